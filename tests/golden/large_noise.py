"""Regenerable inputs of the large-row golden fixtures (golden_large_*.npz).

The fixtures hold only the reference's OUTPUTS. Their inputs are regenerated from committed seeds
on whichever machine runs the test (the build container when make_golden_large.py writes them,
the GPU box when tests/test_gpu_parity.py reads them), so hundreds of MB of recorded noise never
enter the repository:

* points: ``genpose2_amd.synthetic.make_batch(cid, B, 1024)`` (numpy PCG64 per object);
* noise: one numpy PCG64 stream per case, ``standard_normal(dtype=float32)``: the prior (R,9)
  first, then the 2T per-step draws in the order cond_pc_sampler consumes them (corrector z1 of
  step j = draw 2j, predictor z2 = draw 2j+1; samplers.py:148,166).
"""
from __future__ import annotations

import numpy as np

# name -> (sampler, config id of the clouds, B, K, T | None, T0, noise seed)
CASES = {
    "pc_r4800_t100": ("pc", 61, 96, 50, 100, None, 6100),
    "pc_r12800_t100": ("pc", 62, 256, 50, 100, None, 6200),
    "pc_r12800_t500": ("pc", 63, 256, 50, 500, None, 6300),   # the north-star shape itself
    "ode_r4800": ("ode", 64, 96, 50, None, 0.55, 6400),
    "ode_r12800": ("ode", 65, 256, 50, None, 0.55, 6500),
    "pc_cfg5_t100": ("pc", 66, 256, 100, 100, None, 6600),    # config-5 shape (N=2048, K=100) at T=100
}
# points per object where it is not 1024
N_POINTS = {"pc_cfg5_t100": 2048}
# steps j of pc_r12800_t500 whose reference state x_j (the score net's input at step j) and x_{j+1} are
# recorded in golden_large_steps_r12800.npz: single-step pins of the 64-candidate PC tile
STEP_PINS = (1, 400)


def inputs(name: str):
    """(pts (B,N,3), pts_center (B,3), prior (R,9), z1 (T,R,9) | None, z2 (T,R,9) | None)."""
    from genpose2_amd import synthetic
    sampler, cid, B, K, T, _, seed = CASES[name]
    pts, center = synthetic.make_batch(cid, B, N_POINTS.get(name, 1024))
    R = B * K
    rng = np.random.Generator(np.random.PCG64(seed))
    prior = rng.standard_normal((R, 9), dtype=np.float32)
    if sampler != "pc":
        return pts, center, prior, None, None
    z = rng.standard_normal((2 * T, R, 9), dtype=np.float32)
    return pts, center, prior, z[0::2], z[1::2]


def rotation_error_stats(pose: np.ndarray, ref: np.ndarray) -> dict:
    """max / 99.9th percentile / mean of |pose - ref| over the rotation entries (6D columns)."""
    e = np.abs(np.asarray(pose, np.float64)[..., :6] - np.asarray(ref, np.float64)[..., :6])
    return {"max": float(e.max()), "p999": float(np.percentile(e, 99.9)), "mean": float(e.mean())}


def check_calibrated(pose: np.ndarray, g, factor: float = 2.0) -> dict:
    """Parity bar of the large fixtures, calibrated on the reference itself.

    At these sizes the reference's own fp32 trajectories differ from its float64 run by far more than
    the north-star 1e-4 (the untrained score net amplifies rounding along the trajectory; e.g. at
    R=12,800 x T=500 the max rotation error of the reference's fp32 is 1.6e-2). No fp32
    implementation can be held closer to the reference than the reference is to exact arithmetic, so
    the bar is: the implementation's error against the float64 reference run is within `factor` x
    the reference fp32's own error, in max, 99.9th percentile and mean over every rotation entry;
    translations likewise in max absolute error. (ODE, T0=0.55: the reference's own fp32 error at
    R=12,800 is 4.7e-5 max, so the bar there is 9.3e-5 -- inside the north-star 1e-4.)"""
    ref64 = g["pred_pose64"]
    ours = rotation_error_stats(pose, ref64)
    refs = rotation_error_stats(g["pred_pose"], ref64)
    t_ours = float(np.abs(np.asarray(pose, np.float64)[..., 6:] - ref64[..., 6:]).max())
    t_ref = float(np.abs(g["pred_pose"][..., 6:].astype(np.float64) - ref64[..., 6:]).max())
    for k in ("max", "p999", "mean"):
        assert ours[k] <= factor * refs[k], (k, ours, refs)
    assert t_ours <= factor * t_ref, (t_ours, t_ref)
    return {"ours_vs_ref64": ours, "ref32_vs_ref64": refs, "trans_ours": t_ours, "trans_ref32": t_ref}


check_pc_calibrated = check_calibrated


def check_ode(pose: np.ndarray, g) -> dict:
    """Parity bar of the large ODE fixtures: the north-star bar against the reference's fp32 run (rotation
    1e-4 absolute, translation 1e-5 relative to max |t|) and rotation within 1e-4 of its float64 run too.
    The calibrated 2x bar of check_calibrated does not carry over: RK45's step sizes are continuous
    functions of its error norms, so any last-bit change in the right-hand side (a different summation
    order anywhere in the score net) moves the whole step sequence -- with the same nfev -- and the
    solution by up to the solver's tolerance scale (rtol = atol = 1e-5). The reference's fp32 and
    float64 runs share their step sequence, which is why they sit closer to each other (4.7e-5 max at
    R=12,800, 8.4e-6 at R=4,800) than two independently rounded fp32 runs do. Returns the statistics."""
    ref64 = g["pred_pose64"]
    ours = rotation_error_stats(pose, ref64)
    refs = rotation_error_stats(g["pred_pose"], ref64)
    vs32 = rotation_error_stats(pose, g["pred_pose"])
    p = np.asarray(pose, np.float64)
    t_rel = float(np.abs(p[..., 6:] - g["pred_pose"][..., 6:]).max() / np.abs(g["pred_pose"][..., 6:]).max())
    assert vs32["max"] < 1e-4 and ours["max"] < 1e-4 and t_rel < 1e-5, (vs32, ours, t_rel)
    return {"ours_vs_ref32": vs32, "ours_vs_ref64": ours, "ref32_vs_ref64": refs, "trans_rel_vs_ref32": t_rel}
