"""RK45 controller traces of the reference's ODE sampler on golden_ode's fixtures (diagnostic fixture).

For each case (T0=1 with t_eval unset, "t1_none"; T0=0.55 with 20 steps, "t055_s20") this records every
step attempt scipy's RK45 makes inside cond_ode_sampler (networks/gf_algorithms/samplers.py:204-234):
the attempt's t, step size h and RMS error norm (rk.py _estimate_error_norm; the attempt is accepted iff
the norm < 1). Two runs per case:

* "ref32": the reference itself, unmodified (PoseNet.pred_func -> cond_ode_sampler -> solve_ivp), the
  score network in float32 as the reference runs it;
* "ref64": the same solve_ivp call restated here with the reference's network converted to float64 and
  the state passed to it in float64 (samplers.py:210-218 without the float32 cast): the arithmetic-free
  trajectory, to tell which controller decisions are set by the float32 rounding of the score.

Same inputs as make_golden.gen_ode (objects of config 21, prior from PCG64(200), synthetic seed-0 weights).
Outputs: golden_ode_trace.json (the attempts and nfev of both runs and cases) and golden_ode_t1_grid.npz: for
T0=1, both runs' solutions on a fixed grid of 101 times (solve_ivp's dense output, which does not change
the step sequence; post-processed as the reference post-processes xs, samplers.py:251-254: Gram-Schmidt
of the rotation columns, + pts_center), so a trajectory taking different steps can still be compared
state by state, and the float64 run's final pose after the reference's denoise step (samplers.py:240-257).
Run here (imports /root/reference read-only, like make_golden.py).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402
import torch  # noqa: E402


def _trace_patch(log):
    from scipy.integrate._ivp import rk
    orig = rk.RungeKutta._estimate_error_norm

    def est(self, K, h, scale):
        n = orig(self, K, h, scale)
        log.append([float(self.t), float(h), float(n)])
        return n
    rk.RungeKutta._estimate_error_norm = est
    return lambda: setattr(rk.RungeKutta, "_estimate_error_norm", orig)


GRID = np.linspace(1.0, 1e-5, 101)


def post(y, centers):
    """(R*9, n_t) solve_ivp states -> (R, n_t, 9): GS of the rotation columns + pts_center, as the reference
    post-processes xs (samplers.py:250-254)."""
    from utils.misc import normalize_rotation
    n_t = y.shape[1]
    xs = torch.tensor(y).T.reshape(n_t, -1, 9)
    R = xs.shape[1]
    xs = xs.reshape(n_t * R, -1)
    xs[:, :-3] = normalize_rotation(xs[:, :-3], "rot_matrix")
    xs = xs.reshape(n_t, R, -1)
    xs[:, :, -3:] += centers.double().unsqueeze(0).repeat(n_t, 1, 1)
    return xs.permute(1, 0, 2).numpy()


def run_ref32(get_config, PoseNet, T0, steps, d, prior, K, keep=None):
    agent = mg.make_agent(get_config, PoseNet, "score", "ode", steps)
    log, calls = [], {"n": 0}
    import scipy.integrate as si
    import networks.gf_algorithms.samplers as smp
    orig = si.solve_ivp

    def counting(fun, *a, **k):
        def f(t, y):
            calls["n"] += 1
            return fun(t, y)
        if keep is None:
            return orig(f, *a, **k)
        res = orig(f, *a, dense_output=True, **k)   # dense output: same steps, an interpolant besides
        keep["sol"] = res.sol
        return res
    smp.integrate.solve_ivp = counting
    undo = _trace_patch(log)
    try:
        with mg.NoiseFeed(prior, np.zeros((0,), np.float32)):
            agent.pred_func(dict(d), repeat_num=K, T0=T0, return_average_res=True, return_process=True)
    finally:
        smp.integrate.solve_ivp = orig
        undo()
    return log, calls["n"]


def run_ref64(get_config, PoseNet, T0, steps, d, prior, K, keep=None):
    """cond_ode_sampler's solve_ivp (samplers.py:196-234) with the network in float64."""
    import scipy.integrate as si
    import networks.pts_encoder.pointnet2_utils.pointnet2.pointnet2_utils as pu
    agent = mg.make_agent(get_config, PoseNet, "score", "ode", steps)
    net = agent.net.double()
    # the copy ops in the input's dtype (the oracle's C restatement is float32); FPS and ball query keep
    # float32 coordinates, as the reference's CUDA ops take them
    saved = (pu.furthest_point_sample, pu.gather_operation, pu.ball_query, pu.grouping_operation)
    fps0, bq0 = pu.furthest_point_sample, pu.ball_query
    pu.furthest_point_sample = lambda xyz, n: fps0(xyz.float(), n)
    pu.ball_query = lambda r, ns, xyz, nxyz: bq0(r, ns, xyz.float(), nxyz.float())
    pu.gather_operation = lambda f, i: torch.gather(f, 2, i.long().unsqueeze(1).expand(-1, f.shape[1], -1))
    pu.grouping_operation = lambda f, i: torch.gather(
        f, 2, i.long().reshape(i.shape[0], 1, -1).expand(-1, f.shape[1], -1)).reshape(f.shape[0], f.shape[1], *i.shape[1:])
    B = d["pts"].shape[0]
    try:
        with torch.no_grad():   # encoder once per object, then every key repeated K times (posenet_agent.py:503-520)
            feat = net({"pts": d["pts"].double()}, mode="pts_feature")
    finally:
        pu.furthest_point_sample, pu.gather_operation, pu.ball_query, pu.grouping_operation = saved
    dd = {"pts_feat": feat.unsqueeze(1).repeat(1, K, 1).view(B * K, -1)}
    sde_coeff = agent.net.sde_fn
    sigma_T = 0.01 * (50 / 0.01) ** T0                    # ve_prior at T0 (sde.py:15-35), the fixture's draws
    # the reference's initial state exactly: torch.randn(...) * sigma in float32 (samplers.py:197-201)
    x0 = (torch.from_numpy(prior) * sigma_T).numpy().astype(np.float64)
    R = B * K

    def ode_func(t, x):
        xt = torch.tensor(x.reshape(-1, 9), dtype=torch.float64)
        dd["sampled_pose"] = xt
        dd["t"] = torch.ones(R, dtype=torch.float64).unsqueeze(-1) * t
        drift, diffusion = sde_coeff(torch.tensor(t))
        with torch.no_grad():
            s = net(dd, mode="score").numpy().reshape(-1)
        return drift.numpy() - 0.5 * (diffusion.numpy() ** 2) * s
    log, calls = [], {"n": 0}

    def f(t, y):
        calls["n"] += 1
        return ode_func(t, y)
    undo = _trace_patch(log)
    try:
        t_eval = None if steps is None else np.linspace(T0, 1e-5, steps)
        res = si.solve_ivp(f, (T0, 1e-5), x0.reshape(-1), rtol=1e-5, atol=1e-5, method="RK45", t_eval=t_eval,
                           dense_output=keep is not None)
    finally:
        undo()
    if keep is not None:
        keep["sol"] = res.sol
        # the denoise step (samplers.py:240-249) in float64, then GS + pts_center (:255-257)
        from utils.misc import normalize_rotation
        eps = 1e-5
        x = torch.tensor(res.y[:, -1]).reshape(R, 9)
        vec_eps = torch.ones((R, 1), dtype=torch.float64) * eps
        drift, diffusion = sde_coeff(vec_eps)
        dd["sampled_pose"] = x
        dd["t"] = vec_eps
        with torch.no_grad():
            grad = net(dd, mode="score")
        drift = drift - diffusion ** 2 * grad
        x = x + drift * ((1 - eps) / (1000 if steps is None else steps))
        x[:, :-3] = normalize_rotation(x[:, :-3], "rot_matrix")
        x[:, -3:] += d["pts_center"].double().unsqueeze(1).repeat(1, K, 1).view(R, 3)
        keep["pred_pose"] = x.numpy().reshape(B, K, 9)
    return log, calls["n"]


def main():
    get_config, PoseNet = mg.import_reference("ode", None)
    out = {}
    for tag, (T0, steps) in {"t1_none": (1.0, None), "t055_s20": (0.55, 20)}.items():
        B, K = 2, 5
        d = mg.batch(21, B, 1024)
        prior = np.random.Generator(np.random.PCG64(200)).standard_normal((B * K, 9)).astype(np.float32)
        k32, k64 = ({}, {}) if tag == "t1_none" else (None, None)
        l32, n32 = run_ref32(get_config, PoseNet, T0, steps, d, prior, K, k32)
        l64, n64 = run_ref64(get_config, PoseNet, T0, steps, d, prior, K, k64)
        if k32 is not None:
            cen = d["pts_center"].unsqueeze(1).repeat(1, K, 1).view(B * K, 3)
            np.savez_compressed(os.path.join(HERE, "golden_ode_t1_grid.npz"), grid=GRID,
                                xs32=post(k32["sol"](GRID), cen).reshape(B, K, len(GRID), 9),
                                xs64=post(k64["sol"](GRID), cen).reshape(B, K, len(GRID), 9),
                                pred_pose64=k64["pred_pose"], nfev32=np.int64(n32), nfev64=np.int64(n64))
        out[tag] = {"ref32": {"nfev": n32, "attempts": l32}, "ref64": {"nfev": n64, "attempts": l64}}
        print(tag, "ref32 nfev", n32, "attempts", len(l32), "| ref64 nfev", n64, "attempts", len(l64), flush=True)
    with open(os.path.join(HERE, "golden_ode_trace.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
