"""Pin the oracle (CPU restatement) to outputs of the reference itself.

Fixtures: tests/golden/*.npz, produced by tests/golden/make_golden.py from the imported
reference with recorded noise and seeded synthetic weights. Tolerances:
  * index outputs (FPS, ball query, sort orders, DBSCAN labels): exact;
  * fp32 network outputs: |a-b| <= 1e-5 * max|b| (different but valid fp32 summation orders);
  * PC sampler: rotation |a-b| <= 1e-4 (north_star), translation relative to max |t| 1e-5;
  * ODE sampler (scipy RK45, adaptive): T0=0.55 within 1e-5; T0=1.0 the step-size controller
    may take a different accept/reject path, so the bound is the integrator tolerance scale
    (5e-4 abs rotation, 1e-4 relative translation).
"""
import numpy as np
import pytest

from conftest import golden
from oracle import oracle


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("tag", ["n1024", "n2048"])
def test_encoder_levels(tag, score_sd):
    g = golden("encoder")
    feat, levels = oracle.encoder_forward(score_sd, g[f"{tag}_pts"], return_levels=True)
    for lv in range(4):
        assert np.array_equal(levels[lv]["fps_idx"], g[f"{tag}_l{lv}_fps"])
        np.testing.assert_array_equal(levels[lv]["new_xyz"], g[f"{tag}_l{lv}_new_xyz"])
        for b in range(2):
            assert np.array_equal(levels[lv]["ball_idx"][b], g[f"{tag}_l{lv}_ball{b}"])
    for lv in range(5):
        assert rel(levels[lv]["features"][0], g[f"{tag}_l{lv}_feat0"]) < 1e-5
    assert rel(feat, g[f"{tag}_feat"]) < 1e-5


def test_score_and_energy_heads(score_sd, energy_sd):
    g = golden("heads")
    s = oracle.score_forward(score_sd, g["pts_feat"], g["pose"], g["t"])
    # per-row scale: sigma(t) spans 0.01..50 across rows
    err = np.abs(s - g["score"]).max(1) / np.abs(g["score"]).max(1)
    assert err.max() < 1e-5
    e = oracle.energy_forward(energy_sd, g["pts_feat"], g["pose"], g["t"])
    err = np.abs(e - g["energy"]).max(1) / np.abs(g["energy"]).max(1)
    assert err.max() < 1e-5


@pytest.mark.parametrize("name", ["pc_k10_t100", "pc_k50_t20"])
def test_pc_pred_func(name, score_sd):
    g = golden(name)
    K, T = int(g["K"]), int(g["T"])
    pose, q, feat, ex = oracle.pred_func(score_sd, g["pts"], g["pts_center"], K, T, "pc",
                                         g["prior"], g["z1"], g["z2"])
    assert rel(feat, g["pts_feat"]) < 1e-5
    assert np.abs(pose[..., :6] - g["pred_pose"][..., :6]).max() < 1e-4
    assert rel(pose[..., 6:], g["pred_pose"][..., 6:]) < 1e-5
    assert np.abs(q[..., :4] - g["pred_q"][..., :4]).max() < 1e-4
    if "xs" in g.files:
        xs = ex["xs"].reshape(g["xs"].shape)
        assert np.abs(xs[..., :6] - g["xs"][..., :6]).max() < 1e-4


@pytest.mark.parametrize("tag,rot_tol,tr_rel", [("t055_s20", 1e-5, 1e-5), ("t1_none", 5e-4, 1e-4)])
def test_ode_pred_func(tag, rot_tol, tr_rel, score_sd):
    g = golden("ode")
    steps = int(g[f"{tag}_steps"])
    steps = None if steps < 0 else steps
    pose, q, feat, ex = oracle.pred_func(score_sd, g[f"{tag}_pts"], g[f"{tag}_pts_center"], 5, steps,
                                         "ode", g[f"{tag}_prior"], T0=float(g[f"{tag}_T0"]))
    gp = g[f"{tag}_pred_pose"]
    assert pose.dtype == np.float64  # ODE path returns float64
    assert np.abs(pose[..., :6] - gp[..., :6]).max() < rot_tol
    assert rel(pose[..., 6:], gp[..., 6:]) < tr_rel
    if steps is not None:
        assert ex["nfev"] == int(g[f"{tag}_nfev"])
        xs = ex["xs"].reshape(g[f"{tag}_xs"].shape)
        assert np.abs(xs - g[f"{tag}_xs"]).max() < 1e-5 * np.abs(g[f"{tag}_xs"]).max()


def test_tracking_warm_start(score_sd):
    """init_x + small T0 (runners/evaluation_tracking.py:110-127)."""
    g = golden("tracking")
    K, T, T0 = int(g["K"]), int(g["T"]), float(g["T0"])
    pose, q, _, _ = oracle.pred_func(score_sd, g["pts"], g["pts_center"], K, T, "pc", g["prior"], g["z1"], g["z2"],
                                     T0=T0, init_x=g["init_x"])
    assert np.abs(pose[..., :6] - g["pc_pred_pose"][..., :6]).max() < 1e-4
    assert rel(pose[..., 6:], g["pc_pred_pose"][..., 6:]) < 1e-5
    pose, q, _, ex = oracle.pred_func(score_sd, g["pts"], g["pts_center"], K, None, "ode", g["prior"], T0=T0,
                                      init_x=g["init_x"])
    assert np.abs(pose[..., :6] - g["ode_pred_pose"][..., :6]).max() < 1e-4
    assert rel(pose[..., 6:], g["ode_pred_pose"][..., 6:]) < 1e-5
    assert ex["nfev"] == int(g["ode_nfev"])


def test_energy_sort_aggregate_scale(energy_sd, scale_sd):
    g = golden("pipeline")
    e = oracle.get_energy(energy_sd, g["pts"], g["pts_center"], g["pred_pose"], 1e-5)
    assert rel(e, g["energy"]) < 1e-5
    sp, se, _, _ = oracle.sort_poses_by_energy(g["pred_pose"], g["energy"])
    assert np.array_equal(sp, g["sorted_pose"]) and np.array_equal(se, g["sorted_energy"])
    for c in (0, 1):
        a = oracle.aggregate_pose(g["pred_pose"], g["energy"], clustering=c)
        assert np.abs(a - g[f"aggregated_c{c}"]).max() < 1e-4
    a = oracle.aggregate_pose(g["cl_pose"], g["cl_energy"], clustering=1)
    assert np.abs(a - g["cl_aggregated"]).max() < 1e-4
    L = oracle.scale_forward(scale_sd, g["pts_feat"], g["scale_axes"])
    assert rel(L, g["scale_length"]) < 1e-5


def test_stage_glue_oracle_restatements():
    """oracle.points_mean / bbox_length against the reference's own torch expressions
    (datasets_omni6dpose.py:746-752; evaluation_single.py:233-252), typed out op for op."""
    import torch
    rng = np.random.default_rng(4)
    B, N = 3, 1000
    pcl = rng.normal(size=(B, N, 3)).astype(np.float32) * 0.05 + np.array([0.0, 0.1, 0.7], np.float32)
    ref_center = torch.mean(torch.from_numpy(pcl)[:, :, :3], dim=1).numpy()
    np.testing.assert_allclose(oracle.points_mean(pcl), ref_center, rtol=1e-6, atol=1e-7)
    q = rng.normal(size=(B, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    pose = np.zeros((B, 4, 4), np.float32)
    pose[:, :3, :3] = oracle.quaternion_to_matrix(q.astype(np.float32))
    pose[:, :3, 3] = ref_center
    pose[:, 3, 3] = 1
    p = torch.from_numpy(pcl)
    rotation = torch.from_numpy(pose)[:, :3, :3]
    rotation_t = torch.transpose(rotation, 1, 2)
    translation = torch.from_numpy(pose)[:, :3, 3]
    p = p - translation.unsqueeze(1)
    p = p.reshape(-1, 3, 1)
    rotation_t = torch.repeat_interleave(rotation_t, N, dim=0)
    p = torch.bmm(rotation_t, p).reshape(-1, N, 3)
    ref_len, _ = torch.max(torch.abs(p), dim=1)
    ref_len *= 2
    np.testing.assert_allclose(oracle.bbox_length(pcl, pose), ref_len.numpy(), rtol=2e-6, atol=1e-7)


# ---------------------------------------------------------------- large-row fixtures (> 4096 rows)
def test_pc_large_rows_calibrated(score_sd):
    """R = 4800 (B=96, K=50), T=100: the oracle (another fp32 rounding of the same sampler) is held to
    the reference's own fp32-vs-float64 error budget (tests/golden/large_noise.py)."""
    import large_noise
    g = golden("large_pc_r4800_t100")
    _, _, B, K, T, _, _ = large_noise.CASES["pc_r4800_t100"]
    pts, center, prior, z1, z2 = large_noise.inputs("pc_r4800_t100")
    pose, q, _, _ = oracle.pred_func(score_sd, pts, center, K, T, "pc", prior, z1, z2)
    large_noise.check_pc_calibrated(pose, g)
    assert rel(pose[..., 6:], g["pred_pose"][..., 6:]) < 1e-5


def test_ode_large_rows(score_sd):
    """R = 4800, the shipped ODE setting (T0=0.55, RK45): identical nfev, the calibrated bar against the
    float64 reference, and 1e-4 / 1e-5 against the fp32 reference."""
    import large_noise
    g = golden("large_ode_r4800")
    _, _, B, K, _, T0, _ = large_noise.CASES["ode_r4800"]
    pts, center, prior, _, _ = large_noise.inputs("ode_r4800")
    pose, q, _, ex = oracle.pred_func(score_sd, pts, center, K, None, "ode", prior, T0=T0)
    assert ex["nfev"] == int(g["nfev"])
    large_noise.check_calibrated(pose, g)
    assert np.abs(pose[..., :6] - g["pred_pose"][..., :6]).max() < 1e-4
    assert rel(pose[..., 6:], g["pred_pose"][..., 6:]) < 1e-5


def test_fus_encoder_levels():
    """Pointnet2ClsMSGFus (DINO-pointwise fused encoder) restatement vs the reference's own module
    (golden_fus.npz, tests/golden/make_golden_fus.py): per-level SA output, fused input, transformer
    output, the level-3 relative-PE bias and the final feature."""
    import make_golden_fus as mf
    from genpose2_amd import synthetic, weights
    g = golden("fus")
    sd = weights.synthetic_state_dict("score_pointwise")
    pts, _ = synthetic.make_batch(mf.CID, mf.B, mf.N)
    feat, levels = oracle.fus_encoder_forward(sd, pts, mf.rgb_features(mf.B, mf.N), return_levels=True)
    for lv in range(5):
        if levels[lv]["fps_idx"] is not None:
            assert np.array_equal(levels[lv]["fps_idx"], g[f"l{lv}_fps"])
        for k in ("sa", "tf", "fused"):
            if f"l{lv}_{k}" in g:
                assert rel(levels[lv][k][0], g[f"l{lv}_{k}"]) < 1e-5, (lv, k)
    assert rel(levels[3]["bias"][0], g["l3_bias"]) < 1e-6
    assert rel(feat, g["feat"]) < 1e-5


def test_energy_rank_aggregate_r12800_subset(energy_sd):
    """golden_large_energy_r12800 (EnergyNet + sort + aggregation at config 4's shape) on its first 12
    objects: the oracle's energies within 1e-5 of max|ref| per object, the sort order identical, the
    aggregated 4x4 within 1e-5 -- plain and clustered candidate sets."""
    import large_noise
    from genpose2_amd import synthetic
    g = golden("large_energy_r12800")
    src = str(g["src"])
    _, cid, B, K, _, _, _ = large_noise.CASES[src]
    n = 12
    pts, center = synthetic.make_batch(cid, B, 1024)
    pts, center = pts[:n], center[:n]
    plain = golden(f"large_{src}")["pred_pose"][:n]
    for pose, e_ref, idx, agg_ref, c in ((plain, g["energy"], g["sort_idx"], g["aggregated_c0"], 0),
                                         (g["cl_pose"][:n], g["cl_energy"], g["cl_sort_idx"], g["cl_aggregated_c1"], 1)):
        e = oracle.get_energy(energy_sd, pts, center, pose, 1e-5)
        err = np.abs(e - e_ref[:n]).reshape(n, -1).max(1) / np.abs(e_ref[:n]).reshape(n, -1).max(1)
        assert err.max() < 1e-5
        sp, _, _, _ = oracle.sort_poses_by_energy(pose, e)
        ii = idx[:n].astype(np.int64)
        np.testing.assert_array_equal(sp[..., :6], np.take_along_axis(pose, ii[..., 0:1], 1)[..., :6])
        np.testing.assert_array_equal(sp[..., 6:], np.take_along_axis(pose, ii[..., 1:2], 1)[..., 6:])
        agg = oracle.aggregate_pose(pose, e, clustering=c)
        assert np.abs(agg[:, :3, :3] - agg_ref[:n, :3, :3]).max() < 1e-5
        assert rel(agg[:, :3, 3], agg_ref[:n, :3, 3]) < 1e-5


def test_img_encoder_and_gather_vs_reference():
    """ImgEncoder (img_encoder.py:48-100) and the patch -> point gather (posenet.py:146-192) restated in the
    oracle, against the reference's own outputs (golden_img.npz, tests/golden/make_golden_img.py):
    near-one-hot ("hard") and spread ("soft") geometric attention, out-of-range roi pixels clamped."""
    import make_golden_img as mi
    from genpose2_amd import weights
    g = golden("img")
    sd = weights.synthetic_state_dict("score_pointwise", seed=0)
    for tag, (B, scale, seed) in mi.CASES.items():
        layers = mi.dino_layers(B, scale, seed)
        final, parts = oracle.img_encoder_forward(sd, layers, return_parts=True)
        assert rel(final[0], g[f"{tag}_final0"]) < 1e-5, tag
        np.testing.assert_allclose(final.astype(np.float64).sum(axis=(1, 2)), g[f"{tag}_final_sum"], rtol=1e-5)
        assert rel(parts["edge"], g[f"{tag}_edge"]) < 1e-5
        assert rel(parts["layer_w"], g[f"{tag}_layer_w"]) < 1e-5
        xs, ys = mi.roi_pixels(B, 1024, seed)
        gathered = oracle.gather_patch_points(final, xs, ys)
        assert rel(gathered[0, :64], g[f"{tag}_gather0"]) < 1e-5
