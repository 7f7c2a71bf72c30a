"""The north-star configurations at full size on a real MI355X, against the reference where a reference
run fits this container (tests/golden/make_golden_large.py) and through size-independent properties
where it does not.

* EnergyNet + ranking + aggregation at config 4's shape (R = 12,800) on the reference's own poses:
  energies within 1e-5 of max|ref| per object, the sort order identical, the aggregated 4x4 within
  1e-5 (rotation absolute, translation relative) -- with and without DBSCAN, and on a clustered
  candidate set where DBSCAN re-averages every object.
* Config 5's shape (B=256, N=2048, K=100: R = 25,600 rows, two passes of 64-candidate PC tiles) at
  T=100: the N=2048 encoder output at 1e-5, the PC poses at the calibrated bar
  (large_noise.check_calibrated), ScaleNet lengths at 1e-5.
* Single-step pins at R = 12,800: from the reference's own state x_j, one PC step (Langevin corrector
  with the batch's grad_norm, predictor, Gram-Schmidt) against the reference's x_{j+1}, for both
  arithmetic paths -- translation 1e-5 relative; rotation within 2x the reference's own fp32 error
  against a float64 step from the same x_j, and 1e-5 absolute against the reference where that step
  is well conditioned (step 400: the reference's own error 2.4e-7; step 1, at sigma(1) = 50, it is
  1.5e-4). This holds the 64-candidate tile itself to the bar, independent of trajectory chaos.
* Config 5 at its full T=1000 with device noise: determinism, Philox == the same draws injected,
  orthonormal rotations, unit quaternions, finite ScaleNet lengths.
"""
import numpy as np
import pytest
import torch

from conftest import ARITHS, ARITHS3, golden, set_arith

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _agent(**kw):
    from genpose2_amd.agent import PoseNet
    from genpose2_amd.config import GenPoseConfig
    return PoseNet(GenPoseConfig(device=DEV, **kw)).eval()


def _rot_abs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def _rel(a, b):
    b = np.asarray(b, np.float64)
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def _check_agg(got, want):
    assert _rot_abs(got[:, :3, :3], want[:, :3, :3]) < 1e-5
    assert _rel(got[:, :3, 3], want[:, :3, 3]) < 1e-5
    assert np.array_equal(got[:, 3], want[:, 3])


def _obj_rel(a, b):
    B = b.shape[0]
    return np.abs(np.asarray(a, np.float64) - b).reshape(B, -1).max(1) / np.abs(b).reshape(B, -1).max(1)


def _rank_mismatches(e, idx_ref, e64, tol):
    """Positions where our descending order (energy column j) differs from the reference's; each must be
    a near-tie: the float64 energies of the two candidates differ by less than `tol` x the object's
    max |energy| (fp32 rounding can order them either way)."""
    bad = []
    order = np.argsort(-e, axis=1, kind="stable")
    for j in range(2):
        for b, k in zip(*np.nonzero(order[..., j] != idx_ref[..., j])):
            a, r = order[b, k, j], idx_ref[b, k, j]
            scale = np.abs(e64[b]).max()
            if abs(e64[b, a, j] - e64[b, r, j]) > tol * scale:
                bad.append((b, k, j))
    return int((order != idx_ref).sum()), bad


@pytest.mark.parametrize("arith", ARITHS)
def test_energy_rank_aggregate_r12800_vs_reference(arith):
    """Config 4's EnergyNet leg on the reference's own 12,800 PC candidates: energies within 1e-5 of
    max|ref| per object, the sort order identical, the aggregated 4x4 (with and without DBSCAN) within
    1e-5. A clustered candidate set (every object re-averaged by DBSCAN) has energies whose pose . score
    sums cancel ~100x: there the reference's own fp32 energies sit up to 9.6e-6 from its float64 run,
    so the bar is calibrated on it (max over objects within 2x the reference's own error), the order
    may differ only at near-ties inside that error, the kept top-20 sets must equal the reference's at every
    (object, column) pair except where the fixture itself holds a boundary near-tie (one pair), and the
    aggregation is held at 1e-5 from the reference's energies (the aggregation alone) and from ours on every
    object whose kept sets are the reference's."""
    import large_noise
    from genpose2_amd import aggregate, synthetic
    g = golden("large_energy_r12800")
    src = str(g["src"])
    _, cid, B, K, _, _, _ = large_noise.CASES[src]
    pts, center = synthetic.make_batch(cid, B, 1024)
    agent = _agent(agent_type="energy")
    set_arith(agent, arith)
    data = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
    keep = int(K * 0.4)

    def energies(pose_np):
        pose = torch.from_numpy(pose_np).to(DEV)
        e = agent.get_energy(dict(data), pose, T=1e-5, mode="test", extract_feature=True)
        assert e.shape == (B, K, 2) and e.dtype == torch.float32
        return pose, e

    def sorted_ok(pose, e, pose_np, idx):
        sp = aggregate.sort_poses_by_energy(pose, e)[0].cpu().numpy()
        want_rot = np.take_along_axis(pose_np, idx[..., 0:1], 1)[..., :6]
        want_tr = np.take_along_axis(pose_np, idx[..., 1:2], 1)[..., 6:]
        return np.array_equal(sp[..., :6], want_rot) and np.array_equal(sp[..., 6:], want_tr)

    # ---- the sampler's candidates
    pose_np = golden(f"large_{src}")["pred_pose"]
    pose, e = energies(pose_np)
    err = _obj_rel(e.cpu().numpy(), g["energy"])
    print(arith, "plain: energy vs ref32 max", err.max())
    assert err.max() < 1e-5, err.max()
    idx = g["sort_idx"].astype(np.int64)
    assert sorted_ok(pose, e, pose_np, idx)               # ranking identical to the reference's
    for c in (0, 1):
        for en in (torch.from_numpy(g["energy"]).to(DEV), e):
            got = aggregate.aggregate_pose(pose, en, 0.4, c, 0.05, 0.1667, retain_num=keep)
            _check_agg(got.cpu().numpy(), g[f"aggregated_c{c}"])

    # ---- clustered candidates (cancellation-heavy energies)
    pose_np = g["cl_pose"]
    pose, e = energies(pose_np)
    e_np = e.cpu().numpy()
    own = _obj_rel(g["cl_energy"], g["cl_energy64"])
    ours = _obj_rel(e_np, g["cl_energy64"])
    print(arith, "clustered: energy vs ref64 max", ours.max(), "reference fp32's own", own.max(),
          "vs ref32 max", _obj_rel(e_np, g["cl_energy"]).max())
    assert ours.max() <= 2 * own.max()
    idx = g["cl_sort_idx"].astype(np.int64)
    n_diff, bad = _rank_mismatches(e_np, idx, g["cl_energy64"], 2 * own.max())
    print(arith, "clustered: order positions differing from the reference", n_diff, "(not near-ties:", len(bad), ")")
    assert not bad, bad[:5]
    if arith == "fast":
        # the default arithmetic ranks the clustered set exactly as the reference does (the energy epilogue sums in
        # torch-CPU's order, gp_score.hip head_eval_kernel); exact fp32 MFMA differs at near-ties only (checked above)
        assert n_diff == 0, n_diff
    got = aggregate.aggregate_pose(pose, torch.from_numpy(g["cl_energy"]).to(DEV), 0.4, 1, 0.05, 0.1667,
                                   retain_num=keep)
    _check_agg(got.cpu().numpy(), g["cl_aggregated_c1"])
    # kept sets (top `keep` per object and energy column, evaluation_single.py:181-182): ours may differ from
    # the reference's only at (object, column) pairs whose float64 energies of the reference's rank-keep and
    # rank-keep+1 candidates are a near-tie within the reference's own fp32 error (the fixture holds 1 such pair)
    ties = _kept_set_boundary_ties(idx, g["cl_energy64"], keep, 2 * own)
    diff = [(b, j) for b in range(B) for j in range(2)
            if set(np.argsort(-e_np[b, :, j], kind="stable")[:keep]) != set(idx[b, :keep, j])]
    print(arith, f"clustered: kept sets differing from the reference at {len(diff)} of {2 * B} (object, column) "
          f"pairs {diff}; boundary near-ties in the reference fixture: {sorted(ties)}")
    assert set(diff) <= ties, sorted(set(diff) - ties)
    same = sorted({b for b in range(B)} - {b for b, _ in diff})
    got = aggregate.aggregate_pose(pose, e, 0.4, 1, 0.05, 0.1667, retain_num=keep).cpu().numpy()
    _check_agg(got[same], g["cl_aggregated_c1"][same])


def _kept_set_boundary_ties(idx_ref, e64, keep, tol):
    """(object, column) pairs whose reference order places candidates at ranks keep-1 and keep (0-based) with
    float64 energies within tol[b] x the object's max |energy| (tol: per object, twice the reference fp32's own
    error there): the kept set may flip there under fp32 rounding."""
    out = set()
    for b in range(idx_ref.shape[0]):
        scale = np.abs(e64[b]).max()
        for j in range(2):
            a, c = idx_ref[b, keep - 1, j], idx_ref[b, keep, j]
            if abs(e64[b, a, j] - e64[b, c, j]) <= tol[b] * scale:
                out.add((b, j))
    return out


@pytest.mark.parametrize("arith", ARITHS)
def test_config5_shape_vs_reference(arith):
    """B=256, N=2048, K=100 (R=25,600: 400 PC workgroups, two passes), T=100, reference noise."""
    import large_noise
    from genpose2_amd.agent import NoiseFeed
    name = "pc_cfg5_t100"
    g = golden(f"large_{name}")
    _, _, B, K, T, _, _ = large_noise.CASES[name]
    pts, center, prior, z1, z2 = large_noise.inputs(name)
    assert pts.shape == (256, 2048, 3) and B * K == 25600
    agent = _agent(sampling_steps=T)
    set_arith(agent, arith)
    agent.noise_feed = NoiseFeed(torch.from_numpy(prior), torch.from_numpy(np.ascontiguousarray(z1)),
                                 torch.from_numpy(np.ascontiguousarray(z2)))
    del z1, z2
    data = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
    pose, q = agent.pred_func(data, repeat_num=K)
    feat = data["pts_feat"].cpu().numpy()
    err = np.abs(feat - g["pts_feat"]).max(1) / np.abs(g["pts_feat"]).max(1)
    assert err.max() < 1e-5, err.max()
    p = pose.cpu().numpy()
    stats = large_noise.check_calibrated(p, g)
    print(name, arith, stats)
    assert _rel(p[..., 6:], g["pred_pose"][..., 6:]) < 1e-5
    assert torch.isfinite(q).all()
    scale = _agent(agent_type="scale")
    _, length = scale.pred_scale_func({"pts_feat": torch.from_numpy(g["pts_feat"]).to(DEV),
                                       "axes": torch.from_numpy(g["scale_axes"]).to(DEV)})
    assert _rel(length.cpu().numpy(), g["scale_length"]) < 1e-5


@pytest.mark.parametrize("arith", ARITHS3)
def test_pc_single_step_pins_r12800(arith):
    import large_noise
    g = golden("large_steps_r12800")
    src = str(g["src"])
    _, _, B, K, T, _, _ = large_noise.CASES[src]
    pts, center, prior, z1, z2 = large_noise.inputs(src)
    agent = _agent(sampling_steps=T)
    set_arith(agent, arith)
    cdev = torch.from_numpy(center).to(DEV)
    feat = agent.encoder.forward(torch.from_numpy(pts).to(DEV))
    pobj = agent.heads.object_proj(feat)
    tab, tproj = agent._pc_table(T)
    c_rows = np.repeat(center, K, 0)                     # (R,3): object of row r is r // K
    for j in (int(s) for s in g["steps"]):
        x = torch.from_numpy(g[f"x_{j}"]).to(DEV).contiguous()
        zz1 = torch.from_numpy(np.ascontiguousarray(z1[j:j + 2])).to(DEV)
        zz2 = torch.from_numpy(np.ascontiguousarray(z2[j:j + 2])).to(DEV)
        # a 2-step call over grid rows j, j+1: its xs[:, 0] is the state after step j, + pts_center
        _, _, xs = agent.heads.pc_sample(pobj, tproj[j:j + 2], tab[j:j + 2], x, K, cdev, z1=zz1, z2=zz2,
                                         want_xs=True)
        got = xs[:, 0].cpu().numpy()
        want = g[f"x_{j + 1}"].copy()
        want[:, 6:] = want[:, 6:] + c_rows                  # samplers.py:173 in fp32, as the kernel does
        rot = _rot_abs(got[:, :6], want[:, :6])
        tr = _rel(got[:, 6:], want[:, 6:])
        x64 = g[f"x64_{j + 1}"]
        own = _rot_abs(g[f"x_{j + 1}"][:, :6], x64[:, :6])             # the reference's own fp32 step error
        mine = _rot_abs(got[:, :6], x64[:, :6])
        print(f"step {j} ({arith}): rotation {rot:.2e} abs vs ref32, {mine:.2e} vs float64 (reference's own "
              f"{own:.2e}), translation {tr:.2e} rel")
        assert tr < 1e-5 and mine <= 2 * own, (j, rot, mine, own, tr)
        if own < 5e-6:   # a well-conditioned step: the north-star bar against the reference itself
            assert rot < 1e-5, (j, rot)


def _score64(sd, feat, x, t32):
    """PoseScoreNet.forward (scorenet.py:215-275) in float64 from fp32 features, poses and time value."""
    from genpose2_amd import arch, weights
    p = {k: v.astype(np.float64) for k, v in weights.head_params(sd).items()}
    t = float(t32)
    xp = t * p["gfp_w"] * 2.0 * np.pi
    tf = np.maximum(p["te_w"] @ np.concatenate([np.sin(xp), np.cos(xp)]) + p["te_b"], 0.0)
    h = np.maximum(x.astype(np.float64) @ p["pe0_w"].T + p["pe0_b"], 0.0)
    pf = np.maximum(h @ p["pe2_w"].T + p["pe2_b"], 0.0)
    out = []
    for k in range(3):
        u = np.maximum(feat @ p["h1_pts"][k].T + p["h1_t"][k] @ tf + pf @ p["h1_pose"][k].T + p["h1_b"][k], 0.0)
        out.append(u @ p["h2_w"][k].T + p["h2_b"][k])
    sig = arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** t
    return np.concatenate(out, 1) / (sig + 1e-7)


def test_head_gemm_arith_vs_float64_r12800():
    """The head kernels' arithmetic, free of trajectory chaos: one score evaluation of the 12,800 states the
    reference's PC run entered steps 1 and 400 with (golden_large_steps_r12800), with the same fp32 features
    (exact-fp32 encoder) and fp32 object/time rows, in the f16x3 GEMMs (default) and in exact fp32 MFMA,
    against the same network in float64. The f16x3 GEMMs form every product of the fp32 operands to ~2^-33
    and accumulate hi*hi with one MFMA rounding per 32-deep chunk (v_mfma_f32_16x16x32_f16 measured at
    ~0.9 x 2^-24 of its largest term per 33 terms vs v_mfma_f32_16x16x4_f32's ~0.6 per 5,
    scripts/mfma_round_probe.hip), so over the 256-deep GEMMs their error is below exact fp32's: the
    mean and 99.9th percentile of the score error are asserted <= exact fp32's, max printed."""
    import large_noise
    from genpose2_amd import weights
    g = golden("large_steps_r12800")
    src = str(g["src"])
    _, _, B, K, T, _, _ = large_noise.CASES[src]
    pts, _, _, _, _ = large_noise.inputs(src)
    agent = _agent(sampling_steps=T)
    agent.encoder.set_arith("f32")
    feat = agent.encoder.forward(torch.from_numpy(pts).to(DEV))
    pobj = agent.heads.object_proj(feat)
    tab, tproj = agent._pc_table(T)
    feat_rows = np.repeat(feat.cpu().numpy().astype(np.float64), K, 0)
    sd = weights.synthetic_state_dict("score")
    for j in (int(s) for s in g["steps"]):
        x = torch.from_numpy(g[f"x_{j}"]).to(DEV).contiguous()
        ref = _score64(sd, feat_rows, g[f"x_{j}"], tab[j, 0])
        scale = np.abs(ref).max(1, keepdims=True)
        stats = {}
        for arith in ("f16x3", "f32"):
            agent.heads.set_arith(arith)
            s = agent.heads.score(pobj, tproj[j], float(tab[j, 1]), x, K).cpu().numpy().astype(np.float64)
            e = np.abs(s - ref) / scale
            stats[arith] = {"max": float(e.max()), "p999": float(np.percentile(e, 99.9)), "mean": float(e.mean())}
        print(f"step {j} score vs float64 (per-row relative): f16x3 {stats['f16x3']}  exact fp32 {stats['f32']}")
        for arith in stats:
            assert stats[arith]["max"] < 1e-5, (j, arith, stats)
        assert stats["f16x3"]["mean"] <= stats["f32"]["mean"] and stats["f16x3"]["p999"] <= stats["f32"]["p999"], stats
    agent.heads.set_arith("f16x3")


def test_config5_full_t1000_properties():
    """Config 5 at full size (B=256, N=2048, K=100, T=1000) with device Philox noise."""
    from genpose2_amd import device, synthetic
    B, N, K, T = 256, 2048, 100, 1000
    R = B * K
    pts, center = synthetic.make_batch(5, B, N)
    data = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
    a1 = _agent(sampling_steps=T, noise_seed=11)
    a2 = _agent(sampling_steps=T, noise_seed=11)
    d1 = dict(data)
    p1, q1 = a1.pred_func(d1, repeat_num=K)
    p2, q2 = a2.pred_func(dict(data), repeat_num=K)
    assert p1.shape == (B, K, 9) and torch.isfinite(p1).all() and torch.isfinite(q1).all()
    assert torch.equal(p1, p2) and torch.equal(q1, q2)
    r = p1.reshape(-1, 9).double()
    b1, b2 = r[:, :3], r[:, 3:6]
    assert (b1.norm(dim=1) - 1).abs().max() < 1e-5 and (b2.norm(dim=1) - 1).abs().max() < 1e-5
    assert (b1 * b2).sum(1).abs().max() < 1e-5
    assert (q1[..., :4].double().norm(dim=-1) - 1).abs().max() < 1e-5
    # the same run with its Philox draws injected (1.8 GB of noise on the device) is bit-identical
    heads = a1.heads
    feat = d1["pts_feat"]
    pobj = heads.object_proj(feat)
    tab, tproj = a1._pc_table(T)
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    x0 = torch.randn((R, 9), generator=g, device=DEV) * 50.0
    seed = 77
    res_p, q_p, _ = heads.pc_sample(pobj, tproj, tab, x0.clone(), K, data["pts_center"], seed=seed)
    z1 = torch.empty((T, R, 9), device=DEV)
    z2 = torch.empty((T, R, 9), device=DEV)
    for j in range(T):
        z1[j] = device.randn(seed, 2 * j, R, 9, DEV)
        z2[j] = device.randn(seed, 2 * j + 1, R, 9, DEV)
    res_i, q_i, _ = heads.pc_sample(pobj, tproj, tab, x0.clone(), K, data["pts_center"], z1=z1, z2=z2)
    assert torch.equal(res_p, res_i) and torch.equal(q_p, q_i)
    del z1, z2
    scale = _agent(agent_type="scale")
    axes = torch.eye(3, device=DEV).expand(B, 3, 3).contiguous()
    _, length = scale.pred_scale_func({"pts_feat": feat, "axes": axes})
    assert length.shape == (B, 3) and torch.isfinite(length).all()
