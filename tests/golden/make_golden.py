"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the build container (it reads /root/reference read-only; the GPU box never
runs it). The reference is imported as a Python package with:
  * stub modules for imports that are off the hot path (ipdb, tensorboardX, cv2, torchvision,
    cutoop, and the CUDA extension ``pointnet2_cuda``);
  * the four PointNet++ CUDA ops replaced at module-attribute level by the oracle's CPU
    restatement (the reference has no CPU implementation);
  * seeded synthetic weights (genpose2_amd.weights) loaded with load_state_dict;
  * torch.randn / torch.randn_like fed from recorded standard-normal buffers, so the
    stochastic samplers are reproducible by any implementation (SURVEY §7 "Hard parts" 1).

Everything else -- SA modules, SharedMLP, ScoreNet/EnergyNet, the PC and ODE samplers
(with scipy RK45), pred_func/get_energy, sort_poses_by_energy, the rotation utilities,
ScaleNet -- is the reference's own code. The aggregation stage re-traces the call sequence
of runners/evaluation_single.py:160-219 over the reference's functions (that runner is a
script with module-level data loading and cannot be imported).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

import torch  # noqa: E402

from genpose2_amd import synthetic, weights  # noqa: E402
from oracle import oracle  # noqa: E402

torch.set_num_threads(8)


class _StubModule(types.ModuleType):
    """Module whose unknown attributes are inert placeholders (off-path imports only)."""

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        return type(item, (), {})


def _stub(name, **attrs):
    m = _StubModule(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def import_reference(sampler: str, steps):
    for n in ("ipdb",):
        _stub(n, set_trace=lambda *a, **k: None)
    _stub("pointnet2_cuda")
    _stub("tensorboardX", SummaryWriter=object)
    _stub("cv2")
    _stub("torchvision")
    _stub("torchvision.utils")
    for n in ("cutoop", "cutoop.eval_utils", "cutoop.rotation"):
        _stub(n)
    argv = ["ref", "--dino", "none", "--device", "cpu", "--sampler_mode", sampler]
    if steps is not None:
        argv += ["--sampling_steps", str(steps)]
    sys.argv = argv
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import networks.pts_encoder.pointnet2_utils.pointnet2.pointnet2_utils as pu

    pu.furthest_point_sample = lambda xyz, n: torch.from_numpy(
        oracle.furthest_point_sample(xyz.numpy(), n))
    pu.gather_operation = lambda f, i: torch.from_numpy(
        oracle.gather_operation(f.contiguous().numpy(), i.numpy()))
    pu.ball_query = lambda r, ns, xyz, nxyz: torch.from_numpy(
        oracle.ball_query(r, ns, xyz.numpy(), nxyz.numpy()))
    pu.grouping_operation = lambda f, i: torch.from_numpy(
        oracle.grouping_operation(f.contiguous().numpy(), i.numpy()))
    from configs.config import get_config
    from networks.posenet_agent import PoseNet
    return get_config, PoseNet


class NoiseFeed:
    """Replaces torch.randn / torch.randn_like with recorded standard-normal draws."""

    def __init__(self, prior: np.ndarray, zs: np.ndarray):
        self.prior, self.zs, self.i = prior, zs, 0
        self._randn, self._randn_like = torch.randn, torch.randn_like

    def __enter__(self):
        def randn(*shape, **kw):
            shape = tuple(shape[0]) if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else shape
            assert tuple(shape) == self.prior.shape, (shape, self.prior.shape)
            return torch.from_numpy(self.prior.copy())

        def randn_like(x, **kw):
            z = torch.from_numpy(self.zs[self.i].copy())
            assert z.shape == x.shape
            self.i += 1
            return z

        torch.randn, torch.randn_like = randn, randn_like
        return self

    def __exit__(self, *a):
        torch.randn, torch.randn_like = self._randn, self._randn_like


def make_agent(get_config, PoseNet, agent_type, sampler, steps):
    cfg = get_config()
    cfg.agent_type = agent_type
    cfg.sampler_mode = [sampler]
    cfg.sampling_steps = steps
    agent = PoseNet(cfg)
    sd = weights.synthetic_state_dict(agent_type, seed=0)
    agent.net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    agent.eval()
    return agent


def batch(config_id, B, N, tile_every=0):
    pts, _ = synthetic.make_batch(config_id, B, N, n_unique_every=tile_every)
    t = torch.from_numpy(pts)
    return {"pts": t, "pts_center": torch.mean(t, dim=1)}


def gen_encoder(get_config, PoseNet):
    agent = make_agent(get_config, PoseNet, "score", "pc", 20)
    out = {}
    for tag, (cid, B, N) in {"n1024": (11, 3, 1024), "n2048": (12, 2, 2048)}.items():
        d = batch(cid, B, N, tile_every=3)
        xyz, feats = d["pts"], None
        enc = agent.net.pts_encoder
        with torch.no_grad():
            for lv, sa in enumerate(enc.SA_modules):
                new_xyz, feats, fidx = sa(xyz, feats, return_idx=True)
                if fidx is not None:
                    out[f"{tag}_l{lv}_fps"] = fidx.numpy()
                    out[f"{tag}_l{lv}_new_xyz"] = new_xyz.numpy()
                    for b, grp in enumerate(sa.groupers):
                        out[f"{tag}_l{lv}_ball{b}"] = oracle.ball_query(
                            grp.radius, grp.nsample, xyz.numpy(), new_xyz.numpy())
                out[f"{tag}_l{lv}_feat0"] = feats[0].numpy()   # first object only
                xyz = new_xyz if new_xyz is not None else xyz
            feat = agent.net(d, mode="pts_feature")
        out[f"{tag}_pts"] = d["pts"].numpy()
        out[f"{tag}_feat"] = feat.numpy()
    np.savez_compressed(os.path.join(HERE, "golden_encoder.npz"), **out)


def gen_heads(get_config, PoseNet):
    rng = np.random.Generator(np.random.PCG64(7))
    R = 32
    pts_feat = np.maximum(rng.normal(size=(R, 1024)), 0).astype(np.float32)
    pose = rng.normal(size=(R, 9)).astype(np.float32)
    pose[:, 6:] *= 0.3
    t = np.exp(np.linspace(np.log(1e-5), 0.0, R)).astype(np.float32)[:, None]
    out = dict(pts_feat=pts_feat, pose=pose, t=t)
    for kind in ("score", "energy"):
        agent = make_agent(get_config, PoseNet, kind, "pc", 20)
        data = {"pts_feat": torch.from_numpy(pts_feat), "rgb_feat": None,
                "sampled_pose": torch.from_numpy(pose), "t": torch.from_numpy(t)}
        with torch.no_grad():
            y = agent.net(data, mode="score" if kind == "score" else "energy")
        out[kind] = y.numpy()
    np.savez_compressed(os.path.join(HERE, "golden_heads.npz"), **out)


def gen_pc(get_config, PoseNet, name, cid, B, K, T, tile_every=2):
    agent = make_agent(get_config, PoseNet, "score", "pc", T)
    d = batch(cid, B, 1024, tile_every=tile_every)
    rng = np.random.Generator(np.random.PCG64(100 + cid))
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    zs = rng.standard_normal((2 * T, B * K, 9)).astype(np.float32)
    with NoiseFeed(prior, zs) as nf:
        pose, q, q_avg, proc = agent.pred_func(d, repeat_num=K, return_average_res=True,
                                               return_process=True)
        assert nf.i == 2 * T
    out = dict(pts=d["pts"].numpy(), pts_center=d["pts_center"].numpy(), prior=prior,
               z1=zs[0::2], z2=zs[1::2], pred_pose=pose.numpy(), pred_q=q.numpy(),
               pred_q_avg=q_avg.numpy(), pts_feat=d["pts_feat"].numpy(), K=K, T=T)
    if T <= 100:
        out["xs"] = proc.numpy()
    np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), **out)
    return d, pose


def gen_ode(get_config, PoseNet):
    out = {}
    for tag, (T0, steps) in {"t1_none": (1.0, None), "t055_s20": (0.55, 20)}.items():
        agent = make_agent(get_config, PoseNet, "score", "ode", steps)
        B, K = 2, 5
        d = batch(21, B, 1024)
        prior = np.random.Generator(np.random.PCG64(200)).standard_normal((B * K, 9)).astype(np.float32)
        import scipy.integrate as si
        calls = {"n": 0}
        orig = si.solve_ivp

        def counting(fun, *a, **k):
            def f(t, y):
                calls["n"] += 1
                return fun(t, y)
            return orig(f, *a, **k)

        import networks.gf_algorithms.samplers as smp
        smp.integrate.solve_ivp = counting
        try:
            with NoiseFeed(prior, np.zeros((0,), np.float32)):
                pose, q, _, proc = agent.pred_func(d, repeat_num=K, T0=T0, return_average_res=True,
                                                   return_process=True)
        finally:
            smp.integrate.solve_ivp = orig
        out[f"{tag}_pts"] = d["pts"].numpy()
        out[f"{tag}_pts_center"] = d["pts_center"].numpy()
        out[f"{tag}_prior"] = prior
        out[f"{tag}_pred_pose"] = pose.numpy()
        out[f"{tag}_pred_q"] = q.numpy()
        out[f"{tag}_xs"] = proc.numpy()
        out[f"{tag}_nfev"] = np.int64(calls["n"])
        out[f"{tag}_T0"] = np.float64(T0)
        out[f"{tag}_steps"] = np.int64(-1 if steps is None else steps)
    np.savez_compressed(os.path.join(HERE, "golden_ode.npz"), **out)


def gen_pipeline(get_config, PoseNet):
    """score (PC) -> energy -> sort -> aggregate (clustering on/off) -> scale."""
    B, K, T = 4, 50, 20
    d, pose = gen_pc(get_config, PoseNet, "pc_k50_t20", 31, B, K, T, tile_every=0)
    pts_feat = d["pts_feat"]
    e_agent = make_agent(get_config, PoseNet, "energy", "pc", T)
    d2 = {"pts": d["pts"], "pts_center": d["pts_center"]}
    energy = e_agent.get_energy(d2, pose, T=1e-5, mode="test", extract_feature=True)

    from networks.reward import sort_poses_by_energy
    from utils.misc import average_quaternion_batch, get_rot_matrix
    from utils.transforms.rotation_conversions import matrix_to_quaternion, quaternion_to_matrix
    from sklearn.cluster import DBSCAN
    sorted_pose, sorted_energy = sort_poses_by_energy(pose, energy)
    keep = int(K * 0.4)
    out = dict(pts=d["pts"].numpy(), pts_center=d["pts_center"].numpy(), pred_pose=pose.numpy(),
               energy=energy.numpy(), sorted_pose=sorted_pose.numpy(),
               sorted_energy=sorted_energy.numpy(), pts_feat=pts_feat.numpy())
    for clustering in (0, 1):
        good = sorted_pose[:, :keep, :]
        rm = get_rot_matrix(good[:, :, :-3].reshape(B * keep, -1), "rot_matrix")
        qw = matrix_to_quaternion(rm).reshape(B, keep, -1)
        agg_q = average_quaternion_batch(qw)
        if clustering:
            for j in range(B):
                D = 1 - torch.sum(qw[j].unsqueeze(0) * qw[j].unsqueeze(1), dim=2) ** 2
                labels = DBSCAN(eps=0.05, min_samples=int(0.1667 * keep)).fit(D.numpy()).labels_
                if np.any(labels >= 0):
                    best = np.argmax(np.bincount(labels[labels >= 0]))
                    agg_q[j] = average_quaternion_batch(qw[j, labels == best].unsqueeze(0))[0]
                out[f"labels_{j}"] = labels
        agg = torch.zeros(B, 4, 4)
        agg[:, 3, 3] = 1
        agg[:, :3, :3] = quaternion_to_matrix(agg_q)
        agg[:, :3, 3] = torch.mean(good[:, :, -3:], dim=1)
        out[f"aggregated_c{clustering}"] = agg.numpy()
    # clustered candidate sets (untrained weights give no clusters): exercises DBSCAN (F9)
    rng = np.random.Generator(np.random.PCG64(300))
    from utils.misc import get_pose_representation
    base = [torch.from_numpy(synthetic._random_rotation(rng)).float() for _ in range(3)]
    cl_pose = torch.zeros(B, K, 9)
    for j in range(B):
        for k in range(K):
            c = base[(k * (j + 1)) % 3] if k % 5 else base[0]
            noise = torch.from_numpy(synthetic._random_rotation(rng)).float()
            w = 0.02 * (1 + j)
            Rk = c @ (torch.eye(3) * (1 - w) + noise * w)
            cl_pose[j, k, :6] = get_pose_representation(Rk[None], "rot_matrix")[0]
            cl_pose[j, k, 6:] = torch.from_numpy(rng.normal(size=3)).float()
    cl_energy = torch.from_numpy(rng.normal(size=(B, K, 2)).astype(np.float32))
    sp, _ = sort_poses_by_energy(cl_pose, cl_energy)
    good = sp[:, :keep, :]
    rm = get_rot_matrix(good[:, :, :-3].reshape(B * keep, -1), "rot_matrix")
    qw = matrix_to_quaternion(rm).reshape(B, keep, -1)
    agg_q = average_quaternion_batch(qw)
    for j in range(B):
        D = 1 - torch.sum(qw[j].unsqueeze(0) * qw[j].unsqueeze(1), dim=2) ** 2
        labels = DBSCAN(eps=0.05, min_samples=int(0.1667 * keep)).fit(D.numpy()).labels_
        if np.any(labels >= 0):
            best = np.argmax(np.bincount(labels[labels >= 0]))
            agg_q[j] = average_quaternion_batch(qw[j, labels == best].unsqueeze(0))[0]
        out[f"cl_labels_{j}"] = labels
    agg = torch.zeros(B, 4, 4)
    agg[:, 3, 3] = 1
    agg[:, :3, :3] = quaternion_to_matrix(agg_q)
    agg[:, :3, 3] = torch.mean(good[:, :, -3:], dim=1)
    out.update(cl_pose=cl_pose.numpy(), cl_energy=cl_energy.numpy(), cl_aggregated=agg.numpy())

    s_agent = make_agent(get_config, PoseNet, "scale", "pc", T)
    axes = torch.from_numpy(out["aggregated_c1"][:, :3, :3].copy())
    _, length = s_agent.pred_scale_func({"pts_feat": pts_feat, "rgb_feat": None, "axes": axes})
    out["scale_axes"] = axes.numpy()
    out["scale_length"] = length.numpy()
    np.savez_compressed(os.path.join(HERE, "golden_pipeline.npz"), **out)


def gen_tracking(get_config, PoseNet):
    """Warm start as runners/evaluation_tracking.py:110-127 calls it: init_x = previous pose with
    pts_center subtracted from its translation, small T0. PC uses init_x as-is
    and ignores T0 (posenet.py:241-253); ODE starts at prior(sigma(T0)) + init_x (samplers.py:197-201)."""
    from utils.misc import get_pose_representation
    B, K, T, T0 = 2, 5, 20, 0.2
    d = batch(41, B, 1024)
    rng = np.random.Generator(np.random.PCG64(400))
    prev = torch.zeros(B, 9)
    for j in range(B):
        Rj = torch.from_numpy(synthetic._random_rotation(rng)).float()
        prev[j, :6] = get_pose_representation(Rj[None], "rot_matrix")[0]
        prev[j, 6:] = d["pts_center"][j] + torch.from_numpy(rng.normal(scale=0.01, size=3)).float()
    init_x = prev.clone()
    init_x[:, -3:] -= d["pts_center"]
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    zs = rng.standard_normal((2 * T, B * K, 9)).astype(np.float32)
    out = dict(pts=d["pts"].numpy(), pts_center=d["pts_center"].numpy(), init_x=init_x.numpy(),
               prior=prior, z1=zs[0::2], z2=zs[1::2], K=K, T=T, T0=T0)
    agent = make_agent(get_config, PoseNet, "score", "pc", T)
    with NoiseFeed(prior, zs) as nf:
        pose, q = agent.pred_func(dict(d), repeat_num=K, T0=T0, init_x=init_x.clone())
        assert nf.i == 2 * T
    out.update(pc_pred_pose=pose.numpy(), pc_pred_q=q.numpy())
    agent = make_agent(get_config, PoseNet, "score", "ode", None)
    import scipy.integrate as si
    calls = {"n": 0}
    orig = si.solve_ivp

    def counting(fun, *a, **k):
        def f(t, y):
            calls["n"] += 1
            return fun(t, y)
        return orig(f, *a, **k)

    import networks.gf_algorithms.samplers as smp
    smp.integrate.solve_ivp = counting
    try:
        with NoiseFeed(prior, np.zeros((0,), np.float32)):
            pose, q = agent.pred_func(dict(d), repeat_num=K, T0=T0, init_x=init_x.clone())
    finally:
        smp.integrate.solve_ivp = orig
    out.update(ode_pred_pose=pose.numpy(), ode_pred_q=q.numpy(), ode_nfev=np.int64(calls["n"]))
    np.savez_compressed(os.path.join(HERE, "golden_tracking.npz"), **out)


def gen_ckpt_layout(get_config, PoseNet):
    """The structure of a checkpoint written by the reference's own PoseNet.save_ckpt
    (posenet_agent.py:141-169) for each agent type: top-level keys, every model_state_dict key with
    shape and dtype, the optimizer/scheduler state keys and the clock. Written to a scratch dir, loaded
    back with torch.load(weights_only=True) (what the build's load_ckpt does), summarised as JSON."""
    import json
    import tempfile
    from networks.gf_algorithms.score_utils import ExponentialMovingAverage
    out = {}
    for kind in ("score", "energy", "scale"):
        agent = make_agent(get_config, PoseNet, kind, "pc", 20)
        # save_ckpt writes the EMA shadow weights: restart the EMA from the loaded weights
        agent.ema = ExponentialMovingAverage(agent.net.parameters(), decay=agent.cfg.ema_rate)
        with tempfile.TemporaryDirectory() as tmp:
            agent.model_dir = tmp
            agent.save_ckpt("latest")
            ck = torch.load(os.path.join(tmp, "latest.pth"), map_location="cpu", weights_only=True)
        sd = ck["model_state_dict"]
        mine = weights.synthetic_state_dict(kind, seed=0)
        same = all(np.array_equal(sd[k].numpy(), mine[k]) for k in mine)
        out[kind] = {
            "top_level_keys": sorted(ck),
            "model_state_dict": {k: [list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()},
            "optimizer_state_dict_keys": sorted(ck["optimizer_state_dict"]),
            "scheduler_state_dict_keys": sorted(ck["scheduler_state_dict"]),
            "clock": ck["clock"],
            "weights_equal_synthetic": bool(same),
        }
    with open(os.path.join(HERE, "golden_ckpt_layout.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else None      # e.g. "tracking": that fixture only
    get_config, PoseNet = import_reference("pc", 20)
    if only == "tracking":
        gen_tracking(get_config, PoseNet)
        print("tracking done")
        return
    if only == "ckpt":
        gen_ckpt_layout(get_config, PoseNet)
        print("ckpt layout done")
        return
    gen_encoder(get_config, PoseNet)
    print("encoder done")
    gen_heads(get_config, PoseNet)
    print("heads done")
    gen_pc(get_config, PoseNet, "pc_k10_t100", 1, 4, 10, 100)
    print("pc done")
    gen_pipeline(get_config, PoseNet)
    print("pipeline done")
    gen_ode(get_config, PoseNet)
    print("ode done")


if __name__ == "__main__":
    main()
