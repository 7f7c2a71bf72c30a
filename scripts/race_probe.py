"""Diagnostic for the round-4 one-off multirank mismatch (r4zi): is any stage of the evaluation
pipeline non-deterministic when fresh agents run on recycled device memory while other processes
share the GPU?

Every worker process (all on cuda:0) repeats, REPS times:
  garbage-fill and free 3 x 256 MB of device memory (NaN, 3e38, -1),
  build a fresh EvaluationPipeline (seed-0 synthetic weights, the score agent re-loaded from a seed-7
  reference-format checkpoint, as test_gpu_multirank does on rank 0),
  run it on its object block with the stages split out by hand (EvaluationPipeline.run's order and
  streams: one geometry pass, score encoder, energy encoder on a side stream beside the PC sampler),
and compares every stage with its first repetition bit for bit. Worker 0 takes objects 0..2 and
worker 1 objects 3..4 of the test's 5-object batch; extra workers run a B=256, K=50, T=100 pipeline
as load. Prints one line per (worker, repetition) naming the stages that differ.

usage: python scripts/race_probe.py [--procs 3] [--reps 20] [--out gpurun_out/race.json]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

DEV = "cuda:0"
STAGES = ("score_feat", "energy_feat", "pobj", "pred_pose", "energy", "aggregated", "length")


def _cfg(seed, steps=20, K=20):
    from genpose2_amd.config import GenPoseConfig
    return GenPoseConfig(device=DEV, sampling_steps=steps, eval_repeat_num=K, noise_seed=4, seed=seed)


def garbage():
    bufs = [torch.full((64 << 20,), v, device=DEV) for v in (float("nan"), 3e38, -1.0)]
    torch.cuda.synchronize()
    del bufs


def run_stages(pipe, batch):
    """EvaluationPipeline.run with the intermediates kept (same calls, same streams)."""
    from genpose2_amd import aggregate
    cfg = pipe.cfg
    sa, ea, sc = pipe.score_agent, pipe.energy_agent, pipe.scale_agent
    data = dict(batch)
    main = torch.cuda.current_stream(batch["pts"].device)
    side = pipe._side = pipe._side or torch.cuda.Stream(device=batch["pts"].device)
    edata = {k: batch[k] for k in ("pts", "pts_center")}
    sa.encode_geometry(data)
    edata["enc_geometry"] = data["enc_geometry"]

    def start():
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ea.encode_func(edata)
    sa.after_encode = start
    try:
        pred_pose, _ = sa.pred_func(data=data, repeat_num=cfg.eval_repeat_num, T0=cfg.T0)
    finally:
        sa.after_encode = None
    main.wait_stream(side)
    edata["pts_feat"].record_stream(main)
    energy = ea.get_energy(data=edata, pose_samples=pred_pose, T=1e-5, mode="test", extract_feature=False)
    agg = aggregate.aggregate_pose(pred_pose, energy, cfg.retain_ratio, cfg.clustering, cfg.clustering_eps,
                                   cfg.clustering_minpts, retain_num=int(cfg.eval_repeat_num * cfg.retain_ratio))
    _, length = sc.pred_scale_func({"pts_feat": data["pts_feat"], "rgb_feat": None,
                                    "axes": agg[:, :3, :3].contiguous()})
    pobj = sa.heads.object_proj(data["pts_feat"])
    out = {"score_feat": data["pts_feat"], "energy_feat": edata["pts_feat"], "pobj": pobj, "pred_pose": pred_pose,
           "energy": energy, "aggregated": agg, "length": length}
    return {k: v.detach().cpu().numpy().copy() for k, v in out.items()}


def worker(w, nprocs, reps, ckpt, outdir):
    from genpose2_amd import synthetic
    from genpose2_amd.runner import EvaluationPipeline
    torch.cuda.set_device(0)
    if w < 2:
        pts, center = synthetic.make_batch(12, 5, 1024)
        lo, hi = (0, 3) if w == 0 else (3, 5)
        steps, K = 20, 20
    else:   # load: B=256, K=50, T=100
        pts, center = synthetic.make_batch(2, 256, 1024)
        lo, hi = 0, 256
        steps, K = 100, 50
    batch = {"pts": torch.from_numpy(pts[lo:hi].copy()).to(DEV), "pts_center": torch.from_numpy(center[lo:hi].copy()).to(DEV)}
    first = None
    log = []
    for r in range(reps):
        garbage()
        pipe = EvaluationPipeline(_cfg(0, steps, K), with_scale=True)
        if w < 2:
            pipe.score_agent.load_ckpt(model_dir=ckpt, model_path=True, load_model_only=True)
        out = run_stages(pipe, batch)
        del pipe
        if first is None:
            first = out
            diff = []
        else:
            diff = [k for k in STAGES if not np.array_equal(out[k], first[k], equal_nan=True)]
        rec = {"worker": w, "rep": r, "differ": diff,
               "maxdiff": {k: float(np.nanmax(np.abs(out[k].astype(np.float64) - first[k]))) for k in diff},
               "objects": {k: [int(i) for i in range(out[k].shape[0]) if not np.array_equal(out[k][i], first[k][i], equal_nan=True)]
                           for k in diff}}
        print(json.dumps(rec), flush=True)
        log.append(rec)
        if diff and w < 2:
            np.savez(os.path.join(outdir, f"race_w{w}_r{r}.npz"), **{f"first_{k}": first[k] for k in STAGES},
                     **{f"got_{k}": out[k] for k in STAGES})
    with open(os.path.join(outdir, f"race_w{w}.json"), "w") as f:
        json.dump(log, f)


def sharded_worker(rank, world, port, reps, ckpt, outdir, total):
    """test_gpu_multirank's worker, repeated: ranks build agents from different seeds, rank 0 alone loads the
    checkpoint, ShardedEvaluationPipeline broadcasts over gloo and gathers; rank 0 compares every repetition's
    gathered outputs with its first."""
    import torch.distributed as dist
    from genpose2_amd import synthetic
    from genpose2_amd.runner import ShardedEvaluationPipeline
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    pts, center = synthetic.make_batch(12, total, 1024)
    batch = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
    first, log = None, []
    keys = ("pred_pose", "pts_feat", "energy", "aggregated", "length")
    try:
        for r in range(reps):
            garbage()
            pipe = ShardedEvaluationPipeline(_cfg(seed=0 if rank == 0 else 99), with_scale=True)
            pipe.load_ckpt(score=ckpt if rank == 0 else "/nonexistent/on/this/rank.pth")
            got = pipe.run(batch)
            out = {k: getattr(got, k).cpu().numpy().copy() for k in keys}
            del pipe, got
            if rank == 0:
                if first is None:
                    first = out
                    np.savez(os.path.join(outdir, "race_sharded_first.npz"), **first)
                diff = [k for k in keys if not np.array_equal(out[k], first[k], equal_nan=True)]
                rec = {"rep": r, "differ": diff,
                       "objects": {k: [int(i) for i in range(out[k].shape[0])
                                       if not np.array_equal(out[k][i], first[k][i], equal_nan=True)] for k in diff}}
                print(json.dumps(rec), flush=True)
                log.append(rec)
                if diff:
                    np.savez(os.path.join(outdir, f"race_sharded_r{r}.npz"), **out)
            dist.barrier()
        if rank == 0:
            with open(os.path.join(outdir, "race_sharded.json"), "w") as f:
                json.dump(log, f)
    finally:
        dist.destroy_process_group()


def load_worker(kind, seconds):
    """Background load on the same GPU for `seconds`: 'matmul' (bf16 GEMMs: MFMA-bound), 'mem' (512 MB
    copies: HBM-bound), 'pipeline' (B=256, K=50, T=100 evaluation pipelines: this library's kernels)."""
    t_end = time.time() + seconds
    if kind == "matmul":
        a = torch.randn(8192, 8192, device=DEV, dtype=torch.bfloat16)
        while time.time() < t_end:
            for _ in range(20):
                a = (a @ a).clamp_(-1, 1)
            torch.cuda.synchronize()
    elif kind == "mem":
        x = torch.empty(128 << 20, device=DEV)
        y = torch.empty_like(x)
        while time.time() < t_end:
            for _ in range(20):
                y.copy_(x)
            torch.cuda.synchronize()
    else:
        from genpose2_amd import synthetic
        from genpose2_amd.runner import EvaluationPipeline
        pts, center = synthetic.make_batch(2, 256, 1024)
        batch = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
        pipe = EvaluationPipeline(_cfg(0, 100, 50), with_scale=True)
        while time.time() < t_end:
            pipe.run(batch)
            torch.cuda.synchronize()


def levels_worker(w, nprocs, reps, outdir, geom, load="none", nprobe=4, barrier=None):
    if w >= nprobe:
        torch.cuda.set_device(0)
        load_worker(load, float(os.environ.get("RACE_LOAD_SECONDS", "40")))
        return
    """The Light encoder alone, repeated on recycled memory while the other workers do the same: every
    level's FPS indices, centroids, ball lists and features are compared with the first repetition, so the
    first item that differs names the kernel. Even workers encode 3 objects, odd ones 256."""
    from genpose2_amd import device as dev, synthetic, weights
    torch.cuda.set_device(0)
    B = 3 if w % 2 == 0 else 256
    pts, _ = synthetic.make_batch(12, B, 1024)
    pts = torch.from_numpy(pts).to(DEV)
    enc = dev.EncoderModel(weights.synthetic_state_dict("score", seed=7), torch.device(DEV))
    enc.set_arith(os.environ.get("RACE_ENC_ARITH", "split_f16"))
    first, log = None, []
    for r in range(reps):
        garbage()
        enc._ws = None
        if barrier is not None:   # every probe worker encodes at the same moment
            torch.cuda.synchronize()
            barrier.wait()
        if geom:
            g = enc.geometry(pts)
            feat, ws = enc.forward(pts, return_workspace=True, geometry=g)
        else:
            feat, ws = enc.forward(pts, return_workspace=True)
        lv = enc.levels(B, 1024, ws)
        out = {"feat": feat.cpu().numpy().copy()}
        for i, d in enumerate(lv):
            for k, v in d.items():
                if isinstance(v, list):
                    for j, t in enumerate(v):
                        out[f"l{i}_{k}{j}"] = t.cpu().numpy().copy()
                else:
                    out[f"l{i}_{k}"] = v.cpu().numpy().copy()
        if first is None:
            first = out
        order = [k for k in out]   # levels in order, geometry before features within a level
        diff = [k for k in order if not np.array_equal(out[k], first[k], equal_nan=True)]
        rec = {"worker": w, "B": B, "rep": r, "differ": diff,
               "objects": {k: [int(i) for i in range(out[k].shape[0]) if not np.array_equal(out[k][i], first[k][i], equal_nan=True)]
                           for k in diff[:3]}}
        if diff:
            k = diff[0]
            a, b = out[k].reshape(out[k].shape[0], -1), first[k].reshape(out[k].shape[0], -1)
            bad = np.argwhere(a != b)
            rec["first_item"] = k
            rec["n_elems"] = int(len(bad))
            rec["elems"] = bad[:8].tolist()
            rec["maxdiff"] = float(np.nanmax(np.abs(a.astype(np.float64) - b)))
            for k in [k for k in diff if k.endswith("_features")][:1]:
                a, b = out[k], first[k]          # (B, M, C)
                bad = np.argwhere(a != b)
                rec["level_item"] = k
                rec["level_channels"] = np.bincount(bad[:, 2], minlength=a.shape[2]).tolist()
                rec["level_centroids"] = int(len({(int(x), int(y)) for x, y, _ in bad}))
                rec["level_centroid_list"] = sorted({(int(x), int(y)) for x, y, _ in bad})[:20]
                rec["level_maxdiff"] = float(np.abs(a.astype(np.float64) - b).max())
                if B <= 8 and sum(1 for x in log if x["differ"]) < 3:
                    np.savez(os.path.join(outdir, f"race_levels_w{w}_r{r}.npz"), got=a, first=b)
        print(json.dumps(rec), flush=True)
        log.append(rec)
    with open(os.path.join(outdir, f"race_levels_w{w}.json"), "w") as f:
        json.dump(log, f)


def level0_worker(w, nprocs, reps, outdir, inner=5, into_ws=False, on_device=False, poison=False):
    """Level 0 alone (gp_sa_level: ball query, per-point projection Q0, the narrow MLP kernel), INNER times per
    repetition on a fresh workspace: Q0, both ball lists and the level-0 features compared bit for bit with the
    first call, so a difference names the stage (inputs vs the MLP kernel)."""
    import ctypes
    from genpose2_amd import _lib, device as dev, synthetic, weights
    torch.cuda.set_device(0)
    B = 3 if w % 2 == 0 else 256
    N = 1024
    pts, _ = synthetic.make_batch(12, B, N)
    pts = torch.from_numpy(pts).to(DEV)
    enc = dev.EncoderModel(weights.synthetic_state_dict("score", seed=7), torch.device(DEV))
    lib = _lib.load()
    plib = ctypes.CDLL(os.path.join(REPO, "scripts", "libpoison.so")) if poison else None
    off = np.zeros(25, np.int64)
    lib.gp_encoder_workspace_layout(B, N, off.ctypes.data_as(_lib.c_int64_p))
    q0_bytes = B * N * 48 * 4
    # proj[0] follows feat[0..4] in the layout: its offset is the end of feat[4] rounded up to 256
    q0_off = (int(off[4 * 5 + 4]) + B * 1024 * 4 + 255) // 256 * 256
    first, log = None, []
    for r in range(reps):
        garbage()
        enc._ws = None
        ws = enc.workspace(B, N)
        feat0 = ws[int(off[4]):].view(torch.float32)[: B * 512 * 96].view(B, 512, 96) if into_ws else \
            torch.empty(B, 512, 96, device=DEV)
        lib.gp_encoder_fps(ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                           ctypes.c_void_p(dev.stream_handle(torch.device(DEV))))
        for k in range(inner):
            if poison:   # junk in every CU's LDS and every SIMD's registers before the call (scripts/poison.hip)
                plib.poison_gpu(ctypes.c_uint32(r * 7919 + k * 104729 + w), 2048, ctypes.c_void_p(dev.stream_handle(torch.device(DEV))))
            _lib.check(lib.gp_sa_level(ctypes.c_void_p(enc.wbuf.data_ptr()), enc.offsets.ctypes.data_as(_lib.c_int64_p), 0, 0,
                                       ctypes.c_void_p(pts.data_ptr()), B, N, None, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                       ctypes.c_void_p(feat0.data_ptr()), ctypes.c_void_p(dev.stream_handle(torch.device(DEV)))))
            out = {"q0": ws[q0_off:q0_off + q0_bytes].view(torch.float32).view(B, N, 48),
                   "ball0": ws[int(off[2]):].view(torch.int32)[: B * 512 * 16],
                   "ball1": ws[int(off[3]):].view(torch.int32)[: B * 512 * 32],
                   "cent": ws[int(off[1]):].view(torch.float32)[: B * 512 * 3],
                   "feat0": feat0}
            if on_device:   # compared on the device: no host round trip between calls
                out = {n: v.clone() for n, v in out.items()}
                if first is None:
                    first = out
                diff = [n for n in out if not torch.equal(out[n], first[n])]
                if diff:
                    out = {n: v.cpu().numpy() for n, v in out.items()}
                    first_np = {n: v.cpu().numpy() for n, v in first.items()}
            else:
                out = {n: v.cpu().numpy().copy() for n, v in out.items()}
                if first is None:
                    first = out
                diff = [n for n in out if not np.array_equal(out[n], first[n], equal_nan=True)]
                first_np = first
            rec = {"worker": w, "B": B, "rep": r, "call": k, "differ": diff}
            if diff:
                a, b = out[diff[0]], first_np[diff[0]]
                rec["n_elems"] = int((a != b).sum())
                if "feat0" in diff:
                    bad = np.argwhere(out["feat0"] != first_np["feat0"])
                    rec["feat_objects"] = sorted({int(x) for x in bad[:, 0]})[:20]
                    rec["feat_branch_a"] = int((bad[:, 2] < 32).sum())
                    rec["feat_branch_b"] = int((bad[:, 2] >= 32).sum())
                    rec["feat_maxdiff"] = float(np.abs(out["feat0"].astype(np.float64) - first_np["feat0"]).max())
                    if sum(1 for x in log if x["differ"]) < 4:
                        np.savez(os.path.join(outdir, f"race_level0_w{w}_r{r}_c{k}.npz"), **{f"got_{n}": v for n, v in out.items()},
                                 **{f"first_{n}": v for n, v in first_np.items()})
                print(json.dumps(rec), flush=True)
            log.append(rec)
    with open(os.path.join(outdir, f"race_level0_w{w}.json"), "w") as f:
        json.dump(log, f)


def snap_worker(w, nprocs, reps, outdir):
    """The Light encoder level by level (gp_encoder_fps, then gp_sa_level 0..4 into the workspace's own level
    buffers, as gp_encoder_forward_geom runs them), with every level's features -- and every EARLIER level's
    features again -- copied out right after each level: the first (level, snapshot) that differs from the
    first repetition separates a level computing a wrong value from a later kernel overwriting it."""
    import ctypes
    from genpose2_amd import _lib, arch, device as dev, synthetic, weights
    torch.cuda.set_device(0)
    B = 3 if w % 2 == 0 else 256
    N = 1024
    pts, _ = synthetic.make_batch(12, B, N)
    pts = torch.from_numpy(pts).to(DEV)
    enc = dev.EncoderModel(weights.synthetic_state_dict("score", seed=7), torch.device(DEV))
    lib = _lib.load()
    off = np.zeros(25, np.int64)
    lib.gp_encoder_workspace_layout(B, N, off.ctypes.data_as(_lib.c_int64_p))
    couts = [arch.level_out_channels(lv) for lv in range(5)]
    ms = [arch.NPOINTS[lv] if lv < 4 else 1 for lv in range(5)]
    st = ctypes.c_void_p(dev.stream_handle(torch.device(DEV)))
    first, log = None, []
    for r in range(reps):
        garbage()
        enc._ws = None
        ws = enc.workspace(B, N)
        feat4 = torch.empty(B, 1024, device=DEV)
        _lib.check(lib.gp_encoder_fps(ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()), ws.numel(), st))
        views = [ws[int(off[lv * 5 + 4]):].view(torch.float32)[: B * ms[lv] * couts[lv]] for lv in range(4)] + [feat4.view(-1)]
        if os.environ.get("SNAP_SENTINEL") == "1":   # Q0's buffer set to NaN first: a projection that never lands shows
            q0o = (int(off[4 * 5 + 4]) + B * 1024 * 4 + 255) // 256 * 256
            ws[q0o:q0o + B * N * 48 * 4].view(torch.float32).fill_(float("nan"))
        snaps = {}
        for lv in range(5):
            prev = views[lv - 1] if lv else None
            _lib.check(lib.gp_sa_level(ctypes.c_void_p(enc.wbuf.data_ptr()), enc.offsets.ctypes.data_as(_lib.c_int64_p), lv,
                                       couts[lv - 1] if lv else 0, ctypes.c_void_p(pts.data_ptr()), B, N,
                                       ctypes.c_void_p(prev.data_ptr()) if lv else None, ctypes.c_void_p(ws.data_ptr()),
                                       ws.numel(), ctypes.c_void_p(views[lv].data_ptr()), st))
            if lv == 0:   # level 0's inputs as the MLP saw them (Q0 is reused by level 1 for its row maxima)
                q0_off = (int(off[4 * 5 + 4]) + B * 1024 * 4 + 255) // 256 * 256
                snaps["after0_pts"] = pts.clone()   # the input itself, after the level-0 kernels read it
                snaps["after0_q0"] = ws[q0_off:q0_off + B * N * 48 * 4].clone()
                snaps["after0_ball0"] = ws[int(off[2]):int(off[2]) + B * 512 * 16 * 4].clone()
                snaps["after0_ball1"] = ws[int(off[3]):int(off[3]) + B * 512 * 32 * 4].clone()
                snaps["after0_cent"] = ws[int(off[1]):int(off[1]) + B * 512 * 3 * 4].clone()
            for k in range(lv + 1):
                snaps[f"after{lv}_l{k}"] = views[k].clone()   # kept on the device: compared there
        torch.cuda.synchronize()
        if first is None:
            first = snaps
        diff = [k for k in snaps if not torch.equal(snaps[k], first[k])]
        rec = {"worker": w, "B": B, "rep": r, "differ": diff}
        if "after0_q0" in diff:
            # where Q0 differs: level 1 later writes its per-point row maxima over the first B*512 floats of
            # this buffer, so a stale Q0 from the previous repetition differs exactly there
            qa = snaps["after0_q0"].view(torch.float32).cpu().numpy()
            qf = first["after0_q0"].view(torch.float32).cpu().numpy()
            bad = np.nonzero(qa != qf)[0]
            rec["q0_n"] = int(len(bad))
            rec["q0_first_last"] = [int(bad.min()), int(bad.max())]
            rec["q0_in_rowmax_region"] = int((bad < B * 512).sum())
            rec["q0_nan"] = int(np.isnan(qa).sum())
            rec["q0_got_sample"] = [float(v) for v in qa[bad[:6]]]
            rec["q0_first_sample"] = [float(v) for v in qf[bad[:6]]]
            # per differing point row: which 16-float blocks, and whether the bad block equals the same block of
            # another point's correct row (a wrong source point) -- and which
            QA, QF = qa.reshape(B * N, 3, 16), qf.reshape(B * N, 3, 16)
            rows = sorted({int(i) // 48 for i in bad})
            info = []
            for p in rows[:12]:
                blks = [k for k in range(3) if not np.array_equal(QA[p, k], QF[p, k])]
                src = []
                for k in blks:
                    hit = np.nonzero((QF[:, k] == QA[p, k]).all(1))[0]
                    src.append(int(hit[0]) if len(hit) else -1)
                info.append([p, blks, src])
            rec["q0_rows"] = info
            if B <= 8 and sum(1 for x in log if x["differ"]) < 3:
                np.savez(os.path.join(outdir, f"race_snap_q0_w{w}_r{r}.npz"), got=qa, first=qf)
        if "after0_ball0" in diff:   # which centroids' lists changed, and how
            ga = snaps["after0_ball0"].view(torch.int32).view(B, 512, 16).cpu().numpy()
            gf = first["after0_ball0"].view(torch.int32).view(B, 512, 16).cpu().numpy()
            rows = np.argwhere((ga != gf).any(-1))
            rec["ball0_rows"] = int(len(rows))
            rec["ball0_first_rows"] = rows[:8].tolist()
            rec["ball0_got_first"] = [[ga[tuple(r)].tolist(), gf[tuple(r)].tolist()] for r in rows[:3]]
            # per object: the points in one list but not the other, over all its differing rows
            moved = {}
            for bb, mm in rows:
                d = set(ga[bb, mm].tolist()) ^ set(gf[bb, mm].tolist())
                moved.setdefault(int(bb), set()).update(int(x) for x in d)
            rec["ball0_moved_points"] = {k: sorted(v)[:24] for k, v in list(moved.items())[:12]}
        if "after0_pts" in diff:
            pa = snaps["after0_pts"].cpu().numpy().reshape(-1)
            pf = first["after0_pts"].cpu().numpy().reshape(-1)
            bad = np.nonzero(pa != pf)[0]
            rec["pts_bad_floats"] = bad[:32].tolist()
            rec["pts_got"] = pa[bad[:8]].tolist()
            rec["pts_first"] = pf[bad[:8]].tolist()
        if "after0_l0" in diff:
            a0 = snaps["after0_l0"].view(B, 512, 96).cpu().numpy()
            f0 = first["after0_l0"].view(B, 512, 96).cpu().numpy()
            bad = np.argwhere(a0 != f0)
            rec["l0_objects"] = sorted({int(x) for x in bad[:, 0]})[:20]
            rec["l0_branch_a"] = int((bad[:, 2] < 32).sum())
            rec["l0_branch_b"] = int((bad[:, 2] >= 32).sum())
            rec["l0_maxdiff"] = float(np.abs(a0.astype(np.float64) - f0).max())
        print(json.dumps(rec), flush=True)
        log.append(rec)
    with open(os.path.join(outdir, f"race_snap_w{w}.json"), "w") as f:
        json.dump(log, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fresh", choices=("fresh", "sharded", "levels", "levels_geom", "level0", "level0_ws", "level0_dev", "level0_ws_dev", "level0_poison", "snap"))
    ap.add_argument("--procs", type=int, default=3)
    ap.add_argument("--sync", action="store_true", help="levels modes: probe workers start each repetition together")
    ap.add_argument("--load", default="none", choices=("none", "matmul", "mem", "pipeline"))
    ap.add_argument("--nprobe", type=int, default=None, help="levels modes: workers running the probe (the rest: --load)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--outdir", default=os.path.join(REPO, "gpurun_out"))
    args = ap.parse_args()
    import torch.multiprocessing as mp
    from conftest import write_reference_checkpoint
    os.makedirs(args.outdir, exist_ok=True)
    ckpt = write_reference_checkpoint(os.path.join(tempfile.mkdtemp(), "score.pth"), "score", seed=7)
    t0 = time.time()
    if args.mode == "snap":
        mp.spawn(snap_worker, args=(args.procs, args.reps, args.outdir), nprocs=args.procs, join=True)
        bad, firsts = 0, {}
        for w in range(args.procs):
            with open(os.path.join(args.outdir, f"race_snap_w{w}.json")) as f:
                for r in json.load(f):
                    if r["differ"]:
                        bad += 1
                        firsts[r["differ"][0]] = firsts.get(r["differ"][0], 0) + 1
        print(json.dumps({"mode": "snap", "procs": args.procs, "reps": args.reps, "differing_reps": bad,
                          "first_differing_snapshot": firsts, "lib": os.environ.get("GENPOSE_HIP_LIB", "default"),
                          "seconds": time.time() - t0}))
        return
    if args.mode.startswith("level0"):
        mp.spawn(level0_worker, args=(args.procs, args.reps, args.outdir, 5, "_ws" in args.mode, args.mode.endswith("_dev"),
                                      args.mode.endswith("_poison")), nprocs=args.procs, join=True)
        bad, stages = 0, {}
        for w in range(args.procs):
            with open(os.path.join(args.outdir, f"race_level0_w{w}.json")) as f:
                for r in json.load(f):
                    if r["differ"]:
                        bad += 1
                        stages[",".join(r["differ"])] = stages.get(",".join(r["differ"]), 0) + 1
        print(json.dumps({"mode": args.mode, "procs": args.procs, "reps": args.reps, "differing_calls": bad,
                          "stages": stages, "lib": os.environ.get("GENPOSE_HIP_LIB", "default"),
                          "seconds": time.time() - t0}))
        return
    if args.mode.startswith("levels"):
        nprobe = args.procs if args.nprobe is None else args.nprobe
        import multiprocessing
        barrier = multiprocessing.get_context("spawn").Barrier(nprobe) if args.sync else None
        mp.spawn(levels_worker, args=(args.procs, args.reps, args.outdir, args.mode == "levels_geom", args.load, nprobe,
                                      barrier), nprocs=args.procs, join=True)
        bad = {}
        nbad = 0
        for w in range(nprobe):
            with open(os.path.join(args.outdir, f"race_levels_w{w}.json")) as f:
                for r in json.load(f):
                    if r["differ"]:
                        bad[r["first_item"]] = bad.get(r["first_item"], 0) + 1
                        nbad += 1
        print(json.dumps({"mode": args.mode, "procs": args.procs, "nprobe": nprobe, "load": args.load, "sync": args.sync,
                          "lib": os.environ.get("GENPOSE_HIP_LIB", "default"), "reps": args.reps,
                          "differing_reps": nbad, "first_differing_item": bad,
                          "seconds": time.time() - t0}))
        return
    if args.mode == "sharded":
        from genpose2_amd import shard, synthetic
        from genpose2_amd.runner import EvaluationPipeline
        total, world = 5, 2
        port = 29300 + os.getpid() % 600
        mp.spawn(sharded_worker, args=(world, port, args.reps, ckpt, args.outdir, total), nprocs=world, join=True)
        # the test's per-shard reference, computed once in this process
        pts, center = synthetic.make_batch(12, total, 1024)
        batch = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}
        first = np.load(os.path.join(args.outdir, "race_sharded_first.npz"))
        parts = []
        for r in range(world):
            lo, hi = shard.shard_range(total, world, r)
            ref = EvaluationPipeline(_cfg(seed=0), with_scale=True)
            ref.score_agent.load_ckpt(model_dir=ckpt, model_path=True, load_model_only=True)
            parts.append(ref.run({k: v[lo:hi] for k, v in batch.items()}))
        vs = {k: [int(i) for i in range(total) if not np.array_equal(
            torch.cat([getattr(p, k) for p in parts]).cpu().numpy()[i], first[k][i])] for k in first.files}
        with open(os.path.join(args.outdir, "race_sharded.json")) as f:
            bad = sum(1 for r in json.load(f) if r["differ"])
        print(json.dumps({"mode": "sharded", "reps": args.reps, "differing_reps": bad,
                          "first_rep_vs_single_process_reference": vs, "seconds": time.time() - t0}))
        return
    mp.spawn(worker, args=(args.procs, args.reps, ckpt, args.outdir), nprocs=args.procs, join=True)
    bad = 0
    for w in range(min(args.procs, 2)):
        with open(os.path.join(args.outdir, f"race_w{w}.json")) as f:
            bad += sum(1 for r in json.load(f) if r["differ"])
    print(json.dumps({"procs": args.procs, "reps": args.reps, "differing_reps": bad, "seconds": time.time() - t0}))


if __name__ == "__main__":
    main()
