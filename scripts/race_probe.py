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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fresh", choices=("fresh", "sharded", "levels", "levels_geom"))
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
