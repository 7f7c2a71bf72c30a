"""Benchmark: pose candidates/s (B objects x K candidates x T denoise steps) on MI355X.

One "step" = one pass of the pose-candidate path over one batch of synthetic objects resident in
HBM. Default (--config 4): the north-star shape, i.e. one GPU's shard of BASELINE config 4 --
B=256 objects/GPU, N=1024 points, K=50 candidates, T=500 PC steps, ScoreNet encoder + sampler,
EnergyNet encoder + energy, ranking + aggregation (runners/evaluation_single.py:78-219 per batch).
--config 2 is ScoreNet only at B=64, --config 3 adds EnergyNet at B=64, --config 5 is the B=256,
N=2048, K=100, T=1000 + ScaleNet stress case. PC runs also time the shipped ODE sampler
(T0=0.55) on the same objects and report it under "ode".

Multi-GPU: one process per GPU (torchrun), objects sharded (weak scaling: B objects per GPU),
packed weights broadcast once from rank 0 over RCCL, no collective on the timed data path.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    2: dict(B=64, N=1024, K=50, T=500, energy=False, scale=False),
    3: dict(B=64, N=1024, K=50, T=500, energy=True, scale=False),
    4: dict(B=256, N=1024, K=50, T=500, energy=True, scale=False),   # per GPU of the 8-GPU B=2048 case
    5: dict(B=256, N=2048, K=100, T=1000, energy=False, scale=True),
}
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (and vector) peak
F16_PEAK_TFLOPS = 2516.6   # dense BF16/F16 MFMA: 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes/*/properties"


def count_gpus(env=None):
    """GPUs on this node, counted without any HIP call (the launcher must start its ranks before anything
    touches the GPU): amdsmi's processor handles, else the KFD topology nodes whose gfx_target_version is
    non-zero (CPU nodes report 0); capped by HIP/ROCR/CUDA_VISIBLE_DEVICES. None when neither source can
    be read -- the caller then refuses to launch rather than fall back to torch.cuda.device_count(),
    which calls hipGetDeviceCount in this process when amdsmi is unusable."""
    env = os.environ if env is None else env
    n = None
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        try:
            n = len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:   # not importable, no driver, or no permission: try the KFD topology
        n = None
    if not n:
        found = 0
        for fn in glob.glob(KFD_NODES):
            try:
                with open(fn) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        if k == "gfx_target_version" and int(v) != 0:
                            found += 1
            except (OSError, ValueError):
                continue
        n = found if found else n
    if n is None:
        return None
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if env.get(var):
            n = min(n, len([d for d in env[var].split(",") if d.strip()]))
    return n


def launch_command(argv, gpus, env, device_count, probe=False):
    """How `bench.py --gpus N` runs: None = in this process (N == 1, or already a rank of a launcher
    whose WORLD_SIZE equals N); otherwise the torchrun command that starts N ranks (one per GPU) as a
    CHILD process -- never an exec, and decided before anything touches the GPU. Raises when N GPUs
    are not there or a launcher's WORLD_SIZE disagrees with --gpus, so a 1-GPU box never reports a
    1-rank run as N GPUs."""
    if "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        if ws != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {gpus}")
        return None
    if gpus == 1:
        return None
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus}")
    if not probe and device_count < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but only {device_count} HIP device(s) are visible")
    port = 29000 + os.getpid() % 2000
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_probe(ws, rank):
    """--launch-probe: the launcher's rank plumbing without the GPU (gloo on CPU): every rank joins the
    group, the ranks' ids are summed, rank 0 prints one JSON line."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_probe": True, "n_gpus": ws, "rank_sum": int(t.item())}), flush=True)
    dist.destroy_process_group()


def broadcast_weights(agent, ws):
    """RCCL broadcast of the packed weights (device buffers + host layer tables) from rank 0."""
    if ws > 1:
        from genpose2_amd import shard
        shard.broadcast_agent(agent, src=0)


def cpu_info():
    """CPU model, physical cores and the CPUs this process may run on."""
    model, phys = "unknown", set()
    try:
        with open("/proc/cpuinfo") as f:
            pid = cid = None
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name":
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    cid = v
                elif not k and pid is not None:
                    phys.add((pid, cid))
                    pid = cid = None
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return model, len(phys) or avail, avail


def cpu_threads_default():
    """All physical cores this process may use, capped by the OMP_NUM_THREADS allotment when set. The GPU
    box exports OMP_NUM_THREADS=16: its 128 physical cores serve 8 GPUs, and a one-GPU job's fair share
    is 16 of them, so the baseline runs on that share rather than on cores other jobs on the host hold
    (--cpu-threads overrides)."""
    _, phys, avail = cpu_info()
    n = min(phys, avail)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(cfg, config_id, threads, sample_objects, reps=3):
    """Oracle ("port") timing per BASELINE.md §3: 1 warm-up run, then the median of `reps` runs of the
    SAME workload (every stage the GPU step runs: score encoder, T-step PC sampler with K candidates,
    and for full-pipeline configs the energy encoder + energy + ranking/aggregation, ScaleNet for
    config 5) on a bounded sample of `sample_objects` objects, so the default bench stays within
    minutes. Nothing is extrapolated in steps or candidates; per-object work is independent, so the
    rate (candidate-steps/s) is the sample's own. profiles/r2/cpu_full_vs_sample.json checks it
    against a full-batch run on the GPU host."""
    from genpose2_amd import synthetic, weights
    from oracle import oracle
    torch.set_num_threads(threads)
    Bs, N, K, T = min(sample_objects, cfg["B"]), cfg["N"], cfg["K"], cfg["T"]
    sd = weights.synthetic_state_dict("score")
    sd_e = weights.synthetic_state_dict("energy") if cfg["energy"] else None
    sd_s = weights.synthetic_state_dict("scale") if cfg["scale"] else None
    pts, center = synthetic.make_batch(config_id, Bs, N)
    rng = np.random.Generator(np.random.PCG64(0))
    prior = rng.standard_normal((Bs * K, 9), dtype=np.float32)
    z1 = rng.standard_normal((T, Bs * K, 9), dtype=np.float32)
    z2 = rng.standard_normal((T, Bs * K, 9), dtype=np.float32)

    def run():
        pose, _, feat, _ = oracle.pred_func(sd, pts, center, K, T, "pc", prior, z1, z2)
        axes = np.broadcast_to(np.eye(3, dtype=np.float32), (Bs, 3, 3))
        if sd_e is not None:
            e = oracle.get_energy(sd_e, pts, center, pose, 1e-5)
            axes = oracle.aggregate_pose(pose, e)[:, :3, :3]
        if sd_s is not None:
            oracle.scale_forward(sd_s, feat, np.ascontiguousarray(axes))

    t0 = time.perf_counter()
    run()
    warm = time.perf_counter() - t0
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    model, phys, avail = cpu_info()
    stages = "score encoder + PC sampler" + (" + energy encoder/eval + ranking/aggregation" if cfg["energy"] else "") \
        + (" + ScaleNet" if cfg["scale"] else "")
    out = {"value": Bs * K * T / med, "unit": "pose-candidate-steps/s", "cores": threads, "kind": "port",
           "sample": f"oracle (numpy fp32, the reference's unhoisted score form; sklearn DBSCAN) on {Bs} of the "
                     f"{cfg['B']} objects of config {config_id}, full K={K}, T={T} ({stages}); 1 warm-up "
                     f"({warm:.2f} s) + median of {reps}: {med:.2f} s (runs {', '.join(f'{t:.2f}' for t in ts)} s)",
           "cpu_model": model, "physical_cores": phys, "cpus_available": avail,
           "torch_threads": torch.get_num_threads(),
           "float32_matmul_precision": torch.get_float32_matmul_precision()}
    # the bounded sample against the whole batch, measured once on the GPU host (scripts/cpu_full_vs_sample.py)
    chk = os.path.join(REPO, "profiles", "r2", "cpu_full_vs_sample.json")
    if os.path.exists(chk) and config_id == 4:
        with open(chk) as f:
            c = json.load(f)
        out["full_batch_check"] = {"full_256_objects_value": c["full_256_objects"]["value"],
                                   "sample_16_objects_value": c["sample_16_objects"]["value"],
                                   "threads": c["threads"], "source": os.path.relpath(chk, REPO)}
    # the oracle/reference time ratio measured in the build container on identical
    # inputs (oracle/calibrate_cpu.py). It is a different thread count from this run's (the build
    # container has 8 CPUs; the reference cannot run on the GPU host), so it is reported beside the
    # port's rate, not applied to it.
    for cal in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "cpu_calibration.json")), reverse=True):
        with open(cal) as f:
            c = json.load(f)
        out["calibration_note"] = {"oracle_over_reference_time": round(c["oracle_over_reference"], 3),
                                   "threads": c["threads"], "source": os.path.relpath(cal, REPO),
                                   "applied": False,
                                   # the reference's own CPU rate this ratio implies (value is not changed by it)
                                   "reference_equivalent_value": out["value"] * c["oracle_over_reference"]}
        break
    return out


def rocprof_files(config, dino="none"):
    """Committed rocprofv3 --stats summaries of bench runs of `config` (profiles/r<round>/config<C>_*_kernel_stats.csv;
    DINO-pointwise runs: config<C>_pointwise_*), newest round first, then reverse lexical order within a round:
    deterministic on any checkout (no mtimes)."""
    import re
    out = []
    for fn in glob.glob(os.path.join(REPO, "profiles", "r*", f"config{config}_*kernel_stats.csv")):
        base = os.path.basename(fn)
        if ("_pointwise_" in base) != (dino == "pointwise"):
            continue
        m = re.fullmatch(r"r(\d+)", os.path.basename(os.path.dirname(fn)))
        if m:
            out.append((int(m.group(1)), base, fn))
    return [fn for _, _, fn in sorted(out, reverse=True)]


def load_rocprof(kernel, config, dino="none"):
    """Mean duration of `kernel` (its full instantiation name, e.g. "void pc_step_kernel<4, 8, 3>(...": 64-candidate
    tiles, 8 waves, f16x3 -- the plane count keeps it apart from the round-3 2-plane "<4, 8, true>") in the
    newest committed rocprofv3 --stats summary of a bench run of the same config (so the same row count and
    tile) that holds it, or None."""
    import csv
    for fn in rocprof_files(config, dino):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Name"].startswith(kernel):
                    return {"avg_launch_us": float(row["AverageNs"]) / 1e3, "calls": int(row["Calls"]),
                            "source": os.path.relpath(fn, REPO)}
    return None


def rocprof_top(config, dino="none", n=4):
    """The n kernels with the largest total time in the newest committed rocprofv3 --stats summary of a bench run of
    `config` (DINO-pointwise runs: config<C>_pointwise_*), or None."""
    import csv
    for fn in rocprof_files(config, dino):
        with open(fn) as f:
            rows = sorted(csv.DictReader(f), key=lambda r: -float(r["TotalDurationNs"]))
        return {"source": os.path.relpath(fn, REPO),
                "kernels": [{"name": r["Name"].split("(")[0], "calls": int(r["Calls"]),
                             "avg_us": float(r["AverageNs"]) / 1e3, "percent": float(r["Percentage"])}
                            for r in rows[:n]]}
    return None


def load_traffic(rows, split, tile):
    """HBM(+Infinity Cache) bytes per pc_step launch from the newest committed PMC pass of the same
    kernel instantiation (tile width, arithmetic) and row count (profiles/**/pmc_pc_step*.json,
    scripts/pmc_passes.sh), or None."""
    import re

    def key(fn):   # newest round first, then reverse lexical order (deterministic, no mtimes)
        m = re.search(r"profiles/r(\d+)/", fn.replace(os.sep, "/"))
        return (int(m.group(1)) if m else -1, fn)
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "**", "pmc_pc_step*.json"), recursive=True), key=key)
    for fn in reversed(files):
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        k = d.get("kernel", "")
        if d.get("rows") == rows and k.startswith(f"void pc_step_kernel<{tile // 16}, 8, {3 if split else 0}>"):
            return d.get("hbm_bytes_per_launch")
    return None


def _tile_rows(rows, split):
    from genpose2_amd import _lib
    return _lib.load().gp_pc_tile_rows(rows, int(split))


def report_ode(args, B, N, K, ws, rank, elapsed, nfevs, cfgd):
    """ODE sampler line (report nfev and B*K*nfev/s). The whole pred_func is timed
    (encoder + RK45 on device + host step controller, one 8-byte read per attempted step)."""
    from genpose2_amd import arch
    nfev = float(np.mean(nfevs))
    units = B * K * ws * float(np.sum(nfevs))
    per_call = elapsed / args.steps
    flop = B * K * arch.score_flops_per_candidate_step() * float(np.sum(nfevs))
    if rank == 0:
        print(json.dumps({
            "metric": "pose candidate-RHS evaluations/sec (B objs x K cands x nfev, ODE sampler)",
            "value": units / elapsed, "unit": "pose-candidate-evals/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": per_call * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64 state / f32 score", "data": "synthetic",
            "config": {"workload": f"config{args.config} shape, ODE sampler: B={B} objects/GPU, N={N} pts, K={K}, "
                                   f"T0={args.t0}, RK45 rtol=atol=1e-5 (encoder + sampler per step)",
                       "global_batch": B * ws, "seq_len": nfev, "parallelism": f"dp{ws} (object shards)"},
            "nfev": nfev, "poses_per_s": B * K * ws / per_call,
            "effective_score_tflops": flop / ws / elapsed / 1e12 * ws,
        }), flush=True)


def time_ode_calls(args, cfg, data0, B, K, ws, dev):
    """The shipped evaluation sampler (scripts/eval_single.sh: --sampler_mode ode --T0 0.55, steps unset)
    on the same objects: encoder + device RK45 per pred_func call, 1 warm-up + args.ode_calls timed,
    max over ranks. SURVEY §8d: report nfev and B*K*nfev/s."""
    from genpose2_amd.agent import PoseNet
    agent = PoseNet(cfg.copy(sampler_mode=["ode"], sampling_steps=None)).eval()
    broadcast_weights(agent, ws)
    agent.pred_func(dict(data0), repeat_num=K, T0=0.55)
    torch.cuda.synchronize(dev)
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    from genpose2_amd import arch, ode as ode_mod
    nf = []
    t0 = time.perf_counter()
    for _ in range(args.ode_calls):
        agent.pred_func(dict(data0), repeat_num=K, T0=0.55)
        nf.append(agent.last_nfev)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    # the dominant kernel's time from one more call with each attempt's launch(es) bracketed by HIP events on the
    # launch stream (the events sit between the launches, so that call is not part of the timed ones)
    ode_mod.STAGE_EVENTS = []
    try:
        agent.pred_func(dict(data0), repeat_num=K, T0=0.55)
        torch.cuda.synchronize(dev)
        stage_ms = [a.elapsed_time(b) for a, b, _ in ode_mod.STAGE_EVENTS]
        rows = {r for _, _, r in ode_mod.STAGE_EVENTS}
    finally:
        ode_mod.STAGE_EVENTS = None
    if ws > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    per = el / args.ode_calls
    nfev = float(np.mean(nf))
    out = {"metric": "pose candidate-RHS evaluations/sec (B objs x K cands x nfev, ODE sampler, T0=0.55)",
           "value": B * K * ws * float(np.sum(nf)) / el, "unit": "pose-candidate-evals/s", "nfev": nfev,
           "ms_per_call": per * 1e3, "poses_per_s": B * K * ws / per, "calls": args.ode_calls,
           "workload": f"B={B} objects/GPU, K={K}: encoder + RK45 (rtol=atol=1e-5) + denoise per call"}
    if stage_ms and rows == {B * K}:
        # the dominant kernel: one ode_attempt_kernel per attempted step (the six stage evaluations of every row back
        # to back; GENPOSE2_ODE_FUSED=0: six ode_stage_kernel launches, five stage derivatives then the last stage
        # with y_new and the error partials). The events bracket each attempt's launch(es).
        att_us = float(np.sum(stage_ms)) * 1e3 / len(stage_ms)
        fl = B * K * arch.score_flops_per_candidate_step()
        fast = agent.heads.arith == "f16x3"
        peak = F16_PEAK_TFLOPS / 6 if fast else FP32_PEAK_TFLOPS
        tile = int(_tile_rows(B * K, fast))
        fused = os.environ.get("GENPOSE2_ODE_FUSED", "1")[:1] != "0"
        if fused:
            kname, flop_launch, us = f"void ode_attempt_kernel<{3 if fast else 0}, {tile // 16}>", 6 * fl, att_us
            label = kname
        else:
            kname, flop_launch, us = f"void ode_stage_kernel<0, {3 if fast else 0}, {tile // 16}>", fl, att_us / 6
            label = kname.replace("<0,", "<MODE,")
        out["roofline"] = {"bound": "mfma", "achieved": flop_launch / us / 1e6, "peak": peak, "unit": "TFLOP/s",
                           "frac": flop_launch / us / 1e6 / peak, "kernel": label, "flop_per_launch": flop_launch,
                           "avg_launch_us": us, "us_per_stage_evaluation": att_us / 6, "attempts_timed": len(stage_ms),
                           "stage_ms_per_call": float(np.sum(stage_ms))}
        rp = load_rocprof(kname, args.config)
        if rp is not None:
            rp["achieved"] = flop_launch / (rp["avg_launch_us"] * 1e-6) / 1e12
            rp["frac"] = rp["achieved"] / peak
            out["roofline"]["rocprof"] = rp
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=sorted(CONFIGS),
                    help="4 (default): the north-star shape, one GPU's shard of BASELINE config 4 "
                         "(B=256, K=50, T=500, ScoreNet + EnergyNet + ranking/aggregation)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle CPU baseline threads (0: all physical "
                                                               "cores available, capped by OMP_NUM_THREADS)")
    ap.add_argument("--cpu-sample-objects", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ode-calls", type=int, default=3,
                    help="PC runs: also time this many ODE pred_func calls (shipped setting T0=0.55, RK45) on "
                         "the same objects and report them under 'ode' (0: off)")
    ap.add_argument("--sampler", choices=["pc", "ode"], default="pc",
                    help="ode: the shipped evaluation's sampler (scripts/eval_single.sh: --sampler_mode ode "
                         "--T0 0.55, sampling_steps unset); reports B*K*nfev/s")
    ap.add_argument("--t0", type=float, default=0.55)
    ap.add_argument("--energy-overlap", type=int, default=2, choices=[0, 1, 2],
                    help="2 (default): the EnergyNet encoder runs on a side stream beside the score encoder, "
                         "both ahead of the sampler, which waits for both (config 4: 22.21 ms/step); 0: after "
                         "the sampler on the same stream (22.75); 1: beside the sampler (runner."
                         "EvaluationPipeline). Config 4: 23.12 vs 22.83 "
                         "ms/step, but beside the sampler its workgroups hold CUs at ~45 of the 501 PC-step "
                         "launches per step (up to 1.1 ms each; profiles/r2/energy_overlap_ab.json)")
    ap.add_argument("--share-geometry", type=int, default=1, choices=[0, 1],
                    help="1 (default): the ScoreNet and EnergyNet encoders share one geometry pass per batch "
                         "(FPS indices, centroids and ball lists of every level: gp_encoder_geometry, then "
                         "gp_encoder_forward_geom for both); 0: each encoder computes its own")
    ap.add_argument("--dino", choices=["none", "pointwise"], default="none",
                    help="pointwise: the DINO-pointwise path for the score and energy models (ImgEncoder over synthetic "
                         "DINOv3 layers (B, 256, 384) x 3, patch gather at synthetic roi pixels, Pointnet2ClsMSGFus)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1: encode batch k+1 on a side stream while batch k samples (every timed step "
                         "still encodes and samples one batch; the first encode is not overlapped). "
                         "Off by default: no gain measured (profiles/r1/ab_encoder_pipeline.txt)")
    ap.add_argument("--f32-steps", type=int, default=5,
                    help="PC runs: also time this many steps with every GEMM in exact fp32 (heads and encoders; "
                         "GENPOSE2_HEAD_ARITH=f32 / GENPOSE2_ENC_ARITH=f32) and report them under 'f32_exact' (0: off)")
    ap.add_argument("--pointwise-steps", type=int, default=5,
                    help="Light-encoder PC runs of a full-pipeline config: also time this many steps of the shipped "
                         "scripts' encoder (scripts/eval_single.sh: --dino pointwise) on the same shape and report them "
                         "under 'pointwise' (0: off)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    ndev = 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.launch_probe:
        ndev = count_gpus()
        if ndev is None:
            raise SystemExit(f"bench.py: --gpus {args.gpus}: cannot count the node's GPUs without a HIP call (amdsmi "
                             f"unusable and no KFD topology at {KFD_NODES}); not starting the launcher")
    cmd = launch_command(sys.argv[1:], args.gpus, os.environ, ndev, probe=args.launch_probe)
    if cmd is not None:
        import subprocess
        sys.exit(subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")))
    cfgd = CONFIGS[args.config]
    ws, rank, local = dist_env()
    if args.launch_probe:
        return launch_probe(ws, rank)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from genpose2_amd import aggregate, arch, synthetic
    from genpose2_amd.agent import PoseNet
    from genpose2_amd.config import GenPoseConfig

    B, N, K, T = cfgd["B"], cfgd["N"], cfgd["K"], cfgd["T"]
    ode = args.sampler == "ode"
    from types import SimpleNamespace

    def build_leg(dino):
        """The agents of one pipeline (score, energy, scale as the config asks) and its synthetic objects in HBM."""
        c = GenPoseConfig(device=str(dev), sampling_steps=None if ode else T, eval_repeat_num=K,
                          noise_seed=1234 + rank, sampler_mode=[args.sampler], dino=dino)
        sc = PoseNet(c).eval()
        broadcast_weights(sc, ws)
        en = PoseNet(c.copy(agent_type="energy")).eval() if cfgd["energy"] else None
        sl = PoseNet(c.copy(agent_type="scale")).eval() if cfgd["scale"] else None
        for a in (en, sl):
            if a is not None:
                broadcast_weights(a, ws)
        pts, center = synthetic.make_batch(args.config, B, N, first_object=rank * B)
        d0 = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev)}
        if dino == "pointwise":   # the DINOv3 backbone's layers [2, 6, 11] and roi pixels, synthetic
            rng = np.random.Generator(np.random.PCG64(4242 + rank))
            d0["dino_layers"] = [torch.from_numpy(rng.standard_normal((B, 256, 384), dtype=np.float32)).to(dev)
                                 for _ in range(3)]
            d0["roi_xs"] = torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev)
            d0["roi_ys"] = torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev)
        return SimpleNamespace(score=sc, energy=en, scale=sl, data0=d0, dino=dino, cfg=c)

    main_leg = build_leg(args.dino)
    cfg, score, energy, scale, data0 = main_leg.cfg, main_leg.score, main_leg.energy, main_leg.scale, main_leg.data0

    stream = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    enc_side = torch.cuda.Stream(device=dev)
    samp_ev = []
    pending = []   # --pipeline: the next batch's data dict, its encoder already enqueued on enc_side

    def start_encode():
        d = dict(data0)
        enc_side.wait_stream(stream)
        with torch.cuda.stream(enc_side):
            score.encode_func(d)
        pending.append(d)
    nfevs = []

    def one_step(record=False, last=False, leg=None, evs=None):
        leg = main_leg if leg is None else leg
        evs = samp_ev if evs is None else evs
        score, energy, scale, data0 = leg.score, leg.energy, leg.scale, leg.data0
        pipe = args.pipeline and not ode and leg is main_leg
        if pipe:
            if not pending:          # first step of a run: nothing to overlap with yet
                start_encode()
            data = pending.pop(0)
            stream.wait_stream(enc_side)
            data["pts_feat"].record_stream(stream)
        else:
            data = dict(data0)
        edata = None
        if energy is not None:
            # the energy encoder needs only the points: overlap it with the score sampler
            # (as genpose2_amd.runner.EvaluationPipeline does)
            edata = {k: data0[k] for k in ("pts", "pts_center", "dino_layers", "roi_xs", "roi_ys") if k in data0}
            if args.share_geometry and not pipe:
                score.encode_geometry(data)          # one geometry pass for both encoders of this batch
                edata["enc_geometry"] = data["enc_geometry"]

            def start_energy_encoder():
                side.wait_stream(stream)
                with torch.cuda.stream(side):
                    energy.encode_func(edata)
            score.after_encode = start_energy_encoder if args.energy_overlap == 1 else None
            if args.energy_overlap == 2:
                # both encoders together ahead of the sampler (their latency-bound launches interleave);
                # the sampler then waits for both, so nothing shares CUs with it
                start_energy_encoder()
                score.after_encode = lambda: stream.wait_stream(side)
        if record and not ode:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            # bracket only the PC sampler launches (pc_step_kernel x (T+1)) on the launch stream
            orig = score.heads.pc_sample

            def timed(*a, **k):
                e0.record(stream)
                out = orig(*a, **k)
                e1.record(stream)
                return out
            score.heads.pc_sample = timed
        if pipe:
            # the next batch's encoder runs beside this batch's sampler; after_encode
            # (energy encoder) still starts here, before the sampler
            if not last:
                start_encode()
            if score.after_encode is not None:
                score.after_encode()
            hook, score.after_encode = score.after_encode, None
            pose, _ = score.pred_func(data, repeat_num=K, extract_feature=False)
            score.after_encode = hook
        else:
            pose, _ = score.pred_func(data, repeat_num=K, T0=args.t0 if ode else None)
        if ode:
            nfevs.append(score.last_nfev)
        if record and not ode:
            score.heads.pc_sample = orig
            evs.append((e0, e1))
        if energy is not None:
            if not args.energy_overlap:
                energy.encode_func(edata)
            stream.wait_stream(side)
            edata["pts_feat"].record_stream(stream)
            if "_energy_pobj" in edata:
                edata["_energy_pobj"][1].record_stream(stream)
            e = energy.get_energy(edata, pose, T=1e-5, extract_feature=False)
            agg = aggregate.aggregate_pose(pose, e)
            if scale is not None:
                scale.pred_scale_func({"pts_feat": data["pts_feat"], "axes": agg[:, :3, :3].contiguous()})
        elif scale is not None:
            axes = torch.eye(3, device=dev).expand(B, 3, 3).contiguous()
            scale.pred_scale_func({"pts_feat": data["pts_feat"], "axes": axes})
        return pose

    def timed_steps(n, leg=None, evs=None):
        """n steps between a barrier + device synchronisation on both sides; the max over ranks (s)."""
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(n):
            one_step(record=True, last=True, leg=leg, evs=evs)
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        el = time.perf_counter() - t1
        if ws > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for i in range(args.warmup):
        one_step(last=i == args.warmup - 1)
    torch.cuda.synchronize(dev)
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(record=True, last=i == args.steps - 1)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if ode:
        report_ode(args, B, N, K, ws, rank, elapsed, nfevs[-args.steps:], cfgd)
        if ws > 1:
            dist.destroy_process_group()
        return
    ode_info = time_ode_calls(args, cfg, data0, B, K, ws, dev) if args.ode_calls > 0 else None
    fast = score.heads.arith == "f16x3"
    f32_info = None
    if args.f32_steps > 0 and fast:
        # the same steps with every GEMM in exact fp32 (the arithmetic the reference runs)
        agents = [a for a in (score, energy) if a is not None]
        for a in agents:
            a.heads.set_arith("f32")
            if hasattr(a.encoder, "set_arith"):
                a.encoder.set_arith("f32")
            if getattr(a, "img_encoder", None) is not None:
                a.img_encoder.set_arith("f32")
        n_ev = len(samp_ev)
        one_step(last=True)
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.f32_steps):
            one_step(record=True, last=True)
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        el32 = time.perf_counter() - t1
        if ws > 1:
            t = torch.tensor([el32], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el32 = float(t.item())
        ms32 = float(np.mean([a.elapsed_time(b) for a, b in samp_ev[n_ev:]]))
        del samp_ev[n_ev:]
        for a in agents:
            a.heads.set_arith("f16x3")
            if hasattr(a.encoder, "set_arith"):
                a.encoder.set_arith("split_f16")
            if getattr(a, "img_encoder", None) is not None:
                a.img_encoder.set_arith("split_f16")
        us32 = ms32 / 1e3 / (T + 1) * 1e6
        fl = B * K * arch.score_flops_per_candidate_step()
        k32 = f"void pc_step_kernel<{int(_tile_rows(B * K, False)) // 16}, 8, 0>"
        f32_info = {"value": B * K * T * ws * args.f32_steps / el32, "unit": "pose-candidate-steps/s",
                    "steps": args.f32_steps, "ms_per_step": el32 / args.f32_steps * 1e3,
                    "dtype": "f32 (every GEMM exact fp32 MFMA, v_mfma_f32_16x16x4_f32)",
                    "roofline": {"bound": "mfma", "achieved": fl / us32 / 1e6, "peak": FP32_PEAK_TFLOPS,
                                 "unit": "TFLOP/s", "frac": fl / us32 / 1e6 / FP32_PEAK_TFLOPS,
                                 "avg_launch_us": us32, "kernel": k32}}
        rp32 = load_rocprof(k32, args.config, args.dino)
        if rp32 is not None:
            rp32["achieved"] = fl / (rp32["avg_launch_us"] * 1e-6) / 1e12
            rp32["frac"] = rp32["achieved"] / FP32_PEAK_TFLOPS
            f32_info["roofline"]["rocprof"] = rp32
    pw_info = None
    if args.pointwise_steps > 0 and args.dino == "none" and cfgd["energy"] and not args.pipeline:
        # the shipped scripts' configuration (--dino pointwise): ImgEncoder over synthetic DINOv3 layers, the patch
        # gather and Pointnet2ClsMSGFus for both nets, the same sampler, energy and aggregation
        pw = build_leg("pointwise")
        pw_ev = []
        for _ in range(2):
            one_step(last=True, leg=pw, evs=[])
        elp = timed_steps(args.pointwise_steps, leg=pw, evs=pw_ev)
        pw_samp = float(np.mean([a.elapsed_time(b) for a, b in pw_ev]))
        ms = elp / args.pointwise_steps * 1e3
        pw_info = {"value": B * K * T * ws * args.pointwise_steps / elp, "unit": "pose-candidate-steps/s",
                   "steps": args.pointwise_steps, "ms_per_step": ms, "sampler_ms_per_step": pw_samp,
                   "non_sampler_ms_per_step": ms - pw_samp,
                   "pc_step_avg_launch_us": pw_samp / (T + 1) * 1e3,
                   "workload": f"config{args.config} shape with --dino pointwise (scripts/eval_single.sh): ImgEncoder over "
                               f"synthetic DINOv3 layers (B, 256, 384) x 3, patch gather, Pointnet2ClsMSGFus for the score "
                               f"and energy nets, PC sampler, energy, ranking/aggregation",
                   "rocprof_top": rocprof_top(args.config, "pointwise")}
        del pw
        torch.cuda.empty_cache()
    units = B * K * T * ws * args.steps
    samp_ms = float(np.mean([a.elapsed_time(b) for a, b in samp_ev]))
    per_launch_s = samp_ms / 1e3 / (T + 1)
    flop_launch = B * K * arch.score_flops_per_candidate_step()
    achieved = flop_launch / per_launch_s / 1e12
    # f16x3: the two per-candidate GEMMs run 6 f16 MFMA products per fp32 MAC (three planes per operand),
    # so their MFMA ceiling in algorithmic (fp32) FLOP/s is the dense f16 peak / 6
    peak = F16_PEAK_TFLOPS / 6 if fast else FP32_PEAK_TFLOPS
    up = score.heads.up.t
    wg_bytes = sum(up[k].numel() * up[k].element_size() for k in
                   (("pe2_h", "h1p_h") if fast else ("pe2_w", "h1p_w")))   # streamed per workgroup per step
    tile = int(_tile_rows(B * K, fast))   # the kernel's real tile width
    nwg = -(-B * K // tile)
    if rank == 0:
        out = {
            "metric": "pose candidates/sec (B objs x K cands x T denoise steps)",
            "value": units / elapsed,
            "unit": "pose-candidate-steps/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("f32 (pose_encoder.2 / head-1 GEMMs: f16x3 -- three f16 planes per fp32 operand, six MFMA "
                      "products, products to 2^-33, fp32 accumulation; encoder SA levels 1-3: split-f16, per-level error "
                      "vs float64 within exact fp32 MFMA's: tests/test_gpu_precision.py)") if fast else "f32",
            "data": "synthetic (seeded point clouds, seeded synthetic weights; no checkpoint exists for dino=none)",
            "config": {"workload": f"config{args.config}: B={B} objects/GPU, N={N} pts, K={K} candidates, T={T} PC "
                                   f"steps, {'ScoreNet+EnergyNet+ranking/aggregation' if cfgd['energy'] else 'ScoreNet'}"
                                   f"{' + ScaleNet' if cfgd['scale'] else ''} (encoder + sampler per step)"
                                   f"{', DINO-pointwise fused encoders' if args.dino == 'pointwise' else ''}",
                       "global_batch": B * ws, "seq_len": T, "parallelism": f"dp{ws} (object shards)",
                       "encoder_pipelined": bool(args.pipeline),
                       "shared_geometry": bool(args.share_geometry and cfgd["energy"] and not args.pipeline),
                       "energy_encoder": (["after the sampler", "beside the sampler", "beside the score encoder"]
                                          [args.energy_overlap] if cfgd["energy"] else None)},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": load_traffic(B * K, fast, tile),
                         "kernel": "pc_step_kernel", "arith": score.heads.arith, "flop_per_launch": flop_launch,
                         "avg_launch_us": per_launch_s * 1e6, "sampler_ms_per_step": samp_ms,
                         "fp32_mfma_equiv_frac": achieved / FP32_PEAK_TFLOPS,
                         # every workgroup streams the GEMM weights from L2
                         "l2_weight_stream": {"bytes_per_workgroup": wg_bytes, "workgroups": nwg,
                                              "candidates_per_workgroup": tile,
                                              "GBps_per_CU": wg_bytes / per_launch_s / 1e9,
                                              "TBps_chip": wg_bytes * nwg / per_launch_s / 1e12}},
        }
        rp = load_rocprof(f"void pc_step_kernel<{tile // 16}, 8, {3 if fast else 0}>", args.config, args.dino)
        if rp is not None:   # the committed rocprofv3 --stats of a bench run: its mean launch, same FLOPs
            rp["achieved"] = flop_launch / (rp["avg_launch_us"] * 1e-6) / 1e12
            rp["frac"] = rp["achieved"] / peak
            out["roofline"]["rocprof"] = rp
        if f32_info is not None:
            out["f32_exact"] = f32_info
        if ode_info is not None:
            out["ode"] = ode_info
        if pw_info is not None:
            out["pointwise"] = pw_info
        if not args.no_cpu_baseline and args.dino == "none":
            threads = args.cpu_threads or cpu_threads_default()
            out["cpu_baseline"] = (cpu_baseline(cfgd, args.config, threads, args.cpu_sample_objects)
                                   if ws == 1 else None)
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
