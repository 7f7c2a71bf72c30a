"""CPU-baseline calibration (SURVEY §8d "CPU baseline" (i)): the imported reference and this
oracle timed on identical inputs and thread counts in the build container.

Test infrastructure, like the rest of oracle/: it reads /root/reference (read-only) and so runs
only here, never on the GPU box. bench.py's ``cpu_baseline`` times the oracle on the GPU host
(ii); the ratio recorded here converts that figure into reference-equivalent terms.

Both sides run ``pred_func`` (encoder + PC sampler, injected noise) at the config-2 row count
(B=64 objects, K=50) for two step counts; the difference isolates the per-step cost and the rest
is the per-call cost (encoder, repeats, epilogue). The reference's encoder uses the oracle's C
restatement of the four CUDA ops (the reference has no CPU version of them).

Usage:  python oracle/calibrate_cpu.py [threads] > profiles/r1/cpu_calibration.json
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import torch  # noqa: E402

import make_golden as mg  # noqa: E402  (reference import helpers)
from genpose2_amd import weights  # noqa: E402
from oracle import oracle  # noqa: E402


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    torch.set_num_threads(threads)
    B, K = 64, 50
    steps = (10, 50)
    get_config, PoseNet = mg.import_reference("pc", steps[0])
    d = mg.batch(2, B, 1024)
    sd = weights.synthetic_state_dict("score", seed=0)
    rng = np.random.Generator(np.random.PCG64(5))
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    out = {"B": B, "K": K, "threads": threads, "cpu": platform.processor() or platform.machine(),
           "torch_matmul_precision": torch.get_float32_matmul_precision()}
    # encoder, per object (4 objects)
    agent = mg.make_agent(get_config, PoseNet, "score", "pc", steps[0])
    d4 = {"pts": d["pts"][:4].contiguous(), "pts_center": d["pts_center"][:4].contiguous()}
    with torch.no_grad():
        ref_enc = timed(lambda: agent.net(dict(d4), mode="pts_feature")) / 4
    orc_enc = timed(lambda: oracle.encoder_forward(sd, d4["pts"].numpy())) / 4
    # sampler per step: pred_func at two step counts (the encoder cancels in the difference)
    ref_t, orc_t = {}, {}
    for T in steps:
        zs = rng.standard_normal((2 * T, B * K, 9)).astype(np.float32)
        agent = mg.make_agent(get_config, PoseNet, "score", "pc", T)

        def run_ref():
            with mg.NoiseFeed(prior, zs):
                agent.pred_func(dict(d), repeat_num=K)

        def run_orc():
            oracle.pred_func(sd, d["pts"].numpy(), d["pts_center"].numpy(), K, T, "pc", prior, zs[0::2], zs[1::2])

        ref_t[T] = timed(run_ref, reps=1)
        orc_t[T] = timed(run_orc, reps=1)
    a, b = steps
    for name, t, enc in (("reference", ref_t, ref_enc), ("oracle", orc_t, orc_enc)):
        out[name] = {"encoder_s_per_object": enc, "sampler_s_per_step": (t[b] - t[a]) / (b - a),
                     f"pred_func_T{a}_s": t[a], f"pred_func_T{b}_s": t[b]}
    # the bench workload (config 2: B=64, K=50, T=500): encoder for B objects + T sampler steps
    full = {n: B * out[n]["encoder_s_per_object"] + 500 * out[n]["sampler_s_per_step"] for n in ("reference", "oracle")}
    out["config2_pred_func_s"] = full
    out["oracle_over_reference"] = full["oracle"] / full["reference"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
