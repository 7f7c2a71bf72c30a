"""Per-kernel timing sweep (HIP events on the launch stream) for tuning; not part of the bench contract.

    python scripts/kbench.py [--pc] [--enc]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import arch, sde, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def timeit(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pc", action="store_true")
    ap.add_argument("--enc", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=100)).eval()
    out = {}
    if args.pc or not args.enc:
        T = 100
        tab = sde.pc_step_table(T)
        tproj = agent.heads.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
        for B, K in [(64, 50), (256, 50), (256, 100)]:
            R = B * K
            feat = torch.rand(B, 1024, device=dev)
            pobj = agent.heads.object_proj(feat)
            center = torch.zeros(B, 3, device=dev)
            x0 = torch.randn(R, 9, device=dev) * 50

            def run():
                agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), K, center, seed=1)
            ms = timeit(run)
            us = ms * 1e3 / (T + 1)
            tf = R * arch.score_flops_per_candidate_step() / (us * 1e-6) / 1e12
            out[f"pc_R{R}"] = {"us_per_launch": us, "tflops": tf, "frac": tf / 157.3}
            trow = tproj[:1].contiguous()
            ms2 = timeit(lambda: [agent.heads.score(pobj, trow, 1.0, x0, K) for _ in range(20)])
            out[f"score_eval_R{R}"] = {"us_per_launch": ms2 * 1e3 / 20}
    if args.enc or not args.pc:
        for B, N in [(64, 1024), (256, 2048)]:
            pts, _ = synthetic.make_batch(9, B, N)
            p = torch.from_numpy(pts).to(dev)
            ms = timeit(lambda: agent.encoder.forward(p), reps=3)
            tf = B * arch.encoder_flops_per_object(N) / (ms * 1e-3) / 1e12
            out[f"enc_B{B}_N{N}"] = {"ms": ms, "tflops": tf}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
