"""DINO-pointwise encoder pass: host enqueue time vs GPU time, one encoder alone and the ScoreNet + EnergyNet encoders
side by side (tuning aid, not a test).

    python scripts/pw_probe.py [B]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = 1024
    dev = torch.device("cuda:0")
    cfg = GenPoseConfig(device="cuda:0", sampling_steps=500, dino="pointwise")
    score = PoseNet(cfg).eval()
    energy = PoseNet(cfg.copy(agent_type="energy")).eval()
    pts, center = synthetic.make_batch(4, B, N)
    rng = np.random.Generator(np.random.PCG64(4242))
    d0 = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev),
          "dino_layers": [torch.from_numpy(rng.standard_normal((B, 256, 384), dtype=np.float32)).to(dev)
                          for _ in range(3)],
          "roi_xs": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev),
          "roi_ys": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev)}
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    out = {}

    def one(agent, stream, reps=5):
        host, gpu = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                t0 = time.perf_counter()
                agent.encode_func(dict(d0))
                host.append((time.perf_counter() - t0) * 1e3)
                e1.record(stream)
            torch.cuda.synchronize()
            gpu.append(e0.elapsed_time(e1))
        return float(np.median(host[1:])), float(np.median(gpu[1:]))

    out["score_alone_host_ms"], out["score_alone_gpu_ms"] = one(score, main_s)
    out["energy_alone_host_ms"], out["energy_alone_gpu_ms"] = one(energy, side)

    def both(order, reps=5):
        walls, hosts = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            side.wait_stream(main_s)
            t0 = time.perf_counter()
            for who in order:
                if who == "score":
                    score.encode_func(dict(d0))
                else:
                    with torch.cuda.stream(side):
                        energy.encode_func(dict(d0))
            hosts.append((time.perf_counter() - t0) * 1e3)
            main_s.wait_stream(side)
            e1.record(main_s)
            torch.cuda.synchronize()
            walls.append(e0.elapsed_time(e1))
        return float(np.median(hosts[1:])), float(np.median(walls[1:]))

    out["both_energy_first_host_ms"], out["both_energy_first_gpu_ms"] = both(("energy", "score"))
    out["both_score_first_host_ms"], out["both_score_first_gpu_ms"] = both(("score", "energy"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
