"""Host-side timing of the device-controlled RK45 loop (tuning aid, not a test): per attempt, the
time the host spends enqueueing and waiting for the status word."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import ode, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampler_mode=["ode"], sampling_steps=None)).eval()
    pts, center = synthetic.make_batch(2, 64, 1024)
    data = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev)}
    rec = {"launch": [], "wait": []}
    orig_sync = torch.cuda.Stream.synchronize
    orig_check = ode.check

    def timed_check(rc, what=""):
        t0 = time.perf_counter()
        orig_check(rc, what)
        if what == "ode_auto_attempt":
            rec["launch"].append(time.perf_counter() - t0)

    def timed_sync(self):
        t0 = time.perf_counter()
        orig_sync(self)
        rec["wait"].append(time.perf_counter() - t0)
    for _ in range(2):
        agent.pred_func(dict(data), repeat_num=50, T0=0.55)
    torch.cuda.synchronize()
    torch.cuda.Stream.synchronize = timed_sync
    t0 = time.perf_counter()
    agent.pred_func(dict(data), repeat_num=50, T0=0.55)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    torch.cuda.Stream.synchronize = orig_sync
    print(json.dumps({"wall_ms": wall * 1e3, "n_wait": len(rec["wait"]),
                      "wait_us_mean": float(np.mean(rec["wait"]) * 1e6),
                      "wait_us_min": float(np.min(rec["wait"]) * 1e6)}))


if __name__ == "__main__":
    main()
