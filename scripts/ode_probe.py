"""Per-attempt host/GPU time split of the device RK45 sampler (tuning aid, not a test).

python scripts/ode_probe.py [B] [K]: runs pred_func with the ODE sampler at T0=0.55 and reports,
per attempted step, the host time spent forming scalars, launching, and waiting for the error norm,
next to the GPU time of the attempt's kernels (HIP events)."""
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampler_mode=["ode"], sampling_steps=None)).eval()
    pts, center = synthetic.make_batch(2, B, 1024)
    data = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev)}
    stats = {"scalars": [], "launch": [], "wait": [], "gpu": []}
    orig = ode.DeviceRk45.attempt

    def attempt(self, t, h):
        t0 = time.perf_counter()
        stage_t = [t + c * h for c in ode.C[1:]] + [t + h]
        ode.stage_scalars(stage_t)
        t1 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        self._probe = True
        r = orig(self, t, h)   # includes the scalars again, the launch and the wait
        e1.record()
        t2 = time.perf_counter()
        e1.synchronize()
        stats["scalars"].append(t1 - t0)
        stats["launch"].append(t2 - t1)
        stats["gpu"].append(e0.elapsed_time(e1) / 1e3)
        return r
    for _ in range(2):
        agent.pred_func(dict(data), repeat_num=K, T0=0.55)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.pred_func(dict(data), repeat_num=K, T0=0.55)
    torch.cuda.synchronize()
    plain = time.perf_counter() - t0
    ode.DeviceRk45.attempt = attempt
    agent.pred_func(dict(data), repeat_num=K, T0=0.55)
    torch.cuda.synchronize()
    ode.DeviceRk45.attempt = orig
    out = {"B": B, "K": K, "nfev": agent.last_nfev, "call_ms": plain * 1e3, "attempts": len(stats["gpu"]),
           "per_attempt_us": {k: float(np.mean(v) * 1e6) for k, v in stats.items() if v}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
