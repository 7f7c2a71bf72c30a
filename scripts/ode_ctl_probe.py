"""Device- vs host-controlled RK45 wall time per pred_func (tuning aid, not a test).
python scripts/ode_ctl_probe.py [T0]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    t0 = float(sys.argv[1]) if len(sys.argv) > 1 else 0.55
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampler_mode=["ode"], sampling_steps=None)).eval()
    pts, center = synthetic.make_batch(2, 64, 1024)
    data = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev)}
    out = {"T0": t0}
    for host in (True, False, True, False):
        agent.ode_host_control = host
        for _ in range(2):
            agent.pred_func(dict(data), repeat_num=50, T0=t0)
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(5):
            agent.pred_func(dict(data), repeat_num=50, T0=t0)
        torch.cuda.synchronize()
        out["host" if host else "device"] = {"ms": (time.perf_counter() - a) / 5 * 1e3, "nfev": agent.last_nfev}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
