"""Small fixed workload for rocprofv3 PMC passes: the config-2 PC sampler (R=3200) for a few
steps, plus one encoder pass. Usage: rocprofv3 --pmc ... -- python scripts/pmc_target.py [rows]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import sde, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K, T = 50, 20
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=T)).eval()
    pts, center = synthetic.make_batch(2, B, 1024)
    p = torch.from_numpy(pts).to(dev)
    feat = agent.encoder.forward(p)
    tab = sde.pc_step_table(T)
    tproj = agent.heads.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
    pobj = agent.heads.object_proj(feat)
    x0 = torch.randn(B * K, 9, device=dev) * 50
    agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), K, torch.from_numpy(center).to(dev), seed=1)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
