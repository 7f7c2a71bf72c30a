"""Dump deterministic outputs of the loaded library (GENPOSE_HIP_LIB) for bit-for-bit comparison of
two builds: object projection, time projection, a short Philox PC run and the encoder features.
usage: python scripts/lib_outputs.py OUT.npz"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import sde, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402

dev = torch.device("cuda:0")
agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=20)).eval()
B, K, T = 37, 50, 20
pts, center = synthetic.make_batch(5, B, 1024)
feat = agent.encoder.forward(torch.from_numpy(pts).to(dev))
pobj = agent.heads.object_proj(feat)
tab = sde.pc_step_table(T)
tproj = agent.heads.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
x0 = torch.randn(B * K, 9, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
res, q, _ = agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), K, torch.from_numpy(center).to(dev), seed=1)
np.savez(sys.argv[1], feat=feat.cpu().numpy(), pobj=pobj.cpu().numpy(), tproj=tproj.cpu().numpy(),
         res=res.cpu().numpy(), q=q.cpu().numpy())
