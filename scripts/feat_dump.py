"""Diagnostic: dump the energy agent's encoder features (both arithmetic paths) for the objects of
golden_large_energy_r12800 to gpurun_out/ for a float64 comparison on the host."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402

pts, _ = synthetic.make_batch(63, 256, 1024)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
for ea in ("split_f16", "f32"):
    a = PoseNet(GenPoseConfig(device="cuda:0", agent_type="energy")).eval()
    a.encoder.set_arith(ea)
    f, ws = a.encoder.forward(torch.from_numpy(pts).cuda(), return_workspace=True)
    lv = a.encoder.levels(256, 1024, ws)
    np.savez(os.path.join(REPO, "gpurun_out", f"feat_{ea}.npz"), feat=f.cpu().numpy(),
             **{f"l{i}": lv[i]["features"][16:24].cpu().numpy() for i in range(4)})
print("ok")
