"""Split-f16 vs exact-fp32 PC trajectories on identical inputs and noise (B objects x 50 candidates,
T steps): writes the final poses of both arithmetics to OUT.npz. Run once per library build
(GENPOSE_HIP_LIB) to compare tile widths. usage: python scripts/split_spread.py OUT B T"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402

out, B, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
pts, center = synthetic.make_batch(5, B, 1024)
data = {"pts": torch.from_numpy(pts).to("cuda:0"), "pts_center": torch.from_numpy(center).to("cuda:0")}
res = {}
for arith in ("split_f16", "f32"):
    a = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=T, noise_seed=7)).eval()
    a.heads.set_arith(arith)
    res[arith] = a.pred_func(dict(data), repeat_num=50)[0].cpu().numpy()
np.savez(out, **res)
