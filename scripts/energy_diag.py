"""Diagnostic: EnergyNet error at R=12,800 against golden_large_energy_r12800 (reference fp32 and its
float64 run), both arithmetic paths of the heads and of the encoder, plain and clustered sets."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden")]
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402

g = np.load(os.path.join(REPO, "tests/golden/golden_large_energy_r12800.npz"))
plain = np.load(os.path.join(REPO, "tests/golden/golden_large_pc_r12800_t500.npz"))["pred_pose"]
pts, center = synthetic.make_batch(63, 256, 1024)
data = {"pts": torch.from_numpy(pts).cuda(), "pts_center": torch.from_numpy(center).cuda()}


def rel(a, b):
    return np.abs(a.astype(np.float64) - b).reshape(256, -1).max(1) / np.abs(b).reshape(256, -1).max(1)


for tag, pose in (("", plain), ("cl_", g["cl_pose"])):
    e32, e64 = g[tag + "energy"], g[tag + "energy64"]
    own = rel(e32, e64)
    for ha in ("split_f16", "f32"):
        for ea in ("split_f16", "f32"):
            a = PoseNet(GenPoseConfig(device="cuda:0", agent_type="energy")).eval()
            a.heads.set_arith(ha)
            a.encoder.set_arith(ea)
            e = a.get_energy(dict(data), torch.from_numpy(pose).cuda(), T=1e-5).cpu().numpy()
            v32, v64 = rel(e, e32), rel(e, e64)
            print(f"{tag or 'plain'} heads={ha} enc={ea}: vs ref32 max {v32.max():.2e}; vs ref64 max {v64.max():.2e} "
                  f"(ref32's own {own.max():.2e}); worst ratio ours/own {np.max(v64 / own):.2f}", flush=True)

# the heads alone: the oracle's (numpy fp32) encoder output fed in place of ours
of = os.path.join(REPO, "diag", "oracle_energy_feat.npy")
if os.path.exists(of):
    feat = torch.from_numpy(np.load(of)).cuda()
    for tag, pose in (("", plain), ("cl_", g["cl_pose"])):
        e32, e64 = g[tag + "energy"], g[tag + "energy64"]
        for ha in ("split_f16", "f32"):
            a = PoseNet(GenPoseConfig(device="cuda:0", agent_type="energy")).eval()
            a.heads.set_arith(ha)
            d = dict(data, pts_feat=feat)
            e = a.get_energy(d, torch.from_numpy(pose).cuda(), T=1e-5, extract_feature=False).cpu().numpy()
            print(f"{tag or 'plain'} heads={ha} on the oracle's pts_feat: vs ref32 {rel(e, e32).max():.2e}, "
                  f"vs ref64 {rel(e, e64).max():.2e}", flush=True)
