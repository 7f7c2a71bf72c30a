"""Diagnostic: the PC step kernel's score (NT = 2 / 4 column tiles per workgroup) against the score
evaluation kernel (NT = 1) on the same states. Prints per-row-position error statistics."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import sde  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=2)).eval()
    h = agent.heads
    out = {}
    for B, K in [(4, 16), (96, 50), (256, 50)]:
        R = B * K
        tab = sde.pc_step_table(2)
        tproj = h.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
        pobj = h.object_proj(torch.rand(B, 1024, device=dev))
        center = torch.zeros(B, 3, device=dev)
        x0 = torch.randn(R, 9, device=dev)
        z = torch.zeros(2, R, 9, device=dev)
        _, _, xs = h.pc_sample(pobj, tproj, tab, x0.clone(), K, center, z1=z, z2=z, want_xs=True)
        s_pc = h._pc_ws[: R * 9 * 4].view(torch.float32).view(R, 9).clone()
        s_ev = h.score(pobj, tproj[1:2].contiguous(), float(tab[1, 1]), xs[:, 0].contiguous(), K)
        d = (s_pc - s_ev).abs() / (s_ev.abs().max() + 1e-30)
        rowerr = d.max(dim=1).values.cpu().numpy()
        bad = np.nonzero(rowerr > 1e-4)[0]
        out[f"R{R}"] = {"max_rel": float(d.max()), "bad_rows": int(bad.size), "first_bad": bad[:20].tolist(),
                        "bad_mod64": np.bincount(bad % 64, minlength=64).tolist() if bad.size else [],
                        "bad_cols": np.bincount(np.nonzero(d.cpu().numpy() > 1e-4)[1], minlength=9).tolist()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
