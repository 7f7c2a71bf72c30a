"""Split-f16 token linear (gp_linear_split) timing by shape, with and without the epilogue options, against
torch fp32 for accuracy (tuning aid, not a test). Shapes: the DINO-pointwise transformer linears at B=256.
usage: python scripts/lin_bench.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib  # noqa: E402
from genpose2_amd.fus_encoder import pack_split_linear  # noqa: E402

DEV = "cuda:0"
SHAPES = [   # (name, m tokens, k, n)
    ("L3.linear1", 16384, 1024, 4096), ("L3.linear2", 16384, 4096, 1024), ("L3.qkv", 16384, 1024, 3072),
    ("L2.linear1", 32768, 512, 2048), ("L2.linear2", 32768, 2048, 512), ("L1.linear1", 65536, 256, 1024),
    ("L0.linear1", 131072, 96, 384), ("img.conv", 65536, 3456, 96), ("ragged", 1000, 160, 384),
    ("ragged256", 4000, 224, 512),
]


def vp(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def main():
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    out = []
    only = os.environ.get("LIN_SHAPES")
    for name, m, k, n in SHAPES:
        if only and name not in only.split(","):
            continue
        x = torch.from_numpy(rng.normal(size=(m, k)).astype(np.float32)).to(DEV)
        w = (rng.normal(size=(n, k)) / np.sqrt(k)).astype(np.float32)
        wh = torch.from_numpy(pack_split_linear(w)).to(DEV)
        b = torch.from_numpy(rng.normal(size=n).astype(np.float32) * 0.1).to(DEV)
        y = torch.empty(m, n, device=DEV)
        rmax = x.abs().amax(1).contiguous()
        ymax = torch.empty(m, device=DEV)
        rec = {"shape": name, "m": m, "k": k, "n": n}
        for tag, act, use_ymax in (("relu+ymax", 1, True), ("relu", 1, False), ("none", 0, False)):
            def run():
                _lib.check(lib.gp_linear_split(vp(x), k, m, k, vp(wh), vp(b), n, act, vp(y), n, vp(rmax), 1,
                                               vp(ymax if use_ymax else None), st), "linear_split")
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 5 * 1e3
            rec[tag] = {"us": round(us, 1), "tflops": round(2 * m * n * k / us / 1e6, 1)}
        ref = x @ torch.from_numpy(w).to(DEV).T + b
        rec["max_rel_err"] = float(((y - ref).abs().max() / ref.abs().max()).item())
        # bit pattern digest of the last run's outputs (two builds compare equal iff bit-identical, up to collisions)
        rec["digest"] = int((y.view(torch.int32).to(torch.int64) * torch.arange(1, y.numel() + 1, device=DEV).view_as(y)
                             % 1000003).sum().item())
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del x, y, ref


if __name__ == "__main__":
    main()
