"""Per-layer breakdown of sa_branch_kernel launches from in-kernel s_memtime marks (tuning aid).

    make -C genpose2_amd/csrc OUT=../../variants/satrace/libgenpose_hip.so BUILD=../../variants/satrace/build EXTRA=-DSA_TRACE
    GENPOSE_HIP_LIB=variants/satrace/libgenpose_hip.so python scripts/sa_trace.py [B]
Marks per wave: 0 start, 2L+1 after layer L's MFMA loops + epilogue, 2L+2 after the layer barrier.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib, arch, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    lib = _lib.load()
    fn = lib.gp_debug_sa_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p]
    agent = PoseNet(GenPoseConfig(device="cuda:0")).eval()
    pts, _ = synthetic.make_batch(9, B, 1024)
    p = torch.from_numpy(pts).to("cuda:0")
    agent.encoder.forward(p)
    out = {}
    br = arch.sa_branches()
    for lv in range(5):
        for b in range(2):
            tag = lv * 2 + b
            assert fn(tag, None) == 0
            agent.encoder.forward(p)
            torch.cuda.synchronize()
            buf = np.zeros(8192 * 4 * 8, np.uint64)
            assert fn(-1, buf.ctypes.data) == 0
            nl = 3 if lv < 4 else 2
            tr = buf.reshape(8192, 4, 8).astype(np.int64)
            used = tr[:, 0, 0] != 0
            if not used.any():   # level not run by sa_branch_kernel (narrow levels)
                continue
            tr = tr[used][:, :, : 2 * nl + 1]
            d = np.diff(tr, axis=-1)
            widths = br[lv][b].widths
            rec = {"wgs": int(used.sum()), "lifetime_mean": float((tr[:, :, -1].max(1) - tr[:, :, 0].min(1)).mean())}
            for L in range(nl):
                rec[f"L{L}_{widths[L]}->{widths[L+1]}"] = {"work_mean": float(d[:, :, 2 * L].mean()),
                                                          "work_max": float(d[:, :, 2 * L].max()),
                                                          "barrier_mean": float(d[:, :, 2 * L + 1].mean())}
            out[f"l{lv}b{b}"] = rec
            buf[:] = 0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
