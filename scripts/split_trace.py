"""Phase breakdown of sa_split_kernel (encoder levels 2-3, split-f16) from in-kernel s_memtime marks
(tuning aid). Needs the trace build:
    make -C genpose2_amd/csrc OUT=../../variants/satrace/libgenpose_hip.so BUILD=../../variants/satrace/build EXTRA=-DSA_TRACE
    GENPOSE_HIP_LIB=variants/satrace/libgenpose_hip.so python scripts/split_trace.py [B]
Marks per wave: 0 start, 1 staged + barrier, 2 layer-0 gather + barrier, 3 layer-1 stream, 4 column-max barrier,
5 layer-1 planes written, 6 layer-2 barrier, 7 end (layer-2 stream + pooling)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402

NAMES = ["stage+bar", "gather0+bar", "l1_stream", "colmax+bar", "l1_planes", "l2_bar", "l2_stream+pool"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    lib = _lib.load()
    fn = lib.gp_debug_split_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p]
    agent = PoseNet(GenPoseConfig(device="cuda:0")).eval()
    pts, _ = synthetic.make_batch(9, B, 1024)
    p = torch.from_numpy(pts).to("cuda:0")
    agent.encoder.forward(p)
    out = {"B": B}
    for lv in (2, 3):
        for b in range(2):
            assert fn(lv * 2 + b, None) == 0
            agent.encoder.forward(p)
            torch.cuda.synchronize()
            buf = np.zeros(8192 * 8 * 8, np.uint64)
            assert fn(-1, buf.ctypes.data) == 0
            tr = buf.reshape(8192, 8, 8).astype(np.int64)
            used = tr[:, 0, 0] != 0
            tr = tr[used]
            st = tr[:, :, 0].min(1)
            crit = {}
            prev = st
            for k, nm in enumerate(NAMES, start=1):
                m = tr[:, :, k].max(1)       # the last wave past mark k (barriers align the waves)
                crit[nm] = float((m - prev).mean())
                prev = m
            out[f"l{lv}b{b}"] = {"wgs_traced": int(used.sum()), "critical_path_mean": crit,
                                 "lifetime_mean": float((tr[:, :, 7].max(1) - st).mean())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
