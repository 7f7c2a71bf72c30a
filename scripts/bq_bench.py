"""Ball-query timing at level-0 shapes (B=256, 512 centroids over 1024 points) for a few radii:
how much of the launch is the scan (small radius: few hits, full scan) vs the early exit."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib, synthetic  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    B, N, M = 256, 1024, 512
    pts_np, _ = synthetic.make_batch(4, B, N)
    pts = torch.from_numpy(pts_np).to(dev)
    cent = pts[:, :M].contiguous()
    out = {"extent": float((pts.amax(1) - pts.amin(1)).mean())}
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for r, ns in [(0.01, 16), (0.02, 32), (0.1, 32), (10.0, 32)]:
        idx = torch.zeros(B, M, ns, dtype=torch.int32, device=dev)

        def run():
            _lib.check(lib.gp_ball_query(B, N, M, ctypes.c_float(r), ns, ctypes.c_void_p(cent.data_ptr()),
                                         ctypes.c_void_p(pts.data_ptr()), ctypes.c_void_p(idx.data_ptr()), s))
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        out[f"r{r}_ns{ns}_us"] = (time.perf_counter() - t0) / 20 * 1e6
        out[f"r{r}_hits_mean"] = float((idx != idx[..., :1]).sum(-1).float().mean() + 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
