"""Shader clock under sustained load (calibration aid, not a test): runs one workload back to back for SECONDS
while the caller polls the SMI, and prints the workload's rate.
    python scripts/clock_probe.py {hipblaslt|lsplit} [SECONDS]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib  # noqa: E402
from genpose2_amd.fus_encoder import pack_split_linear  # noqa: E402


def vp(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def main():
    mode = sys.argv[1]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    dev = "cuda:0"
    m, k, n = 16384, 1024, 4096
    if mode == "hipblaslt":
        x = torch.randn(m, k, device=dev, dtype=torch.float16)
        w = torch.randn(n, k, device=dev, dtype=torch.float16)

        def run():
            torch.matmul(x, w.t())
        flop = 2 * m * k * n
    else:
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rng = np.random.default_rng(0)
        x = torch.from_numpy(rng.normal(size=(m, k)).astype(np.float32)).to(dev)
        wh = torch.from_numpy(pack_split_linear((rng.normal(size=(n, k)) / np.sqrt(k)).astype(np.float32))).to(dev)
        b = torch.zeros(n, device=dev)
        y = torch.empty(m, n, device=dev)
        rmax = x.abs().amax(1).contiguous()

        def run():
            _lib.check(lib.gp_linear_split(vp(x), k, m, k, vp(wh), vp(b), n, 1, vp(y), n, vp(rmax), 1, None, st), "ls")
        flop = 2 * m * k * n
    run()
    torch.cuda.synchronize()
    t0 = time.time()
    windows = []
    while time.time() - t0 < secs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        windows.append(round(us, 1))
    print(json.dumps({"mode": mode, "us_per_call_windows": windows, "tflops_first": round(flop / windows[0] / 1e6, 1),
                      "tflops_last": round(flop / windows[-1] / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
