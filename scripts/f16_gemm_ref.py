"""Practical f16 MFMA ceiling on this box: torch.matmul (hipBLASLt) in f16 on the split token linears' shapes,
TFLOP/s of the plain GEMM (calibration aid for linear_split_kernel, whose split-f16 form runs three such
products per weight: not a test).   usage: python scripts/f16_gemm_ref.py"""
import json

import torch

SHAPES = [("L3.linear1", 16384, 1024, 4096), ("L3.linear2", 16384, 4096, 1024), ("L2.linear1", 32768, 512, 2048),
          ("L1.linear1", 65536, 256, 1024), ("big", 16384, 8192, 8192)]


def main():
    dev = "cuda:0"
    for name, m, k, n in SHAPES:
        x = torch.randn(m, k, device=dev, dtype=torch.float16)
        w = torch.randn(n, k, device=dev, dtype=torch.float16)
        for _ in range(3):
            torch.matmul(x, w.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            torch.matmul(x, w.t())
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(json.dumps({"shape": name, "m": m, "k": k, "n": n, "us": round(us, 1),
                          "tflops": round(2 * m * k * n / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
