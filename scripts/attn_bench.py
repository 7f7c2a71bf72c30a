"""Per-level timing of the fused encoder's attention (gp_relpe_bias + gp_mha_attention) at the north-star
batch (B objects; levels n = 512/256/128/64 tokens, d = 96/256/512/1024). Prints one JSON line."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib  # noqa: E402
from genpose2_amd._lib import check  # noqa: E402


def vp(t):
    return ctypes.c_void_p(None if t is None else t.data_ptr())


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    lib = _lib.load()
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    pe = torch.randn(1024, device=dev, generator=g) * 0.3   # gp_relpe_bias reads 824 floats
    res = {"B": B}
    for n, d in ((512, 96), (256, 256), (128, 512), (64, 1024)):
        qkv = torch.randn(B, n, 3 * d, device=dev, generator=g)
        xyz = torch.rand(B, n, 3, device=dev, generator=g)
        bias = torch.empty(B, 8, n, n, device=dev)
        out = torch.empty(B, n, d, device=dev)
        tb = timed(lambda: check(lib.gp_relpe_bias(vp(pe), vp(xyz), B, n, vp(bias), st), "relpe"), reps)
        ta = timed(lambda: check(lib.gp_mha_attention(vp(qkv), vp(bias), B, n, d, vp(out), None, st), "mha"), reps)
        flops = 4.0 * B * 8 * n * n * (d // 8)
        res[f"n{n}"] = {"relpe_ms": round(tb, 4), "attn_ms": round(ta, 4),
                        "attn_tflops": round(flops / ta / 1e9, 2),
                        "bias_gbs": round(B * 8 * n * n * 4 / ta / 1e6, 1)}
        del qkv, xyz, bias, out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
