"""One-off check (not a test): gp_head_object_proj of this tree against another build of the library on the same
weights and features -- bit equality and per-call time.   usage: python scripts/cmp_object_proj.py OTHER.so [B]"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib, arch, device, weights  # noqa: E402


def main():
    other = ctypes.CDLL(sys.argv[1])
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda:0")
    heads = device.HeadModel(weights.synthetic_state_dict("score"), dev)
    feat = torch.randn(B, 1024, device=dev, generator=torch.Generator(dev).manual_seed(3))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for name, lib in (("this", _lib.load()), ("other", other)):
        lib.gp_head_object_proj.argtypes = [ctypes.POINTER(_lib.HeadWeights), ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p]
        pobj = torch.empty(B, 3 * arch.HEAD_HID, device=dev)
        for _ in range(3):
            lib.gp_head_object_proj(ctypes.byref(heads.w), ctypes.c_void_p(feat.data_ptr()), B,
                                    ctypes.c_void_p(pobj.data_ptr()), st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            lib.gp_head_object_proj(ctypes.byref(heads.w), ctypes.c_void_p(feat.data_ptr()), B,
                                    ctypes.c_void_p(pobj.data_ptr()), st)
        torch.cuda.synchronize()
        out[name] = (pobj.clone(), (time.perf_counter() - t0) / 50 * 1e6)
    print({"bit_equal": bool(torch.equal(out["this"][0], out["other"][0])), "us_this": round(out["this"][1], 1),
           "us_other": round(out["other"][1], 1), "B": B})


if __name__ == "__main__":
    main()
