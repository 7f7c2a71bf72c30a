"""Where do the workgroups of a CU-masked stream run? Builds scripts/cu_probe.hip, creates streams with
hipExtStreamCreateWithCUMask and reports, per XCC, the distinct (SE, SH, CU) slots the probe's workgroups
ran on. Masks: "all"; "v" = bits 0..15 plus bit 32x+16 for each x (contiguous bit->XCC numbering puts 17
CUs on XCC 0 and 1 on the others; XCC-interleaved numbering 10 and 2); then, only if the numbering is
interleaved, the split this repo would use (bits 0..199 / 200..255: 25 / 7 CUs per XCC). Prints JSON."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "..", "gpurun_out", "cu_probe.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                           os.path.join(HERE, "cu_probe.hip")])


def mask_words(bits):
    w = [0] * 8
    for i in bits:
        w[i // 32] |= 1 << (i % 32)
    return (ctypes.c_uint32 * 8)(*w)


def run(hip, probe, bits, blocks=2048, spin=2_000_000):
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), 8, mask_words(bits))
    assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
    got = (ctypes.c_uint32 * 8)()
    hip.hipExtStreamGetCUMask(st, 8, got)
    out = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    assert probe.cu_probe(ctypes.c_void_p(out.data_ptr()), blocks, ctypes.c_longlong(spin), st) == 0
    assert hip.hipStreamSynchronize(st) == 0
    hip.hipStreamDestroy(st)
    v = out.cpu().numpy().astype("uint32").reshape(-1, 2)
    per = {}
    for hw, xcc in v:
        slot = ((hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)
        per.setdefault(int(xcc), set()).add(tuple(int(s) for s in slot))
    return {"mask_words": [hex(x) for x in got], "cus_per_xcc": {x: len(s) for x, s in sorted(per.items())},
            "slots": {x: sorted(s) for x, s in sorted(per.items())}}


def main():
    build()
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    probe = ctypes.CDLL(SO)
    probe.cu_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]
    res = {"all": run(hip, probe, range(256))}
    res["v"] = run(hip, probe, list(range(16)) + [32 * x + 16 for x in range(8)])
    print(json.dumps({k: {"cus_per_xcc": r["cus_per_xcc"], "mask": r["mask_words"]} for k, r in res.items()}),
          flush=True)
    c = res["v"]["cus_per_xcc"]
    if len(c) == 8 and all(n == 2 for x, n in c.items() if x != 0) and c.get(0) == 10:
        res["pc200"] = run(hip, probe, range(200))
        res["side56"] = run(hip, probe, range(200, 256))
        print(json.dumps({k: r["cus_per_xcc"] for k, r in res.items()}), flush=True)
    json.dump({k: {kk: (vv if kk != "slots" else {str(a): b for a, b in vv.items()}) for kk, vv in r.items()}
               for k, r in res.items()}, open(os.path.join(HERE, "..", "gpurun_out", "cu_mask_probe.json"), "w"))


if __name__ == "__main__":
    sys.exit(main())
