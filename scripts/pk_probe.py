"""Which instruction pattern of the level-0 projection goes wrong under multi-process load (scripts/pk_probe.hip).

Victim processes run the projection's arithmetic over 1M points, REPS times per variant, and compare every
run with the first bit for bit; load processes keep the GPU's matrix pipes and LDS busy (or run the victim
too). Variants: x3 / x1 (one 12-byte coordinate load vs three 4-byte loads) x pk / nopk (the compiler's
packed-FP32 instructions or none: -fno-slp-vectorize). Prints one JSON line per (process, variant) with the
number of runs that differed and, for the first differing run, which coordinate the wrong rows were computed
without (a least-squares fit of the row to the weights).
usage: python scripts/pk_probe.py [--victims 2] [--loads 2] [--reps 200]
"""
import argparse
import ctypes
import json
import os
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
DEV = "cuda:0"


def victim(w, reps, out_q):
    torch.cuda.set_device(0)
    libs = {"pk": ctypes.CDLL(os.path.join(HERE, "libpkprobe.so")),
            "nopk": ctypes.CDLL(os.path.join(HERE, "libpkprobe_nopk.so"))}
    rng = np.random.default_rng(w)
    npts = 1 << 20
    xyz = torch.from_numpy(rng.normal(size=(npts, 3)).astype(np.float32) * 0.1).to(DEV)
    wt = torch.from_numpy(rng.normal(size=(32, 4)).astype(np.float32)).to(DEV)
    b = torch.from_numpy(rng.normal(size=32).astype(np.float32) * 0.05).to(DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for lib_name, lib in libs.items():
        for var, vname in ((0, "x3"), (1, "x1")):
            out = torch.empty(npts, 32, device=DEV)
            first, bad, info = None, 0, None
            for r in range(reps):
                out.fill_(float("nan"))
                assert lib.pk_proj(var, ctypes.c_void_p(xyz.data_ptr()), ctypes.c_void_p(wt.data_ptr()),
                                   ctypes.c_void_p(b.data_ptr()), npts, ctypes.c_void_p(out.data_ptr()), st) == 0
                if first is None:
                    first = out.clone()
                    continue
                if not torch.equal(out, first):
                    bad += 1
                    if info is None:
                        rows = torch.nonzero((out != first).any(1)).flatten()[:64].cpu().numpy()
                        o = out.cpu().numpy()[rows].astype(np.float64)
                        W = wt.cpu().numpy().astype(np.float64)[:, :3]
                        bb = b.cpu().numpy().astype(np.float64)
                        X = xyz.cpu().numpy()[rows].astype(np.float64)
                        fits = []
                        for i in range(min(8, len(rows))):
                            xf = np.linalg.lstsq(W, o[i] - bb, rcond=None)[0]
                            fits.append([round(float(v), 5) for v in (X[i] - xf)])
                        info = {"rows": rows[:16].tolist(), "x_true_minus_fit": fits}
            res.append({"proc": w, "lib": lib_name, "variant": vname, "reps": reps, "differing_runs": bad, "first_bad": info})
    out_q.put(res)


def loader(w, seconds):
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.join(HERE, "libpkprobe.so"))
    sink = torch.empty(256, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    t_end = time.time() + seconds
    while time.time() < t_end:
        for _ in range(8):
            lib.pk_load(2048, 4096, ctypes.c_void_p(sink.data_ptr()), st)
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--victims", type=int, default=2)
    ap.add_argument("--loads", type=int, default=2)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--load-seconds", type=float, default=60)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=loader, args=(i, args.load_seconds)) for i in range(args.loads)]
    procs += [ctx.Process(target=victim, args=(i, args.reps, q)) for i in range(args.victims)]
    for p in procs:
        p.start()
    for _ in range(args.victims):
        for rec in q.get():
            print(json.dumps(rec), flush=True)
    for p in procs:
        p.join()


if __name__ == "__main__":
    main()
