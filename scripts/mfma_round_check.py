"""Reads scripts/mfma_round_probe's dump and compares every MFMA output with the correctly rounded
fp32 value of C + sum(a*b) (exact rational arithmetic), for v_mfma_f32_16x16x32_f16 and
v_mfma_f32_16x16x4_f32. Operand layout (gfx950): A lane l = 16*kb + i holds row i, k block kb;
B lane l = 16*kb + j holds column j, k block kb; D lane l = 16*rb + j holds rows 4*rb + v, column j.
Usage: python scripts/mfma_round_check.py gpurun_out/mfma_probe.bin [TRIALS [OUT.json]]
"""
import json
import sys
from fractions import Fraction

import numpy as np


def rn32(fr: Fraction) -> np.float32:
    """Correctly rounded fp32 of an exact rational (via float64 twice is not enough in general; use
    the neighbours of the float64 approximation)."""
    x = np.float32(float(fr))
    cands = [x, np.nextafter(x, np.float32(np.inf)), np.nextafter(x, np.float32(-np.inf))]
    return min(cands, key=lambda c: (abs(Fraction(float(c)) - fr), int(np.float32(c).view(np.uint32)) & 1))


def ulps(a: np.float32, b: np.float32) -> int:
    ia, ib = int(np.float32(a).view(np.int32)), int(np.float32(b).view(np.int32))
    ia = ia if ia >= 0 else -(ia & 0x7FFFFFFF)
    ib = ib if ib >= 0 else -(ib & 0x7FFFFFFF)
    return ia - ib


def check(name, A, B, C, D, kper):
    """A (n, 64, kper), B (n, 64, kper), C/D (n, 64, 4). Returns the summary: the ulp histogram against the
    correctly rounded result and the error relative to the largest term (C or a product) in 2^-24 units."""
    n = A.shape[0]
    hist = {}
    worst = 0
    rel = []
    for t in range(n):
        for lane in range(64):
            j, rb = lane & 15, lane >> 4
            for v in range(4):
                i = 4 * rb + v
                terms = [Fraction(float(C[t, lane, v]))]
                for kb in range(4):
                    for jj in range(kper):
                        terms.append(Fraction(float(A[t, 16 * kb + i, jj])) * Fraction(float(B[t, 16 * kb + j, jj])))
                s = sum(terms)
                big = max(abs(x) for x in terms)
                if big:
                    rel.append(float(abs(Fraction(float(D[t, lane, v])) - s) / big) * 2.0 ** 24)
                u = ulps(D[t, lane, v], rn32(s))
                hist[u] = hist.get(u, 0) + 1
                worst = max(worst, abs(u))
    tot = sum(hist.values())
    rel = np.asarray(rel)
    out = {"outputs": tot, "terms_per_output": 4 * kper + 1, "correctly_rounded_frac": hist.get(0, 0) / tot,
           "within_1ulp_frac": sum(v for k, v in hist.items() if abs(k) <= 1) / tot, "max_abs_ulp": worst,
           "err_over_max_term_2^-24": {"mean": float(rel.mean()), "p99": float(np.percentile(rel, 99)),
                                       "max": float(rel.max())}}
    print(name, json.dumps(out))
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mfma_probe.bin"
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(4), np.int32)[0])
        rd = lambda dt, cnt: np.frombuffer(f.read(np.dtype(dt).itemsize * cnt), dt)  # noqa: E731
        ha, hb = rd(np.float16, n * 512).reshape(n, 64, 8), rd(np.float16, n * 512).reshape(n, 64, 8)
        hc, hd = rd(np.float32, n * 256).reshape(n, 64, 4), rd(np.float32, n * 256).reshape(n, 64, 4)
        fa, fb = rd(np.float32, n * 64).reshape(n, 64, 1), rd(np.float32, n * 64).reshape(n, 64, 1)
        fc, fd = rd(np.float32, n * 256).reshape(n, 64, 4), rd(np.float32, n * 256).reshape(n, 64, 4)
    m = min(n, int(sys.argv[2]) if len(sys.argv) > 2 else 64)
    res = {"source": "scripts/mfma_round_probe.hip on one MI355X (gfx950), random operands with exponents "
                     "spread over 2^-6..2^6, accumulators 0 for a quarter of the trials", "trials": m,
           "v_mfma_f32_16x16x32_f16": check("16x16x32_f16", ha[:m], hb[:m], hc[:m], hd[:m], 8),
           "v_mfma_f32_16x16x4_f32": check("16x16x4_f32", fa[:m], fb[:m], fc[:m], fd[:m], 1)}
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
