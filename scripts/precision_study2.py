"""CPU study: split-bf16 MFMA arithmetic on the per-candidate GEMMs only (pose_encoder.2 and the
pose block of head layer 1 -- what the PC kernel streams per step), everything else fp32 as the
kernel computes it, run through the PC sampler against the reference's golden trajectories.

Emulation of v_mfma_f32_16x16x32_bf16: products of bf16 planes are exact, each 32-deep k chunk is
summed exactly (float64) and added to the fp32 accumulator with one rounding; the plane products of a
chunk are accumulated smallest first. A variant "wXaY" splits weights into X bf16 planes and
activations into Y, and keeps the products whose plane indices sum below a cut.
Usage: python scripts/precision_study2.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle  # noqa: E402
from genpose2_amd import arch, weights  # noqa: E402

F32 = np.float32


def bf16(a):
    a = np.ascontiguousarray(a, np.float32)
    b = a.view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def split(a, n):
    out, r = [], a.astype(F32)
    for _ in range(n):
        h = bf16(r)
        out.append(h)
        r = (r - h).astype(F32)
    return out


def split16(a, n):
    out, r = [], a.astype(F32)
    for _ in range(n):
        h = r.astype(np.float16).astype(F32)
        out.append(h)
        r = (r - h).astype(F32)
    return out


def pow2_scale(m):
    """2**e with m * 2**e in [2**14, 2**15): the f16 planes keep their 11 bits for the large values."""
    e = np.where(m > 0, 14 - np.floor(np.log2(np.where(m > 0, m, 1))), 0)
    return np.exp2(e).astype(F32)


def mm_split(x, w, nw, nx, pairs, kind="bf16"):
    """x (R,K) @ w(N,K).T with split MFMAs, fp32 accumulation per 32-deep chunk. kind "f16": f16
    planes of exactly power-of-two scaled operands (per row for x, per layer for w)."""
    if kind == "f16":
        sx = pow2_scale(np.abs(x).max(axis=1))[:, None]
        sw = pow2_scale(np.abs(w).max())
        out = mm_split((x * sx).astype(F32), (w * sw).astype(F32), nw, nx, pairs, "f16raw")
        return (out * (F32(1) / (sx * sw)).astype(F32)).astype(F32)
    sp = split16 if kind == "f16raw" else split
    xs, ws = sp(x, nx), sp(w, nw)
    R, K = x.shape
    acc = np.zeros((R, w.shape[0]), F32)
    for k0 in range(0, K, 32):
        sl = slice(k0, min(K, k0 + 32))
        chunk = np.zeros((R, w.shape[0]), np.float64)
        for i, j in sorted(pairs, key=lambda p: -(p[0] + p[1])):   # smallest products first
            chunk += xs[i][:, sl].astype(np.float64) @ ws[j][:, sl].astype(np.float64).T
        acc = (acc + chunk.astype(F32)).astype(F32)
    return acc


MODE = None


def head_features(sd, pts_feat, pose, t):
    n = "pose_score_net"
    t = np.asarray(t, dtype=F32).reshape(-1, 1)
    W = sd[f"{n}.t_encoder.0.W"].astype(F32)
    x_proj = (t[:, 0][:, None] * W[None, :]) * F32(2) * F32(np.pi)
    t_emb = np.concatenate([np.sin(x_proj), np.cos(x_proj)], axis=-1).astype(F32)
    t_feat = np.maximum(oracle._lin(t_emb, sd[f"{n}.t_encoder.1.weight"], sd[f"{n}.t_encoder.1.bias"]), 0)
    h = np.maximum(oracle._lin(pose.astype(F32), sd[f"{n}.pose_encoder.0.weight"], sd[f"{n}.pose_encoder.0.bias"]), 0)
    w2, b2 = sd[f"{n}.pose_encoder.2.weight"].astype(F32), sd[f"{n}.pose_encoder.2.bias"].astype(F32)
    if MODE is None:
        pose_feat = np.maximum(oracle._lin(h, w2, b2), 0)
    else:
        pose_feat = np.maximum((mm_split(h, w2, *MODE) + b2).astype(F32), 0)
    outs = []
    P = pts_feat.shape[1]
    for hn in arch.HEAD_NAMES:
        W1 = sd[f"{n}.{hn}.0.weight"].astype(F32)
        b1 = sd[f"{n}.{hn}.0.bias"].astype(F32)
        fixed = (np.concatenate([pts_feat.astype(F32), t_feat], axis=-1) @ W1[:, :P + 128].T + b1).astype(F32)
        if MODE is None:
            pose_part = (pose_feat @ W1[:, P + 128:].T).astype(F32)
        else:
            pose_part = mm_split(pose_feat, W1[:, P + 128:], *MODE)
        u = np.maximum((fixed + pose_part).astype(F32), 0)
        outs.append(oracle._lin(u, sd[f"{n}.{hn}.2.weight"], sd[f"{n}.{hn}.2.bias"]))
    return np.concatenate(outs, axis=-1).astype(F32), oracle.ve_sigma(t)


oracle.head_features = head_features


def pairs(nw, nx, cut):
    return [(i, j) for i in range(nx) for j in range(nw) if i + j < cut]


VARIANTS = [("fp32", None),
            ("w2a2 3 products (bf16x3)", (2, 2, pairs(2, 2, 2))),
            ("w2a3 5 products", (2, 3, pairs(2, 3, 3))),
            ("w2a3 6 products", (2, 3, pairs(2, 3, 4))),
            ("w3a3 6 products (bf16x6)", (3, 3, pairs(3, 3, 3)))]
if os.environ.get("STUDY_F16"):   # f16 hi/lo planes of power-of-two scaled operands
    VARIANTS = [("fp32", None), ("f16 w2a2 3 products", (2, 2, pairs(2, 2, 2), "f16")),
                ("f16 w2a2 4 products", (2, 2, pairs(2, 2, 3), "f16"))]


def main():
    import conftest
    sd = weights.synthetic_state_dict("score")
    global MODE
    for name in ["pc_k50_t20", "pc_k10_t100"]:
        g = conftest.golden(name)
        K, T = int(g["K"]), int(g["T"])
        for label, mode in VARIANTS:
            MODE = mode
            pose, q, feat, ex = oracle.pred_func(sd, g["pts"], g["pts_center"], K, T, "pc", g["prior"], g["z1"], g["z2"])
            ref = g["pred_pose"]
            rot = np.abs(pose[..., :6] - ref[..., :6]).max()
            tr = np.abs(pose[..., 6:] - ref[..., 6:]).max() / np.abs(ref[..., 6:]).max()
            print(f"{name:12s} {label:26s} rot_abs {rot:.2e} trans_rel {tr:.2e}", flush=True)


if __name__ == "__main__":
    main()
