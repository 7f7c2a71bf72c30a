"""Host-side packing of model parameters into the layouts the HIP kernels stream.

MFMA A-fragment order (v_mfma_f32_16x16x4_f32, weights as the A operand, output channels as
MFMA rows): for a layer W (n_out, k_in) padded to (16*NT, 16*KG),

    packed[T][g][lane][j] = W[16*T + (lane & 15)][16*g + 4*(lane >> 4) + j]

so that lane l's float4 for k-group g feeds the 4 MFMAs of k-steps 4g..4g+3 and one
wave-instruction reads 1 KiB contiguously. The same channel order (c = 16g + 4q + j) is the
accumulator's native layout, so a layer's output tile T is the next layer's k-group T.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from . import arch, weights


def pad16(v: int) -> int:
    return (v + 15) // 16 * 16


def pack_a_fragments(w: np.ndarray, k_pad: Optional[int] = None, n_pad: Optional[int] = None) -> np.ndarray:
    """(n_out, k_in) -> flat float32 array in A-fragment order (see module docstring)."""
    n_out, k_in = w.shape
    NP = pad16(n_out) if n_pad is None else n_pad
    KP = pad16(k_in) if k_pad is None else k_pad
    wp = np.zeros((NP, KP), np.float32)
    wp[:n_out, :k_in] = w
    NT, KG = NP // 16, KP // 16
    t = wp.reshape(NT, 16, KG, 4, 4)          # [T][i][g][q][j]
    return np.ascontiguousarray(t.transpose(0, 2, 3, 1, 4)).reshape(-1)   # [T][g][q][i][j]


def unpack_a_fragments(p: np.ndarray, n_pad: int, k_pad: int) -> np.ndarray:
    t = p.reshape(n_pad // 16, k_pad // 16, 4, 16, 4).transpose(0, 3, 1, 2, 4)
    return t.reshape(n_pad, k_pad)


def pad_vec(b: np.ndarray, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    out[: b.shape[0]] = b
    return out


# ---------------------------------------------------------------- encoder
def pack_encoder(sd: weights.StateDict) -> Tuple[np.ndarray, np.ndarray]:
    """All SA layers, BN folded, into one flat float32 buffer + int64 offsets [5][2][3][2].

    Layer 0 of each branch has its input channels permuted from the reference's
    [xyz(3) | feats(C)] (pointnet2_utils.py:287-289) to [feats(C) | xyz(3) | 0...] with
    K padded to C + 16, matching the kernel's gathered B operand."""
    folded = weights.encoder_layers(sd)
    chunks: List[np.ndarray] = []
    offsets = np.full((5, 2, 3, 2), -1, np.int64)
    pos = 0

    def add(a: np.ndarray) -> int:
        nonlocal pos
        o = pos
        a = np.ascontiguousarray(a, np.float32).reshape(-1)
        chunks.append(a)
        pos += a.size
        # keep every tensor 16-byte aligned
        padn = (-pos) % 4
        if padn:
            chunks.append(np.zeros(padn, np.float32))
            pos += padn
        return o

    for lv, branches in enumerate(arch.sa_branches()):
        c_prev = 0 if lv == 0 else arch.level_out_channels(lv - 1)
        for br in branches:
            for i, (W, b) in enumerate(folded[lv][br.branch]):
                if i == 0:
                    wp = np.zeros((W.shape[0], c_prev + 16), np.float32)
                    wp[:, :c_prev] = W[:, 3:]
                    wp[:, c_prev:c_prev + 3] = W[:, :3]
                    packed = pack_a_fragments(wp, k_pad=c_prev + 16)
                else:
                    packed = pack_a_fragments(W)
                offsets[lv, br.branch, i, 0] = add(packed)
                offsets[lv, br.branch, i, 1] = add(pad_vec(b, pad16(W.shape[0])))
    return np.concatenate(chunks), offsets


# ---------------------------------------------------------------- score / energy heads
HEAD_FIELDS = ("pe0_w", "pe0_b", "pe2_w", "pe2_b", "h1p_w", "h2_w", "h2_b", "h1pts_t", "h1_b",
               "gfp_w", "te_w_t", "te_b", "h1t_t")


def pack_heads(sd: weights.StateDict) -> Dict[str, np.ndarray]:
    p = weights.head_params(sd)
    H = arch.HEAD_HID
    out = {
        "pe0_w": pack_a_fragments(p["pe0_w"], k_pad=16),
        "pe0_b": p["pe0_b"],
        "pe2_w": pack_a_fragments(p["pe2_w"]),
        "pe2_b": p["pe2_b"],
        "h1p_w": pack_a_fragments(p["h1_pose"].reshape(3 * H, arch.POSE_HID)),
        "h2_w": p["h2_w"].reshape(-1),
        "h2_b": p["h2_b"].reshape(-1),
        "h1pts_t": np.ascontiguousarray(p["h1_pts"].reshape(3 * H, arch.PTS_FEAT_DIM).T),
        "h1_b": p["h1_b"].reshape(-1),
        "gfp_w": p["gfp_w"],
        "te_w_t": np.ascontiguousarray(p["te_w"].T),
        "te_b": p["te_b"],
        "h1t_t": np.ascontiguousarray(p["h1_t"].reshape(3 * H, arch.T_EMB).T),
    }
    return {k: np.ascontiguousarray(v, np.float32) for k, v in out.items()}


SCALE_FIELDS = ("ae0_w", "ae0_b", "ae2_w", "ae2_b", "ft0_w", "ft0_b", "ft2_w", "ft2_b")


def pack_scale(sd: weights.StateDict) -> Dict[str, np.ndarray]:
    m = {"ae0": "axes_encoder.0", "ae2": "axes_encoder.2", "ft0": "fusion_tail_length.0",
         "ft2": "fusion_tail_length.2"}
    out = {}
    for short, key in m.items():
        out[f"{short}_w"] = np.ascontiguousarray(sd[f"{key}.weight"], np.float32)
        out[f"{short}_b"] = np.ascontiguousarray(sd[f"{key}.bias"], np.float32)
    return out
