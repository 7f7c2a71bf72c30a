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
ENC_SPLIT_LEVELS = (1, 2, 3, 4)   # levels whose every layer also gets split-f16 planes: layer 0 of levels 1-3 and
                                  # both GroupAll layers run as token GEMMs (tok_split_gemm_kernel), layers 1-2 of
                                  # level 1 in sa_narrow_split_kernel, of levels 2-3 in sa_split_kernel; level 0
                                  # has planes for layers 1-2 (its 32-wide branch in sa_narrow_mixed_kernel)


def enc_split_layer(lv: int, i: int) -> bool:
    """Whether layer i of level lv carries split-f16 planes."""
    return lv in ENC_SPLIT_LEVELS or i >= 1


def pad32(v: int) -> int:
    return (v + 31) // 32 * 32


def pack_encoder(sd: weights.StateDict, levels=None) -> Tuple[np.ndarray, np.ndarray]:
    """All SA layers, BN folded, into one flat float32 buffer + int64 table [5][2][3][4]:
    [0] offset of the fp32 A fragments, [1] offset of the bias (padded to 32), [2] offset of the
    split-f16 planes (enc_split_layer: every layer of levels 1-4 and layers 1-2 of level 0; -1 for
    level 0's layer 0),
    [3] their power-of-two exponent.

    Layer 0 of each branch has its input channels permuted from the reference's
    [xyz(3) | feats(C)] (pointnet2_utils.py:287-289) to [feats(C) | xyz(3) | 0...] with
    K padded to C + 16, matching the kernel's gathered B operand. The split planes
    (pack_h16_fragments) pad every output count and input depth to 32, the chunk of
    v_mfma_f32_16x16x32_f16 (level 2: 196 channels -> 224)."""
    levels = arch.sa_branches() if levels is None else levels
    folded = weights.encoder_layers(sd, levels)
    chunks: List[np.ndarray] = []
    offsets = np.full((5, 2, 3, 4), -1, np.int64)
    pos = 0

    def add(a: np.ndarray) -> int:
        nonlocal pos
        o = pos
        a = np.ascontiguousarray(a).reshape(-1)
        if a.dtype != np.float32:
            a = a.view(np.float32)     # int32 words of the f16 planes, stored bit for bit
        chunks.append(a)
        pos += a.size
        # keep every tensor 16-byte aligned
        padn = (-pos) % 4
        if padn:
            chunks.append(np.zeros(padn, np.float32))
            pos += padn
        return o

    for lv, branches in enumerate(levels):
        c_prev = branches[0].widths[0] - 3      # input feature channels (the level-0 image features: 384)
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
                offsets[lv, br.branch, i, 1] = add(pad_vec(b, pad32(W.shape[0])))
                if enc_split_layer(lv, i):
                    if i == 0:   # layer 0: the [feats | xyz | 0...] order of the fp32 fragments
                        wq = np.zeros((pad32(W.shape[0]), pad32(c_prev + 3)), np.float32)
                        wq[:W.shape[0], :c_prev] = W[:, 3:]
                        wq[:W.shape[0], c_prev:c_prev + 3] = W[:, :3]
                    else:
                        wq = np.zeros((pad32(W.shape[0]), pad32(W.shape[1])), np.float32)
                        wq[:W.shape[0], :W.shape[1]] = W
                    e = split_exponent(W)
                    offsets[lv, br.branch, i, 2] = add(pack_h16_fragments(wq, e))
                    offsets[lv, br.branch, i, 3] = e
    return np.concatenate(chunks), offsets


# ---------------------------------------------------------------- score / energy heads
HEAD_FIELDS = ("pe0_w", "pe0_b", "pe2_w", "pe2_b", "h1p_w", "h2_w", "h2_b", "h1pts_t", "h1_b",
               "gfp_w", "te_w_t", "te_b", "h1t_t", "pe2_h", "h1p_h", "hsc")


def split_exponent(w: np.ndarray) -> int:
    """e with max|w| * 2**e in [2**14, 2**15): the f16 planes of w * 2**e keep 11 bits and cannot overflow."""
    m = float(np.abs(w).max())
    return 14 - int(np.floor(np.log2(m))) if m > 0 else 0


def pack_h16_fragments(w: np.ndarray, e: int, planes: int = 2) -> np.ndarray:
    """(n_out, k_in) -> bits (int32 words) of the f16 planes of x = w * 2**e in the A-operand order of
    v_mfma_f32_16x16x32_f16. planes = 2: hi = f16(x), lo = f16(x - hi) (the encoder's split-f16
    GEMMs); planes = 3: hi, mid = f16(x - hi), lo = f16(x - hi - mid), every bit of x (the head
    trunk's f16x3 GEMMs, gp_head.h):

        packed[T][c][plane][lane][j] = plane(W[16T + (lane & 15)][32c + 16*(j // 4) + 4*(lane >> 4) + j % 4])

    i.e. chunk c pairs the fp32 accumulator tiles 2c and 2c+1 of the producing layer, so its output
    feeds the B operand without moving data between lanes. One (T, c, plane) is 1 KiB."""
    n_out, k_in = w.shape
    assert n_out % 16 == 0 and k_in % 32 == 0, (n_out, k_in)
    assert planes in (2, 3), planes
    r = (np.asarray(w, np.float32) * np.float32(2.0 ** e)).astype(np.float32)
    ps = []
    for _ in range(planes):
        h = r.astype(np.float16)
        ps.append(h)
        r = (r - h.astype(np.float32)).astype(np.float32)   # exact: r and h agree in their leading bits
    NT, KC = n_out // 16, k_in // 32

    def frag(p):   # [T][i][c][half][q][j4] -> [T][c][q][i][half][j4]: lane = 16q + i, j = 4*half + j4
        return p.reshape(NT, 16, KC, 2, 4, 4).transpose(0, 2, 4, 1, 3, 5)
    out = np.stack([frag(p) for p in ps], axis=2)
    # int32 words (two f16 each): every torch.distributed backend broadcasts int32
    return np.ascontiguousarray(out).reshape(-1).view(np.int32)


HEAD_PLANES = 3   # f16 planes per weight of the head trunk's GEMMs (pe2_h, h1p_h)


def split_constants(p: Dict[str, np.ndarray], e2: int, eh: int) -> np.ndarray:
    """hsc: bounds the split trunk derives its per-candidate activation exponents from
    (|pose_encoder.0 out| <= A0*max|x| + B0, |pose_encoder.2 out| <= A2*bound0 + B2) + weight exponents."""
    a0 = np.abs(p["pe0_w"].astype(np.float64)).sum(1).max()
    a2 = np.abs(p["pe2_w"].astype(np.float64)).sum(1).max()
    b0, b2 = np.abs(p["pe0_b"]).max(), np.abs(p["pe2_b"]).max()
    # rounded up so that the fp32 values stay bounds
    return np.nextafter(np.array([a0, b0, a2, b2], np.float32), np.float32(np.inf)).tolist() + [e2, eh, 0, 0]


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
    out = {k: np.ascontiguousarray(v, np.float32) for k, v in out.items()}
    h1_pose = p["h1_pose"].reshape(3 * H, arch.POSE_HID)
    e2, eh = split_exponent(p["pe2_w"]), split_exponent(h1_pose)
    out["pe2_h"] = pack_h16_fragments(p["pe2_w"], e2, HEAD_PLANES)
    out["h1p_h"] = pack_h16_fragments(h1_pose, eh, HEAD_PLANES)
    out["hsc"] = np.asarray(split_constants(p, e2, eh), np.float32)
    return out


SCALE_FIELDS = ("ae0_w", "ae0_b", "ae2_w", "ae2_b", "ft0_w", "ft0_b", "ft2_w", "ft2_b")


def pack_scale(sd: weights.StateDict) -> Dict[str, np.ndarray]:
    m = {"ae0": "axes_encoder.0", "ae2": "axes_encoder.2", "ft0": "fusion_tail_length.0",
         "ft2": "fusion_tail_length.2"}
    out = {}
    for short, key in m.items():
        out[f"{short}_w"] = np.ascontiguousarray(sd[f"{key}.weight"], np.float32)
        out[f"{short}_b"] = np.ascontiguousarray(sd[f"{key}.bias"], np.float32)
    return out
