"""Model parameters: seeded synthetic manifest, checkpoint loading, BN folding.

The reference ships no checkpoint for the ``--dino none`` configuration, so
parity and benchmarks run on *seeded synthetic weights*. Each state-dict tensor is drawn
from its own numpy PCG64 stream keyed by ``(seed, kind, crc32(key))``; the same code runs
here, in the oracle and on the GPU box, so the weights never have to travel.

Key names are the reference's ``model_state_dict`` keys (GFObjectPose for score/energy,
``networks/posenet.py:27-124``; ScaleNet ``networks/scalenet.py:12-31``), so a real checkpoint
saved by ``PoseNet.save_ckpt`` (``posenet_agent.py:141-169``) loads through the same path.
"""
from __future__ import annotations

import zlib
from typing import Dict, List, Tuple

import numpy as np

from . import arch

StateDict = Dict[str, np.ndarray]
_KIND_ID = {"score": 1, "energy": 2, "scale": 3, "score_pointwise": 4, "energy_pointwise": 5}


# ---------------------------------------------------------------- manifest
def _bn(prefix: str, n: int) -> List[Tuple[str, Tuple[int, ...], str]]:
    out = [(f"{prefix}.{nm}", (n,), rule) for nm, rule in
           (("weight", "bn_gamma"), ("bias", "bn_beta"), ("running_mean", "bn_mean"), ("running_var", "bn_var"))]
    return out + [(f"{prefix}.num_batches_tracked", (), "zero_i64")]


def _sa_manifest(levels) -> List[Tuple[str, Tuple[int, ...], str]]:
    out: List[Tuple[str, Tuple[int, ...], str]] = []
    for lv, branches in enumerate(levels):
        for br in branches:
            w = br.widths
            for i in range(len(w) - 1):
                p = f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}"
                out.append((f"{p}.conv.weight", (w[i + 1], w[i], 1, 1), "conv"))
                out += _bn(f"{p}.bn.bn", w[i + 1])
    return out


def fus_encoder_manifest() -> List[Tuple[str, Tuple[int, ...], str]]:
    """Pointnet2ClsMSGFus(384) (pointnet2.py:255-336): SA levels, per-level relative-PE encoders
    (attention.py:648-671) and transformer blocks (attention.py:414-506, :495-503), and the gated
    fusions of levels 1..4 (attention.py:224-279; C = the previous level's channels)."""
    out = _sa_manifest(arch.fus_sa_branches())
    H, P = arch.FUS_HEADS, arch.FUS_PE_HID
    for lv in range(arch.N_LEVELS):
        d = arch.level_out_channels(lv)
        r = f"pts_encoder.relative_pos_encoders.{lv}"
        out += [(f"{r}.distance_encoder.0.weight", (P, 1), "linear"), (f"{r}.distance_encoder.0.bias", (P,), "linear_bias:1"),
                (f"{r}.distance_encoder.2.weight", (H, P), "linear"), (f"{r}.distance_encoder.2.bias", (H,), f"linear_bias:{P}"),
                (f"{r}.direction_encoder.0.weight", (P, 3), "linear"), (f"{r}.direction_encoder.0.bias", (P,), "linear_bias:3"),
                (f"{r}.direction_encoder.2.weight", (H, P), "linear"), (f"{r}.direction_encoder.2.bias", (H,), f"linear_bias:{P}"),
                (f"{r}.fusion.weight", (H, 2 * H), "linear"), (f"{r}.fusion.bias", (H,), f"linear_bias:{2 * H}")]
    for lv in range(arch.N_LEVELS):
        d = arch.level_out_channels(lv)
        t = f"pts_encoder.transformer_blocks.{lv}"
        for nm in ("wq", "wk", "wv", "wo"):
            out += [(f"{t}.self_attn.{nm}.weight", (d, d), "linear"), (f"{t}.self_attn.{nm}.bias", (d,), f"linear_bias:{d}")]
        f = arch.FUS_FF_MULT * d
        out += [(f"{t}.linear1.weight", (f, d), "linear"), (f"{t}.linear1.bias", (f,), f"linear_bias:{d}"),
                (f"{t}.linear2.weight", (d, f), "linear"), (f"{t}.linear2.bias", (d,), f"linear_bias:{f}"),
                (f"{t}.norm1.weight", (d,), "ln_gamma"), (f"{t}.norm1.bias", (d,), "ln_beta"),
                (f"{t}.norm2.weight", (d,), "ln_gamma"), (f"{t}.norm2.bias", (d,), "ln_beta")]
    for k in range(1, arch.N_LEVELS):
        c, o = arch.level_out_channels(k - 1), arch.DINO_DIM
        c2, cr = 2 * c, (2 * c) // arch.FUS_REDUCTION
        g = f"pts_encoder.feature_fusions.{k - 1}"
        out += [(f"{g}.channel_attention.1.weight", (cr, c2, 1), "conv1d"), (f"{g}.channel_attention.1.bias", (cr,), f"linear_bias:{c2}"),
                (f"{g}.channel_attention.3.weight", (c, cr, 1), "conv1d"), (f"{g}.channel_attention.3.bias", (c,), f"linear_bias:{cr}"),
                (f"{g}.spatial_attention.0.weight", (1, 2, arch.FUS_SPATIAL_K), "conv1d"),
                (f"{g}.gate.0.weight", (c, c2, 1), "conv1d"), (f"{g}.gate.0.bias", (c,), f"linear_bias:{c2}")]
        out += _bn(f"{g}.gate.1", c)
        out += [(f"{g}.original_transform.0.weight", (c, o, 1), "conv1d"),
                (f"{g}.original_transform.0.bias", (c,), f"linear_bias:{o}")]
        out += _bn(f"{g}.original_transform.1", c)
        for m in ("downsample", "output_conv"):
            out += [(f"{g}.{m}.0.weight", (c, c, 1), "conv1d"), (f"{g}.{m}.0.bias", (c,), f"linear_bias:{c}")]
            out += _bn(f"{g}.{m}.1", c)
    return out


def img_encoder_manifest() -> List[Tuple[str, Tuple[int, ...], str]]:
    """ImgEncoder(384, 256, 16) (networks/img_encoder/img_encoder.py:7-46), the --dino pointwise model's
    image branch between the DINOv3 backbone and the patch -> point gather: layer attention
    Linear(d, d/2) -> ReLU -> Linear(d/2, 1), the relative-position embedding (900, d/4) of the geometric
    attention, the 3x3 edge conv (d/4, d, 3, 3), and the two branch weights (nn.Parameter 0.2 / 0.1)."""
    d = arch.DINO_DIM
    p = "img_encoder"
    return [(f"{p}.layer_attn.0.weight", (d // 2, d), "linear"), (f"{p}.layer_attn.0.bias", (d // 2,), f"linear_bias:{d}"),
            (f"{p}.layer_attn.2.weight", (1, d // 2), "linear"), (f"{p}.layer_attn.2.bias", (1,), f"linear_bias:{d // 2}"),
            (f"{p}.rel_pos_emb.weight", (arch.IMG_REL_EMB, d // 4), "embedding"),
            (f"{p}.edge_guide.0.weight", (d // 4, d, 3, 3), "conv1d"),
            (f"{p}.edge_guide.0.bias", (d // 4,), f"linear_bias:{d * 9}"),
            (f"{p}.geo_weight", (), "const:0.2"), (f"{p}.edge_weight", (), "const:0.1")]


def manifest(kind: str) -> List[Tuple[str, Tuple[int, ...], str]]:
    """(key, shape, init rule) for every tensor of the model selected by ``kind``.
    ``*_pointwise``: the --dino pointwise model (Pointnet2ClsMSGFus encoder, ImgEncoder, the same heads;
    the frozen DINOv3 backbone ahead of the ImgEncoder is not part of it: its weights are absent,
    SURVEY §8c)."""
    out: List[Tuple[str, Tuple[int, ...], str]] = []
    if kind in ("score", "energy", "score_pointwise", "energy_pointwise"):
        out += fus_encoder_manifest() + img_encoder_manifest() if kind.endswith("_pointwise") \
            else _sa_manifest(arch.sa_branches())
        n = "pose_score_net"
        out += [(f"{n}.pose_encoder.0.weight", (arch.POSE_HID, arch.POSE_DIM), "linear"),
                (f"{n}.pose_encoder.0.bias", (arch.POSE_HID,), "linear_bias:9"),
                (f"{n}.pose_encoder.2.weight", (arch.POSE_HID, arch.POSE_HID), "linear"),
                (f"{n}.pose_encoder.2.bias", (arch.POSE_HID,), "linear_bias:256"),
                (f"{n}.t_encoder.0.W", (arch.GFP_HALF,), "gfp"),
                (f"{n}.t_encoder.1.weight", (arch.T_EMB, arch.T_EMB), "linear"),
                (f"{n}.t_encoder.1.bias", (arch.T_EMB,), "linear_bias:128")]
        for h in arch.HEAD_NAMES:
            out += [(f"{n}.{h}.0.weight", (arch.HEAD_HID, arch.HEAD_IN), "linear"),
                    (f"{n}.{h}.0.bias", (arch.HEAD_HID,), f"linear_bias:{arch.HEAD_IN}"),
                    (f"{n}.{h}.2.weight", (3, arch.HEAD_HID), "linear"),
                    (f"{n}.{h}.2.bias", (3,), f"linear_bias:{arch.HEAD_HID}")]
    elif kind == "scale":
        e, hdim = arch.SCALE_EMB, arch.SCALE_HID
        out += [("axes_encoder.0.weight", (hdim, e), "linear"),
                ("axes_encoder.0.bias", (hdim,), f"linear_bias:{e}"),
                ("axes_encoder.2.weight", (hdim, hdim), "linear"),
                ("axes_encoder.2.bias", (hdim,), f"linear_bias:{hdim}"),
                ("fusion_tail_length.0.weight", (hdim, arch.PTS_FEAT_DIM + hdim), "linear"),
                ("fusion_tail_length.0.bias", (hdim,), f"linear_bias:{arch.PTS_FEAT_DIM + hdim}"),
                ("fusion_tail_length.2.weight", (3, hdim), "linear"),
                ("fusion_tail_length.2.bias", (3,), f"linear_bias:{hdim}")]
    else:
        raise NotImplementedError(f"kind {kind}")
    return out


def _draw(rng: np.random.Generator, shape, rule: str) -> np.ndarray:
    if rule == "conv":            # He-normal over fan_in: keeps ReLU chains O(1)
        fan_in = int(np.prod(shape[1:]))
        return rng.normal(0.0, np.sqrt(2.0 / fan_in), size=shape)
    if rule == "linear":          # torch nn.Linear default: U(+-1/sqrt(fan_in))
        a = 1.0 / np.sqrt(shape[1])
        return rng.uniform(-a, a, size=shape)
    if rule == "conv1d":          # nn.Conv1d default: U(+-1/sqrt(in * kernel))
        a = 1.0 / np.sqrt(int(np.prod(shape[1:])))
        return rng.uniform(-a, a, size=shape)
    if rule == "ln_gamma":
        return rng.uniform(0.8, 1.2, size=shape)
    if rule == "ln_beta":
        return rng.uniform(-0.1, 0.1, size=shape)
    if rule.startswith("linear_bias:"):
        a = 1.0 / np.sqrt(int(rule.split(":")[1]))
        return rng.uniform(-a, a, size=shape)
    if rule == "bn_gamma":
        return rng.uniform(0.5, 1.5, size=shape)
    if rule == "bn_beta":
        return rng.uniform(-0.2, 0.2, size=shape)
    if rule == "bn_mean":
        return rng.uniform(-0.02, 0.02, size=shape)
    if rule == "bn_var":
        return rng.uniform(0.5, 1.5, size=shape)
    if rule == "embedding":       # nn.Embedding default: N(0, 1)
        return rng.normal(0.0, 1.0, size=shape)
    if rule.startswith("const:"):  # nn.Parameter(torch.tensor(v))
        return np.full(shape, float(rule.split(":")[1]))
    if rule == "gfp":             # GaussianFourierProjection: randn(64) * 30 (scorenet.py:84)
        return rng.normal(0.0, 1.0, size=shape) * arch.GFP_SCALE
    raise ValueError(rule)


def synthetic_state_dict(kind: str, seed: int = 0) -> StateDict:
    """Deterministic synthetic weights for ``kind`` (score | energy | scale)."""
    sd: StateDict = {}
    for key, shape, rule in manifest(kind):
        if rule == "zero_i64":
            sd[key] = np.zeros(shape, dtype=np.int64)
            continue
        ss = np.random.SeedSequence([seed, _KIND_ID[kind], zlib.crc32(key.encode())])
        rng = np.random.Generator(np.random.PCG64(ss))
        sd[key] = _draw(rng, shape, rule).astype(np.float32)
    return sd


def load_checkpoint(path: str) -> StateDict:
    """``PoseNet.load_ckpt`` file format (``posenet_agent.py:171-203``), loaded safely."""
    import os
    import torch
    if not os.path.exists(path):
        raise ValueError("Checkpoint {} not exists.".format(path))
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = ckpt["model_state_dict"] if "model_state_dict" in ckpt else ckpt
    return {k.replace("module.", "", 1) if k.startswith("module.") else k: v.numpy()
            for k, v in sd.items()}


def check_keys(sd: StateDict, kind: str) -> None:
    """Strict key/shape check, like ``load_state_dict(strict=True)``."""
    want = {k: s for k, s, _ in manifest(kind)}
    missing = [k for k in want if k not in sd]
    unexpected = [k for k in sd if k not in want]
    if missing or unexpected:
        raise RuntimeError(f"Error(s) in loading state_dict: missing={missing[:5]} "
                           f"unexpected={unexpected[:5]}")
    for k, s in want.items():
        if tuple(sd[k].shape) != tuple(s):
            raise RuntimeError(f"size mismatch for {k}: {tuple(sd[k].shape)} vs {s}")


# ---------------------------------------------------------------- folding
def fold_conv_bn(sd: StateDict, prefix: str) -> Tuple[np.ndarray, np.ndarray]:
    """Conv2d 1x1 (no bias) -> BatchNorm2d(eval) folded into (W (out,in), b (out,)).

    Reference: ``_ConvBase`` conv -> bn -> relu (``pytorch_utils.py:58-106``); BN eval uses
    running stats with eps 1e-5. Folding is done in float64 then rounded once to fp32.
    """
    w = sd[f"{prefix}.conv.weight"].astype(np.float64)[:, :, 0, 0]
    g = sd[f"{prefix}.bn.bn.weight"].astype(np.float64)
    be = sd[f"{prefix}.bn.bn.bias"].astype(np.float64)
    mu = sd[f"{prefix}.bn.bn.running_mean"].astype(np.float64)
    var = sd[f"{prefix}.bn.bn.running_var"].astype(np.float64)
    scale = g / np.sqrt(var + arch.BN_EPS)
    return (w * scale[:, None]).astype(np.float32), (be - mu * scale).astype(np.float32)


def encoder_layers(sd: StateDict, levels=None) -> List[List[List[Tuple[np.ndarray, np.ndarray]]]]:
    """[level][branch][layer] -> (W_folded (out,in), b_folded (out,)); `levels` = arch.sa_branches() (default)
    or arch.fus_sa_branches() (the fused encoder's SA levels)."""
    out = []
    for lv, branches in enumerate(arch.sa_branches() if levels is None else levels):
        lvl = []
        for br in branches:
            layers = []
            for i in range(len(br.widths) - 1):
                layers.append(fold_conv_bn(sd, f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}"))
            lvl.append(layers)
        out.append(lvl)
    return out


def head_params(sd: StateDict) -> Dict[str, np.ndarray]:
    """Score/energy head tensors, with the first head layer split into its column blocks
    [pts 1024 | t 128 | pose 256] (concat order ``scorenet.py:249``/``energynet.py:155``)."""
    n = "pose_score_net"
    p: Dict[str, np.ndarray] = {
        "pe0_w": sd[f"{n}.pose_encoder.0.weight"], "pe0_b": sd[f"{n}.pose_encoder.0.bias"],
        "pe2_w": sd[f"{n}.pose_encoder.2.weight"], "pe2_b": sd[f"{n}.pose_encoder.2.bias"],
        "gfp_w": sd[f"{n}.t_encoder.0.W"],
        "te_w": sd[f"{n}.t_encoder.1.weight"], "te_b": sd[f"{n}.t_encoder.1.bias"],
    }
    P, T = arch.PTS_FEAT_DIM, arch.T_EMB
    h1 = np.stack([sd[f"{n}.{h}.0.weight"] for h in arch.HEAD_NAMES])   # (3,256,1408)
    p["h1_pts"] = np.ascontiguousarray(h1[:, :, :P])                     # (3,256,1024)
    p["h1_t"] = np.ascontiguousarray(h1[:, :, P:P + T])                  # (3,256,128)
    p["h1_pose"] = np.ascontiguousarray(h1[:, :, P + T:])                # (3,256,256)
    p["h1_b"] = np.stack([sd[f"{n}.{h}.0.bias"] for h in arch.HEAD_NAMES])   # (3,256)
    p["h2_w"] = np.stack([sd[f"{n}.{h}.2.weight"] for h in arch.HEAD_NAMES])  # (3,3,256)
    p["h2_b"] = np.stack([sd[f"{n}.{h}.2.bias"] for h in arch.HEAD_NAMES])    # (3,3)
    return {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in p.items()}


def fold_conv1d_bn(sd: StateDict, prefix: str) -> Tuple[np.ndarray, np.ndarray]:
    """Conv1d k=1 with bias -> BatchNorm1d(eval) (the Sequential(Conv1d, BatchNorm1d, act) blocks of
    GatedAttentionFusion, attention.py:262-281) folded in float64: W' = s W, b' = s (b - mean) + beta."""
    w = sd[f"{prefix}.0.weight"].astype(np.float64)[:, :, 0]
    b = sd[f"{prefix}.0.bias"].astype(np.float64)
    g = sd[f"{prefix}.1.weight"].astype(np.float64)
    be = sd[f"{prefix}.1.bias"].astype(np.float64)
    mu = sd[f"{prefix}.1.running_mean"].astype(np.float64)
    var = sd[f"{prefix}.1.running_var"].astype(np.float64)
    s = g / np.sqrt(var + arch.BN_EPS)
    return (w * s[:, None]).astype(np.float32), (s * (b - mu) + be).astype(np.float32)
