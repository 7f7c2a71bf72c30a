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
_KIND_ID = {"score": 1, "energy": 2, "scale": 3}


# ---------------------------------------------------------------- manifest
def manifest(kind: str) -> List[Tuple[str, Tuple[int, ...], str]]:
    """(key, shape, init rule) for every tensor of the model selected by ``kind``."""
    out: List[Tuple[str, Tuple[int, ...], str]] = []
    if kind in ("score", "energy"):
        for lv, branches in enumerate(arch.sa_branches()):
            for br in branches:
                w = br.widths
                for i in range(len(w) - 1):
                    p = f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}"
                    out.append((f"{p}.conv.weight", (w[i + 1], w[i], 1, 1), "conv"))
                    for nm, rule in (("weight", "bn_gamma"), ("bias", "bn_beta"),
                                     ("running_mean", "bn_mean"), ("running_var", "bn_var")):
                        out.append((f"{p}.bn.bn.{nm}", (w[i + 1],), rule))
                    out.append((f"{p}.bn.bn.num_batches_tracked", (), "zero_i64"))
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


def encoder_layers(sd: StateDict) -> List[List[List[Tuple[np.ndarray, np.ndarray]]]]:
    """[level][branch][layer] -> (W_folded (out,in), b_folded (out,))."""
    out = []
    for lv, branches in enumerate(arch.sa_branches()):
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
