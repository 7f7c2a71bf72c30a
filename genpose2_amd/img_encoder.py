"""The --dino pointwise image branch on device: ``ImgEncoder`` (networks/img_encoder/img_encoder.py:6-100) and
the patch -> point gather of ``GFObjectPose.extract_pts_feature`` (networks/posenet.py:136-192).

Input: the three DINOv3 intermediate layers the reference takes from its frozen backbone
(``self.dino.get_intermediate_layers(roi_rgb, n=[2, 6, 11], reshape=False, norm=True,
return_class_token=False)``, posenet.py:138-144), (B, 256, 384) each. The backbone itself needs a hub
checkout and weights that are not part of this build: PoseNet takes its output as
``data["dino_layers"]``, or calls a backbone module the caller sets as ``PoseNet.dino``.

Every computation is a call into libgenpose_hip.so (gp_img_encoder, gp_gather_patch_points); the host only
forms the position table once per weight load (like BN folding): ``rel_pos_emb(rel_pos_idx).sum(-1)``
with torch's own row sums, as the reference computes it.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _lib, arch, weights
from ._lib import check
from .device import require_device_tensor, stream_handle


def geo_table(sd: weights.StateDict, prefix: str = "img_encoder", grid: int = arch.IMG_GRID) -> np.ndarray:
    """(np, np) float32: [i][j] = rel_pos_emb row sum at clamp((c_j - c_i + g - 1) . (2g - 1, 1)), the
    multiplier of the geometric attention scores (img_encoder.py:17-34, 68-76)."""
    h = grid
    coords = np.stack(np.meshgrid(np.arange(h), np.arange(h), indexing="ij"), -1).reshape(-1, 2)
    rel = coords[None, :, :] - coords[:, None, :] + (h - 1)
    E = torch.from_numpy(np.ascontiguousarray(sd[f"{prefix}.rel_pos_emb.weight"], dtype=np.float32))
    idx = np.clip(rel[..., 0] * (2 * (h - 1) + 1) + rel[..., 1], 0, E.shape[0] - 1)
    return np.ascontiguousarray(E.sum(dim=-1).numpy()[idx], dtype=np.float32)


def pack_img_encoder(sd: weights.StateDict, prefix: str = "img_encoder") -> Dict[str, np.ndarray]:
    """Device buffers of gp_img_encoder2: the fp32 weights as stored, plus the layer-attention Linear and the edge
    conv (as its (d/4, 9d) im2col rows) in gp_linear_split's split-f16 layout (``*_h``)."""
    from .fus_encoder import pack_split_linear
    g = lambda k: np.ascontiguousarray(sd[f"{prefix}.{k}"], dtype=np.float32)  # noqa: E731
    out = {"la_w1": g("layer_attn.0.weight"), "la_b1": g("layer_attn.0.bias"),
           "la_w2": g("layer_attn.2.weight").reshape(-1), "geo_table": geo_table(sd, prefix),
           "conv_w": g("edge_guide.0.weight"), "conv_b": g("edge_guide.0.bias")}
    out["la_w1_h"] = pack_split_linear(out["la_w1"])
    out["conv_w_h"] = pack_split_linear(out["conv_w"].reshape(out["conv_w"].shape[0], -1))
    # position-major (k index (ky * 3 + kx) * d + channel) for gp_img_encoder3's implicit im2col GEMM
    out["conv_w_hp"] = pack_split_linear(
        np.ascontiguousarray(out["conv_w"].transpose(0, 2, 3, 1)).reshape(out["conv_w"].shape[0], -1))
    return out


def pack_img_scalars(sd: weights.StateDict, prefix: str = "img_encoder") -> np.ndarray:
    """[la_b2, relu(geo_weight), relu(edge_weight)] (host scalars of gp_img_encoder), float32."""
    v = [float(np.asarray(sd[f"{prefix}.layer_attn.2.bias"]).reshape(-1)[0]),
         max(float(sd[f"{prefix}.geo_weight"]), 0.0), max(float(sd[f"{prefix}.edge_weight"]), 0.0)]
    return np.array(v, np.float32)


def _vp(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(None if t is None else t.data_ptr())


class ImgEncoderModel:
    """ImgEncoder(384, 256, 16) + the patch -> point gather on device."""

    def __init__(self, sd: weights.StateDict, device: torch.device):
        self.lib = _lib.load()
        self.device = device
        self.t = {k: torch.from_numpy(v).to(device) for k, v in pack_img_encoder(sd).items()}
        self.scalars = pack_img_scalars(sd)
        self._ws: Optional[torch.Tensor] = None
        self.set_arith(os.environ.get("GENPOSE2_ENC_ARITH", "split_f16"))

    def set_arith(self, arith: str) -> None:
        """GEMM arithmetic of the layer-attention Linear and the edge conv: "split_f16" (gp_linear_split, as
        the fused encoder's token linears) or "f32" (exact fp32 MFMA)."""
        if arith not in ("split_f16", "f32"):
            raise ValueError(f"unknown encoder arithmetic {arith!r} (split_f16 | f32)")
        self.arith = arith

    @property
    def table(self) -> np.ndarray:
        return self.scalars

    def set_table(self, scalars: np.ndarray) -> None:
        self.scalars = np.ascontiguousarray(scalars, np.float32).reshape(3)

    def _s(self):
        return ctypes.c_void_p(stream_handle(self.device))

    def forward(self, layers: Sequence[torch.Tensor], return_parts: bool = False):
        """layers: three (B, np, d) tensors -> (B, np, d) [, {"layer_w": (B, np, 3), "edge": (B, d/4)}]."""
        if len(layers) != 3:
            raise ValueError(f"ImgEncoder takes the 3 DINOv3 intermediate layers [2, 6, 11], got {len(layers)}")
        ls = [require_device_tensor(v, f"dino layer {i}") for i, v in enumerate(layers)]
        B, n, d = ls[0].shape
        if any(tuple(v.shape) != (B, n, d) for v in ls):
            raise ValueError("the three DINOv3 layers must have one shape (B, np, d)")
        split = self.arith == "split_f16"
        # the edge conv's split GEMM with implicit im2col (gp_img_encoder3), or over a formed column buffer
        # (gp_img_encoder2, GENPOSE2_IMG_IMPLICIT=0: same products, another summation order)
        implicit = os.environ.get("GENPOSE2_IMG_IMPLICIT", "1")[:1] != "0"
        need = int(self.lib.gp_img_encoder3_workspace_size(B, n, d, int(split)) if implicit
                   else self.lib.gp_img_encoder_workspace_size(B, n, d))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        out = torch.empty((B, n, d), dtype=torch.float32, device=self.device)
        lw = torch.empty((B, n, 3), dtype=torch.float32, device=self.device) if return_parts else None
        edge = torch.empty((B, d // 4), dtype=torch.float32, device=self.device) if return_parts else None
        b2, gg, eg = (float(v) for v in self.scalars)
        fn = self.lib.gp_img_encoder3 if implicit else self.lib.gp_img_encoder2
        conv_h = self.t["conv_w_hp" if implicit else "conv_w_h"]
        check(fn(_vp(ls[0]), _vp(ls[1]), _vp(ls[2]), B, n, d, _vp(self.t["la_w1"]), _vp(self.t["la_b1"]),
                 _vp(self.t["la_w2"]), b2, _vp(self.t["geo_table"]), _vp(self.t["conv_w"]), _vp(self.t["conv_b"]), gg,
                 eg, _vp(self.t["la_w1_h"] if split else None), _vp(conv_h if split else None), _vp(out), _vp(lw),
                 _vp(edge), _vp(self._ws), self._ws.numel(), self._s()), "img_encoder")
        if return_parts:
            return out, {"layer_w": lw, "edge": edge}
        return out

    def gather(self, feat: torch.Tensor, roi_xs: torch.Tensor, roi_ys: torch.Tensor) -> torch.Tensor:
        """posenet.py:146-192: (B, np, d) patch features at pos = (roi_xs // 14) * 16 + roi_ys // 14 (clamped)
        -> (B, N, d) per-point features."""
        feat = require_device_tensor(feat, "feat")
        B, n, d = feat.shape
        # the dataloader's roi pixels may still be on the host (process_batch passes them through)
        xs = require_device_tensor(torch.as_tensor(roi_xs).to(self.device), "roi_xs", torch.int32)
        ys = require_device_tensor(torch.as_tensor(roi_ys).to(self.device), "roi_ys", torch.int32)
        if xs.shape != ys.shape or xs.dim() != 2 or xs.shape[0] != B:
            raise ValueError(f"roi_xs / roi_ys must both be (B={B}, N), got {tuple(xs.shape)} / {tuple(ys.shape)}")
        N = xs.shape[1]
        out = torch.empty((B, N, d), dtype=torch.float32, device=self.device)
        check(self.lib.gp_gather_patch_points(_vp(feat), B, n, d, _vp(xs), _vp(ys), N, arch.IMG_PATCH_PX,
                                              arch.IMG_GRID, _vp(out), self._s()), "gather_patch_points")
        return out
