"""DINO-pointwise fused encoder (``Pointnet2ClsMSGFus(384)``, networks/pts_encoder/pointnet2.py:255-388)
on device.

The reference selects it with ``--dino pointwise`` (posenet.py:75-77): its point-cloud input is
``concat([pts, rgb_feat])`` with ``rgb_feat (B, N, 384)`` the per-point DINOv3 features gathered at the
points' image patches (posenet.py:136-197). The DINOv3 backbone and ImgEncoder need weights that are not
available, so this model starts from ``rgb_feat``; everything after it runs here:

* SA levels: ``gp_encoder_fps`` + ``gp_sa_level`` (the Light levels with 384 image channels entering
  level 0);
* after every level, TransformerBlockWithRelativePE (attention.py:491-533): fused QKV ``gp_linear``,
  the EfficientRelativePositionalEncoding bias (``gp_relpe_bias``, attention.py:680-735),
  ``gp_mha_attention``, ``gp_linear`` (wo), ``gp_add_layernorm``, the FFN (``gp_linear`` x2), LayerNorm;
* before levels 1..4, GatedAttentionFusion (attention.py:284-325) of the level input with the image
  features interpolated along the point index (pointnet2.py:343-354): ``gp_interp_points``, the
  BN-folded original_transform / gate / output_conv as ``gp_linear``, ``gp_fusion_attend``,
  ``gp_fusion_mix``. Dropout is the identity (eval).

Token tensors are point-major (B, n, C). The reference's dead gather of ``features`` at the end of each
level (pointnet2.py:370-377) is not executed.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib, arch, pack, weights
from ._lib import check
from .device import EncoderGeometry, require_device_tensor, stream_handle

_ACT = {"none": 0, "relu": 1, "sigmoid": 2, "gate_mix": 3}   # gate_mix: gp_linear_split only


def _vp(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(None if t is None else t.data_ptr())


def pack_relpe(sd: weights.StateDict, prefix: str) -> np.ndarray:
    """The 1024-float layout gp_relpe_bias reads (include/genpose_hip.h): the 504 raw parameters, then the
    fusion layer composed with the two second layers (float64, rounded once): A = Wf[:, :8] Wd2 and
    B = Wf[:, 8:] Wo2 stored [head][u], c = Wf [bd2; bo2] + bf; then the
    direction encoder's first weight transposed to [axis][u]."""
    g = lambda k: np.asarray(sd[f"{prefix}.{k}"], np.float32).reshape(-1)  # noqa: E731
    out = np.zeros(1024, np.float32)
    parts = [g("distance_encoder.0.weight"), g("distance_encoder.0.bias"), g("distance_encoder.2.weight"),
             g("distance_encoder.2.bias"), g("direction_encoder.0.weight"), g("direction_encoder.0.bias"),
             g("direction_encoder.2.weight"), g("direction_encoder.2.bias"), g("fusion.weight"), g("fusion.bias")]
    v = np.concatenate(parts)
    assert v.size == 504
    out[:504] = v
    h, hid = arch.FUS_HEADS, arch.FUS_PE_HID
    wd2 = v[32:160].reshape(h, hid).astype(np.float64)
    bd2 = v[160:168].astype(np.float64)
    wo2 = v[232:360].reshape(h, hid).astype(np.float64)
    bo2 = v[360:368].astype(np.float64)
    wf = v[368:496].reshape(h, 2 * h).astype(np.float64)
    bf = v[496:504].astype(np.float64)
    out[512:640] = (wf[:, :h] @ wd2).reshape(-1)
    out[640:768] = (wf[:, h:] @ wo2).reshape(-1)
    out[768:776] = wf[:, :h] @ bd2 + wf[:, h:] @ bo2 + bf
    out[776:824] = v[168:216].reshape(hid, 3).T.reshape(-1)     # direction_encoder.0 weight as [axis][u]
    return out


def pack_fus_blocks(sd: weights.StateDict) -> Dict[str, np.ndarray]:
    """Transformer, relative-PE and gated-fusion parameters, row-major fp32 (BN folded into the fusion convs)."""
    out: Dict[str, np.ndarray] = {}
    p = "pts_encoder."
    for lv in range(arch.N_LEVELS):
        t = f"{p}transformer_blocks.{lv}"
        out[f"tf{lv}.qkv.w"] = np.concatenate([sd[f"{t}.self_attn.{n}.weight"] for n in ("wq", "wk", "wv")])
        out[f"tf{lv}.qkv.b"] = np.concatenate([sd[f"{t}.self_attn.{n}.bias"] for n in ("wq", "wk", "wv")])
        out[f"tf{lv}.wo.w"], out[f"tf{lv}.wo.b"] = sd[f"{t}.self_attn.wo.weight"], sd[f"{t}.self_attn.wo.bias"]
        for k in ("linear1", "linear2", "norm1", "norm2"):
            out[f"tf{lv}.{k}.w"], out[f"tf{lv}.{k}.b"] = sd[f"{t}.{k}.weight"], sd[f"{t}.{k}.bias"]
        out[f"pe{lv}"] = pack_relpe(sd, f"{p}relative_pos_encoders.{lv}")
    for k in range(1, arch.N_LEVELS):
        g = f"{p}feature_fusions.{k - 1}"
        for m in ("original_transform", "gate", "output_conv"):
            out[f"fu{k}.{m}.w"], out[f"fu{k}.{m}.b"] = weights.fold_conv1d_bn(sd, f"{g}.{m}")
        out[f"fu{k}.ca1.w"] = sd[f"{g}.channel_attention.1.weight"][:, :, 0]
        out[f"fu{k}.ca1.b"] = sd[f"{g}.channel_attention.1.bias"]
        out[f"fu{k}.ca3.w"] = sd[f"{g}.channel_attention.3.weight"][:, :, 0]
        out[f"fu{k}.ca3.b"] = sd[f"{g}.channel_attention.3.bias"]
        out[f"fu{k}.sp.w"] = sd[f"{g}.spatial_attention.0.weight"].reshape(2, arch.FUS_SPATIAL_K)
    out = {k: np.ascontiguousarray(v, np.float32) for k, v in out.items()}
    for name in SPLIT_LINEARS:
        out[f"{name}.wh"] = pack_split_linear(out[f"{name}.w"])
    return out


# token linears that also carry split-f16 planes (gp_linear_split): every one with k % 32 == 0
SPLIT_LINEARS = tuple(f"tf{lv}.{m}" for lv in range(arch.N_LEVELS) for m in ("qkv", "wo", "linear1", "linear2")) + \
    tuple(f"fu{k}.{m}" for k in range(1, arch.N_LEVELS) for m in ("original_transform", "gate", "output_conv"))


def pack_split_linear(w: np.ndarray) -> np.ndarray:
    """gp_linear_split's weight buffer (int32 words): [e, 0, 0, 0] then the f16 hi / lo planes of W * 2**e
    (pack.pack_h16_fragments) with W's rows zero-padded to a multiple of 128."""
    n, k = w.shape
    wp = np.zeros((-(-n // 128) * 128, k), np.float32)
    wp[:n] = w
    e = pack.split_exponent(w)
    return np.concatenate([np.array([e, 0, 0, 0], np.int32), pack.pack_h16_fragments(wp, e)])


class FusEncoderModel:
    """Pointnet2ClsMSGFus(384) on device: forward(pts (B,N,3), rgb_feat (B,N,384)) -> (B, 1024)."""

    def __init__(self, sd: weights.StateDict, device: torch.device):
        self.lib = _lib.load()
        self.device = device
        buf, offs = pack.pack_encoder(sd, arch.fus_sa_branches())
        self.wbuf = torch.from_numpy(buf).to(device)
        self._table = np.ascontiguousarray(offs, np.int64)
        self.arith = "split_f16"
        self.t = {k: torch.from_numpy(v).to(device) for k, v in pack_fus_blocks(sd).items()}
        self._ws: Optional[torch.Tensor] = None
        self._bias: Optional[torch.Tensor] = None
        self._fws: Optional[torch.Tensor] = None
        self._rmax: Optional[torch.Tensor] = None
        self._gen = 0   # bumped whenever this model writes geometry into its workspace
        self.fused_bias = os.environ.get("GENPOSE2_FUSED_RELPE", "1") == "1"
        self.set_arith(os.environ.get("GENPOSE2_ENC_ARITH", "split_f16"))

    @property
    def table(self) -> np.ndarray:
        """Host SA layer table (offsets + split-f16 exponents), broadcast with the device buffers."""
        return self._table

    def set_table(self, table: np.ndarray) -> None:
        self._table = np.ascontiguousarray(table, np.int64).reshape(self._table.shape)
        self.set_arith(self.arith)

    def set_arith(self, arith: str) -> None:
        """GEMM arithmetic of the SA levels and of the token linears: "split_f16" (f16 hi/lo MFMA products
        with per-token activation scaling; gp_linear_split for every linear of >= 1024 tokens) or "f32"
        (exact fp32 MFMA everywhere)."""
        if arith not in ("split_f16", "f32"):
            raise ValueError(f"unknown encoder arithmetic {arith!r} (split_f16 | f32)")
        t = self._table.copy()
        if arith == "f32":
            t[..., 2] = -1
        self.arith = arith
        self.offsets = np.ascontiguousarray(t.reshape(-1), np.int64)

    def _s(self):
        return ctypes.c_void_p(stream_handle(self.device))

    # ------------------------------------------------------------ primitives
    def linear(self, x: torch.Tensor, w: str, act: str = "none", out: Optional[torch.Tensor] = None,
               rmax: Optional[torch.Tensor] = None, ymax: Optional[torch.Tensor] = None) -> torch.Tensor:
        """y = act(x W^T + b). Split arithmetic: ``rmax`` = x's row maxima when the producer already has
        them; ``ymax`` (m floats) receives y's row maxima for the next linear."""
        W, b = self.t[f"{w}.w"], self.t[f"{w}.b"]
        lead, k = x.shape[:-1], x.shape[-1]
        m = int(np.prod(lead)) if lead else 1
        n = W.shape[0]
        y = torch.empty(lead + (n,), dtype=torch.float32, device=self.device) if out is None else out
        if self.split_linear(w, m):
            flags = 0
            if rmax is not None:
                flags = 1
            else:
                if self._rmax is None or self._rmax.numel() < m:
                    self._rmax = torch.empty(m, dtype=torch.float32, device=self.device)
                rmax = self._rmax
            check(self.lib.gp_linear_split(_vp(x), k, m, k, _vp(self.t[f"{w}.wh"]), _vp(b), n, _ACT[act], _vp(y), n,
                                           _vp(rmax), flags, _vp(ymax), self._s()), f"linear_split {w}")
        else:
            check(self.lib.gp_linear(_vp(x), k, m, k, _vp(W), _vp(b), n, _ACT[act], _vp(y), n, self._s()),
                  f"linear {w}")
        return y

    def split_linear(self, w: str, m: int) -> bool:
        return self.arith == "split_f16" and m >= 1024 and f"{w}.wh" in self.t

    def add_ln(self, x: torch.Tensor, r: torch.Tensor, name: str, ymax: Optional[torch.Tensor] = None) -> torch.Tensor:
        d = x.shape[-1]
        y = torch.empty_like(x)
        check(self.lib.gp_add_layernorm(_vp(x), _vp(r), x.numel() // d, d, _vp(self.t[f"{name}.w"]),
                                        _vp(self.t[f"{name}.b"]), ctypes.c_float(arch.LN_EPS), _vp(y), _vp(ymax),
                                        self._s()), f"add_layernorm {name}")
        return y

    def _rowmax_buf(self, m: int, use: bool) -> Optional[torch.Tensor]:
        return torch.empty(m, dtype=torch.float32, device=self.device) if use else None

    def transformer(self, lv: int, x: torch.Tensor, xyz: Optional[torch.Tensor]) -> torch.Tensor:
        """TransformerBlockWithRelativePE.forward (attention.py:505-533), eval mode."""
        B, n, d = x.shape
        if n == 1 and xyz is None:
            # one token per object (GroupAll level): softmax over one key is exactly 1, so the attention
            # output is v itself -- only the wv rows of the fused QKV are evaluated
            W, bq = self.t[f"tf{lv}.qkv.w"][2 * d:], self.t[f"tf{lv}.qkv.b"][2 * d:]
            att = torch.empty_like(x)
            check(self.lib.gp_linear(_vp(x), d, B, d, _vp(W), _vp(bq), d, 0, _vp(att), d, self._s()), "linear wv")
            amax = None
        else:
            amax = self._rowmax_buf(B * n, self.split_linear(f"tf{lv}.wo", B * n))
            att = self.attention(lv, x, xyz, amax)
        # split linears take their input's row maxima from the producer (LayerNorm, linear1's epilogue)
        xmax = self._rowmax_buf(B * n, self.split_linear(f"tf{lv}.linear1", B * n))
        hmax = self._rowmax_buf(B * n, self.split_linear(f"tf{lv}.linear2", B * n))
        x1 = self.add_ln(x, self.linear(att, f"tf{lv}.wo", rmax=amax), f"tf{lv}.norm1", ymax=xmax)
        f = self.linear(self.linear(x1, f"tf{lv}.linear1", "relu", rmax=xmax, ymax=hmax), f"tf{lv}.linear2", rmax=hmax)
        return self.add_ln(x1, f, f"tf{lv}.norm2")

    def attention(self, lv: int, x: torch.Tensor, xyz: Optional[torch.Tensor],
                  amax: Optional[torch.Tensor] = None) -> torch.Tensor:
        """MultiheadAttentionWithRelativePE core (attention.py:436-488): fused QKV, relative-PE bias, heads
        (amax: receives the output's row maxima)."""
        B, n, d = x.shape
        qkv = self.linear(x, f"tf{lv}.qkv")
        att = torch.empty_like(x)
        if xyz is None:
            check(self.lib.gp_mha_attention(_vp(qkv), None, B, n, d, _vp(att), _vp(amax), self._s()), "mha_attention")
        elif d // arch.FUS_HEADS <= 16 and self.fused_bias:
            # level 0: the bias evaluated in the attention kernel's registers (no (B, 8, n, n) buffer, 2.1 GB
            # at B=256); at level 1 (head dim 32) the kernel holds one wave per SIMD and the two-kernel path
            # is faster (0.45 vs 0.73 ms)
            check(self.lib.gp_mha_relpe_attention(_vp(qkv), _vp(xyz), _vp(self.t[f"pe{lv}"]), B, n, d, _vp(att),
                                                  _vp(amax), self._s()), "mha_relpe_attention")
        else:
            need = int(self.lib.gp_relpe_bias_bytes(B, n)) // 4
            if self._bias is None or self._bias.numel() < need:
                self._bias = torch.empty(need, dtype=torch.float32, device=self.device)
            check(self.lib.gp_relpe_bias(_vp(self.t[f"pe{lv}"]), _vp(xyz), B, n, _vp(self._bias), self._s()),
                  "relpe_bias")
            check(self.lib.gp_mha_attention(_vp(qkv), _vp(self._bias), B, n, d, _vp(att), _vp(amax), self._s()),
                  "mha_attention")
        return att

    def fusion(self, k: int, cur: torch.Tensor, orig: torch.Tensor, omax: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
        """GatedAttentionFusion.forward (attention.py:284-325) with orig already at cur's point count (omax: its
        row maxima, when the interpolation produced them)."""
        B, n, c = cur.shape
        ot = self.linear(orig, f"fu{k}.original_transform", "relu", rmax=omax)
        gcat = torch.empty((B, n, 2 * c), dtype=torch.float32, device=self.device)
        t = self.t
        need = int(self.lib.gp_fusion_attend_workspace_size(B, n, c))
        if self._fws is None or self._fws.numel() < need:
            self._fws = torch.empty(need, dtype=torch.uint8, device=self.device)
        gmax = self._rowmax_buf(B * n, self.split_linear(f"fu{k}.gate", B * n))
        check(self.lib.gp_fusion_attend(_vp(cur), _vp(ot), B, n, c, _vp(t[f"fu{k}.ca1.w"]), _vp(t[f"fu{k}.ca1.b"]),
                                        _vp(t[f"fu{k}.ca3.w"]), _vp(t[f"fu{k}.ca3.b"]), _vp(t[f"fu{k}.sp.w"]),
                                        _vp(gcat), _vp(gmax), _vp(self._fws), self._fws.numel(), self._s()),
              "fusion_attend")
        if self.split_linear(f"fu{k}.gate", B * n):   # the gate linear's epilogue does the mix
            fmax = self._rowmax_buf(B * n, self.split_linear(f"fu{k}.output_conv", B * n))
            fused = self.linear(gcat, f"fu{k}.gate", "gate_mix", rmax=gmax, ymax=fmax)
            return self.linear(fused, f"fu{k}.output_conv", "relu", rmax=fmax)
        g = self.linear(gcat, f"fu{k}.gate", "sigmoid")
        fused = torch.empty_like(cur)
        check(self.lib.gp_fusion_mix(_vp(g), _vp(gcat), B * n, c, _vp(fused), self._s()), "fusion_mix")
        return self.linear(fused, f"fu{k}.output_conv", "relu")

    def interp(self, x: torch.Tensor, n_out: int, ymax: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, n_in, c = x.shape
        y = torch.empty((B, n_out, c), dtype=torch.float32, device=self.device)
        check(self.lib.gp_interp_points(_vp(x), B, n_in, c, n_out, _vp(y), _vp(ymax), self._s()), "interp_points")
        return y

    # ------------------------------------------------------------ forward
    def workspace(self, b: int, n: int) -> torch.Tensor:
        need = int(self.lib.gp_encoder_workspace_size(b, n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def geometry(self, pts: torch.Tensor) -> EncoderGeometry:
        """FPS indices, centroids and both ball lists of every level (gp_encoder_geometry) into this model's
        workspace, for this encoder and any other encoder of the same points (forward(geometry=...)): the ScoreNet
        and EnergyNet fused encoders of one batch then share one geometry pass (the ball query then runs once per
        level, not once per encoder and level). Valid until this model encodes again."""
        key = (require_device_tensor(pts, "pts").data_ptr(), tuple(pts.shape[:2]))
        pts = require_device_tensor(pts, "pts")
        B, N, C = pts.shape
        if C != 3:
            pts = pts[..., :3].contiguous()
        ws = self.workspace(B, N)
        self._gen += 1
        cur = torch.cuda.current_stream(self.device)
        check(self.lib.gp_encoder_geometry(_vp(pts), B, N, _vp(ws), ws.numel(), ctypes.c_void_p(cur.cuda_stream)),
              "encoder_geometry")
        ev = torch.cuda.Event()
        ev.record(cur)
        return EncoderGeometry(ws, ev, key, self, self._gen)

    def forward(self, pts: torch.Tensor, rgb_feat: torch.Tensor, return_levels: bool = False,
                geometry: Optional[EncoderGeometry] = None):
        """geometry: from geometry() on the same points (this model's or another fused encoder's): the levels then
        read its FPS indices, centroids and ball lists (gp_sa_level_geom) after the stream waits for it."""
        key = (require_device_tensor(pts, "pts").data_ptr(), tuple(pts.shape[:2]))
        pts = require_device_tensor(pts, "pts")
        rgb_feat = require_device_tensor(rgb_feat, "rgb_feat")
        B, N, C = pts.shape
        if C != 3:
            pts = pts[..., :3].contiguous()
        if tuple(rgb_feat.shape) != (B, N, arch.DINO_DIM):
            raise ValueError(f"rgb_feat must be ({B}, {N}, {arch.DINO_DIM}), got {tuple(rgb_feat.shape)}")
        ws = self.workspace(B, N)
        if geometry is None:
            self._gen += 1   # the self-contained pass rewrites the geometry in this workspace
            check(self.lib.gp_encoder_fps(_vp(pts), B, N, _vp(ws), ws.numel(), self._s()), "encoder_fps")
            geo = None
        else:
            if geometry.key != key:
                raise ValueError("encoder geometry was computed for other points")
            if geometry.producer is not None and geometry.producer._gen != geometry.gen:
                raise ValueError("encoder geometry is stale: its model encoded other points since")
            torch.cuda.current_stream(self.device).wait_event(geometry.event)
            geo = geometry.ws
            if geo is not ws:
                geo.record_stream(torch.cuda.current_stream(self.device))
        off = np.zeros(25, np.int64)
        check(self.lib.gp_encoder_workspace_layout(B, N, off.ctypes.data_as(_lib.c_int64_p)))
        orig, feats = rgb_feat, rgb_feat
        levels: List[dict] = []
        for lv in range(arch.N_LEVELS):
            rec = {}
            if lv > 0:
                omax = None
                if orig.shape[1] != feats.shape[1]:
                    omax = self._rowmax_buf(B * feats.shape[1],
                                            self.split_linear(f"fu{lv}.original_transform", B * feats.shape[1]))
                    orig = self.interp(orig, feats.shape[1], ymax=omax)
                feats = self.fusion(lv, feats, orig, omax)
                rec["fused"] = feats
            m = arch.NPOINTS[lv] if lv < 4 else 1
            cout = arch.level_out_channels(lv)
            sa = torch.empty((B, m, cout), dtype=torch.float32, device=self.device)
            if geo is None:
                check(self.lib.gp_sa_level(_vp(self.wbuf), self.offsets.ctypes.data_as(_lib.c_int64_p), lv,
                                           feats.shape[2], _vp(pts), B, N, _vp(feats), _vp(ws), ws.numel(), _vp(sa),
                                           self._s()), f"sa_level {lv}")
            else:
                check(self.lib.gp_sa_level_geom(_vp(self.wbuf), self.offsets.ctypes.data_as(_lib.c_int64_p), lv,
                                                feats.shape[2], _vp(pts), B, N, _vp(feats), _vp(geo), _vp(ws),
                                                ws.numel(), _vp(sa), self._s()), f"sa_level_geom {lv}")
            gsrc = ws if geo is None else geo
            xyz = gsrc[off[lv * 5 + 1]:].view(torch.float32)[: B * m * 3].view(B, m, 3) if lv < 4 else None
            feats = self.transformer(lv, sa, xyz)
            rec.update(sa=sa, tf=feats)
            levels.append(rec)
        out = feats.reshape(B, arch.PTS_FEAT_DIM)
        return (out, levels) if return_levels else out
