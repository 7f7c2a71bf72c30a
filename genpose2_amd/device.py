"""Device-resident models: packed weights in HBM + thin calls into libgenpose_hip.so.

PyTorch is used only for device memory, the current HIP stream and host<->device copies; every
computation on the path is a call into the HIP library.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib, arch, pack, weights
from ._lib import check


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device_tensor(t: torch.Tensor, name: str, dtype=torch.float32) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must live on a HIP device (got {t.device}); the path has no CPU fallback")
    return t.to(dtype).contiguous()


class _Uploaded:
    def __init__(self, arrays: Dict[str, np.ndarray], device: torch.device):
        self.t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in arrays.items()}

    def ptr(self, k: str) -> int:
        return self.t[k].data_ptr()


class EncoderGeometry:
    """Geometry of one point batch in an encoder workspace (EncoderModel.geometry): valid until the producing
    model recomputes geometry in that workspace (its next geometry() or forward() without a geometry), which
    forward(geometry=...) detects through the producer's generation counter; ``event`` marks its completion on
    the producing stream. Refilling the points tensor in place also invalidates it (not detectable: the key is
    the tensor's address and shape). ``event0`` (or None) marks level 0's geometry alone: levels 1-3 were
    computed on a side stream after it, so a consumer can start level 0 before they are done."""

    def __init__(self, ws: torch.Tensor, event, key, producer=None, gen: int = 0, event0=None):
        self.ws, self.event, self.key = ws, event, key   # key: (points tensor address, (B, N))
        self.producer, self.gen = producer, gen
        self.event0 = event0


class EncoderModel:
    """Pointnet2ClsMSG(0), Light cfg, on device (gp_encoder_forward)."""

    def __init__(self, sd: weights.StateDict, device: torch.device):
        self.lib = _lib.load()
        self.device = device
        buf, offs = pack.pack_encoder(sd)
        self.wbuf = torch.from_numpy(buf).to(device)
        self._table = np.ascontiguousarray(offs, np.int64)     # [5][2][3][4] (gp_encoder_forward)
        self._ws: Optional[torch.Tensor] = None
        self._gen = 0   # bumped whenever this model writes geometry into its workspace
        # geometry(): levels 1-3 of the FPS chain and ball lists on a side stream, beside level 0's MLPs
        self.geometry_overlap = os.environ.get("GENPOSE2_GEOM_OVERLAP", "1") == "1"
        self._geo_stream: Optional[torch.cuda.Stream] = None
        # completion of the last side-stream geometry write into self._ws: every later write into the
        # workspace (geometry() again, forward() without a geometry) is ordered after it on its stream
        self._geo_event: Optional[torch.cuda.Event] = None
        self.set_arith(os.environ.get("GENPOSE2_ENC_ARITH", "split_f16"))

    @property
    def table(self) -> np.ndarray:
        """The host layer table [5][2][3][4] (offsets and split-f16 exponents derived from the weight
        values): part of the model's state beside ``wbuf``, so a weight broadcast carries it too."""
        return self._table

    def set_table(self, table: np.ndarray) -> None:
        table = np.ascontiguousarray(table, np.int64).reshape(self._table.shape)
        self._table = table
        self.set_arith(self.arith)

    def set_arith(self, arith: str) -> None:
        """GEMM arithmetic of SA levels 1-3 and GroupAll: "split_f16" (f16 hi/lo MFMA products with
        per-column activation scaling: sa_narrow_split_kernel, sa_split_kernel, tok_split_gemm_kernel)
        or "f32" (exact fp32 MFMA)."""
        if arith not in ("split_f16", "f32"):
            raise ValueError(f"unknown encoder arithmetic {arith!r} (split_f16 | f32)")
        t = self._table.copy()
        if arith == "f32":
            t[..., 2] = -1
        self.arith = arith
        self.offsets = np.ascontiguousarray(t.reshape(-1), np.int64)

    def workspace(self, b: int, n: int) -> torch.Tensor:
        need = int(self.lib.gp_encoder_workspace_size(b, n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _after_side_writes(self, cur) -> None:
        """Order the current stream after this model's outstanding side-stream geometry writes."""
        if self._geo_event is not None:
            cur.wait_event(self._geo_event)

    @staticmethod
    def _xyz(pts: torch.Tensor) -> torch.Tensor:
        pts = require_device_tensor(pts, "pts")
        if pts.dim() != 3 or pts.shape[2] < 3:
            raise ValueError("pts must be (B, N, 3+)")
        return pts if pts.shape[2] == 3 else pts[..., :3].contiguous()

    def geometry(self, pts: torch.Tensor) -> "EncoderGeometry":
        """FPS indices, centroids and ball lists of every level (gp_encoder_geometry) into this model's
        workspace, for this model and any other encoder of the same points (forward(geometry=...))."""
        key = (require_device_tensor(pts, "pts").data_ptr(), tuple(pts.shape[:2]))
        pts = self._xyz(pts)
        B, N, _ = pts.shape
        ws = self.workspace(B, N)
        self._gen += 1
        cur = torch.cuda.current_stream(self.device)
        self._after_side_writes(cur)
        if not self.geometry_overlap:
            check(self.lib.gp_encoder_geometry(ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()),
                                               ws.numel(), ctypes.c_void_p(cur.cuda_stream)), "encoder_geometry")
            ev = torch.cuda.Event()
            ev.record(cur)
            return EncoderGeometry(ws, ev, key, self, self._gen)
        # level 0 here; levels 1-3 (their FPS reads level 0's centroids) on the side stream after it
        check(self.lib.gp_encoder_geometry_levels(ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()),
                                                  ws.numel(), 0, 1, ctypes.c_void_p(cur.cuda_stream)),
              "encoder_geometry level 0")
        ev0 = torch.cuda.Event()
        ev0.record(cur)
        if self._geo_stream is None:
            self._geo_stream = torch.cuda.Stream(device=self.device)
        side = self._geo_stream
        side.wait_event(ev0)
        check(self.lib.gp_encoder_geometry_levels(ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()),
                                                  ws.numel(), 1, 4, ctypes.c_void_p(side.cuda_stream)),
              "encoder_geometry levels 1-3")
        ws.record_stream(side)
        pts.record_stream(side)
        ev = torch.cuda.Event()
        ev.record(side)
        self._geo_event = ev
        return EncoderGeometry(ws, ev, key, self, self._gen, event0=ev0)

    def forward(self, pts: torch.Tensor, return_workspace: bool = False,
                geometry: Optional["EncoderGeometry"] = None):
        """geometry: from geometry() on the same points (this model's or another encoder's); the call then
        runs only the per-level MLPs (gp_encoder_forward_geom), after the stream waits for it."""
        key = (require_device_tensor(pts, "pts").data_ptr(), tuple(pts.shape[:2]))
        pts = self._xyz(pts)
        B, N, _ = pts.shape
        feat = torch.empty((B, arch.PTS_FEAT_DIM), dtype=torch.float32, device=self.device)
        ws = self.workspace(B, N)
        self._after_side_writes(torch.cuda.current_stream(self.device))
        st = ctypes.c_void_p(stream_handle(self.device))
        if geometry is None:
            self._gen += 1   # the self-contained pass rewrites the geometry in this workspace
            check(self.lib.gp_encoder_forward(
                ctypes.c_void_p(self.wbuf.data_ptr()), self.offsets.ctypes.data_as(_lib.c_int64_p),
                ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                ctypes.c_void_p(feat.data_ptr()), st), "encoder_forward")
        else:
            if geometry.key != key:
                raise ValueError("encoder geometry was computed for other points")
            if geometry.producer is not None and geometry.producer._gen != geometry.gen:
                raise ValueError("encoder geometry is stale: its model encoded other points since")
            cur = torch.cuda.current_stream(self.device)
            # level 0 may start once its own geometry is there (event0), levels 1-4 after all of it
            spans = ((0, 1, geometry.event0), (1, 5, geometry.event)) if geometry.event0 is not None else \
                ((0, 5, geometry.event),)
            for first, last, ev in spans:
                cur.wait_event(ev)
                check(self.lib.gp_encoder_forward_geom_levels(
                    ctypes.c_void_p(self.wbuf.data_ptr()), self.offsets.ctypes.data_as(_lib.c_int64_p),
                    ctypes.c_void_p(pts.data_ptr()), B, N, ctypes.c_void_p(geometry.ws.data_ptr()),
                    ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(feat.data_ptr()), first, last, st),
                    "encoder_forward_geom")
            if geometry.ws is not ws:
                geometry.ws.record_stream(torch.cuda.current_stream(self.device))
        return (feat, ws) if return_workspace else feat

    def levels(self, b: int, n: int, ws: torch.Tensor):
        """Views of the per-level intermediates in the workspace (for parity tests)."""
        off = np.zeros(25, np.int64)
        check(self.lib.gp_encoder_workspace_layout(b, n, off.ctypes.data_as(_lib.c_int64_p)))
        out = []
        couts = [arch.level_out_channels(lv) for lv in range(5)]
        for lv in range(5):
            m = arch.NPOINTS[lv] if lv < 4 else 1
            d = {}
            if lv < 4:
                d["fps_idx"] = ws[off[lv * 5]:].view(torch.int32)[: b * m].view(b, m)
                d["new_xyz"] = ws[off[lv * 5 + 1]:].view(torch.float32)[: b * m * 3].view(b, m, 3)
                d["ball_idx"] = [ws[off[lv * 5 + 2 + i]:].view(torch.int32)[: b * m * ns].view(b, m, ns)
                                 for i, ns in enumerate(arch.NSAMPLES[lv])]
            if lv < 4:
                d["features"] = ws[off[lv * 5 + 4]:].view(torch.float32)[: b * m * couts[lv]].view(b, m, couts[lv])
            out.append(d)
        return out


class HeadModel:
    """PoseScoreNet / PoseEnergyNet heads (Rx_Ry_and_T) on device."""

    def __init__(self, sd: weights.StateDict, device: torch.device):
        self.lib = _lib.load()
        self.device = device
        self.up = _Uploaded(pack.pack_heads(sd), device)
        self.set_arith(os.environ.get("GENPOSE2_HEAD_ARITH", "f16x3"))
        self._pc_ws: Optional[torch.Tensor] = None

    def set_arith(self, arith: str) -> None:
        """Per-candidate GEMM arithmetic of every head kernel (PC step, score/energy eval, ODE stages):
        "f16x3" (pose_encoder.2 and head layer 1's pose block on f16 MFMA with three planes per operand
        and six products: every bit of the fp32 operands, products to ~2^-33, fp32 accumulation;
        gp_head.h) or "f32" (exact fp32 MFMA, v_mfma_f32_16x16x4_f32)."""
        if arith not in ("f16x3", "f32"):
            raise ValueError(f"unknown head arithmetic {arith!r} (f16x3 | f32)")
        ptrs = {k: self.up.ptr(k) for k in pack.HEAD_FIELDS}
        if arith == "f32":
            ptrs.update(pe2_h=None, h1p_h=None, hsc=None)
        self.arith = arith
        self.w = _lib.HeadWeights(**ptrs)

    def _s(self):
        return ctypes.c_void_p(stream_handle(self.device))

    def object_proj(self, feat: torch.Tensor) -> torch.Tensor:
        feat = require_device_tensor(feat, "pts_feat")
        B = feat.shape[0]
        pobj = torch.empty((B, 3 * arch.HEAD_HID), dtype=torch.float32, device=self.device)
        check(self.lib.gp_head_object_proj(ctypes.byref(self.w), ctypes.c_void_p(feat.data_ptr()), B,
                                           ctypes.c_void_p(pobj.data_ptr()), self._s()), "head_object_proj")
        return pobj

    def time_proj(self, t: torch.Tensor) -> torch.Tensor:
        t = require_device_tensor(t.reshape(-1), "t")
        out = torch.empty((t.numel(), 3 * arch.HEAD_HID), dtype=torch.float32, device=self.device)
        check(self.lib.gp_head_time_proj(ctypes.byref(self.w), ctypes.c_void_p(t.data_ptr()), t.numel(),
                                         ctypes.c_void_p(out.data_ptr()), self._s()), "head_time_proj")
        return out

    def score(self, pobj, tproj_row, sigma: float, x: torch.Tensor, k: int, out=None) -> torch.Tensor:
        x = require_device_tensor(x, "x")
        R = x.shape[0]
        out = torch.empty((R, arch.POSE_DIM), dtype=torch.float32, device=self.device) if out is None else out
        check(self.lib.gp_score_eval(ctypes.byref(self.w), ctypes.c_void_p(pobj.data_ptr()),
                                     ctypes.c_void_p(tproj_row.data_ptr()), ctypes.c_float(sigma),
                                     ctypes.c_void_p(x.data_ptr()), R, k, ctypes.c_void_p(out.data_ptr()),
                                     self._s()), "score_eval")
        return out

    def energy(self, pobj, tproj_row, sigma: float, pose: torch.Tensor, k: int) -> torch.Tensor:
        pose = require_device_tensor(pose, "pose")
        R = pose.shape[0]
        out = torch.empty((R, 2), dtype=torch.float32, device=self.device)
        check(self.lib.gp_energy_eval(ctypes.byref(self.w), ctypes.c_void_p(pobj.data_ptr()),
                                      ctypes.c_void_p(tproj_row.data_ptr()), ctypes.c_float(sigma),
                                      ctypes.c_void_p(pose.data_ptr()), R, k, ctypes.c_void_p(out.data_ptr()),
                                      self._s()), "energy_eval")
        return out

    def pc_sample(self, pobj, tproj, step_tab: np.ndarray, x: torch.Tensor, k: int, pts_center: torch.Tensor,
                  z1=None, z2=None, seed: int = 0, snr: float = arch.SNR, want_xs: bool = False, global_batch=None):
        """gp_pc_sample; with ``global_batch`` (shard.GlobalBatch) gp_pc_sample_global: this rank's rows of one
        call on the whole batch (grad_norm over every shard's rows, one partials all-gather per step)."""
        R = x.shape[0]
        T = step_tab.shape[0]
        need = int(self.lib.gp_pc_workspace_size(R))
        if self._pc_ws is None or self._pc_ws.numel() < need:
            self._pc_ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        res = torch.empty((R, 9), dtype=torch.float32, device=self.device)
        q = torch.empty((R, 7), dtype=torch.float32, device=self.device)
        xs = torch.empty((R, T, 9), dtype=torch.float32, device=self.device) if want_xs else None
        tab = np.ascontiguousarray(step_tab, np.float32)
        if global_batch is not None:
            from .shard import PartialsExchange
            gb = global_batch
            if z1 is not None or z2 is not None:
                raise ValueError("global-batch sampling draws its noise on the device (z1 / z2 not supported)")
            rows_total, rows_max = gb.total * k, gb.per_max * k
            if R != (gb.hi - gb.lo) * k:
                raise ValueError(f"global-batch shard: {R} rows for objects [{gb.lo}, {gb.hi}) x {k}")
            n = int(self.lib.gp_pc_global_partials(rows_total, rows_max, gb.world, int(self.w.pe2_h is not None)))
            part = torch.zeros(2 * n, dtype=torch.float32, device=self.device)
            ex = PartialsExchange(part, n, gb)
            rc = self.lib.gp_pc_sample_global(
                ctypes.byref(self.w), ctypes.c_void_p(pobj.data_ptr()), ctypes.c_void_p(tproj.data_ptr()),
                tab.ctypes.data_as(ctypes.c_void_p), T, ctypes.c_void_p(x.data_ptr()), R, k,
                ctypes.c_void_p(pts_center.data_ptr()), ctypes.c_uint64(seed), ctypes.c_float(snr),
                ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(_ptr(xs)),
                rows_total, gb.lo * k, gb.rank, gb.world, rows_max, ctypes.c_void_p(part.data_ptr()), ex.fn, None,
                ctypes.c_void_p(self._pc_ws.data_ptr()), self._pc_ws.numel(), self._s())
            if ex.error is not None:
                raise RuntimeError("pc_sample_global: partials exchange failed") from ex.error
            check(rc, "pc_sample_global")
            return res, q, xs
        check(self.lib.gp_pc_sample(
            ctypes.byref(self.w), ctypes.c_void_p(pobj.data_ptr()), ctypes.c_void_p(tproj.data_ptr()),
            tab.ctypes.data_as(ctypes.c_void_p), T, ctypes.c_void_p(x.data_ptr()), R, k,
            ctypes.c_void_p(pts_center.data_ptr()), ctypes.c_void_p(_ptr(z1)), ctypes.c_void_p(_ptr(z2)),
            ctypes.c_uint64(seed), ctypes.c_float(snr), ctypes.c_void_p(res.data_ptr()),
            ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(_ptr(xs)), ctypes.c_void_p(self._pc_ws.data_ptr()),
            self._pc_ws.numel(), self._s()), "pc_sample")
        return res, q, xs


    def ode_denoise(self, pobj, t32: float, sigma: float, g2: float, step: float, x: torch.Tensor, k: int,
                    pts_center: torch.Tensor, ws: torch.Tensor):
        """cond_ode_sampler's final denoise + epilogue (gp_ode_denoise) -> pose (R,9), q (R,7) fp64."""
        R = x.numel() // arch.POSE_DIM
        pose = torch.empty((R, arch.POSE_DIM), dtype=torch.float64, device=self.device)
        q = torch.empty((R, 7), dtype=torch.float64, device=self.device)
        check(self.lib.gp_ode_denoise(
            ctypes.byref(self.w), ctypes.c_void_p(pobj.data_ptr()), t32, sigma, g2, step,
            ctypes.c_void_p(x.data_ptr()), R, k, ctypes.c_void_p(require_device_tensor(pts_center, "pts_center").data_ptr()),
            ctypes.c_void_p(pose.data_ptr()), ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
            ws.numel(), self._s()), "ode_denoise")
        return pose, q


class ScaleModel:
    def __init__(self, sd: weights.StateDict, device: torch.device):
        self.lib = _lib.load()
        self.device = device
        self.up = _Uploaded(pack.pack_scale(sd), device)
        self.w = _lib.ScaleWeights(**{k: self.up.ptr(k) for k in pack.SCALE_FIELDS})

    def forward(self, axes: torch.Tensor, pts_feat: torch.Tensor) -> torch.Tensor:
        axes = require_device_tensor(axes, "axes")
        pts_feat = require_device_tensor(pts_feat, "pts_feat")
        B = axes.shape[0]
        out = torch.empty((B, 3), dtype=torch.float32, device=self.device)
        check(self.lib.gp_scale_forward(ctypes.byref(self.w), ctypes.c_void_p(axes.data_ptr()),
                                        ctypes.c_void_p(pts_feat.data_ptr()), B, ctypes.c_void_p(out.data_ptr()),
                                        ctypes.c_void_p(stream_handle(self.device))), "scale_forward")
        return out


def pose_epilogue_f64(pose: torch.Tensor, k: int, pts_center: torch.Tensor):
    lib = _lib.load()
    pose = pose.contiguous()
    q = torch.empty((pose.shape[0], 7), dtype=torch.float64, device=pose.device)
    check(lib.gp_pose_epilogue_f64(ctypes.c_void_p(pose.data_ptr()), pose.shape[0], k,
                                   ctypes.c_void_p(require_device_tensor(pts_center, "pts_center").data_ptr()),
                                   ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(stream_handle(pose.device))),
          "pose_epilogue_f64")
    return pose, q


def points_mean(pts: torch.Tensor) -> torch.Tensor:
    """gp_points_mean: (B,N,C>=3) -> (B,3) mean of the first three channels over the points."""
    pts = require_device_tensor(pts, "pts")
    B, N, C = pts.shape
    out = torch.empty((B, 3), dtype=torch.float32, device=pts.device)
    check(_lib.load().gp_points_mean(ctypes.c_void_p(pts.data_ptr()), B, N, C, ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(stream_handle(pts.device))), "points_mean")
    return out


def bbox_length(pcl: torch.Tensor, pose: torch.Tensor) -> torch.Tensor:
    """gp_bbox_length: raw points (B,N,C>=3) and aggregated poses (B,4,4) -> (B,3) box lengths."""
    pcl = require_device_tensor(pcl, "pcl")
    pose = require_device_tensor(pose, "pose")
    B, N, C = pcl.shape
    if pose.shape != (B, 4, 4):
        raise ValueError(f"pose must be ({B},4,4), got {tuple(pose.shape)}")
    out = torch.empty((B, 3), dtype=torch.float32, device=pcl.device)
    check(_lib.load().gp_bbox_length(ctypes.c_void_p(pcl.data_ptr()), B, N, C, ctypes.c_void_p(pose.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream_handle(pcl.device))),
          "bbox_length")
    return out


def randn(seed: int, stream: int, rows: int, cols: int, device) -> torch.Tensor:
    """gp_randn: the device draws gp_pc_sample uses (streams 2j / 2j+1 for step j, cols = 9)."""
    lib = _lib.load()
    out = torch.empty((rows, cols), dtype=torch.float32, device=device)
    check(lib.gp_randn(ctypes.c_uint64(seed), ctypes.c_uint32(stream), rows, cols, ctypes.c_void_p(out.data_ptr()),
                       ctypes.c_void_p(stream_handle(out.device))), "randn")
    return out
