"""Drop-in for the reference's ``pointnet2_utils`` forward ops
(networks/pts_encoder/pointnet2_utils/pointnet2/pointnet2_utils.py), backed by
libgenpose_hip.so instead of the CUDA extension ``pointnet2_cuda``.

Same names, argument meaning, layouts, dtypes (int32 indices) and output allocation as the
reference's autograd Functions' forward passes. Backward passes are out of scope
(inference-only build) and raise. The fused encoder (device.EncoderModel) does not go through
these per-op calls; they exist so that code written against the reference op API runs unchanged.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import torch
import torch.nn as nn

from . import _lib
from .device import require_device_tensor, stream_handle


def _s(t: torch.Tensor):
    return ctypes.c_void_p(stream_handle(t.device))


def furthest_point_sample(xyz: torch.Tensor, npoint: int) -> torch.Tensor:
    """(B, N, 3) -> (B, npoint) int32 (pointnet2_utils.py:14-44)."""
    assert xyz.is_contiguous()
    xyz = require_device_tensor(xyz, "xyz")
    B, N, _ = xyz.size()
    out = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
    _lib.check(_lib.load().gp_furthest_point_sampling(B, N, npoint, ctypes.c_void_p(xyz.data_ptr()), None,
                                                      ctypes.c_void_p(out.data_ptr()), _s(xyz)),
               "furthest_point_sample")
    return out


def gather_operation(features: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """(B, C, N), (B, npoint) -> (B, C, npoint) (pointnet2_utils.py:47-85)."""
    assert features.is_contiguous() and idx.is_contiguous()
    B, npoint = idx.size()
    _, C, N = features.size()
    out = torch.empty((B, C, npoint), dtype=torch.float32, device=features.device)
    _lib.check(_lib.load().gp_gather_points(B, C, N, npoint, ctypes.c_void_p(features.data_ptr()),
                                            ctypes.c_void_p(idx.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                            _s(features)), "gather_operation")
    return out


def grouping_operation(features: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """(B, C, N), (B, npoint, nsample) -> (B, C, npoint, nsample) (pointnet2_utils.py:176-223)."""
    assert features.is_contiguous() and idx.is_contiguous()
    B, nfeatures, nsample = idx.size()
    _, C, N = features.size()
    out = torch.empty((B, C, nfeatures, nsample), dtype=torch.float32, device=features.device)
    _lib.check(_lib.load().gp_group_points(B, C, N, nfeatures, nsample, ctypes.c_void_p(features.data_ptr()),
                                           ctypes.c_void_p(idx.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                           _s(features)), "grouping_operation")
    return out


def ball_query(radius: float, nsample: int, xyz: torch.Tensor, new_xyz: torch.Tensor) -> torch.Tensor:
    """-> (B, npoint, nsample) int32 (pointnet2_utils.py:226-256)."""
    assert new_xyz.is_contiguous() and xyz.is_contiguous()
    B, N, _ = xyz.size()
    npoint = new_xyz.size(1)
    idx = torch.empty((B, npoint, nsample), dtype=torch.int32, device=xyz.device)  # fully written
    _lib.check(_lib.load().gp_ball_query(B, N, npoint, ctypes.c_float(radius), nsample,
                                         ctypes.c_void_p(new_xyz.data_ptr()), ctypes.c_void_p(xyz.data_ptr()),
                                         ctypes.c_void_p(idx.data_ptr()), _s(xyz)), "ball_query")
    return idx


class QueryAndGroup(nn.Module):
    """pointnet2_utils.py:259-298."""

    def __init__(self, radius: float, nsample: int, use_xyz: bool = True):
        super().__init__()
        self.radius, self.nsample, self.use_xyz = radius, nsample, use_xyz

    def forward(self, xyz: torch.Tensor, new_xyz: torch.Tensor, features: torch.Tensor = None) -> torch.Tensor:
        idx = ball_query(self.radius, self.nsample, xyz, new_xyz)
        grouped_xyz = grouping_operation(xyz.transpose(1, 2).contiguous(), idx)
        grouped_xyz -= new_xyz.transpose(1, 2).unsqueeze(-1)
        if features is not None:
            grouped_features = grouping_operation(features, idx)
            return torch.cat([grouped_xyz, grouped_features], dim=1) if self.use_xyz else grouped_features
        assert self.use_xyz, "Cannot have not features and not use xyz as a feature!"
        return grouped_xyz


class GroupAll(nn.Module):
    """pointnet2_utils.py:301-328."""

    def __init__(self, use_xyz: bool = True):
        super().__init__()
        self.use_xyz = use_xyz

    def forward(self, xyz: torch.Tensor, new_xyz: torch.Tensor, features: torch.Tensor = None):
        grouped_xyz = xyz.transpose(1, 2).unsqueeze(2)
        if features is not None:
            grouped_features = features.unsqueeze(2)
            return torch.cat([grouped_xyz, grouped_features], dim=1) if self.use_xyz else grouped_features
        return grouped_xyz
