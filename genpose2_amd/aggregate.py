"""Ranking and aggregation of pose candidates (runner side of the path).

* ``sort_poses_by_energy``  <- networks/reward.py:131-155 (rotation part ordered by the rotation
  energy, translation part by the translation energy, both descending)
* ``aggregate_pose``        <- runners/evaluation_single.py:160-219 (top retain_ratio*K, quaternion
  average, optional DBSCAN re-average of the largest cluster, mean translation, 4x4)

Both run as ONE launch of ``gp_rank_aggregate`` (csrc/gp_aggregate.hip) over the whole batch; the
reference does a per-object host loop with .cpu().numpy() round trips and sklearn DBSCAN. The torch
rotation helpers below serve ``PoseNet.pred_func(return_average_res=True)`` (posenet_agent.py:560),
which the reference also runs as torch ops on device.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _lib
from .device import require_device_tensor, stream_handle


def _rank_aggregate(poses: torch.Tensor, energy: torch.Tensor, retain: int, clustering: int, eps: float,
                    min_samples: int, want_sorted: bool):
    poses = require_device_tensor(poses, "pred_pose")
    energy = require_device_tensor(energy, "pred_energy")
    bs, K = poses.shape[:2]
    if tuple(poses.shape) != (bs, K, 9) or tuple(energy.shape) != (bs, K, 2):
        raise ValueError(f"pred_pose {tuple(poses.shape)} / pred_energy {tuple(energy.shape)}: need (B,K,9)/(B,K,2)")
    agg = torch.empty((bs, 4, 4), dtype=torch.float32, device=poses.device)
    sp = torch.empty_like(poses) if want_sorted else None
    se = torch.empty_like(energy) if want_sorted else None
    vp = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else None)  # noqa: E731
    _lib.check(_lib.load().gp_rank_aggregate(vp(poses), vp(energy), bs, K, retain, int(bool(clustering)),
                                             float(eps), int(min_samples), vp(agg), vp(sp), vp(se),
                                             ctypes.c_void_p(stream_handle(poses.device))), "rank_aggregate")
    return agg, sp, se


def sort_poses_by_energy(poses: torch.Tensor, energy: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (sorted_pose (B,K,9), sorted_energy (B,K,2)); ties keep the lower candidate index."""
    _, sp, se = _rank_aggregate(poses.to(torch.float32), energy.to(torch.float32), 1, 0, 0.0, 1, True)
    return sp, se


def average_quaternion_batch(Q: torch.Tensor, weights: torch.Tensor = None) -> torch.Tensor:
    if weights is None:
        weights = torch.ones((Q.shape[0], Q.shape[1]), device=Q.device, dtype=Q.dtype) / Q.shape[1]
    weight_sum = torch.sum(weights, dim=-1)
    oq = ((Q[:, :, 0:1] > 0).to(Q.dtype) - 0.5) * 2 * Q
    A = torch.einsum("abi,abk->abik", oq, oq)
    A = torch.sum(torch.einsum("abij,ab->abij", A, weights), 1)
    A = A / weight_sum.reshape(A.shape[0], 1, 1)
    q = torch.linalg.eigh(A)[1][:, :, -1]
    return ((q[:, 0:1] > 0).to(Q.dtype) - 0.5) * 2 * q


def rot6_to_matrix(d6: torch.Tensor) -> torch.Tensor:
    """get_rot_matrix(.., 'rot_matrix'): columns b1, b2, b1 x b2 (misc.py:152-153)."""
    a1, a2 = d6[..., :3], d6[..., 3:6]
    b1 = torch.nn.functional.normalize(a1, dim=-1)
    b2 = torch.nn.functional.normalize(a2 - (b1 * a2).sum(-1, keepdim=True) * b1, dim=-1)
    b3 = torch.cross(b1, b2, dim=-1)
    return torch.stack((b1, b2, b3), dim=-2).permute(0, 2, 1)


def matrix_to_quaternion(m: torch.Tensor) -> torch.Tensor:
    """rotation_conversions.py:102-161 (wxyz, no sign standardisation)."""
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = torch.unbind(m.reshape(m.shape[:-2] + (9,)), -1)
    qa = torch.stack([1.0 + m00 + m11 + m22, 1.0 + m00 - m11 - m22, 1.0 - m00 + m11 - m22,
                      1.0 - m00 - m11 + m22], -1)
    q_abs = torch.where(qa > 0, torch.sqrt(torch.clamp(qa, min=0)), torch.zeros_like(qa))
    cand = torch.stack([
        torch.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        torch.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], -1),
        torch.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], -1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], -1)], -2)
    cand = cand / (2.0 * q_abs[..., None].clamp(min=0.1))
    idx = q_abs.argmax(-1)
    return torch.gather(cand, -2, idx[..., None, None].expand(idx.shape + (1, 4)))[..., 0, :]


def quaternion_to_matrix(q: torch.Tensor) -> torch.Tensor:
    """rotation_conversions.py:41-70."""
    r, i, j, k = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def aggregate_pose(pred_pose: torch.Tensor, pred_energy: torch.Tensor, retain_ratio: float = 0.4,
                   clustering: int = 1, clustering_eps: float = 0.05, clustering_minpts: float = 0.1667,
                   retain_num: Optional[int] = None):
    """evaluation_single.py:160-219 for one batch -> (B, 4, 4) float32 on pred_pose's device.

    retain_num: the runner's ``int(cfg.eval_repeat_num * cfg.retain_ratio)`` (:180); defaults to
    int(K * retain_ratio) for a batch of K candidates per object."""
    K = pred_pose.shape[1]
    keep = int(K * retain_ratio) if retain_num is None else int(retain_num)
    if keep < 1:
        raise ValueError(f"retain_ratio {retain_ratio} keeps no candidate of K={K}")
    if keep > K:   # the reference's reshape(bs * retain_num, -1) fails the same way
        raise ValueError(f"retain_num {keep} exceeds the {K} candidates per object")
    agg, _, _ = _rank_aggregate(pred_pose.to(torch.float32), pred_energy.to(torch.float32), keep, clustering,
                                clustering_eps, int(clustering_minpts * keep), False)
    return agg
