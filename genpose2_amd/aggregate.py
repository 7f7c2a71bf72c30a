"""Ranking and aggregation of pose candidates (runner side of the path).

* ``sort_poses_by_energy``      <- networks/reward.py:131-155 (rotation part ordered by the
  rotation energy, translation part by the translation energy, both descending)
* ``average_quaternion_batch``  <- utils/misc.py:295-317 (w>0 orientation, weighted outer
  products, top eigenvector, w>0 orientation of the result)
* ``aggregate_pose``            <- runners/evaluation_single.py:160-219 (top retain_ratio*K,
  average, optional DBSCAN re-average of the largest cluster, mean translation, 4x4)
* ``dbscan_labels``             restates sklearn.cluster.DBSCAN(eps, min_samples) with its
  default Euclidean metric applied to the ROWS of the quaternion distance matrix:
  core points have >= min_samples neighbours within eps (self included), clusters grow by
  depth-first expansion from core points in index order.

Device tensors stay on device; the per-object DBSCAN labelling (<= 20 points each) runs on the
host, as in the reference (ranked "next" for a device kernel in SURVEY §8f).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch


def sort_poses_by_energy(poses: torch.Tensor, energy: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    sorted_energy, order = torch.sort(energy, descending=True, dim=1, stable=True)
    o_rot, o_tr = order[..., 0], order[..., 1]
    sp = torch.gather(poses, 1, o_rot.unsqueeze(-1).expand(-1, -1, poses.shape[-1])).clone()
    sp[..., -3:] = torch.gather(poses, 1, o_tr.unsqueeze(-1).expand(-1, -1, poses.shape[-1]))[..., -3:]
    return sp, sorted_energy


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


def dbscan_labels(X: np.ndarray, eps: float, min_samples: int) -> np.ndarray:
    """sklearn DBSCAN (metric='euclidean', algorithm brute) on the rows of X."""
    X = np.asarray(X, np.float64)
    n = X.shape[0]
    d = np.sqrt(np.maximum(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1), 0.0))
    nbrs = [np.nonzero(d[i] <= eps)[0] for i in range(n)]
    core = np.array([len(v) >= min_samples for v in nbrs])
    labels = np.full(n, -1, np.int64)
    label = 0
    for i in range(n):
        if labels[i] != -1 or not core[i]:
            continue
        stack = [i]
        while stack:
            p = stack.pop()
            if labels[p] != -1:
                continue
            labels[p] = label
            if core[p]:
                stack.extend(int(j) for j in nbrs[p][::-1] if labels[j] == -1)
        label += 1
    return labels


def aggregate_pose(pred_pose: torch.Tensor, pred_energy: torch.Tensor, retain_ratio: float = 0.4,
                   clustering: int = 1, clustering_eps: float = 0.05, clustering_minpts: float = 0.1667):
    """evaluation_single.py:160-219 for one batch: -> (B, 4, 4) float32 on pred_pose's device."""
    bs, K = pred_pose.shape[:2]
    pred_pose = pred_pose.to(torch.float32)
    sp, _ = sort_poses_by_energy(pred_pose, pred_energy.to(pred_pose.device))
    keep = int(K * retain_ratio)
    good = sp[:, :keep, :]
    q = matrix_to_quaternion(rot6_to_matrix(good[:, :, :6].reshape(bs * keep, -1))).reshape(bs, keep, 4)
    qa = average_quaternion_batch(q)
    if clustering:
        D = 1 - torch.sum(q.unsqueeze(1) * q.unsqueeze(2), dim=3) ** 2    # (bs, keep, keep)
        Dh = D.cpu().numpy()
        for j in range(bs):
            labels = dbscan_labels(Dh[j], clustering_eps, int(clustering_minpts * keep))
            if np.any(labels >= 0):
                best = int(np.argmax(np.bincount(labels[labels >= 0])))
                sel = torch.from_numpy(labels == best).to(q.device)
                qa[j] = average_quaternion_batch(q[j, sel].unsqueeze(0))[0]
    out = torch.zeros(bs, 4, 4, device=pred_pose.device)
    out[:, 3, 3] = 1
    out[:, :3, :3] = quaternion_to_matrix(qa)
    out[:, :3, 3] = torch.mean(good[:, :, -3:], dim=1)
    return out
