"""ORACLE — test infrastructure only.

CPU restatement (numpy float32, + plain C for the serial point ops in ``pointops.c``) of the
reference's pose-candidate path. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker /
CPU baseline. The product path (``genpose2_amd``) never imports it.

Each function cites the reference lines it restates. Parity of this restatement against
the reference itself is pinned by ``tests/golden/*.npz`` (generated here by importing the
reference read-only: ``tests/golden/make_golden.py``) and checked in
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from genpose2_amd import arch, weights

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
F32 = np.float32


# ============================================================ native point ops (pointops.c)
def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liboracle_pointops.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = ctypes.CDLL(path)
        fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
        lib.oracle_fps.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip]
        lib.oracle_ball_query.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_int, fp, fp, ip]
        lib.oracle_fps_block_size.argtypes = [ctypes.c_int]
        lib.oracle_fps_block_size.restype = ctypes.c_int
        _LIB = lib
    return _LIB


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def furthest_point_sample(xyz: np.ndarray, npoint: int) -> np.ndarray:
    """``FurthestPointSampling.forward`` (pointnet2_utils.py:14-44 -> sampling_gpu.cu:94-209)."""
    xyz = np.ascontiguousarray(xyz, dtype=F32)
    B, N, _ = xyz.shape
    idx = np.zeros((B, npoint), dtype=np.int32)
    _lib().oracle_fps(_fp(xyz), B, N, npoint, _ip(idx))
    return idx


def ball_query(radius: float, nsample: int, xyz: np.ndarray, new_xyz: np.ndarray) -> np.ndarray:
    """``BallQuery.forward`` (pointnet2_utils.py:226-256 -> ball_query_gpu.cu:9-45)."""
    xyz = np.ascontiguousarray(xyz, dtype=F32)
    new_xyz = np.ascontiguousarray(new_xyz, dtype=F32)
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    idx = np.zeros((B, M, nsample), dtype=np.int32)
    _lib().oracle_ball_query(B, N, M, F32(radius), nsample, _fp(new_xyz), _fp(xyz), _ip(idx))
    return idx


def grouping_operation(features: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """(B,C,N),(B,M,ns) -> (B,C,M,ns) (group_points_gpu.cu:47-66)."""
    B = features.shape[0]
    return np.stack([features[b][:, idx[b]] for b in range(B)]).astype(F32)


def gather_operation(features: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """(B,C,N),(B,M) -> (B,C,M) (sampling_gpu.cu:8-24)."""
    B = features.shape[0]
    return np.stack([features[b][:, idx[b]] for b in range(B)]).astype(F32)


# ============================================================ encoder (Pointnet2ClsMSG)
def _conv_bn_relu(x: np.ndarray, sd, prefix: str) -> np.ndarray:
    """Conv2d 1x1 (no bias) -> BatchNorm2d(eval) -> ReLU (pytorch_utils.py:58-106), through the same
    torch CPU operators the reference's SharedMLP calls (one thread pool with the rest of the CPU
    baseline: numpy's OpenBLAS beside torch's OpenMP pool oversubscribes the cores)."""
    import torch
    import torch.nn.functional as tf
    t = lambda k: torch.from_numpy(np.ascontiguousarray(sd[f"{prefix}.{k}"], dtype=F32))  # noqa: E731
    y = tf.conv2d(torch.from_numpy(np.ascontiguousarray(x, dtype=F32)), t("conv.weight"))
    y = tf.batch_norm(y, t("bn.bn.running_mean"), t("bn.bn.running_var"), t("bn.bn.weight"), t("bn.bn.bias"),
                      training=False, eps=arch.BN_EPS)
    return torch.relu(y).numpy()


def encoder_forward(sd, pts: np.ndarray, return_levels: bool = False):
    """``Pointnet2ClsMSG.forward`` (pointnet2.py:244-252) over ``_PointnetSAModuleBase.forward``
    (pointnet2_modules.py:19-74), QueryAndGroup/GroupAll (pointnet2_utils.py:259-328).

    pts: (B, N, 3) un-centred camera-frame points. Returns (B, 1024)."""
    xyz = np.ascontiguousarray(pts[..., :3], dtype=F32)
    feats = None  # (B, C, N)
    levels = []
    for lv, branches in enumerate(arch.sa_branches()):
        npoint = arch.NPOINTS[lv]
        if npoint is not None:
            fidx = furthest_point_sample(xyz, npoint)
            new_xyz = gather_operation(xyz.transpose(0, 2, 1), fidx).transpose(0, 2, 1).copy()
        else:
            fidx, new_xyz = None, None
        outs, bq = [], []
        for br in branches:
            if npoint is not None:
                idx = ball_query(br.radius, br.nsample, xyz, new_xyz)
                bq.append(idx)
                gx = grouping_operation(xyz.transpose(0, 2, 1), idx)
                gx = gx - new_xyz.transpose(0, 2, 1)[..., None]
                grouped = gx if feats is None else np.concatenate(
                    [gx, grouping_operation(feats, idx)], axis=1)
            else:  # GroupAll: raw xyz + features, (B, 3+C, 1, N)
                gx = xyz.transpose(0, 2, 1)[:, :, None, :]
                grouped = gx if feats is None else np.concatenate([gx, feats[:, :, None, :]], axis=1)
            h = grouped.astype(F32)
            for i in range(len(br.widths) - 1):
                h = _conv_bn_relu(h, sd, f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}")
            outs.append(h.max(axis=3))  # max_pool2d over nsample
        feats = np.concatenate(outs, axis=1).astype(F32)  # (B, C_out, npoint or 1)
        levels.append(dict(fps_idx=fidx, new_xyz=new_xyz, ball_idx=bq, features=feats))
        if new_xyz is not None:
            xyz = new_xyz
    out = feats[:, :, 0]
    return (out, levels) if return_levels else out


# ============================================================ SDE helpers (sde.py:15-35)
def ve_sigma(t):
    """sigma_min * (sigma_max/sigma_min) ** t, in the dtype of ``t`` (sde.py:15-18). Evaluated
    with torch's CPU pow, the function the reference calls (numpy's pow differs by 1 ulp)."""
    import torch
    t = np.asarray(t)
    dt = t.dtype if t.dtype in (np.float32, np.float64) else np.float64
    tt = torch.from_numpy(np.ascontiguousarray(t, dtype=dt))
    return (arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** tt).numpy().astype(dt)


def ve_diffusion(t):
    """sigma(t) * sqrt(2 (ln sigma_max - ln sigma_min)) (sde.py:21-27)."""
    s = np.asarray(ve_sigma(t))
    return (s * s.dtype.type(arch.DIFFUSION_SCALE)).astype(s.dtype)


def gram_schmidt(rot6: np.ndarray) -> np.ndarray:
    """``normalize_rotation(.., 'rot_matrix')`` (misc.py:327-344) via rotation_6d_to_matrix
    (rotation_conversions.py:556-577): b1 = n(a1), b2 = n(a2 - (b1.a2) b1)."""
    a1, a2 = rot6[:, :3], rot6[:, 3:6]
    dt = rot6.dtype.type
    b1 = a1 / np.maximum(np.linalg.norm(a1, axis=-1, keepdims=True), dt(1e-12))
    b2 = a2 - (b1 * a2).sum(-1, keepdims=True) * b1
    b2 = b2 / np.maximum(np.linalg.norm(b2, axis=-1, keepdims=True), dt(1e-12))
    return np.concatenate([b1, b2], axis=-1).astype(rot6.dtype)


# ============================================================ score / energy MLP
def _lin(x, w, b):
    """nn.Linear as the reference calls it (torch CPU F.linear)."""
    import torch
    import torch.nn.functional as tf
    c = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=F32))  # noqa: E731
    return tf.linear(c(x), c(w), c(b)).numpy()


def head_features(sd, pts_feat, pose, t):
    """Shared trunk of PoseScoreNet.forward (scorenet.py:236-249) / PoseEnergyNet.get_energy
    (energynet.py:152-157): returns (f (R,9) before the sigma division, std (R,1))."""
    n = "pose_score_net"
    t = np.asarray(t, dtype=F32).reshape(-1, 1)
    W = sd[f"{n}.t_encoder.0.W"].astype(F32)
    x_proj = (t[:, 0][:, None] * W[None, :]) * F32(2) * F32(np.pi)   # scorenet.py:87
    t_emb = np.concatenate([np.sin(x_proj), np.cos(x_proj)], axis=-1).astype(F32)
    t_feat = np.maximum(_lin(t_emb, sd[f"{n}.t_encoder.1.weight"], sd[f"{n}.t_encoder.1.bias"]), 0)
    h = np.maximum(_lin(pose.astype(F32), sd[f"{n}.pose_encoder.0.weight"], sd[f"{n}.pose_encoder.0.bias"]), 0)
    pose_feat = np.maximum(_lin(h, sd[f"{n}.pose_encoder.2.weight"], sd[f"{n}.pose_encoder.2.bias"]), 0)
    total = np.concatenate([pts_feat.astype(F32), t_feat, pose_feat], axis=-1)
    outs = []
    for hn in arch.HEAD_NAMES:
        u = np.maximum(_lin(total, sd[f"{n}.{hn}.0.weight"], sd[f"{n}.{hn}.0.bias"]), 0)
        outs.append(_lin(u, sd[f"{n}.{hn}.2.weight"], sd[f"{n}.{hn}.2.bias"]))
    return np.concatenate(outs, axis=-1).astype(F32), ve_sigma(t)


def score_forward(sd, pts_feat, pose, t):
    """PoseScoreNet.forward with Rx_Ry_and_T heads (scorenet.py:215-275)."""
    f, std = head_features(sd, pts_feat, pose, t)
    return (f / (std + F32(1e-7))).astype(F32)


def energy_forward(sd, pts_feat, pose, t):
    """PoseEnergyNet.get_energy, energy_mode IP, s_theta score, norm identical, decoupled_rt
    (energynet.py:151-208) -> (R, 2) [rot, trans]."""
    f, std = head_features(sd, pts_feat, pose, t)
    s = (f / std).astype(F32)
    pose = pose.astype(F32)
    return np.stack([(pose[:, :6] * s[:, :6]).sum(-1), (pose[:, 6:] * s[:, 6:]).sum(-1)], -1).astype(F32)


# ============================================================ samplers
def time_grid(num_steps: int, eps: float = arch.SAMPLING_EPS) -> np.ndarray:
    """``torch.linspace(1.0, eps, num_steps)`` (samplers.py:129) as float32."""
    import torch
    return torch.linspace(1.0, eps, num_steps).numpy().astype(F32)


def pc_sample(score_fn: Callable, x0: np.ndarray, pts_center_rows: np.ndarray, num_steps: int,
              z1: np.ndarray, z2: np.ndarray, snr: float = arch.SNR):
    """``cond_pc_sampler`` (samplers.py:113-177) with injected noise.

    x0: (R,9) initial state (prior sample or init_x); z1/z2: (T,R,9) the two randn_like draws
    per step (Langevin :148, predictor :166). Returns (xs (R,T,9), mean_x (R,9))."""
    ts = time_grid(num_steps)
    step_size = F32(ts[0] - ts[1])
    x = x0.astype(F32).copy()
    R = x.shape[0]
    xs = []
    ls_coef = F32(snr * np.sqrt(arch.POSE_DIM))
    mean_x = x
    for k, t in enumerate(ts):
        grad = score_fn(x, np.full((R, 1), t, dtype=F32)).astype(F32)
        grad_norm = F32(np.linalg.norm(grad, axis=-1).astype(F32).mean(dtype=F32))
        ls = F32(2) * (ls_coef / grad_norm) ** 2
        x = (x + ls * grad + np.sqrt(F32(2) * ls) * z1[k]).astype(F32)
        x[:, :3] /= np.linalg.norm(x[:, :3], axis=-1, keepdims=True)
        x[:, 3:6] /= np.linalg.norm(x[:, 3:6], axis=-1, keepdims=True)
        g = ve_diffusion(np.full((R, 1), t, dtype=F32))
        drift = -(g ** 2) * grad
        mean_x = (x + drift * step_size).astype(F32)
        x = (mean_x + g * np.sqrt(step_size) * z2[k]).astype(F32)
        x[:, :6] = gram_schmidt(x[:, :6])
        xs.append(x.copy())
    xs = np.stack(xs, axis=0)
    xs[:, :, 6:] += pts_center_rows[None].astype(F32)
    mean_x = mean_x.copy()
    mean_x[:, 6:] += pts_center_rows.astype(F32)
    mean_x[:, :6] = gram_schmidt(mean_x[:, :6])
    return xs.transpose(1, 0, 2), mean_x


def ode_sample(score_fn: Callable, x0: np.ndarray, pts_center_rows: np.ndarray, T0: float,
               num_steps: Optional[int], eps: float = arch.SAMPLING_EPS,
               atol: float = 1e-5, rtol: float = 1e-5, denoise: bool = True):
    """``cond_ode_sampler`` (samplers.py:180-258): probability-flow ODE through scipy RK45
    (the reference's own integrator, scipy/integrate/_ivp/rk.py), float64 state.

    x0: (R,9) float32 initial state (prior(T0) [+ init_x]). Returns (xs, x) float64, nfev."""
    from scipy import integrate
    R = x0.shape[0]

    def ode_func(t, y):
        x = y.reshape(-1, arch.POSE_DIM).astype(F32)
        tt = np.full((R, 1), F32(t), dtype=F32)   # ones(bs).unsqueeze(-1) * t (float32)
        s = score_fn(x, tt).astype(F32).reshape(-1)
        g = ve_diffusion(np.float64(t))            # sde_coeff(torch.tensor(t)) is float64
        return 0.0 - 0.5 * (g ** 2) * s.astype(np.float64)

    t_eval = None if num_steps is None else np.linspace(T0, eps, num_steps)
    res = integrate.solve_ivp(ode_func, (T0, eps), x0.reshape(-1).astype(np.float64),
                              rtol=rtol, atol=atol, method="RK45", t_eval=t_eval)
    xs = res.y.T.reshape(-1, R, arch.POSE_DIM).copy()
    x = res.y[:, -1].reshape(R, arch.POSE_DIM).copy()
    if denoise:
        ve = np.full((R, 1), F32(eps), dtype=F32)
        g = ve_diffusion(ve)
        grad = score_fn(x.astype(F32), ve).astype(F32)
        drift = (F32(0) - g ** 2 * grad).astype(F32)
        x = x + drift.astype(np.float64) * ((1 - eps) / (1000 if num_steps is None else num_steps))
    n_t = xs.shape[0]
    flat = xs.reshape(n_t * R, -1)
    flat[:, :6] = gram_schmidt(flat[:, :6])
    xs = flat.reshape(n_t, R, -1)
    xs[:, :, 6:] += pts_center_rows[None].astype(F32).astype(np.float64)
    x[:, :6] = gram_schmidt(x[:, :6])
    x[:, 6:] += pts_center_rows.astype(F32).astype(np.float64)
    return xs.transpose(1, 0, 2), x, int(res.nfev)


# ============================================================ device noise (gp_randn)
def philox4x32_10(ctr: np.ndarray, key: np.ndarray) -> np.ndarray:
    """Philox4x32-10 (Salmon et al., SC'11; Random123's philox4x32 with its round constants):
    ctr (..., 4) uint32, key (..., 2) uint32 -> (..., 4) uint32. Pinned by the Random123
    known-answer vectors in tests/test_oracle_pointops.py."""
    c = [np.asarray(ctr[..., j], np.uint64) for j in range(4)]
    k0 = np.asarray(key[..., 0], np.uint64)
    k1 = np.asarray(key[..., 1], np.uint64)
    m32 = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & m32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & m32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & m32
        k1 = (k1 + np.uint64(0xBB67AE85)) & m32
    return np.stack(c, -1).astype(np.uint32)


def randn(seed: int, stream: int, rows: int, cols: int) -> np.ndarray:
    """gp_randn's draws in float64: counter {row, col//4, stream, 0x5EED}, key = seed halves,
    u = ((v >> 8) + 1) / 2^24, Box-Muller (cos, sin) pairs (csrc/gp_common.h philox_normal4)."""
    nb = (cols + 3) // 4
    r, b = np.meshgrid(np.arange(rows, dtype=np.uint64), np.arange(nb, dtype=np.uint64), indexing="ij")
    ctr = np.stack([r, b, np.full_like(r, stream), np.full_like(r, 0x5EED)], -1)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], np.uint64)
    v = philox4x32_10(ctr, np.broadcast_to(key, ctr.shape[:-1] + (2,)))
    u = ((v >> 8).astype(np.float64) + 1.0) / 16777216.0
    rad0, rad1 = np.sqrt(-2.0 * np.log(u[..., 0])), np.sqrt(-2.0 * np.log(u[..., 2]))
    a0, a1 = 2 * np.pi * u[..., 1], 2 * np.pi * u[..., 3]
    z = np.stack([rad0 * np.cos(a0), rad0 * np.sin(a0), rad1 * np.cos(a1), rad1 * np.sin(a1)], -1)
    return z.reshape(rows, nb * 4)[:, :cols]


# ============================================================ rotations (rotation_conversions.py)
def rot6_to_matrix(rot6: np.ndarray) -> np.ndarray:
    """get_rot_matrix(.., 'rot_matrix') = rotation_6d_to_matrix(x).permute(0,2,1): columns
    b1, b2, b3 (misc.py:152-153, rotation_conversions.py:556-577)."""
    g = gram_schmidt(rot6)
    b1, b2 = g[:, :3], g[:, 3:6]
    b3 = np.cross(b1, b2)
    return np.stack([b1, b2, b3], axis=-1).astype(rot6.dtype)


def matrix_to_quaternion(m: np.ndarray) -> np.ndarray:
    """rotation_conversions.py:102-161 (no sign standardisation), wxyz."""
    m = np.asarray(m)
    dt = m.dtype.type
    m00, m01, m02 = m[..., 0, 0], m[..., 0, 1], m[..., 0, 2]
    m10, m11, m12 = m[..., 1, 0], m[..., 1, 1], m[..., 1, 2]
    m20, m21, m22 = m[..., 2, 0], m[..., 2, 1], m[..., 2, 2]
    qa = np.stack([dt(1) + m00 + m11 + m22, dt(1) + m00 - m11 - m22,
                   dt(1) - m00 + m11 - m22, dt(1) - m00 - m11 + m22], -1)
    q_abs = np.where(qa > 0, np.sqrt(np.maximum(qa, 0)), dt(0)).astype(m.dtype)
    cand = np.stack([
        np.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        np.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], -1),
        np.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], -1),
        np.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], -1)], -2)
    cand = cand / (dt(2) * np.maximum(q_abs[..., None], dt(0.1)))
    sel = q_abs.argmax(-1)
    return np.take_along_axis(cand, sel[..., None, None].repeat(4, -1), -2)[..., 0, :].astype(m.dtype)


def quaternion_to_matrix(q: np.ndarray) -> np.ndarray:
    """rotation_conversions.py:41-70."""
    r, i, j, k = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    two_s = 2.0 / (q * q).sum(-1)
    o = np.stack([1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                  two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                  two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)], -1)
    return o.reshape(q.shape[:-1] + (3, 3)).astype(q.dtype)


def pose_to_quat_rows(res: np.ndarray) -> np.ndarray:
    """pred_func tail (posenet_agent.py:554-556): [quat_wxyz(GS(res[:, :6])), res[:, 6:]]."""
    q = matrix_to_quaternion(rot6_to_matrix(res[:, :6]))
    return np.concatenate([q, res[:, 6:]], -1)


def average_quaternion_batch(Q: np.ndarray) -> np.ndarray:
    """misc.py:295-317 (uniform weights)."""
    n = Q.shape[1]
    w = np.full((Q.shape[0], n), 1.0 / n, dtype=Q.dtype)
    oq = ((Q[:, :, 0:1] > 0).astype(Q.dtype) - Q.dtype.type(0.5)) * 2 * Q
    A = np.einsum("abi,abk->abik", oq, oq)
    A = (A * w[:, :, None, None]).sum(1) / w.sum(-1)[:, None, None]
    _, vec = np.linalg.eigh(A)
    q = vec[:, :, -1]
    return (((q[:, 0:1] > 0).astype(Q.dtype) - Q.dtype.type(0.5)) * 2 * q).astype(Q.dtype)


# ============================================================ ranking / aggregation
def sort_poses_by_energy(poses: np.ndarray, energy: np.ndarray):
    """reward.py:131-155: rotation part ordered by energy[...,0] desc, translation part by
    energy[...,1] desc."""
    import torch   # torch.sort(descending=True) as reward.py:144 calls it: NaN first, ties keep index order
    o_rot = torch.sort(torch.from_numpy(np.ascontiguousarray(energy[..., 0])), dim=1, descending=True,
                       stable=True)[1].numpy()
    o_tr = torch.sort(torch.from_numpy(np.ascontiguousarray(energy[..., 1])), dim=1, descending=True,
                      stable=True)[1].numpy()
    sp = np.take_along_axis(poses, o_rot[..., None], 1).copy()
    sp[..., 6:] = np.take_along_axis(poses, o_tr[..., None], 1)[..., 6:]
    se = np.stack([np.take_along_axis(energy[..., 0], o_rot, 1),
                   np.take_along_axis(energy[..., 1], o_tr, 1)], -1)
    return sp, se, o_rot, o_tr


def dbscan_labels(X: np.ndarray, eps: float, min_samples: int) -> np.ndarray:
    """sklearn DBSCAN(eps, min_samples), metric='euclidean', on the rows of X, restated as the
    device kernel runs it (csrc/gp_aggregate.hip): core points have >= min_samples neighbours
    within eps (self included); clusters grow from core points in index order; border points
    join the first cluster that reaches them. Pinned against sklearn in tests/test_cpu_host.py."""
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


def aggregate_pose(pred_pose: np.ndarray, pred_energy: np.ndarray, retain_ratio=0.4,
                   clustering=1, clustering_eps=0.05, clustering_minpts=0.1667):
    """evaluation_single.py:160-219 for one batch -> (B,4,4) float32."""
    from sklearn.cluster import DBSCAN
    bs, K = pred_pose.shape[:2]
    sp, _, _, _ = sort_poses_by_energy(pred_pose, pred_energy)
    keep = int(K * retain_ratio)
    good = sp[:, :keep]
    R = rot6_to_matrix(good[:, :, :6].reshape(bs * keep, -1))
    q = matrix_to_quaternion(R).reshape(bs, keep, 4)
    qa = average_quaternion_batch(q)
    if clustering:
        for j in range(bs):
            D = 1 - (q[j][None] * q[j][:, None]).sum(2) ** 2
            labels = DBSCAN(eps=clustering_eps, min_samples=int(clustering_minpts * keep)).fit(
                D.astype(np.float32)).labels_
            if np.any(labels >= 0):
                best = np.argmax(np.bincount(labels[labels >= 0]))
                qa[j] = average_quaternion_batch(q[j, labels == best][None])[0]
    out = np.zeros((bs, 4, 4), dtype=np.float32)
    out[:, 3, 3] = 1
    out[:, :3, :3] = quaternion_to_matrix(qa)
    out[:, :3, 3] = good[:, :, 6:].mean(1)
    return out


# ============================================================ stage glue
def points_mean(pts: np.ndarray) -> np.ndarray:
    """process_batch's pts_center (datasets_omni6dpose.py:746-752): mean of pts[:, :, :3] over points."""
    return pts[..., :3].astype(np.float64).mean(1).astype(F32)


def bbox_length(pcl: np.ndarray, pose: np.ndarray) -> np.ndarray:
    """inference_scale without a ScaleNet checkpoint (evaluation_single.py:233-252):
    2 * max_n |R^T (p_n - t)| per axis, fp32 as the reference's CPU tensors."""
    R = pose[:, :3, :3].astype(F32)
    t = pose[:, :3, 3].astype(F32)
    d = (pcl[..., :3].astype(F32) - t[:, None, :]).astype(F32)              # (B, N, 3)
    q = np.einsum("bji,bnj->bni", R, d).astype(F32)                          # bmm(R^T, d)
    return (np.abs(q).max(1) * 2).astype(F32)


# ============================================================ ScaleNet
def encode_axes(axes: np.ndarray, dim: int) -> np.ndarray:
    """genpose_utils.py:8-18."""
    bs = axes.shape[0]
    a = axes.reshape(bs, -1, 1).astype(F32)
    e = (2.0 ** np.arange(dim, dtype=F32)).reshape(1, 1, -1)
    return np.concatenate([np.sin(e * a).reshape(bs, -1), np.cos(e * a).reshape(bs, -1)], -1).astype(F32)


def scale_forward(sd, pts_feat: np.ndarray, axes: np.ndarray) -> np.ndarray:
    """ScaleNet.forward (scalenet.py:33-49) -> (B,3)."""
    emb = encode_axes(axes, arch.SCALE_EMB // 18)
    h = np.maximum(_lin(emb, sd["axes_encoder.0.weight"], sd["axes_encoder.0.bias"]), 0)
    h = np.maximum(_lin(h, sd["axes_encoder.2.weight"], sd["axes_encoder.2.bias"]), 0)
    tot = np.concatenate([pts_feat.astype(F32), h], -1)
    u = np.maximum(_lin(tot, sd["fusion_tail_length.0.weight"], sd["fusion_tail_length.0.bias"]), 0)
    return _lin(u, sd["fusion_tail_length.2.weight"], sd["fusion_tail_length.2.bias"])


# ============================================================ whole pred_func (PC / ODE)
def pred_func(sd, pts: np.ndarray, pts_center: np.ndarray, repeat_num: int, num_steps: int,
              sampler: str, prior: np.ndarray, z1=None, z2=None, T0: Optional[float] = None,
              init_x: Optional[np.ndarray] = None):
    """``PoseNet.pred_func`` (posenet_agent.py:490-584) with injected noise.

    prior: (B*K, 9) standard-normal draw (scaled here by sigma(T)). Returns
    (pred_pose (B,K,9), pred_q (B,K,7), pts_feat (B,1024), extra)."""
    B = pts.shape[0]
    K = repeat_num
    feat = encoder_forward(sd, pts)
    feat_rows = np.repeat(feat, K, axis=0)
    center_rows = np.repeat(pts_center.astype(F32), K, axis=0)

    def score_fn(x, t):
        return score_forward(sd, feat_rows, x, t)

    if sampler == "pc":
        sig = F32(arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** 1.0)
        x0 = (prior.astype(F32) * sig).astype(F32) if init_x is None else np.repeat(init_x, K, 0)
        xs, res = pc_sample(score_fn, x0, center_rows, num_steps, z1, z2)
        extra = dict(xs=xs)
    elif sampler == "ode":
        T0 = arch.SDE_T if T0 is None else T0
        sig = F32(arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** T0)
        x0 = (prior.astype(F32) * sig).astype(F32)
        if init_x is not None:
            x0 = (np.repeat(init_x, K, 0).astype(F32) + x0).astype(F32)
        xs, res, nfev = ode_sample(score_fn, x0, center_rows, T0, num_steps)
        extra = dict(xs=xs, nfev=nfev)
    else:
        raise NotImplementedError(sampler)
    q = pose_to_quat_rows(res)
    return res.reshape(B, K, -1), q.reshape(B, K, -1), feat, extra


def get_energy(sd, pts: np.ndarray, pts_center: np.ndarray, pose_samples: np.ndarray, T: float):
    """``PoseNet.get_energy(mode='test', extract_feature=True)`` (posenet_agent.py:608-705)."""
    B, K = pose_samples.shape[:2]
    feat = encoder_forward(sd, pts)
    rows = pose_samples.reshape(B * K, -1).astype(F32).copy()
    rows[:, 6:] -= np.repeat(pts_center.astype(F32), K, axis=0)
    t = np.full((B * K, 1), F32(T), dtype=F32)
    return energy_forward(sd, np.repeat(feat, K, 0), rows, t).reshape(B, K, 2)


# ============================================================ DINO-pointwise fused encoder (Pointnet2ClsMSGFus)
def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=F32))


def sa_level(sd, prefix: str, lv: int, branches, xyz: np.ndarray, feats: Optional[np.ndarray]):
    """One PointnetSAModuleMSG level (pointnet2_modules.py:19-124) over (B,N,3) xyz and (B,C,N) features:
    FPS + gather, ball query + group per branch, SharedMLP, max-pool. Returns (new_xyz | None, (B,C_out,M))."""
    npoint = arch.NPOINTS[lv]
    if npoint is not None:
        fidx = furthest_point_sample(xyz, npoint)
        new_xyz = gather_operation(xyz.transpose(0, 2, 1), fidx).transpose(0, 2, 1).copy()
    else:
        fidx, new_xyz = None, None
    outs = []
    for br in branches:
        if npoint is not None:
            idx = ball_query(br.radius, br.nsample, xyz, new_xyz)
            gx = grouping_operation(xyz.transpose(0, 2, 1), idx) - new_xyz.transpose(0, 2, 1)[..., None]
            grouped = gx if feats is None else np.concatenate([gx, grouping_operation(feats, idx)], axis=1)
        else:
            gx = xyz.transpose(0, 2, 1)[:, :, None, :]
            grouped = gx if feats is None else np.concatenate([gx, feats[:, :, None, :]], axis=1)
        h = grouped.astype(F32)
        for i in range(len(br.widths) - 1):
            h = _conv_bn_relu(h, sd, f"{prefix}SA_modules.{lv}.mlps.{br.branch}.layer{i}")
        outs.append(h.max(axis=3))
    return new_xyz, fidx, np.concatenate(outs, axis=1).astype(F32)


def relative_bias(sd, prefix: str, xyz: np.ndarray) -> np.ndarray:
    """EfficientRelativePositionalEncoding.forward (attention.py:680-735): rel[b,i,j] = xyz[j] - xyz[i];
    distance / direction encoders (Linear -> ReLU -> Linear), fusion Linear(16, 8) -> (B, 8, N, N)."""
    import torch
    import torch.nn.functional as tf
    w = lambda k: _t(sd[f"{prefix}.{k}"])  # noqa: E731
    x = _t(xyz)
    rel = x.unsqueeze(1) - x.unsqueeze(2)
    dist = torch.norm(rel, dim=-1, keepdim=True)
    db = tf.linear(torch.relu(tf.linear(dist, w("distance_encoder.0.weight"), w("distance_encoder.0.bias"))),
                   w("distance_encoder.2.weight"), w("distance_encoder.2.bias"))
    direction = rel / (torch.norm(rel, dim=-1, keepdim=True) + 1e-7)
    ob = tf.linear(torch.relu(tf.linear(direction, w("direction_encoder.0.weight"), w("direction_encoder.0.bias"))),
                   w("direction_encoder.2.weight"), w("direction_encoder.2.bias"))
    fused = tf.linear(torch.cat([db, ob], dim=-1), w("fusion.weight"), w("fusion.bias"))
    return fused.permute(0, 3, 1, 2).contiguous().numpy()


def transformer_block(sd, prefix: str, x: np.ndarray, bias: Optional[np.ndarray]) -> np.ndarray:
    """TransformerBlockWithRelativePE.forward (attention.py:505-533) over MultiheadAttentionWithRelativePE
    (attention.py:436-488), eval mode (dropout = identity). x (B, C, N) -> (B, C, N)."""
    import math
    import torch
    import torch.nn.functional as tf
    w = lambda k: _t(sd[f"{prefix}.{k}"])  # noqa: E731
    xt = _t(x).transpose(1, 2).contiguous()
    Bn, Nn, C = xt.shape
    H = arch.FUS_HEADS
    hd = C // H

    def heads(nm):
        return tf.linear(xt, w(f"self_attn.{nm}.weight"), w(f"self_attn.{nm}.bias")).view(Bn, Nn, H, hd).transpose(1, 2)
    q, k, v = heads("wq"), heads("wk"), heads("wv")
    s = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(hd)
    if bias is not None:
        s = s + _t(bias)
    o = torch.matmul(torch.softmax(s, dim=-1), v).transpose(1, 2).contiguous().view(Bn, Nn, C)
    o = tf.linear(o, w("self_attn.wo.weight"), w("self_attn.wo.bias"))
    xt = tf.layer_norm(xt + o, (C,), w("norm1.weight"), w("norm1.bias"), arch.LN_EPS)
    f = tf.linear(torch.relu(tf.linear(xt, w("linear1.weight"), w("linear1.bias"))), w("linear2.weight"), w("linear2.bias"))
    xt = tf.layer_norm(xt + f, (C,), w("norm2.weight"), w("norm2.bias"), arch.LN_EPS)
    return xt.transpose(1, 2).contiguous().numpy()


def _conv1d_bn(x, sd, prefix, act):
    """Conv1d(k=1, bias) -> BatchNorm1d(eval) -> act (attention.py:262-281 Sequentials)."""
    import torch
    import torch.nn.functional as tf
    w = lambda k: _t(sd[f"{prefix}.{k}"])  # noqa: E731
    y = tf.conv1d(x, w("0.weight"), w("0.bias"))
    y = tf.batch_norm(y, w("1.running_mean"), w("1.running_var"), w("1.weight"), w("1.bias"), training=False,
                      eps=arch.BN_EPS)
    return act(y)


def gated_fusion(sd, prefix: str, cur: np.ndarray, orig: np.ndarray) -> np.ndarray:
    """GatedAttentionFusion.forward (attention.py:284-325): cur (B, C, N), orig (B, 384, N) -> (B, C, N)."""
    import torch
    import torch.nn.functional as tf
    w = lambda k: _t(sd[f"{prefix}.{k}"])  # noqa: E731
    c, o = _t(cur), _t(orig)
    ot = _conv1d_bn(o, sd, f"{prefix}.original_transform", torch.relu)
    ca = torch.mean(torch.cat([c, ot], dim=1), dim=2, keepdim=True)          # AdaptiveAvgPool1d(1)
    ca = torch.relu(tf.conv1d(ca, w("channel_attention.1.weight"), w("channel_attention.1.bias")))
    ca = torch.sigmoid(tf.conv1d(ca, w("channel_attention.3.weight"), w("channel_attention.3.bias")))
    sp_in = torch.cat([torch.max(c, dim=1, keepdim=True)[0], torch.mean(c, dim=1, keepdim=True)], dim=1)
    sp = torch.sigmoid(tf.conv1d(sp_in, w("spatial_attention.0.weight"), None, padding=arch.FUS_SPATIAL_K // 2))
    att = ot * ca * sp
    g = _conv1d_bn(torch.cat([c, att], dim=1), sd, f"{prefix}.gate", torch.sigmoid)
    fused = g * c + (1 - g) * att
    return _conv1d_bn(fused, sd, f"{prefix}.output_conv", torch.relu).numpy()


def interp_points(x: np.ndarray, n_out: int) -> np.ndarray:
    """F.interpolate(x, size=n_out, mode="linear", align_corners=False) along the point index
    (pointnet2.py:344-350): x (B, C, N)."""
    import torch.nn.functional as tf
    return tf.interpolate(_t(x), size=n_out, mode="linear", align_corners=False).numpy()


def fus_encoder_forward(sd, pts: np.ndarray, rgb_feat: np.ndarray, return_levels: bool = False):
    """Pointnet2ClsMSGFus.forward (pointnet2.py:331-380), eval mode: pts (B,N,3), rgb_feat (B,N,384) -> (B,1024).
    The reference's gather of `features` at the end of each level (:370-377) feeds nothing and is omitted."""
    p = "pts_encoder."
    xyz = np.ascontiguousarray(pts[..., :3], dtype=F32)
    orig = np.ascontiguousarray(rgb_feat.transpose(0, 2, 1), dtype=F32)    # (B, 384, N)
    feats = orig
    levels = []
    for lv, branches in enumerate(arch.fus_sa_branches()):
        rec = {}
        if lv > 0:
            if orig.shape[2] != feats.shape[2]:
                orig = interp_points(orig, feats.shape[2])
            feats = gated_fusion(sd, f"{p}feature_fusions.{lv - 1}", feats, orig)
            rec["fused"] = feats
        new_xyz, fidx, feats = sa_level(sd, p, lv, branches, xyz, feats)
        rec.update(sa=feats, fps_idx=fidx)
        bias = relative_bias(sd, f"{p}relative_pos_encoders.{lv}", new_xyz) if new_xyz is not None else None
        feats = transformer_block(sd, f"{p}transformer_blocks.{lv}", feats, bias)
        rec["tf"] = feats
        if lv == 3:
            rec["bias"] = bias
        levels.append(rec)
        if new_xyz is not None:
            xyz = new_xyz
    out = feats[:, :, 0]
    return (out, levels) if return_levels else out


# ============================================================ ImgEncoder + patch gather (--dino pointwise)
def img_geo_bias(sd, prefix: str = "img_encoder", grid: int = arch.IMG_GRID) -> np.ndarray:
    """rel_pos_emb(rel_pos_idx).sum(-1) of ImgEncoder.forward (img_encoder.py:68-76, rel_coords :18-34):
    (np, np) with [i][j] = sum_d E[clamp((c_j - c_i + h - 1) . (2h - 1, 1), 0, 899)][d], c_p = (p // h, p % h)."""
    import torch
    h = grid
    coords = np.stack(np.meshgrid(np.arange(h), np.arange(h), indexing="ij"), -1).reshape(-1, 2)
    rel = coords[None, :, :] - coords[:, None, :] + (h - 1)
    E = torch.from_numpy(np.ascontiguousarray(sd[f"{prefix}.rel_pos_emb.weight"], dtype=F32))
    idx = np.clip(rel[..., 0] * (2 * (h - 1) + 1) + rel[..., 1], 0, E.shape[0] - 1)
    return E.sum(dim=-1).numpy()[idx]


def img_encoder_forward(sd, layers, prefix: str = "img_encoder", return_parts: bool = False):
    """ImgEncoder.forward (networks/img_encoder/img_encoder.py:48-100), eval: three (B, np, d) DINOv3
    intermediate layers -> (B, np, d): layer attention (softmax over the 3 layers), geometric attention
    (G G^T x the position table, softmax, . fused), 3x3 edge conv -> ReLU -> mean, final mix."""
    import torch
    import torch.nn.functional as tf
    t = lambda k: torch.from_numpy(np.ascontiguousarray(sd[f"{prefix}.{k}"], dtype=F32))  # noqa: E731
    f = torch.stack([torch.from_numpy(np.ascontiguousarray(v, dtype=F32)) for v in layers], 1)   # (B, 3, np, d)
    B, _, n, d = f.shape
    h = int(round(n ** 0.5))
    s = tf.linear(torch.relu(tf.linear(f, t("layer_attn.0.weight"), t("layer_attn.0.bias"))),
                  t("layer_attn.2.weight"), t("layer_attn.2.bias"))                           # (B, 3, np, 1)
    w = torch.softmax(s, dim=1)
    fused = (f * w).sum(dim=1)                                                               # (B, np, d)
    g = fused[:, :, d // 4:]
    attn = torch.softmax(torch.matmul(g, g.transpose(1, 2)) * torch.from_numpy(img_geo_bias(sd, prefix, h)), dim=-1)
    geo = torch.matmul(attn, fused)
    sp = fused.transpose(1, 2).reshape(B, d, h, h)
    edge = torch.relu(tf.conv2d(sp, t("edge_guide.0.weight"), t("edge_guide.0.bias"), padding=1)).mean(dim=(2, 3))
    final = fused + torch.relu(t("geo_weight")) * geo + torch.relu(t("edge_weight")) * (fused * edge.repeat(1, 4)[:, None, :])
    if return_parts:
        return final.numpy(), {"layer_w": w[..., 0].numpy(), "edge": edge.numpy(), "fused": fused.numpy()}
    return final.numpy()


def gather_patch_points(feat: np.ndarray, xs: np.ndarray, ys: np.ndarray, patch_px: int = arch.IMG_PATCH_PX,
                        grid: int = arch.IMG_GRID) -> np.ndarray:
    """posenet.py:146-192: pos = (roi_xs // 14) * 16 + roi_ys // 14 (floor division), clamped to the patch
    range, then torch.gather along the patch axis: (B, np, d) -> (B, N, d)."""
    pos = np.clip((np.asarray(xs) // patch_px) * grid + np.asarray(ys) // patch_px, 0, feat.shape[1] - 1)
    return np.take_along_axis(feat, pos[..., None].astype(np.int64), 1)
