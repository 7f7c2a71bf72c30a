"""Synthetic segmented object point clouds (SURVEY §8d "Synthetic inputs").

Per object: points on the surface of a random box or ellipsoid (half-extents U[2,10] cm),
random SO(3) rotation, centre at z~U[0.5,1.0] m, x,y~U[-0.1,0.1] m, Gaussian jitter 1 mm.
Seed = 1000*config_id + object index (numpy PCG64), so every machine regenerates the same
clouds. ``n_unique < n_points`` reproduces the dataset's tile padding
(``datasets_omni6dpose.py:455-471``), which creates exact duplicate points (FPS ties).

``make_batch`` returns the two keys the path reads from ``process_batch``
(``datasets_omni6dpose.py:708-752``): ``pts`` (B,N,3) un-centred and ``pts_center`` (B,3)
= mean of pts.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


def _random_rotation(rng: np.random.Generator) -> np.ndarray:
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def object_cloud(seed: int, n_points: int = 1024, n_unique: Optional[int] = None) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    n_u = n_points if n_unique is None else n_unique
    half = rng.uniform(0.02, 0.10, size=3)
    if rng.uniform() < 0.5:   # box surface: pick a face, uniform on it
        face = rng.integers(0, 6, size=n_u)
        p = rng.uniform(-1.0, 1.0, size=(n_u, 3))
        ax = face // 2
        p[np.arange(n_u), ax] = np.where(face % 2 == 0, -1.0, 1.0)
        p = p * half
    else:                     # ellipsoid surface
        d = rng.normal(size=(n_u, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        p = d * half
    R = _random_rotation(rng)
    centre = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.5, 1.0)])
    p = p @ R.T + centre + rng.normal(scale=1e-3, size=(n_u, 3))
    if n_u < n_points:        # tile padding, datasets_omni6dpose.py:455-471
        p = np.concatenate([np.tile(p, (n_points // n_u, 1)), p[: n_points % n_u]], axis=0)
    return p.astype(np.float32)


def make_batch(config_id: int, batch: int, n_points: int = 1024, n_unique_every: int = 0,
               first_object: int = 0):
    """(pts (B,N,3) float32, pts_center (B,3) float32). Every ``n_unique_every``-th object
    (if >0) is tile-padded from 300 unique points."""
    pts = np.stack([
        object_cloud(1000 * config_id + first_object + i, n_points,
                     300 if (n_unique_every and (first_object + i) % n_unique_every == 0) else None)
        for i in range(batch)])
    return pts, pts.mean(axis=1).astype(np.float32)
