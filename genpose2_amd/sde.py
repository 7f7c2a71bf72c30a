"""VE SDE scalars, formed exactly as the reference forms them (so the per-step constants handed
to the kernels are bit-identical to the reference's): networks/gf_algorithms/sde.py:15-35,110-119
and the time grid of cond_pc_sampler (samplers.py:129-130).

These are host-side control values (T scalars per call), not per-candidate work."""
from __future__ import annotations

import numpy as np
import torch

from . import arch

_DIFF_SCALE_T = torch.sqrt(torch.tensor(2 * (np.log(arch.SIGMA_MAX) - np.log(arch.SIGMA_MIN))))  # float64


def sigma(t: torch.Tensor) -> torch.Tensor:
    """ve_marginal_prob std: sigma_min * (sigma_max / sigma_min) ** t (dtype of t)."""
    return arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** t


def diffusion(t: torch.Tensor) -> torch.Tensor:
    """ve_sde diffusion coefficient sigma(t) * sqrt(2 (ln sigma_max - ln sigma_min))."""
    return sigma(t) * _DIFF_SCALE_T


def prior_sigma(T: float = arch.SDE_T) -> float:
    """ve_prior scale sigma(T) as a python float (sde.py:30-34)."""
    return arch.SIGMA_MIN * (arch.SIGMA_MAX / arch.SIGMA_MIN) ** T


def pc_step_table(num_steps: int, eps: float = arch.SAMPLING_EPS) -> np.ndarray:
    """(T, 5) float32 rows {t, sigma(t), g(t), dt, sqrt(dt)} for cond_pc_sampler."""
    ts = torch.linspace(1.0, eps, num_steps)
    step_size = ts[0] - ts[1]
    bt = ts.unsqueeze(-1)                       # batch_time_step values (one per step)
    sig = sigma(bt)[:, 0]
    g = diffusion(bt)[:, 0]
    tab = torch.stack([ts, sig, g, step_size.expand(num_steps), torch.sqrt(step_size).expand(num_steps)], 1)
    return tab.to(torch.float32).numpy().copy()
