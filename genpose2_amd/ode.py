"""Probability-flow ODE sampler (cond_ode_sampler, samplers.py:180-258) with a device-resident
Dormand-Prince 5(4) integrator.

The reference hands the float64 state to scipy ``solve_ivp(method="RK45")`` on the host and pays
one device->host and one host->device copy per right-hand-side evaluation (samplers.py:207-219).
Here the state, the 7 stages and every stage combination stay in HBM (float64); the score is the
HIP head kernel; only the step controller's scalars (one RMS error norm per attempted step) cross
to the host. The controller restates scipy's published RK45 (scipy 1.15 ``_ivp/rk.py``:
``rk_step``, ``_step_impl``, ``RkDenseOutput``; ``_ivp/common.py``: ``select_initial_step``,
RMS ``norm``; ``_ivp/ivp.py`` t_eval handling), which the reference pins only as
``scipy`` (requirements.txt:2, commented ``scipy==1.12.0``).
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Tuple

import numpy as np
import torch

# Dormand-Prince tableau as in scipy RK45
_C = [0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0]
_A = [[], [1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9],
      [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
      [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]]
_B = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]
_E = [-71 / 57600, 0.0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40]
_P = np.array([
    [1, -8048581381 / 2820520608, 8663915743 / 2820520608, -12715105075 / 11282082432],
    [0, 0, 0, 0],
    [0, 131558114200 / 32700410799, -68118460800 / 10900136933, 87487479700 / 32700410799],
    [0, -1754552775 / 470086768, 14199869525 / 1410260304, -10690763975 / 1880347072],
    [0, 127303824393 / 49829197408, -318862633887 / 49829197408, 701980252875 / 199316789632],
    [0, -282668133 / 205662961, 2019193451 / 616988883, -1453857185 / 822651844],
    [0, 40617522 / 29380423, -110615467 / 29380423, 69997945 / 29380423]])
SAFETY, MIN_FACTOR, MAX_FACTOR = 0.9, 0.2, 10.0
ERR_EXP = -1.0 / 5.0


def _rms(x: torch.Tensor) -> float:
    return float(torch.linalg.vector_norm(x).item()) / math.sqrt(x.numel())


def _lin(coefs, ks, h=None):
    acc = None
    for c, k in zip(coefs, ks):
        if c == 0.0:
            continue
        acc = k * c if acc is None else acc + k * c
    if acc is None:
        acc = torch.zeros_like(ks[0])
    return acc * h if h is not None else acc


def rk45_solve(fun: Callable[[float, torch.Tensor], torch.Tensor], t0: float, y0: torch.Tensor, t_bound: float,
               rtol: float = 1e-5, atol: float = 1e-5, t_eval: Optional[np.ndarray] = None):
    """Integrate y' = fun(t, y) from t0 to t_bound. Returns (ts (n,), ys (n, *y.shape), nfev)."""
    nfev = [0]

    def f(t, y):
        nfev[0] += 1
        return fun(t, y)

    direction = 1.0 if t_bound > t0 else -1.0
    t, y = float(t0), y0.clone()
    fy = f(t, y)
    # select_initial_step (order = error_estimator_order = 4)
    interval = abs(t_bound - t0)
    scale = atol + y.abs() * rtol
    d0, d1 = _rms(y / scale), _rms(fy / scale)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    h0 = min(h0, interval)
    y1 = y + (h0 * direction) * fy
    f1 = f(t + h0 * direction, y1)
    d2 = _rms((f1 - fy) / scale) / h0
    h1 = max(1e-6, h0 * 1e-3) if (d1 <= 1e-15 and d2 <= 1e-15) else (0.01 / max(d1, d2)) ** (1 / 5)
    h_abs = min(100 * h0, h1, interval)

    ts, ys = [], []
    if t_eval is None:
        ts.append(t)
        ys.append(y.clone())
    else:
        t_eval = np.asarray(t_eval, dtype=np.float64)
        if direction < 0:
            t_eval = t_eval[::-1]
            t_eval_i = t_eval.shape[0]
        else:
            t_eval_i = 0
    K = [None] * 7
    status = None
    while status is None:
        # ---- OdeSolver.step -> _step_impl
        min_step = 10 * abs(np.nextafter(t, direction * np.inf) - t)
        h_abs = min(max(h_abs, min_step), np.inf)
        accepted, rejected = False, False
        while not accepted:
            if h_abs < min_step:
                raise RuntimeError("RK45: required step size is less than spacing between numbers")
            h = h_abs * direction
            t_new = t + h
            if direction * (t_new - t_bound) > 0:
                t_new = t_bound
            h = t_new - t
            h_abs = abs(h)
            K[0] = fy
            for s in range(1, 6):
                K[s] = f(t + _C[s] * h, y + _lin(_A[s], K[:s], h))
            y_new = y + _lin(_B, K[:6]) * h
            f_new = f(t + h, y_new)
            K[6] = f_new
            scale = atol + torch.maximum(y.abs(), y_new.abs()) * rtol
            err = _rms(_lin(_E, K) * h / scale)
            if err < 1:
                factor = MAX_FACTOR if err == 0 else min(MAX_FACTOR, SAFETY * err ** ERR_EXP)
                if rejected:
                    factor = min(1.0, factor)
                h_abs *= factor
                accepted = True
            else:
                h_abs *= max(MIN_FACTOR, SAFETY * err ** ERR_EXP)
                rejected = True
        t_old, y_old = t, y
        t, y, fy = t_new, y_new, f_new
        if direction * (t - t_bound) >= 0:
            status = 0
        # ---- solve_ivp output collection
        if t_eval is None:
            ts.append(t)
            ys.append(y.clone())
        else:
            if direction > 0:
                new_i = int(np.searchsorted(t_eval, t, side="right"))
                step_t = t_eval[t_eval_i:new_i]
            else:
                new_i = int(np.searchsorted(t_eval, t, side="left"))
                step_t = t_eval[new_i:t_eval_i][::-1]
            if step_t.size > 0:
                Q = torch.stack(K, -1) @ torch.from_numpy(_P).to(y.device)        # (n, 4)
                hh = t - t_old
                for te in step_t:
                    x = (te - t_old) / hh
                    p = torch.tensor(np.cumprod(np.tile(x, 4)), dtype=torch.float64, device=y.device)
                    ts.append(float(te))
                    ys.append(hh * (Q @ p) + y_old)
                t_eval_i = new_i
    return np.asarray(ts), torch.stack(ys, 0), nfev[0]
