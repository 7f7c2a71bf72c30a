"""Probability-flow ODE sampler (cond_ode_sampler, samplers.py:180-258) with a device-resident
Dormand-Prince 5(4) integrator.

The reference hands the float64 state to scipy ``solve_ivp(method="RK45")`` on the host and pays
one device->host and one host->device copy per right-hand-side evaluation (samplers.py:207-219).
Here the state, the 7 stage derivatives and every stage combination stay in HBM (float64): one
HIP launch per stage (``gp_ode_attempt`` fuses the stage combination, the score heads and the
error estimate). Only the step controller's scalars cross to the host: one 8-byte error norm per
attempted step.

The controller (``rk45_drive``) restates scipy's published RK45 line by line, with the same
Python/NumPy scalar types (scipy 1.15 ``_ivp/rk.py``: ``RK45``, ``rk_step``, ``_step_impl``,
``RkDenseOutput``; ``_ivp/common.py``: ``select_initial_step``, RMS ``norm``; ``_ivp/base.py``:
``OdeSolver.step``; ``_ivp/ivp.py``: ``solve_ivp`` t_eval handling). The reference pins scipy only as
``scipy`` (requirements.txt:2, commented ``scipy==1.12.0``). The arithmetic lives in a backend:
``DeviceRk45`` (HIP, the product path) or ``NumpyRk45`` (scipy's own NumPy expressions; used by the
CPU tests to hold the controller to ``solve_ivp`` exactly).
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
import warnings
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib, arch, sde
from ._lib import check

# Dormand-Prince tableau exactly as scipy's RK45 class attributes
C = np.array([0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1])
A = np.array([
    [0, 0, 0, 0, 0],
    [1 / 5, 0, 0, 0, 0],
    [3 / 40, 9 / 40, 0, 0, 0],
    [44 / 45, -56 / 15, 32 / 9, 0, 0],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729, 0],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]])
B = np.array([35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84])
E = np.array([-71 / 57600, 0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40])
P = np.array([
    [1, -8048581381 / 2820520608, 8663915743 / 2820520608, -12715105075 / 11282082432],
    [0, 0, 0, 0],
    [0, 131558114200 / 32700410799, -68118460800 / 10900136933, 87487479700 / 32700410799],
    [0, -1754552775 / 470086768, 14199869525 / 1410260304, -10690763975 / 1880347072],
    [0, 127303824393 / 49829197408, -318862633887 / 49829197408, 701980252875 / 199316789632],
    [0, -282668133 / 205662961, 2019193451 / 616988883, -1453857185 / 822651844],
    [0, 40617522 / 29380423, -110615467 / 29380423, 69997945 / 29380423]])
N_STAGES = 6
ERROR_ESTIMATOR_ORDER = 4
SAFETY, MIN_FACTOR, MAX_FACTOR = 0.9, 0.2, 10
ERROR_EXPONENT = -1 / (ERROR_ESTIMATOR_ORDER + 1)


# ============================================================================ controller
def initial_step(be, t0: float, tf: float, direction):
    """RK45.__init__: f = fun(t0, y0) and h_abs = select_initial_step(...) (common.py), over backend
    `be` (rhs0, init_norms, rhs_euler, diff_norm). Returns (h_abs, nfev)."""
    interval_length = abs(tf - t0)
    if interval_length == 0.0:
        raise ValueError("RK45: empty integration interval (T0 == eps)")
    nfev = 1
    be.rhs0(t0)
    d0, d1 = be.init_norms()
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = 1e-6
    else:
        h0 = 0.01 * d0 / d1
    h0 = min(h0, interval_length)
    be.rhs_euler(t0 + h0 * direction, h0 * direction)
    nfev += 1
    d2 = be.diff_norm() / h0
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = max(1e-6, h0 * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1 / (ERROR_ESTIMATOR_ORDER + 1))
    return min(100 * h0, h1, interval_length, np.inf), nfev


def rk45_drive(be, t0: float, t_bound: float, rtol: float = 1e-5, atol: float = 1e-5,
               t_eval: Optional[np.ndarray] = None, keep_all: bool = True, trace: Optional[list] = None):
    """solve_ivp(fun, (t0, t_bound), y0, method="RK45", rtol, atol, t_eval) over backend `be`.

    `be` holds y0 and provides: set_t_eval, rhs0(t), init_norms(), rhs_euler(t, h), diff_norm(),
    attempt(t, h) -> error norm, dense(t_old, t, lo, hi), accept(t_old, t), keep_y(keep, first).
    Returns (ts, nfev, status); the outputs stay in the backend (``be.ys`` for t_eval=None, the
    dense rows otherwise). With keep_all=False
    only the final output is kept (the value ``res.y[:, -1]`` that pred_func uses). ``trace``: a list that
    receives [t, h, error norm] per step attempt (scipy's _estimate_error_norm; accepted iff norm < 1).
    """
    t0, tf = map(float, (t0, t_bound))                          # ivp.py: t0, tf = map(float, t_span)
    direction = np.sign(tf - t0) if tf != t0 else 1             # base.py OdeSolver.__init__
    if t_eval is not None:
        t_eval = np.asarray(t_eval)
        if np.any(t_eval < min(t0, tf)) or np.any(t_eval > max(t0, tf)):
            raise ValueError("Values in `t_eval` are not within `t_span`.")
        if tf > t0:
            t_eval_i = 0
        else:
            t_eval = t_eval[::-1]
            t_eval_i = t_eval.shape[0]
        be.set_t_eval(np.ascontiguousarray(t_eval), direction, keep_all)
    h_abs, nfev = initial_step(be, t0, tf, direction)
    ts: List[float] = [t0] if t_eval is None else []
    if t_eval is None:
        be.keep_y(keep_all, first=True)
    t = t0
    status = None
    while status is None:
        # ---- OdeSolver.step (t == t_bound cannot hold here: the loop ends when t reaches it)
        # ---- RK45._step_impl
        min_step = 10 * np.abs(np.nextafter(t, direction * np.inf) - t)
        if h_abs > np.inf:
            h_abs = np.inf
        elif h_abs < min_step:
            h_abs = min_step
        step_accepted = False
        step_rejected = False
        failed = False
        while not step_accepted:
            if h_abs < min_step:
                failed = True
                break
            h = h_abs * direction
            t_new = t + h
            if direction * (t_new - tf) > 0:
                t_new = tf
            h = t_new - t
            h_abs = np.abs(h)
            error_norm = be.attempt(t, h)
            nfev += N_STAGES
            if trace is not None:
                trace.append([float(t), float(h), float(error_norm)])
            if error_norm < 1:
                if error_norm == 0:
                    factor = MAX_FACTOR
                else:
                    factor = min(MAX_FACTOR, SAFETY * error_norm ** ERROR_EXPONENT)
                if step_rejected:
                    factor = min(1, factor)
                h_abs *= factor
                step_accepted = True
            else:
                h_abs *= max(MIN_FACTOR, SAFETY * error_norm ** ERROR_EXPONENT)
                step_rejected = True
        if failed:
            # solve_ivp returns (status -1) with the outputs collected so far; the reference then
            # uses res.y[:, -1] as is
            warnings.warn("RK45: required step size is less than spacing between numbers.")
            status = -1
            if t_eval is None and not keep_all:
                be.keep_y(True, first=False)
            break
        t_old = t
        t = t_new
        if direction * (t - tf) >= 0:
            status = 0
        # ---- solve_ivp output collection
        if t_eval is None:
            ts.append(t)
            be.accept(t_old, t)
            be.keep_y(keep_all or status is not None, first=False)
        else:
            if direction > 0:
                t_eval_i_new = int(np.searchsorted(t_eval, t, side="right"))
                lo, hi = t_eval_i, t_eval_i_new
            else:
                t_eval_i_new = int(np.searchsorted(t_eval, t, side="left"))
                lo, hi = t_eval_i_new, t_eval_i
            if hi > lo:
                be.dense(t_old, t, lo, hi)
                ts.extend(t_eval[lo:hi][::-1] if direction < 0 else t_eval[lo:hi])
                t_eval_i = t_eval_i_new
            be.accept(t_old, t)
    return np.asarray(ts, dtype=np.float64), nfev, status


# ============================================================================ NumPy backend
class NumpyRk45:
    """scipy's own expressions (rk.py rk_step, _estimate_error_norm, RkDenseOutput; common.py norm)
    over an arbitrary fun(t, y). Used by the CPU tests to hold the controller to solve_ivp."""

    def __init__(self, fun, y0: np.ndarray, rtol: float = 1e-5, atol: float = 1e-5):
        self.fun = fun
        self.y = np.asarray(y0, dtype=float)
        self.rtol, self.atol = rtol, atol
        self.K = np.empty((N_STAGES + 1, self.y.shape[0]), dtype=self.y.dtype)
        self.ys: List[np.ndarray] = []
        self.dense_rows: List[Tuple[float, np.ndarray]] = []

    @staticmethod
    def _norm(x):
        return np.linalg.norm(x) / x.size ** 0.5

    def set_t_eval(self, t_eval, direction, keep_all):
        self.t_eval, self.direction = t_eval, direction

    def rhs0(self, t):
        self.f = self.fun(t, self.y)

    def init_norms(self):
        self.scale0 = self.atol + np.abs(self.y) * self.rtol
        return self._norm(self.y / self.scale0), self._norm(self.f / self.scale0)

    def rhs_euler(self, t, h):
        y1 = self.y + h * self.f
        self.f1 = self.fun(t, y1)

    def diff_norm(self):
        return self._norm((self.f1 - self.f) / self.scale0)

    def attempt(self, t, h):
        K, y = self.K, self.y
        K[0] = self.f
        for s, (a, c) in enumerate(zip(A[1:], C[1:]), start=1):
            dy = np.dot(K[:s].T, a[:s]) * h
            K[s] = self.fun(t + c * h, y + dy)
        y_new = y + h * np.dot(K[:-1].T, B)
        f_new = self.fun(t + h, y_new)
        K[-1] = f_new
        self.y_new, self.f_new = y_new, f_new
        scale = self.atol + np.maximum(np.abs(y), np.abs(y_new)) * self.rtol
        return self._norm(np.dot(K.T, E) * h / scale)

    def accept(self, t_old, t):
        self.y_old = self.y
        self.y, self.f = self.y_new, self.f_new

    def keep_y(self, keep, first):
        if keep:
            self.ys.append(self.y.copy())

    def dense(self, t_old, t, lo, hi):
        Q = self.K.T.dot(P)
        h = t - t_old
        te = self.t_eval[lo:hi][::-1] if self.direction < 0 else self.t_eval[lo:hi]
        x = (te - t_old) / h
        p = np.cumprod(np.tile(x, (Q.shape[1], 1)), axis=0)
        y = h * np.dot(Q, p)
        y += self.y[:, None]
        for j in range(te.shape[0]):
            self.dense_rows.append((float(te[j]), y[:, j]))


# ============================================================================ HIP backend
def _ptr_array(ts) -> ctypes.Array:
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


_A6 = np.zeros((6, 6), dtype=np.float64)
_A6[:, :5] = A
_A6 = np.ascontiguousarray(_A6)
_B6 = np.ascontiguousarray(B, dtype=np.float64)
_E7 = np.ascontiguousarray(E, dtype=np.float64)
_P74 = np.ascontiguousarray(P, dtype=np.float64)


def time_scalars(t):
    """Per-RHS scalars exactly as ode_func forms them (samplers.py:209-216): the score model sees
    t32 = float32(t) and sigma(t32) in fp32; the coefficient is -(0.5 * g^2) with
    g = sde_coeff(torch.tensor(t)) -- float32 when t is a Python float (the first evaluation at
    t0, ivp.py maps t_span to float), float64 for the NumPy scalars of every later evaluation."""
    t32 = float(np.float32(t))
    sig = float(sde.sigma(torch.tensor([t32], dtype=torch.float32))[0])
    g = sde.diffusion(torch.tensor(t)).numpy()
    coef = -(0.5 * (g ** 2))
    return t32, sig, float(coef)


def stage_scalars(ts: List[float]):
    """time_scalars for the 6 stage times of one attempt in one vectorised pass (the stage times
    are NumPy float64, so g is float64). Bitwise equal to per-value time_scalars
    (tests/test_cpu_host.py::test_ode_stage_scalars_vectorised)."""
    tt = np.asarray(ts, dtype=np.float64)
    t32 = tt.astype(np.float32)
    sig = sde.sigma(torch.from_numpy(t32)).numpy().astype(np.float32)
    g = sde.diffusion(torch.from_numpy(tt)).numpy()
    coef = -(0.5 * (g ** 2))
    return (np.ascontiguousarray(t32), np.ascontiguousarray(sig), np.ascontiguousarray(coef, dtype=np.float64))


class DeviceRk45:
    """State y, K_0..K_6 and y_new as fp64 (R*9) device tensors; every RHS is a HIP launch."""

    def __init__(self, heads, pobj: torch.Tensor, y0: torch.Tensor, k: int, rtol: float = 1e-5,
                 atol: float = 1e-5):
        self.lib = _lib.load()
        self.h = heads
        self.dev = heads.device
        self.pobj = pobj
        self.R = y0.numel() // arch.POSE_DIM
        self.n = self.R * arch.POSE_DIM
        self.k = int(k)
        self.rtol, self.atol = float(rtol), float(atol)
        self.y = y0.reshape(-1).to(self.dev, torch.float64).contiguous()
        self.K = [torch.empty(self.n, dtype=torch.float64, device=self.dev) for _ in range(N_STAGES + 1)]
        self.f1 = torch.empty(self.n, dtype=torch.float64, device=self.dev)
        nb = int(self.lib.gp_ode_workspace_size(self.R))
        self.ws = torch.empty(nb, dtype=torch.uint8, device=self.dev)
        self.scal = torch.zeros(8, dtype=torch.float64, device=self.dev)   # [d0, d1, d2, err]
        self.ys: List[torch.Tensor] = []
        self.dense_out: Optional[torch.Tensor] = None
        self.t_eval_dev = None

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _rhs(self, t, kin, acoef, h, kout):
        t32, sig, coef = time_scalars(t)
        nk = len(kin)
        karr = _ptr_array(kin) if nk else None
        aarr = (ctypes.c_double * nk)(*acoef) if nk else None
        check(self.lib.gp_ode_rhs(ctypes.byref(self.h.w), ctypes.c_void_p(self.pobj.data_ptr()), t32, sig, coef,
                                  ctypes.c_void_p(self.y.data_ptr()), karr, aarr, nk, float(h), self.R, self.k,
                                  ctypes.c_void_p(kout.data_ptr()), ctypes.c_void_p(self.ws.data_ptr()),
                                  self.ws.numel(), self._s()), "ode_rhs")

    def set_t_eval(self, t_eval, direction, keep_all):
        self.t_eval = t_eval
        self.direction = direction
        self.keep_all = keep_all
        self.t_eval_dev = torch.from_numpy(np.ascontiguousarray(t_eval, dtype=np.float64)).to(self.dev)
        rows = t_eval.shape[0] if keep_all else 1
        self.dense_out = torch.empty((rows, self.n), dtype=torch.float64, device=self.dev)
        self.n_dense = 0    # t_eval points collected so far (solve_ivp order: the first n_dense rows)

    def rhs0(self, t):
        self._rhs(t, [], [], 0.0, self.K[0])

    def init_norms(self):
        check(self.lib.gp_ode_init_norms(ctypes.c_void_p(self.y.data_ptr()), ctypes.c_void_p(self.K[0].data_ptr()),
                                         None, self.n, self.atol, self.rtol, ctypes.c_void_p(self.scal.data_ptr()),
                                         self._s()), "ode_init_norms")
        v = self.scal[:2].cpu().numpy()
        return v[0], v[1]

    def rhs_euler(self, t, h):
        self._rhs(t, [self.K[0]], [1.0], h, self.f1)

    def diff_norm(self):
        check(self.lib.gp_ode_init_norms(ctypes.c_void_p(self.y.data_ptr()), ctypes.c_void_p(self.K[0].data_ptr()),
                                         ctypes.c_void_p(self.f1.data_ptr()), self.n, self.atol, self.rtol,
                                         ctypes.c_void_p(self.scal.data_ptr()), self._s()), "ode_init_norms")
        return self.scal[2:3].cpu().numpy()[0]

    def attempt(self, t, h):
        stage_t = [t + c * h for c in C[1:]] + [t + h]   # rk_step: fun(t + c * h, ...) for s = 1..5, then t + h
        t32, sig, coef = stage_scalars(stage_t)
        self.y_new = torch.empty(self.n, dtype=torch.float64, device=self.dev)
        check(self.lib.gp_ode_attempt(
            ctypes.byref(self.h.w), ctypes.c_void_p(self.pobj.data_ptr()), t32.ctypes.data_as(ctypes.c_void_p),
            sig.ctypes.data_as(ctypes.c_void_p), coef.ctypes.data_as(ctypes.c_void_p),
            ctypes.c_void_p(self.y.data_ptr()), _ptr_array(self.K), _A6.ctypes.data_as(ctypes.c_void_p),
            _B6.ctypes.data_as(ctypes.c_void_p), _E7.ctypes.data_as(ctypes.c_void_p), float(h), self.rtol,
            self.atol, self.R, self.k, ctypes.c_void_p(self.y_new.data_ptr()),
            ctypes.c_void_p(self.scal[3:].data_ptr()), ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(),
            self._s()), "ode_attempt")
        return self.scal[3:4].cpu().numpy()[0]

    def accept(self, t_old, t):
        self.y_old = self.y
        self.y = self.y_new
        self.K[0], self.K[N_STAGES] = self.K[N_STAGES], self.K[0]   # FSAL: f = f_new

    def keep_y(self, keep, first):
        if keep:
            self.ys.append(self.y)

    def dense(self, t_old, t, lo, hi):
        """Called before accept(): self.y is still the step's y_old, K the step's stages."""
        h = t - t_old
        if self.keep_all:
            i0, i1, base, rev = lo, hi, (self.t_eval.shape[0] - 1 if self.direction < 0 else 0), int(self.direction < 0)
            self.n_dense += max(0, hi - lo)
        else:   # only the final t_eval point (t_bound side) is kept
            last = 0 if self.direction < 0 else self.t_eval.shape[0] - 1
            if not (lo <= last < hi):
                return
            i0, i1, base, rev = last, last + 1, last, 0
        check(self.lib.gp_ode_dense(_ptr_array(self.K), _P74.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.c_void_p(self.y.data_ptr()), ctypes.c_void_p(self.t_eval_dev.data_ptr()),
                                    i0, i1, base, rev, float(t_old), float(h), self.n,
                                    ctypes.c_void_p(self.dense_out.data_ptr()), self._s()), "ode_dense")

    def outputs(self) -> torch.Tensor:
        """(n_t, R*9) fp64 outputs in solve_ivp order (all kept, or only the last). After a failed
        solve (status -1) with keep_all, only the t_eval points collected before the failure."""
        if self.dense_out is not None:
            return self.dense_out[: self.n_dense] if self.keep_all else self.dense_out
        return torch.stack(self.ys, 0)


class GlobalDeviceRk45(DeviceRk45):
    """DeviceRk45 for one shard of a global-batch solve (shard.GlobalBatch ``gb``: this rank holds the rows of
    objects [gb.lo, gb.hi), K each, of one solve_ivp call on the whole batch). select_initial_step's norms are
    taken over the WHOLE batch's y0, f0 and f1 (each shard's rows all-gathered: the same vectors and the same
    summation order as one call), and rk45_device drives the attempts through gp_ode_auto_attempt_global (the
    error norm over every shard's partials)."""

    def __init__(self, heads, pobj: torch.Tensor, y0: torch.Tensor, k: int, gb, rtol: float = 1e-5,
                 atol: float = 1e-5):
        super().__init__(heads, pobj, y0, k, rtol, atol)
        if self.R != (gb.hi - gb.lo) * self.k:
            raise ValueError(f"global-batch shard: {self.R} rows for objects [{gb.lo}, {gb.hi}) x {self.k}")
        self.gb = gb
        self.n_total = gb.total * self.k * arch.POSE_DIM
        self._y_full = self._f0_full = None

    def _full(self, v: torch.Tensor) -> torch.Tensor:
        from . import shard
        return shard.gather_shard_rows(v.view(self.R, arch.POSE_DIM), self.gb, self.k).reshape(-1).contiguous()

    def set_t_eval(self, t_eval, direction, keep_all):
        raise NotImplementedError("global-batch RK45 keeps only the final output (rk45_device)")

    def init_norms(self):
        self._y_full, self._f0_full = self._full(self.y), self._full(self.K[0])
        check(self.lib.gp_ode_init_norms(ctypes.c_void_p(self._y_full.data_ptr()),
                                         ctypes.c_void_p(self._f0_full.data_ptr()), None, self.n_total, self.atol,
                                         self.rtol, ctypes.c_void_p(self.scal.data_ptr()), self._s()), "ode_init_norms")
        v = self.scal[:2].cpu().numpy()
        return v[0], v[1]

    def diff_norm(self):
        f1 = self._full(self.f1)
        check(self.lib.gp_ode_init_norms(ctypes.c_void_p(self._y_full.data_ptr()),
                                         ctypes.c_void_p(self._f0_full.data_ptr()), ctypes.c_void_p(f1.data_ptr()),
                                         self.n_total, self.atol, self.rtol, ctypes.c_void_p(self.scal.data_ptr()),
                                         self._s()), "ode_init_norms")
        self._y_full = self._f0_full = None
        return self.scal[2:3].cpu().numpy()[0]

    def attempt(self, t, h):
        raise NotImplementedError("global-batch RK45 runs the device controller (rk45_device)")


# ============================================================================ device-controlled driver
class OdeCtl(ctypes.Structure):
    """Host mirror of the device controller record (gp_ode.hip OdeCtl)."""
    _fields_ = [("t", ctypes.c_double), ("h_abs", ctypes.c_double), ("t_old", ctypes.c_double),
                ("h_last", ctypes.c_double), ("h", ctypes.c_double), ("t_new", ctypes.c_double),
                ("h_abs_loc", ctypes.c_double), ("coef", ctypes.c_double * 6), ("t32", ctypes.c_float * 6),
                ("sig", ctypes.c_float * 6), ("status", ctypes.c_int), ("active", ctypes.c_int),
                ("rejected", ctypes.c_int), ("nfev", ctypes.c_int), ("n_acc", ctypes.c_int), ("yi", ctypes.c_int),
                ("kidx", ctypes.c_int * 7)]


_STATUS_OFF = OdeCtl.status.offset
_SIDE = {}   # device -> (side stream, pinned status word), created once


def _side_resources(dev):
    r = _SIDE.get(dev)
    if r is None:
        r = (torch.cuda.Stream(device=dev), torch.empty(1, dtype=torch.int32).pin_memory())
        _SIDE[dev] = r
    return r


# Measurement hook (bench.py): when a list, every attempt's six stage launches are bracketed by a pair of
# timing events on the launch stream, appended as (start, end, rows); the final no-op attempt is not recorded.
STAGE_EVENTS: Optional[list] = None


def _attempts_evented(launch, ws, rec, stream, side, stat, be, max_attempts: int) -> int:
    """The attempt loop with an event after each control launch and a 4-byte status copy on a side stream
    (GENPOSE2_ODE_ZC=0). Returns the index n of the attempt whose successor's control ended the solve."""
    launch(0, 3)
    n = 0
    while True:
        launch(n + 1, 1)                       # decides attempt n, prepares attempt n+1
        ev = torch.cuda.Event()
        ev.record(stream)
        timing = STAGE_EVENTS is not None
        if timing:
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record(stream)
        launch(n + 1, 2)                       # attempt n+1 (no-op if attempt n ended the solve)
        if timing:
            s1.record(stream)
        off = ((n + 2) & 1) * rec + _STATUS_OFF
        side.wait_event(ev)
        with torch.cuda.stream(side):
            stat.copy_(ws[off:off + 4].view(torch.int32), non_blocking=True)
        side.synchronize()
        if int(stat[0]) != 0:
            return n
        if timing:
            STAGE_EVENTS.append((s0, s1, be.R))
        n += 1
        if n > max_attempts:
            raise RuntimeError("RK45: attempt limit reached")


_HSTAT_FREE = {}            # device -> free (pinned words, device address) pairs
_HSTAT_LOCK = threading.Lock()
_HIP = None


def _host_status_words(dev):
    """Lease 4 pinned int32 words the device can write, with their device-side address (hipHostGetDevicePointer
    checks that the pinned allocation is mapped for the device), or (None, None) if it cannot (the caller then
    keeps the evented loop). One lease per solve: concurrent solves on one device never share the words. Return
    it with _release_status_words."""
    global _HIP
    with _HSTAT_LOCK:
        free = _HSTAT_FREE.setdefault(dev, [])
        if free:
            return free.pop()
    h = torch.full((4,), -1, dtype=torch.int32).pin_memory()
    dp = ctypes.c_void_p()
    try:
        if _HIP is None:
            _HIP = ctypes.CDLL("libamdhip64.so")
        rc = _HIP.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(h.data_ptr()), 0)
    except OSError:
        rc = -1
    return (h, dp.value) if rc == 0 and dp.value else (None, None)


_CTL_FREE = {}              # device -> free pinned staging buffers of one controller record


def _ctl_staging(dev, nbytes: int) -> torch.Tensor:
    """A pinned host buffer for the initial controller record (its copy to the device is then asynchronous), leased
    per solve like the status words; return it with _release_ctl_staging once the stream has drained."""
    with _HSTAT_LOCK:
        free = _CTL_FREE.setdefault(dev, [])
        if free:
            return free.pop()
    return torch.empty(nbytes, dtype=torch.uint8).pin_memory()


def _release_ctl_staging(dev, buf: torch.Tensor) -> None:
    with _HSTAT_LOCK:
        _CTL_FREE.setdefault(dev, []).append(buf)


def _release_status_words(dev, lease) -> None:
    if lease[0] is not None:
        with _HSTAT_LOCK:
            _HSTAT_FREE.setdefault(dev, []).append(lease)


def _attempts_polled(call, be, stream, lease, max_attempts: int, timeout_s: float = 60.0) -> int:
    """The attempt loop with nothing between a control launch and its stage launch: the control kernel of
    attempt n writes 4 n + (status + 1) into word n & 3 of a host-mapped pinned buffer (gp_ode_auto_attempt_hs),
    and the host, one attempt ahead, polls that word. Same launches, same order, same bits as the evented loop."""
    h, hdev = lease
    hv = h.numpy()
    hv[:] = -1
    hp = ctypes.c_void_p(hdev)

    def launch(n, what):
        call(n, what, hp)

    timing = STAGE_EVENTS is not None

    def attempt(n):
        if not timing:
            launch(n, 3)
            return None
        launch(n, 1)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        launch(n, 2)
        s1.record(stream)
        return s0, s1

    attempt(0)
    n = 0
    while True:
        evs = attempt(n + 1)                   # control n+1 decides attempt n and prepares n+1; then attempt n+1
        want = n + 1
        t_end = time.monotonic() + timeout_s
        while (int(hv[want & 3]) >> 2) != want:
            if time.monotonic() > t_end:
                raise RuntimeError(f"RK45: no status from the control kernel of attempt {want} in {timeout_s} s")
        status = (int(hv[want & 3]) & 3) - 1
        if status != 0:
            return n
        if evs is not None:
            STAGE_EVENTS.append((evs[0], evs[1], be.R))
        n += 1
        if n > max_attempts:
            raise RuntimeError("RK45: attempt limit reached")


def rk45_device(be: DeviceRk45, t0: float, t_bound: float, t_eval: Optional[np.ndarray] = None,
                max_attempts: int = 100000):
    """solve_ivp(..., method="RK45", t_eval) with the step controller on the device.

    select_initial_step runs host-side exactly as in rk45_drive; every attempted step is then
    gp_ode_auto_attempt: the control kernel of attempt n decides attempt n-1 and prepares attempt
    n, the stage kernels follow. The host keeps one attempt enqueued ahead and reads only the
    status word of the newest controller record, so the device never waits for the host.
    Returns (x (R*9) fp64 -- the value ``res.y[:, -1]`` that cond_ode_sampler continues from --,
    nfev, status)."""
    lib = be.lib
    if ctypes.sizeof(OdeCtl) != int(lib.gp_ode_ctl_size()):
        raise RuntimeError("OdeCtl layout does not match libgenpose_hip.so")
    t0, tf = map(float, (t0, t_bound))
    direction = np.sign(tf - t0) if tf != t0 else 1
    if t_eval is not None:
        t_eval = np.asarray(t_eval, dtype=np.float64)
        if np.any(t_eval < min(t0, tf)) or np.any(t_eval > max(t0, tf)):
            raise ValueError("Values in `t_eval` are not within `t_span`.")
    # everything that does not depend on the initial step is set up before select_initial_step's two norm reads, so
    # the host has only h_abs and the controller record to form between the second read and the first attempt
    dev = be.dev
    gb = be.gb if isinstance(be, GlobalDeviceRk45) else None
    ex = None
    nbytes = int(lib.gp_ode_auto_workspace_size(be.R))
    if gb is not None:
        from .shard import PartialsExchange
        rows_total, rows_max = gb.total * be.k, gb.per_max * be.k
        part_n = int(lib.gp_ode_global_partials(rows_total, rows_max, gb.world, int(be.h.w.pe2_h is not None)))
        nbytes = max(nbytes, int(lib.gp_ode_global_workspace_size(part_n)))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if gb is not None:
        # every shard's partials, zero where a short last shard has no workgroup (their sum's fixed order is the
        # single call's)
        off = int(lib.gp_ode_auto_partials_offset())
        part = ws[off:off + 8 * part_n].view(torch.float64)
        part.zero_()
        ex = PartialsExchange(part, part_n, gb)
    rec = ctypes.sizeof(OdeCtl)
    ybuf = [be.y, torch.empty_like(be.y)]
    kbuf = list(be.K)
    karr = _ptr_array(kbuf)
    stream = torch.cuda.current_stream(dev)
    side, stat = _side_resources(dev)
    args = (float(tf), float(direction), be.rtol, be.atol, arch.SIGMA_MIN, arch.SIGMA_MAX / arch.SIGMA_MIN,
            float(sde._DIFF_SCALE_T), ctypes.c_void_p(ybuf[0].data_ptr()), ctypes.c_void_p(ybuf[1].data_ptr()), karr,
            _A6.ctypes.data_as(ctypes.c_void_p), _B6.ctypes.data_as(ctypes.c_void_p),
            _E7.ctypes.data_as(ctypes.c_void_p), be.R, be.k, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
            ctypes.c_void_p(stream.cuda_stream))

    w, pobj = ctypes.byref(be.h.w), ctypes.c_void_p(be.pobj.data_ptr())

    def call(n, what, hp):
        if ex is not None:
            rc = lib.gp_ode_auto_attempt_global(w, pobj, n, what, *args[:15], rows_total, gb.lo * be.k, gb.rank,
                                                gb.world, rows_max, ex.fn, None, *args[15:17], hp, args[17])
            if ex.error is not None:
                raise RuntimeError("ode_auto_attempt_global: partials exchange failed") from ex.error
            check(rc, "ode_auto_attempt_global")
        elif hp is not None:
            check(lib.gp_ode_auto_attempt_hs(w, pobj, n, what, *args[:-1], hp, args[-1]), "ode_auto_attempt")
        else:
            check(lib.gp_ode_auto_attempt(w, pobj, n, what, *args), "ode_auto_attempt")

    def launch(n, what):
        call(n, what, None)

    lease = _host_status_words(dev) if os.environ.get("GENPOSE2_ODE_ZC", "1")[:1] != "0" else (None, None)
    stage = _ctl_staging(dev, rec)
    try:
        h_abs, nfev = initial_step(be, t0, tf, direction)
        c0 = OdeCtl(t=t0, h_abs=float(h_abs), nfev=nfev)
        c0.kidx[:] = list(range(N_STAGES + 1))
        ctypes.memmove(stage.data_ptr(), ctypes.addressof(c0), rec)
        ws[:rec].copy_(stage, non_blocking=True)   # pinned: enqueued, no host wait
        if lease[0] is not None:
            n = _attempts_polled(call, be, stream, lease, max_attempts)
        else:
            n = _attempts_evented(launch, ws, rec, stream, side, stat, be, max_attempts)
    finally:
        # the device may still write the words (the speculative next control) until the stream drains, and the
        # controller record's copy may still read the staging buffer
        stream.synchronize()
        _release_status_words(dev, lease)
        _release_ctl_staging(dev, stage)
    last = ((n + 2) & 1) * rec

    ctl = OdeCtl.from_buffer_copy(bytes(ws[last:last + rec].cpu().numpy()))
    if ctl.status < 0:
        warnings.warn("RK45: required step size is less than spacing between numbers.")
    x = ybuf[ctl.yi]
    if t_eval is not None and ctl.status > 0:
        # res.y[:, -1] is the dense output of the final step at t_eval's last point (= t_bound)
        step_k = [kbuf[ctl.kidx[j]] for j in range(N_STAGES + 1)]
        step_k[0], step_k[N_STAGES] = step_k[N_STAGES], step_k[0]     # undo the FSAL swap
        tev = torch.tensor([t_eval[-1]], dtype=torch.float64, device=dev)
        out = torch.empty((1, be.n), dtype=torch.float64, device=dev)
        check(lib.gp_ode_dense(_ptr_array(step_k), _P74.ctypes.data_as(ctypes.c_void_p),
                               ctypes.c_void_p(ybuf[ctl.yi ^ 1].data_ptr()), ctypes.c_void_p(tev.data_ptr()), 0, 1, 0,
                               0, float(ctl.t_old), float(ctl.t - ctl.t_old), be.n, ctypes.c_void_p(out.data_ptr()),
                               ctypes.c_void_p(stream.cuda_stream)), "ode_dense")
        x = out[0]
    return x, int(ctl.nfev), int(ctl.status)
