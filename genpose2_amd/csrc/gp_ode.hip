// Probability-flow ODE sampler on device: Dormand-Prince 5(4) stages fused with the score heads.
//
// Reference: cond_ode_sampler (networks/gf_algorithms/samplers.py:180-258) hands the float64 state
// to scipy solve_ivp(method="RK45") and pays a device->host and host->device copy per right-hand
// side. Here an RK45 stage is a fused kernel body: the stage combination y + (sum_j a_j K_j) * h (fp64,
// scipy rk.py rk_step order) is formed in the prologue, cast to the fp32 pose the score model sees
// (samplers.py:210), the head trunk evaluates the score, and the epilogue writes
// K_s = -(0.5 g(t)^2) * score in fp64 (samplers.py:216). The last stage of an attempted step also
// writes y_new and the per-workgroup sum of (err / scale)^2 of scipy's error estimator
// (_estimate_error_norm, rk.py); ode_norm_kernel reduces it in a fixed order. The step
// controller's scalars stay on the host (genpose2_amd/ode.py): one 8-byte read per attempt. The
// device-controlled attempts (gp_ode_auto_attempt) run all six stages of an attempt in one launch
// (ode_attempt_kernel); the host-controlled ones launch each stage (ode_stage_kernel).
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "gp_head.h"

#define ODE_NK 7   // Dormand-Prince stages incl. the FSAL derivative

// Device-resident RK45 controller state (the device-controlled path, gp_ode_auto_*). One copy per
// attempt parity: the control kernel of attempt n reads ctl[n & 1] and writes ctl[(n + 1) & 1], the
// stage kernels of attempt n read ctl[(n + 1) & 1]. Field order fixed (doubles, floats, ints) so the
// host mirror (genpose2_amd/ode.py OdeCtl) has the same layout.
struct OdeCtl {
    double t, h_abs;              // solver time; step size carried to the next step (scipy self.h_abs)
    double t_old, h_last;         // last accepted step (dense output)
    double h, t_new, h_abs_loc;   // the prepared attempt (scipy _step_impl locals h, t_new, h_abs)
    double coef[6];               // -(0.5 g(t_s)^2) of the attempt's 6 stage times
    float t32[6], sig[6];         // float32(t_s), sigma(t32)
    int status;                   // 0 running, 1 finished, -1 step size below spacing (scipy failure)
    int active;                   // the prepared attempt runs
    int rejected;                 // scipy step_rejected within the current step
    int nfev, n_acc, yi;          // RHS evaluations, accepted steps, y buffer holding the state
    int kidx[ODE_NK];             // K slot permutation (FSAL swaps slots 0 and 6 on acceptance)
};
static_assert(sizeof(OdeCtl) == 208, "OdeCtl layout is mirrored on the host");

struct OdeStageArgs {
    gp_head_weights w;
    const float* pobj;
    const float* tproj;          // (768) time row of this stage's t (host-controlled calls)
    float sigma;                 // sigma(t32), fp32 (score = f / (sigma + 1e-7))
    double coef;                 // -(0.5 * g(t)^2)
    const double* y;             // (R,9) state at the step's start
    const double* k[ODE_NK];     // stage derivatives combined into this stage's input
    double a[ODE_NK];            // y_in = y + (sum_{j<nk} a_j K_j) * h
    int nk;
    double h;
    double* kout;                // (R,9) this stage's derivative
    // final stage of an attempt (MODE 1): y_new out and the error-estimator partials
    double* ynew;
    double e[ODE_NK];            // error weights over K_0..K_6 (K_6 = this stage)
    double rtol, atol;
    double* part;                // (nwg) sum over the workgroup's elements of (err/scale)^2
    int part_off;                // index of this launch's first partial (global-batch shards: the single call's
                                 // workgroup index of this shard's first row tile; 0 otherwise)
    int rows, kper;
    // device-controlled attempts: state, time rows and buffers resolved from ctl
    const OdeCtl* ctl;           // null for host-controlled calls
    const float* tproj6;         // (6,768) rows of the prepared attempt
    double* ybuf[2];
    double* kbuf[ODE_NK];
    int stage;                   // 1..6
};

// One RK45 stage for the workgroup's rows. MODE 0: stage derivative. MODE 1: last stage of an attempt
// (y_new, K_6, error partials). y_in = y + (sum_{j<nk} acoef_j K_j) h, K_out = coef * score(f32(y_in), t).
template <int MODE, int PL, int NT>
__device__ __forceinline__ void ode_stage_body(const OdeStageArgs& a, const double* y, const double* const* kin,
                                               const double* acoef, int nk, double h, double coef, float sigma,
                                               const float* tproj, double* kout, double* ynew,
                                               HeadSmem<NT, EVAL_WV, PL>& sm, int* obj, double* y0s, double* y1s,
                                               double* esq, const SplitScalars& hs) {
    constexpr int ROWS = 16 * NT;
    constexpr int NTH = EVAL_WV * 64;
    constexpr bool SPLIT = PL != 0;
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * ROWS;
    stage_small_weights<NT, EVAL_WV, 0, !SPLIT>(a.w, sm);
    for (int i = tid; i < ROWS * 16; i += NTH) {
        const int c = i >> 4, j = i & 15;
        const int r = r0 + c;
        float xv = 0.f;
        if (r < a.rows && j < 9) {
#pragma clang fp contract(off)
            const size_t e = (size_t)r * 9 + j;
            const double yv = y[e];
            double yi = yv;
            if (nk > 0) {
                double acc = kin[0][e] * acoef[0];
                for (int s = 1; s < nk; ++s) acc = acc + kin[s][e] * acoef[s];
                yi = yv + acc * h;
            }
            xv = (float)yi;   // torch.tensor(x, dtype=torch.float32) (samplers.py:210)
            if (MODE == 1) {
                y0s[c * 9 + j] = yv;
                y1s[c * 9 + j] = yi;
                ynew[e] = yi;
            }
        }
        sm.xin[i] = xv;
    }
    if (tid < ROWS) {
        const int r = r0 + tid;
        obj[tid] = (r < a.rows ? r : a.rows - 1) / a.kper;
    }
    if constexpr (SPLIT)
        head_trunk_x3<NT, EVAL_WV>(a.w, a.pobj, tproj, obj, sm, 0, hs);
    else
        head_trunk<NT, EVAL_WV>(a.w, a.pobj, tproj, obj, sm);
    double sq = 0.0;   // this thread's (err/scale)^2 terms, its elements in increasing order
    for (int e9 = tid; e9 < ROWS * 9; e9 += NTH) {
#pragma clang fp contract(off)
        const int c = e9 / 9, o = e9 - c * 9;
        const int r = r0 + c;
        if (r < a.rows) {
            const size_t e = (size_t)r * 9 + o;
            const float s = fdiv(head_out(sm, c, o), fadd(sigma, 1e-7f));
            const double kv = coef * (double)s;
            kout[e] = kv;
            if (MODE == 1) {
                // scipy: err = (K^T E) * h / scale, scale = atol + max(|y|, |y_new|) * rtol
                double acc = kin[0][e] * a.e[0];
                for (int s2 = 1; s2 < ODE_NK - 1; ++s2) acc = acc + kin[s2][e] * a.e[s2];
                acc = acc + kv * a.e[ODE_NK - 1];
                const double y0 = y0s[c * 9 + o], y1 = y1s[c * 9 + o];
                const double sc = a.atol + fmax(fabs(y0), fabs(y1)) * a.rtol;
                const double er = (acc * h) / sc;
                sq += er * er;
            }
        }
    }
    if (MODE == 1) {
        // workgroup partial in a fixed order: per-thread sums, xor tree per wave, waves in order
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off, 64);
        if ((tid & 63) == 0) esq[tid >> 6] = sq;
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
            for (int v = 0; v < EVAL_WV; ++v) t += esq[v];
            a.part[a.part_off + blockIdx.x] = t;
        }
    }
}

// MODE 0: stage derivative. MODE 1: last stage of an attempt (y_new, K_6, error partials).
// NT column tiles of 16 candidates per workgroup (head_pick_nt: 32 / 64 candidates from 4097 / 8193 rows
// with the split-f16 trunk, as the PC step).
template <int MODE, int PL, int NT>   // PL 0: exact fp32 GEMMs, X3P: f16x3
__global__ __launch_bounds__(EVAL_WV * 64) void ode_stage_kernel(OdeStageArgs a) {
    constexpr int ROWS = 16 * NT;
    constexpr int NTH = EVAL_WV * 64;
    __shared__ HeadSmem<NT, EVAL_WV, PL> sm;
    constexpr bool SPLIT = PL != 0;
    __shared__ int obj[ROWS];
    __shared__ double y0s[ROWS * 9], y1s[ROWS * 9], esq[NTH];
    SplitScalars hs = {};
    if constexpr (SPLIT) hs = load_split_scalars(a.w);
    const double* y = a.y;
    const double* kin[ODE_NK];
#pragma unroll
    for (int j = 0; j < ODE_NK; ++j) kin[j] = a.k[j];
    double h = a.h, coef = a.coef;
    float sigma = a.sigma;
    const float* tproj = a.tproj;
    double* kout = a.kout;
    double* ynew = a.ynew;
    if (a.ctl != nullptr) {   // device-controlled: skip when no attempt was prepared
        const OdeCtl* c = a.ctl;
        if (!c->active) return;
        y = a.ybuf[c->yi];
#pragma unroll
        for (int j = 0; j < ODE_NK; ++j) kin[j] = a.kbuf[c->kidx[j]];
        h = c->h;
        coef = c->coef[a.stage - 1];
        sigma = c->sig[a.stage - 1];
        tproj = a.tproj6 + (size_t)(a.stage - 1) * 768;
        kout = a.kbuf[c->kidx[a.stage]];
        ynew = a.ybuf[c->yi ^ 1];
    }
    ode_stage_body<MODE, PL, NT>(a, y, kin, a.a, a.nk, h, coef, sigma, tproj, kout, ynew, sm, obj, y0s, y1s, esq, hs);
}

// A whole device-controlled attempt in one launch: the six stages run back to back in every workgroup
// (a stage needs only its own rows' earlier stages, so no grid-wide step separates them -- only the
// controller's accept / reject between attempts does). Stage s combines K_0..K_{s-1} with tableau row
// A[s] (stage 6: B, y_new and the error partials), exactly as the six stage launches do: bit-identical,
// without five kernel boundaries (each ~3 us of tail, boundary and refill at config 4). The K_s a stage
// writes are read back by other threads of the workgroup after the stage's barrier (the workgroup-scope
// release / acquire of __syncthreads orders the global stores before those loads).
struct OdeTableau {
    double A[36], B[6];
};
template <int PL, int NT>
__global__ __launch_bounds__(EVAL_WV * 64) void ode_attempt_kernel(OdeStageArgs a, OdeTableau tb) {
    constexpr int ROWS = 16 * NT;
    constexpr int NTH = EVAL_WV * 64;
    __shared__ HeadSmem<NT, EVAL_WV, PL> sm;
    constexpr bool SPLIT = PL != 0;
    __shared__ int obj[ROWS];
    __shared__ double y0s[ROWS * 9], y1s[ROWS * 9], esq[NTH];
    // the tableau and the K slots of this attempt in LDS: read per use (wave-uniform), not held in registers
    // across the six stages
    __shared__ double tab[42];
    __shared__ const double* kin[ODE_NK];
    const OdeCtl* c = a.ctl;
    if (!c->active) return;
    const int tid = threadIdx.x;
    if (tid < 36) tab[tid] = tb.A[tid];
    else if (tid < 42) tab[tid] = tb.B[tid - 36];
    else if (tid < 42 + ODE_NK) kin[tid - 42] = a.kbuf[c->kidx[tid - 42]];
    const double* y = a.ybuf[c->yi];
    const double h = c->h;
    __syncthreads();
    for (int s = 1; s < 6; ++s) {
        if (s > 1) __syncthreads();   // stage s-1's K stores and its reads of the staged weights are done
        // per stage (L2-resident): held across the stages they would add to the trunk's register peak
        SplitScalars hs = {};
        if constexpr (SPLIT) hs = load_split_scalars(a.w);
        ode_stage_body<0, PL, NT>(a, y, kin, tab + s * 6, s, h, c->coef[s - 1], c->sig[s - 1],
                                  a.tproj6 + (size_t)(s - 1) * 768, const_cast<double*>(kin[s]), nullptr, sm, obj,
                                  y0s, y1s, esq, hs);
    }
    __syncthreads();
    SplitScalars hs = {};
    if constexpr (SPLIT) hs = load_split_scalars(a.w);
    ode_stage_body<1, PL, NT>(a, y, kin, tab + 36, 6, h, c->coef[5], c->sig[5], a.tproj6 + (size_t)5 * 768,
                              const_cast<double*>(kin[6]), a.ybuf[c->yi ^ 1], sm, obj, y0s, y1s, esq, hs);
}

// Stage-kernel launch of `nt` column tiles per workgroup (1 for the exact-fp32 trunk).
template <int MODE>
static void ode_launch_stage(const OdeStageArgs& a, int nt, hipStream_t st) {
    const int nwg = (a.rows + 16 * nt - 1) / (16 * nt);
    const dim3 grid(nwg), blk(EVAL_WV * 64);
    if (!a.w.pe2_h)
        hipLaunchKernelGGL((ode_stage_kernel<MODE, 0, 1>), grid, blk, 0, st, a);
    else if (nt == 4)
        hipLaunchKernelGGL((ode_stage_kernel<MODE, X3P, 4>), grid, blk, 0, st, a);
    else if (nt == 2)
        hipLaunchKernelGGL((ode_stage_kernel<MODE, X3P, 2>), grid, blk, 0, st, a);
    else
        hipLaunchKernelGGL((ode_stage_kernel<MODE, X3P, 1>), grid, blk, 0, st, a);
}

static int ode_nt(const gp_head_weights* w, int rows) { return head_pick_nt(rows, w->pe2_h != nullptr); }
static int ode_nwg(const gp_head_weights* w, int rows) {
    const int nt = ode_nt(w, rows);
    return (rows + 16 * nt - 1) / (16 * nt);
}

// Sum of part[0..n) by a 256-thread workgroup in a fixed order (strided per-thread sums, xor
// shuffles within each wave, the four wave sums in wave order): every caller that reduces the same
// partials gets the same bits. `red` is 4 doubles of LDS.
__device__ __forceinline__ double block_sum_f64(const double* __restrict__ part, int n, double* red) {
    double t = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) t += part[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

// out[0] = sqrt(sum(part[0..n))) / sqrt(count): scipy's RMS norm over the error partials.
__global__ __launch_bounds__(256) void ode_norm_kernel(const double* __restrict__ part, int n, double count,
                                                       double* __restrict__ out) {
    __shared__ double red[4];
    const double t = block_sum_f64(part, n, red);
    if (threadIdx.x == 0) out[0] = sqrt(t) / sqrt(count);
}

// select_initial_step norms (scipy _ivp/common.py): scale = atol + |y0| rtol;
// f1 == NULL: out[0] = rms(y0 / scale), out[1] = rms(f0 / scale); else out[2] = rms((f1 - f0) / scale).
__global__ __launch_bounds__(1024) void ode_init_norms_kernel(const double* __restrict__ y0,
                                                              const double* __restrict__ f0,
                                                              const double* __restrict__ f1, long long n,
                                                              double atol, double rtol, double* __restrict__ out) {
#pragma clang fp contract(off)
    __shared__ double r0[16], r1[16];
    double s0 = 0.0, s1 = 0.0;
    // each thread's elements i = tid + 1024 j in increasing j, as one load per step would add them; the loads of
    // IL consecutive steps are issued together (a load per dependent add waited a full memory round trip each:
    // 76 -> 42 us per call at R = 12,800; the rest is the fp64 divisions of one workgroup)
    constexpr int IL = 8;
    long long i0 = threadIdx.x;
    for (; i0 + 1024LL * (IL - 1) < n; i0 += 1024LL * IL) {
        double yv[IL], fa[IL], fb[IL];
#pragma unroll
        for (int j = 0; j < IL; ++j) {
            yv[j] = y0[i0 + 1024LL * j];
            fa[j] = f0[i0 + 1024LL * j];
        }
        if (f1 != nullptr) {
#pragma unroll
            for (int j = 0; j < IL; ++j) fb[j] = f1[i0 + 1024LL * j];
        } else {
#pragma unroll
            for (int j = 0; j < IL; ++j) fb[j] = 0.0;
        }
#pragma unroll
        for (int j = 0; j < IL; ++j) {
            const double sc = atol + fabs(yv[j]) * rtol;
            if (f1 == nullptr) {
                const double u = yv[j] / sc, v = fa[j] / sc;
                s0 += u * u;
                s1 += v * v;
            } else {
                const double v = (fb[j] - fa[j]) / sc;
                s0 += v * v;
            }
        }
    }
    for (long long i = i0; i < n; i += 1024) {
        const double sc = atol + fabs(y0[i]) * rtol;
        if (f1 == nullptr) {
            const double u = y0[i] / sc, v = f0[i] / sc;
            s0 += u * u;
            s1 += v * v;
        } else {
            const double v = (f1[i] - f0[i]) / sc;
            s0 += v * v;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        s0 += __shfl_xor(s0, off, 64);
        s1 += __shfl_xor(s1, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        r0[threadIdx.x >> 6] = s0;
        r1[threadIdx.x >> 6] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 16; ++i) {
            r0[0] += r0[i];
            r1[0] += r1[i];
        }
    }
    if (threadIdx.x == 0) {
        const double rn = sqrt((double)n);
        if (f1 == nullptr) {
            out[0] = sqrt(r0[0]) / rn;
            out[1] = sqrt(r1[0]) / rn;
        } else {
            out[2] = sqrt(r0[0]) / rn;
        }
    }
}

// Dense output of an accepted step (scipy RkDenseOutput, rk.py): for each requested t_eval point
// te = tev[i], x = (te - t_old) / h, p = cumprod([x, x, x, x]), y = h * (Q p) + y_old with
// Q = K^T P. Writes out[(i - i_base) * n + e] for i in [i0, i1).
struct OdeDenseArgs {
    const double* k[ODE_NK];
    double P[ODE_NK][4];
    const double* y_old;
    const double* tev;
    int i0, i1, i_base;
    double t_old, h;
    double* out;
    long long n;
    int reverse;   // out row = (i_base - i) instead of (i - i_base)
};

__global__ __launch_bounds__(256) void ode_dense_kernel(OdeDenseArgs a) {
#pragma clang fp contract(off)
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= a.n) return;
    double Q[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        double acc = a.k[0][e] * a.P[0][m];
        for (int j = 1; j < ODE_NK; ++j) acc = acc + a.k[j][e] * a.P[j][m];
        Q[m] = acc;
    }
    const double yo = a.y_old[e];
    for (int i = a.i0; i < a.i1; ++i) {
        const double x = (a.tev[i] - a.t_old) / a.h;
        const double p1 = x, p2 = p1 * x, p3 = p2 * x, p4 = p3 * x;
        const double d = ((Q[0] * p1 + Q[1] * p2) + Q[2] * p3) + Q[3] * p4;
        const long long row = a.reverse ? (long long)(a.i_base - i) : (long long)(i - a.i_base);
        a.out[row * a.n + e] = a.h * d + yo;
    }
}

// Final denoise (samplers.py:240-249) + epilogue: grad = score(float(x), eps) in fp32,
// mean_x = x + (0 - g^2 grad) * c (fp32 product, fp64 sum), then GS of [:6], + pts_center, quaternion
// (posenet_agent.py:554-556). Writes pose (R,9) fp64 and q (R,7) fp64. The score runs on the stage kernels'
// trunk and tile (f16x3, 64 candidates per workgroup at R >= 8193; exact fp32 without the f16 planes).
struct OdeDenoiseArgs {
    gp_head_weights w;
    const float* pobj;
    const float* tproj;
    float sigma;
    float g2;        // diffusion(eps)^2 in fp32
    float step;      // (1 - eps) / num_steps as fp32
    const double* x;
    const float* center;
    double* pose;
    double* q;
    int rows, kper;
};

template <int PL, int NT>   // PL 0: exact fp32 trunk, X3P: f16x3 (the stage kernels' arithmetic)
__global__ __launch_bounds__(EVAL_WV * 64) void ode_denoise_kernel(OdeDenoiseArgs a) {
    constexpr int ROWS = 16 * NT;
    constexpr int NTH = EVAL_WV * 64;
    __shared__ HeadSmem<NT, EVAL_WV, PL> sm;
    __shared__ int obj[ROWS];
    __shared__ double xm[ROWS * 9];
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * ROWS;
    SplitScalars hs = {};
    if constexpr (PL != 0) hs = load_split_scalars(a.w);
    stage_small_weights<NT, EVAL_WV, 0, PL == 0>(a.w, sm);
    for (int i = tid; i < ROWS * 16; i += NTH) {
        const int c = i >> 4, j = i & 15;
        const int r = r0 + c;
        sm.xin[i] = (r < a.rows && j < 9) ? (float)a.x[(size_t)r * 9 + j] : 0.f;
    }
    if (tid < ROWS) {
        const int r = r0 + tid;
        obj[tid] = (r < a.rows ? r : a.rows - 1) / a.kper;
    }
    if constexpr (PL != 0)
        head_trunk_x3<NT, EVAL_WV>(a.w, a.pobj, a.tproj, obj, sm, 0, hs);
    else
        head_trunk<NT, EVAL_WV>(a.w, a.pobj, a.tproj, obj, sm);
    for (int e9 = tid; e9 < ROWS * 9; e9 += NTH) {
#pragma clang fp contract(off)
        const int c = e9 / 9, o = e9 - c * 9;
        const int r = r0 + c;
        if (r < a.rows) {
            const float grad = fdiv(head_out(sm, c, o), fadd(a.sigma, 1e-7f));
            const float drift = 0.0f - a.g2 * grad;
            xm[e9] = a.x[(size_t)r * 9 + o] + (double)(drift * a.step);
        }
    }
    __syncthreads();
    if (tid < ROWS && r0 + tid < a.rows) {
        const int r = r0 + tid;
        double v[9], qq[4];
#pragma unroll
        for (int j = 0; j < 9; ++j) v[j] = xm[tid * 9 + j];
        gram_schmidt6<double>(v);
        const float* cen = a.center + (size_t)obj[tid] * 3;
        v[6] += (double)ld1(cen);
        v[7] += (double)ld1(cen + 1);
        v[8] += (double)ld1(cen + 2);
        quat_from_gs<double>(v, qq);
#pragma unroll
        for (int j = 0; j < 9; ++j) a.pose[(size_t)r * 9 + j] = v[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) a.q[(size_t)r * 7 + j] = qq[j];
#pragma unroll
        for (int j = 0; j < 3; ++j) a.q[(size_t)r * 7 + 4 + j] = v[6 + j];
    }
}

// Time rows of up to 6 stage times passed by value (no host->device copy per attempt); each row is
// split over ODE_ROW_CHUNKS workgroups.
#define ODE_ROW_CHUNKS 8
struct OdeTimes {
    float t[6];
};
__global__ __launch_bounds__(HT) void ode_time_rows_kernel(gp_head_weights w, OdeTimes tv, float* __restrict__ out) {
    __shared__ float emb[128];
    __shared__ float tf[128];
    constexpr int PER = 768 / ODE_ROW_CHUNKS;
    time_row(w, tv.t[blockIdx.x], emb, tf, out + (size_t)blockIdx.x * 768, blockIdx.y * PER, blockIdx.y * PER + PER);
}

// ------------------------------------------------------------------------------ C ABI
// Workspace: 6 time rows (6 x 768 fp32) | per-workgroup error partials (fp64).
static size_t ode_part_offset() { return 6 * 768 * sizeof(float); }

extern "C" size_t gp_ode_workspace_size(int rows) {
    return ode_part_offset() + sizeof(double) * (((size_t)rows + 15) / 16) + 256;
}

static int ode_launch_times(const gp_head_weights* w, const float* t32, int nt, void* ws, hipStream_t stream) {
    OdeTimes tv = {};
    for (int i = 0; i < nt; ++i) tv.t[i] = t32[i];
    hipLaunchKernelGGL(ode_time_rows_kernel, dim3(nt, ODE_ROW_CHUNKS), dim3(HT), 0, stream, *w, tv,
                       static_cast<float*>(ws));
    return gp_check_launch("ode_time_rows_kernel");
}

extern "C" int gp_ode_rhs(const gp_head_weights* w, const float* pobj, float t32, float sigma, double coef,
                          const double* y, const double* const* kin, const double* acoef, int nk, double h, int rows,
                          int k, double* kout, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    GP_REQUIRE(w && pobj && y && kout && workspace && rows >= 1 && k >= 1, "ode_rhs: bad arguments");
    GP_REQUIRE(nk >= 0 && nk < ODE_NK && (nk == 0 || (kin && acoef)), "ode_rhs: nk must be in [0, 6]");
    GP_REQUIRE(workspace_bytes >= gp_ode_workspace_size(rows), "ode_rhs: workspace too small");
    OdeStageArgs a = {};
    a.w = *w;
    a.pobj = pobj;
    a.tproj = static_cast<const float*>(workspace);
    a.sigma = sigma;
    a.coef = coef;
    a.y = y;
    for (int j = 0; j < nk; ++j) {
        GP_REQUIRE(kin[j] != nullptr, "ode_rhs: null stage pointer");
        a.k[j] = kin[j];
        a.a[j] = acoef[j];
    }
    a.nk = nk;
    a.h = h;
    a.kout = kout;
    a.rows = rows;
    a.kper = k;
    int rc = ode_launch_times(w, &t32, 1, workspace, stream);
    if (rc) return rc;
    ode_launch_stage<0>(a, ode_nt(w, rows), stream);
    return gp_check_launch("ode_stage_kernel");
}

extern "C" int gp_ode_attempt(const gp_head_weights* w, const float* pobj, const float* t32_6, const float* sigma_6,
                              const double* coef_6, const double* y, double* const* kslots, const double* tableau_a,
                              const double* b, const double* e, double h, double rtol, double atol, int rows, int k,
                              double* ynew, double* err_out, void* workspace, size_t workspace_bytes,
                              hipStream_t stream) {
    GP_REQUIRE(w && pobj && t32_6 && sigma_6 && coef_6 && y && kslots && tableau_a && b && e && ynew && err_out &&
                   workspace && rows >= 1 && k >= 1,
               "ode_attempt: bad arguments");
    GP_REQUIRE(workspace_bytes >= gp_ode_workspace_size(rows), "ode_attempt: workspace too small");
    for (int j = 0; j < ODE_NK; ++j) GP_REQUIRE(kslots[j] != nullptr, "ode_attempt: null K slot");
    const int nwg = ode_nwg(w, rows), nt = ode_nt(w, rows);
    const float* tproj = static_cast<const float*>(workspace);
    double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + ode_part_offset());
    int rc = ode_launch_times(w, t32_6, 6, workspace, stream);
    if (rc) return rc;
    OdeStageArgs a = {};
    a.w = *w;
    a.pobj = pobj;
    a.y = y;
    a.h = h;
    a.rows = rows;
    a.kper = k;
    a.rtol = rtol;
    a.atol = atol;
    for (int j = 0; j < ODE_NK; ++j) a.k[j] = kslots[j];
    // stages 1..5: K_s = f(t + c_s h, y + (sum_{j<s} A[s][j] K_j) h)   (tableau_a: 6x6 row-major)
    for (int s = 1; s < 6; ++s) {
        a.tproj = tproj + (size_t)(s - 1) * 768;
        a.sigma = sigma_6[s - 1];
        a.coef = coef_6[s - 1];
        a.nk = s;
        for (int j = 0; j < s; ++j) a.a[j] = tableau_a[s * 6 + j];
        a.kout = kslots[s];
        ode_launch_stage<0>(a, nt, stream);
    }
    // y_new = y + (sum_{j<6} B_j K_j) h ; K_6 = f(t + h, y_new) ; error partials
    a.tproj = tproj + (size_t)5 * 768;
    a.sigma = sigma_6[5];
    a.coef = coef_6[5];
    a.nk = 6;
    for (int j = 0; j < 6; ++j) a.a[j] = b[j];
    for (int j = 0; j < ODE_NK; ++j) a.e[j] = e[j];
    a.kout = kslots[6];
    a.ynew = ynew;
    a.part = part;
    ode_launch_stage<1>(a, nt, stream);
    hipLaunchKernelGGL(ode_norm_kernel, dim3(1), dim3(256), 0, stream, (const double*)part, nwg,
                       (double)rows * 9.0, err_out);
    return gp_check_launch("ode_stage_kernel<final>");
}

extern "C" int gp_ode_init_norms(const double* y0, const double* f0, const double* f1, long long n, double atol,
                                 double rtol, double* out, hipStream_t stream) {
    GP_REQUIRE(y0 && f0 && out && n >= 1, "ode_init_norms: bad arguments");
    hipLaunchKernelGGL(ode_init_norms_kernel, dim3(1), dim3(1024), 0, stream, y0, f0, f1, n, atol, rtol, out);
    return gp_check_launch("ode_init_norms_kernel");
}

extern "C" int gp_ode_dense(const double* const* kslots, const double* P7x4, const double* y_old,
                            const double* t_eval, int i0, int i1, int i_base, int reverse, double t_old, double h,
                            long long n, double* out, hipStream_t stream) {
    GP_REQUIRE(kslots && P7x4 && y_old && t_eval && out && n >= 1 && i1 >= i0, "ode_dense: bad arguments");
    if (i1 == i0) return GP_OK;
    OdeDenseArgs a = {};
    for (int j = 0; j < ODE_NK; ++j) {
        GP_REQUIRE(kslots[j] != nullptr, "ode_dense: null K slot");
        a.k[j] = kslots[j];
        for (int m = 0; m < 4; ++m) a.P[j][m] = P7x4[j * 4 + m];
    }
    a.y_old = y_old;
    a.tev = t_eval;
    a.i0 = i0;
    a.i1 = i1;
    a.i_base = i_base;
    a.reverse = reverse;
    a.t_old = t_old;
    a.h = h;
    a.out = out;
    a.n = n;
    hipLaunchKernelGGL(ode_dense_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
    return gp_check_launch("ode_dense_kernel");
}

extern "C" int gp_ode_denoise(const gp_head_weights* w, const float* pobj, float t32, float sigma, float g2,
                              float step, const double* x, int rows, int k, const float* pts_center, double* pose,
                              double* q, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    GP_REQUIRE(w && pobj && x && pts_center && pose && q && workspace && rows >= 1 && k >= 1,
               "ode_denoise: bad arguments");
    GP_REQUIRE(workspace_bytes >= gp_ode_workspace_size(rows), "ode_denoise: workspace too small");
    int rc = ode_launch_times(w, &t32, 1, workspace, stream);
    if (rc) return rc;
    OdeDenoiseArgs a = {};
    a.w = *w;
    a.pobj = pobj;
    a.tproj = static_cast<const float*>(workspace);
    a.sigma = sigma;
    a.g2 = g2;
    a.step = step;
    a.x = x;
    a.center = pts_center;
    a.pose = pose;
    a.q = q;
    a.rows = rows;
    a.kper = k;
    // the stage kernels' trunk and tile (exact fp32 without the f16 planes)
    const int nt = ode_nt(w, rows);
    const dim3 grid((rows + 16 * nt - 1) / (16 * nt)), blk(EVAL_WV * 64);
    if (!w->pe2_h)
        hipLaunchKernelGGL((ode_denoise_kernel<0, 1>), grid, blk, 0, stream, a);
    else if (nt == 4)
        hipLaunchKernelGGL((ode_denoise_kernel<X3P, 4>), grid, blk, 0, stream, a);
    else if (nt == 2)
        hipLaunchKernelGGL((ode_denoise_kernel<X3P, 2>), grid, blk, 0, stream, a);
    else
        hipLaunchKernelGGL((ode_denoise_kernel<X3P, 1>), grid, blk, 0, stream, a);
    return gp_check_launch("ode_denoise_kernel");
}

// ============================================================================ device-controlled RK45
// The host-controlled path above reads one error norm per attempt (a device->host round trip per
// attempt, ~30% of the sampler's wall time at config 2). Here the step controller itself runs on
// the device: ode_control_kernel of attempt n decides attempt n-1 (scipy _step_impl's
// accept/reject and step-size update from its error norm) and prepares attempt n (min_step check,
// h, t_new, the 6 stage times and their scalars, and their time rows), so the host only enqueues
// attempts one ahead and reads a status word. Stage scalars use device pow(); the host path uses
// glibc's through torch: the two can differ in the last bit (tests/test_gpu_parity.py compares
// the two paths).
struct OdeConsts {
    double t_bound, direction, rtol, atol;
    double sig_min, base, diff_scale;   // sigma(t) = sig_min * base^t; g = sigma(t) * diff_scale
    double count;                       // elements of the state (R*9) for the RMS norm
    int nwg;                            // error partials
};

#define ODE_CTL_CHUNKS 8   // workgroups per stage time row (768 / 8 outputs each)

// hstat (optional, host-mapped memory): word n & 3 receives 4 n + (status + 1) once attempt n is decided and prepared,
// so a host can follow the solve without an event and a copy between the control and the stage launches
__global__ __launch_bounds__(HT) void ode_control_kernel(gp_head_weights w, const OdeCtl* __restrict__ cin,
                                                         OdeCtl* __restrict__ cout, const double* __restrict__ part,
                                                         int decide, OdeConsts k, float* __restrict__ tproj6,
                                                         int* __restrict__ hstat, int n) {
#pragma clang fp contract(off)
    __shared__ double red[4];
    __shared__ OdeCtl s;
    __shared__ float emb[128], tf[128];
    const int tid = threadIdx.x;
    // error norm of attempt n-1 (the same fixed order in every workgroup)
    const double esum = decide ? block_sum_f64(part, k.nwg, red) : 0.0;
    if (tid == 0) {
        OdeCtl c = *cin;
        const double dir = k.direction;
        if (decide && c.active) {   // scipy RK45._step_impl, after rk_step / _estimate_error_norm
            const double err = sqrt(esum) / sqrt(k.count);
            c.nfev += 6;
            if (err < 1.0) {
                double factor = err == 0.0 ? 10.0 : fmin(10.0, 0.9 * pow(err, -0.2));
                if (c.rejected) factor = fmin(1.0, factor);
                c.h_abs = c.h_abs_loc * factor;
                c.t_old = c.t;
                c.h_last = c.h;
                c.t = c.t_new;
                c.yi ^= 1;
                const int k0 = c.kidx[0];
                c.kidx[0] = c.kidx[ODE_NK - 1];
                c.kidx[ODE_NK - 1] = k0;
                c.n_acc += 1;
                c.rejected = 0;
                if (dir * (c.t - k.t_bound) >= 0.0) c.status = 1;
            } else {
                c.h_abs_loc *= fmax(0.2, 0.9 * pow(err, -0.2));
                c.rejected = 1;
            }
        }
        c.active = 0;
        if (c.status == 0) {   // prepare the next attempt
            const double min_step = 10.0 * fabs(nextafter(c.t, dir * INFINITY) - c.t);
            double ha = c.rejected ? c.h_abs_loc : (c.h_abs < min_step ? min_step : c.h_abs);
            if (ha < min_step) {
                c.status = -1;
            } else {
                double h = ha * dir;
                double t_new = c.t + h;
                if (dir * (t_new - k.t_bound) > 0.0) t_new = k.t_bound;
                h = t_new - c.t;
                c.h = h;
                c.t_new = t_new;
                c.h_abs_loc = fabs(h);
                c.active = 1;
            }
        }
        s = c;
    }
    __syncthreads();
    if (!s.active) {
        if (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
            *cout = s;
            if (hstat != nullptr) {
                __threadfence_system();
                reinterpret_cast<volatile int*>(hstat)[n & 3] = 4 * n + s.status + 1;
            }
        }
        return;
    }
    // stage times t + c_s h (s = 1..5) and t + h, one thread each (rk.py rk_step)
    if (tid < 6) {
        const double cs[5] = {1.0 / 5.0, 3.0 / 10.0, 4.0 / 5.0, 8.0 / 9.0, 1.0};
        const double ts = tid < 5 ? s.t + cs[tid] * s.h : s.t + s.h;
        const float t32 = (float)ts;
        s.t32[tid] = t32;
        s.sig[tid] = fmul((float)k.sig_min, (float)pow(k.base, (double)t32));
        const double g = (k.sig_min * pow(k.base, ts)) * k.diff_scale;
        s.coef[tid] = -(0.5 * (g * g));
    }
    __syncthreads();
    if (tid == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
        *cout = s;
        if (hstat != nullptr) {
            __threadfence_system();
            reinterpret_cast<volatile int*>(hstat)[n & 3] = 4 * n + s.status + 1;
        }
    }
    // time row slice of stage blockIdx.x: outputs [chunk * 96, chunk * 96 + 96)
    constexpr int PER = 768 / ODE_CTL_CHUNKS;
    time_row(w, s.t32[blockIdx.x], emb, tf, tproj6 + (size_t)blockIdx.x * 768, blockIdx.y * PER, blockIdx.y * PER + PER);
}

// Device-controlled attempts as one fused launch (default) or six stage launches (GENPOSE2_ODE_FUSED=0: the
// same bits; for A/B and the equality test).
static bool ode_fused() {
    const char* v = getenv("GENPOSE2_ODE_FUSED");
    return v == nullptr || v[0] != '0';
}

// Workspace of the device-controlled path: ctl[2] | time rows (6 x 768 fp32) | error partials.
static size_t auto_tproj_off() { return 2 * sizeof(OdeCtl); }
static size_t auto_part_off() { return auto_tproj_off() + 6 * 768 * sizeof(float); }

extern "C" size_t gp_ode_ctl_size(void) { return sizeof(OdeCtl); }

extern "C" size_t gp_ode_auto_workspace_size(int rows) {
    return auto_part_off() + sizeof(double) * (((size_t)rows + 15) / 16) + 256;
}

// A global-batch shard of one RK45 solve on the whole batch: the tiling of the single call (nt from rows_total), this
// shard's partials at part_off of part_n, the error norm over every shard's partials and rows_total * 9 elements,
// and after each attempt an exchange that brings every shard's partials to every rank before the next control.
struct OdeGlobal {
    int rows_total, part_n, part_off;
    gp_ode_exchange_fn exchange;
    void* ctx;
};

static size_t ode_auto_ws_bytes(int part_n) { return auto_part_off() + sizeof(double) * (size_t)part_n + 256; }

static int ode_auto_attempt_impl(const gp_head_weights* w, const float* pobj, int n, int what, double t_bound,
                                 double direction, double rtol, double atol, double sig_min, double base,
                                 double diff_scale, double* y0, double* y1, double* const* kslots,
                                 const double* tableau_a, const double* b, const double* e, int rows, int k,
                                 const OdeGlobal* g, void* workspace, size_t workspace_bytes, int* hstat,
                                 hipStream_t stream) {
    GP_REQUIRE(w && pobj && y0 && y1 && kslots && tableau_a && b && e && workspace && rows >= 1 && k >= 1 && n >= 0,
               "ode_auto_attempt: bad arguments");
    for (int j = 0; j < ODE_NK; ++j) GP_REQUIRE(kslots[j] != nullptr, "ode_auto_attempt: null K slot");
    char* ws = static_cast<char*>(workspace);
    OdeCtl* ctl = reinterpret_cast<OdeCtl*>(ws);
    float* tproj6 = reinterpret_cast<float*>(ws + auto_tproj_off());
    double* part = reinterpret_cast<double*>(ws + auto_part_off());
    const int nt = ode_nt(w, g ? g->rows_total : rows);
    const int nwg = (rows + 16 * nt - 1) / (16 * nt);   // this call's workgroups
    const int part_n = g ? g->part_n : nwg;
    GP_REQUIRE(!g || (g->part_off >= 0 && g->part_off + nwg <= part_n),
               "ode_auto_attempt: shard partials [%d, %d) outside %d", g ? g->part_off : 0, g ? g->part_off + nwg : 0,
               part_n);
    GP_REQUIRE(workspace_bytes >= ode_auto_ws_bytes(part_n), "ode_auto_attempt: workspace too small");
    OdeConsts kc = {t_bound, direction, rtol, atol, sig_min, base, diff_scale,
                    (double)(g ? g->rows_total : rows) * 9.0, part_n};
    OdeCtl* cin = ctl + (n & 1);
    OdeCtl* cout = ctl + ((n + 1) & 1);
    GP_REQUIRE(what >= 1 && what <= 3, "ode_auto_attempt: what must be 1 (control), 2 (stages) or 3 (both)");
    if (what & 1) {
        hipLaunchKernelGGL(ode_control_kernel, dim3(6, ODE_CTL_CHUNKS), dim3(HT), 0, stream, *w, (const OdeCtl*)cin,
                           cout, (const double*)part, n > 0 ? 1 : 0, kc, tproj6, hstat, n);
        const int rc = gp_check_launch("ode_control_kernel");
        if (rc || !(what & 2)) return rc;
    }
    OdeStageArgs a = {};
    a.w = *w;
    a.pobj = pobj;
    a.rows = rows;
    a.kper = k;
    a.part_off = g ? g->part_off : 0;
    a.rtol = rtol;
    a.atol = atol;
    a.ctl = cout;
    a.tproj6 = tproj6;
    a.ybuf[0] = y0;
    a.ybuf[1] = y1;
    for (int j = 0; j < ODE_NK; ++j) a.kbuf[j] = kslots[j];
    if (ode_fused()) {   // one launch per attempt (ode_attempt_kernel)
        OdeTableau tb;
        for (int j = 0; j < 36; ++j) tb.A[j] = tableau_a[j];
        for (int j = 0; j < 6; ++j) tb.B[j] = b[j];
        for (int j = 0; j < ODE_NK; ++j) a.e[j] = e[j];
        a.part = part;
        const dim3 grid(nwg), blk(EVAL_WV * 64);
        if (!w->pe2_h)
            hipLaunchKernelGGL((ode_attempt_kernel<0, 1>), grid, blk, 0, stream, a, tb);
        else if (nt == 4)
            hipLaunchKernelGGL((ode_attempt_kernel<X3P, 4>), grid, blk, 0, stream, a, tb);
        else if (nt == 2)
            hipLaunchKernelGGL((ode_attempt_kernel<X3P, 2>), grid, blk, 0, stream, a, tb);
        else
            hipLaunchKernelGGL((ode_attempt_kernel<X3P, 1>), grid, blk, 0, stream, a, tb);
        const int rc = gp_check_launch("ode_attempt_kernel");
        if (rc || !g) return rc;
        GP_REQUIRE(g->exchange(g->ctx, n, part, part_n, stream) == 0, "ode_auto_attempt: partials exchange of attempt %d",
                   n);
        return GP_OK;
    }
    for (int s = 1; s < 6; ++s) {
        a.stage = s;
        a.nk = s;
        for (int j = 0; j < s; ++j) a.a[j] = tableau_a[s * 6 + j];
        ode_launch_stage<0>(a, nt, stream);
    }
    a.stage = 6;
    a.nk = 6;
    for (int j = 0; j < 6; ++j) a.a[j] = b[j];
    for (int j = 0; j < ODE_NK; ++j) a.e[j] = e[j];
    a.part = part;
    ode_launch_stage<1>(a, nt, stream);
    const int rc = gp_check_launch("ode_stage_kernel<auto>");
    if (rc || !g) return rc;
    GP_REQUIRE(g->exchange(g->ctx, n, part, part_n, stream) == 0, "ode_auto_attempt: partials exchange of attempt %d", n);
    return GP_OK;
}

extern "C" int gp_ode_auto_attempt(const gp_head_weights* w, const float* pobj, int n, int what,
                                   double t_bound, double direction, double rtol, double atol, double sig_min,
                                   double base, double diff_scale, double* y0, double* y1,
                                   double* const* kslots, const double* tableau_a, const double* b,
                                   const double* e, int rows, int k, void* workspace, size_t workspace_bytes,
                                   hipStream_t stream) {
    return ode_auto_attempt_impl(w, pobj, n, what, t_bound, direction, rtol, atol, sig_min, base, diff_scale, y0, y1,
                                 kslots, tableau_a, b, e, rows, k, nullptr, workspace, workspace_bytes, nullptr, stream);
}

extern "C" int gp_ode_auto_attempt_hs(const gp_head_weights* w, const float* pobj, int n, int what,
                                      double t_bound, double direction, double rtol, double atol, double sig_min,
                                      double base, double diff_scale, double* y0, double* y1,
                                      double* const* kslots, const double* tableau_a, const double* b,
                                      const double* e, int rows, int k, void* workspace, size_t workspace_bytes,
                                      int* host_status, hipStream_t stream) {
    GP_REQUIRE(host_status != nullptr, "ode_auto_attempt_hs: null status words");
    return ode_auto_attempt_impl(w, pobj, n, what, t_bound, direction, rtol, atol, sig_min, base, diff_scale, y0, y1,
                                 kslots, tableau_a, b, e, rows, k, nullptr, workspace, workspace_bytes, host_status,
                                 stream);
}

extern "C" int gp_ode_global_partials(int rows_total, int shard_rows_max, int shards, int split) {
    if (rows_total < 1 || shard_rows_max < 1 || shards < 1) return 0;
    const int tile = 16 * head_pick_nt(rows_total, split != 0);
    return shards * ((shard_rows_max + tile - 1) / tile);
}

extern "C" size_t gp_ode_global_workspace_size(int part_n) { return part_n >= 1 ? ode_auto_ws_bytes(part_n) : 0; }

extern "C" size_t gp_ode_auto_partials_offset(void) { return auto_part_off(); }

extern "C" int gp_ode_auto_attempt_global(const gp_head_weights* w, const float* pobj, int n, int what,
                                          double t_bound, double direction, double rtol, double atol, double sig_min,
                                          double base, double diff_scale, double* y0, double* y1,
                                          double* const* kslots, const double* tableau_a, const double* b,
                                          const double* e, int rows, int k, int rows_total, int row_off, int shard,
                                          int shards, int shard_rows_max, gp_ode_exchange_fn exchange, void* ctx,
                                          void* workspace, size_t workspace_bytes, int* host_status,
                                          hipStream_t stream) {
    GP_REQUIRE(w && exchange, "ode_auto_attempt_global: null pointer");
    GP_REQUIRE(shards >= 1 && shard >= 0 && shard < shards && rows >= 1 && rows <= shard_rows_max && row_off >= 0 &&
                   row_off + rows <= rows_total,
               "ode_auto_attempt_global: shard %d of %d, rows [%d, %d) of %d (at most %d per shard)", shard, shards,
               row_off, row_off + rows, rows_total, shard_rows_max);
    const int tile = 16 * ode_nt(w, rows_total);
    const int per = (shard_rows_max + tile - 1) / tile;
    OdeGlobal g = {rows_total, shards * per, shard * per, exchange, ctx};
    return ode_auto_attempt_impl(w, pobj, n, what, t_bound, direction, rtol, atol, sig_min, base, diff_scale, y0, y1,
                                 kslots, tableau_a, b, e, rows, k, &g, workspace, workspace_bytes, host_status, stream);
}

// ============================================================================ whole sampler (C hosts)
// cond_ode_sampler (samplers.py:180-258) in one call for hosts without Python: select_initial_step
// (scipy _ivp/common.py) from two host-scalar RHS evaluations, then the device-controlled attempts
// (gp_ode_auto_attempt) kept one attempt ahead of a 4-byte status read, the dense output at eps when
// `steps` > 0 (t_eval = linspace(T0, eps, steps): only its last point reaches cond_ode_sampler), the
// final denoise step and the epilogue (gp_ode_denoise). genpose2_amd/ode.py (rk45_device) and
// agent.py (PoseNet._ode) are the Python form of the same sequence.
namespace {
// Dormand-Prince tableau exactly as scipy's RK45 class attributes (rk.py)
const double kA6[36] = {0, 0, 0, 0, 0, 0,
                        1.0 / 5, 0, 0, 0, 0, 0,
                        3.0 / 40, 9.0 / 40, 0, 0, 0, 0,
                        44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0, 0,
                        19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0, 0,
                        9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656, 0};
const double kB6[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
const double kE7[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40};
const double kP74[28] = {1, -8048581381.0 / 2820520608, 8663915743.0 / 2820520608, -12715105075.0 / 11282082432,
                         0, 0, 0, 0,
                         0, 131558114200.0 / 32700410799, -68118460800.0 / 10900136933, 87487479700.0 / 32700410799,
                         0, -1754552775.0 / 470086768, 14199869525.0 / 1410260304, -10690763975.0 / 1880347072,
                         0, 127303824393.0 / 49829197408, -318862633887.0 / 49829197408, 701980252875.0 / 199316789632,
                         0, -282668133.0 / 205662961, 2019193451.0 / 616988883, -1453857185.0 / 822651844,
                         0, 40617522.0 / 29380423, -110615467.0 / 29380423, 69997945.0 / 29380423};
constexpr double kSigMin = 0.01, kBase = 50.0 / 0.01;

double diff_scale() { return sqrt(2.0 * (log(50.0) - log(0.01))); }
// sigma(t32) as sde.py forms it for a float32 tensor: f32(0.01) * 5000^t32 (power correctly rounded)
float sigma32(float t32) { return 0.01f * (float)pow(kBase, (double)t32); }

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

struct OdeSampleLayout {
    size_t y[2], k[ODE_NK], f1, dense, scal, rhs_ws, auto_ws, total;
};
OdeSampleLayout ode_sample_layout(int rows) {
    OdeSampleLayout L = {};
    const size_t vec = align256((size_t)rows * 9 * sizeof(double));
    size_t off = 0;
    for (int i = 0; i < 2; ++i) { L.y[i] = off; off += vec; }
    for (int j = 0; j < ODE_NK; ++j) { L.k[j] = off; off += vec; }
    L.f1 = off; off += vec;
    L.dense = off; off += vec;
    L.scal = off; off += 256;
    L.rhs_ws = off; off += align256(gp_ode_workspace_size(rows));
    L.auto_ws = off; off += align256(gp_ode_auto_workspace_size(rows));
    L.total = off;
    return L;
}

// Host resources of gp_ode_sample's status reads (a pinned int and an event on the stream's device),
// leased from a per-device pool for one call and returned after it. A per-thread cache bound them to
// the first device a thread used, which breaks a host that drives several GPUs from one thread (or a
// cgo host, whose goroutines move between OS threads); creating them per call would cost a
// device-synchronising hipHostFree. The pool holds at most as many readers per device as calls ever
// ran on it at once.
struct StatusReader {
    int* pinned;
    hipEvent_t ev;
    int dev;
};
std::mutex g_status_mu;
std::vector<StatusReader> g_status_pool;

struct StatusLease {
    StatusReader r{nullptr, nullptr, -1};
    hipStream_t stream = nullptr;
    bool pending = false;   // a status copy into r.pinned was enqueued and may not have landed yet
    int acquire(hipStream_t s) {
        stream = s;
        int cur = 0, dev = 0;
        if (hipGetDevice(&cur) != hipSuccess) return -1;
        dev = cur;
        if (s != nullptr && hipStreamGetDevice(s, &dev) != hipSuccess) return -1;
        {
            std::lock_guard<std::mutex> lk(g_status_mu);
            for (size_t i = 0; i < g_status_pool.size(); ++i)
                if (g_status_pool[i].dev == dev) {
                    r = g_status_pool[i];
                    g_status_pool.erase(g_status_pool.begin() + (long)i);
                    return 0;
                }
        }
        if (dev != cur && hipSetDevice(dev) != hipSuccess) return -1;
        r.dev = dev;
        bool ok = hipHostMalloc(reinterpret_cast<void**>(&r.pinned), 64, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&r.ev, hipEventDisableTiming) == hipSuccess;
        if (!ok) {   // a partial creation frees what it made (nothing of it is pooled)
            if (r.pinned != nullptr) (void)hipHostFree(r.pinned);
            r.pinned = nullptr;
            r.ev = nullptr;
        }
        if (dev != cur) (void)hipSetDevice(cur);
        return ok ? 0 : -1;
    }
    ~StatusLease() {
        if (r.pinned == nullptr || r.ev == nullptr) return;
        // an early return between the status copy and its wait leaves the copy in flight: it must land
        // before another call can lease this pinned word (if the stream cannot be drained, the reader is
        // dropped rather than pooled)
        if (pending && hipStreamSynchronize(stream) != hipSuccess) return;
        std::lock_guard<std::mutex> lk(g_status_mu);
        g_status_pool.push_back(r);
    }
};
}  // namespace

__global__ void f32_to_f64_kernel(const float* __restrict__ in, double* __restrict__ out, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (double)in[i];
}

extern "C" size_t gp_ode_sample_workspace_size(int rows) { return rows >= 1 ? ode_sample_layout(rows).total : 0; }

extern "C" int gp_ode_sample(const gp_head_weights* w, const float* pobj, const float* x0, int rows, int k, double T0,
                             double eps, int steps, double rtol, double atol, const float* pts_center, double* pose,
                             double* q, int* nfev_out, int* status_out, void* workspace, size_t workspace_bytes,
                             hipStream_t stream) {
    GP_REQUIRE(w && pobj && x0 && pts_center && pose && q && workspace && rows >= 1 && k >= 1 && steps >= 0,
               "ode_sample: bad arguments");
    GP_REQUIRE(T0 != eps, "ode_sample: empty integration interval (T0 == eps)");
    GP_REQUIRE(steps != 1, "ode_sample: steps must be 0 (t_eval unset) or >= 2");
    const OdeSampleLayout L = ode_sample_layout(rows);
    GP_REQUIRE(workspace_bytes >= L.total, "ode_sample: workspace too small (gp_ode_sample_workspace_size)");
    StatusLease status;
    GP_REQUIRE(status.acquire(stream) == 0, "ode_sample: pinned status word / event");
    char* ws = static_cast<char*>(workspace);
    double* y[2] = {reinterpret_cast<double*>(ws + L.y[0]), reinterpret_cast<double*>(ws + L.y[1])};
    double* K[ODE_NK];
    for (int j = 0; j < ODE_NK; ++j) K[j] = reinterpret_cast<double*>(ws + L.k[j]);
    double* f1 = reinterpret_cast<double*>(ws + L.f1);
    double* dense = reinterpret_cast<double*>(ws + L.dense);
    double* scal = reinterpret_cast<double*>(ws + L.scal);
    void* rws = ws + L.rhs_ws;
    void* aws = ws + L.auto_ws;
    const size_t rws_b = gp_ode_workspace_size(rows), aws_b = gp_ode_auto_workspace_size(rows);
    const long long n = (long long)rows * 9;
    const double t0 = T0, tf = eps, dir = tf > t0 ? 1.0 : -1.0;
    const double dscale = diff_scale();
    int rc;
    hipLaunchKernelGGL(f32_to_f64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x0, y[0], n);
    if ((rc = gp_check_launch("f32_to_f64_kernel"))) return rc;

    // ---- select_initial_step (scipy common.py), as genpose2_amd/ode.py initial_step
    {   // f(t0): solve_ivp hands t0 as a Python float, so ode_func's g is float32 sigma * float64 scale
        const float t32 = (float)t0;
        const double g = (double)sigma32(t32) * dscale;
        if ((rc = gp_ode_rhs(w, pobj, t32, sigma32(t32), -(0.5 * (g * g)), y[0], nullptr, nullptr, 0, 0.0, rows, k,
                             K[0], rws, rws_b, stream)))
            return rc;
    }
    if ((rc = gp_ode_init_norms(y[0], K[0], nullptr, n, atol, rtol, scal, stream))) return rc;
    double hs[3];
    GP_REQUIRE(hipMemcpyAsync(hs, scal, 2 * sizeof(double), hipMemcpyDeviceToHost, stream) == hipSuccess &&
                   hipStreamSynchronize(stream) == hipSuccess, "ode_sample: norm read");
    const double d0 = hs[0], d1 = hs[1], interval = fabs(tf - t0);
    double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    h0 = fmin(h0, interval);
    {   // f(t0 + h0 dir, y0 + h0 dir f0): a NumPy float64 time from here on
        const double t = t0 + h0 * dir;
        const double g = kSigMin * pow(kBase, t) * dscale;
        const double a1 = 1.0;
        const double* kin[1] = {K[0]};
        if ((rc = gp_ode_rhs(w, pobj, (float)t, sigma32((float)t), -(0.5 * (g * g)), y[0], kin, &a1, 1, h0 * dir,
                             rows, k, f1, rws, rws_b, stream)))
            return rc;
    }
    if ((rc = gp_ode_init_norms(y[0], K[0], f1, n, atol, rtol, scal, stream))) return rc;
    GP_REQUIRE(hipMemcpyAsync(hs + 2, scal + 2, sizeof(double), hipMemcpyDeviceToHost, stream) == hipSuccess &&
                   hipStreamSynchronize(stream) == hipSuccess, "ode_sample: norm read");
    const double d2 = hs[2] / h0;
    const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 1.0 / 5.0);
    const double h_abs = fmin(fmin(100 * h0, h1), interval);

    // ---- device-controlled attempts, one enqueued ahead of the status read
    OdeCtl c0 = {};
    c0.t = t0;
    c0.h_abs = h_abs;
    c0.nfev = 2;
    for (int j = 0; j < ODE_NK; ++j) c0.kidx[j] = j;
    GP_REQUIRE(hipMemcpyAsync(aws, &c0, sizeof(OdeCtl), hipMemcpyHostToDevice, stream) == hipSuccess &&
                   hipStreamSynchronize(stream) == hipSuccess, "ode_sample: controller record");
    auto launch = [&](int a, int what) {
        return gp_ode_auto_attempt(w, pobj, a, what, tf, dir, rtol, atol, kSigMin, kBase, dscale, y[0], y[1], K,
                                   kA6, kB6, kE7, rows, k, aws, aws_b, stream);
    };
    const int rec = (int)sizeof(OdeCtl);
    const int stat_off = (int)offsetof(OdeCtl, status);
    int a = 0;
    int* hs_dev = nullptr;   // the pinned words as the device addresses them, if it can
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&hs_dev), status.r.pinned, 0) != hipSuccess) {
        hs_dev = nullptr;
        (void)hipGetLastError();
    }
    if (hs_dev != nullptr) {
        // polled: the control kernel of attempt n writes 4 n + (status + 1) into pinned word n & 3; nothing sits
        // between a control launch and its stage launch (gp_ode_auto_attempt_hs)
        volatile int* hv = status.r.pinned;
        for (int i = 0; i < 4; ++i) hv[i] = -1;
        auto launch_hs = [&](int n) {
            return gp_ode_auto_attempt_hs(w, pobj, n, 3, tf, dir, rtol, atol, kSigMin, kBase, dscale, y[0], y[1], K,
                                          kA6, kB6, kE7, rows, k, aws, aws_b, hs_dev, stream);
        };
        status.pending = true;   // the device writes the words until the stream drains
        if ((rc = launch_hs(0))) return rc;
        for (;; ++a) {
            GP_REQUIRE(a < 100000, "ode_sample: attempt limit reached");
            if ((rc = launch_hs(a + 1))) return rc;   // decides attempt a, prepares and runs a + 1
            const int want = a + 1;
            const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(60);
            int v;
            while (((v = hv[want & 3]) >> 2) != want)
                GP_REQUIRE(std::chrono::steady_clock::now() < t_end, "ode_sample: no status from attempt %d", want);
            if ((v & 3) - 1 != 0) break;
        }
    } else {
        if ((rc = launch(0, 3))) return rc;
        for (;; ++a) {
            GP_REQUIRE(a < 100000, "ode_sample: attempt limit reached");
            if ((rc = launch(a + 1, 1))) return rc;   // decides attempt a, prepares a + 1
            const char* src = static_cast<const char*>(aws) + ((a + 2) & 1) * rec + stat_off;
            status.pending = true;
            GP_REQUIRE(hipMemcpyAsync(status.r.pinned, src, 4, hipMemcpyDeviceToHost, stream) == hipSuccess &&
                           hipEventRecord(status.r.ev, stream) == hipSuccess, "ode_sample: status read");
            if ((rc = launch(a + 1, 2))) return rc;   // attempt a + 1 (a no-op once the solve has ended)
            GP_REQUIRE(hipEventSynchronize(status.r.ev) == hipSuccess, "ode_sample: status wait");
            status.pending = false;
            if (*status.r.pinned != 0) break;
        }
    }
    OdeCtl c;
    GP_REQUIRE(hipMemcpyAsync(&c, static_cast<const char*>(aws) + ((a + 2) & 1) * rec, sizeof(OdeCtl),
                              hipMemcpyDeviceToHost, stream) == hipSuccess &&
                   hipStreamSynchronize(stream) == hipSuccess, "ode_sample: final record");
    status.pending = false;
    if (status_out) *status_out = c.status;
    if (nfev_out) *nfev_out = c.nfev;
    GP_REQUIRE(!(c.status < 0 && steps > 0),
               "ode_sample: RK45 failed (step size below the spacing of t) with t_eval set: the collected t_eval "
               "outputs need the host controller (genpose2_amd/ode.py rk45_drive)");
    const double* x = y[c.yi];
    if (steps > 0 && c.status > 0) {   // res.y[:, -1]: the final step's dense output at t_eval[-1] = eps
        const double* ks[ODE_NK];
        for (int j = 0; j < ODE_NK; ++j) ks[j] = K[c.kidx[j]];
        std::swap(ks[0], ks[ODE_NK - 1]);   // undo the FSAL swap of the accepted step
        GP_REQUIRE(hipMemcpyAsync(scal + 7, &eps, sizeof(double), hipMemcpyHostToDevice, stream) == hipSuccess &&
                       hipStreamSynchronize(stream) == hipSuccess, "ode_sample: t_eval");
        if ((rc = gp_ode_dense(ks, kP74, y[c.yi ^ 1], scal + 7, 0, 1, 0, 0, c.t_old, c.t - c.t_old, n, dense, stream)))
            return rc;
        x = dense;
    }
    // ---- denoise (samplers.py:240-249) with eps's scalars: a float32 1-element tensor for g
    const float te = (float)eps;
    const float sig = sigma32(te);
    const float g = sig * (float)dscale;
    const float step = (float)((1.0 - eps) / (steps > 0 ? steps : 1000));
    return gp_ode_denoise(w, pobj, te, sig, g * g, step, x, rows, k, pts_center, pose, q, rws, rws_b, stream);
}
