// Score / energy heads and the fused PC sampling step for gfx950.
//
// Reference: PoseScoreNet.forward (networks/gf_algorithms/scorenet.py:215-275), PoseEnergyNet.get_energy
// (energynet.py:151-208), cond_pc_sampler (samplers.py:113-177), VE SDE (sde.py:15-35).
//
// Hoisting. The first head layer Linear(1408 -> 3x256) sees [pts_feat | t_feat | pose_feat]. The pts
// block is constant per object and the t block is constant per step, so they are computed once
// (gp_head_object_proj: B x 1024 x 768, gp_head_time_proj: T x 128 x 768) and enter the per-candidate
// GEMM as the accumulator's initial value. Per candidate-step only pose 9->256->256 -> 3x256 and the
// block-diagonal 3x(256->3) remain: 0.5335 MFLOP instead of the reference's 2.336 MFLOP.
//
// Tiling. A workgroup (8 waves) owns 16 candidates. Candidates are MFMA columns, output channels are
// MFMA rows, so weights are the streamed A operand (packed per lane by pack.py: coalesced 1 KiB
// loads) and activations stay in the accumulator-native LDS layout between layers. The two
// per-candidate GEMMs run as split-f16 MFMA (gp_head.h head_trunk_split) when gp_head_weights
// carries the packed f16 planes, exact f32 MFMA (v_mfma_f32_16x16x4_f32) otherwise.
//
// PC step fusion. The Langevin step size uses the mean score norm over ALL rows of the call
// (samplers.py:143), a grid-wide dependency. Launch i therefore (a) finishes step i-1 for its own
// rows -- reading the per-tile norm partials every tile wrote in launch i-1, summed in one fixed
// order so every workgroup derives the identical grad_norm -- and (b) evaluates the score at step i
// and publishes its tile's partial. The kernel boundary is the only grid-wide synchronisation.

#include "gp_common.h"


// Phase timestamps for tuning builds only (make EXTRA=-DPC_TRACE; read by scripts/pc_trace.py). Per wave of the
// first 256 workgroups, three launch slots (step parity; 2 = the finalize launch i = steps): slots 0..15
// shader-clock stamps (s_memtime) of the marks, 16 / 17 the constant 100 MHz clock (s_memrealtime) at marks 0 / 8
// (workgroup start / end on one chip-wide time base: s_memtime runs per XCD at the current shader clock), 18 the
// HW_ID register | XCC_ID << 32.
#ifdef PC_TRACE
constexpr int PC_TR_SLOTS = 20;
__device__ unsigned long long g_pc_trace[3 * 256 * 8 * PC_TR_SLOTS];
#define PC_TR_AT(k) g_pc_trace[((trace_slot * 256 + blockIdx.x) * 8 + (threadIdx.x >> 6)) * PC_TR_SLOTS + (k)]
#define PC_MARK(k)                                                                                       \
    do {                                                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) {                                               \
            PC_TR_AT(k) = __builtin_amdgcn_s_memtime();                                                  \
            if ((k) == 0 || (k) == 8) PC_TR_AT(16 + ((k) == 8)) = __builtin_amdgcn_s_memrealtime();      \
            if ((k) == 0)                                                                                \
                PC_TR_AT(18) = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) | \
                               ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32); \
        }                                                                                                \
    } while (0)
extern "C" int gp_debug_pc_trace(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pc_trace), sizeof(g_pc_trace)) == hipSuccess ? 0 : -1;
}
#else
#define PC_MARK(k) ((void)trace_slot)
#endif
#include "gp_head.h"

// ============================================================================ hoist kernels
__global__ __launch_bounds__(HT) void object_proj_kernel(gp_head_weights w, const float* __restrict__ feat,
                                                         float* __restrict__ pobj) {
    __shared__ float sf[1024];
    const int b = blockIdx.y;
    for (int i = threadIdx.x; i < 1024; i += HT) sf[i] = feat[(size_t)b * 1024 + i];
    __syncthreads();
    const int o = blockIdx.x * HT + threadIdx.x;  // 0..767
#if HOIST64
    pobj[(size_t)b * 768 + o] = (float)(dot_f64<1024>(w.h1pts_t + o, 768, sf) + (double)w.h1_b[o]);
#else
    pobj[(size_t)b * 768 + o] = dot_chains<1024, 32>(w.h1pts_t + o, 768, sf) + w.h1_b[o];
#endif
}

extern "C" int gp_head_object_proj(const gp_head_weights* w, const float* pts_feat, int b, float* pobj,
                                   hipStream_t stream) {
    GP_REQUIRE(w && pts_feat && pobj && b >= 0, "head_object_proj: bad arguments");
    if (!b) return GP_OK;
    hipLaunchKernelGGL(object_proj_kernel, dim3(3, b), dim3(HT), 0, stream, *w, pts_feat, pobj);
    return gp_check_launch("object_proj_kernel");
}

__global__ __launch_bounds__(HT) void time_proj_kernel(gp_head_weights w, const float* __restrict__ tv,
                                                       float* __restrict__ tproj) {
    __shared__ float emb[128];
    __shared__ float tf[128];
    const int k = blockIdx.x;
    time_row(w, tv[k], emb, tf, tproj + (size_t)k * 768);
}

extern "C" int gp_head_time_proj(const gp_head_weights* w, const float* t, int nt, float* tproj,
                                 hipStream_t stream) {
    GP_REQUIRE(w && t && tproj && nt >= 0, "head_time_proj: bad arguments");
    if (!nt) return GP_OK;
    hipLaunchKernelGGL(time_proj_kernel, dim3(nt), dim3(HT), 0, stream, *w, t, tproj);
    return gp_check_launch("time_proj_kernel");
}

// ============================================================================ score / energy eval
template <int MODE, int PL>  // MODE 0: score f/(sigma+1e-7), 1: energy (IP, decoupled); PL 0: exact fp32, X3P: f16x3
__global__ __launch_bounds__(EVAL_WV * 64) void head_eval_kernel(gp_head_weights w, const float* __restrict__ pobj,
                                                       const float* __restrict__ tproj, float sigma,
                                                       const float* __restrict__ x, int rows, int kper,
                                                       float* __restrict__ out) {
    __shared__ HeadSmem<1, EVAL_WV, PL> sm;
    constexpr bool SPLIT = PL != 0;
    __shared__ int obj[16];
    const int r0 = blockIdx.x * 16;
    SplitScalars hs = {};
    if constexpr (SPLIT) hs = load_split_scalars(w);
    stage_small_weights<1, EVAL_WV, 0, !SPLIT>(w, sm);
    for (int i = threadIdx.x; i < 256; i += EVAL_WV * 64) {
        const int c = i >> 4, j = i & 15;
        const int r = r0 + c;
        sm.xin[i] = (r < rows && j < 9) ? x[(size_t)r * 9 + j] : 0.f;
    }
    if (threadIdx.x < 16) {
        const int r = r0 + threadIdx.x;
        obj[threadIdx.x] = (r < rows ? r : rows - 1) / kper;
    }
    if constexpr (SPLIT)
        head_trunk_x3<1, EVAL_WV>(w, pobj, tproj, obj, sm, 0, hs);
    else
        head_trunk<1, EVAL_WV>(w, pobj, tproj, obj, sm);
    if (MODE == 0) {
        if (threadIdx.x < 144) {
            const int c = threadIdx.x / 9, o = threadIdx.x - c * 9;
            if (r0 + c < rows) out[(size_t)(r0 + c) * 9 + o] = fdiv(head_out(sm, c, o), fadd(sigma, 1e-7f));
        }
    } else {
        // energy = [sum_{o<6} pose_o * s_o, sum_{o>=6} pose_o * s_o] with s = f / sigma (energynet.py:175-193):
        // each product rounded on its own (no contraction), summed in the order torch's CPU sum takes over a
        // contiguous row -- ((((p0 + p4) + p5) + p1) + p2) + p3 for the six rotation entries, (p6 + p7) + p8
        // for the translation (checked against torch.sum on 200k random rows) -- so rows whose energies tie
        // to the last bits in the reference rank as they do there
        if (threadIdx.x < 32) {
            const int c = threadIdx.x >> 1, part = threadIdx.x & 1;
            if (r0 + c < rows) {
                float p[9];
#pragma unroll
                for (int o = 0; o < 9; ++o) p[o] = fmul(sm.xin[c * 16 + o], fdiv(head_out(sm, c, o), sigma));
                const float e = part ? fadd(fadd(p[6], p[7]), p[8])
                                     : fadd(fadd(fadd(fadd(fadd(p[0], p[4]), p[5]), p[1]), p[2]), p[3]);
                out[(size_t)(r0 + c) * 2 + part] = e;
            }
        }
    }
}

extern "C" int gp_score_eval(const gp_head_weights* w, const float* pobj, const float* tproj_row, float sigma,
                             const float* x, int rows, int k, float* score, hipStream_t stream) {
    GP_REQUIRE(w && pobj && tproj_row && x && score && rows >= 0 && k >= 1, "score_eval: bad arguments");
    if (!rows) return GP_OK;
    if (w->pe2_h)
        hipLaunchKernelGGL((head_eval_kernel<0, X3P>), dim3((rows + 15) / 16), dim3(EVAL_WV * 64), 0, stream, *w, pobj, tproj_row,
                       sigma, x, rows, k, score);
    else
        hipLaunchKernelGGL((head_eval_kernel<0, 0>), dim3((rows + 15) / 16), dim3(EVAL_WV * 64), 0, stream, *w, pobj, tproj_row,
                       sigma, x, rows, k, score);
    return gp_check_launch("head_eval_kernel<score>");
}

extern "C" int gp_energy_eval(const gp_head_weights* w, const float* pobj, const float* tproj_row, float sigma,
                              const float* pose, int rows, int k, float* energy, hipStream_t stream) {
    GP_REQUIRE(w && pobj && tproj_row && pose && energy && rows >= 0 && k >= 1, "energy_eval: bad arguments");
    if (!rows) return GP_OK;
    if (w->pe2_h)
        hipLaunchKernelGGL((head_eval_kernel<1, X3P>), dim3((rows + 15) / 16), dim3(EVAL_WV * 64), 0, stream, *w, pobj, tproj_row,
                       sigma, pose, rows, k, energy);
    else
        hipLaunchKernelGGL((head_eval_kernel<1, 0>), dim3((rows + 15) / 16), dim3(EVAL_WV * 64), 0, stream, *w, pobj, tproj_row,
                       sigma, pose, rows, k, energy);
    return gp_check_launch("head_eval_kernel<energy>");
}

// ============================================================================ PC sampler
struct PCStep {       // one row of step_tab: {t, sigma, g, dt, sqrt_dt}
    float t, sigma, g, dt, sqrt_dt;
};

struct PCArgs {
    gp_head_weights w;
    const float* pobj;
    const float* tproj;   // (T, 768)
    float* x;             // (R, 9) state
    float* s;             // (R, 9) score of the previous step
    float* part;          // (2, part_n) per-workgroup sums of row score norms; this call's workgroups write
                          // entries [part_off, part_off + nwg) of a slot
    int part_n, part_off; // entries summed for grad_norm (nwg / 0 for a call on its own rows; every shard's
                          // workgroups in shard order for a global-batch call, gp_pc_sample_global)
    int norm_rows;        // rows grad_norm averages over (rows, or the global batch's)
    int row_off;          // global index of row 0 (the Philox draws' row counter)
    float* zbuf;          // (2 slots, 2 streams, R, 9) Philox draws: launch i writes step i's into slot
                          // i&1 while its wave 0 reads step i-1's from the other slot (no ordering
                          // between the waves of a workgroup is needed)
    const float* z1;      // (T, R, 9) or null -> Philox
    const float* z2;
    uint64_t seed;
    const float* center;  // (B, 3)
    float* res;           // (R, 9)
    float* q;             // (R, 7)
    float* xs;            // (R, T, 9) or null
    int rows, kper, steps, nwg;
    float ls_coef;        // snr * sqrt(pose_dim)
};

// One update wave's part of step i-1 -> i for its 16 rows (wave g owns rows 16g .. 16g+15, four lanes per row:
// part p < 3 owns elements [3p, 3p+3) -- rot6 columns a1, a2, translation; lane 4c+3 only pads the row).
// gacc: the lane's share of sum_r ||s_r|| over every row of step i-1, summed by the caller in the fixed
// lane / index order both kernels share, so every workgroup derives the identical grad_norm. x3: this lane's
// entries of x (updated in place); sv, z1v, z2v: its entries of the previous score and the two draws.
// Writes xin (the trunk's input), the split trunk's per-column scales, obj, and the outputs (x when store_x,
// the trajectory, res / q at the last step).
template <int NT, int WV, int PL>
__device__ __forceinline__ void pc_update_rows(const PCArgs& a, int i, const PCStep& prev, HeadSmem<NT, WV, PL>& sm,
                                               int* obj, int g, int lane, int r0, float gacc, float (&x3)[3],
                                               const float (&sv)[3], const float (&z1v)[3], const float (&z2v)[3],
                                               const SplitScalars& hs, bool store_x, int trace_slot) {
#pragma clang fp contract(off)
    constexpr bool SPLIT = PL != 0;
    const int p = lane & 3;
    const int e0 = 3 * (p < 3 ? p : 0);
    if (lane < 16) {
        const int r = r0 + 16 * g + lane;
        obj[16 * g + lane] = (r < a.rows ? r : a.rows - 1) / a.kper;
    }
    PC_MARK(10);
    gacc = wave_sum(gacc);
    PC_MARK(11);
    const int c = 16 * g + (lane >> 2);
    const int r = r0 + c;
    const bool upd = i > 0 && r < a.rows && p < 3;
    if (upd) {
        const float gn = udiv(gacc, (float)a.norm_rows);
        const float ratio = udiv(a.ls_coef, gn);
        const float ls = 2.0f * (ratio * ratio);
        const float sq2ls = usqrt(2.0f * ls);
        float mean[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) x3[k] = (x3[k] + ls * sv[k]) + sq2ls * z1v[k];
        if (p < 2) {   // x[:, :3] /= ||x[:, :3]||, x[:, 3:6] /= ||x[:, 3:6]|| (samplers.py:157-160)
            const float nn = usqrt((x3[0] * x3[0] + x3[1] * x3[1]) + x3[2] * x3[2]);
            x3[0] = udiv(x3[0], nn); x3[1] = udiv(x3[1], nn); x3[2] = udiv(x3[2], nn);
        }
        // reverse-SDE Euler-Maruyama predictor (samplers.py:163-166; sign as in the reference)
        const float g2 = prev.g * prev.g;
        const float gs = prev.g * prev.sqrt_dt;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float drift = 0.0f - g2 * sv[k];
            mean[k] = x3[k] + drift * prev.dt;
            x3[k] = mean[k] + gs * z2v[k];
        }
        gram_schmidt6_quad(x3, p, lane);
        // the centre only where it is added (the trajectory, the last step): the loads are atomic (gp_common.h
        // ld1), which the compiler does not drop when their values go unused
        float cen[3] = {0.f, 0.f, 0.f};
        if (a.xs || i == a.steps) {
            const float* cp = a.center + (size_t)(r / a.kper) * 3;
            cen[0] = ld1(cp);
            cen[1] = ld1(cp + 1);
            cen[2] = ld1(cp + 2);
        }
        if (a.xs) {
            float* o = a.xs + ((size_t)r * a.steps + (i - 1)) * 9 + e0;
#pragma unroll
            for (int k = 0; k < 3; ++k) o[k] = p == 2 ? x3[k] + cen[k] : x3[k];
        }
        if (i == a.steps) {  // res = mean_x of the last step (+centre, GS), samplers.py:174-177
            if (p == 2) {
                mean[0] += cen[0];
                mean[1] += cen[1];
                mean[2] += cen[2];
            }
            gram_schmidt6_quad(mean, p, lane);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                a.res[(size_t)r * 9 + e0 + k] = mean[k];
                sm.xu[c * 9 + e0 + k] = mean[k];   // gathered below for the quaternion
            }
        }
        if (store_x || i == a.steps) {
#pragma unroll
            for (int k = 0; k < 3; ++k) a.x[(size_t)r * 9 + e0 + k] = x3[k];
        }
    }
    if (i == a.steps) {
        wave_sync();
        if (p == 0 && r < a.rows) {
            float m9[9], qq[4];
#pragma unroll
            for (int j = 0; j < 9; ++j) m9[j] = sm.xu[c * 9 + j];
            quat_from_gs<float>(m9, qq);
#pragma unroll
            for (int j = 0; j < 4; ++j) a.q[(size_t)r * 7 + j] = qq[j];
            a.q[(size_t)r * 7 + 4] = m9[6];
            a.q[(size_t)r * 7 + 5] = m9[7];
            a.q[(size_t)r * 7 + 6] = m9[8];
        }
    }
    if (p < 3) {
#pragma unroll
        for (int k = 0; k < 3; ++k) sm.xin[c * 16 + e0 + k] = (r < a.rows) ? x3[k] : 0.f;
    } else {
#pragma unroll
        for (int j = 9; j < 16; ++j) sm.xin[c * 16 + j] = 0.f;
    }
    if constexpr (SPLIT) {
        // this row's split-trunk scales, from the entries just written to xin (max |x| over the row's four
        // lanes by DPP), once here instead of in all eight waves of the trunk
        float m = (p < 3 && r < a.rows) ? fmaxf(fmaxf(fabsf(x3[0]), fabsf(x3[1])), fabsf(x3[2])) : 0.f;
        m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xF, 0xF, true)));
        m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x4E, 0xF, 0xF, true)));
        if (p == 0) {
            const ColScales cs = split_col_scales(m, hs);
            sm.cscl[c][0] = f32x4{cs.s1, cs.s2, cs.u2, cs.uh};
            sm.cscl[c][1] = f32x4{cs.sh, 0.f, 0.f, 0.f};
        }
    }
}

// Draws for the update of step i (applied one launch / iteration later), made while waves 0..NT-1 update:
// 2 streams x 3 blocks of 4 normals per row, streams 2i (corrector) and 2i+1 (predictor). dst(st, r, e)
// receives normal e < 9 of stream st for row r.
template <int NT, int WV, typename Dst>
__device__ __forceinline__ void pc_make_draws(const PCArgs& a, int i, int r0, Dst dst) {
    constexpr int ROWS = NT * 16;
    for (int e = tid_x() - 64 * NT; e < ROWS * 6; e += (WV - NT) * 64) {
        const int c = e / 6, st = (e - c * 6) / 3, blk = e - c * 6 - st * 3;
        const int r = r0 + c;
        if (r < a.rows) {
            const f32x4 v = philox_normal4(a.seed, (uint32_t)(st + 2 * i), (uint32_t)(a.row_off + r), (uint32_t)blk);
            dst(st, c, blk * 4 + 0, v.x);
            if (blk < 2) {
                dst(st, c, blk * 4 + 1, v.y);
                dst(st, c, blk * 4 + 2, v.z);
                dst(st, c, blk * 4 + 3, v.w);
            }
        }
    }
}

// s = f / (sigma + 1e-7) for the workgroup's rows (a lane per (row, output): 4 rows per wave as 16-lane rows,
// outputs 0..8 valid, row norms by a DPP row sum) handed to put(c, o, s); the waves' partials of sum_r ||s_r||
// combined in wave order after one barrier. Returns the workgroup partial (valid in thread 0).
template <int NT, int WV, int PL, typename Put>
__device__ __forceinline__ float pc_score_norm(const PCArgs& a, const PCStep& cur, HeadSmem<NT, WV, PL>& sm, int r0,
                                               int wid, int lane, Put put) {
    constexpr int ROWS = NT * 16;
    const float den = fadd(cur.sigma, 1e-7f);
    float wsum = 0.f;
    for (int cg = wid; cg < ROWS / 4; cg += WV) {
        const int c = 4 * cg + (lane >> 4), o = lane & 15;
        const int r = r0 + c;
        float v = 0.f;
        if (o < 9 && r < a.rows) {
            v = fdiv(head_out(sm, c, o), den);
            put(c, o, v);
        }
        wsum += rows_sum(sqrtf(row16_sum(fmul(v, v))));
    }
    if (lane == 0) sm.scratch[wid] = wsum;
    __syncthreads();
    float t = 0.f;
    if (wid == 0 && lane == 0) {
#pragma unroll
        for (int v = 0; v < WV; ++v) t += sm.scratch[v];
    }
    return t;
}

// Launch i in [0, steps]: finish step i-1 (if i > 0), then score at step i (if i < steps).
// Waves 0..NT-1 run the update, one 16-row column tile each (their global loads, the draws and the
// grad-norm reduction overlap), while the other waves make the next step's draws, stage the small
// weights and issue their first weight-stream loads; one barrier (inside the trunk) joins them.
template <int NT, int WV, int PL>   // PL 0: exact fp32 GEMMs, X3P: f16x3
__global__ __launch_bounds__(WV * 64) void pc_step_kernel(PCArgs a, int i, PCStep cur, PCStep prev) {
    constexpr int ROWS = NT * 16;
    static_assert(NT < WV, "at least one wave besides the update waves");
    __shared__ HeadSmem<NT, WV, PL> sm;
    constexpr bool SPLIT = PL != 0;
    __shared__ int obj[ROWS];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r0 = blockIdx.x * ROWS;
    const int trace_slot = i == a.steps ? 2 : (i & 1);
    SplitScalars hs = {};
    if constexpr (SPLIT) hs = load_split_scalars<WV>(a.w);   // in flight across the update
    PC_MARK(0);
    if (wid < NT) {
        // ---- every load first and unconditional (rows clamped: a guarded load becomes a branch,
        //      and the compiler then drains the first batch before issuing the next): the
        //      grad-norm partials of step i-1, then this lane's elements of x, s and the two draws.
        const int g = wid;
        const bool inj = a.z1 != nullptr;
        const float* zslot = a.zbuf + (size_t)((i - 1) & 1) * 2 * a.rows * 9;
        const float* z1p = inj ? a.z1 + ((size_t)(i > 0 ? i - 1 : 0) * a.rows) * 9 : zslot;
        const float* z2p = inj ? a.z2 + ((size_t)(i > 0 ? i - 1 : 0) * a.rows) * 9 : zslot + (size_t)a.rows * 9;
        const float* part = a.part + (size_t)((i - 1) & 1) * a.part_n;
        float pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pv[u] = part[min(lane + 64 * u, a.part_n - 1)];
        const int p = lane & 3;
        const int e0 = 3 * (p < 3 ? p : 0);
        float x3[3], sv[3], z1v[3], z2v[3];
        {
            const size_t e = (size_t)min(r0 + 16 * g + (lane >> 2), a.rows - 1) * 9 + e0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                x3[k] = ld1(a.x + e + k);
                sv[k] = ld1(a.s + e + k);
                z1v[k] = ld1(z1p + e + k);
                z2v[k] = ld1(z2p + e + k);
            }
        }
        // grad_norm = mean_r ||s_r|| over all rows of step i-1 (samplers.py:143); unused at i=0
        float gacc = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) gacc += lane + 64 * u < a.part_n ? pv[u] : 0.f;
        for (int t0 = 512; t0 < a.part_n; t0 += 512) {
#pragma unroll
            for (int u = 0; u < 8; ++u) pv[u] = part[min(t0 + lane + 64 * u, a.part_n - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) gacc += t0 + lane + 64 * u < a.part_n ? pv[u] : 0.f;
        }
        PC_MARK(9);
        pc_update_rows<NT, WV, PL>(a, i, prev, sm, obj, g, lane, r0, gacc, x3, sv, z1v, z2v, hs, true, trace_slot);
        PC_MARK(12);
    }
    if (i == a.steps) return;  // finalize launch: no score evaluation
    if (wid >= NT && a.z1 == nullptr)
        pc_make_draws<NT, WV>(a, i, r0, [&](int st, int c, int e, float v) {
            a.zbuf[((size_t)((i & 1) * 2 + st) * a.rows + r0 + c) * 9 + e] = v;
        });
    stage_small_weights<NT, WV, 64 * NT, !SPLIT>(a.w, sm);
    if constexpr (SPLIT)
        head_trunk_x3<NT, WV, true>(a.w, a.pobj, a.tproj + (size_t)i * 768, obj, sm, trace_slot, hs);
    else
        head_trunk<NT, WV>(a.w, a.pobj, a.tproj + (size_t)i * 768, obj, sm, trace_slot);
    PC_MARK(7);
    const float t = pc_score_norm<NT, WV, PL>(a, cur, sm, r0, wid, lane,
                                              [&](int c, int o, float v) { a.s[(size_t)(r0 + c) * 9 + o] = v; });
    if (tid == 0) a.part[(size_t)(i & 1) * a.part_n + a.part_off + blockIdx.x] = t;
    PC_MARK(8);
}

// Device standard normals in the PC sampler's draw layout: out[r][c] = philox_normal4(seed, stream,
// r, c / 4)[c % 4]. gp_pc_sample's draws of step j are streams 2j (corrector) and 2j+1 (predictor)
// with cols = 9, so a sampler run fed these as z1/z2 reproduces its Philox run exactly.
__global__ void randn_kernel(uint64_t seed, uint32_t stream, int rows, int cols, float* __restrict__ out) {
    const int nb = (cols + 3) >> 2;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)rows * nb) return;
    const int r = (int)(e / nb), blk = (int)(e - (long long)r * nb);
    const f32x4 v = philox_normal4(seed, stream, (uint32_t)r, (uint32_t)blk);
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (4 * blk + k < cols) out[(size_t)r * cols + 4 * blk + k] = vv[k];
}

extern "C" int gp_randn(uint64_t seed, uint32_t stream, int rows, int cols, float* out, hipStream_t hs) {
    GP_REQUIRE(rows >= 0 && cols >= 1 && (out || rows == 0), "randn: bad arguments");
    if (!rows) return GP_OK;
    const long long n = (long long)rows * ((cols + 3) >> 2);
    hipLaunchKernelGGL(randn_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, hs, seed, stream, rows, cols, out);
    return gp_check_launch("randn_kernel");
}

extern "C" size_t gp_pc_workspace_size(int rows) {
    const size_t ntiles = ((size_t)rows + 15) / 16;
    // s (R,9) | grad-norm partials (2, ntiles) | Philox draws (2 slots, 2 streams, R, 9)
    return sizeof(float) * ((size_t)rows * 9 * 5 + 2 * ntiles) + 256;
}

// Candidates per PC-step workgroup that gp_pc_sample picks for `rows` (split: head weights with
// the f16 planes) -- lets callers size their accounting from the kernel's real tiling.
extern "C" int gp_pc_tile_rows(int rows, int split) { return 16 * head_pick_nt(rows, split != 0); }

// cond_pc_sampler's time grid and VE SDE scalars (samplers.py:129-130, sde.py:15-27) as float32 rows
// {t, sigma(t), g(t), dt, sqrt(dt)} -- the table genpose2_amd/sde.py forms with torch, for hosts
// without Python. t is torch.linspace(1, eps, T) in float32 as torch computes it on the CPU: step =
// (eps - 1) / (T - 1) rounded once, t_i = 1 + step * i for i < T/2 and eps - step * (T - 1 - i) above,
// each with a single rounding. sigma = f32(0.01) * 5000^t with the power correctly rounded (torch's
// CPU pow is Sleef's 1-ulp vector routine: the two agree within 1 ulp, tests/test_cpu_host.py);
// g = sigma * f32(sqrt(2 ln 5000)) in float32; dt = t_0 - t_1; sqrt(dt) correctly rounded (torch's
// Sleef sqrt can be 1 ulp off it).
extern "C" int gp_pc_step_table(int steps, float eps, float* out) {
    GP_REQUIRE(out && steps >= 2, "pc_step_table: need steps >= 2 and an output of steps x 5 floats");
    const float start = 1.0f, end = eps;
    const float step = (end - start) / (float)(steps - 1);
    const int half = steps / 2;
    const float diff_scale = (float)sqrt(2.0 * (log(50.0) - log(0.01)));
    float t0 = 0.f, t1 = 0.f;
    for (int i = 0; i < steps; ++i) {
        const float t = i < half ? fmaf(step, (float)i, start) : fmaf(-step, (float)(steps - 1 - i), end);
        if (i == 0) t0 = t;
        if (i == 1) t1 = t;
        out[5 * i] = t;
    }
    const float dt = t0 - t1, sdt = sqrtf(t0 - t1);
    for (int i = 0; i < steps; ++i) {
        const float t = out[5 * i];
        const float sig = 0.01f * (float)pow(5000.0, (double)t);
        out[5 * i + 1] = sig;
        out[5 * i + 2] = sig * diff_scale;
        out[5 * i + 3] = dt;
        out[5 * i + 4] = sdt;
    }
    return GP_OK;
}

// The shared body of gp_pc_sample and gp_pc_sample_global: nt column tiles per workgroup, grad_norm over
// part_n partials of `part` averaged over norm_rows, exchange (if any) after every scoring launch.
static int pc_sample_impl(const gp_head_weights* w, const float* pobj, const float* tproj, const float* step_tab,
                          int steps, float* x, int rows, int k, const float* pts_center, const float* z1,
                          const float* z2, uint64_t seed, float snr, float* res, float* q, float* xs, void* workspace,
                          size_t workspace_bytes, int nt, float* part, int part_n, int part_off, int norm_rows,
                          int row_off, gp_pc_exchange_fn exchange, void* ctx, hipStream_t stream) {
    GP_REQUIRE(w && pobj && tproj && step_tab && x && pts_center && res && q && workspace,
               "pc_sample: null pointer");
    GP_REQUIRE(steps >= 2 && rows >= 1 && k >= 1, "pc_sample: need steps>=2, rows>=1, k>=1");
    GP_REQUIRE((z1 == nullptr) == (z2 == nullptr), "pc_sample: z1/z2 must both be given or both null");
    GP_REQUIRE(workspace_bytes >= gp_pc_workspace_size(rows), "pc_sample: workspace too small");
    // split-f16 GEMMs when the packed planes are given (gp_head_weights), exact fp32 otherwise
    const bool split = w->pe2_h != nullptr;
    GP_REQUIRE(!split || (w->h1p_h && w->hsc), "pc_sample: pe2_h, h1p_h and hsc must be given together");
    PCArgs a;
    a.w = *w;
    a.pobj = pobj;
    a.tproj = tproj;
    a.x = x;
    a.s = static_cast<float*>(workspace);
    a.zbuf = a.s + (size_t)rows * 9 + 2 * (((size_t)rows + 15) / 16);
    a.z1 = z1;
    a.z2 = z2;
    a.seed = seed;
    a.center = pts_center;
    a.res = res;
    a.q = q;
    a.xs = xs;
    a.rows = rows;
    a.kper = k;
    a.steps = steps;
    a.nwg = (rows + 16 * nt - 1) / (16 * nt);
    a.part = part != nullptr ? part : a.s + (size_t)rows * 9;
    a.part_n = part != nullptr ? part_n : a.nwg;
    a.part_off = part != nullptr ? part_off : 0;
    a.norm_rows = norm_rows;
    a.row_off = row_off;
    a.ls_coef = snr * 3.0f;  // snr * sqrt(pose_dim=9) in fp32 (0.48 rounds identically)
    GP_REQUIRE(a.part_off >= 0 && a.part_off + a.nwg <= a.part_n, "pc_sample: partials [%d, %d) outside %d entries",
               a.part_off, a.part_off + a.nwg, a.part_n);
    const dim3 grid(a.nwg);
    for (int i = 0; i <= steps; ++i) {
        PCStep cur = {}, prev = {};
        if (i < steps) cur = PCStep{step_tab[5 * i], step_tab[5 * i + 1], step_tab[5 * i + 2], step_tab[5 * i + 3],
                                    step_tab[5 * i + 4]};
        if (i > 0) prev = PCStep{step_tab[5 * (i - 1)], step_tab[5 * (i - 1) + 1], step_tab[5 * (i - 1) + 2],
                                 step_tab[5 * (i - 1) + 3], step_tab[5 * (i - 1) + 4]};
        if (nt == 4)
            hipLaunchKernelGGL((pc_step_kernel<4, PC_WV1, X3P>), grid, dim3(PC_WV1 * 64), 0, stream, a, i, cur, prev);
        else if (nt == 2)
            hipLaunchKernelGGL((pc_step_kernel<2, PC_WV1, X3P>), grid, dim3(PC_WV1 * 64), 0, stream, a, i, cur, prev);
        else if (split)
            hipLaunchKernelGGL((pc_step_kernel<1, PC_WV1, X3P>), grid, dim3(PC_WV1 * 64), 0, stream, a, i, cur, prev);
        else
            hipLaunchKernelGGL((pc_step_kernel<1, PC_WV1, 0>), grid, dim3(PC_WV1 * 64), 0, stream, a, i, cur, prev);
        if (exchange != nullptr && i < steps) {   // launch i's partials -> every shard before launch i + 1 reads them
            const int rc = gp_check_launch("pc_step_kernel");
            if (rc) return rc;
            GP_REQUIRE(exchange(ctx, i, a.part + (size_t)(i & 1) * a.part_n, a.part_n, stream) == 0,
                       "pc_sample_global: the partials exchange of step %d failed", i);
        }
    }
    return gp_check_launch("pc_step_kernel");
}

extern "C" int gp_pc_sample(const gp_head_weights* w, const float* pobj, const float* tproj, const float* step_tab,
                            int steps, float* x, int rows, int k, const float* pts_center, const float* z1,
                            const float* z2, uint64_t seed, float snr, float* res, float* q, float* xs,
                            void* workspace, size_t workspace_bytes, hipStream_t stream) {
    GP_REQUIRE(w != nullptr, "pc_sample: null pointer");
    return pc_sample_impl(w, pobj, tproj, step_tab, steps, x, rows, k, pts_center, z1, z2, seed, snr, res, q, xs,
                          workspace, workspace_bytes, head_pick_nt(rows, w->pe2_h != nullptr), nullptr, 0, 0, rows, 0,
                          nullptr, nullptr, stream);
}

extern "C" int gp_pc_global_partials(int rows_total, int shard_rows_max, int shards, int split) {
    if (rows_total < 1 || shard_rows_max < 1 || shards < 1) return 0;
    const int tile = 16 * head_pick_nt(rows_total, split != 0);
    return shards * ((shard_rows_max + tile - 1) / tile);
}

extern "C" int gp_pc_sample_global(const gp_head_weights* w, const float* pobj, const float* tproj,
                                   const float* step_tab, int steps, float* x, int rows, int k,
                                   const float* pts_center, uint64_t seed, float snr, float* res, float* q, float* xs,
                                   int rows_total, int row_off, int shard, int shards, int shard_rows_max,
                                   float* part, gp_pc_exchange_fn exchange, void* ctx, void* workspace,
                                   size_t workspace_bytes, hipStream_t stream) {
    GP_REQUIRE(w && part && exchange, "pc_sample_global: null pointer");
    GP_REQUIRE(shards >= 1 && shard >= 0 && shard < shards && rows >= 1 && rows <= shard_rows_max &&
                   row_off >= 0 && row_off + rows <= rows_total,
               "pc_sample_global: shard %d of %d, rows [%d, %d) of %d (at most %d per shard)", shard, shards, row_off,
               row_off + rows, rows_total, shard_rows_max);
    const int nt = head_pick_nt(rows_total, w->pe2_h != nullptr);   // the tiling of one call on the whole batch
    const int per = (shard_rows_max + 16 * nt - 1) / (16 * nt);
    return pc_sample_impl(w, pobj, tproj, step_tab, steps, x, rows, k, pts_center, nullptr, nullptr, seed, snr, res, q,
                          xs, workspace, workspace_bytes, nt, part, shards * per, shard * per, rows_total, row_off,
                          exchange, ctx, stream);
}

// ============================================================================ ODE epilogue (fp64)
__global__ void pose_epilogue_f64_kernel(double* pose, int rows, int kper, const float* center, double* q) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    double v[9];
    for (int j = 0; j < 9; ++j) v[j] = pose[(size_t)r * 9 + j];
    gram_schmidt6<double>(v);
    const float* c = center + (size_t)(r / kper) * 3;
    v[6] += (double)ld1(c);
    v[7] += (double)ld1(c + 1);
    v[8] += (double)ld1(c + 2);
    double qq[4];
    quat_from_gs<double>(v, qq);
    for (int j = 0; j < 9; ++j) pose[(size_t)r * 9 + j] = v[j];
    for (int j = 0; j < 4; ++j) q[(size_t)r * 7 + j] = qq[j];
    for (int j = 0; j < 3; ++j) q[(size_t)r * 7 + 4 + j] = v[6 + j];
}

extern "C" int gp_pose_epilogue_f64(double* pose, int rows, int k, const float* pts_center, double* q,
                                    hipStream_t stream) {
    GP_REQUIRE(pose && pts_center && q && rows >= 0 && k >= 1, "pose_epilogue_f64: bad arguments");
    if (!rows) return GP_OK;
    hipLaunchKernelGGL(pose_epilogue_f64_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, pose, rows, k,
                       pts_center, q);
    return gp_check_launch("pose_epilogue_f64_kernel");
}

// ============================================================================ ScaleNet
// ScaleNet.forward (scalenet.py:33-49) with encode_axes (genpose_utils.py:8-18). 0.88 MFLOP per
// object: one workgroup per object, VALU dot products.
__global__ __launch_bounds__(HT) void scale_kernel(gp_scale_weights w, const float* __restrict__ axes,
                                                   const float* __restrict__ feat, float* __restrict__ len) {
    __shared__ float emb[180];
    __shared__ float h1[256];
    __shared__ float tot[1280];
    __shared__ float u[256];
    const int b = blockIdx.x, i = threadIdx.x;
    if (i < 90) {  // embedding[(fn, a, e)] = fn(2^e * axes[a]), a<9, e<10
        const int a = i / 10, e = i - a * 10;
        const float v = fmul((float)(1 << e), axes[(size_t)b * 9 + a]);
        emb[i] = sinf(v);
        emb[90 + i] = cosf(v);
    }
    for (int c = i; c < 1024; c += HT) tot[c] = feat[(size_t)b * 1024 + c];
    __syncthreads();
    {
        float acc = 0.f;
        for (int c = 0; c < 180; ++c) acc += w.ae0_w[i * 180 + c] * emb[c];
        h1[i] = fmaxf(acc + w.ae0_b[i], 0.f);
    }
    __syncthreads();
    {
        float acc = 0.f;
        for (int c = 0; c < 256; ++c) acc += w.ae2_w[i * 256 + c] * h1[c];
        tot[1024 + i] = fmaxf(acc + w.ae2_b[i], 0.f);
    }
    __syncthreads();
    {
        float acc = 0.f;
        for (int c = 0; c < 1280; ++c) acc += w.ft0_w[(size_t)i * 1280 + c] * tot[c];
        u[i] = fmaxf(acc + w.ft0_b[i], 0.f);
    }
    __syncthreads();
    if (i < 3) {
        float acc = 0.f;
        for (int c = 0; c < 256; ++c) acc += w.ft2_w[i * 256 + c] * u[c];
        len[(size_t)b * 3 + i] = acc + w.ft2_b[i];
    }
}

extern "C" int gp_scale_forward(const gp_scale_weights* w, const float* axes, const float* pts_feat, int b,
                                float* length, hipStream_t stream) {
    GP_REQUIRE(w && axes && pts_feat && length && b >= 0, "scale_forward: bad arguments");
    if (!b) return GP_OK;
    hipLaunchKernelGGL(scale_kernel, dim3(b), dim3(HT), 0, stream, *w, axes, pts_feat, length);
    return gp_check_launch("scale_kernel");
}
