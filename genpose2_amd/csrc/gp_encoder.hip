// PointNet++ MSG set-abstraction encoder for gfx950 (Pointnet2ClsMSG(0), Light config:
// networks/pts_encoder/pointnet2.py:77-89, 211-252; SA module pointnet2_modules.py:19-124).
//
// The reference materialises every grouped tensor (B, 3+C, M, ns) in HBM (group_points_gpu.cu)
// and runs each 1x1 conv + BN + ReLU as a separate cuDNN call, then max-pools. Here one kernel
// per (level, branch) does gather -> 2-3 BN-folded layers -> ReLU -> max-pool with the grouped
// tile never leaving the CU:
//   * grouped rows are MFMA columns (16 per column tile), output channels are MFMA rows, so
//     the weights are the streamed A operand (packed once by genpose2_amd/pack.py into the
//     exact per-lane fragment order: one 1 KiB coalesced load feeds 4 MFMAs per column tile);
//   * layer-0 B fragments are gathered straight from the previous level's point-major
//     features (one float4 = 4 channels of one neighbour per lane) with the relative xyz as the
//     last k-group (input channels are permuted [feats | xyz | pad] so feature float4s align);
//   * inter-layer activations live in LDS in the MFMA accumulator's native layout, so a layer
//     writes and the next reads 1 KiB per wave-instruction, linear and conflict-free;
//   * the max over nsample is taken on the accumulators with 16-lane shuffles.
// Exact f32 MFMA (v_mfma_f32_16x16x4_f32): no precision is traded.
#include <algorithm>

#include "gp_common.h"
#include "gp_fps.h"
#include "gp_head.h"   // split-f16 helpers: mfma_h, split_pair, stream_hk_step, rows_max, exp2i, ilog2f

int gp_launch_fps_chain(const float* xyz, int b, int nlev, const int* n, const int* m, int* const* idx,
                        float* const* nxyz, hipStream_t st);
int gp_launch_ball_query2(int b, int n, int m, float ra, float rb, int nsa, int nsb, const float* new_xyz,
                          const float* xyz, int* idxa, int* idxb, hipStream_t st);

struct SAArgs {
    int n_prev, c_prev, m, ns, cols;  // cols = columns per object (m*ns, or n_prev for group-all)
    const float* xyz_prev;            // (B, n_prev, 3)
    const float* feat_prev;           // (B, n_prev, c_prev) or null
    const float* cent;                // (B, m, 3) or null (group-all: raw xyz)
    const int* nbr;                   // (B, m, ns) or null (group-all)
    int nlayers;
    const float* w[3];
    const float* bias[3];
    int kg[3];                        // k-groups (k_pad / 16)
    int nt[3];                        // output tiles (n_pad / 16)
    float* out;                       // (B, m, c_out_total)
    int c_out_total, out_off;
    int buf1_off;                     // float4 offset of the second LDS buffer
    int tag;                          // level * 2 + branch (tuning traces)
    // layer 0 by per-point projection (levels 0-3): h0(c, s) = relu(Q[nbr] - W0_xyz . x_c), where
    // Q[p] = W0_feat . f_p + W0_xyz . x_p + b0 was computed once per point by proj_kernel
    const float* qin;                 // (B, n_prev, q_stride) or null -> layer 0 by MFMA
    int q_stride, q_off;
    float* proj_out;                  // proj_kernel: Q output (B, n_prev, q_stride) at q_off
};

// Per-wave layer timestamps for tuning builds only (make EXTRA=-DSA_TRACE; scripts/sa_trace.py).
#ifdef SA_TRACE
__device__ unsigned long long g_sa_trace[8192 * 4 * 8];
__device__ int g_sa_trace_sel = -1;
#define SA_MARK(k)                                                                                         \
    do {                                                                                                   \
        const int wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                               \
        if (a.tag == g_sa_trace_sel && (threadIdx.x & 63) == 0 && wg_ < 8192)                              \
            g_sa_trace[(wg_ * 4 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime();          \
    } while (0)
extern "C" int gp_debug_sa_trace(int sel, unsigned long long* host) {
    if (host) return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sa_trace), sizeof(g_sa_trace)) == hipSuccess ? 0 : -1;
    void* ptr = nullptr;
    if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(g_sa_trace)) != hipSuccess || hipMemset(ptr, 0, sizeof(g_sa_trace)) != hipSuccess)
        return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sa_trace_sel), &sel, sizeof(int)) == hipSuccess ? 0 : -1;
}
// split-f16 levels (8 waves per workgroup): marks 0 start, 1 staged + barrier, 2 layer-0 gather + barrier,
// 3 layer-1 stream done, 4 column-max barrier, 5 layer-1 planes written, 6 layer-2 barrier, 7 end
__device__ unsigned long long g_split_trace[8192 * 8 * 8];
__device__ int g_split_trace_sel = -1;
#define SPLIT_MARK(a, k)                                                                                   \
    do {                                                                                                   \
        const int wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                               \
        if ((a).tag == g_split_trace_sel && (threadIdx.x & 63) == 0 && wg_ < 8192)                         \
            g_split_trace[(wg_ * 8 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime();       \
    } while (0)
extern "C" int gp_debug_split_trace(int sel, unsigned long long* host) {
    if (host) return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_split_trace), sizeof(g_split_trace)) == hipSuccess ? 0 : -1;
    void* ptr = nullptr;
    if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(g_split_trace)) != hipSuccess || hipMemset(ptr, 0, sizeof(g_split_trace)) != hipSuccess)
        return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_split_trace_sel), &sel, sizeof(int)) == hipSuccess ? 0 : -1;
}
#else
#define SA_MARK(k) ((void)0)
#define SPLIT_MARK(a, k) ((void)0)
#endif

constexpr int SA_THREADS = 256;
#ifndef SA_RING
#define SA_RING 2        // k-groups of operands in flight + 1
#endif

// One layer for the CTW column tiles [cbase, cbase+CTW) of this wave and the output tiles
// wt*TC, wt*TC + WT*TC, ... (WT = waves sharing the columns). Layers narrower than 4*TC output
// tiles split the workgroup's columns over waves instead of leaving waves idle.
template <int CT, int CTW, int TC, int SPAN>
__device__ __forceinline__ void sa_layer(const SAArgs& a, f32x4* lds, int L, int b, int col0, int cbase,
                                         int wt, int WT, int ibeg, int iend) {
    const int lane = threadIdx.x & 63;
    const int q = lane >> 4, nn = lane & 15;
    const int KG = a.kg[L], NT = a.nt[L];
    const int voff = lane * 16;
    const int tpc = a.ns >> 4;
    const __amdgpu_buffer_rsrc_t W = make_rsrc(a.w[L], (uint32_t)(NT * KG) * 1024u);
    const f32x4* in_lds = (L == 1) ? lds : lds + a.buf1_off;   // L>=1 reads buffer (L-1)&1
    f32x4* out_lds = (L == 0) ? lds : lds + a.buf1_off;         // L<last writes buffer L&1
    const bool last = (L == a.nlayers - 1);
    const int feat_groups = a.c_prev >> 4;

    // layer 0: per-lane gathered neighbour of each of this wave's column tiles + xyz fragment
    int pi[CTW];
    bool valid[CTW];
    f32x4 bx[CTW];
    if (L == 0) {
#pragma unroll
        for (int c = 0; c < CTW; ++c) {
            const int col = col0 + (cbase + c) * 16 + nn;
            valid[c] = col < a.cols;
            const int m = col / a.ns, s = col - m * a.ns;
            int p = 0;
            if (valid[c]) p = a.nbr ? a.nbr[((size_t)b * a.m + m) * a.ns + s] : s;
            pi[c] = p;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (valid[c] && q == 0) {
                const float* px = a.xyz_prev + ((size_t)b * a.n_prev + p) * 3;
                if (a.cent) {  // grouped_xyz -= new_xyz (pointnet2_utils.py:281-282)
                    const float* cc = a.cent + ((size_t)b * a.m + m) * 3;
                    v = f32x4{fsub(ld1(px), ld1(cc)), fsub(ld1(px + 1), ld1(cc + 1)), fsub(ld1(px + 2), ld1(cc + 2)), 0.f};
                } else {       // GroupAll keeps raw xyz (pointnet2_utils.py:316-324)
                    v = f32x4{ld1(px), ld1(px + 1), ld1(px + 2), 0.f};
                }
            }
            bx[c] = v;
        }
    }
    // entries [ibeg, iend) of this wave's output tiles wt, wt+WT, wt+2WT, ... (round robin keeps
    // waves within one tile of each other), TC of them per pass
    for (int i0 = ibeg; i0 < iend; i0 += TC) {
        int Tt[TC];
#pragma unroll
        for (int t = 0; t < TC; ++t) Tt[t] = (i0 + t < iend) ? wt + (i0 + t) * WT : NT;   // NT = none
        f32x4 acc[TC][CTW];
#pragma unroll
        for (int t = 0; t < TC; ++t)
#pragma unroll
            for (int c = 0; c < CTW; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
        // operand fetch for k-group g: A = packed weights (buffer load, SGPR offset), B = the
        // gathered neighbour features (layer 0) or the previous layer in LDS
        auto fetch = [&](int g, f32x4 (&af)[TC], f32x4 (&bf)[CTW]) {
#pragma unroll
            for (int t = 0; t < TC; ++t)
                af[t] = (Tt[t] < NT) ? ldbuf4(W, voff, (Tt[t] * KG + g) * 1024) : f32x4{0.f, 0.f, 0.f, 0.f};
            if (L == 0) {
                if (g < feat_groups) {
#pragma unroll
                    for (int c = 0; c < CTW; ++c)
                        bf[c] = valid[c] ? ld4(a.feat_prev + ((size_t)b * a.n_prev + pi[c]) * a.c_prev + 16 * g + 4 * q)
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
                } else {
#pragma unroll
                    for (int c = 0; c < CTW; ++c) bf[c] = bx[c];
                }
            } else {
#pragma unroll
                for (int c = 0; c < CTW; ++c) bf[c] = in_lds[(g * CT + cbase + c) * 64 + lane];
            }
        };
        // k-step outermost so consecutive MFMAs use different accumulators
        auto compute = [&](const f32x4 (&af)[TC], const f32x4 (&bf)[CTW]) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int t = 0; t < TC; ++t)
#pragma unroll
                    for (int c = 0; c < CTW; ++c) acc[t][c] = mfma4(af[t][j], bf[c][j], acc[t][c]);
        };
        // SA_RING-slot ring: the operands of k-groups g+1 .. g+SA_RING-1 are in flight while g
        // computes; sched_barrier keeps the compiler from sinking the loads next to their MFMAs
        f32x4 ra[SA_RING][TC], rb[SA_RING][CTW];
#pragma unroll
        for (int u = 0; u < SA_RING - 1; ++u)
            if (u < KG) fetch(u, ra[u], rb[u]);
        for (int g = 0; g < KG; g += SA_RING) {
#pragma unroll
            for (int u = 0; u < SA_RING; ++u) {
                if (g + u < KG) {
                    if (g + u + SA_RING - 1 < KG)
                        fetch(g + u + SA_RING - 1, ra[(u + SA_RING - 1) % SA_RING], rb[(u + SA_RING - 1) % SA_RING]);
                    __builtin_amdgcn_sched_barrier(0);
                    compute(ra[u], rb[u]);
                }
            }
        }
#pragma unroll
        for (int t = 0; t < TC; ++t) {
            const int T = Tt[t];
            if (T >= NT) continue;
            const f32x4 bias = ld4(a.bias[L] + 16 * T + 4 * q);
            if (!last) {
#pragma unroll
                for (int c = 0; c < CTW; ++c) out_lds[(T * CT + cbase + c) * 64 + lane] = relu4(acc[t][c] + bias);
            } else if (a.proj_out) {   // per-point projection: pre-activation, point-major
#pragma unroll
                for (int c = 0; c < CTW; ++c) {
                    const int col = col0 + (cbase + c) * 16 + nn;
                    if (col < a.cols)
                        st4(a.proj_out + ((size_t)b * a.n_prev + col) * a.q_stride + a.q_off + 16 * T + 4 * q,
                            acc[t][c] + bias);
                }
            } else {
                // max over nsample: across the centroid's SPAN column tiles, then 16 lanes
#pragma unroll
                for (int cb = 0; cb < CTW; cb += SPAN) {
                    f32x4 v = relu4(acc[t][cb] + bias);
#pragma unroll
                    for (int u = 1; u < SPAN; ++u) {
                        const f32x4 w2 = relu4(acc[t][cb + u] + bias);
                        v = f32x4{__builtin_elementwise_maximum(v.x, w2.x), __builtin_elementwise_maximum(v.y, w2.y),
                                  __builtin_elementwise_maximum(v.z, w2.z), __builtin_elementwise_maximum(v.w, w2.w)};
                    }
                    v = row16_max4(v);
                    const int colc = col0 + (cbase + cb) * 16;
                    if (nn == 0 && colc < a.cols) {
                        const int m = colc / a.ns;
                        float* o = a.out + ((size_t)b * a.m + m) * a.c_out_total + a.out_off + 16 * T + 4 * q;
                        if (tpc <= SPAN) {
                            st4(o, v);
                        } else {  // centroid split over workgroups: post-ReLU values are >= 0
                            unsigned int* u = reinterpret_cast<unsigned int*>(o);
                            atomicMax(u + 0, __float_as_uint(v.x));
                            atomicMax(u + 1, __float_as_uint(v.y));
                            atomicMax(u + 2, __float_as_uint(v.z));
                            atomicMax(u + 3, __float_as_uint(v.w));
                        }
                    }
                }
            }
        }
    }
}

// Layer 0 from the per-point projection: for each (output tile, column tile) pair of the workgroup,
// h0 = relu(Q[nbr(col)] - W0_xyz . x_centroid) into LDS buffer 0 in the accumulator layout. The
// xyz weights are read from the packed layer-0 fragments (k-group c_prev/16, lanes 0..15).
template <int CT>
__device__ __forceinline__ void sa_gather0(const SAArgs& a, f32x4* lds, int b, int col0) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int q = lane >> 4, nn = lane & 15;
    const int NT0 = a.nt[0], KG0 = a.kg[0], gx = a.c_prev >> 4, H0p = NT0 * 16;
    const f32x4* w0 = reinterpret_cast<const f32x4*>(a.w[0]);
    // W0_xyz . x_c for this workgroup's centroids, once, into the (still unused) second buffer
    const int mfirst = col0 / a.ns;
    const int mlast = min((col0 + CT * 16 - 1) / a.ns, a.m - 1);
    float* cx = reinterpret_cast<float*>(lds + a.buf1_off);
    for (int e = tid; e < (mlast - mfirst + 1) * H0p; e += SA_THREADS) {
        const int c = e / H0p, ch = e - (e / H0p) * H0p;
        const float* cc = a.cent + ((size_t)b * a.m + mfirst + c) * 3;
        const f32x4 w = w0[((ch >> 4) * KG0 + gx) * 64 + (ch & 15)];   // W0[ch][c_prev + 0..2]
        cx[e] = (w.x * ld1(cc) + w.y * ld1(cc + 1)) + w.z * ld1(cc + 2);
    }
    int pcol[CT], mcol[CT];
    bool ok[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int col = col0 + ct * 16 + nn;
        ok[ct] = col < a.cols;
        const int m = ok[ct] ? col / a.ns : 0, s = ok[ct] ? col - (col / a.ns) * a.ns : 0;
        mcol[ct] = m - mfirst;
        pcol[ct] = ok[ct] ? a.nbr[((size_t)b * a.m + m) * a.ns + s] : 0;
    }
    __syncthreads();
    // this wave's (output tile, column tile) pairs, 8 at a time: all Q gathers in flight first
    constexpr int PB = 8;
    for (int p0 = wid; p0 < NT0 * CT; p0 += 4 * PB) {
        f32x4 qv[PB];
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            const int pr = p0 + 4 * u;
            const int T = pr / CT, ct = pr - (pr / CT) * CT;
            qv[u] = (pr < NT0 * CT && ok[ct])
                        ? ld4(a.qin + ((size_t)b * a.n_prev + pcol[ct]) * a.q_stride + a.q_off + 16 * T + 4 * q)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            const int pr = p0 + 4 * u;
            if (pr >= NT0 * CT) break;
            const int T = pr / CT, ct = pr - (pr / CT) * CT;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (ok[ct]) {
                const f32x4 c4 = ld4(cx + mcol[ct] * H0p + 16 * T + 4 * q);
                v = relu4(qv[u] - c4);
            }
            lds[(T * CT + ct) * 64 + lane] = v;
        }
    }
}

// A layer in passes whose tile counts match the wave's tiles exactly (a pass of TC tiles computes
// all TC accumulators, so a short last pass would burn MFMAs on absent tiles).
template <int CT, int CTW, int SPAN, int MAXTC>
__device__ __forceinline__ void sa_layer_fit(const SAArgs& a, f32x4* lds, int L, int b, int col0, int cbase, int wt,
                                             int WT) {
    const int nt = a.nt[L];
    const int cnt = nt > wt ? (nt - wt + WT - 1) / WT : 0;
    if constexpr (MAXTC >= 8) {
        if (cnt == 8) return sa_layer<CT, CTW, 8, SPAN>(a, lds, L, b, col0, cbase, wt, WT, 0, cnt);
    }
    if constexpr (MAXTC >= 7) {
        if (cnt == 7) return sa_layer<CT, CTW, 7, SPAN>(a, lds, L, b, col0, cbase, wt, WT, 0, cnt);
    }
    if constexpr (MAXTC >= 6) {
        if (cnt == 6) return sa_layer<CT, CTW, 6, SPAN>(a, lds, L, b, col0, cbase, wt, WT, 0, cnt);
    }
    // passes of 4 tiles, then the remainder as one exact pass
    const int full = cnt & ~3, rem = cnt - full;
    if (full) sa_layer<CT, CTW, 4, SPAN>(a, lds, L, b, col0, cbase, wt, WT, 0, full);
    if (rem == 1) sa_layer<CT, CTW, 1, SPAN>(a, lds, L, b, col0, cbase, wt, WT, full, cnt);
    else if (rem == 2) sa_layer<CT, CTW, 2, SPAN>(a, lds, L, b, col0, cbase, wt, WT, full, cnt);
    else if (rem == 3) sa_layer<CT, CTW, 3, SPAN>(a, lds, L, b, col0, cbase, wt, WT, full, cnt);
}

template <int CT, int TC, int SPAN, int MAXTC>
__device__ __forceinline__ void sa_body(const SAArgs& a, f32x4* lds) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.y;
    const int col0 = blockIdx.x * CT * 16;
    SA_MARK(0);
    int L0 = 0;
    if (a.qin) {
        sa_gather0<CT>(a, lds, b, col0);
        SA_MARK(1);
        __syncthreads();
        SA_MARK(2);
        L0 = 1;
    }
    for (int L = L0; L < a.nlayers; ++L) {
        // waves over columns: 4 / (output tiles this layer can feed at TC per wave), kept >= the
        // pooling span on the last layer
        const int nt = a.nt[L];
        int wc = nt >= 4 * TC ? 1 : (nt > TC ? 2 : 4);
        if (wc > CT) wc = CT;
        if (L == a.nlayers - 1)
            while (wc > 1 && CT / wc < SPAN) wc >>= 1;
        const int wt = wid / wc, WT = 4 / wc;
        if (wc == 1) {
            sa_layer_fit<CT, CT, SPAN, MAXTC>(a, lds, L, b, col0, 0, wt, WT);
        } else if (wc == 2) {
            if constexpr (CT >= 2 && CT / 2 >= 1) sa_layer_fit<CT, CT / 2, (SPAN <= CT / 2 ? SPAN : 1), MAXTC>(
                a, lds, L, b, col0, (wid % 2) * (CT / 2), wt, WT);
        } else {
            if constexpr (CT >= 4) sa_layer_fit<CT, CT / 4, 1, MAXTC>(a, lds, L, b, col0, (wid % 4) * (CT / 4), wt, WT);
        }
        SA_MARK(1 + 2 * L);
        __syncthreads();
        SA_MARK(2 + 2 * L);
    }
}

// Both branches of a level (or both branch projections) in one launch: blockIdx.z = branch.
// Each branch keeps its own column count, layer widths and pooling span.
template <int CT, int SPAN0, int SPAN1, int MAXTC>
__global__ __launch_bounds__(SA_THREADS, 2) void sa_pair_kernel(SAArgs a0, SAArgs a1) {
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
    if (blockIdx.z == 0) {
        if ((int)blockIdx.x * CT * 16 < a0.cols) sa_body<CT, 4, SPAN0, MAXTC>(a0, lds);
    } else {
        if ((int)blockIdx.x * CT * 16 < a1.cols) sa_body<CT, 4, SPAN1, MAXTC>(a1, lds);
    }
}

// ============================================================================ split-f16 levels (2, 3)
// Layers 1 and 2 of a level as split-f16 MFMA GEMMs (v_mfma_f32_16x16x32_f16, three products of
// hi/lo planes with fp32 accumulation, as the head trunk): per 32-deep chunk w_lo*a_hi + w_hi*a_lo
// + w_hi*a_hi, ~22 significant bits per operand. The activation planes take a per-COLUMN power-of-two
// scale from the column's actual maximum (a column is one grouped neighbour: its scale multiplies
// out of every output of that column), so the split keeps ~22 bits wherever the values lie:
//   * layer 0 (relu(Q[nbr] - W0_xyz . x_c), the per-point projection) is gathered by waves 0..CT-1,
//     one 16-column tile each; the lane's values and a 4-lane max give the column maximum directly;
//   * layer 1's outputs are spread over the waves by output chunk: every wave publishes its partial
//     column maxima in LDS before the barrier that retires the reads of layer 0's planes, then
//     writes its chunks' planes over them (one activation buffer, no extra barrier).
// Weights carry a per-layer exponent (pack.pack_encoder). Wave w owns output chunks w, w+8, ...: the
// two waves sharing a SIMD (w, w+4) split a level-3 branch-1 layer 1's 12 chunks 2 + 1.
// 64 columns per workgroup: every weight fragment streamed from L2 feeds 4 column tiles x 3 MFMAs.
constexpr int SPLIT_WV = 8;

struct SplitArgs {
    int n_prev, m, ns, cols;          // cols = m * ns, a multiple of the workgroup's 16*CT columns
    const float* qin;                 // layer-0 projection Q (B, n_prev, q_stride), pre-activation
    int q_stride, q_off;
    const float* w0;                  // packed fp32 layer 0 (its xyz k-group gives W0_xyz)
    int kg0, gx;
    const int* nbr;                   // (B, m, ns)
    const float* cent;                // (B, m, 3)
    const float* w[2];                // split planes of layers 1, 2 (pack_h16_fragments)
    const float* bias[2];             // padded to 32
    int ew[2];                        // weight exponents
    float* out;                       // (B, m, c_out_total)
    int c_out_total, out_off;
    int tag;                          // level * 2 + branch (tuning traces)
};

// IEEE maximum (v_maximum3_f32: no quieting of non-canonical MFMA outputs first, three operands per
// instruction); equal to fmaxf for every non-NaN value
__device__ __forceinline__ float fmax2(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float max4(f32x4 v) { return fmax2(fmax2(fmax2(v.x, v.y), v.z), v.w); }
__device__ __forceinline__ f32x4 vmax4(f32x4 a, f32x4 b) {
    return f32x4{fmax2(a.x, b.x), fmax2(a.y, b.y), fmax2(a.z, b.z), fmax2(a.w, b.w)};
}
// Max-pooling before the bias and ReLU: x -> relu(x + b) is monotonic and rounding is monotonic, so
// relu(max_n x_n + b) equals max_n relu(x_n + b) bit for bit -- the pools take the max of the unscaled
// accumulators (scales are exact powers of two) and add the bias once per pooled output.
constexpr float NEG_BIG = -3.0e38f;

// Column exponent: E with the column maximum in [2^E, 2^(E+1)); all-zero columns get E = -100.
__device__ __forceinline__ int col_exponent(float m) { return m > 1e-30f ? ilog2f(m) : -100; }

// Layer-0 planes of column tile ct: lane (q, n) gathers column n's channels 32c + 4q + j and
// 32c + 16 + 4q + j (j < 4) of every chunk c -- exactly its B fragments.
// Neighbour index and centroid of lane column n of column tile ct: loaded at kernel entry, one round trip
// ahead of the layer-0 gather that depends on them.
__device__ __forceinline__ int split_gather0_pre(const SplitArgs& a, int b, int col0, int ct, int lane) {
    const int g = col0 + ct * 16 + (lane & 15);
    if (g >= a.cols) return 0;   // past the last centroid (ragged last workgroup)
    const int m = g / a.ns, s = g - (g / a.ns) * a.ns;
    return a.nbr[((size_t)b * a.m + m) * a.ns + s];
}

// The centroid term of layer 0, W0_xyz . x_c, for each of the workgroup's centroids and layer-0 channels
// (P[ci][ch], ci = the workgroup's ci-th centroid), computed once per workgroup: every column of a 16-column
// tile shares its centroid, so the gather reads it as one broadcast LDS read per 4 channels instead of
// recomputing it from (wx, wy, wz) in all 16 lanes. Same expression and order as before: bit-identical.
template <int CT, int KC0>
__device__ __forceinline__ void split_centroid_term(const SplitArgs& a, float* P, int b, int col0, int tid) {
#pragma clang fp contract(off)
    const int nci = 16 * CT / a.ns, mi0 = col0 / a.ns;
    for (int idx = tid; idx < nci * KC0 * 32; idx += SPLIT_WV * 64) {
        const int ci = idx / (KC0 * 32), ch = idx - ci * (KC0 * 32);
        const int mi = min(mi0 + ci, a.m - 1);   // past the last centroid: any value (never stored)
        const float* cc = a.cent + ((size_t)b * a.m + mi) * 3;
        const f32x4 w = ld4(a.w0 + ((size_t)((ch >> 4) * a.kg0 + a.gx) * 64 + (ch & 15)) * 4);
        P[idx] = (w.x * ld1(cc) + w.y * ld1(cc + 1)) + w.z * ld1(cc + 2);
    }
}

// The lane's layer-0 projection row of its neighbour (the gathered Q values of chunk c, half h),
// loaded at kernel entry so the loads overlap the centroid-term staging and its barrier.
template <int KC0>
__device__ __forceinline__ void split_gather0_load(const SplitArgs& a, int b, int p, int lane, f32x4 (&v)[KC0][2]) {
    const float* qrow = a.qin + ((size_t)b * a.n_prev + p) * a.q_stride + a.q_off + 4 * (lane >> 4);
#pragma unroll
    for (int c = 0; c < KC0; ++c) {
        v[c][0] = ld4(qrow + 32 * c);
        v[c][1] = ld4(qrow + 32 * c + 16);
    }
}

template <int CT, int KC0>
__device__ __forceinline__ void split_gather0(const SplitArgs& a, f16x8* X, int* e0s, const f32x4* P4, int col0,
                                              int ct, int lane, f32x4 (&v)[KC0][2]) {
#pragma clang fp contract(off)
    const int q = lane >> 4, n = lane & 15;
    const int col = ct * 16 + n;
    const int ci = (col0 + ct * 16) / a.ns - col0 / a.ns;   // the tile's centroid within the workgroup
    const f32x4* pc = P4 + ci * KC0 * 8 + q;                 // channels 32 c + 16 h + 4 q .. + 3: pc[8 c + 4 h]
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < KC0; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float r[4];
            const f32x4 t = pc[8 * c + 4 * h];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                r[j] = relu1(v[c][h][j] - t[j]);
                mx = fmax2(mx, r[j]);
            }
            v[c][h] = f32x4{r[0], r[1], r[2], r[3]};
        }
    const int E = col_exponent(rows_max(mx));
    const float sc = exp2i(14 - E);
#pragma unroll
    for (int c = 0; c < KC0; ++c) {
        f16x8 hi, lo;
        split_pair(v[c][0], v[c][1], sc, hi, lo);
        X[((c * CT + ct) * 2 + 0) * 64 + lane] = hi;
        X[((c * CT + ct) * 2 + 1) * 64 + lane] = lo;
    }
    if (q == 0) e0s[col] = E;
}

// Layer 1 for this wave's NC output chunks (wid, wid + 8, ...): primes its weight ring, gathers layer
// 0 (waves < CT), streams, and leaves the planes of its outputs in X (over layer 0's) plus every
// column's exponent in e1[ct] (for lane column n). Executes the same two barriers in every wave.
template <int CT, int KC0, int NC, int D>
__device__ __forceinline__ void split_layer1(const SplitArgs& a, f16x8* X, int* e0s, float* pm, const f32x4* P4,
                                             int b, int col0, int wid, int lane, int oc1, int (&e1)[CT],
                                             f32x4 (&gq)[KC0][2], bool loaded, int pnb) {
    const int q = lane >> 4, n = lane & 15;
    float pmax[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) pmax[ct] = 0.f;
    if constexpr (NC == 0) {
        if (wid < CT) {
            if (!loaded) split_gather0_load<KC0>(a, b, pnb, lane, gq);
            split_gather0<CT, KC0>(a, X, e0s, P4, col0, wid, lane, gq);
        }
        __syncthreads();
        if (q == 0)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) pm[(ct * 16 + n) * SPLIT_WV + wid] = 0.f;
        __syncthreads();
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            float M = 0.f;
            {   // the column's SPLIT_WV wave partials, column-major: two 16-byte reads
                const f32x4 p0 = ld4(&pm[(ct * 16 + n) * SPLIT_WV]), p1 = ld4(&pm[(ct * 16 + n) * SPLIT_WV + 4]);
                const float pw[SPLIT_WV] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
                for (int w = 0; w < SPLIT_WV; ++w) M = fmaxf(M, pw[w]);
            }
            e1[ct] = col_exponent(M);
        }
    } else {
        int T[2 * NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            T[2 * i] = 2 * (wid + SPLIT_WV * i);
            T[2 * i + 1] = T[2 * i] + 1;
        }
        const __amdgpu_buffer_rsrc_t W = make_rsrc(a.w[0], (uint32_t)(2 * oc1) * KC0 * 2048u);
        const int voff = lane * 16;
        f16x8 ring[D + 1][2 * NC][2];
        f32x4 acc[2 * NC][CT];
#pragma unroll
        for (int t = 0; t < 2 * NC; ++t)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        stream_hk_step<KC0, 0, D, 2 * NC, CT, D>(W, T, X, lane, voff, ring, acc);
        if (wid < CT) {
            if (!loaded) split_gather0_load<KC0>(a, b, pnb, lane, gq);
            split_gather0<CT, KC0>(a, X, e0s, P4, col0, wid, lane, gq);
        }
        __syncthreads();
        SPLIT_MARK(a, 2);
        stream_hk_step<KC0, D, KC0 + D, 2 * NC, CT, D>(W, T, X, lane, voff, ring, acc);
        SPLIT_MARK(a, 3);
        // unscale (exact powers of two), bias, ReLU, partial column maxima
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const float u = exp2i(e0s[ct * 16 + n] - 14 - a.ew[0]);
#pragma unroll
            for (int t = 0; t < 2 * NC; ++t) {
                acc[t][ct] = relu4(acc[t][ct] * u + ld4(a.bias[0] + 16 * T[t] + 4 * q));
                pmax[ct] = fmax2(pmax[ct], max4(acc[t][ct]));
            }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const float M = rows_max(pmax[ct]);
            if (q == 0) pm[(ct * 16 + n) * SPLIT_WV + wid] = M;
        }
        __syncthreads();   // every read of layer 0's planes is done; the partial maxima are visible
        SPLIT_MARK(a, 4);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            float M = 0.f;
            {   // the column's SPLIT_WV wave partials, column-major: two 16-byte reads
                const f32x4 p0 = ld4(&pm[(ct * 16 + n) * SPLIT_WV]), p1 = ld4(&pm[(ct * 16 + n) * SPLIT_WV + 4]);
                const float pw[SPLIT_WV] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
                for (int w = 0; w < SPLIT_WV; ++w) M = fmaxf(M, pw[w]);
            }
            e1[ct] = col_exponent(M);
            const float sc = exp2i(14 - e1[ct]);
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int oc = wid + SPLIT_WV * i;
                f16x8 hi, lo;
                split_pair(acc[2 * i][ct], acc[2 * i + 1][ct], sc, hi, lo);
                X[((oc * CT + ct) * 2 + 0) * 64 + lane] = hi;
                X[((oc * CT + ct) * 2 + 1) * 64 + lane] = lo;
            }
        }
        SPLIT_MARK(a, 5);
    }
}

// Layer 2 for this wave's NC output chunks, ReLU, and the max over each centroid's ns columns
// (ns = 16: one column tile, 32: two) written to the level's point-major output.
template <int CT, int KC1, int NC, int D>
__device__ __forceinline__ void split_layer2(const SplitArgs& a, const f16x8* X, const int (&e1)[CT], int b,
                                             int col0, int wid, int lane, int oc2) {
    static_assert(NC >= 1, "every wave owns a layer-2 chunk");
    const int q = lane >> 4, n = lane & 15;
    int T[2 * NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        T[2 * i] = 2 * (wid + SPLIT_WV * i);
        T[2 * i + 1] = T[2 * i] + 1;
    }
    const __amdgpu_buffer_rsrc_t W = make_rsrc(a.w[1], (uint32_t)(2 * oc2) * KC1 * 2048u);
    const int voff = lane * 16;
    f16x8 ring[D + 1][2 * NC][2];
    f32x4 acc[2 * NC][CT];
#pragma unroll
    for (int t = 0; t < 2 * NC; ++t)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    stream_hk_step<KC1, 0, D, 2 * NC, CT, D>(W, T, X, lane, voff, ring, acc);
    __syncthreads();   // layer 1's planes are complete
    SPLIT_MARK(a, 6);
    stream_hk_step<KC1, D, KC1 + D, 2 * NC, CT, D>(W, T, X, lane, voff, ring, acc);
    const int span = a.ns >> 4;   // column tiles per centroid (1 or 2)
#pragma unroll
    for (int t = 0; t < 2 * NC; ++t) {
        const f32x4 bias = ld4(a.bias[1] + 16 * T[t] + 4 * q);
        f32x4 v[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) v[ct] = relu4(acc[t][ct] * exp2i(e1[ct] - 14 - a.ew[1]) + bias);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            if (span == 2) {
                if (ct & 1) continue;
                v[ct] = vmax4(v[ct], v[ct + 1]);
            }
            const float r = row16_max_scatter4(v[ct], n);   // channel 16 T[t] + 4 q + (n >> 2)
            const int mi = (col0 + ct * 16) / a.ns;
            if ((n & 3) == 0 && mi < a.m) a.out[((size_t)b * a.m + mi) * a.c_out_total + a.out_off + 16 * T[t] + 4 * q + (n >> 2)] = r;
        }
    }
}

template <int CT, int D, int KC0, int OC1, int OC2>
__device__ __forceinline__ void sa_split_body(const SplitArgs& a, char* smem) {
    constexpr int C = 16 * CT, KX = KC0 > OC1 ? KC0 : OC1;
    f16x8* X = reinterpret_cast<f16x8*>(smem);                       // [chunk][ct][plane][lane]
    float* P = reinterpret_cast<float*>(smem + (size_t)KX * CT * 2048);   // [centroid][channel] W0_xyz . x_c
    float* pm = P + CT * KC0 * 32;                                   // [column][wave] partial maxima
    int* e0s = reinterpret_cast<int*>(pm + SPLIT_WV * C);           // layer-0 column exponents
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.y, col0 = blockIdx.x * C;
    SPLIT_MARK(a, 0);
    // level 3 (256-wide layer 0): the gather's loads go out before the centroid-term barrier; level 2
    // issues them after it (its 64 registers would not fit the 128 of two workgroups per CU)
    constexpr bool EARLY = KC0 >= 8;
    f32x4 gq[KC0][2];
    const int pnb = wid < CT ? split_gather0_pre(a, b, col0, wid, lane) : 0;
    split_centroid_term<CT, KC0>(a, P, b, col0, tid);
    // after the centroid terms' loads (vmcnt counts in order: issued before them, the gather loads would
    // be waited for there)
    if (EARLY && wid < CT) split_gather0_load<KC0>(a, b, pnb, lane, gq);
    if constexpr (EARLY) {
        // LDS-only barrier: the centroid terms' stores are complete (lgkmcnt), the gather loads stay in
        // flight across it (__syncthreads would wait for them: vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
        __syncthreads();
    }
    SPLIT_MARK(a, 1);
    int e1[CT];
    // layer-1 output chunks of this wave: wid, wid + 8, ... below OC1
    constexpr int NC1_HI = (OC1 + SPLIT_WV - 1) / SPLIT_WV;
    const int nc1 = wid < OC1 % SPLIT_WV || OC1 % SPLIT_WV == 0 ? NC1_HI : NC1_HI - 1;
    if (nc1 == NC1_HI)
        split_layer1<CT, KC0, NC1_HI, D>(a, X, e0s, pm, reinterpret_cast<const f32x4*>(P), b, col0, wid, lane, OC1, e1, gq, EARLY, pnb);
    else
        split_layer1<CT, KC0, (NC1_HI > 0 ? NC1_HI - 1 : 0), D>(a, X, e0s, pm, reinterpret_cast<const f32x4*>(P), b, col0, wid, lane, OC1, e1, gq, EARLY, pnb);
    static_assert(OC2 % SPLIT_WV == 0, "layer-2 chunks spread evenly over the waves");
    split_layer2<CT, OC1, OC2 / SPLIT_WV, D>(a, X, e1, b, col0, wid, lane, OC2);
    SPLIT_MARK(a, 7);
}

// Both branches of a level per launch (blockIdx.z = branch).
// CT column tiles per workgroup (whole centroids; the last workgroup of a branch may be ragged), D
// 32-deep weight chunks in flight per layer.
// MINB: workgroups per CU the register budget is held to (2 at level 2, whose LDS fits two: 128 VGPRs).
template <int CT, int D, int KC0, int OC1A, int OC2A, int OC1B, int OC2B, int MINB = 1>
__global__ __launch_bounds__(SPLIT_WV * 64) __attribute__((amdgpu_waves_per_eu(2 * MINB))) void sa_split_kernel(SplitArgs a0, SplitArgs a1) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (blockIdx.z == 0) {
        if ((int)blockIdx.x * 16 * CT < a0.cols) sa_split_body<CT, D, KC0, OC1A, OC2A>(a0, smem);
    } else {
        if ((int)blockIdx.x * 16 * CT < a1.cols) sa_split_body<CT, D, KC0, OC1B, OC2B>(a1, smem);
    }
}

// Column tiles per workgroup at levels 2 / 3 and the weight ring depth. Level 3 (101 KB of LDS at 4
// tiles: one workgroup per CU either way) takes 6 tiles, the most LDS holds: every weight fragment
// streamed from L2 then feeds 6 column tiles (1.69 -> 1.31 ms at B=256). Level 2 keeps 4 tiles, two
// workgroups per CU whose gather and barrier phases overlap each other's streams (8 tiles: 0.87 ->
// 1.40 ms).
#ifndef SPLIT_CT2
#define SPLIT_CT2 4
#endif
#ifndef SPLIT_CT3
#define SPLIT_CT3 6
#endif
#ifndef SPLIT_D2
#define SPLIT_D2 2
#endif
#ifndef SPLIT_D3
#define SPLIT_D3 2
#endif

template <int CT, int KC0, int OC1>
static size_t sa_split_lds() {
    constexpr int KX = KC0 > OC1 ? KC0 : OC1;
    return (size_t)KX * CT * 2048 + sizeof(float) * CT * KC0 * 32 + sizeof(float) * SPLIT_WV * 16 * CT + sizeof(int) * 16 * CT;
}

// ============================================================================ narrow levels
// Levels 0 and 1 (layers <= 128 wide): every wave owns whole centroids and runs layer 1, layer 2
// and the max-pool for them entirely in registers -- the accumulator of one layer is the next
// layer's B operand as is, so there is no LDS round trip and no barrier after the weights are
// staged. Layer 0 comes from the per-point projection (relu(Q[nbr] - W0_xyz . x_c)).
struct NarrowArgs {
    const float* qin;      // (B, n_prev, q_stride)
    int q_stride, q_off, n_prev;
    const float* w0;       // packed layer 0 (for its xyz columns), KG0 k-groups
    int kg0, gx;           // k-groups of layer 0, index of its xyz k-group
    const float* w1;       // packed layer 1 / 2 and biases
    const float* b1;
    const float* w2;
    const float* b2;
    const int* nbr;        // (B, m, ns)
    const float* cent;     // (B, m, 3)
    int m, ns, nobj;
    float* out;            // (B, m, c_out_total)
    int c_out_total, out_off;
    const float* w1h;      // split-f16 planes of layers 1 / 2 (sa_narrow_split_kernel) and their exponents
    const float* w2h;
    int ew1, ew2;
};

// A centroid's gathered layer-0 projections (SPAN column tiles x KG k-groups) and its coordinates.
// The task loops run a two-stage software pipeline over a wave's centroids: the neighbour indices
// of centroid i+2 and the projection rows of centroid i+1 are in flight while centroid i computes,
// so the dependent index -> row round trips leave the critical path.
template <int SPAN, int KG>
struct NarrowGather {
    f32x4 q[SPAN][KG];
    float cx, cy, cz;
};

template <int SPAN>
__device__ __forceinline__ void narrow_nbr(const NarrowArgs& a, int task, int nn, int (&p)[SPAN]) {
#pragma unroll
    for (int ct = 0; ct < SPAN; ++ct) p[ct] = a.nbr[(size_t)task * a.ns + ct * 16 + nn];
}

// W0_xyz . x_c for the lane's layer-0 channels 16g + 4q + j: the same for every column of a centroid
template <int KG>
__device__ __forceinline__ const f32x4* narrow_centroid_term(const f32x4* sW0x, int q, float cx, float cy, float cz,
                                                             f32x4 (&cw)[KG]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int g = 0; g < KG; ++g) {
        float r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f32x4 wx = sW0x[16 * g + 4 * q + j];
            r[j] = (wx.x * cx + wx.y * cy) + wx.z * cz;
        }
        cw[g] = f32x4{r[0], r[1], r[2], r[3]};
    }
    return cw;
}

template <int SPAN, int KG>
__device__ __forceinline__ void narrow_fetch(const NarrowArgs& a, int task, const int (&p)[SPAN], int q,
                                             NarrowGather<SPAN, KG>& g) {
    const int b = task / a.m;
    const float* cc = a.cent + (size_t)task * 3;
    g.cx = ld1(cc);
    g.cy = ld1(cc + 1);
    g.cz = ld1(cc + 2);
#pragma unroll
    for (int ct = 0; ct < SPAN; ++ct) {
        const float* qrow = a.qin + ((size_t)b * a.n_prev + p[ct]) * a.q_stride + a.q_off + 4 * q;
#pragma unroll
        for (int g2 = 0; g2 < KG; ++g2) g.q[ct][g2] = ld4(qrow + 16 * g2);
    }
}

template <int KG1, int NT1, int NT2, int SPAN>
__device__ __forceinline__ void narrow_branch(const NarrowArgs& a, f32x4* lds) {
    constexpr int KG2 = NT1;
    constexpr int NA1 = NT1 * KG1 * 64, NA2 = NT2 * KG2 * 64;
    f32x4* sA1 = lds;
    f32x4* sA2 = sA1 + NA1;
    f32x4* sW0x = sA2 + NA2;              // [KG1*16] (wx, wy, wz, 0) per layer-0 output channel
    float* sB1 = reinterpret_cast<float*>(sW0x + KG1 * 16);
    float* sB2 = sB1 + NT1 * 16;
    const int tid = threadIdx.x;
    for (int i = tid; i < NA1; i += SA_THREADS) sA1[i] = ld4(a.w1 + (size_t)i * 4);
    for (int i = tid; i < NA2; i += SA_THREADS) sA2[i] = ld4(a.w2 + (size_t)i * 4);
    for (int ch = tid; ch < KG1 * 16; ch += SA_THREADS)   // packed layer-0 fragment of channel ch, q = 0
        sW0x[ch] = ld4(a.w0 + ((size_t)((ch >> 4) * a.kg0 + a.gx) * 64 + (ch & 15)) * 4);
    for (int i = tid; i < NT1 * 16; i += SA_THREADS) sB1[i] = a.b1[i];
    for (int i = tid; i < NT2 * 16; i += SA_THREADS) sB2[i] = a.b2[i];
    __syncthreads();
    const int lane = tid & 63, q = lane >> 4, nn = lane & 15;
    const int nw = gridDim.x * (SA_THREADS / 64);
    const int total = a.nobj * a.m;
    int task = blockIdx.x * (SA_THREADS / 64) + (tid >> 6);
    if (task >= total) return;
    int pn[SPAN];
    NarrowGather<SPAN, KG1> cur, nxt;
    f32x4 cwv[KG1];
    narrow_nbr<SPAN>(a, task, nn, pn);
    narrow_fetch<SPAN, KG1>(a, task, pn, q, cur);
    if (task + nw < total) narrow_nbr<SPAN>(a, task + nw, nn, pn);
    for (; task < total; task += nw) {
        if (task + nw < total) {
            narrow_fetch<SPAN, KG1>(a, task + nw, pn, q, nxt);
            if (task + 2 * nw < total) narrow_nbr<SPAN>(a, task + 2 * nw, nn, pn);
        }
        const float cx = cur.cx, cy = cur.cy, cz = cur.cz;
        f32x4 rmax[NT2];
#pragma unroll
        for (int t = 0; t < NT2; ++t) rmax[t] = f32x4{NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};   // pre-bias maxima
        const f32x4* cw = narrow_centroid_term<KG1>(sW0x, q, cx, cy, cz, cwv);
#pragma unroll
        for (int ct = 0; ct < SPAN; ++ct) {
            f32x4 bf[KG1];
#pragma unroll
            for (int g = 0; g < KG1; ++g) {
                float r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) r[j] = relu1(fsub(cur.q[ct][g][j], cw[g][j]));
                bf[g] = f32x4{r[0], r[1], r[2], r[3]};
            }
            f32x4 acc1[NT1];
#pragma unroll
            for (int t = 0; t < NT1; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < KG1; ++g) {
                f32x4 af[NT1];
#pragma unroll
                for (int t = 0; t < NT1; ++t) af[t] = sA1[(t * KG1 + g) * 64 + lane];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int t = 0; t < NT1; ++t) acc1[t] = mfma4(af[t][j], bf[g][j], acc1[t]);
                __builtin_amdgcn_sched_barrier(0);   // bound the live A fragments to one k-group
            }
#pragma unroll
            for (int t = 0; t < NT1; ++t) acc1[t] = relu4(acc1[t] + ld4(&sB1[16 * t + 4 * q]));
            f32x4 acc2[NT2];
#pragma unroll
            for (int t = 0; t < NT2; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < KG2; ++g) {
                f32x4 af[NT2];
#pragma unroll
                for (int t = 0; t < NT2; ++t) af[t] = sA2[(t * KG2 + g) * 64 + lane];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int t = 0; t < NT2; ++t) acc2[t] = mfma4(af[t][j], acc1[g][j], acc2[t]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int t = 0; t < NT2; ++t) rmax[t] = vmax4(rmax[t], acc2[t]);
            __builtin_amdgcn_sched_barrier(0);
        }
        float* o = a.out + (size_t)task * a.c_out_total + a.out_off + 4 * q;
#pragma unroll
        for (int t = 0; t < NT2; ++t) {
            const int j = nn >> 2;   // row16_max_scatter4 leaves channel 16 t + 4 q + j in this quad
            const float r = relu1(row16_max_scatter4(rmax[t], nn) + sB2[16 * t + 4 * q + j]);
            if ((nn & 3) == 0) o[16 * t + j] = r;
        }
        cur = nxt;
    }
}

// Narrow level with layers 1-2 as split-f16 MFMA (v_mfma_f32_16x16x32_f16, three products of hi/lo
// planes, fp32 accumulation, as sa_split_kernel) and per-column power-of-two activation scaling. A
// column's values sit in the four lanes (q, n) of its column index n, so the column maximum is a 4-lane
// max of registers: layer 0's from the gathered projection, layer 1's from its accumulators. The
// accumulator tiles 2c, 2c+1 of one layer are chunk c of the next layer's B operand as is, so the
// activations never leave registers. KC0 = 32-deep chunks of layer 0's output (its width / 32).
template <int KC0, int NT1, int NT2, int SPAN>
__device__ __forceinline__ void narrow_branch_split(const NarrowArgs& a, f32x4* lds) {
    constexpr int KG1 = 2 * KC0, KC1 = NT1 / 2;
    static_assert(NT1 % 2 == 0, "layer-1 tiles pair into 32-deep chunks");
    constexpr int NA1 = NT1 * KC0 * 2 * 64, NA2 = NT2 * KC1 * 2 * 64;   // f16x8 fragments
    f16x8* sA1 = reinterpret_cast<f16x8*>(lds);
    f16x8* sA2 = sA1 + NA1;
    f32x4* sW0x = reinterpret_cast<f32x4*>(sA2 + NA2);
    float* sB1 = reinterpret_cast<float*>(sW0x + KG1 * 16);
    float* sB2 = sB1 + NT1 * 16;
    const int tid = threadIdx.x;
    for (int i = tid; i < NA1; i += SA_THREADS) sA1[i] = __builtin_bit_cast(f16x8, ld4(a.w1h + (size_t)i * 4));
    for (int i = tid; i < NA2; i += SA_THREADS) sA2[i] = __builtin_bit_cast(f16x8, ld4(a.w2h + (size_t)i * 4));
    for (int ch = tid; ch < KG1 * 16; ch += SA_THREADS)
        sW0x[ch] = ld4(a.w0 + ((size_t)((ch >> 4) * a.kg0 + a.gx) * 64 + (ch & 15)) * 4);
    for (int i = tid; i < NT1 * 16; i += SA_THREADS) sB1[i] = a.b1[i];
    for (int i = tid; i < NT2 * 16; i += SA_THREADS) sB2[i] = a.b2[i];
    __syncthreads();
    const int lane = tid & 63, q = lane >> 4, nn = lane & 15;
    const int nw = gridDim.x * (SA_THREADS / 64);
    const int total = a.nobj * a.m;
    int task = blockIdx.x * (SA_THREADS / 64) + (tid >> 6);
    if (task >= total) return;
    int pn[SPAN];
    NarrowGather<SPAN, KG1> cur, nxt;
    f32x4 cwv[KG1];
    narrow_nbr<SPAN>(a, task, nn, pn);
    narrow_fetch<SPAN, KG1>(a, task, pn, q, cur);
    if (task + nw < total) narrow_nbr<SPAN>(a, task + nw, nn, pn);
    for (; task < total; task += nw) {
        if (task + nw < total) {
            narrow_fetch<SPAN, KG1>(a, task + nw, pn, q, nxt);
            if (task + 2 * nw < total) narrow_nbr<SPAN>(a, task + 2 * nw, nn, pn);
        }
        const float cx = cur.cx, cy = cur.cy, cz = cur.cz;
        f32x4 rmax[NT2];
#pragma unroll
        for (int t = 0; t < NT2; ++t) rmax[t] = f32x4{NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};   // pre-bias maxima
        const f32x4* cw = narrow_centroid_term<KG1>(sW0x, q, cx, cy, cz, cwv);
#pragma unroll
        for (int ct = 0; ct < SPAN; ++ct) {
            f32x4 bf[KG1];
            float mx = 0.f;
#pragma unroll
            for (int g = 0; g < KG1; ++g) {
                float r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    r[j] = relu1(fsub(cur.q[ct][g][j], cw[g][j]));
                    mx = fmax2(mx, r[j]);
                }
                bf[g] = f32x4{r[0], r[1], r[2], r[3]};
            }
            // layer 0 -> chunk planes at the column's scale
            const int E0 = col_exponent(rows_max(mx));
            f16x8 h0[KC0], l0[KC0];
#pragma unroll
            for (int c = 0; c < KC0; ++c) split_pair(bf[2 * c], bf[2 * c + 1], exp2i(14 - E0), h0[c], l0[c]);
            f32x4 acc1[NT1];
#pragma unroll
            for (int t = 0; t < NT1; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < KC0; ++c) {
#pragma unroll
                for (int t = 0; t < NT1; ++t) {
                    const f16x8 ah = sA1[((t * KC0 + c) * 2 + 0) * 64 + lane];
                    const f16x8 al = sA1[((t * KC0 + c) * 2 + 1) * 64 + lane];
                    acc1[t] = mfma_h(al, h0[c], acc1[t]);
                    acc1[t] = mfma_h(ah, l0[c], acc1[t]);
                    acc1[t] = mfma_h(ah, h0[c], acc1[t]);
                }
            }
            const float u0 = exp2i(E0 - 14 - a.ew1);
            float m1 = 0.f;
#pragma unroll
            for (int t = 0; t < NT1; ++t) {
                acc1[t] = relu4(acc1[t] * u0 + ld4(&sB1[16 * t + 4 * q]));
                m1 = fmax2(m1, max4(acc1[t]));
            }
            const int E1 = col_exponent(rows_max(m1));
            f16x8 h1[KC1], l1[KC1];
#pragma unroll
            for (int c = 0; c < KC1; ++c) split_pair(acc1[2 * c], acc1[2 * c + 1], exp2i(14 - E1), h1[c], l1[c]);
            f32x4 acc2[NT2];
#pragma unroll
            for (int t = 0; t < NT2; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < KC1; ++c) {
#pragma unroll
                for (int t = 0; t < NT2; ++t) {
                    const f16x8 ah = sA2[((t * KC1 + c) * 2 + 0) * 64 + lane];
                    const f16x8 al = sA2[((t * KC1 + c) * 2 + 1) * 64 + lane];
                    acc2[t] = mfma_h(al, h1[c], acc2[t]);
                    acc2[t] = mfma_h(ah, l1[c], acc2[t]);
                    acc2[t] = mfma_h(ah, h1[c], acc2[t]);
                }
            }
            const float u1 = exp2i(E1 - 14 - a.ew2);
#pragma unroll
            for (int t = 0; t < NT2; ++t) rmax[t] = vmax4(rmax[t], acc2[t] * u1);
            __builtin_amdgcn_sched_barrier(0);
        }
        float* o = a.out + (size_t)task * a.c_out_total + a.out_off + 4 * q;
#pragma unroll
        for (int t = 0; t < NT2; ++t) {
            const int j = nn >> 2;   // row16_max_scatter4 leaves channel 16 t + 4 q + j in this quad
            const float r = relu1(row16_max_scatter4(rmax[t], nn) + sB2[16 * t + 4 * q + j]);
            if ((nn & 3) == 0) o[16 * t + j] = r;
        }
        cur = nxt;
    }
}

// FPS levels run beside a narrow level's MLP as extra workgroups (blockIdx.y == 0, one per
// object): the chain's later levels depend only on the previous level's centroids, so they need
// not sit on the critical path. Level l+1 reads level l's sampled coordinates.
struct FpsSide {
    int nlev;               // 0: none
    int n[2], m[2], nb[2], jbits[2];
    const float* in;        // (B, n[0], 3)
    int* idx[2];            // (B, m_l)
    float* nxyz[2];         // (B, m_l, 3)
    int nobj;
};

static size_t fps_side_lds(const FpsSide& f) {
    return f.nlev ? FPS_RED_BYTES + sizeof(float) * 3 * ((size_t)f.n[0] + f.m[0]) + sizeof(int) * (size_t)f.m[0] : 0;
}

__device__ __forceinline__ void fps_side(const FpsSide& f, char* smem) {
    const int b = blockIdx.x;
    if (b >= f.nobj) return;
    void* s_red = smem;
    float* cur = reinterpret_cast<float*>(smem + FPS_RED_BYTES);
    float* nxt = cur + 3 * f.n[0];
    int* s_idx = reinterpret_cast<int*>(nxt + 3 * f.m[0]);
    const float* src = f.in + (size_t)b * f.n[0] * 3;
    for (int i = threadIdx.x; i < 3 * f.n[0]; i += FPS_THREADS) cur[i] = src[i];
    __syncthreads();
    for (int l = 0; l < f.nlev; ++l) {
        if (f.n[l] <= FPS_THREADS)
            fps_run<1>(cur, f.n[l], f.m[l], f.nb[l], f.jbits[l], s_red, s_idx, nxt);
        else if (f.n[l] <= 2 * FPS_THREADS)
            fps_run<2>(cur, f.n[l], f.m[l], f.nb[l], f.jbits[l], s_red, s_idx, nxt);
        else
            fps_run<4>(cur, f.n[l], f.m[l], f.nb[l], f.jbits[l], s_red, s_idx, nxt);
        __syncthreads();
        int* gi = f.idx[l] + (size_t)b * f.m[l];
        float* gx = f.nxyz[l] + (size_t)b * f.m[l] * 3;
        for (int i = threadIdx.x; i < f.m[l]; i += FPS_THREADS) gi[i] = s_idx[i];
        for (int i = threadIdx.x; i < 3 * f.m[l]; i += FPS_THREADS) gx[i] = nxt[i];
        __syncthreads();
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
}

// Both branches of a narrow level in one launch (blockIdx.y = 1 + branch), plus FPS side work.
template <int KG1a, int NT1a, int NT2a, int SPANa, int KG1b, int NT1b, int NT2b, int SPANb>
__global__ __launch_bounds__(SA_THREADS) void sa_narrow_kernel(NarrowArgs a0, NarrowArgs a1, FpsSide f) {
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
    // FPS first (blockIdx.y == 0): the dispatcher issues workgroups in linear order, so the
    // latency-bound FPS chain starts at once instead of behind the 1024 MLP workgroups
    if (blockIdx.y == 0)
        fps_side(f, reinterpret_cast<char*>(lds));
    else if (blockIdx.y == 1)
        narrow_branch<KG1a, NT1a, NT2a, SPANa>(a0, lds);
    else
        narrow_branch<KG1b, NT1b, NT2b, SPANb>(a1, lds);
}

// Level 1 with split-f16 layers 1-2 (both branches), FPS levels 2-3 beside it.
template <int KC0a, int NT1a, int NT2a, int SPANa, int KC0b, int NT1b, int NT2b, int SPANb>
__global__ __launch_bounds__(SA_THREADS) void sa_narrow_split_kernel(NarrowArgs a0, NarrowArgs a1, FpsSide f) {
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
    if (blockIdx.y == 0)
        fps_side(f, reinterpret_cast<char*>(lds));
    else if (blockIdx.y == 1)
        narrow_branch_split<KC0a, NT1a, NT2a, SPANa>(a0, lds);
    else
        narrow_branch_split<KC0b, NT1b, NT2b, SPANb>(a1, lds);
}

// Level 0: the 16-wide branch in exact fp32 (its layer 0 does not fill a 32-deep chunk), the 32-wide
// branch with split-f16 layers 1-2 (5x fewer MFMA cycles than fp32 16x16x4), FPS level 1 beside them.
template <int KG1a, int NT1a, int NT2a, int SPANa, int KC0b, int NT1b, int NT2b, int SPANb>
__global__ __launch_bounds__(SA_THREADS) void sa_narrow_mixed_kernel(NarrowArgs a0, NarrowArgs a1, FpsSide f) {
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
#ifdef NARROW_PROBE   // timing probes only (results are wrong): 1 = FPS only, 2 = branch a only, 3 = branch b only
    if (blockIdx.y != (NARROW_PROBE - 1)) return;
#endif
    if (blockIdx.y == 0)
        fps_side(f, reinterpret_cast<char*>(lds));
    else if (blockIdx.y == 1)
        narrow_branch<KG1a, NT1a, NT2a, SPANa>(a0, lds);
    else
        narrow_branch_split<KC0b, NT1b, NT2b, SPANb>(a1, lds);
}

static size_t narrow_split_lds(int kc0, int nt1, int nt2) {
    return 16 * ((size_t)nt1 * kc0 * 2 * 64 + (size_t)nt2 * (nt1 / 2) * 2 * 64 + (size_t)2 * kc0 * 16) +
           sizeof(float) * 16 * (nt1 + nt2);
}

static size_t narrow_lds(int kg1, int nt1, int nt2) {
    return sizeof(f32x4) * ((size_t)nt1 * kg1 * 64 + (size_t)nt2 * nt1 * 64 + kg1 * 16) + sizeof(float) * 16 * (nt1 + nt2);
}

// ============================================================================ split-f16 token GEMMs
// Per-point GEMMs of the encoder as token GEMMs: points are MFMA columns, outputs MFMA rows, both
// operands staged through LDS per 32-deep chunk (weights: pack_h16_fragments planes; points: fp32 rows
// split into hi/lo f16 on the way in at a per-point power-of-two scale from the point's max |x|), three
// products per chunk with fp32 accumulation as the other split levels. Workgroup tile: 64*WO outputs x
// 64*(8/WO) points, 8 waves as WO (outputs) x 8/WO (points) of 64 x 64; two LDS stages, one barrier per
// chunk.
//   MODE 0 (GroupAll layer 0, both branches in one launch): y = relu(W0 [f | xyz] + b) point-major, and
//          per point and branch the max of y (atomicMax on the bits of a float >= 0) for layer 1's scale;
//   MODE 1 (GroupAll layer 1): relu(W1 y + b), max over each object's 64 points (one wave's block), out;
//   MODE 2 (levels 1-3, per-point layer-0 projection Q = W0 [f | xyz] + b, no activation): y.
struct TokArgs {
    const float* x0[2];    // per branch: first input block, row-major (M, ld0), k0 columns
    int ld0, k0;
    const float* x1;       // second input block (M, ld1), k1 columns (null when k1 = 0)
    int ld1, k1;
    int M, KC;             // points; 32-deep chunks of the padded input
    const float* rmax[2];  // per branch: per-point max |x| over its input row
    const float* w[2];     // per branch: split planes, bias (padded to 32), weight exponent
    const float* bias[2];
    int ew[2];
    int nbpb;              // output blocks (64 * WO wide) per branch
    float* y;              // MODE 0/2: (M, ldy), branch br's outputs from column ycol[br]
    int ldy, ycol[2];
    unsigned* ymax;        // MODE 0: [2][M] max of y per point and branch
    float* out;            // MODE 1: (M / 64, ldo), branch br's outputs from column out_off[br]
    int ldo, out_off[2];
};
constexpr int TG_THREADS = 512;
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
template <int WO>
constexpr size_t tg_lds_bytes() {   // two stages of (4*WO weight + 4*(8/WO) point) tiles of 2 KiB + exponents
    return 2 * (size_t)(4 * WO + 4 * (8 / WO)) * 2048 + sizeof(int) * 64 * (8 / WO);
}

// max |x| over each point's input row [x0 | x1]: 16 lanes per point (16-byte loads when the rows
// allow), 16 points per 256-thread workgroup, the max over the 16 lanes by DPP (fmaxf, as the
// one-wave-per-point form this replaces: a wave per point spent its time in dispatch, 30-64 us per
// call at B=256)
template <int CTRL>
__device__ __forceinline__ float dpp_fmax(float v) {
    return fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true)));
}
__global__ __launch_bounds__(256) void tok_rowmax_kernel(const float* __restrict__ x0, int ld0, int k0,
                                                         const float* __restrict__ x1, int ld1, int k1, int M,
                                                         float* __restrict__ rmax) {
    const int r = blockIdx.x * 16 + (threadIdx.x >> 4), sub = threadIdx.x & 15;
    float m = 0.f;
    if (r < M) {   // no early exit: every lane of a 16-lane row takes part in the DPP max below
        const float* row = x0 + (size_t)r * ld0;
        if (((k0 | ld0) & 3) == 0 && (reinterpret_cast<uintptr_t>(x0) & 15) == 0) {
            for (int k = 4 * sub; k < k0; k += 64) {
                const f32x4 v = ld4(row + k);
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            }
        } else {
            for (int k = sub; k < k0; k += 16) m = fmaxf(m, fabsf(row[k]));
        }
        for (int k = sub; k < k1; k += 16) m = fmaxf(m, fabsf(x1[(size_t)r * ld1 + k]));
    }
    m = dpp_fmax<0xB1>(m);    // quad_perm [1,0,3,2]
    m = dpp_fmax<0x4E>(m);    // quad_perm [2,3,0,1]
    m = dpp_fmax<0x141>(m);   // row_half_mirror
    m = dpp_fmax<0x140>(m);   // row_mirror
    if (sub == 0 && r < M) rmax[r] = m;
}

template <int MODE, int WO>
__global__ __launch_bounds__(TG_THREADS) void tok_split_gemm_kernel(TokArgs a) {
    constexpr int WT = 8 / WO, BM = 64 * WT;
    constexpr int NA = 4 * WO * 128, NB = 4 * WT * 128;   // f16x8 fragments per stage
    extern __shared__ __attribute__((aligned(16))) f16x8 tg_lds[];
    auto sA = [&](int st) { return tg_lds + st * (NA + NB); };
    auto sB = [&](int st) { return tg_lds + st * (NA + NB) + NA; };
    int* eT = reinterpret_cast<int*>(tg_lds + 2 * (NA + NB));
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, n = lane & 15;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int br = blockIdx.x / a.nbpb, nblk = blockIdx.x - br * a.nbpb;
    const int m0 = blockIdx.y * BM, T0 = nblk * 4 * WO;
    const f16x8* W = reinterpret_cast<const f16x8*>(a.w[br]);
    const float* X0 = a.x0[br];
    // staging roles: weight fragments tid + 512u (u < WO); point rows (tid + 512u) / 8 (u < WT), k-group g
    const int g = tid & 7;
    int row[WT];
    float sc[WT];
#pragma unroll
    for (int u = 0; u < WT; ++u) {
        const int r = (tid + 512 * u) >> 3;
        row[u] = m0 + r;
        const int E = col_exponent(row[u] < a.M ? a.rmax[br][row[u]] : 0.f);
        sc[u] = exp2i(14 - E);
        if (g == 0) eT[r] = E;
    }
    auto fetch_x = [&](int r, int col) -> f32x4 {
        if (r >= a.M) return f32x4{0.f, 0.f, 0.f, 0.f};
        if (col + 4 <= a.k0) return ld4(X0 + (size_t)r * a.ld0 + col);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = col + j;
            v[j] = k < a.k0 ? X0[(size_t)r * a.ld0 + k] : (k - a.k0 < a.k1 ? a.x1[(size_t)r * a.ld1 + k - a.k0] : 0.f);
        }
        return f32x4{v[0], v[1], v[2], v[3]};
    };
    auto load = [&](int c, f32x4 (&ra)[WO], f32x4 (&rb)[WT]) {
#pragma unroll
        for (int u = 0; u < WO; ++u) {
            const int idx = tid + 512 * u;
            ra[u] = ld4(reinterpret_cast<const float*>(W + ((size_t)(T0 + (idx >> 7)) * a.KC + c) * 128 + (idx & 127)));
        }
#pragma unroll
        for (int u = 0; u < WT; ++u) rb[u] = fetch_x(row[u], 32 * c + 4 * g);
    };
    auto store = [&](int s, const f32x4 (&ra)[WO], const f32x4 (&rb)[WT]) {
#pragma unroll
        for (int u = 0; u < WO; ++u) sA(s)[tid + 512 * u] = __builtin_bit_cast(f16x8, ra[u]);
#pragma unroll
        for (int u = 0; u < WT; ++u) {
#pragma clang fp contract(off)
            const int r = (tid + 512 * u) >> 3, ln = 16 * (g & 3) + (r & 15), half = g >> 2;
            f16x4 hi, lo;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float x = rb[u][j] * sc[u];
                const _Float16 h = (_Float16)x;
                hi[j] = h;
                lo[j] = (_Float16)(x - (float)h);
            }
            reinterpret_cast<f16x4*>(&sB(s)[((r >> 4) * 2 + 0) * 64 + ln])[half] = hi;
            reinterpret_cast<f16x4*>(&sB(s)[((r >> 4) * 2 + 1) * 64 + ln])[half] = lo;
        }
    };
    const int wo = wid % WO, wt = wid / WO;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 ra[WO], rb[WT];
    load(0, ra, rb);
    store(0, ra, rb);
    __syncthreads();
    for (int c = 0; c < a.KC; ++c) {
        const int s = c & 1;
        if (c + 1 < a.KC) load(c + 1, ra, rb);
        f16x8 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bh[j] = sB(s)[((4 * wt + j) * 2 + 0) * 64 + lane];
            bl[j] = sB(s)[((4 * wt + j) * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x8 ah = sA(s)[((4 * wo + i) * 2 + 0) * 64 + lane];
            const f16x8 al = sA(s)[((4 * wo + i) * 2 + 1) * 64 + lane];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma_h(al, bh[j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma_h(ah, bl[j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma_h(ah, bh[j], acc[i][j]);
        }
        if (c + 1 < a.KC) store(s ^ 1, ra, rb);
        __syncthreads();
    }
    // epilogue: unscale (exact powers of two), bias, ReLU (MODE 0/1)
    const float* bias = a.bias[br];
    if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int pc = (4 * wt + j) * 16 + n, r = m0 + pc;
            const float u = exp2i(eT[pc] - 14 - a.ew[br]);
            float cm = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = (T0 + 4 * wo + i) * 16 + 4 * q;
                f32x4 v = acc[i][j] * u + ld4(bias + o);
                if constexpr (MODE == 0) {
                    v = relu4(v);
                    cm = fmax2(cm, max4(v));
                }
                if (r < a.M) st4(a.y + (size_t)r * a.ldy + a.ycol[br] + o, v);
            }
            if constexpr (MODE == 0) {
                cm = rows_max(cm);
                if (q == 0 && r < a.M) atomicMax(a.ymax + (size_t)br * a.M + r, __float_as_uint(cm));
            }
        }
    } else {
        f32x4 pm[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) pm[i] = f32x4{NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};   // pre-bias maxima
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int pc = (4 * wt + j) * 16 + n;
            const float u = exp2i(eT[pc] - 14 - a.ew[br]);
#pragma unroll
            for (int i = 0; i < 4; ++i) pm[i] = vmax4(pm[i], acc[i][j] * u);
        }
        const int obj = (m0 + 64 * wt) >> 6;   // the wave's 64 points are one object
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = n >> 2;   // row16_max_scatter4 leaves channel ... + 4 q + j in this quad
            const float r = relu1(row16_max_scatter4(pm[i], n) + bias[(T0 + 4 * wo + i) * 16 + 4 * q + j]);
            if ((n & 3) == 0 && obj * 64 < a.M) a.out[(size_t)obj * a.ldo + a.out_off[br] + (T0 + 4 * wo + i) * 16 + 4 * q + j] = r;
        }
    }
}

// Level-0 projection without point features (Light encoder, c_prev = 0): Q[p] = W0_xyz . x_p + b for
// both branches, a thread per (point, 4 channels), from the packed layer-0 fragments' xyz k-group (lane
// ch % 16 of tile ch / 16 holds (wx, wy, wz, 0)). The fma chain in k order is what the fp32 MFMA path
// (sa_pair_kernel) computes.
// The branch is the grid's y index, so its weight / bias pointers are picked by a wave-uniform index
// (scalar loads of the kernel arguments). Picked per lane, as this kernel once did, they were read with
// VECTOR loads from the kernel-argument segment, which the dispatch does not make coherent for the vector
// caches: with other processes' kernels on the GPU, a wave now and then read another dispatch's stale
// pointer and projected its points with the other branch's bias -- the one-off wrong level-0 features
// behind the round-4 multirank mismatch (scripts/race_probe.py; tests/test_cpu_host.py checks every kernel
// of the library for vector loads from the argument segment).
#ifndef PROJ_DIAG
#define PROJ_DIAG 0
#endif
struct ProjXyzArgs {
    const float* xyz;       // (B * n, 3)
    int npts;               // B * n
    const float* w0[2];     // packed layer-0 fragments (k-groups kg0 = 1, xyz group 0)
    const float* b0[2];
    int ch[2];              // padded channel counts (16 | 32)
    float* q;               // (B * n, q_stride): branch 0's channels, then branch 1's
    int q_stride;
};
__global__ __launch_bounds__(256) void proj_xyz_kernel(ProjXyzArgs a) {
    const int br = blockIdx.y;   // wave-uniform
    const int g4 = a.ch[br] / 4, qoff = br ? a.ch[0] : 0;
    const float* w0 = a.w0[br];
    const float* b0 = a.b0[br];
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (size_t)a.npts * g4) return;
    const int p = (int)(t / g4), g = (int)(t - (size_t)p * g4);
    const int c0 = 4 * g;
    const float x = ld1(a.xyz + (size_t)p * 3 + 0), y = ld1(a.xyz + (size_t)p * 3 + 1), z = ld1(a.xyz + (size_t)p * 3 + 2);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ch = c0 + j;
        const f32x4 w = ld4(w0 + ((size_t)(ch >> 4) * 64 + (ch & 15)) * 4);
        float acc = __builtin_fmaf(w.x, x, 0.f);
#if PROJ_DIAG & 2   // diagnostic: opaque values between the chains, so no packed-FP32 (v_pk_fma_f32) forms
        asm volatile("" : "+v"(acc));
#endif
        acc = __builtin_fmaf(w.y, y, acc);
#if PROJ_DIAG & 2
        asm volatile("" : "+v"(acc));
#endif
        acc = __builtin_fmaf(w.z, z, acc);
#if PROJ_DIAG & 2
        asm volatile("" : "+v"(acc));
#endif
        v[j] = acc + b0[ch];
#if PROJ_DIAG & 2
        asm volatile("" : "+v"(v[j]));
#endif
    }
    st4(a.q + (size_t)p * a.q_stride + qoff + 4 * g, f32x4{v[0], v[1], v[2], v[3]});
}

// Per-point layer-0 projection with point features (the DINO-pointwise level 0: c_prev = 384 rgb channels + xyz),
// both branches in one workgroup: Q[p] = W0 [f_p | x_p] + b, exact fp32 MFMA. Each wave owns 16 * CTW consecutive
// points and every output tile of both branches (NT0 + NT1): a point's row is read once and each A fragment (the
// packed layer-0 weights, from L2) feeds CTW column tiles; the k-groups of A and of the B operand (the rows, the xyz
// group last) are kept RING deep in flight. Per
// accumulator the MFMA sequence is sa_layer's projection pass (k-group g outer, its four k-steps j inner, the same
// operands): the same bits, where sa_pair_kernel read each row once per branch with one k-group in flight.
#ifndef PROJ_FEAT_CTW
#define PROJ_FEAT_CTW 4
#endif
#ifndef PROJ_FEAT_RING
#define PROJ_FEAT_RING 2
#endif
struct ProjFeatArgs {
    const float* feat;     // (npts, c_prev) point-major
    const float* xyz;      // (npts, 3)
    int npts, c_prev;      // points over all objects; channels (a multiple of 16)
    const float* w0[2];    // packed layer-0 fragments of each branch ((c_prev + 16) / 16 k-groups per tile)
    const float* b0[2];    // biases, padded to 16
    float* q;              // (npts, q_stride): branch 0's channels, then branch 1's
    int q_stride;
};
template <int NT0, int NT1, int CTW, int RING>
__global__ __launch_bounds__(256) void proj_feat_kernel(ProjFeatArgs a) {
    constexpr int NT = NT0 + NT1;
    const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p0 = (blockIdx.x * 4 + wid) * 16 * CTW;
    if (p0 >= a.npts) return;   // whole waves leave together
    const int FG = a.c_prev >> 4, KG = FG + 1;
    const __amdgpu_buffer_rsrc_t W0 = make_rsrc(a.w0[0], (uint32_t)(NT0 * KG) * 1024u);
    const __amdgpu_buffer_rsrc_t W1 = make_rsrc(a.w0[1], (uint32_t)(NT1 * KG) * 1024u);
    const int voff = lane * 16;
    bool ok[CTW];
    const float* row[CTW];
    f32x4 bx[CTW];   // the xyz k-group: raw coordinates in lanes q == 0 (channels c_prev + 0..2)
#pragma unroll
    for (int c = 0; c < CTW; ++c) {
        const int p = p0 + 16 * c + n;
        ok[c] = p < a.npts;
        row[c] = a.feat + (size_t)(ok[c] ? p : 0) * a.c_prev + 4 * q;
        bx[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (ok[c] && q == 0) {
            const float* px = a.xyz + (size_t)p * 3;
            bx[c] = f32x4{ld1(px), ld1(px + 1), ld1(px + 2), 0.f};
        }
    }
    f32x4 acc[NT][CTW];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int c = 0; c < CTW; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    // every A fragment (weights, L2) feeds CTW column tiles
    auto fetch = [&](int g, f32x4 (&af)[NT], f32x4 (&bf)[CTW]) {
#pragma unroll
        for (int t = 0; t < NT0; ++t) af[t] = ldbuf4(W0, voff, (t * KG + g) * 1024);
#pragma unroll
        for (int t = 0; t < NT1; ++t) af[NT0 + t] = ldbuf4(W1, voff, (t * KG + g) * 1024);
#pragma unroll
        for (int c = 0; c < CTW; ++c) bf[c] = g < FG ? (ok[c] ? ld4(row[c] + 16 * g) : f32x4{0.f, 0.f, 0.f, 0.f}) : bx[c];
    };
    auto compute = [&](const f32x4 (&af)[NT], const f32x4 (&bf)[CTW]) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int c = 0; c < CTW; ++c) acc[t][c] = mfma4(af[t][j], bf[c][j], acc[t][c]);
    };
    f32x4 ra[RING][NT], rb[RING][CTW];
#pragma unroll
    for (int u = 0; u < RING - 1; ++u)
        if (u < KG) fetch(u, ra[u], rb[u]);
    for (int g0 = 0; g0 < KG; g0 += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            const int g = g0 + u;
            if (g < KG) {
                if (g + RING - 1 < KG) fetch(g + RING - 1, ra[(u + RING - 1) % RING], rb[(u + RING - 1) % RING]);
                __builtin_amdgcn_sched_barrier(0);
                compute(ra[u], rb[u]);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int br = t < NT0 ? 0 : 1, T = t < NT0 ? t : t - NT0;
        const f32x4 bias = ld4(a.b0[br] + 16 * T + 4 * q);
#pragma unroll
        for (int c = 0; c < CTW; ++c)
            if (ok[c])
                st4(a.q + (size_t)(p0 + 16 * c + n) * a.q_stride + 4 * q + (br ? 16 * NT0 : 0) + 16 * T, acc[t][c] + bias);
    }
}

// ============================================================================ host side
static const int kNpoint[4] = {512, 256, 128, 64};
static const int kNs[2] = {16, 32};
static const float kRadius[4][2] = {{0.01f, 0.02f}, {0.02f, 0.04f}, {0.04f, 0.08f}, {0.08f, 0.16f}};
static const int kWidths[5][2][4] = {
    {{3, 16, 16, 32}, {3, 32, 32, 64}},
    {{99, 64, 64, 128}, {99, 64, 96, 128}},
    {{259, 128, 196, 256}, {259, 128, 196, 256}},
    {{515, 256, 256, 512}, {515, 256, 384, 512}},
    {{1027, 512, 512, 0}, {1027, 512, 512, 0}}};
static const int kCout[5] = {96, 256, 512, 1024, 1024};

static inline int pad16(int v) { return (v + 15) & ~15; }

struct EncLayout {
    size_t fps[4], nxyz[4], ball[4][2], feat[5], proj[4], total;
};

// Per-point layer-0 projection width of level l (both branches, each padded to 16).
static inline int proj_stride(int l) { return pad16(kWidths[l][0][1]) + pad16(kWidths[l][1][1]); }

static EncLayout enc_layout(int B, int N) {
    EncLayout L;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    for (int l = 0; l < 4; ++l) {
        const size_t M = kNpoint[l];
        L.fps[l] = take(sizeof(int) * B * M);
        L.nxyz[l] = take(sizeof(float) * B * M * 3);
        L.ball[l][0] = take(sizeof(int) * B * M * kNs[0]);
        L.ball[l][1] = take(sizeof(int) * B * M * kNs[1]);
    }
    for (int l = 0; l < 5; ++l) L.feat[l] = take(sizeof(float) * B * (l < 4 ? kNpoint[l] : 1) * kCout[l]);
    for (int l = 0; l < 4; ++l)
        L.proj[l] = take(sizeof(float) * B * (size_t)(l == 0 ? N : kNpoint[l - 1]) * proj_stride(l));
    L.total = off;
    return L;
}

extern "C" size_t gp_encoder_workspace_size(int b, int n) { return enc_layout(b, n).total; }

extern "C" int gp_encoder_workspace_layout(int b, int n, int64_t* offsets) {
    GP_REQUIRE(offsets, "encoder_workspace_layout: null offsets");
    const EncLayout L = enc_layout(b, n);
    for (int l = 0; l < 5; ++l) {
        offsets[l * 5 + 0] = l < 4 ? (int64_t)L.fps[l] : -1;
        offsets[l * 5 + 1] = l < 4 ? (int64_t)L.nxyz[l] : -1;
        offsets[l * 5 + 2] = l < 4 ? (int64_t)L.ball[l][0] : -1;
        offsets[l * 5 + 3] = l < 4 ? (int64_t)L.ball[l][1] : -1;
        offsets[l * 5 + 4] = (int64_t)L.feat[l];
    }
    return GP_OK;
}

template <int CT>
static size_t sa_lds(SAArgs& a) {
    size_t buf0 = 0, buf1 = 0;
    if (a.nlayers >= 2) buf0 = (size_t)CT * 16 * a.nt[0] * 16;                 // floats
    if (a.nlayers >= 3) buf1 = (size_t)CT * 16 * a.nt[1] * 16;
    a.buf1_off = (int)(buf0 / 4);
    return (buf0 + buf1) * sizeof(float);
}

template <int CT>
static int sa_span(const SAArgs& a) {
    const int tpc = a.ns / 16;
    return tpc < CT ? tpc : CT;
}

// One launch for a pair of branches (a0 on blockIdx.z = 0, a1 on 1).
template <int CT, int MAXTC = 4>
static int launch_pair(SAArgs a0, SAArgs a1, int B, hipStream_t st) {
    const size_t lds = std::max(sa_lds<CT>(a0), sa_lds<CT>(a1));
    if (lds > 160 * 1024) {
        gp_set_error("sa_pair_kernel: LDS %zu bytes exceeds 160 KiB", lds);
        return GP_ERR_UNSUPPORTED;
    }
    const int blocks = std::max((a0.cols + CT * 16 - 1) / (CT * 16), (a1.cols + CT * 16 - 1) / (CT * 16));
    const int s0 = sa_span<CT>(a0), s1 = sa_span<CT>(a1);
    const dim3 grid(blocks, B, 2), blk(SA_THREADS);
#define GP_SA_PAIR(S0, S1)                                                                     \
    if (s0 == S0 && s1 == S1) {                                                                \
        hipLaunchKernelGGL((sa_pair_kernel<CT, S0, S1, MAXTC>), grid, blk, lds, st, a0, a1);   \
        return gp_check_launch("sa_pair_kernel");                                              \
    }
    if constexpr (CT == 2) {
        GP_SA_PAIR(1, 2) GP_SA_PAIR(2, 2) GP_SA_PAIR(1, 1)
    } else {
        GP_SA_PAIR(4, 4) GP_SA_PAIR(1, 2) GP_SA_PAIR(2, 2) GP_SA_PAIR(1, 1)
    }
#undef GP_SA_PAIR
    gp_set_error("sa_pair_kernel: unsupported spans %d/%d", s0, s1);
    return GP_ERR_UNSUPPORTED;
}

// Row of the packed-layer table (pack.pack_encoder, [5][2][3][4]): {fp32 fragments, bias, split
// planes or -1, split exponent}.
static inline const int64_t* enc_layer(const int64_t* tab, int l, int br, int i) { return tab + ((l * 2 + br) * 3 + i) * 4; }

// Per-call view of the encoder workspace (enc_layout) and the packed layer table.
// geo: the workspace that holds (or receives) the geometry -- FPS indices, centroids, ball lists -- which
// depends only on the points; another encoder's workspace when two models encode the same points
// (gp_encoder_forward_geom). geo_ready: the ball lists are already there (no ball query per level).
struct EncCtx {
    const float* wbuf;
    const int64_t* tab;
    const float* pts;
    int B, N;
    char* ws;
    char* geo;
    bool geo_ready;
    EncLayout L;
    int* fidx[4];
    float* nxyz[4];
    int nin[4], mout[4];
};

static EncCtx enc_ctx(const float* wbuf, const int64_t* layer_off, const float* pts, int B, int N, void* workspace,
                      void* geometry = nullptr) {
    EncCtx c;
    c.wbuf = wbuf;
    c.tab = layer_off;
    c.pts = pts;
    c.B = B;
    c.N = N;
    c.ws = static_cast<char*>(workspace);
    c.geo = geometry ? static_cast<char*>(geometry) : c.ws;
    c.geo_ready = geometry != nullptr;
    c.L = enc_layout(B, N);
    for (int l = 0; l < 4; ++l) {
        c.fidx[l] = reinterpret_cast<int*>(c.geo + c.L.fps[l]);
        c.nxyz[l] = reinterpret_cast<float*>(c.geo + c.L.nxyz[l]);
        c.nin[l] = l == 0 ? N : kNpoint[l - 1];
        c.mout[l] = kNpoint[l];
    }
    return c;
}

// Per-point layer-0 projection of level l (1-3) as a split-f16 token GEMM (MODE 2): Q = W0 [f | xyz] + b
// for both branches into qbuf (B, n_prev, proj_stride). The per-point maxima go to level l-1's
// projection buffer, free once level l-1 has run.
static int run_proj_split(const EncCtx& c, int l, int c_prev, const float* feat_prev, const float* xyz_prev,
                          int n_prev, float* qbuf, hipStream_t st) {
    const int B = c.B, M = B * n_prev, w = kWidths[l][0][1];
    GP_REQUIRE(w == kWidths[l][1][1] && (w == 64 || w == 128 || w == 256) && feat_prev && c_prev % 4 == 0,
               "encoder: level %d projection of width %d has no split tile", l, w);
    float* rmax = reinterpret_cast<float*>(c.ws + c.L.proj[l - 1]);
    hipLaunchKernelGGL(tok_rowmax_kernel, dim3((M + 15) / 16), dim3(256), 0, st, feat_prev, c_prev, c_prev, xyz_prev, 3,
                       3, M, rmax);
    TokArgs a = {};
    a.M = M;
    a.nbpb = 1;
    for (int br = 0; br < 2; ++br) {
        const int64_t* o = enc_layer(c.tab, l, br, 0);
        a.x0[br] = feat_prev;
        a.rmax[br] = rmax;
        a.w[br] = c.wbuf + o[2];
        a.bias[br] = c.wbuf + o[1];
        a.ew[br] = (int)o[3];
        a.ycol[br] = br == 0 ? 0 : pad16(w);
    }
    a.ld0 = c_prev;
    a.k0 = c_prev;
    a.x1 = xyz_prev;
    a.ld1 = 3;
    a.k1 = 3;
    a.KC = (c_prev + 3 + 31) / 32;
    a.y = qbuf;
    a.ldy = proj_stride(l);
#define GP_PROJ(WO)                                                                                          \
    hipLaunchKernelGGL((tok_split_gemm_kernel<2, WO>), dim3(2, (M + 64 * (8 / WO) - 1) / (64 * (8 / WO))), \
                       dim3(TG_THREADS), tg_lds_bytes<WO>(), st, a)
    if (w == 256) GP_PROJ(4);
    else if (w == 128) GP_PROJ(2);
    else GP_PROJ(1);
#undef GP_PROJ
    return gp_check_launch("tok_split_gemm_kernel (projection)");
}

// GroupAll as two split-f16 token GEMMs (tok_split_gemm_kernel) when the table carries both layers' planes.
// Scratch: layer 0's output (B*64 x 1024) in level 3's projection buffer, the per-point maxima in level
// 2's, both free once level 3 has run.
static int run_groupall_split(const EncCtx& c, const float* feat_prev, float* out, hipStream_t st) {
    const int B = c.B, P = kNpoint[3], M = B * P;
    const int k_in = kCout[3];
    GP_REQUIRE(P == 64 && kWidths[4][0][1] == 512 && kWidths[4][1][1] == 512 && kWidths[4][0][2] == 512 &&
                   kWidths[4][1][2] == 512 && kWidths[4][0][0] == k_in + 3,
               "encoder: GroupAll split path expects 64 points of %d + 3 channels", k_in);
    float* y0 = reinterpret_cast<float*>(c.ws + c.L.proj[3]);
    float* rmax0 = reinterpret_cast<float*>(c.ws + c.L.proj[2]);
    unsigned* ymax = reinterpret_cast<unsigned*>(rmax0 + M);
    GP_REQUIRE((size_t)kNpoint[2] * proj_stride(3) >= (size_t)P * 1024 && (size_t)kNpoint[1] * proj_stride(2) >= 3u * P,
               "encoder: GroupAll scratch does not fit the projection buffers");
    const float* xyz = c.nxyz[3];
    hipLaunchKernelGGL(tok_rowmax_kernel, dim3((M + 15) / 16), dim3(256), 0, st, feat_prev, k_in, k_in, xyz, 3, 3, M,
                       rmax0);
    if (hipMemsetAsync(ymax, 0, sizeof(unsigned) * 2 * (size_t)M, st) != hipSuccess)
        return gp_check_launch("groupall memset");
    TokArgs a = {};
    a.M = M;
    a.nbpb = 2;
    for (int br = 0; br < 2; ++br) {
        const int64_t* o = enc_layer(c.tab, 4, br, 0);
        a.x0[br] = feat_prev;
        a.rmax[br] = rmax0;
        a.w[br] = c.wbuf + o[2];
        a.bias[br] = c.wbuf + o[1];
        a.ew[br] = (int)o[3];
    }
    a.ld0 = k_in;
    a.k0 = k_in;
    a.x1 = xyz;
    a.ld1 = 3;
    a.k1 = 3;
    a.KC = (k_in + 3 + 31) / 32;
    a.y = y0;
    a.ldy = 1024;
    a.ycol[0] = 0;
    a.ycol[1] = 512;
    a.ymax = ymax;
    const dim3 grid(4, (M + 127) / 128);
    hipLaunchKernelGGL((tok_split_gemm_kernel<0, 4>), grid, dim3(TG_THREADS), tg_lds_bytes<4>(), st, a);
    TokArgs b = {};
    b.M = M;
    b.nbpb = 2;
    for (int br = 0; br < 2; ++br) {
        const int64_t* o = enc_layer(c.tab, 4, br, 1);
        b.x0[br] = y0 + 512 * br;
        b.rmax[br] = reinterpret_cast<const float*>(ymax) + (size_t)br * M;
        b.w[br] = c.wbuf + o[2];
        b.bias[br] = c.wbuf + o[1];
        b.ew[br] = (int)o[3];
        b.out_off[br] = 512 * br;
    }
    b.ld0 = 1024;
    b.k0 = 512;
    b.KC = 16;
    b.out = out;
    b.ldo = kCout[4];
    hipLaunchKernelGGL((tok_split_gemm_kernel<1, 4>), grid, dim3(TG_THREADS), tg_lds_bytes<4>(), st, b);
    return gp_check_launch("tok_split_gemm_kernel");
}

// One SA level l (ball query, per-point layer 0, layers 1-2 + max-pool) over the FPS results already
// in the workspace. feat_prev (B, n_prev, c_prev) point-major or null (c_prev = 0); out (B, M_l, C_l).
// side: FPS levels that ride along as extra workgroups of the narrow launches (gp_encoder_forward),
// or null when the FPS chain ran whole beforehand (gp_encoder_fps).
static int run_sa_level(const EncCtx& c, int l, int c_prev, const float* feat_prev, float* out, bool side,
                        hipStream_t st) {
    const int B = c.B;
    const float* wbuf = c.wbuf;
    const int64_t* layer_off = c.tab;
    const float* xyz_prev = l == 0 ? c.pts : c.nxyz[l - 1];
    const int n_prev = l == 0 ? c.N : kNpoint[l - 1];
    int rc = GP_OK;
    int* b0 = nullptr;
    int* b1 = nullptr;
    if (l < 4) {
        b0 = reinterpret_cast<int*>(c.geo + c.L.ball[l][0]);
        b1 = reinterpret_cast<int*>(c.geo + c.L.ball[l][1]);
        if (!c.geo_ready) {
            rc = gp_launch_ball_query2(B, n_prev, kNpoint[l], kRadius[l][0], kRadius[l][1], kNs[0], kNs[1], c.nxyz[l],
                                       xyz_prev, b0, b1, st);
            if (rc) return rc;
        }
    }
    // layer 0 once per input point for both branches (levels 0-3)
    float* qbuf = l < 4 ? reinterpret_cast<float*>(c.ws + c.L.proj[l]) : nullptr;
    if (l < 4) {
        int q_off = 0;
        SAArgs pp[2];
        for (int br = 0; br < 2; ++br) {
            SAArgs& pa = pp[br];
            pa = {};
            pa.n_prev = n_prev;
            pa.c_prev = c_prev;
            pa.m = 1;
            pa.ns = n_prev;
            pa.cols = n_prev;
            pa.xyz_prev = xyz_prev;
            pa.feat_prev = feat_prev;
            pa.nlayers = 1;
            const int64_t* o = enc_layer(layer_off, l, br, 0);
            GP_REQUIRE(o[0] >= 0 && o[1] >= 0, "encoder: missing layer %d/%d/0", l, br);
            pa.w[0] = wbuf + o[0];
            pa.bias[0] = wbuf + o[1];
            pa.kg[0] = (pa.c_prev + 16) / 16;
            pa.nt[0] = pad16(kWidths[l][br][1]) / 16;
            pa.proj_out = qbuf;
            pa.q_stride = proj_stride(l);
            pa.q_off = q_off;
            pa.tag = 16 + l * 2 + br;
            q_off += pad16(kWidths[l][br][1]);
        }
        const bool split0 = l >= 1 && enc_layer(layer_off, l, 0, 0)[2] >= 0 && enc_layer(layer_off, l, 1, 0)[2] >= 0;
        if (l == 0 && c_prev == 0) {   // xyz only: 3 multiply-adds per channel
            ProjXyzArgs pa = {};
            pa.xyz = xyz_prev;
            pa.npts = B * n_prev;
            for (int br = 0; br < 2; ++br) {
                pa.w0[br] = pp[br].w[0];
                pa.b0[br] = pp[br].bias[0];
                pa.ch[br] = pad16(kWidths[0][br][1]);
            }
            GP_REQUIRE(pa.ch[0] + pa.ch[1] == proj_stride(0), "encoder: level-0 projection layout");
            pa.q = qbuf;
            pa.q_stride = proj_stride(0);
            const size_t threads = (size_t)pa.npts * std::max(pa.ch[0], pa.ch[1]) / 4;   // per branch (grid y)
            hipLaunchKernelGGL(proj_xyz_kernel, dim3((unsigned)((threads + 255) / 256), 2), dim3(256), 0, st, pa);
            rc = gp_check_launch("proj_xyz_kernel");
        } else if (l == 0 && !split0 && c_prev % 16 == 0 && pad16(kWidths[0][0][1]) == 16 &&
                   pad16(kWidths[0][1][1]) == 32) {   // point features at level 0 (DINO-pointwise)
            ProjFeatArgs pa = {};
            pa.feat = feat_prev;
            pa.xyz = xyz_prev;
            pa.npts = B * n_prev;
            pa.c_prev = c_prev;
            for (int br = 0; br < 2; ++br) {
                pa.w0[br] = pp[br].w[0];
                pa.b0[br] = pp[br].bias[0];
            }
            pa.q = qbuf;
            pa.q_stride = proj_stride(0);
            GP_REQUIRE(feat_prev && pa.q_stride == 48, "encoder: level-0 feature projection layout");
            constexpr int CTW = PROJ_FEAT_CTW;   // points per wave / 16
            hipLaunchKernelGGL((proj_feat_kernel<1, 2, CTW, PROJ_FEAT_RING>), dim3((pa.npts + 64 * CTW - 1) / (64 * CTW)),
                               dim3(256), 0, st, pa);
            rc = gp_check_launch("proj_feat_kernel");
        } else {
            rc = split0 ? run_proj_split(c, l, c_prev, feat_prev, xyz_prev, n_prev, qbuf, st)
                        : launch_pair<4>(pp[0], pp[1], B, st);
        }
        if (rc) return rc;
    }
    if (l == 4 && enc_layer(layer_off, 4, 0, 0)[2] >= 0 && enc_layer(layer_off, 4, 0, 1)[2] >= 0 &&
        enc_layer(layer_off, 4, 1, 0)[2] >= 0 && enc_layer(layer_off, 4, 1, 1)[2] >= 0)
        return run_groupall_split(c, feat_prev, out, st);
    if (l == 4) {  // group-all pools with atomicMax when a centroid spans workgroups
        if (hipMemsetAsync(out, 0, sizeof(float) * B * kCout[4], st) != hipSuccess)
            return gp_check_launch("encoder memset");
    }
    if (l <= 1) {   // narrow levels: one launch, wave-independent centroids
        NarrowArgs na[2];
        int out_off = 0, q_off = 0;
        for (int br = 0; br < 2; ++br) {
            NarrowArgs& n = na[br];
            n = {};
            n.qin = qbuf;
            n.q_stride = proj_stride(l);
            n.q_off = q_off;
            q_off += pad16(kWidths[l][br][1]);
            n.n_prev = n_prev;
            const int64_t* o0 = enc_layer(layer_off, l, br, 0);
            const int64_t* o1 = enc_layer(layer_off, l, br, 1);
            const int64_t* o2 = enc_layer(layer_off, l, br, 2);
            GP_REQUIRE(o1[0] >= 0 && o2[0] >= 0, "encoder: missing layers of %d/%d", l, br);
            n.w0 = wbuf + o0[0];
            n.c_out_total = kCout[l];
            n.kg0 = (c_prev + 16) / 16;
            n.gx = c_prev / 16;
            n.w1 = wbuf + o1[0];
            n.b1 = wbuf + o1[1];
            n.w2 = wbuf + o2[0];
            n.b2 = wbuf + o2[1];
            n.nbr = br == 0 ? b0 : b1;
            n.cent = c.nxyz[l];
            n.m = kNpoint[l];
            n.ns = kNs[br];
            n.nobj = B;
            n.out = out;
            n.out_off = out_off;
            out_off += kWidths[l][br][3];
            n.w1h = o1[2] >= 0 ? wbuf + o1[2] : nullptr;
            n.w2h = o2[2] >= 0 ? wbuf + o2[2] : nullptr;
            n.ew1 = (int)o1[3];
            n.ew2 = (int)o2[3];
        }
        FpsSide fs = {};   // nobj = 0: the FPS row of workgroups returns at once
        if (side) {
            fs.nlev = l == 0 ? 1 : 2;          // level 0 launch: FPS level 1; level 1 launch: FPS levels 2, 3
            fs.in = c.nxyz[l];
            fs.nobj = B;
            for (int k = 0; k < fs.nlev; ++k) {
                const int lv = l == 0 ? 1 : 2 + k;
                fs.n[k] = c.nin[lv];
                fs.m[k] = c.mout[lv];
                const FpsGeom g = fps_geom(c.nin[lv]);
                fs.nb[k] = g.nb;
                fs.jbits[k] = g.jbits;
                fs.idx[k] = c.fidx[lv];
                fs.nxyz[k] = c.nxyz[lv];
            }
        }
        const dim3 grid(std::max(512, B), 3);
        if (l == 0 && na[1].w1h && na[1].w2h) {
            const size_t lds = std::max({narrow_lds(1, 1, 2), narrow_split_lds(1, 2, 4), fps_side_lds(fs)});
#ifdef GP_NARROW_SEQ   // diagnostic builds only: the two branches as two launches (no co-resident mix)
            NarrowArgs n0 = na[0], n1 = na[1];
            n0.nobj = 0;
            n1.nobj = 0;
            hipLaunchKernelGGL((sa_narrow_mixed_kernel<1, 1, 2, 1, 1, 2, 4, 2>), grid, dim3(SA_THREADS), lds, st,
                               na[0], n1, fs);
            hipLaunchKernelGGL((sa_narrow_mixed_kernel<1, 1, 2, 1, 1, 2, 4, 2>), grid, dim3(SA_THREADS), lds, st,
                               n0, na[1], FpsSide{});
#else
            hipLaunchKernelGGL((sa_narrow_mixed_kernel<1, 1, 2, 1, 1, 2, 4, 2>), grid, dim3(SA_THREADS), lds, st,
                               na[0], na[1], fs);
#endif
        } else if (l == 0) {
            const size_t lds = std::max({narrow_lds(1, 1, 2), narrow_lds(2, 2, 4), fps_side_lds(fs)});
            hipLaunchKernelGGL((sa_narrow_kernel<1, 1, 2, 1, 2, 2, 4, 2>), grid, dim3(SA_THREADS), lds, st, na[0],
                               na[1], fs);
        } else if (na[0].w1h && na[0].w2h && na[1].w1h && na[1].w2h) {
            const size_t lds = std::max({narrow_split_lds(2, 4, 8), narrow_split_lds(2, 6, 8), fps_side_lds(fs)});
            hipLaunchKernelGGL((sa_narrow_split_kernel<2, 4, 8, 1, 2, 6, 8, 2>), grid, dim3(SA_THREADS), lds, st,
                               na[0], na[1], fs);
        } else {
            const size_t lds = std::max({narrow_lds(4, 4, 8), narrow_lds(4, 6, 8), fps_side_lds(fs)});
            hipLaunchKernelGGL((sa_narrow_kernel<4, 4, 8, 1, 4, 6, 8, 2>), grid, dim3(SA_THREADS), lds, st, na[0],
                               na[1], fs);
        }
        return gp_check_launch("sa_narrow_kernel");
    }
    // levels 2-3: split-f16 kernel when the table carries the planes (pack.pack_encoder)
    if ((l == 2 || l == 3) && enc_layer(layer_off, l, 0, 1)[2] >= 0 && enc_layer(layer_off, l, 0, 2)[2] >= 0 &&
        enc_layer(layer_off, l, 1, 1)[2] >= 0 && enc_layer(layer_off, l, 1, 2)[2] >= 0) {
        const int CT = l == 2 ? SPLIT_CT2 : SPLIT_CT3;
        SplitArgs sp[2];
        int off_out = 0;
        for (int br = 0; br < 2; ++br) {
            SplitArgs& a = sp[br];
            a = {};
            a.n_prev = n_prev;
            a.m = kNpoint[l];
            a.ns = kNs[br];
            a.cols = a.m * a.ns;
            a.qin = qbuf;
            a.q_stride = proj_stride(l);
            a.q_off = br == 0 ? 0 : pad16(kWidths[l][0][1]);
            const int64_t* o0 = enc_layer(layer_off, l, br, 0);
            a.w0 = wbuf + o0[0];
            a.kg0 = (c_prev + 16) / 16;
            a.gx = c_prev / 16;
            a.nbr = br == 0 ? b0 : b1;
            a.cent = c.nxyz[l];
            for (int i = 0; i < 2; ++i) {
                const int64_t* o = enc_layer(layer_off, l, br, i + 1);
                a.w[i] = wbuf + o[2];
                a.bias[i] = wbuf + o[1];
                a.ew[i] = (int)o[3];
            }
            a.out = out;
            a.c_out_total = kCout[l];
            a.out_off = off_out;
            a.tag = l * 2 + br;
            off_out += kWidths[l][br][3];
            GP_REQUIRE((16 * CT) % a.ns == 0, "encoder: level %d centroids of %d columns straddle %d-column tiles",
                       l, a.ns, 16 * CT);
        }
        const int cmax = std::max(sp[0].cols, sp[1].cols);
        const dim3 grid((cmax + 16 * CT - 1) / (16 * CT), B, 2), blk(SPLIT_WV * 64);
        if (l == 2) {
            const size_t lds = sa_split_lds<SPLIT_CT2, 4, 7>();
            hipLaunchKernelGGL((sa_split_kernel<SPLIT_CT2, SPLIT_D2, 4, 7, 8, 7, 8, 2>), grid, blk, lds, st, sp[0], sp[1]);
        } else {
            const size_t lds = std::max(sa_split_lds<SPLIT_CT3, 8, 8>(), sa_split_lds<SPLIT_CT3, 8, 12>());
            hipLaunchKernelGGL((sa_split_kernel<SPLIT_CT3, SPLIT_D3, 8, 8, 16, 12, 16>), grid, blk, lds, st, sp[0],
                               sp[1]);
        }
        return gp_check_launch("sa_split_kernel");
    }
    int out_off = 0;
    SAArgs sa[2];
    for (int br = 0; br < 2; ++br) {
        SAArgs& a = sa[br];
        a = {};
        a.n_prev = n_prev;
        a.c_prev = c_prev;
        a.m = l < 4 ? kNpoint[l] : 1;
        a.ns = l < 4 ? kNs[br] : n_prev;
        a.cols = a.m * a.ns;
        a.xyz_prev = xyz_prev;
        a.feat_prev = feat_prev;
        a.cent = l < 4 ? c.nxyz[l] : nullptr;
        a.nbr = l < 4 ? (br == 0 ? b0 : b1) : nullptr;
        a.nlayers = l < 4 ? 3 : 2;
        for (int i = 0; i < a.nlayers; ++i) {
            const int64_t* o = enc_layer(layer_off, l, br, i);
            GP_REQUIRE(o[0] >= 0 && o[1] >= 0, "encoder: missing layer %d/%d/%d", l, br, i);
            a.w[i] = wbuf + o[0];
            a.bias[i] = wbuf + o[1];
            const int kin = i == 0 ? a.c_prev + 16 : pad16(kWidths[l][br][i]);
            a.kg[i] = kin / 16;
            a.nt[i] = pad16(kWidths[l][br][i + 1]) / 16;
        }
        a.out = out;
        a.tag = l * 2 + br;
        if (l < 4) {
            a.qin = qbuf;
            a.q_stride = proj_stride(l);
            a.q_off = br == 0 ? 0 : pad16(kWidths[l][0][1]);
        }
        a.c_out_total = kCout[l];
        a.out_off = out_off;
        out_off += kWidths[l][br][a.nlayers];
        if (a.ns % 16 != 0) {
            gp_set_error("encoder: nsample %d not a multiple of 16", a.ns);
            return GP_ERR_UNSUPPORTED;
        }
    }
    // levels 2-3 at 32 columns (LDS ping-pong <= 80 KiB: 2-3 workgroups per CU), GroupAll split
    // over 2 workgroups per (object, branch) with atomicMax pooling; both branches per launch
    // levels 3-4: one pass of up to 8 tiles per wave per layer (2 workgroups per CU either way);
    // level 2 keeps 4-tile passes: its 131 VGPRs fit 3 workgroups per CU, a 7-tile pass's 191 only
    // 2 (measured 725 vs 764 us)
    return l == 2 ? launch_pair<2, 4>(sa[0], sa[1], B, st) : launch_pair<2, 8>(sa[0], sa[1], B, st);
}

static int enc_check(const float* wbuf, const int64_t* layer_off, const float* pts, int B, int N, void* workspace,
                     size_t workspace_bytes) {
    GP_REQUIRE(wbuf && layer_off && pts && workspace, "encoder: null pointer");
    GP_REQUIRE(B >= 1 && N >= kNpoint[0] && N <= 8192, "encoder: need 1<=b and 512<=n<=8192 (b=%d n=%d)", B, N);
    const size_t need = enc_layout(B, N).total;
    GP_REQUIRE(workspace_bytes >= need, "encoder: workspace %zu < %zu", workspace_bytes, need);
    return GP_OK;
}

extern "C" int gp_encoder_forward(const float* wbuf, const int64_t* layer_off, const float* pts, int B, int N,
                                  void* workspace, size_t workspace_bytes, float* feat, hipStream_t st) {
    int rc = enc_check(wbuf, layer_off, pts, B, N, workspace, workspace_bytes);
    if (rc) return rc;
    GP_REQUIRE(feat, "encoder_forward: null feat");
    const EncCtx c = enc_ctx(wbuf, layer_off, pts, B, N, workspace);
    // FPS level 0 here; levels 1-3 run beside the level-0 / level-1 MLP launches (FpsSide)
#ifdef GP_NO_FPS_SIDE   // diagnostic builds only: the whole FPS chain up front, no FPS workgroups beside the MLPs
    rc = gp_launch_fps_chain(pts, B, 4, c.nin, c.mout, (int* const*)c.fidx, (float* const*)c.nxyz, st);
    constexpr bool side = false;
#else
    rc = gp_launch_fps_chain(pts, B, 1, c.nin, c.mout, (int* const*)c.fidx, (float* const*)c.nxyz, st);
    constexpr bool side = true;
#endif
    if (rc) return rc;
    for (int l = 0; l < 5; ++l) {
        const float* fprev = l == 0 ? nullptr : reinterpret_cast<const float*>(c.ws + c.L.feat[l - 1]);
        float* out = l < 4 ? reinterpret_cast<float*>(c.ws + c.L.feat[l]) : feat;
        rc = run_sa_level(c, l, l == 0 ? 0 : kCout[l - 1], fprev, out, side, st);
        if (rc) return rc;
    }
    return GP_OK;
}

extern "C" int gp_encoder_fps(const float* pts, int B, int N, void* workspace, size_t workspace_bytes, hipStream_t st) {
    const float dummy = 0.f;
    const int64_t tab = 0;
    int rc = enc_check(&dummy, &tab, pts, B, N, workspace, workspace_bytes);
    if (rc) return rc;
    const EncCtx c = enc_ctx(nullptr, nullptr, pts, B, N, workspace);
    return gp_launch_fps_chain(pts, B, 4, c.nin, c.mout, (int* const*)c.fidx, (float* const*)c.nxyz, st);
}

// The geometry of every level in one pass: the FPS chain of all four levels, then the ball lists of both
// radii per level. Another encoder of the same points then skips all of it (gp_encoder_forward_geom).
extern "C" int gp_encoder_geometry_levels(const float* pts, int B, int N, void* workspace, size_t workspace_bytes,
                                          int first, int last, hipStream_t st) {
    const float dummy = 0.f;
    const int64_t tab = 0;
    int rc = enc_check(&dummy, &tab, pts, B, N, workspace, workspace_bytes);
    if (rc) return rc;
    GP_REQUIRE(first >= 0 && first < last && last <= 4, "encoder_geometry_levels: levels [%d, %d) of 4", first, last);
    const EncCtx c = enc_ctx(nullptr, nullptr, pts, B, N, workspace);
    // levels first.. sample from level first-1's centroids (already in the workspace)
    rc = gp_launch_fps_chain(first == 0 ? pts : c.nxyz[first - 1], B, last - first, c.nin + first, c.mout + first,
                             (int* const*)c.fidx + first, (float* const*)c.nxyz + first, st);
    if (rc) return rc;
    for (int l = first; l < last; ++l) {
        const float* xyz_prev = l == 0 ? pts : c.nxyz[l - 1];
        rc = gp_launch_ball_query2(B, c.nin[l], kNpoint[l], kRadius[l][0], kRadius[l][1], kNs[0], kNs[1], c.nxyz[l],
                                   xyz_prev, reinterpret_cast<int*>(c.ws + c.L.ball[l][0]),
                                   reinterpret_cast<int*>(c.ws + c.L.ball[l][1]), st);
        if (rc) return rc;
    }
    return GP_OK;
}

// gp_encoder_forward over geometry that gp_encoder_geometry left in `geometry` (a workspace of the same
// (B, N) layout; it may be `workspace` itself): only the per-level MLPs run, their scratch in `workspace`.
extern "C" int gp_encoder_geometry(const float* pts, int B, int N, void* workspace, size_t workspace_bytes,
                                   hipStream_t st) {
    return gp_encoder_geometry_levels(pts, B, N, workspace, workspace_bytes, 0, 4, st);
}

extern "C" int gp_encoder_forward_geom_levels(const float* wbuf, const int64_t* layer_off, const float* pts, int B,
                                              int N, const void* geometry, void* workspace, size_t workspace_bytes,
                                              float* feat, int first, int last, hipStream_t st) {
    int rc = enc_check(wbuf, layer_off, pts, B, N, workspace, workspace_bytes);
    if (rc) return rc;
    GP_REQUIRE(feat && geometry, "encoder_forward_geom: null feat or geometry");
    GP_REQUIRE(first >= 0 && first < last && last <= 5, "encoder_forward_geom_levels: levels [%d, %d) of 5", first, last);
    const EncCtx c = enc_ctx(wbuf, layer_off, pts, B, N, workspace, const_cast<void*>(geometry));
    for (int l = first; l < last; ++l) {
        const float* fprev = l == 0 ? nullptr : reinterpret_cast<const float*>(c.ws + c.L.feat[l - 1]);
        float* out = l < 4 ? reinterpret_cast<float*>(c.ws + c.L.feat[l]) : feat;
        rc = run_sa_level(c, l, l == 0 ? 0 : kCout[l - 1], fprev, out, false, st);
        if (rc) return rc;
    }
    return GP_OK;
}

extern "C" int gp_encoder_forward_geom(const float* wbuf, const int64_t* layer_off, const float* pts, int B, int N,
                                       const void* geometry, void* workspace, size_t workspace_bytes, float* feat,
                                       hipStream_t st) {
    return gp_encoder_forward_geom_levels(wbuf, layer_off, pts, B, N, geometry, workspace, workspace_bytes, feat, 0, 5,
                                          st);
}

static int sa_level_impl(const float* wbuf, const int64_t* layer_off, int level, int c_prev, const float* pts, int B,
                         int N, const float* feat_prev, const void* geometry, void* workspace, size_t workspace_bytes,
                         float* out, hipStream_t st) {
    int rc = enc_check(wbuf, layer_off, pts, B, N, workspace, workspace_bytes);
    if (rc) return rc;
    GP_REQUIRE(level >= 0 && level < 5 && out, "sa_level: level %d out of range or null out", level);
    GP_REQUIRE(level == 0 ? (c_prev % 16 == 0 && c_prev >= 0 && c_prev <= 1024) : c_prev == kCout[level - 1],
               "sa_level: level %d takes c_prev = %d (got %d)", level, level ? kCout[level - 1] : 0, c_prev);
    GP_REQUIRE(c_prev == 0 || feat_prev, "sa_level: c_prev %d needs feat_prev", c_prev);
    const EncCtx c = enc_ctx(wbuf, layer_off, pts, B, N, workspace, const_cast<void*>(geometry));
    return run_sa_level(c, level, c_prev, feat_prev, out, false, st);
}

extern "C" int gp_sa_level(const float* wbuf, const int64_t* layer_off, int level, int c_prev, const float* pts, int B,
                           int N, const float* feat_prev, void* workspace, size_t workspace_bytes, float* out,
                           hipStream_t st) {
    return sa_level_impl(wbuf, layer_off, level, c_prev, pts, B, N, feat_prev, nullptr, workspace, workspace_bytes, out,
                         st);
}

// gp_sa_level over the geometry gp_encoder_geometry left in `geometry` (FPS indices, centroids and both ball lists of
// every level; it may be `workspace` itself): no ball query runs, the level's scratch goes to `workspace`. Two fused
// encoders of the same points (the ScoreNet's and the EnergyNet's) then share one geometry pass, as the Light
// encoders do (gp_encoder_forward_geom).
extern "C" int gp_sa_level_geom(const float* wbuf, const int64_t* layer_off, int level, int c_prev, const float* pts,
                                int B, int N, const float* feat_prev, const void* geometry, void* workspace,
                                size_t workspace_bytes, float* out, hipStream_t st) {
    GP_REQUIRE(geometry, "sa_level_geom: null geometry");
    return sa_level_impl(wbuf, layer_off, level, c_prev, pts, B, N, feat_prev, geometry, workspace, workspace_bytes,
                         out, st);
}
