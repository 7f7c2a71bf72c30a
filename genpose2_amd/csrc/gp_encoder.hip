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
#include "gp_common.h"

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
#else
#define SA_MARK(k) ((void)0)
#endif

constexpr int SA_THREADS = 256;

// One layer for the CTW column tiles [cbase, cbase+CTW) of this wave and the output tiles
// wt*TC, wt*TC + WT*TC, ... (WT = waves sharing the columns). Layers narrower than 4*TC output
// tiles split the workgroup's columns over waves instead of leaving waves idle.
template <int CT, int CTW, int TC, int SPAN>
__device__ __forceinline__ void sa_layer(const SAArgs& a, f32x4* lds, int L, int b, int col0, int cbase,
                                         int wt, int WT) {
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
                    v = f32x4{fsub(px[0], cc[0]), fsub(px[1], cc[1]), fsub(px[2], cc[2]), 0.f};
                } else {       // GroupAll keeps raw xyz (pointnet2_utils.py:316-324)
                    v = f32x4{px[0], px[1], px[2], 0.f};
                }
            }
            bx[c] = v;
        }
    }
    for (int T0 = wt * TC; T0 < NT; T0 += WT * TC) {
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
                af[t] = (T0 + t < NT) ? ldbuf4(W, voff, ((T0 + t) * KG + g) * 1024) : f32x4{0.f, 0.f, 0.f, 0.f};
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
        // two-slot ping-pong: the operands of k-group g+1 are in flight while g computes;
        // sched_barrier keeps the compiler from sinking the loads back next to their MFMAs
        f32x4 aA[TC], bA[CTW], aB[TC], bB[CTW];
        fetch(0, aA, bA);
        for (int g = 0; g < KG; g += 2) {
            if (g + 1 < KG) fetch(g + 1, aB, bB);
            __builtin_amdgcn_sched_barrier(0);
            compute(aA, bA);
            if (g + 2 < KG) fetch(g + 2, aA, bA);
            __builtin_amdgcn_sched_barrier(0);
            if (g + 1 < KG) compute(aB, bB);
        }
#pragma unroll
        for (int t = 0; t < TC; ++t) {
            const int T = T0 + t;
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
                        v = f32x4{fmaxf(v.x, w2.x), fmaxf(v.y, w2.y), fmaxf(v.z, w2.z), fmaxf(v.w, w2.w)};
                    }
#pragma unroll
                    for (int off = 8; off >= 1; off >>= 1) {
                        v.x = fmaxf(v.x, __shfl_xor(v.x, off, 64));
                        v.y = fmaxf(v.y, __shfl_xor(v.y, off, 64));
                        v.z = fmaxf(v.z, __shfl_xor(v.z, off, 64));
                        v.w = fmaxf(v.w, __shfl_xor(v.w, off, 64));
                    }
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
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q = lane >> 4, nn = lane & 15;
    const int NT0 = a.nt[0], KG0 = a.kg[0], gx = a.c_prev >> 4;
    const f32x4* w0 = reinterpret_cast<const f32x4*>(a.w[0]);
    int pcol[CT], mcol[CT];
    bool ok[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int col = col0 + ct * 16 + nn;
        ok[ct] = col < a.cols;
        const int m = ok[ct] ? col / a.ns : 0, s = ok[ct] ? col - (col / a.ns) * a.ns : 0;
        mcol[ct] = m;
        pcol[ct] = ok[ct] ? a.nbr[((size_t)b * a.m + m) * a.ns + s] : 0;
    }
    for (int pr = wid; pr < NT0 * CT; pr += 4) {
        const int T = pr / CT, ct = pr - (pr / CT) * CT;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (ok[ct]) {
            const f32x4 qv = ld4(a.qin + ((size_t)b * a.n_prev + pcol[ct]) * a.q_stride + a.q_off + 16 * T + 4 * q);
            const float* cc = a.cent + ((size_t)b * a.m + mcol[ct]) * 3;
            const float cx = cc[0], cy = cc[1], cz = cc[2];
            float r[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f32x4 wx = w0[(T * KG0 + gx) * 64 + 4 * q + j];   // W0[16T+4q+j][c_prev + 0..2]
                r[j] = fmaxf(qv[j] - ((wx.x * cx + wx.y * cy) + wx.z * cz), 0.f);
            }
            v = f32x4{r[0], r[1], r[2], r[3]};
        }
        lds[(T * CT + ct) * 64 + lane] = v;
    }
}

template <int CT, int TC, int SPAN>
__global__ __launch_bounds__(SA_THREADS, 2) void sa_branch_kernel(SAArgs a) {
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
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
            sa_layer<CT, CT, TC, SPAN>(a, lds, L, b, col0, 0, wt, WT);
        } else if (wc == 2) {
            if constexpr (CT >= 2 && CT / 2 >= 1) sa_layer<CT, CT / 2, TC, (SPAN <= CT / 2 ? SPAN : 1)>(
                a, lds, L, b, col0, (wid % 2) * (CT / 2), wt, WT);
        } else {
            if constexpr (CT >= 4) sa_layer<CT, CT / 4, TC, 1>(a, lds, L, b, col0, (wid % 4) * (CT / 4), wt, WT);
        }
        SA_MARK(1 + 2 * L);
        __syncthreads();
        SA_MARK(2 + 2 * L);
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
static int launch_sa(const SAArgs& a, int B, hipStream_t st) {
    size_t buf0 = 0, buf1 = 0;
    if (a.nlayers >= 2) buf0 = (size_t)CT * 16 * a.nt[0] * 16;                 // floats
    if (a.nlayers >= 3) buf1 = (size_t)CT * 16 * a.nt[1] * 16;
    SAArgs args = a;
    args.buf1_off = (int)(buf0 / 4);
    const size_t lds = (buf0 + buf1) * sizeof(float);
    if (lds > 160 * 1024) {
        gp_set_error("sa_branch_kernel: LDS %zu bytes exceeds 160 KiB", lds);
        return GP_ERR_UNSUPPORTED;
    }
    const int blocks = (a.cols + CT * 16 - 1) / (CT * 16);
    const int tpc = a.ns / 16;
    const int span = tpc < CT ? tpc : CT;
    if (span == 1)
        hipLaunchKernelGGL((sa_branch_kernel<CT, 4, 1>), dim3(blocks, B), dim3(SA_THREADS), lds, st, args);
    else if (span == 2)
        hipLaunchKernelGGL((sa_branch_kernel<CT, 4, 2>), dim3(blocks, B), dim3(SA_THREADS), lds, st, args);
    else if (span == 4 && CT >= 4)
        hipLaunchKernelGGL((sa_branch_kernel<(CT >= 4 ? CT : 4), 4, 4>), dim3(blocks, B), dim3(SA_THREADS), lds, st,
                           args);
    else {
        gp_set_error("sa_branch_kernel: unsupported span %d", span);
        return GP_ERR_UNSUPPORTED;
    }
    return gp_check_launch("sa_branch_kernel");
}

extern "C" int gp_encoder_forward(const float* wbuf, const int64_t* layer_off, const float* pts, int B, int N,
                                  void* workspace, size_t workspace_bytes, float* feat, hipStream_t st) {
    GP_REQUIRE(wbuf && layer_off && pts && workspace && feat, "encoder_forward: null pointer");
    GP_REQUIRE(B >= 1 && N >= kNpoint[0] && N <= 8192, "encoder_forward: need 1<=b and 512<=n<=8192 (b=%d n=%d)",
               B, N);
    const EncLayout L = enc_layout(B, N);
    GP_REQUIRE(workspace_bytes >= L.total, "encoder_forward: workspace %zu < %zu", workspace_bytes, L.total);
    char* ws = static_cast<char*>(workspace);
    int* fidx[4];
    float* nxyz[4];
    int nin[4], mout[4];
    for (int l = 0; l < 4; ++l) {
        fidx[l] = reinterpret_cast<int*>(ws + L.fps[l]);
        nxyz[l] = reinterpret_cast<float*>(ws + L.nxyz[l]);
        nin[l] = l == 0 ? N : kNpoint[l - 1];
        mout[l] = kNpoint[l];
    }
    int rc = gp_launch_fps_chain(pts, B, 4, nin, mout, fidx, nxyz, st);
    if (rc) return rc;
    for (int l = 0; l < 5; ++l) {
        const float* xyz_prev = l == 0 ? pts : nxyz[l - 1];
        const int n_prev = l == 0 ? N : kNpoint[l - 1];
        int* b0 = nullptr;
        int* b1 = nullptr;
        if (l < 4) {
            b0 = reinterpret_cast<int*>(ws + L.ball[l][0]);
            b1 = reinterpret_cast<int*>(ws + L.ball[l][1]);
            rc = gp_launch_ball_query2(B, n_prev, kNpoint[l], kRadius[l][0], kRadius[l][1], kNs[0], kNs[1], nxyz[l],
                                       xyz_prev, b0, b1, st);
            if (rc) return rc;
        }
        // layer 0 once per input point for both branches (levels 0-3)
        float* qbuf = l < 4 ? reinterpret_cast<float*>(ws + L.proj[l]) : nullptr;
        if (l < 4) {
            int q_off = 0;
            for (int br = 0; br < 2; ++br) {
                SAArgs pa = {};
                pa.n_prev = n_prev;
                pa.c_prev = l == 0 ? 0 : kCout[l - 1];
                pa.m = 1;
                pa.ns = n_prev;
                pa.cols = n_prev;
                pa.xyz_prev = xyz_prev;
                pa.feat_prev = l == 0 ? nullptr : reinterpret_cast<const float*>(ws + L.feat[l - 1]);
                pa.nlayers = 1;
                const int64_t* o = layer_off + ((l * 2 + br) * 3 + 0) * 2;
                GP_REQUIRE(o[0] >= 0 && o[1] >= 0, "encoder_forward: missing layer %d/%d/0", l, br);
                pa.w[0] = wbuf + o[0];
                pa.bias[0] = wbuf + o[1];
                pa.kg[0] = (pa.c_prev + 16) / 16;
                pa.nt[0] = pad16(kWidths[l][br][1]) / 16;
                pa.proj_out = qbuf;
                pa.q_stride = proj_stride(l);
                pa.q_off = q_off;
                pa.tag = 16 + l * 2 + br;
                q_off += pad16(kWidths[l][br][1]);
                rc = launch_sa<4>(pa, B, st);
                if (rc) return rc;
            }
        }
        float* out = l < 4 ? reinterpret_cast<float*>(ws + L.feat[l]) : feat;
        if (l == 4) {  // group-all pools with atomicMax when a centroid spans workgroups
            if (hipMemsetAsync(out, 0, sizeof(float) * B * kCout[4], st) != hipSuccess)
                return gp_check_launch("encoder memset");
        }
        int out_off = 0;
        for (int br = 0; br < 2; ++br) {
            SAArgs a = {};
            a.n_prev = n_prev;
            a.c_prev = l == 0 ? 0 : kCout[l - 1];
            a.m = l < 4 ? kNpoint[l] : 1;
            a.ns = l < 4 ? kNs[br] : n_prev;
            a.cols = a.m * a.ns;
            a.xyz_prev = xyz_prev;
            a.feat_prev = l == 0 ? nullptr : reinterpret_cast<const float*>(ws + L.feat[l - 1]);
            a.cent = l < 4 ? nxyz[l] : nullptr;
            a.nbr = l < 4 ? (br == 0 ? b0 : b1) : nullptr;
            a.nlayers = l < 4 ? 3 : 2;
            for (int i = 0; i < a.nlayers; ++i) {
                const int64_t* o = layer_off + ((l * 2 + br) * 3 + i) * 2;
                GP_REQUIRE(o[0] >= 0 && o[1] >= 0, "encoder_forward: missing layer %d/%d/%d", l, br, i);
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
                gp_set_error("encoder_forward: nsample %d not a multiple of 16", a.ns);
                return GP_ERR_UNSUPPORTED;
            }
            // level 3 at 32 columns (its 640-channel LDS ping-pong), GroupAll split over 2 workgroups
            // per (object, branch) with atomicMax pooling (4x the workgroups of one per object)
            rc = (l >= 3) ? launch_sa<2>(a, B, st) : launch_sa<4>(a, B, st);
            if (rc) return rc;
        }
    }
    return GP_OK;
}
