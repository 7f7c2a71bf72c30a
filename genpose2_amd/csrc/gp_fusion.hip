// Blocks of the DINO-pointwise fused encoder (Pointnet2ClsMSGFus, networks/pts_encoder/pointnet2.py:255-388)
// that sit between its SA levels, for gfx950:
//   * token linears (nn.Linear / Conv1d k=1, BN folded on the host) as exact-fp32 MFMA GEMMs;
//   * residual + LayerNorm (TransformerBlockWithRelativePE, attention.py:505-533);
//   * the relative-PE bias of EfficientRelativePositionalEncoding (attention.py:680-735), all 8 heads of
//     a point pair from one evaluation of its distance / direction MLPs;
//   * biased multi-head attention (MultiheadAttentionWithRelativePE, attention.py:436-488), flash-style:
//     QK^T and PV on exact-fp32 MFMA, K / V staged in LDS, an online softmax;
//   * GatedAttentionFusion's channel / spatial attention and gating (attention.py:284-325).
// Token tensors are point-major (b, n, C): the reference's (b, C, n) transposed, so one token's channels
// are contiguous and every linear is a row-major GEMM over b*n rows.
#include "gp_common.h"
#include "gp_head.h"   // split-f16 helpers: f16x8, mfma_h, exp2i, ilog2f, rows_max

constexpr int FUS_THREADS = 256;
#define FUS_TRY(x)                        \
    do {                                  \
        const int rc_ = (x);              \
        if (rc_ != GP_OK) return rc_;     \
    } while (0)
constexpr int FUS_HEADS = 8;

__device__ __forceinline__ float sigmoidf(float v) { return 1.0f / (1.0f + expf(-v)); }

// ============================================================================ token linear (MFMA)
// y[r, o] = act(sum_k x[r, k] w[o, k] + bias[o]). 4 waves as 2 (tokens) x 2 (outputs); a wave owns TM
// token tiles x TN output tiles of 16. MFMA A = w rows (output channels), B = x rows (tokens): lane
// (q, r) feeds float4 k-slices 16g + 4q .. +3 of row r of both, so one 16-deep k-group is 4 MFMAs per
// tile pair and the accumulator holds 4 consecutive output channels of one token (a float4 store).
template <int TM, int TN, int ACT>
__global__ __launch_bounds__(FUS_THREADS) void linear_kernel(const float* __restrict__ x, int ldx, int m, int k,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias, int n,
                                                             float* __restrict__ y, int ldy) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q = lane >> 4, r = lane & 15;
    const int tok0 = blockIdx.x * (32 * TM) + (wid & 1) * (16 * TM);
    const int ot0 = blockIdx.y * (2 * TN) + (wid >> 1) * TN;   // first output tile of this wave
    const int ntile = n >> 4;
    const float* xp[TM];
    const float* wp[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) xp[t] = x + (size_t)min(tok0 + 16 * t + r, m - 1) * ldx + 4 * q;
#pragma unroll
    for (int u = 0; u < TN; ++u) wp[u] = w + (size_t)(16 * min(ot0 + u, ntile - 1) + r) * k + 4 * q;
    f32x4 acc[TN][TM];
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int t = 0; t < TM; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int KG = k >> 4;
    f32x4 xa[TM], wa[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) xa[t] = ld4(xp[t]);
#pragma unroll
    for (int u = 0; u < TN; ++u) wa[u] = ld4(wp[u]);
    for (int g = 0; g < KG; ++g) {
        f32x4 xb[TM], wb[TN];
        const int gn = (g + 1 < KG ? g + 1 : g) * 16;
#pragma unroll
        for (int t = 0; t < TM; ++t) xb[t] = ld4(xp[t] + gn);
#pragma unroll
        for (int u = 0; u < TN; ++u) wb[u] = ld4(wp[u] + gn);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int u = 0; u < TN; ++u)
#pragma unroll
                for (int t = 0; t < TM; ++t) acc[u][t] = mfma4(wa[u][j], xa[t][j], acc[u][t]);
#pragma unroll
        for (int t = 0; t < TM; ++t) xa[t] = xb[t];
#pragma unroll
        for (int u = 0; u < TN; ++u) wa[u] = wb[u];
    }
#pragma unroll
    for (int u = 0; u < TN; ++u) {
        const int T = ot0 + u;
        if (T >= ntile) continue;
        const f32x4 bv = bias ? ld4(bias + 16 * T + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            const int tok = tok0 + 16 * t + r;
            if (tok >= m) continue;
            f32x4 v = acc[u][t] + bv;
            if (ACT == 1) v = relu4(v);
            if (ACT == 2) v = f32x4{sigmoidf(v.x), sigmoidf(v.y), sigmoidf(v.z), sigmoidf(v.w)};
            st4(y + (size_t)tok * ldy + 16 * T + 4 * q, v);
        }
    }
}

// LDS-tiled form for large token counts: a workgroup owns 128 tokens x (32 * WN) outputs, 4 waves as 2 x 2
// of 64 tokens x (16 * WN) outputs, so every fragment read from LDS feeds 4 (or WN) MFMAs and every
// operand element is fetched from L2 once per workgroup. K advances 32 per stage through two LDS buffers
// (one barrier per stage; the next stage's global loads are in flight while this stage computes). Both
// operands are stored in LDS in fragment order [k-group][q][row] x float4: a lane's ds_read_b128 of row r,
// k-slice q lands in a distinct bank group (conflict-free).
constexpr int LK_BM = 128, LK_KC = 32;
template <int WN, int ACT>
__global__ __launch_bounds__(FUS_THREADS, 2) void linear_lds_kernel(const float* __restrict__ x, int ldx, int m, int k,
                                                                    const float* __restrict__ w,
                                                                    const float* __restrict__ bias, int n,
                                                                    float* __restrict__ y, int ldy) {
    constexpr int BN = 32 * WN;                        // outputs per workgroup
    constexpr int XF4 = LK_BM * LK_KC / 4, WF4 = BN * LK_KC / 4;   // float4s per stage
    __shared__ f32x4 sx[2][XF4];
    __shared__ f32x4 sw[2][WF4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int q = lane >> 4, r = lane & 15;
    const int tok0 = blockIdx.x * LK_BM, out0 = blockIdx.y * BN;
    const int ntile = n >> 4;
    // staging: float4 e of a stage = (row, k-group g, slice qq); loads are row-major coalesced
    constexpr int XPT = XF4 / FUS_THREADS, WPT = (WF4 + FUS_THREADS - 1) / FUS_THREADS;
    const float* xs[XPT];
    int xdst[XPT];
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
        const int e = tid + u * FUS_THREADS, row = e >> 3, g = (e >> 2) & 1, qq = e & 3;
        xs[u] = x + (size_t)min(tok0 + row, m - 1) * ldx + 16 * g + 4 * qq;
        xdst[u] = (g * 4 + qq) * LK_BM + row;
    }
    const float* ws[WPT];
    int wdst[WPT];
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
        const int e = min(tid + u * FUS_THREADS, WF4 - 1), row = e >> 3, g = (e >> 2) & 1, qq = e & 3;
        ws[u] = w + (size_t)min(out0 + row, n - 1) * k + 16 * g + 4 * qq;
        wdst[u] = (g * 4 + qq) * BN + row;
    }
    f32x4 px[XPT], pw[WPT];
    auto fetch = [&](int kk) {
#pragma unroll
        for (int u = 0; u < XPT; ++u) px[u] = ld4(xs[u] + kk);
#pragma unroll
        for (int u = 0; u < WPT; ++u) pw[u] = ld4(ws[u] + kk);
    };
    auto stash = [&](int b) {
#pragma unroll
        for (int u = 0; u < XPT; ++u) sx[b][xdst[u]] = px[u];
#pragma unroll
        for (int u = 0; u < WPT; ++u)
            if (WF4 % FUS_THREADS == 0 || tid + u * FUS_THREADS < WF4) sw[b][wdst[u]] = pw[u];
    };
    const int wm = wid & 1, wn = wid >> 1;
    f32x4 acc[WN][4];
#pragma unroll
    for (int a = 0; a < WN; ++a)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int stages = k / LK_KC;
    fetch(0);
    stash(0);
    __syncthreads();
    for (int s = 0; s < stages; ++s) {
        const int b = s & 1;
        if (s + 1 < stages) fetch((s + 1) * LK_KC);
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x4 af[WN], bf[4];
#pragma unroll
            for (int a = 0; a < WN; ++a) af[a] = sw[b][(g * 4 + q) * BN + wn * 16 * WN + 16 * a + r];
#pragma unroll
            for (int t = 0; t < 4; ++t) bf[t] = sx[b][(g * 4 + q) * LK_BM + wm * 64 + 16 * t + r];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int a = 0; a < WN; ++a)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[a][t] = mfma4(af[a][j], bf[t][j], acc[a][t]);
        }
        if (s + 1 < stages) stash(b ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < WN; ++a) {
        const int T = (out0 >> 4) + wn * WN + a;
        if (T >= ntile) continue;
        const f32x4 bv = bias ? ld4(bias + 16 * T + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int tok = tok0 + wm * 64 + 16 * t + r;
            if (tok >= m) continue;
            f32x4 v = acc[a][t] + bv;
            if (ACT == 1) v = relu4(v);
            if (ACT == 2) v = f32x4{sigmoidf(v.x), sigmoidf(v.y), sigmoidf(v.z), sigmoidf(v.w)};
            st4(y + (size_t)tok * ldy + 16 * T + 4 * q, v);
        }
    }
}

template <int WN, int ACT>
static void launch_linear_lds(const float* x, int ldx, int m, int k, const float* w, const float* bias, int n, float* y,
                              int ldy, hipStream_t st) {
    const dim3 grid((m + LK_BM - 1) / LK_BM, (n + 32 * WN - 1) / (32 * WN));
    hipLaunchKernelGGL((linear_lds_kernel<WN, ACT>), grid, dim3(FUS_THREADS), 0, st, x, ldx, m, k, w, bias, n, y, ldy);
}

template <int TN, int ACT, int TM = 2>
static void launch_linear(const float* x, int ldx, int m, int k, const float* w, const float* bias, int n, float* y,
                          int ldy, hipStream_t st) {
    const dim3 grid((m + 32 * TM - 1) / (32 * TM), ((n >> 4) + 2 * TN - 1) / (2 * TN));
    hipLaunchKernelGGL((linear_kernel<TM, TN, ACT>), grid, dim3(FUS_THREADS), 0, st, x, ldx, m, k, w, bias, n, y, ldy);
}

template <int TN>
static void launch_linear_act(int act, const float* x, int ldx, int m, int k, const float* w, const float* bias, int n,
                              float* y, int ldy, hipStream_t st) {
    if (act == 0) launch_linear<TN, 0>(x, ldx, m, k, w, bias, n, y, ldy, st);
    else if (act == 1) launch_linear<TN, 1>(x, ldx, m, k, w, bias, n, y, ldy, st);
    else launch_linear<TN, 2>(x, ldx, m, k, w, bias, n, y, ldy, st);
}

extern "C" int gp_linear(const float* x, int ldx, int m, int k, const float* w, const float* bias, int n, int act,
                         float* y, int ldy, hipStream_t st) {
    GP_REQUIRE(x && w && y && m >= 0, "linear: null pointer");
    GP_REQUIRE(k >= 16 && k % 16 == 0 && n >= 16 && n % 16 == 0, "linear: k=%d and n=%d must be multiples of 16", k, n);
    GP_REQUIRE(ldx >= k && ldy >= n && ldx % 4 == 0 && ldy % 4 == 0, "linear: strides ldx=%d ldy=%d", ldx, ldy);
    GP_REQUIRE(((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)bias) % 16 == 0,
               "linear: pointers must be 16-byte aligned");
    GP_REQUIRE(act >= 0 && act <= 2, "linear: act %d", act);
    if (!m) return GP_OK;
    if (m >= 1024 && k % LK_KC == 0 && n >= 64) {   // LDS-tiled: 128 tokens x 128 (or 64) outputs per workgroup
        const bool wide = n % 128 == 0;   // else 64-output columns (n = 96, 192, 288: less padding)
#define GP_LIN_LDS(WN)                                                                                     \
        if (act == 0) launch_linear_lds<WN, 0>(x, ldx, m, k, w, bias, n, y, ldy, st);                      \
        else if (act == 1) launch_linear_lds<WN, 1>(x, ldx, m, k, w, bias, n, y, ldy, st);                 \
        else launch_linear_lds<WN, 2>(x, ldx, m, k, w, bias, n, y, ldy, st);
        if (wide) { GP_LIN_LDS(4) } else { GP_LIN_LDS(2) }
#undef GP_LIN_LDS
        return gp_check_launch("linear_lds_kernel");
    }
    // few tokens (the GroupAll level's one token per object): 32 x 32 tiles, so that the grid still covers the
    // chip (m = 256, n = 1024: 256 workgroups instead of 32)
    if ((long long)((m + 63) / 64) * ((n + 127) / 128) < 256 && n % 32 == 0) {
        if (act == 0) launch_linear<1, 0, 1>(x, ldx, m, k, w, bias, n, y, ldy, st);
        else if (act == 1) launch_linear<1, 1, 1>(x, ldx, m, k, w, bias, n, y, ldy, st);
        else launch_linear<1, 2, 1>(x, ldx, m, k, w, bias, n, y, ldy, st);
        return gp_check_launch("linear_kernel");
    }
    // output tiles per wave: the widest that divides n into whole workgroup columns
    if (n % 128 == 0) launch_linear_act<4>(act, x, ldx, m, k, w, bias, n, y, ldy, st);
    else if (n % 96 == 0) launch_linear_act<3>(act, x, ldx, m, k, w, bias, n, y, ldy, st);
    else if (n % 64 == 0) launch_linear_act<2>(act, x, ldx, m, k, w, bias, n, y, ldy, st);
    else launch_linear_act<1>(act, x, ldx, m, k, w, bias, n, y, ldy, st);
    return gp_check_launch("linear_kernel");
}

// ============================================================================ token linear (split-f16 MFMA)
// The same y = act(x W^T + b) with each fp32 operand split into f16 hi / lo planes at a power-of-two scale
// (W: one exponent per matrix, packed on the host by pack.pack_h16_fragments; x: per token from its row
// max |x|, split on the way into LDS) and three v_mfma_f32_16x16x32_f16 products (hi.hi + hi.lo + lo.hi)
// accumulated in fp32 -- the encoder's split arithmetic (tok_split_gemm_kernel), 16x the MACs per MFMA of
// the fp32 path. Workgroup: 64*WO outputs x 16*JT*(8/WO) tokens, 8 waves of 64 outputs x 16*JT tokens, two
// LDS stages of one 32-deep chunk, one barrier per chunk. JT = 8 (WO = 4): every A fragment read from LDS
// feeds 8 token tiles instead of 4, so the LDS traffic per MFMA drops by a third.
constexpr int SL_THREADS = 512;
#ifndef SL_DMA
#define SL_DMA 1   // A planes global -> LDS by global_load_lds_dwordx4 (0: through registers and ds_write)
#endif
#ifndef SL_DIAG
#define SL_DIAG 0     // timing diagnostics of linear_split_kernel's chunk loop (wrong results): see the loop
#endif
// 16 bytes per lane from global memory straight into LDS at lds + 16 * lane (lds wave-uniform)
__device__ __forceinline__ void lds_dma16(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
// every outstanding memory operation of the wave has completed (the LDS copies above included)
__device__ __forceinline__ void wait_all_mem() { __builtin_amdgcn_s_waitcnt(0); }
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
struct SplitLinArgs {
    const float* x;
    int ldx, m, k;
    const float* rmax;    // per-token max |x| (m)
    const int32_t* w;     // [ew, 0, 0, 0] (W was scaled by 2^ew), then the planes [tile][chunk][plane][lane] f16x8
    const float* bias;
    int n;
    float* y;
    int ldy;
    unsigned* ymax;       // or null: per-row max |y| (bits of a float >= 0 order as unsigned: atomicMax)
    // IM = 1 (implicit im2col of a 3x3 / pad 1 conv): x is the (objects, g*g pixels, d) feature map, row r = pixel
    // (r / gg, r % gg) of object r / gg, k = 9 d in position-major order (k index = (ky * 3 + kx) * d + channel):
    // chunk c reads the 32 channels (c % d32) * 32.. of neighbour c / d32 -- zeros outside the grid
    int im_g, im_d32;
};
template <int WO, int JT = 4>
constexpr size_t sl_lds_bytes() {
    return 2 * (size_t)(4 * WO + JT * (8 / WO)) * 2048 + sizeof(int) * 16 * JT * (8 / WO);
}

__global__ __launch_bounds__(256) void fus_rowmax_kernel(const float* __restrict__ x, int ldx, int m, int k,
                                                         float* __restrict__ rmax) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= m) return;
    const float* row = x + (size_t)r * ldx;
    float v = 0.f;
    for (int c = 4 * lane; c < k; c += 256) {
        const f32x4 t = ld4(row + c);
        v = fmaxf(v, fmaxf(fmaxf(fabsf(t.x), fabsf(t.y)), fmaxf(fabsf(t.z), fabsf(t.w))));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    if (lane == 0) rmax[r] = v;
}

template <int WO, int ACT, int JT = 4, int IM = 0>
__global__ __launch_bounds__(SL_THREADS) void linear_split_kernel(SplitLinArgs a) {
    // RU: (token row, k-group pair) items per thread. Item (row br, k-groups bq and bq + 4) fills one 16-byte
    // B-fragment entry per plane, and a wave's 16-lane store phases cover 16 rows of one k-group: entries of
    // distinct banks (8 threads a row writing 8-byte halves conflicted 4-way: 43 % of LDS cycles)
    constexpr int WT = 8 / WO, BM = 16 * JT * WT, RU = BM / 128;
    constexpr int NA = 4 * WO * 128, NB = JT * WT * 128;   // f16x8 fragments per stage
    extern __shared__ __attribute__((aligned(16))) f16x8 sl_lds[];
    auto sA = [&](int st) { return sl_lds + st * (NA + NB); };
    auto sB = [&](int st) { return sl_lds + st * (NA + NB) + NA; };
    int* eT = reinterpret_cast<int*>(sl_lds + 2 * (NA + NB));
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, nn = lane & 15;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0 = blockIdx.y * BM, T0 = blockIdx.x * 4 * WO;
    const int KC = a.k >> 5;
    const int ew = a.w[0];
    const f16x8* W = reinterpret_cast<const f16x8*>(a.w + 4);
    int row[RU], brow[RU], bq[RU];
    float sc[RU];
    int py[RU], px[RU];   // IM: the row's pixel
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        const int idx = tid + SL_THREADS * u;
        brow[u] = (idx & 15) + 16 * (idx >> 6);
        bq[u] = (idx >> 4) & 3;
        row[u] = m0 + brow[u];
        const float mx = row[u] < a.m ? a.rmax[row[u]] : 0.f;
        const int E = mx > 1e-30f ? ilog2f(mx) : -100;
        sc[u] = exp2i(14 - E);
        if (bq[u] == 0) eT[brow[u]] = E;
        if constexpr (IM) {
            const int p = row[u] % (a.im_g * a.im_g);
            py[u] = p / a.im_g;
            px[u] = p - py[u] * a.im_g;
        }
    }
    // x of chunk c for item u: its two 16-byte k-groups (IM: the neighbour pixel's channels, zeros off the grid)
    auto xload = [&](int c, int u, f32x4& v0, f32x4& v1) {
        if constexpr (IM) {
            const int k9 = c / a.im_d32, cc = c - k9 * a.im_d32;   // wave-uniform
            const int dy = k9 / 3 - 1, dx = k9 - (k9 / 3) * 3 - 1;
            const int yy = py[u] + dy, xx = px[u] + dx;
            const bool in = row[u] < a.m && yy >= 0 && yy < a.im_g && xx >= 0 && xx < a.im_g;
            const float* xr = a.x + (size_t)(in ? row[u] + dy * a.im_g + dx : 0) * a.ldx + 32 * cc + 4 * bq[u];
            v0 = in ? ld4(xr) : f32x4{0.f, 0.f, 0.f, 0.f};
            v1 = in ? ld4(xr + 16) : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
            const float* xr = a.x + (size_t)row[u] * a.ldx + 32 * c + 4 * bq[u];
            v0 = row[u] < a.m ? ld4(xr) : f32x4{0.f, 0.f, 0.f, 0.f};
            v1 = row[u] < a.m ? ld4(xr + 16) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // A (the packed weight planes, stored as they are): SL_DMA copies them global -> LDS directly
    // (global_load_lds_dwordx4: no registers, no ds_write; the wave's 64 lanes fill 1 KB at its LDS base)
    auto load = [&](int c, int sdst, f32x4 (&ra)[WO], f32x4 (&rb)[2 * RU]) {
#pragma unroll
        for (int u = 0; u < WO; ++u) {
            const int idx = tid + SL_THREADS * u;
            const f16x8* src = W + ((size_t)(T0 + (idx >> 7)) * KC + c) * 128 + (idx & 127);
#if SL_DMA
            lds_dma16(src, sA(sdst) + (idx & ~63));
            (void)ra;
#else
            (void)sdst;
            ra[u] = ld4(reinterpret_cast<const float*>(src));
#endif
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) xload(c, u, rb[2 * u], rb[2 * u + 1]);
    };
    auto store = [&](int s, const f32x4 (&ra)[WO], const f32x4 (&rb)[2 * RU]) {
#if !SL_DMA
#pragma unroll
        for (int u = 0; u < WO; ++u) sA(s)[tid + SL_THREADS * u] = __builtin_bit_cast(f16x8, ra[u]);
#else
        (void)ra;
#endif
#pragma unroll
        for (int u = 0; u < RU; ++u) {
#pragma clang fp contract(off)
            const int r = brow[u], ln = 16 * bq[u] + (r & 15);
            f16x8 hi, lo;   // k-groups bq (halves 0-3) and bq + 4 (halves 4-7)
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float x = rb[2 * u + h2][j] * sc[u];
                    const _Float16 h = (_Float16)x;
                    hi[4 * h2 + j] = h;
                    lo[4 * h2 + j] = (_Float16)(x - (float)h);
                }
            sB(s)[((r >> 4) * 2 + 0) * 64 + ln] = hi;
            sB(s)[((r >> 4) * 2 + 1) * 64 + ln] = lo;
        }
    };
    const int wo = wid % WO, wt = wid / WO;
    f32x4 acc[4][JT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 ra[WO], rb[2 * RU];
    load(0, 0, ra, rb);
    store(0, ra, rb);
    if constexpr (SL_DMA) wait_all_mem();   // the direct-to-LDS copies have landed
    __syncthreads();
    for (int c = 0; c < KC; ++c) {
        const int s = c & 1;
#if SL_DIAG
        // timing diagnostic (wrong results): bit 1 no x loads / split / B stores after chunk 0, bit 2 no weight
        // copies after chunk 0, bit 4 no barrier wait on memory (the loop's vmcnt(0) dropped)
        if (c + 1 < KC) {
            if constexpr ((SL_DIAG & 2) == 0)
#pragma unroll
                for (int u = 0; u < WO; ++u) {
                    const int idx = tid + SL_THREADS * u;
                    lds_dma16(W + ((size_t)(T0 + (idx >> 7)) * KC + c + 1) * 128 + (idx & 127), sA(s ^ 1) + (idx & ~63));
                }
            if constexpr ((SL_DIAG & 1) == 0)
#pragma unroll
                for (int u = 0; u < RU; ++u) xload(c + 1, u, rb[2 * u], rb[2 * u + 1]);
        }
#else
        if (c + 1 < KC) load(c + 1, s ^ 1, ra, rb);
#endif
        if constexpr (JT == 4) {
            f16x8 bh[JT], bl[JT];
#pragma unroll
            for (int j = 0; j < JT; ++j) {
                bh[j] = sB(s)[((JT * wt + j) * 2 + 0) * 64 + lane];
                bl[j] = sB(s)[((JT * wt + j) * 2 + 1) * 64 + lane];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f16x8 ah = sA(s)[((4 * wo + i) * 2 + 0) * 64 + lane];
                const f16x8 al = sA(s)[((4 * wo + i) * 2 + 1) * 64 + lane];
#pragma unroll
                for (int j = 0; j < JT; ++j) acc[i][j] = mfma_h(al, bh[j], acc[i][j]);
#pragma unroll
                for (int j = 0; j < JT; ++j) acc[i][j] = mfma_h(ah, bl[j], acc[i][j]);
#pragma unroll
                for (int j = 0; j < JT; ++j) acc[i][j] = mfma_h(ah, bh[j], acc[i][j]);
            }
        } else {
            // the wave's four A tiles held for the chunk, the token tiles' planes read two at a time (the 8 x 4
            // accumulators leave no room for all 16 B fragments); the same three products per tile, in order
            f16x8 ah[4], al[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ah[i] = sA(s)[((4 * wo + i) * 2 + 0) * 64 + lane];
                al[i] = sA(s)[((4 * wo + i) * 2 + 1) * 64 + lane];
            }
#pragma unroll
            for (int j0 = 0; j0 < JT; j0 += 2) {
                f16x8 bh[2], bl[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    bh[j] = sB(s)[((JT * wt + j0 + j) * 2 + 0) * 64 + lane];
                    bl[j] = sB(s)[((JT * wt + j0 + j) * 2 + 1) * 64 + lane];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j0 + j] = mfma_h(al[i], bh[j], acc[i][j0 + j]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j0 + j] = mfma_h(ah[i], bl[j], acc[i][j0 + j]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j0 + j] = mfma_h(ah[i], bh[j], acc[i][j0 + j]);
            }
        }
#if SL_DIAG
        if ((SL_DIAG & 1) == 0 && c + 1 < KC) store(s ^ 1, ra, rb);
        if constexpr ((SL_DIAG & 4) == 0) wait_all_mem();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
        if (c + 1 < KC) store(s ^ 1, ra, rb);
        if constexpr (SL_DMA) wait_all_mem();
        __syncthreads();
#endif
    }
    // epilogue: unscale (exact powers of two), bias, activation; the accumulator of tile (i, j) holds outputs
    // 4q..4q+3 of output tile T0 + 4 wo + i for token (JT wt + j) * 16 + nn
#pragma unroll
    for (int j = 0; j < JT; ++j) {
        const int pc = (JT * wt + j) * 16 + nn, r = m0 + pc;
        const float u = exp2i(eT[pc] - 14 - ew);
        float ym = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = (T0 + 4 * wo + i) * 16 + 4 * q;
            if (o >= a.n || r >= a.m) continue;
            f32x4 v = acc[i][j] * u + ld4(a.bias + o);
            if (ACT == 1) v = relu4(v);
            if (ACT >= 2) v = f32x4{sigmoidf(v.x), sigmoidf(v.y), sigmoidf(v.z), sigmoidf(v.w)};
            if (ACT == 3) {   // GatedAttentionFusion's mix: g * cur + (1 - g) * att, x = [cur | att]
#pragma clang fp contract(off)
                const f32x4 cu = ld4(a.x + (size_t)r * a.ldx + o), at = ld4(a.x + (size_t)r * a.ldx + a.n + o);
                v = f32x4{v.x * cu.x + (1.0f - v.x) * at.x, v.y * cu.y + (1.0f - v.y) * at.y,
                          v.z * cu.z + (1.0f - v.z) * at.z, v.w * cu.w + (1.0f - v.w) * at.w};
            }
            ym = fmaxf(ym, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            st4(a.y + (size_t)r * a.ldy + o, v);
        }
        if (a.ymax) {   // one atomic per (row, wave): the max over the wave's 64 outputs of the row
            ym = rows_max(ym);
            if (q == 0 && r < a.m) atomicMax(a.ymax + r, __float_as_uint(ym));
        }
    }
}

// 256-token workgroups (JT = 8) when they still give the chip at least two workgroups per CU; GENPOSE2_LSPLIT_JT=4
// keeps the 128-token tiles (tuning)
#ifndef SL_JT8_DEFAULT
#define SL_JT8_DEFAULT 1
#endif
static bool sl_wide_tokens(int m, int npad) {
    const char* env = getenv("GENPOSE2_LSPLIT_JT");
    const bool on = env ? env[0] == '8' : SL_JT8_DEFAULT != 0;
    return on && (long long)((m + 255) / 256) * (npad / 256) >= 512;
}

extern "C" size_t gp_linear_split_words(int n, int k) {
    if (n < 1 || k < 32) return 0;
    return 4 + (size_t)((n + 127) / 128 * 128) * k;
}

extern "C" int gp_linear_split(const float* x, int ldx, int m, int k, const int32_t* wpk, const float* bias, int n,
                               int act, float* y, int ldy, float* rmax, int flags, float* ymax, hipStream_t st) {
    GP_REQUIRE(x && wpk && bias && y && rmax && m >= 0, "linear_split: null pointer");
    GP_REQUIRE(k >= 32 && k % 32 == 0 && n >= 16 && n % 16 == 0, "linear_split: k=%d (multiple of 32), n=%d (of 16)", k, n);
    GP_REQUIRE(ldx >= k && ldy >= n && ldx % 4 == 0 && ldy % 4 == 0, "linear_split: strides ldx=%d ldy=%d", ldx, ldy);
    GP_REQUIRE(((uintptr_t)x | (uintptr_t)wpk | (uintptr_t)y | (uintptr_t)bias) % 16 == 0,
               "linear_split: pointers must be 16-byte aligned");
    GP_REQUIRE(act >= 0 && act <= 3 && (flags & ~GP_LINEAR_RMAX_GIVEN) == 0, "linear_split: act %d flags %d", act, flags);
    GP_REQUIRE(act != 3 || k == 2 * n, "linear_split: the gate mix (act 3) takes x = [cur | att], k = 2n (k=%d n=%d)", k, n);
    if (!m) return GP_OK;
    if (!(flags & GP_LINEAR_RMAX_GIVEN)) {
        hipLaunchKernelGGL(fus_rowmax_kernel, dim3((m + 3) / 4), dim3(256), 0, st, x, ldx, m, k, rmax);
        FUS_TRY(gp_check_launch("fus_rowmax_kernel"));
    }
    if (ymax && hipMemsetAsync(ymax, 0, sizeof(float) * (size_t)m, st) != hipSuccess)
        return gp_check_launch("linear_split ymax memset");
    SplitLinArgs a{x, ldx, m, k, rmax, wpk, bias, n, y, ldy, reinterpret_cast<unsigned*>(ymax), 0, 0};
    const int npad = (n + 127) / 128 * 128;
#define GP_LSPLIT(WO, JT)                                                                                          \
    {                                                                                                          \
        constexpr int BM = 16 * JT * (8 / WO);                                                                 \
        const dim3 grid(npad / (64 * WO), (m + BM - 1) / BM);                                                  \
        constexpr size_t lds = sl_lds_bytes<WO, JT>();                                                         \
        if (act == 0) hipLaunchKernelGGL((linear_split_kernel<WO, 0, JT>), grid, dim3(SL_THREADS), lds, st, a); \
        else if (act == 1) hipLaunchKernelGGL((linear_split_kernel<WO, 1, JT>), grid, dim3(SL_THREADS), lds, st, a); \
        else if (act == 2) hipLaunchKernelGGL((linear_split_kernel<WO, 2, JT>), grid, dim3(SL_THREADS), lds, st, a); \
        else hipLaunchKernelGGL((linear_split_kernel<WO, 3, JT>), grid, dim3(SL_THREADS), lds, st, a); \
    }
    if (npad % 256 == 0 && sl_wide_tokens(m, npad)) GP_LSPLIT(4, 8)
    else if (npad % 256 == 0) GP_LSPLIT(4, 4)
    else GP_LSPLIT(2, 4)
#undef GP_LSPLIT
    return gp_check_launch("linear_split_kernel");
}

// relu(conv3x3(f) + bias) over every pixel of b objects of a g x g grid (stride 1, zero padding 1) as the split
// linear with implicit im2col: f (b, g*g, d) pixel-major, wpk = pack_split_linear of the weight in position-major
// order ((n, 3, 3, d) rows: k index (ky * 3 + kx) * d + channel), rmax[b * g * g] = max |x| over each pixel's im2col
// row (its in-grid neighbours' channel maxima), y (b * g * g, n). No (b g^2, 9 d) column buffer is formed.
int gp_linear_split_conv3x3(const float* f, int b, int g, int d, const int32_t* wpk, const float* bias, int n,
                            float* y, const float* rmax, hipStream_t st) {
    GP_REQUIRE(f && wpk && bias && y && rmax && b >= 0 && g >= 1, "conv3x3_split: bad arguments");
    GP_REQUIRE(d % 32 == 0 && n >= 16 && n % 16 == 0, "conv3x3_split: d=%d (multiple of 32), n=%d (of 16)", d, n);
    GP_REQUIRE(((uintptr_t)f | (uintptr_t)wpk | (uintptr_t)y | (uintptr_t)bias) % 16 == 0,
               "conv3x3_split: pointers must be 16-byte aligned");
    const int m = b * g * g, k = 9 * d;
    if (!m) return GP_OK;
    SplitLinArgs a{f, d, m, k, rmax, wpk, bias, n, y, n, nullptr, g, d / 32};
    const int npad = (n + 127) / 128 * 128;
#define GP_LSPLIT_IM(WO)                                                                                       \
    {                                                                                                          \
        constexpr int BM = 16 * 4 * (8 / WO);                                                                  \
        const dim3 grid(npad / (64 * WO), (m + BM - 1) / BM);                                                  \
        constexpr size_t lds = sl_lds_bytes<WO, 4>();                                                          \
        hipLaunchKernelGGL((linear_split_kernel<WO, 1, 4, 1>), grid, dim3(SL_THREADS), lds, st, a);            \
    }
    if (npad % 256 == 0) GP_LSPLIT_IM(4)
    else GP_LSPLIT_IM(2)
#undef GP_LSPLIT_IM
    return gp_check_launch("linear_split_kernel<im2col>");
}

// ============================================================================ residual + LayerNorm
// L lanes per row (16 for d <= 256, else 64; up to 4 float4 per lane in registers), torch's biased variance.
// ymax (optional): max |y| per row, for a split-arithmetic consumer (gp_linear_split's GP_LINEAR_RMAX_GIVEN).
template <int L>
__device__ __forceinline__ float group_sum(float v) { return L == 16 ? row16_sum(v) : wave_sum(v); }
template <int L>
__device__ __forceinline__ float group_max(float v) {
    v = row16_max(v);
    if constexpr (L == 64) v = rows_max(v);
    return v;
}
template <int L>
__global__ __launch_bounds__(FUS_THREADS) void add_layernorm_kernel(const float* x,
                                                                    const float* __restrict__ r, int m, int d,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta, float eps,
                                                                    float* y, float* __restrict__ ymax) {   // y may alias x
#pragma clang fp contract(off)
    const int sub = threadIdx.x & (L - 1);
    const int row = (int)(((long long)blockIdx.x * FUS_THREADS + threadIdx.x) / L);
    if (row >= m) return;   // whole L-lane groups leave together
    const float* xr = x + (size_t)row * d;
    const float* rr = r + (size_t)row * d;
    f32x4 v[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = 4 * (sub + L * i);
        v[i] = c < d ? ld4(xr + c) + ld4(rr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = group_sum<L>(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = 4 * (sub + L * i);
        if (c < d) {
            const f32x4 u = v[i] - mean;
            s2 += (u.x * u.x + u.y * u.y) + (u.z * u.z + u.w * u.w);
        }
    }
    const float rstd = 1.0f / sqrtf(group_sum<L>(s2) / (float)d + eps);
    float* yr = y + (size_t)row * d;
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = 4 * (sub + L * i);
        if (c < d) {
            const f32x4 o = ((v[i] - mean) * rstd) * ld4(gamma + c) + ld4(beta + c);
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            st4(yr + c, o);
        }
    }
    if (ymax) {
        mx = group_max<L>(mx);
        if (sub == 0) ymax[row] = mx;
    }
}

extern "C" int gp_add_layernorm(const float* x, const float* r, int m, int d, const float* gamma, const float* beta,
                                float eps, float* y, float* ymax, hipStream_t st) {
    GP_REQUIRE(x && r && gamma && beta && y && m >= 0, "add_layernorm: null pointer");
    GP_REQUIRE(d >= 4 && d <= 1024 && d % 4 == 0, "add_layernorm: d=%d not a multiple of 4 in [4, 1024]", d);
    GP_REQUIRE(((uintptr_t)x | (uintptr_t)r | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) % 16 == 0,
               "add_layernorm: pointers must be 16-byte aligned");
    if (!m) return GP_OK;
    if (d <= 256)
        hipLaunchKernelGGL(add_layernorm_kernel<16>, dim3((unsigned)(((long long)m * 16 + FUS_THREADS - 1) / FUS_THREADS)),
                           dim3(FUS_THREADS), 0, st, x, r, m, d, gamma, beta, eps, y, ymax);
    else
        hipLaunchKernelGGL(add_layernorm_kernel<64>, dim3((m + 3) / 4), dim3(FUS_THREADS), 0, st, x, r, m, d, gamma, beta,
                           eps, y, ymax);
    return gp_check_launch("add_layernorm_kernel");
}

// ============================================================================ relative-PE bias
// Packed pe (gp_relpe_bias in genpose_hip.h): distance Linear(1,16)/ReLU/Linear(16,8), direction
// Linear(3,16)/ReLU/Linear(16,8), fusion Linear(16,8) over [distance | direction]. The fusion layer is
// linear, so the host composes it with the two second layers: bias_h = A_h . hd + B_h . ho + c_h
// (pe[512:776), composed in float64) -- 256 multiply-adds per pair instead of 384, done as packed fp32
// FMAs over pairs of hidden units like the first layers (direction weights transposed at pe[776:824)). The result is the reference's
// up to rounding order (fused multiply-adds, the composition); the distance and direction are as it
// rounds them.
// with the weights in scalar registers (uniform loads). One thread per pair, all 8
// heads. Stored as the reference's relative_bias, bias[b][h][i][j] (query i, key j): consecutive threads
// take consecutive keys j, so the stores are coalesced, and an attention lane reads its 4 consecutive
// keys of a 16-key tile as one 16-byte load.
typedef float f32x2 __attribute__((ext_vector_type(2)));
// The 8 heads' bias of one pair from rel = xyz[key] - xyz[query] (shared by relpe_bias_kernel and the
// fused mha_relpe_kernel, so both produce the same bits).
__device__ __forceinline__ void relpe_heads(const float* __restrict__ pe, float rx, float ry, float rz,
                                            float (&out)[FUS_HEADS]) {
    float dist, dx, dy, dz;
    {
#pragma clang fp contract(off)
        dist = sqrtf((rx * rx + ry * ry) + rz * rz);
        const float den = dist + 1e-7f;
        dx = rx / den;
        dy = ry / den;
        dz = rz / den;
    }
    // first layers as fused multiply-adds (bias first), hidden units u = 2 u2, 2 u2 + 1 per packed FMA
    const f32x2* W1d = reinterpret_cast<const f32x2*>(pe);          // dist.0.w
    const f32x2* B1d = reinterpret_cast<const f32x2*>(pe + 16);     // dist.0.b
    const f32x2* W1o = reinterpret_cast<const f32x2*>(pe + 776);    // dir.0.w transposed: [axis][u]
    const f32x2* B1o = reinterpret_cast<const f32x2*>(pe + 216);    // dir.0.b
    f32x2 hd[8], ho[8];
    const f32x2 d2 = {dist, dist}, x2 = {dx, dx}, y2 = {dy, dy}, z2 = {dz, dz};
#pragma unroll
    for (int u2 = 0; u2 < 8; ++u2) {
        const f32x2 a = __builtin_elementwise_fma(d2, W1d[u2], B1d[u2]);
        f32x2 c = __builtin_elementwise_fma(x2, W1o[u2], B1o[u2]);
        c = __builtin_elementwise_fma(y2, W1o[8 + u2], c);
        c = __builtin_elementwise_fma(z2, W1o[16 + u2], c);
        hd[u2] = f32x2{fmaxf(a.x, 0.f), fmaxf(a.y, 0.f)};
        ho[u2] = f32x2{fmaxf(c.x, 0.f), fmaxf(c.y, 0.f)};
    }
    // composed second layers: head h accumulates the even / odd hidden units in the two halves
    const f32x2* A2 = reinterpret_cast<const f32x2*>(pe + 512);   // [h][u]
    const f32x2* B2 = reinterpret_cast<const f32x2*>(pe + 640);
#pragma unroll
    for (int h = 0; h < FUS_HEADS; ++h) {
        f32x2 acc = {pe[768 + h], 0.f};
#pragma unroll
        for (int u2 = 0; u2 < 8; ++u2) acc = __builtin_elementwise_fma(hd[u2], A2[8 * h + u2], acc);
#pragma unroll
        for (int u2 = 0; u2 < 8; ++u2) acc = __builtin_elementwise_fma(ho[u2], B2[8 * h + u2], acc);
        out[h] = acc.x + acc.y;
    }
}

__global__ __launch_bounds__(FUS_THREADS) void relpe_bias_kernel(const float* __restrict__ pe,
                                                                 const float* __restrict__ xyz, int n,
                                                                 float* __restrict__ bias) {
    const int b = blockIdx.y;
    const long long e = (long long)blockIdx.x * FUS_THREADS + threadIdx.x;
    if (e >= (long long)n * n) return;
    const int i = (int)(e / n), j = (int)(e - (long long)i * n);
    const float* pi = xyz + ((size_t)b * n + i) * 3;
    const float* pj = xyz + ((size_t)b * n + j) * 3;
    float rx, ry, rz;
    {
#pragma clang fp contract(off)
        rx = ld1(pj) - ld1(pi);   // xyz[j] - xyz[i]
        ry = ld1(pj + 1) - ld1(pi + 1);
        rz = ld1(pj + 2) - ld1(pi + 2);
    }
    float hb[FUS_HEADS];
    relpe_heads(pe, rx, ry, rz, hb);
    const size_t hs = (size_t)n * n;
    float* bp = bias + (size_t)b * FUS_HEADS * hs + (size_t)i * n + j;
#pragma unroll
    for (int h = 0; h < FUS_HEADS; ++h) bp[h * hs] = hb[h];
}

extern "C" size_t gp_relpe_bias_bytes(int b, int n) { return sizeof(float) * (size_t)b * FUS_HEADS * n * n; }

extern "C" int gp_relpe_bias(const float* pe, const float* xyz, int b, int n, float* bias, hipStream_t st) {
    GP_REQUIRE(pe && xyz && bias && b >= 0 && n >= 1 && n <= 4096, "relpe_bias: bad arguments");
    if (!b) return GP_OK;
    const long long pairs = (long long)n * n;
    hipLaunchKernelGGL(relpe_bias_kernel, dim3((unsigned)((pairs + FUS_THREADS - 1) / FUS_THREADS), b),
                       dim3(FUS_THREADS), 0, st, pe, xyz, n, bias);
    return gp_check_launch("relpe_bias_kernel");
}

// ============================================================================ biased attention
// Flash-style on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32). Workgroup = 64 queries (4 waves x 16) of one
// (object, head); a wave keeps its 16 queries' Q^T fragments and O^T accumulators in registers and walks
// the keys in LDS chunks of KC (K row-major, V transposed), 64 keys per softmax block:
//   S^T = K Q^T          A = K rows (keys), B = Q^T: the D tile holds keys 4q + r of query l & 15 -- which is
//                        exactly the B-operand layout of the next product, so P never leaves registers;
//   s = S^T / sqrt(hd) + bias (a lane's 4 keys are consecutive in the bias row: one 16-byte load), keys >= n
//   masked;
//   online softmax per query: m' = max(m, block max), O *= exp(m - m'), l = l exp(m - m') + sum exp(s - m');
//   O^T += V^T P^T       A = V^T (dims x keys, from the transposed LDS copy), B = P^T.
// out = O / l. Head dims are zero-padded to a multiple of 16 (12 -> 16). The grid is 1-D and XCD-aware:
// the query blocks of one (object, head) land on one XCD, so its K / V are read into one L2.
// (q.k / sqrt(hd) is taken as q.k * (1 / sqrt(hd)): within an ulp of torch's division. The softmax is
// torch's result up to rounding: the online rescaling replaces its two passes.)
template <int HDP>
__global__ __launch_bounds__(FUS_THREADS) void mha_kernel(const float* __restrict__ qkv,
                                                          const float* __restrict__ bias, int n, int d, int hd,
                                                          int nqb, float* __restrict__ out, unsigned* __restrict__ ymax) {
    constexpr int NG = HDP / 16;      // 16-deep k-groups of S, 16-row dim tiles of O
    constexpr int KC = 4096 / HDP;    // keys per LDS chunk (37 KB at every head dim)
    constexpr int KS = HDP + 4;       // K row stride (floats)
    constexpr int VS = KC + 4;        // V^T row stride
    __shared__ __attribute__((aligned(16))) float ks[KC * KS];
    __shared__ __attribute__((aligned(16))) float vt[HDP * VS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int qg = lane >> 4, nl = lane & 15;
    const int G = gridDim.x;                                   // a multiple of 8 (8 heads)
    const int t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
    const int qb = t % nqb, hb = t / nqb, h = hb & (FUS_HEADS - 1), b = hb / FUS_HEADS;
    const size_t ld = 3 * (size_t)d;
    const float* base = qkv + (size_t)b * n * ld;
    const int i = qb * 64 + wid * 16 + nl;
    const int ii = i < n ? i : n - 1;
    f32x4 qf[NG], o[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int c = 16 * g + 4 * qg;
        qf[g] = c < hd ? ld4(base + (size_t)ii * ld + h * hd + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        o[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const float inv = 1.0f / sqrtf((float)hd);
    const float* brow = bias ? bias + (((size_t)b * FUS_HEADS + h) * n + ii) * n : nullptr;   // + key
    const bool bvec = (n & 3) == 0;   // 16-byte aligned rows
    float m = -INFINITY, lsum = 0.f;
    for (int c0 = 0; c0 < n; c0 += KC) {
        const int kn = min(KC, n - c0), k16 = (kn + 15) & ~15;
        __syncthreads();
        for (int e = threadIdx.x; e < k16 * (HDP / 4); e += FUS_THREADS) {
            const int j = e / (HDP / 4), c = 4 * (e - j * (HDP / 4));
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
            if (j < kn && c < hd) {
                const float* row = base + (size_t)(c0 + j) * ld + h * hd + c;
                kv = ld4(row + d);
                vv = ld4(row + 2 * d);
            }
            st4(ks + j * KS + c, kv);
            vt[(c + 0) * VS + j] = vv.x;
            vt[(c + 1) * VS + j] = vv.y;
            vt[(c + 2) * VS + j] = vv.z;
            vt[(c + 3) * VS + j] = vv.w;
        }
        __syncthreads();
        for (int kb = 0; kb < k16; kb += 64) {
            const int nt = min(4, (k16 - kb) >> 4);
            f32x4 s[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {      // bias loads first: their latency hides under the S MFMAs
                bv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (brow && u < nt) {
                    const int j0 = c0 + kb + 16 * u + 4 * qg;
                    if (bvec && j0 < n) {
                        bv[u] = ld4(brow + j0);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (j0 + r < n) bv[u][r] = brow[j0 + r];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (u < nt) {
                    const float* kr = ks + (kb + 16 * u + nl) * KS + 4 * qg;
#pragma unroll
                    for (int g = 0; g < NG; ++g) s[u] = mfma_kgroup(ld4(kr + 16 * g), qf[g], s[u]);
                }
            }
            float bmax = -INFINITY;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j0 = c0 + kb + 16 * u + 4 * qg;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v;
                    {
#pragma clang fp contract(off)
                        v = s[u][r] * inv + bv[u][r];
                    }
                    s[u][r] = (u < nt && j0 + r < n) ? v : -INFINITY;
                    bmax = fmaxf(bmax, s[u][r]);
                }
            }
            const float mn = fmaxf(m, rows_max(bmax));
            const float alpha = expf(m - mn);
            m = mn;
            float ps = 0.f;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    s[u][r] = expf(s[u][r] - mn);
                    ps += s[u][r];
                }
            lsum = lsum * alpha + ps;
#pragma unroll
            for (int g = 0; g < NG; ++g) o[g] *= alpha;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u < nt) {
                    const float* vr = vt + nl * VS + kb + 16 * u + 4 * qg;
#pragma unroll
                    for (int g = 0; g < NG; ++g) o[g] = mfma_kgroup(ld4(vr + 16 * g * VS), s[u], o[g]);
                }
        }
    }
    const float rl = 1.0f / rows_sum(lsum);
    float mx = 0.f;
    if (i < n) {
        float* op = out + ((size_t)b * n + i) * d + h * hd;
#pragma unroll
        for (int g = 0; g < NG; ++g)
            if (16 * g + 4 * qg < hd) {
                const f32x4 v = o[g] * rl;
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                st4(op + 16 * g + 4 * qg, v);
            }
    }
    if (ymax) {   // the query row's max |out| over this head, merged over the 8 heads' workgroups
        mx = rows_max(mx);
        if (qg == 0 && i < n) atomicMax(ymax + (size_t)b * n + i, __float_as_uint(mx));
    }
}

extern "C" int gp_mha_attention(const float* qkv, const float* bias, int b, int n, int d, float* out, float* ymax,
                                hipStream_t st) {
    GP_REQUIRE(qkv && out && b >= 0 && n >= 1, "mha_attention: bad arguments");
    GP_REQUIRE(d % (4 * FUS_HEADS) == 0, "mha_attention: d=%d must be a multiple of 32", d);
    GP_REQUIRE(((uintptr_t)qkv | (uintptr_t)out) % 16 == 0, "mha_attention: pointers must be 16-byte aligned");
    if (!b) return GP_OK;
    const int hd = d / FUS_HEADS;
    const int nqb = (n + 63) / 64;
    GP_REQUIRE((long long)nqb * FUS_HEADS * b < (1LL << 31), "mha_attention: grid too large");
    const dim3 grid((unsigned)(nqb * FUS_HEADS * b));
    if (ymax && hipMemsetAsync(ymax, 0, sizeof(float) * (size_t)b * n, st) != hipSuccess)
        return gp_check_launch("mha_attention ymax memset");
    unsigned* ym = reinterpret_cast<unsigned*>(ymax);
#define GP_MHA(HDP) hipLaunchKernelGGL((mha_kernel<HDP>), grid, dim3(FUS_THREADS), 0, st, qkv, bias, n, d, hd, nqb, out, ym)
    if (hd <= 16) GP_MHA(16);
    else if (hd <= 32) GP_MHA(32);
    else if (hd <= 64) GP_MHA(64);
    else if (hd <= 128) GP_MHA(128);
    else { gp_set_error("mha_attention: head dim %d > 128", hd); return GP_ERR_UNSUPPORTED; }
#undef GP_MHA
    return gp_check_launch("mha_kernel");
}

// ============================================================================ attention with in-register bias
// MultiheadAttentionWithRelativePE with its EfficientRelativePositionalEncoding bias evaluated where it is
// used: a wave owns 16 queries and ALL 8 heads, so the relative-PE MLP of a (query, key) pair is evaluated
// once (relpe_heads, the bits gp_relpe_bias writes) for the 8 heads' score tiles that hold that pair in the
// same lane and register -- S^T = K Q^T puts keys 4q + r of query l & 15 in lane l, register r, for every
// head. No (B, 8, n, n) bias buffer is written or read (2.1 GB at level 0, B = 256). K / V^T of all heads
// and the keys' xyz are staged per chunk in LDS; per 16-key tile: the 8 heads' S^T on MFMA, the 4 pairs'
// bias on VALU (their latency under those MFMAs), one online-softmax update per head, O^T += V^T P^T.
// Head dims <= 32 (levels 0 and 1: the levels whose n^2 made the bias buffer large).
template <int HDP>
__global__ __launch_bounds__(FUS_THREADS) void mha_relpe_kernel(const float* __restrict__ qkv,
                                                                const float* __restrict__ xyz,
                                                                const float* __restrict__ pe, int n, int d, int hd,
                                                                int nqb, float* __restrict__ out,
                                                                float* __restrict__ ymax) {
    constexpr int NG = HDP / 16;
    constexpr int KC = HDP == 16 ? 64 : 32;   // keys per LDS chunk (69 / 68 KB: two workgroups per CU)
    constexpr int DP = FUS_HEADS * HDP;       // all heads, each padded to HDP
    constexpr int KS = DP + 4, VS = KC + 4;
    __shared__ __attribute__((aligned(16))) float ks[KC * KS];
    __shared__ __attribute__((aligned(16))) float vt[DP * VS];
    __shared__ float kx[KC * 3];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int qg = lane >> 4, nl = lane & 15;
    const int G = gridDim.x;   // XCD-aware: the query blocks of one object on one XCD when G % 8 == 0
    const int t = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : (int)blockIdx.x;
    const int qb = t % nqb, b = t / nqb;
    const size_t ld = 3 * (size_t)d;
    const float* base = qkv + (size_t)b * n * ld;
    const int i = qb * 64 + wid * 16 + nl;
    const int ii = i < n ? i : n - 1;
    const float px = ld1(xyz + ((size_t)b * n + ii) * 3), py = ld1(xyz + ((size_t)b * n + ii) * 3 + 1),
                pz = ld1(xyz + ((size_t)b * n + ii) * 3 + 2);
    f32x4 qf[FUS_HEADS][NG], o[FUS_HEADS][NG];
    float m[FUS_HEADS], lsum[FUS_HEADS];
#pragma unroll
    for (int h = 0; h < FUS_HEADS; ++h) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int c = 16 * g + 4 * qg;
            qf[h][g] = c < hd ? ld4(base + (size_t)ii * ld + h * hd + c) : f32x4{0.f, 0.f, 0.f, 0.f};
            o[h][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        m[h] = -INFINITY;
        lsum[h] = 0.f;
    }
    const float inv = 1.0f / sqrtf((float)hd);
    for (int c0 = 0; c0 < n; c0 += KC) {
        const int kn = min(KC, n - c0), k16 = (kn + 15) & ~15;
        __syncthreads();
        for (int e = threadIdx.x; e < k16 * (DP / 4); e += FUS_THREADS) {
            const int j = e / (DP / 4), cc = 4 * (e - j * (DP / 4));
            const int h = cc / HDP, c = cc - h * HDP;
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
            if (j < kn && c < hd) {
                const float* row = base + (size_t)(c0 + j) * ld + h * hd + c;
                kv = ld4(row + d);
                vv = ld4(row + 2 * d);
            }
            st4(ks + j * KS + cc, kv);
            vt[(cc + 0) * VS + j] = vv.x;
            vt[(cc + 1) * VS + j] = vv.y;
            vt[(cc + 2) * VS + j] = vv.z;
            vt[(cc + 3) * VS + j] = vv.w;
        }
        for (int e = threadIdx.x; e < kn * 3; e += FUS_THREADS) kx[e] = xyz[((size_t)b * n + c0) * 3 + e];
        __syncthreads();
        for (int kt = 0; kt < k16; kt += 16) {
            f32x4 s[FUS_HEADS];
#pragma unroll
            for (int h = 0; h < FUS_HEADS; ++h) {
                s[h] = f32x4{0.f, 0.f, 0.f, 0.f};
                const float* kr = ks + (kt + nl) * KS + h * HDP + 4 * qg;
#pragma unroll
                for (int g = 0; g < NG; ++g) s[h] = mfma_kgroup(ld4(kr + 16 * g), qf[h][g], s[h]);
            }
            float bb[4][FUS_HEADS];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = kt + 4 * qg + r;
                if (j < kn) {
                    float rx, ry, rz;
                    {
#pragma clang fp contract(off)
                        rx = ld1(kx + 3 * j) - px;   // xyz[key] - xyz[query]; 4-byte LDS reads (gp_common.h ld1)
                        ry = ld1(kx + 3 * j + 1) - py;
                        rz = ld1(kx + 3 * j + 2) - pz;
                    }
                    relpe_heads(pe, rx, ry, rz, bb[r]);
                } else {
#pragma unroll
                    for (int h = 0; h < FUS_HEADS; ++h) bb[r][h] = 0.f;
                }
            }
#pragma unroll
            for (int h = 0; h < FUS_HEADS; ++h) {
                float bm = -INFINITY;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v;
                    {
#pragma clang fp contract(off)
                        v = s[h][r] * inv + bb[r][h];
                    }
                    s[h][r] = kt + 4 * qg + r < kn ? v : -INFINITY;
                    bm = fmaxf(bm, s[h][r]);
                }
                const float mn = fmaxf(m[h], rows_max(bm));
                const float alpha = expf(m[h] - mn);
                m[h] = mn;
                float ps = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    s[h][r] = expf(s[h][r] - mn);
                    ps += s[h][r];
                }
                lsum[h] = lsum[h] * alpha + ps;
                const float* vr = vt + (h * HDP + nl) * VS + kt + 4 * qg;
#pragma unroll
                for (int g = 0; g < NG; ++g) o[h][g] = mfma_kgroup(ld4(vr + 16 * g * VS), s[h], o[h][g] * alpha);
            }
        }
    }
    float mx = 0.f;
#pragma unroll
    for (int h = 0; h < FUS_HEADS; ++h) {
        const float rl = 1.0f / rows_sum(lsum[h]);
        if (i < n) {
            float* op = out + ((size_t)b * n + i) * d + h * hd;
#pragma unroll
            for (int g = 0; g < NG; ++g)
                if (16 * g + 4 * qg < hd) {
                    const f32x4 v = o[h][g] * rl;
                    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                    st4(op + 16 * g + 4 * qg, v);
                }
        }
    }
    if (ymax) {   // this wave holds the query's whole row (all heads)
        mx = rows_max(mx);
        if (qg == 0 && i < n) ymax[(size_t)b * n + i] = mx;
    }
}

extern "C" int gp_mha_relpe_attention(const float* qkv, const float* xyz, const float* pe, int b, int n, int d,
                                      float* out, float* ymax, hipStream_t st) {
    GP_REQUIRE(qkv && xyz && pe && out && b >= 0 && n >= 1, "mha_relpe_attention: bad arguments");
    GP_REQUIRE(d % (4 * FUS_HEADS) == 0 && d / FUS_HEADS <= 32,
               "mha_relpe_attention: d=%d (head dims that are multiples of 4, up to 32)", d);
    GP_REQUIRE(((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)pe) % 16 == 0,
               "mha_relpe_attention: pointers must be 16-byte aligned");
    if (!b) return GP_OK;
    const int hd = d / FUS_HEADS;
    const int nqb = (n + 63) / 64;
    GP_REQUIRE((long long)nqb * b < (1LL << 31), "mha_relpe_attention: grid too large");
    const dim3 grid((unsigned)(nqb * b));
    if (hd <= 16)
        hipLaunchKernelGGL((mha_relpe_kernel<16>), grid, dim3(FUS_THREADS), 0, st, qkv, xyz, pe, n, d, hd, nqb, out, ymax);
    else
        hipLaunchKernelGGL((mha_relpe_kernel<32>), grid, dim3(FUS_THREADS), 0, st, qkv, xyz, pe, n, d, hd, nqb, out, ymax);
    return gp_check_launch("mha_relpe_kernel");
}

// ============================================================================ gated fusion
// F.interpolate(linear, align_corners=False) along points (upsample_linear1d's source index and lambda): a
// wave per output point, float4 channels; ymax (optional): max |y| per output row.
__global__ __launch_bounds__(FUS_THREADS) void interp_points_kernel(const float* __restrict__ x, int n_in, int c,
                                                                    int n_out, float* __restrict__ y,
                                                                    float* __restrict__ ymax) {
#pragma clang fp contract(off)
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int o = blockIdx.x * (FUS_THREADS / 64) + (threadIdx.x >> 6);
    if (o >= n_out) return;
    const float scale = (float)n_in / (float)n_out;
    float src = scale * ((float)o + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    int i0 = (int)src;
    i0 = i0 < n_in - 1 ? i0 : n_in - 1;
    const int i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
    float l1 = src - (float)i0;
    l1 = fminf(fmaxf(l1, 0.f), 1.f);
    const float l0 = 1.0f - l1;
    const float* x0 = x + ((size_t)b * n_in + i0) * c;
    const float* x1 = x + ((size_t)b * n_in + i1) * c;
    float* yr = y + ((size_t)b * n_out + o) * c;
    float mx = 0.f;
    for (int ch = 4 * lane; ch < c; ch += 256) {
        const f32x4 a = ld4(x0 + ch), v = ld4(x1 + ch);
        const f32x4 r = f32x4{l0 * a.x + l1 * v.x, l0 * a.y + l1 * v.y, l0 * a.z + l1 * v.z, l0 * a.w + l1 * v.w};
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fmaxf(fabsf(r.z), fabsf(r.w))));
        st4(yr + ch, r);
    }
    if (ymax) {
        mx = rows_max(row16_max(mx));
        if (lane == 0) ymax[(size_t)b * n_out + o] = mx;
    }
}

extern "C" int gp_interp_points(const float* x, int b, int n_in, int c, int n_out, float* y, float* ymax,
                                hipStream_t st) {
    GP_REQUIRE(x && y && b >= 0 && n_in >= 1 && n_out >= 1 && c >= 4 && c % 4 == 0,
               "interp_points: bad arguments (c must be a multiple of 4)");
    GP_REQUIRE(((uintptr_t)x | (uintptr_t)y) % 16 == 0, "interp_points: pointers must be 16-byte aligned");
    if (!b) return GP_OK;
    hipLaunchKernelGGL(interp_points_kernel, dim3((n_out + 3) / 4, b), dim3(FUS_THREADS), 0, st, x, n_in, c, n_out, y, ymax);
    return gp_check_launch("interp_points_kernel");
}

// GatedAttentionFusion's attention stage as four chip-filling steps (the per-object statistics are
// batch-parallel reductions; the two 1x1 convs of the channel attention are (b x 2c) GEMMs on MFMA):
//   1. colmean[b][ch] = mean over tokens of [cur | ot] (AdaptiveAvgPool1d(1));
//   2. tstat[b][t] = (max, mean) over channels of cur (the spatial attention's two input rows);
//   3. ca = sigmoid(ca3(relu(ca1(colmean)))) via gp_linear;
//   4. gcat = [cur | (ot * ca) * sp], sp[t] = sigmoid(conv1d_7([max ; mean]))[t] (zero padding 3).
// Step 1: lanes are channels (coalesced rows), the 4 waves take tokens t = w mod 4, summed in a fixed order.
__global__ __launch_bounds__(FUS_THREADS) void fusion_colmean_kernel(const float* __restrict__ cur,
                                                                     const float* __restrict__ ot, int n, int c,
                                                                     float* __restrict__ colmean) {
#pragma clang fp contract(off)
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, b = blockIdx.y;
    const int ch = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (ch < 2 * c) {
        const float* src = (ch < c ? cur + ch : ot + (ch - c)) + (size_t)b * n * c;
        int t = wid;
        for (; t + 12 < n; t += 16) {
            const float v0 = src[(size_t)t * c], v1 = src[(size_t)(t + 4) * c];
            const float v2 = src[(size_t)(t + 8) * c], v3 = src[(size_t)(t + 12) * c];
            s += v0;
            s += v1;
            s += v2;
            s += v3;
        }
        for (; t < n; t += 4) s += src[(size_t)t * c];
    }
    part[wid][lane] = s;
    __syncthreads();
    if (wid == 0 && ch < 2 * c)
        colmean[(size_t)b * 2 * c + ch] = ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane])) / (float)n;
}

// Step 2: a wave per token.
__global__ __launch_bounds__(FUS_THREADS) void fusion_tokstat_kernel(const float* __restrict__ cur, int n, int c,
                                                                     float* __restrict__ tstat) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63, b = blockIdx.y;
    const int t = blockIdx.x * (FUS_THREADS / 64) + (threadIdx.x >> 6);
    if (t >= n) return;
    const float* row = cur + ((size_t)b * n + t) * c;
    float mxv = -INFINITY, s = 0.f;
    for (int ch = lane; ch < c; ch += 64) {
        const float v = row[ch];
        mxv = fmaxf(mxv, v);
        s += v;
    }
    for (int off = 32; off >= 1; off >>= 1) mxv = fmaxf(mxv, __shfl_xor(mxv, off, 64));
    s = wave_sum(s);
    if (lane == 0) {
        tstat[((size_t)b * n + t) * 2] = mxv;
        tstat[((size_t)b * n + t) * 2 + 1] = s / (float)c;
    }
}

// Step 4: a wave per token (c % 4 == 0); gmax (optional): max |gcat| per token, for the gate linear.
__global__ __launch_bounds__(FUS_THREADS) void fusion_gcat_kernel(const float* __restrict__ cur,
                                                                  const float* __restrict__ ot, int n, int c,
                                                                  const float* __restrict__ ca,
                                                                  const float* __restrict__ tstat,
                                                                  const float* __restrict__ sp_w,
                                                                  float* __restrict__ gcat, float* __restrict__ gmax) {
#pragma clang fp contract(off)
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int t = blockIdx.x * (FUS_THREADS / 64) + (threadIdx.x >> 6);
    if (t >= n) return;
    const float* ts = tstat + (size_t)b * n * 2;
    float sv = 0.f;
#pragma unroll
    for (int u = 0; u < 7; ++u) {
        const int tt = t + u - 3;
        if (tt >= 0 && tt < n) sv += sp_w[u] * ts[2 * tt] + sp_w[7 + u] * ts[2 * tt + 1];
    }
    const float sp = sigmoidf(sv);
    const size_t src = ((size_t)b * n + t) * c;
    float* g = gcat + ((size_t)b * n + t) * 2 * c;
    float mx = 0.f;
    for (int ch = 4 * lane; ch < c; ch += 256) {
        const f32x4 cv = ld4(cur + src + ch), ov = ld4(ot + src + ch), cav = ld4(ca + (size_t)b * c + ch);
        const f32x4 av = f32x4{(ov.x * cav.x) * sp, (ov.y * cav.y) * sp, (ov.z * cav.z) * sp, (ov.w * cav.w) * sp};
        st4(g + ch, cv);
        st4(g + c + ch, av);
        mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(fabsf(cv.x), fabsf(cv.y)), fmaxf(fabsf(cv.z), fabsf(cv.w))),
                             fmaxf(fmaxf(fabsf(av.x), fabsf(av.y)), fmaxf(fabsf(av.z), fabsf(av.w)))));
    }
    if (gmax) {
        mx = rows_max(row16_max(mx));
        if (lane == 0) gmax[(size_t)b * n + t] = mx;
    }
}

static size_t fus_align(size_t floats) { return (floats + 63) & ~(size_t)63; }

extern "C" size_t gp_fusion_attend_workspace_size(int b, int n, int c) {
    if (b < 0 || n < 1 || c < 1) return 0;
    const size_t B = (size_t)b;
    return sizeof(float) * (fus_align(B * 2 * c) + fus_align(B * (c / 2)) + fus_align(B * c) + fus_align(B * 2 * n));
}

extern "C" int gp_fusion_attend(const float* cur, const float* ot, int b, int n, int c, const float* ca1_w,
                                const float* ca1_b, const float* ca3_w, const float* ca3_b, const float* sp_w,
                                float* gcat, float* gmax, void* ws, size_t ws_bytes, hipStream_t st) {
    GP_REQUIRE(cur && ot && ca1_w && ca1_b && ca3_w && ca3_b && sp_w && gcat && b >= 0, "fusion_attend: null pointer");
    GP_REQUIRE(n >= 1 && c >= 32 && c % 32 == 0, "fusion_attend: n=%d c=%d (c must be a multiple of 32)", n, c);
    GP_REQUIRE(((uintptr_t)cur | (uintptr_t)ot | (uintptr_t)gcat | (uintptr_t)ws) % 16 == 0,
               "fusion_attend: pointers must be 16-byte aligned");
    if (!b) return GP_OK;
    GP_REQUIRE(ws && ws_bytes >= gp_fusion_attend_workspace_size(b, n, c), "fusion_attend: workspace %zu < %zu bytes",
               ws_bytes, gp_fusion_attend_workspace_size(b, n, c));
    const size_t B = (size_t)b;
    float* colmean = static_cast<float*>(ws);
    float* hid = colmean + fus_align(B * 2 * c);
    float* ca = hid + fus_align(B * (c / 2));
    float* tstat = ca + fus_align(B * c);
    hipLaunchKernelGGL(fusion_colmean_kernel, dim3((2 * c + 63) / 64, b), dim3(FUS_THREADS), 0, st, cur, ot, n, c, colmean);
    FUS_TRY(gp_check_launch("fusion_colmean_kernel"));
    hipLaunchKernelGGL(fusion_tokstat_kernel, dim3((n + 3) / 4, b), dim3(FUS_THREADS), 0, st, cur, n, c, tstat);
    FUS_TRY(gp_check_launch("fusion_tokstat_kernel"));
    FUS_TRY(gp_linear(colmean, 2 * c, b, 2 * c, ca1_w, ca1_b, c / 2, 1, hid, c / 2, st));
    FUS_TRY(gp_linear(hid, c / 2, b, c / 2, ca3_w, ca3_b, c, 2, ca, c, st));
    hipLaunchKernelGGL(fusion_gcat_kernel, dim3((n + 3) / 4, b), dim3(FUS_THREADS), 0, st, cur, ot, n, c, ca, tstat, sp_w,
                       gcat, gmax);
    return gp_check_launch("fusion_gcat_kernel");
}

__global__ __launch_bounds__(FUS_THREADS) void fusion_mix_kernel(const float* __restrict__ g,
                                                                 const float* __restrict__ gcat, long long total,
                                                                 int c, float* __restrict__ out) {
#pragma clang fp contract(off)
    const long long e = (long long)blockIdx.x * FUS_THREADS + threadIdx.x;
    if (e >= total) return;
    const long long r = e / c;
    const int ch = (int)(e - r * c);
    const float gv = g[e];
    const float* row = gcat + (size_t)r * 2 * c;
    out[e] = gv * row[ch] + (1.0f - gv) * row[c + ch];
}

extern "C" int gp_fusion_mix(const float* g, const float* gcat, int rows, int c, float* out, hipStream_t st) {
    GP_REQUIRE(g && gcat && out && rows >= 0 && c >= 1, "fusion_mix: bad arguments");
    const long long total = (long long)rows * c;
    if (!total) return GP_OK;
    hipLaunchKernelGGL(fusion_mix_kernel, dim3((unsigned)((total + FUS_THREADS - 1) / FUS_THREADS)), dim3(FUS_THREADS),
                       0, st, g, gcat, total, c, out);
    return gp_check_launch("fusion_mix_kernel");
}
