// Shared score-head trunk for gfx950: LDS layout, streamed-weight MFMA layers, and pose helpers.
// Used by the PC sampler / score / energy kernels (gp_score.hip) and the ODE stage kernels
// (gp_ode.hip). Reference: PoseScoreNet.forward (networks/gf_algorithms/scorenet.py:215-275).
#pragma once
#include "gp_common.h"

constexpr int HT = 256;          // threads per workgroup
constexpr int HID = 256;         // pose/head hidden width
constexpr int KG_HID = HID / 16; // k-groups over a 256-wide activation
#ifndef PC_WV1
#define PC_WV1 8                 // waves per workgroup, 16-candidate PC tiles
#endif
#ifndef EVAL_WV
#define EVAL_WV 8                // waves per workgroup, score/energy evaluation
#endif
#ifndef PC_D2
#define PC_D2 3                  // k-groups of pose_encoder.2 weights kept in flight
#endif
#ifndef HEAD_PREFETCH
#define HEAD_PREFETCH 2          // k-groups of head-layer-1 weights kept in flight
#endif


// Phase stamps (PC_MARK) are defined by the including file; no-op by default.
#ifndef PC_MARK
#define PC_MARK(k) ((void)trace_slot)
#endif


// The thread id behind an opaque copy: per-lane values derived from it are computed where they are used and
// cannot be hoisted out of an enclosing loop (a trunk run once per loop iteration kept hoisted lane addresses
// live across every trunk and spilled them, their reloads draining the weight ring)
__device__ __forceinline__ int tid_x() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// ============================================================================ shared head trunk
// NT = column tiles (16 candidates each) per workgroup. PL = 0: the exact-fp32 trunk's activations
// (fp32, accumulator-native); PL = 3: the f16x3 trunk's (three f16 planes per value, 6 B).
template <int NT, int WV, int PL = 0>
struct HeadSmem {
    // 64-candidate tiles (NT = 4) alias pose_encoder.2's output onto pose_encoder.0's (written after
    // a barrier that retires every read of act1), so one workgroup still fits the 160 KiB of a CU
    static constexpr bool kAliasAct = NT >= 4;
    static constexpr int kAct = PL ? (HID / 32) * NT * PL * 64 : KG_HID * NT * 64;   // 16-byte entries
    float xin[NT * 16 * 16];           // input poses, [col][16] (9 used)
    f32x4 act1[kAct];                  // pose_encoder.0 output: [g][ct][lane] (fp32) / [chunk][ct][plane][lane]
    f32x4 act2[kAliasAct ? 4 : kAct];  // pose_encoder.2 output (act1 when aliased)
    // per-wave head-layer-2 partials, wave-minor (head_out reads a row), indexed [v][n][wave] by the
    // value v = (head * NT + column tile) * 3 + output and the column n within the tile: the order the
    // split trunk's reduce-scatter leaves them in (row q of the wave holds values 4g + q); padded to
    // whole groups of four values
    static constexpr int kRedV = (9 * NT + 3) / 4 * 4;
    float red[kRedV][16][WV];
    float xu[NT * 16 * 9];             // PC: last-step mean rows, gathered for the quaternion
    float scratch[WV * 64];
    // small per-launch weights staged once per workgroup (their loads overlap the PC update); the
    // f16x3 trunk holds pose_encoder.0's fragments and bias in registers (SplitScalars)
    f32x4 pe0w[PL ? 1 : 16 * 64];      // pose_encoder.0 packed A fragments
    float pe0b[PL ? 1 : HID], pe2b[HID];
    float h2w[9 * HID];                // head layer 2, [head*3 + out][256]
    float h2b[12];
    f32x4 cscl[NT * 16][2];            // split trunk: per-column scales {s1, s2, u2, uh}, {sh} (ColScales)
};

// Threads [FIRST, WV*64) copy the small weights into LDS.
// PE0 = false: pose_encoder.0's fragments and bias are not staged (the split trunk holds them in
// registers from kernel entry, SplitScalars).
template <int NT, int WV, int FIRST = 0, bool PE0 = true, int PL>
__device__ __forceinline__ void stage_small_weights(const gp_head_weights& w, HeadSmem<NT, WV, PL>& sm) {
    static_assert(PE0 || PL, "the fp32 trunk reads pose_encoder.0 from LDS");
    constexpr int NTH = WV * 64 - FIRST;
    const int t0 = (int)threadIdx.x - FIRST;
    if (t0 < 0) return;
    if constexpr (PE0)
        for (int i = t0; i < 16 * 64; i += NTH) sm.pe0w[i] = ld4(w.pe0_w + (size_t)i * 4);
    for (int i = t0; i < HID; i += NTH) {
        if constexpr (PE0) sm.pe0b[i] = w.pe0_b[i];
        sm.pe2b[i] = w.pe2_b[i];
    }
    for (int i = t0; i < 9 * HID / 4; i += NTH) st4(&sm.h2w[i * 4], ld4(w.h2_w + (size_t)i * 4));
    if (t0 < 9) sm.h2b[t0] = w.h2_b[t0];
}

// Head output o of column c (valid after head_trunk): bias + the per-wave partials in wave order.
template <int NT, int WV, int PL>
__device__ __forceinline__ float head_out(const HeadSmem<NT, WV, PL>& sm, int c, int o) {
    const int h = o / 3;
    const int v = (h * NT + (c >> 4)) * 3 + (o - 3 * h);
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < WV; ++w) acc += sm.red[v][c & 15][w];
    return sm.h2b[o] + acc;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// acc[t][ct] += sum_g A(tile T[t], k-group g) . B(k-group g, column tile ct) over KG k-groups.
// A fragments stream from global (L2-resident packed weights) through a (D+1)-slot register ring
// so that the loads of k-group g+D are in flight while k-group g feeds the MFMAs; B fragments
// come from LDS. Loads are raw buffer loads: the tile/k-group offset is a wave-uniform SGPR
// (soffset) and the only per-lane address is lane*16 (voffset), so the fully unrolled ring needs
// no 64-bit address registers. Every ring index is a compile-time constant.
// Steps G..GEND-1 of the pipelined stream (step G issues k-group G's loads and computes k-group
// G-D). Steps 0..D-1 only prime the ring, so they can be issued early (before a barrier).
template <int G, int GEND, int TT, int NT, int KG, int D>
__device__ __forceinline__ void stream_step(__amdgpu_buffer_rsrc_t W, const int (&T)[TT], const f32x4* __restrict__ B,
                                            int lane, int voff, f32x4 (&ring)[D + 1][TT], f32x4 (&acc)[TT][NT]) {
    if constexpr (G < GEND) {
        if constexpr (G < KG) {
#pragma unroll
            for (int t = 0; t < TT; ++t) ring[G % (D + 1)][t] = ldbuf4(W, voff, (T[t] * KG + G) * 1024);
        }
        // keep the prefetch where it is: without this fence the scheduler sinks every load next to
        // its MFMAs and waits vmcnt(0) per k-group (checked in the .s)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (G >= D) {
            constexpr int GG = G - D;
            f32x4 bf[NT];
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) bf[ct] = B[(GG * NT + ct) * 64 + lane];
            // k-step outermost: consecutive MFMAs hit different accumulators (16x16x4 f32 has a
            // 40-cycle dependent latency vs a 32-cycle issue interval)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int ct = 0; ct < NT; ++ct)
                        acc[t][ct] = mfma4(ring[GG % (D + 1)][t][j], bf[ct][j], acc[t][ct]);
        }
        stream_step<G + 1, GEND, TT, NT, KG, D>(W, T, B, lane, voff, ring, acc);
    }
}

// acc[t][ct] += sum_g A(tile T[t], k-group g) . B(k-group g, column tile ct) over KG k-groups.
// A fragments stream from global (L2-resident packed weights) through a (D+1)-slot register ring
// so that the loads of k-group g+D are in flight while k-group g feeds the MFMAs; B fragments
// come from LDS. Loads are raw buffer loads: the tile/k-group offset is a wave-uniform SGPR
// (soffset) and the only per-lane address is lane*16 (voffset). The k-group loop is unrolled by
// template recursion, so every ring index is a compile-time constant (no scratch).
template <int TT, int NT, int KG, int D>
__device__ __forceinline__ void stream_layer(__amdgpu_buffer_rsrc_t W, const int (&T)[TT],
                                             const f32x4* __restrict__ B, int lane, f32x4 (&acc)[TT][NT]) {
    f32x4 ring[D + 1][TT];
    stream_step<0, KG + D, TT, NT, KG, D>(W, T, B, lane, lane * 16, ring, acc);
}

// Computes the head outputs (read with head_out) for the candidates of this workgroup. Starts with
// the workgroup barrier that publishes sm.xin, obj_of_col and the staged weights (callers write
// them before the call without a barrier of their own; the first weight loads are issued before it).
// `obj_of_col` maps column -> object row of pobj; `tproj` is the 768-vector of this time value.
template <int NT, int WV>
__device__ __forceinline__ void head_trunk(const gp_head_weights& w, const float* __restrict__ pobj,
                           const float* __restrict__ tproj, const int* obj_of_col, HeadSmem<NT, WV>& sm,
                           int trace_slot = 0) {
    constexpr int TPW = 16 / WV;   // output tiles per wave and per 256-wide layer
    static_assert(!HeadSmem<NT, WV>::kAliasAct, "the exact-fp32 trunk keeps separate activation buffers");
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (SGPR)
    const int q = lane >> 4, n = lane & 15;
    const int voff = lane * 16;
    const __amdgpu_buffer_rsrc_t W2 = make_rsrc(w.pe2_w, HID * HID * 4);
    const __amdgpu_buffer_rsrc_t WH = make_rsrc(w.h1p_w, 3 * HID * HID * 4);
    constexpr int D2 = PC_D2, DH = HEAD_PREFETCH;
    int T2[TPW], TH[3 * TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) T2[t] = wid * TPW + t;
#pragma unroll
    for (int h = 0; h < 3; ++h)
#pragma unroll
        for (int t = 0; t < TPW; ++t) TH[h * TPW + t] = h * 16 + wid * TPW + t;
    f32x4 acc2[TPW][NT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) acc2[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 ring2[D2 + 1][TPW];
    // prime pose_encoder.2's weight ring before pose_encoder.0 (no B operand read yet)
    stream_step<0, D2, TPW, NT, KG_HID, D2>(W2, T2, sm.act1, lane, voff, ring2, acc2);
    __syncthreads();
    PC_MARK(1);
    // ---- pose_encoder.0 (9 -> 256), one k-group
    {
        f32x4 bf[NT];
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) bf[ct] = ld4(&sm.xin[(ct * 16 + n) * 16 + 4 * q]);
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            const int T = wid * TPW + t;
            const f32x4 a = sm.pe0w[T * 64 + lane];
            const f32x4 bias = ld4(&sm.pe0b[16 * T + 4 * q]);
#pragma unroll
            for (int ct = 0; ct < NT; ++ct)
                sm.act1[(T * NT + ct) * 64 + lane] = relu4(mfma_kgroup(a, bf[ct], f32x4{0.f, 0.f, 0.f, 0.f}) + bias);
        }
    }
    __syncthreads();
    PC_MARK(2);
    // ---- pose_encoder.2 (256 -> 256): TPW output tiles per wave
    // the last PE2_TAIL k-groups of pose_encoder.2 run after the head-layer-1 accumulator-init loads
    // (hoisted pts/t blocks) are issued, so their latency hides behind MFMAs
    constexpr int PE2_TAIL = 4;
    stream_step<D2, KG_HID + D2 - PE2_TAIL, TPW, NT, KG_HID, D2>(W2, T2, sm.act1, lane, voff, ring2, acc2);
    f32x4 tpv[3 * TPW], pov[3 * TPW][NT];
#pragma unroll
    for (int i = 0; i < 3 * TPW; ++i) {
        const int T = TH[i];
        tpv[i] = ld4(tproj + 16 * T + 4 * q);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) pov[i][ct] = ld4(pobj + (size_t)obj_of_col[ct * 16 + n] * (3 * HID) + 16 * T + 4 * q);
    }
    stream_step<KG_HID + D2 - PE2_TAIL, KG_HID + D2, TPW, NT, KG_HID, D2>(W2, T2, sm.act1, lane, voff, ring2, acc2);
    // ---- head layer 1 prologue, issued before the barrier: the first DH k-groups of the pose-block
    //      weights
    PC_MARK(3);
    f32x4 acc[3 * TPW][NT];
#pragma unroll
    for (int i = 0; i < 3 * TPW; ++i)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) acc[i][ct] = pov[i][ct] + tpv[i];
    f32x4 ringh[DH + 1][3 * TPW];
    stream_step<0, DH, 3 * TPW, NT, KG_HID, DH>(WH, TH, sm.act2, lane, voff, ringh, acc);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const f32x4 bias = ld4(&sm.pe2b[16 * T2[t] + 4 * q]);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) sm.act2[(T2[t] * NT + ct) * 64 + lane] = relu4(acc2[t][ct] + bias);
    }
    __syncthreads();
    PC_MARK(4);
    // ---- head layer 1 (pose block 256 -> 3x256): 3*TPW output tiles per wave
    stream_step<DH, KG_HID + DH, 3 * TPW, NT, KG_HID, DH>(WH, TH, sm.act2, lane, voff, ringh, acc);
    PC_MARK(5);
    // ---- ReLU -> head layer 2 (block diagonal 3 x (256 -> 3)) partial dot products
#pragma unroll
    for (int h = 0; h < 3; ++h) {
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
            float p0 = 0.f, p1 = 0.f, p2 = 0.f;
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const f32x4 u = relu4(acc[h * TPW + t][ct]);
                const int ch = 16 * (wid * TPW + t) + 4 * q;
                const f32x4 w0 = ld4(&sm.h2w[(h * 3 + 0) * HID + ch]);
                const f32x4 w1 = ld4(&sm.h2w[(h * 3 + 1) * HID + ch]);
                const f32x4 w2 = ld4(&sm.h2w[(h * 3 + 2) * HID + ch]);
                p0 += u.x * w0.x + u.y * w0.y + u.z * w0.z + u.w * w0.w;
                p1 += u.x * w1.x + u.y * w1.y + u.z * w1.z + u.w * w1.w;
                p2 += u.x * w2.x + u.y * w2.y + u.z * w2.z + u.w * w2.w;
            }
            p0 = rows_sum(p0);
            p1 = rows_sum(p1);
            p2 = rows_sum(p2);
            if (q == 0) {
                sm.red[(h * NT + ct) * 3 + 0][n][wid] = p0;
                sm.red[(h * NT + ct) * 3 + 1][n][wid] = p1;
                sm.red[(h * NT + ct) * 3 + 2][n][wid] = p2;
            }
        }
    }
    __syncthreads();
    PC_MARK(6);
}

// ============================================================================ f16 MFMA helpers
// Split-f16 arithmetic on v_mfma_f32_16x16x32_f16 (16x the fp32 MFMA rate on gfx950). An operand is
// scaled by an exact power of two and split into f16 planes: x = hi + lo (hi = f16(x), lo = f16(x - hi),
// ~22 significant bits; the encoder's SA levels 1-3 and token GEMMs, gp_encoder.hip) or x = hi + mid + lo
// (every bit of an fp32 value: the head trunk below).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int KC_HID = HID / 32;   // 32-deep chunks over a 256-wide activation

__device__ __forceinline__ f32x4 mfma_h(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// 2^e (e clamped to the normal range) and floor(log2(v)) of a normal v > 0, both exact
__device__ __forceinline__ float exp2i(int e) {
    e = e < -126 ? -126 : (e > 127 ? 127 : e);
    return __uint_as_float((uint32_t)(e + 127) << 23);
}
__device__ __forceinline__ int ilog2f(float v) { return (int)((__float_as_uint(v) >> 23) & 0xff) - 127; }
// max over lanes l, l^16, l^32, l^48
__device__ __forceinline__ float rows_max(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// hi/lo planes of the 32-deep chunk made of two accumulator tiles (u: tile 2c, v: tile 2c+1), times
// s. Lane (q, n) holds k = 4q + j (j < 4) from u and 16 + 4q + j - 4 from v: the k order pack.py's
// pack_h16_fragments gives the weights.
__device__ __forceinline__ void split_pair(f32x4 u, f32x4 v, float s, f16x8& hi, f16x8& lo) {
#pragma clang fp contract(off)
    const float x[8] = {u.x * s, u.y * s, u.z * s, u.w * s, v.x * s, v.y * s, v.z * s, v.w * s};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)x[j];
        hi[j] = h;
        lo[j] = (_Float16)(x[j] - (float)h);
    }
}

// stream_step on f16 planes over KC 32-deep chunks: ring slot = [tile][hi, lo] of one chunk (2 x 1 KiB
// per tile, weights packed by pack.pack_h16_fragments as [T][chunk][plane][lane]); B = activation
// planes in LDS, [chunk][ct][hi, lo][lane].
template <int KC, int G, int GEND, int TT, int NT, int D>
__device__ __forceinline__ void stream_hk_step(__amdgpu_buffer_rsrc_t W, const int (&T)[TT], const f16x8* __restrict__ B,
                                               int lane, int voff, f16x8 (&ring)[D + 1][TT][2], f32x4 (&acc)[TT][NT]) {
    if constexpr (G < GEND) {
        if constexpr (G < KC) {
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    ring[G % (D + 1)][t][p] =
                        __builtin_bit_cast(f16x8, ldbuf4(W, voff, ((T[t] * KC + G) * 2 + p) * 1024));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (G >= D && NT > 4) {
            // wide column blocks (encoder levels 2-3): one column tile's planes live at a time
            constexpr int GG = G - D, S = GG % (D + 1);
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) {
                const f16x8 bh = B[((GG * NT + ct) * 2 + 0) * 64 + lane];
                const f16x8 bl = B[((GG * NT + ct) * 2 + 1) * 64 + lane];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][ct] = mfma_h(ring[S][t][1], bh, acc[t][ct]);
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][ct] = mfma_h(ring[S][t][0], bl, acc[t][ct]);
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][ct] = mfma_h(ring[S][t][0], bh, acc[t][ct]);
            }
        } else if constexpr (G >= D) {
            constexpr int GG = G - D, S = GG % (D + 1);
            f16x8 bh[NT], bl[NT];
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) {
                bh[ct] = B[((GG * NT + ct) * 2 + 0) * 64 + lane];
                bl[ct] = B[((GG * NT + ct) * 2 + 1) * 64 + lane];
            }
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int ct = 0; ct < NT; ++ct) acc[t][ct] = mfma_h(ring[S][t][1], bh[ct], acc[t][ct]);
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int ct = 0; ct < NT; ++ct) acc[t][ct] = mfma_h(ring[S][t][0], bl[ct], acc[t][ct]);
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int ct = 0; ct < NT; ++ct) acc[t][ct] = mfma_h(ring[S][t][0], bh[ct], acc[t][ct]);
        }
        stream_hk_step<KC, G + 1, GEND, TT, NT, D>(W, T, B, lane, voff, ring, acc);
    }
}


// The split trunk's activation bounds and weight exponents (gp_head_weights.hsc). Loaded at kernel entry by
// the callers: read where they are used, their round trip (a cold L2 line after the kernel boundary) sat
// on the critical path between the PC update and pose_encoder.0.
// Also this wave's pose_encoder.0 A fragments and bias (output tiles 2 wid, 2 wid + 1 of an 8-wave
// workgroup): loaded at kernel entry instead of being staged through LDS for every launch.
constexpr int HSPLIT_WV = 8;   // waves per workgroup of the split-trunk kernels
struct SplitScalars {
    float A0, B0, A2, B2;
    int ew2, ewh;
    f32x4 pe0a[4], pe0b[4];   // this wave's 16 / WV output tiles (entries past them unused)
};
template <int WV = HSPLIT_WV>
__device__ __forceinline__ SplitScalars load_split_scalars(const gp_head_weights& w) {
    static_assert(WV == 4 || WV == 8, "the split trunk runs 4- or 8-wave workgroups");
    const f32x4 a = ld4(w.hsc), b = ld4(w.hsc + 4);
    SplitScalars r{a.x, a.y, a.z, a.w, (int)b.x, (int)b.y, {}, {}};
    const int tid = tid_x();
    const int lane = tid & 63, q = lane >> 4;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
    for (int t = 0; t < 16 / WV; ++t) {
        const int T = wid * (16 / WV) + t;
        r.pe0a[t] = ld4(w.pe0_w + ((size_t)T * 64 + lane) * 4);
        r.pe0b[t] = ld4(w.pe0_b + 16 * T + 4 * q);
    }
    return r;
}

// Sums of four values over the four 16-lane rows, scattered: on return row q of the wave holds the
// total of value q (its column n's sum over lanes n, n+16, n+32, n+48). Three row swaps and three adds
// for four values (a full row sum of each would take eight and eight); the pairs are summed in
// rows_sum's order, (r0 + r1) + (r2 + r3), so each total has rows_sum's bits.
// v_permlane16_swap exchanges the odd rows of its first operand with the even rows of its second;
// v_permlane32_swap the upper half of the first with the lower half of the second.
__device__ __forceinline__ float rows_sum_scatter4(float a, float b, float c, float d) {
    const auto ab = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const auto cd = __builtin_amdgcn_permlane16_swap(__float_as_uint(c), __float_as_uint(d), false, false);
    const float s = __uint_as_float(ab[0]) + __uint_as_float(ab[1]);   // rows: a01, b01, a23, b23
    const float t = __uint_as_float(cd[0]) + __uint_as_float(cd[1]);   // rows: c01, d01, c23, d23
    const auto st = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(t), false, false);
    return __uint_as_float(st[0]) + __uint_as_float(st[1]);            // rows: a, b, c, d
}

// ReLU -> head layer 2 (block diagonal 3 x (256 -> 3)) partials of the split trunk's head-layer-1
// accumulators (scaled domain; uh[ct] undoes the scale, a power of two, so scaling each lane's chain
// before the row sum is exact). Each (column, output) is one fp32 FMA chain over this wave's channels,
// t-major then j, with separately rounded sums across rows and waves (head_out). Scalar FMAs: the
// same chains as v_pk_fma_f32 over column-tile pairs (broadcast weights through op_sel, results in

// A candidate's power-of-two scales of the split trunk from m0 = max |pose entry| (rigorous bounds of
// pose_encoder.0's and .2's outputs, hs): s1 / s2 scale the two activations into [2^14, 2^15) at their
// bound, u2 / uh undo both scales of pose_encoder.2 / head layer 1, sh brings head layer 1's fp32 init
// into the scaled domain. One definition for the trunk and the PC update waves that precompute it.
struct ColScales {
    float s1, s2, u2, uh, sh;
};
__device__ __forceinline__ ColScales split_col_scales(float m0, const SplitScalars& hs) {
    const float b1 = fmaxf(__builtin_fmaf(hs.A0, m0, hs.B0) * 1.0009765625f, 1e-18f);
    const float b2 = fmaxf(__builtin_fmaf(hs.A2, b1, hs.B2) * 1.0009765625f, 1e-18f);
    const int e1 = ilog2f(b1), e2 = ilog2f(b2);
    return ColScales{exp2i(14 - e1), exp2i(14 - e2), exp2i(e1 - 14 - hs.ew2), exp2i(e2 - 14 - hs.ewh),
                     exp2i(14 - e2 + hs.ewh)};
}
// max |x| of a 16-wide xin row held four entries per lane over the four 16-lane rows (the trunk's
// B-operand layout): the bound's m0
__device__ __forceinline__ float xin_row_absmax(f32x4 b) {
    return rows_max(fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)), fmaxf(fabsf(b.z), fabsf(b.w))));
}

// ============================================================================ f16x3 trunk
// The two per-candidate GEMMs (pose_encoder.2 and head layer 1's pose block) on
// v_mfma_f32_16x16x32_f16 with three f16 planes per operand: after an exact power-of-two scaling,
// x = hi + mid + lo with hi = f16(x), mid = f16(x - hi), lo = f16(x - hi - mid) holds every bit of an
// fp32 value (11 + 11 + 11 >= 24 significant bits; only values ~2^-7 below the operand's scale lose
// lo bits to f16 subnormals, an absolute error <= 2^-39 of the scale). Per 32-deep chunk, the six
// products whose plane orders sum to <= 2 (relative sizes 1, 2^-11, 2^-11, 2^-22 x3) are formed; the
// three dropped ones are <= 2^-33 relative, so every product w*a enters the sum to ~2^-33, finer than
// an fp32 FMA. hi*hi accumulates in one fp32 accumulator (one rounding per 32-deep chunk, as the
// MFMA sums its 32 exact f16 products and rounds once), the five cross products in a second one (its
// roundings are 2^-11 smaller), and the two are added once per layer: fewer roundings at full
// magnitude than v_mfma_f32_16x16x4_f32's one per 4-deep step (scripts/precision_study3.py,
// scripts/mfma_round_probe.hip). Six f16 MFMAs per 32x16x16 chunk-tile take 96 cycles against the
// exact fp32 MFMA's 256.
// Weights: per-layer exponents and packed hi/mid/lo planes (pack.pack_h16_fragments, 6 B per weight).
// Activations: a per-candidate exponent from a rigorous bound on the layer's outputs (max|pose| times
// the layer's max row L1 norm plus max|bias|, chained), so no extra barrier is needed and f16 cannot
// overflow. pose_encoder.0 and head layer 2 stay fp32 (VALU / fp32 MFMA).
#ifndef X3_D2
#define X3_D2 2                  // 32-deep chunks of pose_encoder.2 weights kept in flight
#endif
#ifndef X3_DH
#define X3_DH 1                  // 32-deep chunks of head-layer-1 weights kept in flight (2: ab_prio_dh1.json)
#endif
#ifndef X3_PRIO
#define X3_PRIO 0                // 1: alternate the issue priority of a SIMD's two waves per chunk (tuning)
#endif
#ifndef X3_BPIPE
#define X3_BPIPE 1               // B planes read one column tile ahead of their MFMAs (0: just in time;
                                 // profiles/r4/ab_bpipe.json)
#endif
#ifndef X3_CHAIN
#define X3_CHAIN 1               // each tile's correction products back to back (R=25,600 -3 %, R=12,800 even;
                                 // profiles/r4/ab_chain.json)
#endif
#ifndef X3_EPI_EARLY
#define X3_EPI_EARLY 1           // pose_encoder.2 epilogue planes computed before the alias barrier
                                 // (profiles/r4/ab_epi_early.json)
#endif
#ifndef X3_DIAG
#define X3_DIAG 0                // timing diagnostics only (wrong results), bits: 1 no B-plane LDS reads after
                                 // the first, 2 no weight loads after the ring's priming, 4 no head-layer-2
                                 // epilogue between the heads
#endif
#ifndef X3_HEAD_BARRIER
#define X3_HEAD_BARRIER 0        // 1: a workgroup barrier after each head of head layer 1 (tuning)
#endif
constexpr int X3P = 3;           // planes per operand

// x = h + m + l exactly (x finite, |x| < 65504; f16 subnormals aside)
__device__ __forceinline__ void split3(float x, _Float16& h, _Float16& m, _Float16& l) {
#pragma clang fp contract(off)
    h = (_Float16)x;
    const float r = x - (float)h;   // exact: x and h agree in sign and leading bits
    m = (_Float16)r;
    l = (_Float16)(r - (float)m);   // exact likewise; <= 3 significant bits remain
}
// The three planes of the 32-deep chunk made of two accumulator tiles (u: tile 2c, v: tile 2c+1),
// times s, in the k order of pack_h16_fragments (as split_pair).
__device__ __forceinline__ void split3_pair(f32x4 u, f32x4 v, float s, f16x8 (&p)[X3P]) {
#pragma clang fp contract(off)
    const float x[8] = {u.x * s, u.y * s, u.z * s, u.w * s, v.x * s, v.y * s, v.z * s, v.w * s};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        _Float16 h, m, l;
        split3(x[j], h, m, l);
        p[0][j] = h;
        p[1][j] = m;
        p[2][j] = l;
    }
}

// One pipelined step of a 256-deep f16x3 layer: step G issues the loads of chunk G (tile T[t]'s three
// weight planes, 3 KiB per tile: pack_h16_fragments' [T][c][plane][lane]) and computes chunk G - D from
// the ring; B = activation planes in LDS, [chunk][ct][plane][lane]. acc += hi*hi, cor += the five cross
// products, smallest first. The B planes of column tile ct + 1 are read while column tile ct's MFMAs
// run (X3_BPIPE; sched barriers keep the compiler from sinking the reads to their first use, where
// each became an lgkmcnt(0) stall). Steps 0..D-1 only prime the ring (no B or accumulator access), so
// they can run before a barrier or under another phase.
template <int G, int GEND, int TT, int NT, int D>
__device__ __forceinline__ void stream_x3_rec(__amdgpu_buffer_rsrc_t W, const int (&T)[TT], const f16x8* __restrict__ B,
                                              int lane, int voff, f16x8 (&ring)[D + 1][TT][X3P],
                                              f32x4 (&acc)[TT][NT], f32x4 (&cor)[TT][NT], f16x8 (&bc)[X3P]) {
    if constexpr (G < GEND) {
        if constexpr (G < KC_HID && ((X3_DIAG & 2) == 0 || G < D + 1)) {
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int p = 0; p < X3P; ++p)
                    ring[G % (D + 1)][t][p] =
                        __builtin_bit_cast(f16x8, ldbuf4(W, voff, ((T[t] * KC_HID + G) * X3P + p) * 1024));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (G >= D) {
            constexpr int GG = G - D, S = GG % (D + 1);
#if X3_PRIO
            // the two waves of a SIMD (w, w + 4) take turns at issue priority chunk by chunk, so neither runs
            // a whole stream ahead and leaves the other to finish it alone (tuning variant)
            if ((__builtin_amdgcn_readfirstlane(threadIdx.x >> 8) ^ GG) & 1)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
#endif
#if X3_BPIPE
            // B planes one column tile ahead: column tile ct + 1's (or the next chunk's first) reads are in
            // flight during column tile ct's MFMAs
            if constexpr (GG == 0) {
#pragma unroll
                for (int p = 0; p < X3P; ++p) bc[p] = B[p * 64 + lane];
            }
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) {
                f16x8 bn[X3P];
                const int nx = ct + 1 < NT ? (GG * NT + ct + 1) : ((GG + 1) * NT);
                if ((X3_DIAG & 1) == 0 && (ct + 1 < NT || GG + 1 < KC_HID)) {
#pragma unroll
                    for (int p = 0; p < X3P; ++p) bn[p] = B[(nx * X3P + p) * 64 + lane];
                }
#if X3_DIAG & 1
#pragma unroll
                for (int p = 0; p < X3P; ++p) {   // distinct operands per tile, so the MFMAs stay distinct
                    using u4 = __attribute__((ext_vector_type(4))) unsigned;
                    bn[p] = __builtin_bit_cast(f16x8, __builtin_bit_cast(u4, bc[p]) ^ (unsigned)(nx + 1));
                }
#endif
                __builtin_amdgcn_sched_barrier(0);   // the reads stay ahead of this column tile's MFMAs
                const f16x8 b0 = bc[0], b1 = bc[1], b2 = bc[2];
#if X3_CHAIN
                // each tile's five correction products back to back on one accumulator, then the main
                // products (the issue rate itself does not depend on the order, scripts/mfma_chain_probe.hip;
                // this order measured 3 % faster at two passes, even at one)
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    f32x4 c = cor[t][ct];
                    c = mfma_h(ring[S][t][2], b0, c);
                    c = mfma_h(ring[S][t][0], b2, c);
                    c = mfma_h(ring[S][t][1], b1, c);
                    c = mfma_h(ring[S][t][1], b0, c);
                    c = mfma_h(ring[S][t][0], b1, c);
                    cor[t][ct] = c;
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][ct] = mfma_h(ring[S][t][0], b0, acc[t][ct]);
#else
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    f32x4 c = cor[t][ct];
                    c = mfma_h(ring[S][t][2], b0, c);
                    c = mfma_h(ring[S][t][0], b2, c);
                    c = mfma_h(ring[S][t][1], b1, c);
                    c = mfma_h(ring[S][t][1], b0, c);
                    c = mfma_h(ring[S][t][0], b1, c);
                    cor[t][ct] = c;
                    acc[t][ct] = mfma_h(ring[S][t][0], b0, acc[t][ct]);
                }
#endif
                __builtin_amdgcn_sched_barrier(0);
                if (ct + 1 < NT || GG + 1 < KC_HID) {
#pragma unroll
                    for (int p = 0; p < X3P; ++p) bc[p] = bn[p];
                }
            }
#else
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) {
                const f16x8 b0 = B[((GG * NT + ct) * X3P + 0) * 64 + lane];
                const f16x8 b1 = B[((GG * NT + ct) * X3P + 1) * 64 + lane];
                const f16x8 b2 = B[((GG * NT + ct) * X3P + 2) * 64 + lane];
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    f32x4 c = cor[t][ct];
                    c = mfma_h(ring[S][t][2], b0, c);
                    c = mfma_h(ring[S][t][0], b2, c);
                    c = mfma_h(ring[S][t][1], b1, c);
                    c = mfma_h(ring[S][t][1], b0, c);
                    c = mfma_h(ring[S][t][0], b1, c);
                    cor[t][ct] = c;
                    acc[t][ct] = mfma_h(ring[S][t][0], b0, acc[t][ct]);
                }
            }
#endif
        }
        stream_x3_rec<G + 1, GEND, TT, NT, D>(W, T, B, lane, voff, ring, acc, cor, bc);
    }
}
template <int G, int GEND, int TT, int NT, int D>
__device__ __forceinline__ void stream_x3_step(__amdgpu_buffer_rsrc_t W, const int (&T)[TT], const f16x8* __restrict__ B,
                                               int lane, int voff, f16x8 (&ring)[D + 1][TT][X3P],
                                               f32x4 (&acc)[TT][NT], f32x4 (&cor)[TT][NT]) {
    f16x8 bc[X3P];   // X3_BPIPE: the B planes of the next column tile, carried from step to step
    stream_x3_rec<G, GEND, TT, NT, D>(W, T, B, lane, voff, ring, acc, cor, bc);
}

// The fp32 init rows of head layer 1 (hoisted pts + t blocks: pobj of each column's object, tproj) for this
// wave's output tiles of head H: loads issued where their latency hides (under the previous head's epilogue,
// or the pose_encoder.2 epilogue for head 0) and folded into the accumulator at the head's start, so they are
// not live across the MFMA stream.
template <int H, int NT, int TPW>
__device__ __forceinline__ void head_x3_init_load(__amdgpu_buffer_rsrc_t RP, __amdgpu_buffer_rsrc_t RT, const int (&vo)[NT],
                                                  int wid, int lane, f32x4 (&tpv)[TPW], f32x4 (&pov)[TPW][NT]) {
    const int q = lane >> 4;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int T = H * 16 + wid * TPW + t;
        tpv[t] = ldbuf4(RT, 16 * q, 64 * T);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) pov[t][ct] = ldbuf4(RP, vo[ct], 64 * T);
    }
}

// head_trunk with the f16x3 GEMMs (same contract: head_out reads the outputs after it returns).
// Head layer 1 runs one head at a time (2 output tiles per wave and head): the head's fp32 init rows
// enter its main accumulator in the scaled domain (x sh, a power of two: exact), hi*hi accumulates on top
// and the cross products beside it; the next head's first weight chunks and init rows are in flight during
// this head's layer-2 partials.
// PRE: the caller wrote every column's ColScales to sm.cscl before the trunk's first barrier (the PC
// step's update waves, which hold the rows), so the trunk reads them instead of recomputing them in
// every wave.
template <int H, int NT, int WV, int TPW, int DH>
__device__ __forceinline__ void head_x3_head(__amdgpu_buffer_rsrc_t WH, const f16x8* __restrict__ act2h,
                                             __amdgpu_buffer_rsrc_t RP, __amdgpu_buffer_rsrc_t RT, const int (&vo)[NT],
                                             HeadSmem<NT, WV, X3P>& sm, const float (&uh)[NT], const float (&sh)[NT],
                                             int wid, int lane, f16x8 (&ringh)[DH + 1][TPW][X3P],
                                             f32x4 (&tpv)[TPW], f32x4 (&pov)[TPW][NT],
                                             float (&pv)[HeadSmem<NT, WV, X3P>::kRedV]) {
    const int q = lane >> 4, n = lane & 15;
    const int voff = lane * 16;
    int TH[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) TH[t] = H * 16 + wid * TPW + t;
    f32x4 acc[TPW][NT], cor[TPW][NT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
            acc[t][ct] = (pov[t][ct] + tpv[t]) * sh[ct];
            cor[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    stream_x3_step<DH, KC_HID + DH, TPW, NT, DH>(WH, TH, act2h, lane, voff, ringh, acc, cor);
    if constexpr (H < 2) {   // the next head's first chunks and init rows, in flight across this epilogue
        int TN[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) TN[t] = TH[t] + 16;
        stream_x3_step<0, DH, TPW, NT, DH>(WH, TN, act2h, lane, voff, ringh, acc, cor);
        head_x3_init_load<H + 1, NT, TPW>(RP, RT, vo, wid, lane, tpv, pov);
    }
    // nothing below is scheduled into the MFMA stream above: interleaved there, the row swaps of the
    // reduce-scatter reused registers in-flight MFMAs still read (v_permlane*_swap writes both operands)
    __builtin_amdgcn_sched_barrier(0);
    // u = ReLU(scale-undone accumulators) -> head layer 2 (3 outputs) partials: one fp32 FMA chain per
    // (column, output) over this wave's channels, t-major then j
    float p[NT][3];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) p[ct][0] = p[ct][1] = p[ct][2] = 0.f;
#if X3_DIAG & 4
    // timing diagnostic: no layer-2 epilogue between the heads' streams (every accumulator still used)
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
            for (int o = 0; o < 3; ++o) p[ct][o] += acc[t][ct][o] + cor[t][ct][o + 1];
#else
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int ch = 16 * (wid * TPW + t) + 4 * q;
        const f32x4 w0 = ld4(&sm.h2w[(H * 3 + 0) * HID + ch]);
        const f32x4 w1 = ld4(&sm.h2w[(H * 3 + 1) * HID + ch]);
        const f32x4 w2 = ld4(&sm.h2w[(H * 3 + 2) * HID + ch]);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
            const f32x4 u = relu4((acc[t][ct] + cor[t][ct]) * uh[ct]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                p[ct][0] = __builtin_fmaf(u[j], w0[j], p[ct][0]);
                p[ct][1] = __builtin_fmaf(u[j], w1[j], p[ct][1]);
                p[ct][2] = __builtin_fmaf(u[j], w2[j], p[ct][2]);
            }
        }
    }
#endif
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int o = 0; o < 3; ++o) pv[(H * NT + ct) * 3 + o] = p[ct][o];
    // rows reduce-scatter (rows_sum_scatter4) of this head's values where they fill whole groups of four
    if constexpr ((3 * NT) % 4 == 0) {
#pragma unroll
        for (int g = H * 3 * NT / 4; g < (H + 1) * 3 * NT / 4; ++g)
            sm.red[4 * g + q][n][wid] = rows_sum_scatter4(pv[4 * g], pv[4 * g + 1], pv[4 * g + 2], pv[4 * g + 3]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int NT, int WV, bool PRE = false>
__device__ __forceinline__ void head_trunk_x3(const gp_head_weights& w, const float* __restrict__ pobj,
                                              const float* __restrict__ tproj, const int* obj_of_col,
                                              HeadSmem<NT, WV, X3P>& sm, int trace_slot, const SplitScalars hs) {
    constexpr int TPW = 16 / WV;   // output tiles per wave and 256-wide layer; tiles (2c, 2c+1) form chunk c
    static_assert(TPW % 2 == 0, "the f16x3 trunk pairs a wave's output tiles into 32-deep chunks");
    static_assert(TPW <= 4, "SplitScalars carries at most four pose_encoder.0 tiles per wave");
    constexpr int CPW = TPW / 2;
    using SM = HeadSmem<NT, WV, X3P>;
    const int tid = tid_x();
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, n = lane & 15;
    const int voff = lane * 16;
    const __amdgpu_buffer_rsrc_t W2 = make_rsrc(w.pe2_h, HID * HID * 2 * X3P);
    const __amdgpu_buffer_rsrc_t WH = make_rsrc(w.h1p_h, 3 * HID * HID * 2 * X3P);
    f16x8* act1h = reinterpret_cast<f16x8*>(sm.act1);
    f16x8* act2h = reinterpret_cast<f16x8*>(SM::kAliasAct ? sm.act1 : sm.act2);
    constexpr int D2 = X3_D2, DH = X3_DH;
    int T2[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) T2[t] = wid * TPW + t;
    f32x4 acc2[TPW][NT], cor2[TPW][NT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) acc2[t][ct] = cor2[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    f16x8 ring2[D2 + 1][TPW][X3P];
    stream_x3_step<0, D2, TPW, NT, D2>(W2, T2, act1h, lane, voff, ring2, acc2, cor2);
    __syncthreads();
    PC_MARK(1);
    // ---- per-candidate exponents: bound1 >= |pose_encoder.0 out|, bound2 >= |pose_encoder.2 out|
    f32x4 bf[NT];
    float s1[NT], s2[NT], u2[NT], uh[NT], sh[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
        bf[ct] = ld4(&sm.xin[(ct * 16 + n) * 16 + 4 * q]);
        ColScales cs;
        if constexpr (PRE) {
            const f32x4 a = sm.cscl[ct * 16 + n][0];
            cs = ColScales{a.x, a.y, a.z, a.w, sm.cscl[ct * 16 + n][1].x};
        } else {
            cs = split_col_scales(xin_row_absmax(bf[ct]), hs);
        }
        s1[ct] = cs.s1;
        s2[ct] = cs.s2;
        u2[ct] = cs.u2;
        uh[ct] = cs.uh;
        sh[ct] = cs.sh;
    }
    // ---- pose_encoder.0 (9 -> 256) in fp32, one k-group; ReLU, scale, split into the chunk planes
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int Ta = wid * TPW + 2 * c;
        const f32x4 a0 = hs.pe0a[2 * c], a1 = hs.pe0a[2 * c + 1];
        const f32x4 bias0 = hs.pe0b[2 * c], bias1 = hs.pe0b[2 * c + 1];
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
            const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
            f16x8 pl[X3P];
            split3_pair(relu4(mfma_kgroup(a0, bf[ct], z) + bias0), relu4(mfma_kgroup(a1, bf[ct], z) + bias1), s1[ct], pl);
#pragma unroll
            for (int p = 0; p < X3P; ++p) act1h[(((Ta >> 1) * NT + ct) * X3P + p) * 64 + lane] = pl[p];
        }
    }
    __syncthreads();
    PC_MARK(2);
    // ---- pose_encoder.2 (256 -> 256)
    stream_x3_step<D2, KC_HID + D2, TPW, NT, D2>(W2, T2, act1h, lane, voff, ring2, acc2, cor2);
    PC_MARK(3);
    // head layer 1's first chunks and init rows (head 0), in flight across the pose_encoder.2 epilogue
    f16x8 ringh[DH + 1][TPW][X3P];
    {
        int TH0[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) TH0[t] = wid * TPW + t;
        stream_x3_step<0, DH, TPW, NT, DH>(WH, TH0, act2h, lane, voff, ringh, acc2, cor2);
    }
    const __amdgpu_buffer_rsrc_t RP = make_rsrc(pobj, 0x7ffffff0u), RT = make_rsrc(tproj, 3 * HID * 4);
    int vo[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) vo[ct] = obj_of_col[ct * 16 + n] * (3 * HID * 4) + 16 * q;
    f32x4 tpv[TPW], pov[TPW][NT];
    head_x3_init_load<0, NT, TPW>(RP, RT, vo, wid, lane, tpv, pov);
#if X3_EPI_EARLY
    // the epilogue's planes are made before the alias barrier (a wave that finished its stream early does
    // this VALU work while it waits for the last one) and only written after it
    f16x8 pls[CPW][NT][X3P];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int Ta = T2[2 * c];
        const f32x4 bias0 = ld4(&sm.pe2b[16 * Ta + 4 * q]), bias1 = ld4(&sm.pe2b[16 * (Ta + 1) + 4 * q]);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
            split3_pair(relu4((acc2[2 * c][ct] + cor2[2 * c][ct]) * u2[ct] + bias0),
                        relu4((acc2[2 * c + 1][ct] + cor2[2 * c + 1][ct]) * u2[ct] + bias1), s2[ct], pls[c][ct]);
    }
    if constexpr (SM::kAliasAct) __syncthreads();   // act2 overwrites act1: all reads done
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
            for (int p = 0; p < X3P; ++p) act2h[(((T2[2 * c] >> 1) * NT + ct) * X3P + p) * 64 + lane] = pls[c][ct][p];
#else
    if constexpr (SM::kAliasAct) __syncthreads();   // act2 overwrites act1: all reads done
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int Ta = T2[2 * c];
        const f32x4 bias0 = ld4(&sm.pe2b[16 * Ta + 4 * q]), bias1 = ld4(&sm.pe2b[16 * (Ta + 1) + 4 * q]);
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
            f16x8 pl[X3P];
            split3_pair(relu4((acc2[2 * c][ct] + cor2[2 * c][ct]) * u2[ct] + bias0),
                        relu4((acc2[2 * c + 1][ct] + cor2[2 * c + 1][ct]) * u2[ct] + bias1), s2[ct], pl);
#pragma unroll
            for (int p = 0; p < X3P; ++p) act2h[(((Ta >> 1) * NT + ct) * X3P + p) * 64 + lane] = pl[p];
        }
    }
#endif
    __syncthreads();
    PC_MARK(4);
    // ---- head layer 1 (pose block 256 -> 3x256) head by head, each followed by its layer-2 partials
    float pv[SM::kRedV];
#pragma unroll
    for (int v = 9 * NT; v < SM::kRedV; ++v) pv[v] = 0.f;
#if X3_DIAG & 8
    // timing diagnostic: one wave per SIMD runs head layer 1 for its own output tiles and its sibling's (same
    // results), the sibling idles -- the single-wave stream rate inside the kernel
    if (wid < WV / 2) {
        head_x3_head<0, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
        PC_MARK(13);
        head_x3_head<1, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
        PC_MARK(14);
        head_x3_head<2, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
        const int vw = wid + WV / 2;
        int TV[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) TV[t] = vw * TPW + t;
        stream_x3_step<0, DH, TPW, NT, DH>(WH, TV, act2h, lane, voff, ringh, acc2, cor2);
        head_x3_init_load<0, NT, TPW>(RP, RT, vo, vw, lane, tpv, pov);
        head_x3_head<0, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, vw, lane, ringh, tpv, pov, pv);
        head_x3_head<1, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, vw, lane, ringh, tpv, pov, pv);
        head_x3_head<2, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, vw, lane, ringh, tpv, pov, pv);
    }
#else
    head_x3_head<0, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
    if constexpr (X3_HEAD_BARRIER) __syncthreads();
    PC_MARK(13);
    head_x3_head<1, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
    if constexpr (X3_HEAD_BARRIER) __syncthreads();
    PC_MARK(14);
    head_x3_head<2, NT, WV, TPW, DH>(WH, act2h, RP, RT, vo, sm, uh, sh, wid, lane, ringh, tpv, pov, pv);
#endif
    if constexpr (X3_PRIO) __builtin_amdgcn_s_setprio(0);
    PC_MARK(5);
    if constexpr ((3 * NT) % 4 != 0) {
#pragma unroll
        for (int g = 0; g < SM::kRedV / 4; ++g)
            sm.red[4 * g + q][n][wid] = rows_sum_scatter4(pv[4 * g], pv[4 * g + 1], pv[4 * g + 2], pv[4 * g + 3]);
    }
    __syncthreads();
    PC_MARK(6);
}

// ============================================================================ tile width
#ifndef PC_SPLIT_NT2_MIN
#define PC_SPLIT_NT2_MIN 4097   // rows from which the split kernels take 32-candidate tiles (> 256 tiles of 16)
#endif
#ifndef PC_SPLIT_NT4_MIN
#define PC_SPLIT_NT4_MIN 8193   // ... and 64-candidate tiles (> 256 tiles of 32)
#endif
// Column tiles (16 candidates each) per workgroup of the per-candidate head kernels (PC step, ODE stages).
// exact fp32 (scripts/kbench.py): 16 candidates x 8 waves per workgroup beats 32 x 4 at every size
// (R=25,600: 125 vs 153 us/step): 112 VGPRs leave room for two workgroups per CU, while the 32-wide
// tile needs 373 registers (one wave per SIMD).
// split-f16: each workgroup streams the 1 MB of GEMM weights once per launch whatever its width, so
// wider tiles cut the weight stream per candidate once there are enough tiles. One workgroup per CU
// either way (the LDS of a 32- or 64-candidate tile), so the tile width is the smallest that keeps the
// launch within one pass of the 256 CUs, or the widest above that.
static inline int head_pick_nt(int rows, bool split) {
    if (!split) return 1;
    return rows >= PC_SPLIT_NT4_MIN ? 4 : (rows >= PC_SPLIT_NT2_MIN ? 2 : 1);
}

// ============================================================================ pose helpers
template <typename T>
__device__ __forceinline__ T tsqrt(T v);
template <>
__device__ __forceinline__ float tsqrt<float>(float v) { return sqrtf(v); }
template <>
__device__ __forceinline__ double tsqrt<double>(double v) { return sqrt(v); }

// normalize_rotation(.., 'rot_matrix') (misc.py:327-344): rotation_6d_to_matrix GS with
// F.normalize's eps 1e-12 (rotation_conversions.py:571-575).
template <typename T>
__device__ __forceinline__ void gram_schmidt6(T* v) {
#pragma clang fp contract(off)
    T n1 = tsqrt<T>((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    n1 = n1 > (T)1e-12 ? n1 : (T)1e-12;
    const T b0 = v[0] / n1, b1 = v[1] / n1, b2 = v[2] / n1;
    const T d = (b0 * v[3] + b1 * v[4]) + b2 * v[5];
    T c0 = v[3] - d * b0, c1 = v[4] - d * b1, c2 = v[5] - d * b2;
    T n2 = tsqrt<T>((c0 * c0 + c1 * c1) + c2 * c2);
    n2 = n2 > (T)1e-12 ? n2 : (T)1e-12;
    v[0] = b0;
    v[1] = b1;
    v[2] = b2;
    v[3] = c0 / n2;
    v[4] = c1 / n2;
    v[5] = c2 / n2;
}

// Division / square root of the PC update chain: IEEE by default; PC_FAST_UPDATE builds use the
// hardware v_rcp_f32 / v_sqrt_f32 (<= 1 ulp) to shorten wave 0's dependent chain (tuning only).
#ifdef PC_FAST_UPDATE
__device__ __forceinline__ float udiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float usqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
#else
__device__ __forceinline__ float udiv(float a, float b) { return fdiv(a, b); }
__device__ __forceinline__ float usqrt(float x) { return sqrtf(x); }
#endif

// gram_schmidt6 spread over the four lanes of a row (lane part p: 0 -> v[0:3], 1 -> v[3:6],
// 2 -> translation, untouched; 3 idle). Same operations and order as gram_schmidt6<float>.
__device__ __forceinline__ void gram_schmidt6_quad(float* v, int p, int lane) {
#pragma clang fp contract(off)
    float n1 = usqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    n1 = n1 > 1e-12f ? n1 : 1e-12f;
    const float b0 = udiv(v[0], n1), b1 = udiv(v[1], n1), b2 = udiv(v[2], n1);   // meaningful on p == 0
    (void)lane;
    const float B0 = quad_bcast0(b0), B1 = quad_bcast0(b1), B2 = quad_bcast0(b2);
    const float d = (B0 * v[0] + B1 * v[1]) + B2 * v[2];
    float c0 = v[0] - d * B0, c1 = v[1] - d * B1, c2 = v[2] - d * B2;
    float n2 = usqrt((c0 * c0 + c1 * c1) + c2 * c2);
    n2 = n2 > 1e-12f ? n2 : 1e-12f;
    if (p == 0) {
        v[0] = b0; v[1] = b1; v[2] = b2;
    } else if (p == 1) {
        v[0] = udiv(c0, n2); v[1] = udiv(c1, n2); v[2] = udiv(c2, n2);
    }
}

// matrix_to_quaternion (rotation_conversions.py:102-161) of R = [b1 b2 b1xb2] (columns), input
// already Gram-Schmidt'ed; returns wxyz.
template <typename T>
__device__ __forceinline__ void quat_from_gs(const T* v, T* qo) {
#pragma clang fp contract(off)
    // second GS pass as get_rot_matrix applies rotation_6d_to_matrix again (posenet_agent.py:554)
    T g[6] = {v[0], v[1], v[2], v[3], v[4], v[5]};
    gram_schmidt6<T>(g);
    const T b3x = g[1] * g[5] - g[2] * g[4];
    const T b3y = g[2] * g[3] - g[0] * g[5];
    const T b3z = g[0] * g[4] - g[1] * g[3];
    const T m00 = g[0], m01 = g[3], m02 = b3x;
    const T m10 = g[1], m11 = g[4], m12 = b3y;
    const T m20 = g[2], m21 = g[5], m22 = b3z;
    const T one = (T)1;
    T qa[4] = {((one + m00) + m11) + m22, ((one + m00) - m11) - m22, ((one - m00) + m11) - m22,
               ((one - m00) - m11) + m22};
#pragma unroll
    for (int i = 0; i < 4; ++i) qa[i] = qa[i] > (T)0 ? tsqrt<T>(qa[i]) : (T)0;
    int best = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (qa[i] > qa[best]) best = i;
    T c[4];
    if (best == 0) {
        c[0] = qa[0] * qa[0]; c[1] = m21 - m12; c[2] = m02 - m20; c[3] = m10 - m01;
    } else if (best == 1) {
        c[0] = m21 - m12; c[1] = qa[1] * qa[1]; c[2] = m10 + m01; c[3] = m02 + m20;
    } else if (best == 2) {
        c[0] = m02 - m20; c[1] = m10 + m01; c[2] = qa[2] * qa[2]; c[3] = m12 + m21;
    } else {
        c[0] = m10 - m01; c[1] = m20 + m02; c[2] = m21 + m12; c[3] = qa[3] * qa[3];
    }
    const T den = (T)2 * (qa[best] > (T)0.1 ? qa[best] : (T)0.1);
#pragma unroll
    for (int i = 0; i < 4; ++i) qo[i] = c[i] / den;
}

// Head layer-1 t block for one time value (HT threads): tproj = W1_t . relu(W_te . [sin, cos](GFP(t)) + b_te)
// (scorenet.py:77-88 GaussianFourierProjection + t_encoder, the t columns of the first head layer).
// Writes out[o] for o in [o0, o1) (the caller's slice of the 768-row).
// sum_c W[c * stride] * x[c] over N = CH * L terms as CH interleaved fp32 chains (chain j: c = j, j + CH,
// ...) combined by a pairwise tree -- the accumulation pattern of a vectorised CPU GEMM. A single
// N-term chain is ~sqrt(N) roundings deep; the energy's pose . score sums cancel enough to expose it
// (the 1024-term pts block of head layer 1 was 2x the reference's own fp32 error at R=12,800).
template <int N, int CH>
__device__ __forceinline__ float dot_chains(const float* __restrict__ W, size_t stride, const float* x) {
    static_assert(N % CH == 0 && (CH & (CH - 1)) == 0, "N must be a multiple of the power-of-two CH");
    float p[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) p[j] = 0.f;
#pragma unroll 1
    for (int c0 = 0; c0 < N; c0 += CH) {
#pragma unroll
        for (int j = 0; j < CH; ++j) p[j] = fmaf(W[(size_t)(c0 + j) * stride], x[c0 + j], p[j]);
    }
#pragma unroll
    for (int s = CH / 2; s >= 1; s >>= 1)
#pragma unroll
        for (int j = 0; j < s; ++j) p[j] += p[j + s];
    return p[0];
}

// HOIST64 (diagnostic builds): the hoisted head-1 rows' GEMMs (object block, t_encoder, t block) accumulated in
// float64 and rounded once -- how far the order of those sums moves the T0=1 ODE path (tests/test_gpu_parity.py
// test_ode_t1_calibrated_vs_float64). The Fourier embedding stays the reference's float32 computation.
#ifndef HOIST64
#define HOIST64 0
#endif
template <int N>
__device__ __forceinline__ double dot_f64(const float* __restrict__ W, size_t stride, const float* x) {
    double s = 0.0;   // each fp32 x fp32 product is exact in float64
#pragma unroll 8
    for (int c = 0; c < N; ++c) s = fma((double)W[(size_t)c * stride], (double)x[c], s);
    return s;
}

__device__ __forceinline__ void time_row(const gp_head_weights& w, float t, float* emb, float* tf,
                                         float* __restrict__ out, int o0 = 0, int o1 = 768) {
    const int i = threadIdx.x;
    if (i < 64) {  // x_proj = x[:, None] * W[None, :] * 2 * np.pi (scorenet.py:87)
        const float a = fmul(fmul(fmul(t, w.gfp_w[i]), 2.0f), 3.14159265358979323846f);
        emb[i] = sinf(a);
        emb[64 + i] = cosf(a);
    }
    __syncthreads();
#if HOIST64
    if (i < 128) tf[i] = fmaxf((float)(dot_f64<128>(w.te_w_t + i, 128, emb) + (double)w.te_b[i]), 0.f);
    __syncthreads();
    for (int o = o0 + i; o < o1; o += HT) out[o] = (float)dot_f64<128>(w.h1t_t + o, 768, tf);
#else
    if (i < 128) tf[i] = fmaxf(dot_chains<128, 16>(w.te_w_t + i, 128, emb) + w.te_b[i], 0.f);
    __syncthreads();
    for (int o = o0 + i; o < o1; o += HT) out[o] = dot_chains<128, 16>(w.h1t_t + o, 768, tf);
#endif
}
