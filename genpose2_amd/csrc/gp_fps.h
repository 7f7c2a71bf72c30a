// Farthest-point sampling core shared by the FPS kernels (gp_geometry.hip) and the encoder, which
// runs FPS levels as extra workgroups of its MLP launches (gp_encoder.hip). See gp_geometry.hip
// for the tie rule.
#pragma once
#include "gp_common.h"

// ============================================================================ FPS
static inline int fps_block_log2(int n) {  // cuda_utils.h:9-13 (opt_n_threads), exact for n>=1
    int p = 0;
    while ((2 << p) <= n && p < 10) ++p;
    return p;
}

struct FpsGeom {
    int nb;      // log2 of the reference block size
    int jbits;   // bits for k / bs
};

static inline FpsGeom fps_geom(int n) {
    FpsGeom g;
    g.nb = fps_block_log2(n);
    const int jmax = (n - 1) >> g.nb;
    g.jbits = 0;
    while ((1 << g.jbits) <= jmax) ++g.jbits;
    return g;
}

__device__ __forceinline__ uint32_t fps_key(int k, int nb, int jbits) {
    const uint32_t t = (uint32_t)k & ((1u << nb) - 1u);
    const uint32_t rt = nb ? (__brev(t) >> (32 - nb)) : 0u;
    return (rt << jbits) | ((uint32_t)k >> nb);
}

__device__ __forceinline__ int fps_key_to_k(uint32_t key, int nb, int jbits) {
    const uint32_t rt = key >> jbits;
    const uint32_t t = nb ? (__brev(rt) >> (32 - nb)) : 0u;
    return (int)(t + ((key & ((1u << jbits) - 1u)) << nb));
}

constexpr int FPS_THREADS = 256;

constexpr int FPS_RED_BYTES = 2 * 16 * 8;   // double-buffered per-wave 64-bit maxima, up to 16 waves

// The packed (distance, ~key) pair read as an f64. Its high word is a finite non-negative f32, so
// the pattern is a finite non-negative double (exponent field <= 0x7F7, never NaN/Inf) and f64
// order equals the unsigned order of the 64-bit pattern, denormals included (the kernels run with
// f64 denormals preserved: float_denorm_mode_16_64 = 3). One v_max_f64 therefore does the work of
// a 64-bit compare plus two selects. Inline asm keeps LLVM from canonicalising the DPP'd inputs.
__device__ __forceinline__ double fps_pack_f64(float d2, uint32_t low) {
    return __hiloint2double(__float_as_int(d2), (int)low);
}

__device__ __forceinline__ double fps_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int CTRL>
__device__ __forceinline__ double fps_dpp(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Wave-wide max (every lane ends with it): DPP within each 16-lane row, then the gfx950 row
// swaps (v_permlane16_swap / v_permlane32_swap) across rows.
__device__ __forceinline__ double fps_wave_max(double v) {
    v = fps_max(v, fps_dpp<0xB1>(v));    // quad_perm [1,0,3,2]
    v = fps_max(v, fps_dpp<0x4E>(v));    // quad_perm [2,3,0,1]
    v = fps_max(v, fps_dpp<0x141>(v));   // row_half_mirror
    v = fps_max(v, fps_dpp<0x140>(v));   // row_mirror
    {
        const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
        const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
        v = fps_max(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
    }
    {
        const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
        const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
        v = fps_max(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
    }
    return v;
}

// One FPS run over `n` points held in LDS (s_xyz, xyz interleaved). Writes the m indices to
// s_idx and, after the loop, the selected coordinates to s_out (both LDS; s_out may be null).
// Nothing touches global memory inside the iteration loop, so the per-iteration barrier never
// waits on a store. All NTH threads must call it. s_red holds FPS_RED_BYTES.
// Per iteration: distance update + local max of packed pairs, a wave max (6 DPP/swap steps),
// one barrier, then a DPP tree over the per-wave maxima (lane i reads wave i % NW) and the key
// decode on the scalar unit. Points past n carry the packed value 0 (distance 0, low word 0), which
// never beats a real point, so the loop has no bounds branches.
// Measured slower and not kept (level 0 at B=64): carrying the winner's coordinates through the
// exchange instead of re-reading them from s_xyz (411 vs 327 us); two 32-bit DPP maxima (distance,
// then key) instead of one 64-bit maximum of the packed pair (436 vs 309 us).
template <int PMAX, int NTH = FPS_THREADS>
__device__ void fps_run(const float* s_xyz, int n, int m, int nb, int jbits, void* s_red_v, int* s_idx,
                        float* s_out) {
    constexpr int NW = NTH / 64;
    static_assert(NW >= 1 && NW <= 16 && (NW & (NW - 1)) == 0, "NTH must be 64 * 2^k, at most 1024");
    double* s_red = reinterpret_cast<double*>(s_red_v);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float px[PMAX], py[PMAX], pz[PMAX], tmin[PMAX];
    uint32_t low[PMAX];
#pragma unroll
    for (int p = 0; p < PMAX; ++p) {
        const int k = tid + p * NTH;
        const bool ok = k < n;
        px[p] = ok ? s_xyz[3 * k + 0] : 0.f;
        py[p] = ok ? s_xyz[3 * k + 1] : 0.f;
        pz[p] = ok ? s_xyz[3 * k + 2] : 0.f;
        tmin[p] = ok ? 1e10f : 0.f;             // pointnet2_utils.py:32-34
        low[p] = ok ? 0xFFFFFFFFu - fps_key(k, nb, jbits) : 0u;
    }
    if (m <= 0) return;
    if (tid == 0) s_idx[0] = 0;
    const uint32_t kmask = (1u << jbits) - 1u;
    int old = 0;
    for (int j = 1; j < m; ++j) {
        const float x1 = s_xyz[3 * old + 0], y1 = s_xyz[3 * old + 1], z1 = s_xyz[3 * old + 2];
        double best;
#pragma unroll
        for (int p = 0; p < PMAX; ++p) {
            const float d = dist2_ref(px[p], py[p], pz[p], x1, y1, z1);
            const float d2 = fminf(d, tmin[p]);
            tmin[p] = d2;
            best = p ? fps_max(best, fps_pack_f64(d2, low[p])) : fps_pack_f64(d2, low[p]);
        }
        best = fps_wave_max(best);
        double* red = s_red + (j & 1) * 16;
        if (lane == 0) red[wid] = best;
        __syncthreads();
        double v = red[lane & (NW - 1)];
        if constexpr (NW >= 2) v = fps_max(v, fps_dpp<0xB1>(v));
        if constexpr (NW >= 4) v = fps_max(v, fps_dpp<0x4E>(v));
        if constexpr (NW >= 8) v = fps_max(v, fps_dpp<0x141>(v));
        if constexpr (NW >= 16) v = fps_max(v, fps_dpp<0x140>(v));
        const uint32_t key = 0xFFFFFFFFu - (uint32_t)__builtin_amdgcn_readfirstlane(__double2loint(v));
        const uint32_t rt = key >> jbits;
        const uint32_t t = nb ? (__builtin_bitreverse32(rt) >> (32 - nb)) : 0u;
        old = (int)(t + ((key & kmask) << nb));
        if (tid == 0) s_idx[j] = old;
    }
    if (s_out) {
        __syncthreads();
        for (int i = tid; i < 3 * m; i += NTH) {
            const int j = i / 3;
            s_out[i] = s_xyz[3 * s_idx[j] + (i - 3 * j)];
        }
    }
}
