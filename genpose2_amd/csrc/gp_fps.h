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

__device__ __forceinline__ unsigned long long fps_pack(float d2, uint32_t key) {
    return ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned long long)(0xFFFFFFFFu - key);
}

constexpr int FPS_THREADS = 256;

// Wave-wide max of a 64-bit key: DPP steps within each 16-lane row (quad perms, half/full row
// mirror), then the gfx950 row swaps (v_permlane16_swap / v_permlane32_swap) across rows. Every
// lane ends with the maximum; one 64-bit compare per step.
#define GP_DPP_MAX_STEP(CTRL)                                                                   \
    {                                                                                           \
        const uint32_t ohi = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, CTRL, 0xF, 0xF, false); \
        const uint32_t olo = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, CTRL, 0xF, 0xF, false); \
        const bool take = (((unsigned long long)ohi << 32) | olo) > (((unsigned long long)hi << 32) | lo); \
        hi = take ? ohi : hi;                                                                   \
        lo = take ? olo : lo;                                                                   \
    }
#define GP_SWAP_MAX_STEP(SWAP)                                                                  \
    {                                                                                           \
        const auto h = SWAP(hi, hi, false, false);                                              \
        const auto l = SWAP(lo, lo, false, false);                                              \
        const bool take = (((unsigned long long)h[1] << 32) | l[1]) > (((unsigned long long)h[0] << 32) | l[0]); \
        hi = take ? h[1] : h[0];                                                                \
        lo = take ? l[1] : l[0];                                                                \
    }

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
    uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    GP_DPP_MAX_STEP(0xB1)   // quad_perm [1,0,3,2]
    GP_DPP_MAX_STEP(0x4E)   // quad_perm [2,3,0,1]
    GP_DPP_MAX_STEP(0x141)  // row_half_mirror
    GP_DPP_MAX_STEP(0x140)  // row_mirror
    GP_SWAP_MAX_STEP(__builtin_amdgcn_permlane16_swap)
    GP_SWAP_MAX_STEP(__builtin_amdgcn_permlane32_swap)
    const uint32_t rhi = (uint32_t)__builtin_amdgcn_readfirstlane((int)hi);
    const uint32_t rlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
    return ((unsigned long long)rhi << 32) | rlo;
}

constexpr int FPS_RED_BYTES = 2 * 16 * 8;   // double-buffered per-wave 64-bit maxima, up to 16 waves

// One FPS run over `n` points held in LDS (s_xyz, xyz interleaved). Writes the m indices to
// s_idx and the selected coordinates to s_out (both LDS; s_out may be null). Nothing touches
// global memory inside the iteration loop, so the per-iteration barrier never waits on a store.
// All NTH threads must call it. s_red holds FPS_RED_BYTES.
// Measured slower and not kept (level 0 at B=64): carrying the winner's coordinates through the
// exchange instead of re-reading them from s_xyz (411 vs 327 us); two 32-bit DPP maxima (distance,
// then key) instead of one 64-bit maximum of the packed pair (436 vs 309 us).
template <int PMAX, int NTH = FPS_THREADS>
__device__ void fps_run(const float* s_xyz, int n, int m, int nb, int jbits, void* s_red_v, int* s_idx,
                        float* s_out) {
    unsigned long long* s_red = reinterpret_cast<unsigned long long*>(s_red_v);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float px[PMAX], py[PMAX], pz[PMAX], tmin[PMAX];
    uint32_t key[PMAX];
#pragma unroll
    for (int p = 0; p < PMAX; ++p) {
        const int k = tid + p * NTH;
        const bool ok = k < n;
        px[p] = ok ? s_xyz[3 * k + 0] : 0.f;
        py[p] = ok ? s_xyz[3 * k + 1] : 0.f;
        pz[p] = ok ? s_xyz[3 * k + 2] : 0.f;
        tmin[p] = 1e10f;                        // pointnet2_utils.py:32-34
        key[p] = ok ? fps_key(k, nb, jbits) : 0u;
    }
    int old = 0;
    if (m <= 0) return;
    if (tid == 0) s_idx[0] = 0;
    if (tid < 3 && s_out) s_out[tid] = s_xyz[tid];
    for (int j = 1; j < m; ++j) {
        const float x1 = s_xyz[3 * old + 0], y1 = s_xyz[3 * old + 1], z1 = s_xyz[3 * old + 2];
        unsigned long long best = 0ull;
#pragma unroll
        for (int p = 0; p < PMAX; ++p) {
            const int k = tid + p * NTH;
            if (k < n) {
                const float d = dist2_ref(px[p], py[p], pz[p], x1, y1, z1);
                const float d2 = fminf(d, tmin[p]);
                tmin[p] = d2;
                const unsigned long long c = fps_pack(d2, key[p]);
                best = c > best ? c : best;
            }
        }
        best = wave_max_u64(best);
        unsigned long long* red = s_red + (j & 1) * 16;
        if (lane == 0) red[wid] = best;
        __syncthreads();
        unsigned long long b = red[0];
#pragma unroll
        for (int w = 1; w < NTH / 64; ++w) b = red[w] > b ? red[w] : b;
        old = fps_key_to_k(0xFFFFFFFFu - (uint32_t)(b & 0xFFFFFFFFull), nb, jbits);
        if (tid == 0) s_idx[j] = old;
        if (tid < 3 && s_out) s_out[3 * j + tid] = s_xyz[3 * old + tid];
    }
}

