// Shared device helpers for the GenPose++ MI355X kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/genpose_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define GP_WAVE 64

// --------------------------------------------------------------- error plumbing (host)
void gp_set_error(const char* fmt, ...);
int gp_check_launch(const char* what);
// the split linear with implicit im2col of a 3x3 conv (gp_fusion.hip; used by the image encoder, not part of the ABI)
int gp_linear_split_conv3x3(const float* f, int b, int g, int d, const int32_t* wpk, const float* bias, int n,
                            float* y, const float* rmax, hipStream_t st);

#define GP_REQUIRE(cond, ...)                   \
    do {                                        \
        if (!(cond)) {                          \
            gp_set_error(__VA_ARGS__);          \
            return GP_ERR_INVALID;              \
        }                                       \
    } while (0)

// --------------------------------------------------------------- MFMA (exact f32)
// D = A(16x4) * B(4x16) + C.  Lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; C/D lane l
// holds rows 4*(l>>4)+j, column l&15 (j = register 0..3).
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
#ifdef GP_DIAG_NO_MFMA   // diagnostic builds only: one VALU FMA instead (results are meaningless)
    c.x = __builtin_fmaf(a, b, c.x);
    return c;
#else
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#endif
}

// One 16-deep k-group: 4 MFMAs with the lane's A float4 / B float4 (k = 16g + 4q + j).
__device__ __forceinline__ f32x4 mfma_kgroup(const f32x4 a, const f32x4 b, f32x4 c) {
    c = mfma4(a.x, b.x, c);
    c = mfma4(a.y, b.y, c);
    c = mfma4(a.z, b.z, c);
    c = mfma4(a.w, b.w, c);
    return c;
}

// max(v, 0) as one instruction (v_maximum3_f32 v, 0, 0): fmaxf on a value the compiler cannot prove canonical (an MFMA or
// load result) is preceded by a v_max_f32 v, v, v that quiets signalling NaNs, doubling every ReLU.
// IEEE maximum needs no quieting; it propagates NaN as torch.relu does (fmaxf maps NaN to 0).
__device__ __forceinline__ float relu1(float v) { return __builtin_elementwise_maximum(v, 0.f); }
__device__ __forceinline__ f32x4 relu4(f32x4 v) { return f32x4{relu1(v.x), relu1(v.y), relu1(v.z), relu1(v.w)}; }

typedef __attribute__((address_space(3))) void* lds_void_ptr;   // LDS-DMA destination

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// One 4-byte global load that the backend never merges with its neighbours (a relaxed workgroup-scope atomic
// load: a plain global_load_dword, sc0, cached as usual). Three consecutive floats (coordinates, a pose
// row's three entries) are read through it. Observed, not explained: with a merged global_load_dwordx3 feeding
// a packed-FP32 instruction (v_pk_fma_f32 reading the load's register pair), the level-0 projection lost its y
// term in a few 16-lane groups per thousand launches, only while other processes' kernels shared the GPU; with
// 4-byte loads it never did (A/B in DESIGN (c), scripts/race_probe.py). The hardware cause -- wave state lost
// across a context switch between processes -- is a HYPOTHESIS that user code cannot confirm. The guard is
// behavioural (race_probe.py) plus static (tests/test_cpu_host.py: no 12-byte loads, no vector loads from the
// kernel-argument segment). Kernels that still stage data in LDS behind a barrier and were cleared only by
// finite probes (0 differing repetitions), not by construction: the level-0 FPS chain (gp_fps.h), the SA
// gathers (gp_encoder.hip), the relative-PE key coordinates (gp_fusion.hip mha_relpe_kernel) and the PC / ODE
// trunks' activation planes (gp_head.h).
__device__ __forceinline__ float ld1(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Buffer resource over `bytes` bytes at p (p must be wave-uniform: a kernel argument).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 16-byte buffer load: voffset per lane (VGPR), soffset wave-uniform (SGPR).
__device__ __forceinline__ f32x4 ldbuf4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
#ifdef GP_DIAG_NO_WLOAD   // diagnostic builds only: no weight stream (results are meaningless)
    (void)r;
    const float v = (float)(voff + soff) * 1e-9f;
    return f32x4{v, v, v, v};
#else
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
#endif
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// Non-contracted fp32 arithmetic (mirrors the reference's separately rounded ops). hipcc's
// __fmul_rn is a plain multiply that -ffp-contract=fast may still fuse into v_fma, so every
// helper carries its own `fp contract(off)` scope.
__device__ __forceinline__ float fmul(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ float fadd(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ float fsub(float a, float b) {
#pragma clang fp contract(off)
    return a - b;
}
__device__ __forceinline__ float fdiv(float a, float b) {
#pragma clang fp contract(off)
    return a / b;
}

// Squared distance exactly as the reference CUDA text writes it: (dx*dx + dy*dy) + dz*dz
// with every operation rounded separately (no FMA contraction, no reassociation).
__device__ __forceinline__ float dist2_ref(float ax, float ay, float az, float bx, float by, float bz) {
#pragma clang fp contract(off)
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    return (dx * dx + dy * dy) + dz * dz;
}

// --------------------------------------------------------------- cross-lane sums (no LDS)
// DPP within 16-lane rows, then the gfx950 row swaps (v_permlane16_swap / v_permlane32_swap):
// every lane ends with the same bits, and the summation order is fixed, so every workgroup that
// runs the same code reduces identically.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over lanes l, l^16, l^32, l^48 (the four rows' lane n)
__device__ __forceinline__ float rows_sum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// sum over the 16 lanes of each row (every lane of the row ends with the row's sum)
__device__ __forceinline__ float row16_sum(float v) {
    v = dpp_add<0xB1>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x141>(v);   // row_half_mirror
    return dpp_add<0x140>(v);   // row_mirror
}
__device__ __forceinline__ float wave_sum(float v) { return rows_sum(row16_sum(v)); }
// max over the 16 lanes of each row, DPP only (no ds_bpermute round trip through LDS)
template <int CTRL>
__device__ __forceinline__ float dpp_max(float v) {
    // every source lane of these patterns exists, so bound_ctrl never applies. IEEE maximum: a DPP move
    // plus one v_maximum3_f32; fmaxf folded the DPP into v_max but quieted both operands first (four
    // instructions per level on MFMA outputs)
    return __builtin_elementwise_maximum(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true)));
}
__device__ __forceinline__ float row16_max(float v) {
    v = dpp_max<0xB1>(v);
    v = dpp_max<0x4E>(v);
    v = dpp_max<0x141>(v);
    return dpp_max<0x140>(v);
}
__device__ __forceinline__ f32x4 row16_max4(f32x4 v) {
    return f32x4{row16_max(v.x), row16_max(v.y), row16_max(v.z), row16_max(v.w)};
}
// The same four maxima scattered over the row: lane n (n = lane & 15) ends with the max of component
// (n >> 2) & 3, every lane of its quad alike -- 16 instructions instead of row16_max4's 32. Lanes n and
// n ^ 8 first trade halves (x, y stay below 8, z, w above), then each half-row trades with its mirror
// lane 7 - n (the other quad of the half), which leaves one component per quad, reduced over the quad
// by two more DPP levels. Maxima are exact, so the result equals row16_max4's bit for bit.
__device__ __forceinline__ float row16_max_scatter4(f32x4 v, int n) {
    const bool h8 = (n & 8) != 0, h4 = (n & 4) != 0;
    float a0 = h8 ? v.z : v.x, a1 = h8 ? v.w : v.y;
    const float s0 = h8 ? v.x : v.z, s1 = h8 ? v.y : v.w;
    a0 = __builtin_elementwise_maximum(a0, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s0), 0x128, 0xF, 0xF, true)));
    a1 = __builtin_elementwise_maximum(a1, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s1), 0x128, 0xF, 0xF, true)));
    float r = h4 ? a1 : a0;
    const float s = h4 ? a0 : a1;
    r = __builtin_elementwise_maximum(r, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s), 0x141, 0xF, 0xF, true)));
    r = dpp_max<0xB1>(r);
    return dpp_max<0x4E>(r);
}
// value of lane 4*(l/4) (first lane of the quad)
__device__ __forceinline__ float quad_bcast0(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x00, 0xF, 0xF, false));
}

// --------------------------------------------------------------- Philox4x32-10 + Box-Muller
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.z;
        ctr = u32x4{(uint32_t)(p1 >> 32) ^ ctr.y ^ k0, (uint32_t)p1,
                    (uint32_t)(p0 >> 32) ^ ctr.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return ctr;
}

__device__ __forceinline__ float u01(uint32_t v) {  // (0,1]
    return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// 4 standard normals for (seed, stream, row, block): Box-Muller on the hardware transcendentals
// (v_log_f32 = log2, v_sin/v_cos_f32 take revolutions, so sin(2*pi*u) needs no range reduction).
__device__ __forceinline__ f32x4 philox_normal4(uint64_t seed, uint32_t stream, uint32_t row,
                                                uint32_t blk) {
    u32x4 r = philox4x32_10(u32x4{row, blk, stream, 0x5EEDu}, (uint32_t)seed, (uint32_t)(seed >> 32));
    constexpr float kM2Ln2 = -1.3862943611198906f;   // -2 ln 2
    const float r0 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.x)));
    const float r1 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.z)));
    const float a0 = u01(r.y), a1 = u01(r.w);
    return f32x4{r0 * __builtin_amdgcn_cosf(a0), r0 * __builtin_amdgcn_sinf(a0), r1 * __builtin_amdgcn_cosf(a1),
                 r1 * __builtin_amdgcn_sinf(a1)};
}
