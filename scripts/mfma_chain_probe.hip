// Issue rate of v_mfma_f32_16x16x32_f16 by accumulator dependence pattern (tuning aid, not a test).
// One workgroup of W waves (W/4 per SIMD) per CU runs N iterations of 48 MFMAs with every operand in
// registers; cycles per MFMA per SIMD from s_memtime around the loop.
//   pattern 0: 16 accumulators, each MFMA on the next one (dependent distance 16)
//   pattern 1: the f16x3 stream's order per column tile: two tiles' 5-deep correction chains interleaved,
//              then their main products (dependent distance 2), four column tiles in turn
//   pattern 2: one accumulator (dependent distance 1)
//   pattern 3: as 1 but two column tiles at once (dependent distance 4)
//   pattern 4: as 1 but four column tiles at once (dependent distance 8)
//   pattern 5: per column tile, tile 0's five correction products back to back, then tile 1's, then the
//              two main products
//   pattern 6: per column tile and tile: the five correction products back to back, then the main one
//   pattern 7: as 5 over two chunks at once (ten correction products per chain, two main per chain)
//   pattern 10: as 1 with the B operands of the next column tile made by 12 VALU ops (v_xor) per 12 MFMAs
//   pattern 11: as 1 with the B operands of the next column tile read from LDS (3 ds_read_b128 per
//              12 MFMAs, one column tile ahead, as the kernel's X3_BPIPE)
//   pattern 8 / 9: v_mfma_f32_16x16x4_f32, 8 per 32-deep chunk: two tiles alternating / each tile's 8
//              back to back (the exact-fp32 trunk)
// Usage: mfma_chain_probe [ITERS [FILL [WGS]]] (FILL: operand bits, see main; WGS workgroups, 64 default).
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_chain_probe scripts/mfma_chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// issue order pinned: no MFMA moves across another
__device__ __forceinline__ f32x4 mf(f16x8 a, f16x8 b, f32x4 c) {
    const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    return d;
}

__device__ __forceinline__ f32x4 mff(float a, float b, f32x4 c) {
    const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    return d;
}

template <int P, int UNR = 1>
__global__ __launch_bounds__(512) void probe(const f16x8* __restrict__ in, f32x4* __restrict__ out, unsigned long long* cyc, int n) {
    const int l = threadIdx.x & 63;
    f16x8 w[2][3], b[4][3];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) w[t][p] = in[(t * 3 + p) * 64 + l];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int p = 0; p < 3; ++p) b[c][p] = in[(6 + c * 3 + p) * 64 + l];
    f32x4 acc[2][4], cor[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[t][c] = cor[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    __shared__ f16x8 sb[12 * 64];   // pattern 11: four column tiles' B planes
    if (threadIdx.x < 64)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) sb[(c * 3 + p) * 64 + l] = b[c][p];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    // UNR > 1: the iteration loop unrolled UNR times (straight-line code of 48 UNR MFMAs: instruction-cache
    // footprint)
    for (int it = 0; it < n; it += UNR)
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
        if constexpr (P == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        cor[t][c] = mf(w[t][k], b[c][2 - k], cor[t][c]);
                        acc[t][c] = mf(w[t][(k + 1) % 3], b[c][k], acc[t][c]);
                    }
        } else if constexpr (P == 1 || P == 3 || P == 4) {
            constexpr int G = P == 1 ? 1 : (P == 3 ? 2 : 4);
#pragma unroll
            for (int c0 = 0; c0 < 4; c0 += G) {
#pragma unroll
                for (int s = 0; s < 5; ++s)
#pragma unroll
                    for (int c = c0; c < c0 + G; ++c)
#pragma unroll
                        for (int t = 0; t < 2; ++t) cor[t][c] = mf(w[t][(s + 2) % 3], b[c][s % 3], cor[t][c]);
#pragma unroll
                for (int c = c0; c < c0 + G; ++c)
#pragma unroll
                    for (int t = 0; t < 2; ++t) acc[t][c] = mf(w[t][0], b[c][0], acc[t][c]);
            }
        } else if constexpr (P == 5) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 5; ++s) cor[t][c] = mf(w[t][(s + 2) % 3], b[c][s % 3], cor[t][c]);
#pragma unroll
                for (int t = 0; t < 2; ++t) acc[t][c] = mf(w[t][0], b[c][0], acc[t][c]);
            }
        } else if constexpr (P == 6) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
#pragma unroll
                    for (int s = 0; s < 5; ++s) cor[t][c] = mf(w[t][(s + 2) % 3], b[c][s % 3], cor[t][c]);
                    acc[t][c] = mf(w[t][0], b[c][0], acc[t][c]);
                }
        } else if constexpr (P == 7) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 10; ++s) cor[t][c] = mf(w[t][(s + 2) % 3], b[2 * c + s / 5][s % 3], cor[t][c]);
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) acc[t][c] = mf(w[t][0], b[2 * c + s][0], acc[t][c]);
            }
        } else if constexpr (P == 10 || P == 11) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                f16x8 bn[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    using u4 = __attribute__((ext_vector_type(4))) unsigned;
                    if constexpr (P == 10)
                        bn[p] = __builtin_bit_cast(f16x8, __builtin_bit_cast(u4, b[c][p]) ^ (unsigned)(it + c + 1));
                    else
                        bn[p] = sb[(((c + 1) & 3) * 3 + p) * 64 + l];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int s = 0; s < 5; ++s)
#pragma unroll
                    for (int t = 0; t < 2; ++t) cor[t][c] = mf(w[t][(s + 2) % 3], b[c][s % 3], cor[t][c]);
#pragma unroll
                for (int t = 0; t < 2; ++t) acc[t][c] = mf(w[t][0], b[c][0], acc[t][c]);
#pragma unroll
                for (int p = 0; p < 3; ++p) b[(c + 1) & 3][p] = bn[p];
            }
        } else if constexpr (P == 8 || P == 9) {
            // 48 f32 MFMAs: 3 "chunks" of 8 k-steps x 2 tiles
            const float a0 = (float)w[0][0][0], a1 = (float)w[1][0][0], bb = (float)b[0][0][1];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if constexpr (P == 8) {
#pragma unroll
                    for (int k = 0; k < 8; ++k)
#pragma unroll
                        for (int t = 0; t < 2; ++t) acc[t][c] = mff(t ? a1 : a0, bb, acc[t][c]);
                } else {
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int k = 0; k < 8; ++k) acc[t][c] = mff(t ? a1 : a0, bb, acc[t][c]);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 48; ++k) acc[0][0] = mf(w[k & 1][k % 3], b[k & 3][(k >> 2) % 3], acc[0][0]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) s += acc[t][c] + cor[t][c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (l == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

static int g_fill = 0, g_wgs = 64;   // workgroups: one per CU up to 256
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int P, int UNR = 1>
static int run(const f16x8* in, f32x4* out, unsigned long long* cyc, int waves, int n) {
    hipLaunchKernelGGL((probe<P, UNR>), dim3(g_wgs), dim3(64 * waves), 0, 0, in, out, cyc, n);
    CK(hipDeviceSynchronize());
    static unsigned long long h[1024 * 8];
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * g_wgs * waves, hipMemcpyDeviceToHost));
    // the SIMD's time is its LAST wave's (the older wave of a pair wins issue and finishes first, so a
    // mean over waves would overstate the pair's rate)
    double m = 0;
    for (int g = 0; g < g_wgs; ++g) {
        unsigned long long mx = 0;
        for (int i = 0; i < waves; ++i) mx = h[g * waves + i] > mx ? h[g * waves + i] : mx;
        m += (double)mx;
    }
    m /= g_wgs;
    // cycles per MFMA per SIMD: each wave issued 48 n MFMAs; waves / 4 waves share a SIMD
    printf("{\"pattern\": %d, \"unroll\": %d, \"fill\": %d, \"wgs\": %d, \"waves_per_simd\": %d, \"cycles_per_mfma_per_simd\": %.2f}\n", P, UNR, g_fill, g_wgs,
           waves / 4, m / (48.0 * n) / (waves / 4));
    return 0;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    f16x8* in;
    f32x4* out;
    unsigned long long* cyc;
    // operand bits: 0 every f16 0x3131, 1 random normals, 2 random f16 subnormals, 3 a third of the
    // registers (the lo planes) subnormal
    const int fill = argc > 2 ? atoi(argv[2]) : 0;
    g_fill = fill;
    g_wgs = argc > 3 ? atoi(argv[3]) : 64;
    CK(hipMalloc(&in, 18 * 64 * sizeof(f16x8)));
    {
        static unsigned short h[18 * 64 * 8];
        unsigned x = 12345u;
        for (int i = 0; i < 18 * 64 * 8; ++i) {
            x = x * 1664525u + 1013904223u;
            const unsigned r = x >> 8;
            const unsigned short nrm = (unsigned short)(((r & 1) << 15) | ((13 + (r >> 1) % 4) << 10) | ((r >> 3) & 0x3ff));
            const unsigned short sub = (unsigned short)(((r & 1) << 15) | (1 + (r >> 3) % 1023));
            const int reg = i / (64 * 8);   // operand register index: w[t][p] = 0..5, b[c][p] = 6..17
            h[i] = fill == 0 ? 0x3131 : fill == 1 ? nrm : fill == 2 ? sub : (reg % 3 == 2 ? sub : nrm);
        }
        CK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&out, 1024 * 512 * sizeof(f32x4)));
    CK(hipMalloc(&cyc, 1024 * 8 * sizeof(unsigned long long)));
    for (int waves = 4; waves <= 8; waves += 4) {
        if (run<0>(in, out, cyc, waves, n) || run<1>(in, out, cyc, waves, n) || run<2>(in, out, cyc, waves, n) ||
            run<3>(in, out, cyc, waves, n) || run<4>(in, out, cyc, waves, n) || run<5>(in, out, cyc, waves, n) ||
            run<6>(in, out, cyc, waves, n) || run<7>(in, out, cyc, waves, n) || run<8>(in, out, cyc, waves, n) ||
            run<9>(in, out, cyc, waves, n) || run<1, 16>(in, out, cyc, waves, n) || run<1, 64>(in, out, cyc, waves, n) ||
            run<1, 128>(in, out, cyc, waves, n) || run<10>(in, out, cyc, waves, n) || run<11>(in, out, cyc, waves, n))
            return 1;
    }
    return 0;
}
