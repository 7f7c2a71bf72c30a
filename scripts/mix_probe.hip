// Microbenchmark (tuning aid, not product): can f32 VALU FMAs run beside v_mfma_f32_16x16x4_f32 on
// one SIMD? 512-thread workgroups (2 waves per SIMD), one per CU, 256 workgroups.
//   mfma      : waves 0-3 run MFMA chains (8 independent accumulators), waves 4-7 idle
//   valu      : waves 4-7 run v_fmac_f32_dpp row_newbcast chains (the VALU GEMM form), waves 0-3 idle
//   split     : both at once (two waves per SIMD)
//   fill<NF>  : waves 0-3 only, NF VALU fillers after every MFMA in the same instruction stream
// Build: hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o scripts/mix_probe scripts/mix_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int C>
__device__ __forceinline__ void fmac_bcast(float& acc, float x, float w) {
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(x), "v"(w), "n"(C));
}
__device__ __forceinline__ void fmac_plain(float& acc, float x, float w) {
    asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc) : "v"(x), "v"(w));
}

template <int F, int NF, bool DPP>
__device__ __forceinline__ void fillers(float (&v)[16], float x, float w) {
    if constexpr (F < NF) {
        if constexpr (DPP)
            fmac_bcast<F & 15>(v[F & 15], x, w);
        else
            fmac_plain(v[F & 15], x, w);
        fillers<F + 1, NF, DPP>(v, x, w);
    }
}

template <int J, int NF, bool DPP>
__device__ __forceinline__ void body(f32x4 (&acc)[8], float (&v)[16], float a, float b) {
    if constexpr (J < 8) {
        acc[J] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[J], 0, 0, 0);
        // fillers for this gap rotate through the 16 accumulators: v[(J*NF + f) % 16]
        fillers<0, NF, DPP>(*reinterpret_cast<float(*)[16]>(&v[0]), J & 1 ? b : a, J & 1 ? a : b);
        body<J + 1, NF, DPP>(acc, v, a, b);
    }
}

// MODE 0 mfma only, 1 valu only, 2 split (two waves per SIMD), 3 fillers in the MFMA stream
template <int MODE, int NF, bool DPP>
__global__ __launch_bounds__(512) void mix(float* out, long long* cyc, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float a = 1.0f + lane * 1e-3f, b = 0.5f - lane * 1e-3f;
    float sink = 0.f;
    __builtin_amdgcn_s_barrier();
    const long long t0 = __builtin_amdgcn_s_memtime();
    const bool mfma_wave = w < 4 && (MODE == 0 || MODE == 2 || MODE == 3);
    const bool valu_wave = w >= 4 && (MODE == 1 || MODE == 2);
    if (mfma_wave) {
        f32x4 acc[8];
        float v[16];
        for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < 16; ++c) v[c] = 0.f;
        for (int i = 0; i < n; ++i) body<0, MODE == 3 ? NF : 0, DPP>(acc, v, a, b);
        for (int j = 0; j < 8; ++j) sink += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
        for (int c = 0; c < 16; ++c) sink += v[c];
    } else if (valu_wave) {
        float v[16];
        for (int c = 0; c < 16; ++c) v[c] = 0.f;
        for (int i = 0; i < n; ++i) {   // 32 FMAs per iteration (one MFMA's worth of issue time is 8 MFMAs)
            fillers<0, 16, DPP>(v, a, b);
            fillers<0, 16, DPP>(v, b, a);
        }
        for (int c = 0; c < 16; ++c) sink += v[c];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
    out[blockIdx.x * 512 + threadIdx.x] = sink;
}

template <int MODE, int NF, bool DPP>
void run(const char* name, float* out, long long* cyc, int n) {
    const int nwg = 256;
    std::vector<long long> h(nwg * 8);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((mix<MODE, NF, DPP>), dim3(nwg), dim3(512), 0, 0, out, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double m = 0, v = 0;
    for (int g = 0; g < nwg; ++g) {
        for (int w = 0; w < 4; ++w) m += h[g * 8 + w];
        for (int w = 4; w < 8; ++w) v += h[g * 8 + w];
    }
    m /= nwg * 4;
    v /= nwg * 4;
    printf("%-16s waves0-3 %8.0f cyc = %6.1f per 8-MFMA iter (%5.1f / MFMA)   waves4-7 %8.0f cyc (%5.2f / FMA)\n",
           name, m, m / n, m / n / 8, v, v / (n * 32.0));
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8);
    const int n = 256;
    run<0, 0, true>("mfma only", out, cyc, n);
    run<1, 0, true>("valu dpp only", out, cyc, n);
    run<1, 0, false>("valu plain only", out, cyc, n);
    run<2, 0, true>("split dpp", out, cyc, n);
    run<2, 0, false>("split plain", out, cyc, n);
    run<3, 2, true>("fill 2 dpp", out, cyc, n);
    run<3, 4, true>("fill 4 dpp", out, cyc, n);
    run<3, 6, true>("fill 6 dpp", out, cyc, n);
    run<3, 8, true>("fill 8 dpp", out, cyc, n);
    run<3, 4, false>("fill 4 plain", out, cyc, n);
    run<3, 6, false>("fill 6 plain", out, cyc, n);
    return 0;
}
