// Microbenchmark (tuning aid, not product): can f32 VALU work run beside v_mfma_f32_16x16x32_f16 on one SIMD?
// The PC step's serial phases (update, pose_encoder.0, epilogues) are f32 VALU; if another wave's f16 MFMA
// stream on the same SIMD keeps issuing under them, two phase-shifted candidate groups per workgroup can hide
// them. 512-thread workgroups (2 waves per SIMD), one per CU, 256 workgroups.
//   mfma        : waves 0-3 run f16 MFMA chains (8 independent accumulators), waves 4-7 idle
//   valu        : waves 4-7 run f32 FMA chains (plain / packed), waves 0-3 idle
//   split       : both at once (one MFMA wave and one VALU wave per SIMD)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mix16_probe scripts/mix16_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// MODE 3: waves 0-3 only, NF independent f32 FMAs after every MFMA in the same instruction stream (can one wave
// fill its own MFMA shadow with VALU work?)
template <int NF>
__global__ __launch_bounds__(512) void fill(float* out, long long* cyc, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f16x8 a, b;
    for (int k = 0; k < 8; ++k) {
        a[k] = (_Float16)(1.0f + lane * 1e-3f + k * 1e-2f);
        b[k] = (_Float16)(0.5f - lane * 1e-3f + k * 1e-2f);
    }
    float sink = 0.f;
    __builtin_amdgcn_s_barrier();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (w < 4) {
        f32x4 acc[8];
        float v[16];
        for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < 16; ++c) v[c] = lane * 1e-3f + c;
        const float x = 1.0f + lane * 1e-6f, y = 0.999f;
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
#pragma unroll
                for (int f = 0; f < NF; ++f) v[(j * NF + f) & 15] = __builtin_fmaf(v[(j * NF + f) & 15], x, y);
            }
        }
        for (int j = 0; j < 8; ++j) sink += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
        for (int c = 0; c < 16; ++c) sink += v[c];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
    out[blockIdx.x * 512 + threadIdx.x] = sink;
}

template <int NF>
void run_fill(const char* name, float* out, long long* cyc, int n) {
    const int nwg = 256;
    std::vector<long long> h(nwg * 8);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((fill<NF>), dim3(nwg), dim3(512), 0, 0, out, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 4; ++w) m += h[g * 8 + w];
    m /= nwg * 4;
    printf("%-22s mfma waves %9.0f cyc (%5.2f / MFMA with %d f32 FMAs each)\n", name, m, m / (n * 8.0), NF);
}

template <int MODE, bool PK>
__global__ __launch_bounds__(512) void mix(float* out, long long* cyc, int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f16x8 a, b;
    for (int k = 0; k < 8; ++k) {
        a[k] = (_Float16)(1.0f + lane * 1e-3f + k * 1e-2f);
        b[k] = (_Float16)(0.5f - lane * 1e-3f + k * 1e-2f);
    }
    float sink = 0.f;
    __builtin_amdgcn_s_barrier();
    const long long t0 = __builtin_amdgcn_s_memtime();
    const bool mfma_wave = w < 4 && (MODE == 0 || MODE == 2);
    const bool valu_wave = w >= 4 && (MODE == 1 || MODE == 2);
    if (mfma_wave) {
        f32x4 acc[8];
        for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
        }
        for (int j = 0; j < 8; ++j) sink += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
    } else if (valu_wave) {
        // 16 independent chains; 64 FMAs per iteration (plain) or 32 packed FMAs (64 lanes x 2)
        float x = 1.0f + lane * 1e-6f, y = 0.999f;
        if constexpr (PK) {
            f32x2 v[16];
            for (int c = 0; c < 16; ++c) v[c] = f32x2{0.f, 1.f};
            const f32x2 xx = {x, y}, yy = {y, x};
            for (int i = 0; i < n; ++i) {
#pragma unroll
                for (int c = 0; c < 16; ++c) v[c] = __builtin_elementwise_fma(v[c], xx, yy);
#pragma unroll
                for (int c = 0; c < 16; ++c) v[c] = __builtin_elementwise_fma(v[c], yy, xx);
                asm volatile("" : "+v"(v[0]), "+v"(v[5]), "+v"(v[10]), "+v"(v[15]));
            }
            for (int c = 0; c < 16; ++c) sink += v[c].x + v[c].y;
        } else {
            float v[16];
            for (int c = 0; c < 16; ++c) v[c] = 0.f;
            for (int i = 0; i < n; ++i) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 16; ++c) v[c] = __builtin_fmaf(v[c], r & 1 ? x : y, r & 1 ? y : x);
                asm volatile("" : "+v"(v[0]), "+v"(v[5]), "+v"(v[10]), "+v"(v[15]));
            }
            for (int c = 0; c < 16; ++c) sink += v[c];
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
    out[blockIdx.x * 512 + threadIdx.x] = sink;
}

template <int MODE, bool PK>
void run(const char* name, float* out, long long* cyc, int nm, int nv) {
    const int nwg = 256;
    std::vector<long long> h(nwg * 8);
    const int n = MODE == 1 ? nv : nm;
    for (int rep = 0; rep < 2; ++rep) {
        if (MODE == 2) {
            // the MFMA waves run nm iterations, the VALU waves nv: pass nm, VALU waves scale by nv / nm
            hipLaunchKernelGGL((mix<MODE, PK>), dim3(nwg), dim3(512), 0, 0, out, cyc, nm);
        } else {
            hipLaunchKernelGGL((mix<MODE, PK>), dim3(nwg), dim3(512), 0, 0, out, cyc, n);
        }
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
    const double fma_per_iter = 64.0;   // plain: 64 v_fma_f32; packed: 32 v_pk_fma_f32 (64 lane-pairs of work)
    printf("%-22s mfma waves %9.0f cyc (%5.2f / MFMA)   valu waves %9.0f cyc (%5.2f / instr)\n", name, m,
           MODE == 1 ? 0.0 : m / (n * 8.0), v, MODE == 0 ? 0.0 : v / (n * (PK ? 32.0 : fma_per_iter)));
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8);
    const int n = 512;
    run<0, false>("f16 mfma only", out, cyc, n, n);
    run<1, false>("f32 fma only", out, cyc, n, n);
    run<1, true>("pk_fma only", out, cyc, n, n);
    run<2, false>("split f32 fma", out, cyc, n, n);
    run<2, true>("split pk_fma", out, cyc, n, n);
    run_fill<0>("fill 0", out, cyc, n);
    run_fill<2>("fill 2", out, cyc, n);
    run_fill<4>("fill 4", out, cyc, n);
    run_fill<8>("fill 8", out, cyc, n);
    run_fill<12>("fill 12", out, cyc, n);
    return 0;
}
