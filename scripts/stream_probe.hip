// The f16x3 head-layer-1 stream of pc_step_kernel<4, 8, 3> on its own (tuning aid, not a test): one
// workgroup of 8 waves per CU runs stream_x3_step (gp_head.h) over the 3 heads' weight planes with the
// 64-candidate B planes in LDS, exactly as the trunk does, but with no epilogue, barrier or other phase
// between the heads. Prints cycles per MFMA per SIMD (s_memtime), per wave and for the last wave.
// Variants: MODE 0 the trunk's order (every wave: head 0, 1, 2 for its tile pair), MODE 1 a workgroup
// barrier after each head.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I genpose2_amd/csrc -I include -o scripts/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gp_head.h"

#ifndef SP_NT
#define SP_NT 4
#endif
constexpr int NT = SP_NT, WV = 8, TPW = 2, DH = X3_DH;

template <int MODE>
__global__ __launch_bounds__(512) void stream_probe(const void* __restrict__ wplanes, const f16x8* __restrict__ bsrc,
                                                    f32x4* __restrict__ out, unsigned long long* cyc) {
    __shared__ f16x8 act[KC_HID * NT * X3P * 64];   // 96 KiB: [chunk][ct][plane][lane]
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < KC_HID * NT * X3P * 64; i += 512) act[i] = bsrc[i];
    const __amdgpu_buffer_rsrc_t WH = make_rsrc(wplanes, 3 * HID * HID * 2 * X3P);
    const int voff = lane * 16;
    f16x8 ringh[DH + 1][TPW][X3P];
    f32x4 acc[TPW][NT], cor[TPW][NT], keep = f32x4{0.f, 0.f, 0.f, 0.f};
    int TH[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) TH[t] = wid * TPW + t;
    stream_x3_step<0, DH, TPW, NT, DH>(WH, TH, act, lane, voff, ringh, acc, cor);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int h = 0; h < 3; ++h) {
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) acc[t][ct] = cor[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TPW; ++t) TH[t] = h * 16 + wid * TPW + t;
        stream_x3_step<DH, KC_HID + DH, TPW, NT, DH>(WH, TH, act, lane, voff, ringh, acc, cor);
        if (h < 2) {
            int TN[TPW];
#pragma unroll
            for (int t = 0; t < TPW; ++t) TN[t] = TH[t] + 16;
            stream_x3_step<0, DH, TPW, NT, DH>(WH, TN, act, lane, voff, ringh, acc, cor);
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) keep += acc[t][ct] + cor[t][ct];
        if constexpr (MODE == 1) __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = keep;
    if (lane == 0) cyc[blockIdx.x * WV + wid] = t1 - t0;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int MODE>
static int run(const void* w, const f16x8* b, f32x4* out, unsigned long long* cyc, int wgs) {
    hipLaunchKernelGGL(stream_probe<MODE>, dim3(wgs), dim3(512), 0, 0, w, b, out, cyc);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(stream_probe<MODE>, dim3(wgs), dim3(512), 0, 0, w, b, out, cyc);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)wgs * WV);
    CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
    double mean_w[WV] = {0}, last = 0;
    for (int g = 0; g < wgs; ++g) {
        unsigned long long mx = 0;
        for (int w8 = 0; w8 < WV; ++w8) {
            mean_w[w8] += (double)h[(size_t)g * WV + w8] / wgs;
            mx = h[(size_t)g * WV + w8] > mx ? h[(size_t)g * WV + w8] : mx;
        }
        last += (double)mx / wgs;
    }
    // 3 heads x 8 chunks x 48 MFMAs per wave, two waves per SIMD
    printf("{\"mode\": %d, \"wgs\": %d, \"last_wave_cycles\": %.0f, \"cycles_per_mfma_per_simd\": %.2f, \"per_wave\": [", MODE, wgs,
           last, last / (2.0 * 3 * 8 * 48));
    for (int w8 = 0; w8 < WV; ++w8) printf("%s%.0f", w8 ? ", " : "", mean_w[w8]);
    printf("]}\n");
    return 0;
}

int main(int argc, char** argv) {
    const int wgs = argc > 1 ? atoi(argv[1]) : 200;
    const size_t wbytes = (size_t)3 * HID * HID * 2 * X3P;
    std::vector<unsigned short> hw(wbytes / 2), hb((size_t)KC_HID * NT * X3P * 64 * 8);
    unsigned x = 7u;
    auto rnd = [&]() {
        x = x * 1664525u + 1013904223u;
        const unsigned r = x >> 8;
        return (unsigned short)(((r & 1) << 15) | ((11 + (r >> 1) % 6) << 10) | ((r >> 4) & 0x3ff));
    };
    for (auto& v : hw) v = rnd();
    for (auto& v : hb) v = rnd();
    void* w;
    f16x8* b;
    f32x4* out;
    unsigned long long* cyc;
    CK(hipMalloc(&w, wbytes));
    CK(hipMalloc(&b, hb.size() * 2));
    CK(hipMalloc(&out, (size_t)wgs * 512 * sizeof(f32x4)));
    CK(hipMalloc(&cyc, (size_t)wgs * WV * 8));
    CK(hipMemcpy(w, hw.data(), wbytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    if (run<0>(w, b, out, cyc, wgs) || run<1>(w, b, out, cyc, wgs)) return 1;
    return 0;
}
