// How v_mfma_f32_16x16x32_f16 and v_mfma_f32_16x16x4_f32 round: dumps random operand fragments, the
// accumulator input and the MFMA output of many trials to a binary file; scripts/mfma_round_check.py
// compares each output with the correctly rounded fp32 value of C + sum(a*b) computed exactly.
// Build: hipcc -O2 --offload-arch=gfx950 -o scripts/mfma_round_probe scripts/mfma_round_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// one trial per wave: A, B fragments (per lane), C (per lane, 4 values), D out
__global__ void probe_h(const f16x8* a, const f16x8* b, const f32x4* c, f32x4* d) {
    const int l = threadIdx.x & 63, w = blockIdx.x;
    d[w * 64 + l] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[w * 64 + l], b[w * 64 + l], c[w * 64 + l], 0, 0, 0);
}
__global__ void probe_f(const float* a, const float* b, const f32x4* c, f32x4* d) {
    const int l = threadIdx.x & 63, w = blockIdx.x;
    d[w * 64 + l] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[w * 64 + l], b[w * 64 + l], c[w * 64 + l], 0, 0, 0);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 256;   // trials
    const char* out = argc > 2 ? argv[2] : "mfma_probe.bin";
    std::mt19937_64 rng(1234);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::uniform_int_distribution<int> ue(-6, 6);
    std::vector<_Float16> ha((size_t)n * 64 * 8), hb((size_t)n * 64 * 8);
    std::vector<float> fa((size_t)n * 64), fb((size_t)n * 64), hc((size_t)n * 64 * 4), fc((size_t)n * 64 * 4);
    for (auto& v : ha) v = (_Float16)ldexpf(nd(rng), ue(rng));
    for (auto& v : hb) v = (_Float16)ldexpf(nd(rng), ue(rng));
    for (auto& v : fa) v = ldexpf(nd(rng), ue(rng));
    for (auto& v : fb) v = ldexpf(nd(rng), ue(rng));
    // accumulators: zero for a quarter of the trials, random magnitudes otherwise
    for (size_t i = 0; i < hc.size(); ++i) {
        const int trial = (int)(i / 256);
        hc[i] = (trial % 4 == 0) ? 0.f : ldexpf(nd(rng), ue(rng) + 3);
        fc[i] = (trial % 4 == 0) ? 0.f : ldexpf(nd(rng), ue(rng) + 3);
    }
    void *da, *db, *dc, *dd, *ga, *gb, *gc, *gd;
    CK(hipMalloc(&da, ha.size() * 2)); CK(hipMalloc(&db, hb.size() * 2));
    CK(hipMalloc(&dc, hc.size() * 4)); CK(hipMalloc(&dd, hc.size() * 4));
    CK(hipMalloc(&ga, fa.size() * 4)); CK(hipMalloc(&gb, fb.size() * 4));
    CK(hipMalloc(&gc, fc.size() * 4)); CK(hipMalloc(&gd, fc.size() * 4));
    CK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ga, fa.data(), fa.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(gb, fb.data(), fb.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(gc, fc.data(), fc.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe_h, dim3(n), dim3(64), 0, 0, (const f16x8*)da, (const f16x8*)db, (const f32x4*)dc, (f32x4*)dd);
    hipLaunchKernelGGL(probe_f, dim3(n), dim3(64), 0, 0, (const float*)ga, (const float*)gb, (const f32x4*)gc, (f32x4*)gd);
    CK(hipDeviceSynchronize());
    std::vector<float> hd(hc.size()), fd(fc.size());
    CK(hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(fd.data(), gd, fd.size() * 4, hipMemcpyDeviceToHost));
    FILE* f = fopen(out, "wb");
    if (!f) return 1;
    fwrite(&n, 4, 1, f);
    fwrite(ha.data(), 2, ha.size(), f); fwrite(hb.data(), 2, hb.size(), f);
    fwrite(hc.data(), 4, hc.size(), f); fwrite(hd.data(), 4, hd.size(), f);
    fwrite(fa.data(), 4, fa.size(), f); fwrite(fb.data(), 4, fb.size(), f);
    fwrite(fc.data(), 4, fc.size(), f); fwrite(fd.data(), 4, fd.size(), f);
    fclose(f);
    printf("wrote %d trials to %s\n", n, out);
    return 0;
}
