// Diagnostic only (scripts/race_probe.py --mode poison): leaves pseudo-random junk in every CU's LDS and in the
// VGPRs of every SIMD, so a later kernel that reads LDS or registers it never wrote sees values that differ from
// call to call instead of whatever the previous identical kernel happened to leave there.
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/libpoison.so scripts/poison.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// LDS: every dword of the workgroup's allocation; VGPRs: 192 live random values per lane, folded into one
// store so none is dead (the allocation they occupy is what the next wave on that SIMD inherits).
__global__ __launch_bounds__(256) void poison_kernel(uint32_t seed, uint32_t lds_dwords, float* sink) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    for (uint32_t i = threadIdx.x; i < lds_dwords; i += 256) lds[i] = mix(seed ^ (i * 2654435761u) ^ (blockIdx.x << 20));
    float r[192];
#pragma unroll
    for (int k = 0; k < 192; ++k) r[k] = (float)(mix(seed + t * 193u + k) >> 8) * 1e-3f - 8000.f;
    // two rounds of opaque touches: every value is live from its first touch to its second, so all 192 occupy
    // registers at once
#pragma unroll
    for (int k = 0; k < 192; k += 8)
        asm volatile("" : "+v"(r[k]), "+v"(r[k + 1]), "+v"(r[k + 2]), "+v"(r[k + 3]), "+v"(r[k + 4]), "+v"(r[k + 5]),
                          "+v"(r[k + 6]), "+v"(r[k + 7]));
#pragma unroll
    for (int k = 184; k >= 0; k -= 8)
        asm volatile("" : "+v"(r[k]), "+v"(r[k + 1]), "+v"(r[k + 2]), "+v"(r[k + 3]), "+v"(r[k + 4]), "+v"(r[k + 5]),
                          "+v"(r[k + 6]), "+v"(r[k + 7]));
    __syncthreads();
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 192; ++k) acc = acc * 0.999f + r[k] * __uint_as_float(lds[(k * 37 + threadIdx.x) % lds_dwords] | 0x3f800000u);
    if (acc == 1.2345f) sink[t] = acc;
}

// every CU's whole LDS (one 160 KiB workgroup per CU at a time), then the register files (small LDS, as many
// workgroups as the registers allow)
extern "C" int poison_gpu(uint32_t seed, int blocks, hipStream_t st) {
    const uint32_t lds_bytes = 160 * 1024;
    hipLaunchKernelGGL(poison_kernel, dim3(blocks), dim3(256), lds_bytes, st, seed, lds_bytes / 4, nullptr);
    hipLaunchKernelGGL(poison_kernel, dim3(blocks * 4), dim3(256), 4096, st, seed ^ 0x9e3779b9u, 1024u, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
