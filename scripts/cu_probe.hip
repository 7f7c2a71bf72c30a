// Placement probe for CU-masked streams (hipExtStreamCreateWithCUMask): every workgroup spins for a
// bounded number of cycles (so that the grid spreads over every CU its queue may use) and records the
// XCC and HW_ID it ran on. Diagnostic only: scripts/cu_mask_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void cu_probe_kernel(uint32_t* out, long long spin) {
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    if (threadIdx.x == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

extern "C" int cu_probe(uint32_t* out, int blocks, long long spin, hipStream_t st) {
    hipLaunchKernelGGL(cu_probe_kernel, dim3(blocks), dim3(64), 0, st, out, spin);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
