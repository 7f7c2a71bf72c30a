// Diagnostic only (scripts/pk_probe.py): the level-0 projection's arithmetic in isolation, to find which
// instruction pattern returns a wrong value now and then when other processes' kernels share the GPU.
//   proj_x3   : coordinates read as one 12-byte load (global_load_dwordx3), the fma chains left to the compiler
//               (it packs them into v_pk_fma_f32 with op_sel broadcasts of x / y / z) -- the shipped kernel's shape
//   proj_x1   : the same arithmetic, each coordinate read by its own 4-byte load
// Built twice: libpkprobe.so (default target features) and libpkprobe_nopk.so (-packed-fp32-ops: the same
// source without packed-FP32 instructions).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool X3>
__global__ __launch_bounds__(256) void proj_kernel(const float* __restrict__ xyz, const float* __restrict__ w,
                                                   const float* __restrict__ b, int npts, float* __restrict__ out) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (size_t)npts * 8) return;
    const int p = (int)(t / 8), g = (int)(t - (size_t)p * 8);
    float x, y, z;
    if constexpr (X3) {
        x = xyz[(size_t)p * 3 + 0];
        y = xyz[(size_t)p * 3 + 1];
        z = xyz[(size_t)p * 3 + 2];
    } else {
        x = __hip_atomic_load(xyz + (size_t)p * 3 + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        y = __hip_atomic_load(xyz + (size_t)p * 3 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        z = __hip_atomic_load(xyz + (size_t)p * 3 + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ch = 4 * g + j;
        const f32x4 ww = *reinterpret_cast<const f32x4*>(w + ch * 4);
        float acc = __builtin_fmaf(ww.x, x, 0.f);
        acc = __builtin_fmaf(ww.y, y, acc);
        acc = __builtin_fmaf(ww.z, z, acc);
        v[j] = acc + b[ch];
    }
    *reinterpret_cast<f32x4*>(out + (size_t)p * 32 + 4 * g) = f32x4{v[0], v[1], v[2], v[3]};
}

// MFMA- and LDS-heavy load for other processes: keeps every SIMD's matrix pipe and the LDS busy
__global__ __launch_bounds__(256) void load_kernel(float* sink, int iters) {
    __shared__ float lds[8192];
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    h8 a, bb;
    for (int k = 0; k < 8; ++k) {
        a[k] = (_Float16)(threadIdx.x * 0.001f + k);
        bb[k] = (_Float16)(k * 0.01f);
    }
    for (int i = 0; i < iters; ++i) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bb, acc, 0, 0, 0);
        lds[(threadIdx.x * 33 + i) & 8191] = acc.x;
        a[0] = (_Float16)lds[(threadIdx.x * 17 + i) & 8191];
    }
    if (acc.x == 1.2345f) sink[threadIdx.x] = acc.y;
}

extern "C" int pk_proj(int variant, const float* xyz, const float* w, const float* b, int npts, float* out, hipStream_t st) {
    const unsigned blocks = (unsigned)(((size_t)npts * 8 + 255) / 256);
    if (variant == 0)
        hipLaunchKernelGGL(proj_kernel<true>, dim3(blocks), dim3(256), 0, st, xyz, w, b, npts, out);
    else
        hipLaunchKernelGGL(proj_kernel<false>, dim3(blocks), dim3(256), 0, st, xyz, w, b, npts, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int pk_load(int blocks, int iters, float* sink, hipStream_t st) {
    hipLaunchKernelGGL(load_kernel, dim3(blocks), dim3(256), 0, st, sink, iters);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
