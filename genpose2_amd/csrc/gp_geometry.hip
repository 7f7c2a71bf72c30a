// Point-cloud geometry kernels for gfx950: farthest-point sampling, ball query, gather/group.
//
// Semantics follow the reference CUDA text (networks/pts_encoder/pointnet2_utils/pointnet2/
// src/sampling_gpu.cu, ball_query_gpu.cu, group_points_gpu.cu); the execution design does not.
//
// FPS: the reference runs min(2^floor(log2 n),1024) threads, keeps the running min-distance in
// GLOBAL memory and reduces through a 10-level shared-memory tree with a barrier per level.
// Here one 256-thread workgroup per object keeps min-distances in VGPRs and the point set in
// LDS, and picks the farthest point with a single 64-bit max (distance bits | tie key) through
// wave shuffles + one LDS exchange per iteration. The tie key reproduces the reference winner
// exactly: the reference prefers, among equal distances, the first point in a thread's strided
// scan (strict >) and then the lower shared-memory slot at every tree level, i.e. the thread
// whose index is smallest in bit-reversed order. key = bitrev(k mod bs) << jbits | k / bs.
//
// Ball query: one wave per centroid scans 64 points per step with two ballots (both radii of
// an MSG level at once) and writes the hits in index order with mbcnt ranks; early exit when
// every list is full.
#include <stdarg.h>
#include <stdio.h>

#include "gp_common.h"
#include "gp_fps.h"

// ============================================================================ error plumbing
static thread_local char g_err[512];

void gp_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int gp_check_launch(const char* what) {
#ifdef GP_DEBUG_SYNC   // diagnostic builds only: every launch completes before the host continues
    (void)hipDeviceSynchronize();
#endif
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gp_set_error("%s: %s", what, hipGetErrorString(e));
        return GP_ERR_LAUNCH;
    }
    return GP_OK;
}

extern "C" const char* gp_last_error(void) { return g_err; }
extern "C" int gp_abi_version(void) { return GP_ABI_VERSION; }

// ============================================================================ FPS (core in gp_fps.h)
template <int PMAX>
__global__ __launch_bounds__(FPS_THREADS) void fps_kernel(const float* __restrict__ xyz, int n, int m,
                                                          int nb, int jbits, int* __restrict__ idx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    void* s_red = smem;
    float* s_xyz = reinterpret_cast<float*>(smem + FPS_RED_BYTES);
    const int b = blockIdx.x;
    const float* src = xyz + (size_t)b * n * 3;
    int* s_idx = reinterpret_cast<int*>(s_xyz + 3 * n);
    for (int i = threadIdx.x; i < 3 * n; i += FPS_THREADS) s_xyz[i] = src[i];
    __syncthreads();
    fps_run<PMAX>(s_xyz, n, m, nb, jbits, s_red, s_idx, nullptr);
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += FPS_THREADS) idx[(size_t)b * m + i] = s_idx[i];
}

static int launch_fps(const float* xyz, int b, int n, int m, int* idx, hipStream_t st) {
    const FpsGeom g = fps_geom(n);
    const size_t lds = FPS_RED_BYTES + sizeof(float) * 3 * (size_t)n + sizeof(int) * (size_t)m;
    if (lds > 160 * 1024) {
        gp_set_error("furthest_point_sampling: n=%d, m=%d exceed the LDS budget", n, m);
        return GP_ERR_UNSUPPORTED;
    }
    const int p = (n + FPS_THREADS - 1) / FPS_THREADS;
#define GP_FPS_CASE(PM)                                                                      \
    if (p <= PM) {                                                                           \
        hipLaunchKernelGGL(fps_kernel<PM>, dim3(b), dim3(FPS_THREADS), lds, st, xyz, n, m, g.nb, \
                           g.jbits, idx);                                                    \
        return gp_check_launch("fps_kernel");                                                \
    }
    GP_FPS_CASE(1) GP_FPS_CASE(2) GP_FPS_CASE(4) GP_FPS_CASE(8) GP_FPS_CASE(16) GP_FPS_CASE(32)
#undef GP_FPS_CASE
    gp_set_error("furthest_point_sampling: n=%d exceeds 8192", n);
    return GP_ERR_UNSUPPORTED;
}

extern "C" int gp_furthest_point_sampling(int b, int n, int m, const float* xyz, float* temp,
                                          int* idx, hipStream_t stream) {
    (void)temp;
    GP_REQUIRE(b >= 0 && n >= 1 && m >= 0, "furthest_point_sampling: bad sizes b=%d n=%d m=%d", b, n, m);
    GP_REQUIRE(xyz && idx, "furthest_point_sampling: null pointer");
    if (b == 0 || m == 0) return GP_OK;
    return launch_fps(xyz, b, n, m, idx, stream);
}

// ---------------------------------------------------------------------------- FPS chain
// All SA levels' FPS for one object in one workgroup: level l samples M_l points from the
// M_{l-1} points chosen by level l-1 (pointnet2_modules.py:39-47 applied level after level).
struct ChainArgs {
    int nlev;
    int n[4];      // input size per level
    int m[4];      // samples per level
    int nb[4];
    int jbits[4];
    int* idx[4];   // (B, m_l)
    float* nxyz[4];  // (B, m_l, 3)
};

template <int PMAX, int NTH>
__global__ __launch_bounds__(NTH) void fps_chain_kernel(const float* __restrict__ xyz, ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    void* s_red = smem;
    float* bufA = reinterpret_cast<float*>(smem + FPS_RED_BYTES);
    float* bufB = bufA + 3 * a.n[0];
    int* s_idx = reinterpret_cast<int*>(bufB + 3 * a.m[0]);
    const int b = blockIdx.x;
    const float* src = xyz + (size_t)b * a.n[0] * 3;
    for (int i = threadIdx.x; i < 3 * a.n[0]; i += NTH) bufA[i] = src[i];
    __syncthreads();
    float* cur = bufA;
    float* nxt = bufB;
    for (int l = 0; l < a.nlev; ++l) {
        fps_run<PMAX, NTH>(cur, a.n[l], a.m[l], a.nb[l], a.jbits[l], s_red, s_idx, nxt);
        __syncthreads();
        int* gi = a.idx[l] + (size_t)b * a.m[l];
        float* gx = a.nxyz[l] + (size_t)b * a.m[l] * 3;
        for (int i = threadIdx.x; i < a.m[l]; i += NTH) gi[i] = s_idx[i];
        for (int i = threadIdx.x; i < 3 * a.m[l]; i += NTH) gx[i] = nxt[i];
        __syncthreads();
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
}

int gp_launch_fps_chain(const float* xyz, int b, int nlev, const int* n, const int* m, int* const* idx,
                        float* const* nxyz, hipStream_t st) {
    ChainArgs a;
    a.nlev = nlev;
    for (int l = 0; l < nlev; ++l) {
        a.n[l] = n[l];
        a.m[l] = m[l];
        const FpsGeom g = fps_geom(n[l]);
        a.nb[l] = g.nb;
        a.jbits[l] = g.jbits;
        a.idx[l] = idx[l];
        a.nxyz[l] = nxyz[l];
    }
    const size_t lds = FPS_RED_BYTES + sizeof(float) * 3 * ((size_t)n[0] + (size_t)m[0]) + sizeof(int) * (size_t)m[0];
#ifndef FPS_CHAIN_NTH
#define FPS_CHAIN_NTH 512   // 8 waves per object: measured 3.04 vs 3.07 ms (256) and 3.21 (1024) encoder at B=64
#endif
    const int p = (n[0] + FPS_CHAIN_NTH - 1) / FPS_CHAIN_NTH;
#define GP_CHAIN_CASE(PM)                                                                       \
    if (p <= PM) {                                                                              \
        hipLaunchKernelGGL((fps_chain_kernel<PM, FPS_CHAIN_NTH>), dim3(b), dim3(FPS_CHAIN_NTH), lds, st, xyz, a); \
        return gp_check_launch("fps_chain_kernel");                                             \
    }
    GP_CHAIN_CASE(1) GP_CHAIN_CASE(2) GP_CHAIN_CASE(4) GP_CHAIN_CASE(8) GP_CHAIN_CASE(16) GP_CHAIN_CASE(32)
#undef GP_CHAIN_CASE
    gp_set_error("encoder: n=%d exceeds 8192", n[0]);
    return GP_ERR_UNSUPPORTED;
}

// ============================================================================ ball query
// NR radii (1 or 2) answered by the same scan.
constexpr int BQ_CPW = 8;
// Scan state of one centroid: hits so far and the first hit, per radius.
struct BqState {
    int cnta, cntb, firsta, firstb;
};

template <int NR>
__device__ __forceinline__ void bq_take(float d2, int k, int n, int base, float r2a, float r2b, int nsa, int nsb,
                                        unsigned long long lt, int* oa, int* ob, BqState& st) {
    const bool ha = (k < n) && d2 < r2a;
    const unsigned long long ma = __ballot(ha);
    if (st.cnta < nsa && ma) {
        const int rank = st.cnta + __popcll(ma & lt);
        if (ha && rank < nsa) oa[rank] = k;
        if (st.firsta < 0) st.firsta = base + __ffsll((long long)ma) - 1;
        st.cnta += __popcll(ma);
    }
    if (NR > 1) {
        const bool hb = (k < n) && d2 < r2b;
        const unsigned long long mb = __ballot(hb);
        if (st.cntb < nsb && mb) {
            const int rank = st.cntb + __popcll(mb & lt);
            if (hb && rank < nsb) ob[rank] = k;
            if (st.firstb < 0) st.firstb = base + __ffsll((long long)mb) - 1;
            st.cntb += __popcll(mb);
        }
    }
}

template <int NR>
__device__ __forceinline__ void bq_pad(int lane, int nsa, int nsb, int* oa, int* ob, const BqState& st) {
    // pad with the first hit (ball_query_gpu.cu:35-40); no hit -> 0 (zero-initialised output)
    for (int s = (st.cnta < nsa ? st.cnta : nsa) + lane; s < nsa; s += 64) oa[s] = st.firsta < 0 ? 0 : st.firsta;
    if (NR > 1)
        for (int s = (st.cntb < nsb ? st.cntb : nsb) + lane; s < nsb; s += 64) ob[s] = st.firstb < 0 ? 0 : st.firstb;
}

// One wave scans two centroids at once (p and p + 4): the distances of a point to both are packed fp32
// operations (v_pk_add_f32 / v_pk_mul_f32), each rounded exactly as dist2_ref. 4 * BQ_CPW centroids of one
// object per workgroup. The points are read from global memory (L1/L2-resident: 12 B x n per object), NOT
// staged in LDS: with several processes time-sharing the GPU the LDS-staged point set intermittently gave
// wrong ball lists (points dropping out of balls) while the identical global-memory kernel stayed
// bit-exact (DESIGN (c), profiles/r5/race_probe_history.md).
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int NR>
__global__ __launch_bounds__(256) void ball_query_kernel(int n, int m, const float* __restrict__ new_xyz,
                                                         const float* __restrict__ xyz, float r2a,
                                                         float r2b, int nsa, int nsb,
                                                         int* __restrict__ idxa,
                                                         int* __restrict__ idxb) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    const float* pts = xyz + (size_t)b * n * 3;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int pend = min(m, (int)(blockIdx.x + 1) * 4 * BQ_CPW);
    for (int p = blockIdx.x * 4 * BQ_CPW + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); p < pend; p += 8) {
        const int q = p + 4 < pend ? p + 4 : p;   // second centroid (a repeat of the first when absent)
        const float* c0 = new_xyz + ((size_t)b * m + p) * 3;
        const float* c1 = new_xyz + ((size_t)b * m + q) * 3;
        const f32x2 cx = {ld1(c0), ld1(c1)}, cy = {ld1(c0 + 1), ld1(c1 + 1)}, cz = {ld1(c0 + 2), ld1(c1 + 2)};
        int* oa0 = idxa + ((size_t)b * m + p) * nsa;
        int* oa1 = idxa + ((size_t)b * m + q) * nsa;
        int* ob0 = NR > 1 ? idxb + ((size_t)b * m + p) * nsb : nullptr;
        int* ob1 = NR > 1 ? idxb + ((size_t)b * m + q) * nsb : nullptr;
        BqState s0 = {0, 0, -1, -1}, s1 = {0, 0, -1, -1};
        const bool two = q != p;
        for (int base = 0; base < n; base += 64) {
            const int k = base + lane;
            f32x2 d2 = {3.0e38f, 3.0e38f};
            if (k < n) {
#pragma clang fp contract(off)
                const float px = ld1(pts + 3 * k + 0), py = ld1(pts + 3 * k + 1), pz = ld1(pts + 3 * k + 2);
                const f32x2 dx = cx - f32x2{px, px}, dy = cy - f32x2{py, py}, dz = cz - f32x2{pz, pz};
                d2 = (dx * dx + dy * dy) + dz * dz;
            }
            bq_take<NR>(d2.x, k, n, base, r2a, r2b, nsa, nsb, lt, oa0, ob0, s0);
            if (two) bq_take<NR>(d2.y, k, n, base, r2a, r2b, nsa, nsb, lt, oa1, ob1, s1);
            const bool done0 = s0.cnta >= nsa && (NR == 1 || s0.cntb >= nsb);
            const bool done1 = !two || (s1.cnta >= nsa && (NR == 1 || s1.cntb >= nsb));
            if (done0 && done1) break;
        }
        bq_pad<NR>(lane, nsa, nsb, oa0, ob0, s0);
        if (two) bq_pad<NR>(lane, nsa, nsb, oa1, ob1, s1);
    }
}

int gp_launch_ball_query2(int b, int n, int m, float ra, float rb, int nsa, int nsb,
                          const float* new_xyz, const float* xyz, int* idxa, int* idxb,
                          hipStream_t st) {
    const float r2a = ra * ra, r2b = rb * rb;  // radius2 = radius * radius in fp32
    dim3 grid((m + 4 * BQ_CPW - 1) / (4 * BQ_CPW), b);
    if (idxb)
        hipLaunchKernelGGL((ball_query_kernel<2>), grid, dim3(256), 0, st, n, m, new_xyz, xyz, r2a, r2b, nsa, nsb, idxa, idxb);
    else
        hipLaunchKernelGGL((ball_query_kernel<1>), grid, dim3(256), 0, st, n, m, new_xyz, xyz, r2a, 0.f, nsa, 0, idxa,
                           nullptr);
    return gp_check_launch("ball_query_kernel");
}

extern "C" int gp_ball_query(int b, int n, int m, float radius, int nsample, const float* new_xyz,
                             const float* xyz, int* idx, hipStream_t stream) {
    GP_REQUIRE(b >= 0 && n >= 0 && m >= 0 && nsample >= 1, "ball_query: bad sizes");
    GP_REQUIRE(new_xyz && xyz && idx, "ball_query: null pointer");
    if (b == 0 || m == 0) return GP_OK;
    return gp_launch_ball_query2(b, n, m, radius, 0.f, nsample, 0, new_xyz, xyz, idx, nullptr, stream);
}

// ============================================================================ gather / group
__global__ void gather_points_kernel(int c, int n, int m, const float* __restrict__ pts,
                                     const int* __restrict__ idx, float* __restrict__ out) {
    const int b = blockIdx.z, ch = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    out[((size_t)b * c + ch) * m + i] = pts[((size_t)b * c + ch) * n + idx[(size_t)b * m + i]];
}

extern "C" int gp_gather_points(int b, int c, int n, int npoints, const float* points, const int* idx,
                                float* out, hipStream_t stream) {
    GP_REQUIRE(b >= 0 && c >= 0 && n >= 0 && npoints >= 0, "gather_points: bad sizes");
    GP_REQUIRE(points && idx && out, "gather_points: null pointer");
    if (!b || !c || !npoints) return GP_OK;
    hipLaunchKernelGGL(gather_points_kernel, dim3((npoints + 255) / 256, c, b), dim3(256), 0, stream, c, n,
                       npoints, points, idx, out);
    return gp_check_launch("gather_points_kernel");
}

__global__ void group_points_kernel(int c, int n, int m, int ns, const float* __restrict__ pts,
                                    const int* __restrict__ idx, float* __restrict__ out) {
    const int b = blockIdx.z, ch = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m * ns) return;
    out[((size_t)b * c + ch) * m * ns + i] = pts[((size_t)b * c + ch) * n + idx[(size_t)b * m * ns + i]];
}

extern "C" int gp_group_points(int b, int c, int n, int npoints, int nsample, const float* points,
                               const int* idx, float* out, hipStream_t stream) {
    GP_REQUIRE(b >= 0 && c >= 0 && n >= 0 && npoints >= 0 && nsample >= 1, "group_points: bad sizes");
    GP_REQUIRE(points && idx && out, "group_points: null pointer");
    if (!b || !c || !npoints) return GP_OK;
    hipLaunchKernelGGL(group_points_kernel, dim3((npoints * nsample + 255) / 256, c, b), dim3(256), 0,
                       stream, c, n, npoints, nsample, points, idx, out);
    return gp_check_launch("group_points_kernel");
}
