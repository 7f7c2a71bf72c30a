// The --dino pointwise image branch for gfx950: ImgEncoder.forward (networks/img_encoder/img_encoder.py:48-100)
// over the three DINOv3 intermediate layers, and the patch -> point gather of GFObjectPose.extract_pts_feature
// (networks/posenet.py:146-192). Tokens are patch-major (b, np, d) as the backbone returns them.
//
//   layer attention   Linear(d, d/2) -> ReLU on the three layers as one exact-fp32 MFMA GEMM (gp_linear over
//                     3*b*np tokens), then imgenc_layer_fuse_kernel: Linear(d/2, 1), softmax over the layers
//                     and the weighted sum -- a wave per token;
//   edge branch       Conv2d(d, d/4, 3, padding 1) as an im2col GEMM (gp_linear with ReLU, the conv weight
//                     (d/4, d*9) as stored: columns in [c][dy][dx] order) over object chunks, then the mean
//                     over the 16 x 16 pixels in the reference's sequential order;
//   geo attention     S = G G^T (G = the last 3d/4 channels) and O = P F as batched exact-fp32 MFMA GEMMs,
//                     S x (the host-built position table) and the row softmax between them, a wave per row;
//   final mix         (F + relu(geo_w) O) + relu(edge_w) (F x edge[c % (d/4)]), in the reference's order.
#include "gp_common.h"

constexpr int IE_THREADS = 256;

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---------------------------------------------------------------- layer attention fuse
// h: (3, T, hid) = relu(W1 f_l + b1) for the three layers (layer-major), T = b * np tokens.
// s_l = w2 . h_l + b2; a = softmax_l(s) (max, exp(s - max), sum, x * (1 / sum)); fused = (f0 a0 + f1 a1) + f2 a2.
__global__ __launch_bounds__(IE_THREADS) void imgenc_layer_fuse_kernel(const float* __restrict__ h, int hid,
                                                                       const float* __restrict__ w2, float b2,
                                                                       const float* __restrict__ f0,
                                                                       const float* __restrict__ f1,
                                                                       const float* __restrict__ f2, int T, int d,
                                                                       float* __restrict__ fused,
                                                                       float* __restrict__ layer_w) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int tok = blockIdx.x * (IE_THREADS / 64) + (threadIdx.x >> 6);
    if (tok >= T) return;
    float s[3];
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        const float* hr = h + ((size_t)l * T + tok) * hid;
        float acc = 0.f;
        for (int c = lane; c < hid; c += 64) acc += hr[c] * w2[c];
        s[l] = wave_sum_f(acc) + b2;
    }
    const float m = fmaxf(fmaxf(s[0], s[1]), s[2]);
    const float e0 = expf(s[0] - m), e1 = expf(s[1] - m), e2 = expf(s[2] - m);
    const float inv = 1.0f / ((e0 + e1) + e2);
    const float a0 = e0 * inv, a1 = e1 * inv, a2 = e2 * inv;
    if (layer_w && lane < 3) layer_w[(size_t)tok * 3 + lane] = lane == 0 ? a0 : (lane == 1 ? a1 : a2);
    const size_t base = (size_t)tok * d;
    for (int c = lane; c < d; c += 64) fused[base + c] = (f0[base + c] * a0 + f1[base + c] * a1) + f2[base + c] * a2;
}

// ---------------------------------------------------------------- edge branch
// im2col of Conv2d(d, co, 3, padding=1) over spatial_feat = F^T viewed (d, g, g) (img_encoder.py:92):
// col[(b*np + p)][c*9 + dy*3 + dx] = F[b][(y+dy-1)*g + (x+dx-1)][c] inside the grid, 0 outside.
__global__ __launch_bounds__(IE_THREADS) void imgenc_im2col_kernel(const float* __restrict__ f, int np, int g, int d,
                                                                   float* __restrict__ col) {
    const int bp = blockIdx.x;                       // (object, pixel) of this chunk
    const int b = bp / np, p = bp - b * np;
    const int y = p / g, x = p - y * g;
    float* out = col + (size_t)bp * d * 9;
    for (int e = threadIdx.x; e < d * 9; e += IE_THREADS) {
        const int c = e / 9, k = e - c * 9, dy = k / 3, dx = k - dy * 3;
        const int yy = y + dy - 1, xx = x + dx - 1;
        out[e] = (yy >= 0 && yy < g && xx >= 0 && xx < g) ? f[((size_t)b * np + yy * g + xx) * d + c] : 0.f;
    }
}

// Row maxima of the implicit im2col (gp_linear_split_conv3x3): pmax[t] = max |f[t][:]| per pixel (a wave per pixel),
// then rmax[t] = the max of pmax over the pixel's in-grid 3x3 neighbourhood -- the max |x| of its im2col row (the
// zero padding adds 0), bit for bit what a row max over the formed column buffer gives.
__global__ __launch_bounds__(IE_THREADS) void imgenc_pixel_max_kernel(const float* __restrict__ f, int t, int d,
                                                                      float* __restrict__ pmax) {
    const int r = blockIdx.x * (IE_THREADS / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= t) return;
    float v = 0.f;
    for (int c = 4 * lane; c < d; c += 256) {
        const f32x4 x = ld4(f + (size_t)r * d + c);
        v = fmaxf(v, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    if (lane == 0) pmax[r] = v;
}
__global__ void imgenc_nbr_max_kernel(const float* __restrict__ pmax, int t, int g, float* __restrict__ rmax) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= t) return;
    const int p = r % (g * g), y = p / g, x = p - y * g;
    float v = 0.f;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx)
            if (y + dy >= 0 && y + dy < g && x + dx >= 0 && x + dx < g) v = fmaxf(v, pmax[r + dy * g + dx]);
    rmax[r] = v;
}

// edge[b][o] = (sum_p y[b][p][o], p in order) / np -- AdaptiveAvgPool2d(1)'s sequential sum (np = 256: the
// division is exact scaling, as the reference's / kh / kw)
__global__ void imgenc_pool_kernel(const float* __restrict__ y, int nb, int np, int co, float* __restrict__ edge) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nb * co) return;
    const int b = e / co, o = e - b * co;
    const float* yp = y + (size_t)b * np * co + o;
    float s = 0.f;
    int p = 0;
    // 16 loads in flight per step, added in p order (a load per dependent add waited ~600 cycles each)
    for (; p + 16 <= np; p += 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = yp[(size_t)(p + j) * co];
#pragma unroll
        for (int j = 0; j < 16; ++j) s += v[j];
    }
    for (; p < np; ++p) s += yp[(size_t)p * co];
    edge[e] = s / (float)np;
}

// ---------------------------------------------------------------- batched GEMM (exact f32 MFMA)
// C[z][i][j] = sum_k A[z][i][k] B[z][j][k]; A rows i (lda, batch stride sa), B rows j (ldb, sb), C (ldc, sc).
// 4 waves as 2 (i) x 2 (j); a wave owns TM i-tiles x TN j-tiles of 16. Lane (q, r) feeds float4 k-slices
// 16g + 4q .. +3 of row r of both operands (k a multiple of 16, rows 16-byte aligned).
template <int TM, int TN>
__global__ __launch_bounds__(IE_THREADS) void bgemm_nt_kernel(const float* __restrict__ A, int lda, long long sa,
                                                              const float* __restrict__ Bm, int ldb, long long sb,
                                                              float* __restrict__ C, int ldc, long long sc, int M,
                                                              int N, int K) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int q = lane >> 4, r = lane & 15;
    const int z = blockIdx.z;
    A += z * sa;
    Bm += z * sb;
    C += z * sc;
    const int i0 = blockIdx.x * (32 * TM) + (wid & 1) * (16 * TM);
    const int j0 = blockIdx.y * (32 * TN) + (wid >> 1) * (16 * TN);
    const float* ap[TM];
    const float* bp[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) ap[t] = A + (size_t)min(i0 + 16 * t + r, M - 1) * lda + 4 * q;
#pragma unroll
    for (int u = 0; u < TN; ++u) bp[u] = Bm + (size_t)min(j0 + 16 * u + r, N - 1) * ldb + 4 * q;
    f32x4 acc[TN][TM];
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int t = 0; t < TM; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int KG = K >> 4;
    f32x4 aa[TM], ba[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) aa[t] = ld4(ap[t]);
#pragma unroll
    for (int u = 0; u < TN; ++u) ba[u] = ld4(bp[u]);
    for (int g = 0; g < KG; ++g) {
        f32x4 an[TM], bn[TN];
        const int kn = (g + 1 < KG ? g + 1 : g) * 16;
#pragma unroll
        for (int t = 0; t < TM; ++t) an[t] = ld4(ap[t] + kn);
#pragma unroll
        for (int u = 0; u < TN; ++u) bn[u] = ld4(bp[u] + kn);
        // D rows = j (B operand rows as the MFMA A input), columns = i
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
            for (int u = 0; u < TN; ++u)
#pragma unroll
                for (int t = 0; t < TM; ++t) acc[u][t] = mfma4(ba[u][jj], aa[t][jj], acc[u][t]);
#pragma unroll
        for (int t = 0; t < TM; ++t) aa[t] = an[t];
#pragma unroll
        for (int u = 0; u < TN; ++u) ba[u] = bn[u];
    }
#pragma unroll
    for (int u = 0; u < TN; ++u) {
        const int jt = j0 + 16 * u;
        if (jt >= N) continue;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            const int i = i0 + 16 * t + r;
            if (i >= M) continue;
            st4(C + (size_t)i * ldc + jt + 4 * q, acc[u][t]);
        }
    }
}

static void launch_bgemm_nt(const float* A, int lda, long long sa, const float* B, int ldb, long long sb, float* C,
                            int ldc, long long sc, int M, int N, int K, int batch, hipStream_t st) {
    constexpr int TM = 2, TN = 2;
    const dim3 grid((M + 32 * TM - 1) / (32 * TM), (N + 32 * TN - 1) / (32 * TN), batch);
    hipLaunchKernelGGL((bgemm_nt_kernel<TM, TN>), grid, dim3(IE_THREADS), 0, st, A, lda, sa, B, ldb, sb, C, ldc, sc,
                       M, N, K);
}

// F (b, np, d) -> FT (b, d, np), so O = P F is an NT product against FT
__global__ __launch_bounds__(IE_THREADS) void imgenc_transpose_kernel(const float* __restrict__ f, int np, int d,
                                                                      float* __restrict__ ft) {
    __shared__ float tile[32][33];
    const int b = blockIdx.z;
    const int p0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
    for (int yy = ty; yy < 32; yy += 8) {
        const int p = p0 + yy, c = c0 + tx;
        tile[yy][tx] = (p < np && c < d) ? f[((size_t)b * np + p) * d + c] : 0.f;
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {
        const int c = c0 + yy, p = p0 + tx;
        if (c < d && p < np) ft[((size_t)b * d + c) * np + p] = tile[tx][yy];
    }
}

// row softmax of S x table (img_encoder.py:83-85), in place: a wave per (object, query) row of np keys
__global__ __launch_bounds__(IE_THREADS) void imgenc_softmax_kernel(float* __restrict__ s, const float* __restrict__ tab,
                                                                    int rows, int np) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (IE_THREADS / 64) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int i = row % np;
    float* sr = s + (size_t)row * np;
    const float* tr = tab + (size_t)i * np;
    float m = -INFINITY;
    for (int j = lane; j < np; j += 64) m = fmaxf(m, sr[j] * tr[j]);
    m = wave_max_f(m);
    float sum = 0.f;
    for (int j = lane; j < np; j += 64) {
        const float e = expf(sr[j] * tr[j] - m);
        sr[j] = e;
        sum += e;
    }
    const float inv = 1.0f / wave_sum_f(sum);
    for (int j = lane; j < np; j += 64) sr[j] = sr[j] * inv;
}

// final = (F + geo_gate O) + edge_gate (F x edge[c % co])  (img_encoder.py:94-99)
__global__ __launch_bounds__(IE_THREADS) void imgenc_combine_kernel(const float* __restrict__ f,
                                                                    const float* __restrict__ o,
                                                                    const float* __restrict__ edge, int np, int d,
                                                                    int co, float geo_gate, float edge_gate,
                                                                    long long n, float* __restrict__ out) {
#pragma clang fp contract(off)
    const long long e = (long long)blockIdx.x * IE_THREADS + threadIdx.x;
    if (e >= n) return;
    const int c = (int)(e % d);
    const long long b = e / ((long long)np * d);
    const float fv = f[e];
    out[e] = (fv + geo_gate * o[e]) + edge_gate * (fv * edge[b * co + c % co]);
}

// ---------------------------------------------------------------- patch -> point gather
// out[b][n][:] = feat[b][clamp((xs // px) * grid + ys // px, 0, np - 1)][:] (floor division, posenet.py:146-192)
__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ __launch_bounds__(IE_THREADS) void gather_patch_kernel(const float* __restrict__ feat, int np, int d,
                                                                  const int* __restrict__ xs,
                                                                  const int* __restrict__ ys, int n, int px, int grid,
                                                                  float* __restrict__ out) {
    const int b = blockIdx.y;
    const int pt = blockIdx.x * (IE_THREADS / 64) + (threadIdx.x >> 6);
    if (pt >= n) return;
    const int lane = threadIdx.x & 63;
    int pos = floordiv(xs[(size_t)b * n + pt], px) * grid + floordiv(ys[(size_t)b * n + pt], px);
    pos = pos < 0 ? 0 : (pos > np - 1 ? np - 1 : pos);
    const float* src = feat + ((size_t)b * np + pos) * d;
    float* dst = out + ((size_t)b * n + pt) * d;
    for (int c = 4 * lane; c < d; c += 256) st4(dst + c, ld4(src + c));
}

extern "C" int gp_gather_patch_points(const float* feat, int b, int np, int d, const int* xs, const int* ys, int n,
                                      int patch_px, int grid, float* out, hipStream_t st) {
    GP_REQUIRE(feat && xs && ys && out && b >= 0 && np >= 1 && n >= 0 && patch_px >= 1 && grid >= 1,
               "gather_patch_points: bad arguments");
    GP_REQUIRE(d % 4 == 0 && ((uintptr_t)feat | (uintptr_t)out) % 16 == 0,
               "gather_patch_points: d must be a multiple of 4 and the tensors 16-byte aligned");
    if (!b || !n) return GP_OK;
    hipLaunchKernelGGL(gather_patch_kernel, dim3((n + 3) / 4, b), dim3(IE_THREADS), 0, st, feat, np, d, xs, ys, n,
                       patch_px, grid, out);
    return gp_check_launch("gather_patch_kernel");
}

// ---------------------------------------------------------------- host: position table, workspace, driver
extern "C" int gp_img_geo_table(const float* rel_pos_emb, int num_emb, int edim, int grid, float* table) {
    GP_REQUIRE(rel_pos_emb && table && num_emb >= 1 && edim >= 1 && grid >= 2, "img_geo_table: bad arguments");
    const int np = grid * grid, span = 2 * (grid - 1) + 1;
    for (int i = 0; i < np; ++i)
        for (int j = 0; j < np; ++j) {
            const int r0 = j / grid - i / grid + grid - 1, r1 = j % grid - i % grid + grid - 1;
            int idx = r0 * span + r1;
            idx = idx < 0 ? 0 : (idx > num_emb - 1 ? num_emb - 1 : idx);
            float s = 0.f;
            for (int k = 0; k < edim; ++k) s += rel_pos_emb[(size_t)idx * edim + k];
            table[(size_t)i * np + j] = s;
        }
    return GP_OK;
}

namespace {
constexpr int IE_EDGE_CHUNK = 256;  // objects per im2col GEMM (col: chunk * np * 9d floats, 906 MB at np = 256, d = 384):
                                     // 32 gave the split GEMM (n = 96 outputs) only 32 workgroups per launch; 256 objects
                                     // fill the chip (one workgroup per 256 tokens)
size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }
struct ImgLayout {
    size_t h, fused, s, ft, o, col, ey, edge, rmax, total;
};
// implicit: the split edge conv of gp_img_encoder3 (no column buffer; its output and pixel maxima for all objects)
ImgLayout img_layout(int b, int np, int d, bool implicit = false) {
    ImgLayout L = {};
    const int co = d / 4, hid = d / 2, chunk = implicit ? b : (b < IE_EDGE_CHUNK ? b : IE_EDGE_CHUNK);
    size_t off = 0;
    L.h = off;     off += al256(sizeof(float) * 3 * (size_t)b * np * hid);
    L.fused = off; off += al256(sizeof(float) * (size_t)b * np * d);
    L.s = off;     off += al256(sizeof(float) * (size_t)b * np * np);
    L.ft = off;    off += al256(sizeof(float) * (size_t)b * np * d);
    L.o = off;     off += al256(sizeof(float) * (size_t)b * np * d);
    L.col = off;   off += implicit ? al256(sizeof(float) * (size_t)b * np) : al256(sizeof(float) * (size_t)chunk * np * 9 * d);
    L.ey = off;    off += al256(sizeof(float) * (size_t)chunk * np * co);
    L.edge = off;  off += al256(sizeof(float) * (size_t)b * co);
    L.rmax = off;  off += al256(sizeof(float) * (size_t)b * np);   // split GEMMs: per-token row maxima
    L.total = off;
    return L;
}
}  // namespace

extern "C" size_t gp_img_encoder_workspace_size(int b, int np, int d) {
    return b >= 1 && np >= 1 && d >= 4 ? img_layout(b, np, d).total : 0;
}

extern "C" size_t gp_img_encoder3_workspace_size(int b, int np, int d, int split_conv) {
    return b >= 1 && np >= 1 && d >= 4 ? img_layout(b, np, d, split_conv != 0).total : 0;
}

// y = relu(x W^T + b): split-f16 (gp_linear_split, the token linears' arithmetic: per-token power-of-two scaling,
// three f16 products) when the weight planes are given, exact fp32 MFMA (gp_linear) otherwise
static int img_linear_relu(const float* x, int m, int k, const float* w, const int32_t* wh, const float* bias, int n,
                           float* y, float* rmax, hipStream_t st) {
    if (wh) return gp_linear_split(x, k, m, k, wh, bias, n, 1, y, n, rmax, 0, nullptr, st);
    return gp_linear(x, k, m, k, w, bias, n, 1, y, n, st);
}

// implicit: conv_w_h holds the position-major planes and the edge conv runs as gp_linear_split_conv3x3
static int img_encoder_impl(const float* l0, const float* l1, const float* l2, int b, int np, int d,
                            const float* la_w1, const float* la_b1, const float* la_w2, float la_b2,
                            const float* geo_table, const float* conv_w, const float* conv_b, float geo_gate,
                            float edge_gate, const int32_t* la_w1_h, const int32_t* conv_w_h, bool implicit, float* out,
                            float* layer_w, float* edge_out, void* workspace, size_t workspace_bytes, hipStream_t st) {
    GP_REQUIRE(l0 && l1 && l2 && la_w1 && la_b1 && la_w2 && geo_table && conv_w && conv_b && out && workspace,
               "img_encoder: null pointer");
    GP_REQUIRE(b >= 0 && np >= 4 && d % 64 == 0, "img_encoder: need np >= 4 and d a multiple of 64 (d=%d)", d);
    int g = 1;
    while (g * g < np) ++g;
    GP_REQUIRE(g * g == np && np % 16 == 0, "img_encoder: np=%d must be a square grid with np %% 16 == 0", np);
    if (!b) return GP_OK;
    implicit = implicit && conv_w_h != nullptr;
    const ImgLayout L = img_layout(b, np, d, implicit);
    GP_REQUIRE(workspace_bytes >= L.total, "img_encoder: workspace too small (gp_img_encoder%s_workspace_size)",
               implicit ? "3" : "");
    char* ws = static_cast<char*>(workspace);
    float* h = reinterpret_cast<float*>(ws + L.h);
    float* fused = reinterpret_cast<float*>(ws + L.fused);
    float* s = reinterpret_cast<float*>(ws + L.s);
    float* ft = reinterpret_cast<float*>(ws + L.ft);
    float* o = reinterpret_cast<float*>(ws + L.o);
    float* col = reinterpret_cast<float*>(ws + L.col);
    float* ey = reinterpret_cast<float*>(ws + L.ey);
    float* edge = edge_out ? edge_out : reinterpret_cast<float*>(ws + L.edge);
    float* rmax = reinterpret_cast<float*>(ws + L.rmax);
    const int T = b * np, hid = d / 2, co = d / 4;
    int rc;
    // 1. layer attention: Linear(d, d/2) + ReLU over each layer's tokens, then the fuse kernel
    const float* layers[3] = {l0, l1, l2};
    for (int l = 0; l < 3; ++l)
        if ((rc = img_linear_relu(layers[l], T, d, la_w1, la_w1_h, la_b1, hid, h + (size_t)l * T * hid, rmax, st)))
            return rc;
    hipLaunchKernelGGL(imgenc_layer_fuse_kernel, dim3((T + 3) / 4), dim3(IE_THREADS), 0, st, (const float*)h, hid,
                       la_w2, la_b2, l0, l1, l2, T, d, fused, layer_w);
    if ((rc = gp_check_launch("imgenc_layer_fuse_kernel"))) return rc;
    // 2. edge branch: im2col GEMM + ReLU per chunk of objects, then the pixel mean
    if (implicit) {   // the split GEMM gathers its column rows from the feature map itself
        float* pmax = col;   // (b * np) pixel maxima in the implicit layout
        hipLaunchKernelGGL(imgenc_pixel_max_kernel, dim3((T + 3) / 4), dim3(IE_THREADS), 0, st, (const float*)fused, T, d,
                           pmax);
        if ((rc = gp_check_launch("imgenc_pixel_max_kernel"))) return rc;
        hipLaunchKernelGGL(imgenc_nbr_max_kernel, dim3((T + 255) / 256), dim3(256), 0, st, (const float*)pmax, T, g,
                           rmax);
        if ((rc = gp_check_launch("imgenc_nbr_max_kernel"))) return rc;
        if ((rc = gp_linear_split_conv3x3(fused, b, g, d, conv_w_h, conv_b, co, ey, rmax, st))) return rc;
        hipLaunchKernelGGL(imgenc_pool_kernel, dim3((b * co + 255) / 256), dim3(256), 0, st, (const float*)ey, b, np, co,
                           edge);
        if ((rc = gp_check_launch("imgenc_pool_kernel"))) return rc;
    }
    for (int c0 = 0; c0 < (implicit ? 0 : b); c0 += IE_EDGE_CHUNK) {
        const int nb = b - c0 < IE_EDGE_CHUNK ? b - c0 : IE_EDGE_CHUNK;
        hipLaunchKernelGGL(imgenc_im2col_kernel, dim3(nb * np), dim3(IE_THREADS), 0, st,
                           (const float*)(fused + (size_t)c0 * np * d), np, g, d, col);
        if ((rc = gp_check_launch("imgenc_im2col_kernel"))) return rc;
        if ((rc = img_linear_relu(col, nb * np, 9 * d, conv_w, conv_w_h, conv_b, co, ey, rmax, st))) return rc;
        hipLaunchKernelGGL(imgenc_pool_kernel, dim3((nb * co + 255) / 256), dim3(256), 0, st, (const float*)ey, nb, np,
                           co, edge + (size_t)c0 * co);
        if ((rc = gp_check_launch("imgenc_pool_kernel"))) return rc;
    }
    // 3. geometric attention: S = G G^T, softmax(S x table), O = P F
    launch_bgemm_nt(fused + co, d, (long long)np * d, fused + co, d, (long long)np * d, s, np, (long long)np * np, np,
                    np, d - co, b, st);
    if ((rc = gp_check_launch("bgemm_nt_kernel<scores>"))) return rc;
    hipLaunchKernelGGL(imgenc_softmax_kernel, dim3((T + 3) / 4), dim3(IE_THREADS), 0, st, s, geo_table, T, np);
    if ((rc = gp_check_launch("imgenc_softmax_kernel"))) return rc;
    hipLaunchKernelGGL(imgenc_transpose_kernel, dim3((np + 31) / 32, (d + 31) / 32, b), dim3(IE_THREADS), 0, st,
                       (const float*)fused, np, d, ft);
    if ((rc = gp_check_launch("imgenc_transpose_kernel"))) return rc;
    launch_bgemm_nt(s, np, (long long)np * np, ft, np, (long long)np * d, o, d, (long long)np * d, np, d, np, b, st);
    if ((rc = gp_check_launch("bgemm_nt_kernel<values>"))) return rc;
    // 4. final mix
    const long long n = (long long)T * d;
    hipLaunchKernelGGL(imgenc_combine_kernel, dim3((unsigned)((n + IE_THREADS - 1) / IE_THREADS)), dim3(IE_THREADS), 0,
                       st, (const float*)fused, (const float*)o, (const float*)edge, np, d, co, geo_gate, edge_gate, n,
                       out);
    return gp_check_launch("imgenc_combine_kernel");
}

extern "C" int gp_img_encoder2(const float* l0, const float* l1, const float* l2, int b, int np, int d,
                               const float* la_w1, const float* la_b1, const float* la_w2, float la_b2,
                               const float* geo_table, const float* conv_w, const float* conv_b, float geo_gate,
                               float edge_gate, const int32_t* la_w1_h, const int32_t* conv_w_h, float* out,
                               float* layer_w, float* edge_out, void* workspace, size_t workspace_bytes, hipStream_t st) {
    return img_encoder_impl(l0, l1, l2, b, np, d, la_w1, la_b1, la_w2, la_b2, geo_table, conv_w, conv_b, geo_gate,
                            edge_gate, la_w1_h, conv_w_h, false, out, layer_w, edge_out, workspace, workspace_bytes, st);
}

extern "C" int gp_img_encoder3(const float* l0, const float* l1, const float* l2, int b, int np, int d,
                               const float* la_w1, const float* la_b1, const float* la_w2, float la_b2,
                               const float* geo_table, const float* conv_w, const float* conv_b, float geo_gate,
                               float edge_gate, const int32_t* la_w1_h, const int32_t* conv_w_hp, float* out,
                               float* layer_w, float* edge_out, void* workspace, size_t workspace_bytes, hipStream_t st) {
    return img_encoder_impl(l0, l1, l2, b, np, d, la_w1, la_b1, la_w2, la_b2, geo_table, conv_w, conv_b, geo_gate,
                            edge_gate, la_w1_h, conv_w_hp, true, out, layer_w, edge_out, workspace, workspace_bytes, st);
}

extern "C" int gp_img_encoder(const float* l0, const float* l1, const float* l2, int b, int np, int d,
                              const float* la_w1, const float* la_b1, const float* la_w2, float la_b2,
                              const float* geo_table, const float* conv_w, const float* conv_b, float geo_gate,
                              float edge_gate, float* out, float* layer_w, float* edge_out, void* workspace,
                              size_t workspace_bytes, hipStream_t st) {
    return gp_img_encoder2(l0, l1, l2, b, np, d, la_w1, la_b1, la_w2, la_b2, geo_table, conv_w, conv_b, geo_gate,
                           edge_gate, nullptr, nullptr, out, layer_w, edge_out, workspace, workspace_bytes, st);
}
