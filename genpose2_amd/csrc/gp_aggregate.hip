// Candidate ranking and pose aggregation on device (one workgroup of 64 threads per object).
//
// Reference: sort_poses_by_energy (networks/reward.py:131-155), aggregate_pose
// (runners/evaluation_single.py:160-219), average_quaternion_batch (utils/misc.py:295-317),
// rotation_6d_to_matrix / matrix_to_quaternion / quaternion_to_matrix
// (utils/transforms/rotation_conversions.py:41-161,556-577) and sklearn DBSCAN(eps, min_samples)
// applied with its default Euclidean metric to the ROWS of the quaternion distance matrix
// (SURVEY F9). The reference runs this as a host loop over objects with .cpu().numpy() round trips.
//
//  1. ranks by descending rotation / translation energy (ties -> lower candidate index);
//  2. top `retain` rotations (by rotation energy) and translations (by translation energy);
//  3. quaternion (wxyz) of each kept rotation, sign-oriented weighted outer-product mean, top
//     eigenvector by cyclic Jacobi on the 4x4 in fp64 (the reference calls fp32 eigh);
//  4. optional DBSCAN over the kept set (core: >= min_samples neighbours within eps incl. itself;
//     clusters grown depth-first from core points in index order), re-average of the largest
//     cluster (first label on count ties, numpy argmax);
//  5. mean translation, 4x4 [R t; 0 1].
#include "gp_common.h"

constexpr int AGG_THREADS = 64;
constexpr int AGG_MAXK = 1024;
constexpr int AGG_MAXKEEP = 128;

// normalize_rotation -> rotation_6d_to_matrix -> matrix_to_quaternion, fp32 (as the reference).
__device__ __forceinline__ void rot6_to_quat(const float* v, float* q) {
#pragma clang fp contract(off)
    float n1 = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    n1 = n1 > 1e-12f ? n1 : 1e-12f;
    const float b0 = v[0] / n1, b1 = v[1] / n1, b2 = v[2] / n1;
    const float d = (b0 * v[3] + b1 * v[4]) + b2 * v[5];
    float c0 = v[3] - d * b0, c1 = v[4] - d * b1, c2 = v[5] - d * b2;
    float n2 = sqrtf((c0 * c0 + c1 * c1) + c2 * c2);
    n2 = n2 > 1e-12f ? n2 : 1e-12f;
    c0 /= n2; c1 /= n2; c2 /= n2;
    const float b3x = b1 * c2 - b2 * c1, b3y = b2 * c0 - b0 * c2, b3z = b0 * c1 - b1 * c0;
    // matrix columns b1, b2, b3 (get_rot_matrix permutes rotation_6d_to_matrix's rows)
    const float m00 = b0, m01 = c0, m02 = b3x, m10 = b1, m11 = c1, m12 = b3y, m20 = b2, m21 = c2, m22 = b3z;
    float qa[4] = {((1.f + m00) + m11) + m22, ((1.f + m00) - m11) - m22, ((1.f - m00) + m11) - m22,
                   ((1.f - m00) - m11) + m22};
#pragma unroll
    for (int i = 0; i < 4; ++i) qa[i] = qa[i] > 0.f ? sqrtf(qa[i]) : 0.f;
    int best = 0;
    float qb = qa[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (qa[i] > qb) { qb = qa[i]; best = i; }
    float c[4];
    if (best == 0) { c[0] = qa[0] * qa[0]; c[1] = m21 - m12; c[2] = m02 - m20; c[3] = m10 - m01; }
    else if (best == 1) { c[0] = m21 - m12; c[1] = qa[1] * qa[1]; c[2] = m10 + m01; c[3] = m02 + m20; }
    else if (best == 2) { c[0] = m02 - m20; c[1] = m10 + m01; c[2] = qa[2] * qa[2]; c[3] = m12 + m21; }
    else { c[0] = m10 - m01; c[1] = m20 + m02; c[2] = m21 + m12; c[3] = qa[3] * qa[3]; }
    const float den = 2.f * (qb > 0.1f ? qb : 0.1f);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = c[i] / den;
}

// Top eigenvector of a symmetric 4x4 (cyclic Jacobi, fp64), oriented so that w >= 0 is kept and
// w <= 0 flipped exactly as ((q[0] > 0) - 0.5) * 2 * q does.
__device__ void top_eigvec4(double A[4][4], float* out) {
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int r = p + 1; r < 4; ++r) off += A[p][r] * A[p][r];
        const double diag = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2] + A[3][3] * A[3][3];
        if (off <= 1e-36 * diag || off < 1e-300) break;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int r = p + 1; r < 4; ++r) {
                if (A[p][r] == 0.0) continue;
                const double theta = (A[r][r] - A[p][p]) / (2.0 * A[p][r]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; ++k) {  // A <- J^T A J
                    const double akp = A[k][p], akr = A[k][r];
                    A[k][p] = c * akp - s * akr;
                    A[k][r] = s * akp + c * akr;
                }
                for (int k = 0; k < 4; ++k) {
                    const double apk = A[p][k], ark = A[r][k];
                    A[p][k] = c * apk - s * ark;
                    A[r][k] = s * apk + c * ark;
                }
                for (int k = 0; k < 4; ++k) {
                    const double vkp = V[k][p], vkr = V[k][r];
                    V[k][p] = c * vkp - s * vkr;
                    V[k][r] = s * vkp + c * vkr;
                }
            }
    }
    // column of the largest eigenvalue (register selects, no dynamic indexing)
    double lam = A[0][0], v[4] = {V[0][0], V[1][0], V[2][0], V[3][0]};
#pragma unroll
    for (int c = 1; c < 4; ++c)
        if (A[c][c] > lam) {
            lam = A[c][c];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = V[i][c];
        }
    const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
    const double sgn = (v[0] / nrm > 0.0) ? 1.0 : -1.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = (float)(sgn * v[i] / nrm);
}

// Does candidate (b, j) come before (a, i) in torch.sort(descending=True) order? NaN sorts as the
// largest value (torch's comparator), equal keys (NaN with NaN too) keep the lower index first.
__device__ __forceinline__ bool precedes(float b, int j, float a, int i) {
    const bool an = a != a, bn = b != b;
    if (an || bn) return bn && (!an || j < i);
    return b > a || (b == a && j < i);
}

struct AggSmem {
    int rank_rot[AGG_MAXK];
    int rank_tr[AGG_MAXK];
    int ord_rot[AGG_MAXKEEP];
    int ord_tr[AGG_MAXKEEP];
    float q[AGG_MAXKEEP][4];
    float qo[AGG_MAXKEEP][4];   // w-oriented copies
    float D[AGG_MAXKEEP][AGG_MAXKEEP + 1];
    unsigned char adj[AGG_MAXKEEP][AGG_MAXKEEP];   // |D_i - D_j|_2 <= eps
    int ncount[AGG_MAXKEEP];
    int label[AGG_MAXKEEP];
    int stack[AGG_MAXKEEP];
    float qavg[4];
};

__global__ __launch_bounds__(AGG_THREADS) void rank_aggregate_kernel(
    const float* __restrict__ poses, const float* __restrict__ energy, int K, int keep, int clustering,
    float eps, int min_samples, float* __restrict__ agg, float* __restrict__ sorted_pose,
    float* __restrict__ sorted_energy) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    AggSmem& sm = *reinterpret_cast<AggSmem*>(smem_raw);
    const int b = blockIdx.x, tid = threadIdx.x;
    const float* P = poses + (size_t)b * K * 9;
    const float* E = energy + (size_t)b * K * 2;
    // ---- 1. descending ranks, ties by lower index (stable); a total order, so the ranks are a
    //         permutation whatever the energies hold (precedes(): NaN first, as torch.sort orders it)
    for (int i = tid; i < K; i += AGG_THREADS) {
        const float er = E[2 * i], et = E[2 * i + 1];
        int rr = 0, rt = 0;
        for (int j = 0; j < K; ++j) {
            rr += precedes(E[2 * j], j, er, i);
            rt += precedes(E[2 * j + 1], j, et, i);
        }
        sm.rank_rot[i] = rr;
        sm.rank_tr[i] = rt;
    }
    __syncthreads();
    for (int i = tid; i < K; i += AGG_THREADS) {
        if (sm.rank_rot[i] < keep) sm.ord_rot[sm.rank_rot[i]] = i;
        if (sm.rank_tr[i] < keep) sm.ord_tr[sm.rank_tr[i]] = i;
        if (sorted_pose) {  // sorted_poses: rotation part by rotation rank, translation by translation rank
            float* o = sorted_pose + ((size_t)b * K + sm.rank_rot[i]) * 9;
            for (int c = 0; c < 6; ++c) o[c] = P[9 * i + c];
            float* ot = sorted_pose + ((size_t)b * K + sm.rank_tr[i]) * 9;
            for (int c = 6; c < 9; ++c) ot[c] = P[9 * i + c];
        }
        if (sorted_energy) {
            sorted_energy[((size_t)b * K + sm.rank_rot[i]) * 2 + 0] = E[2 * i];
            sorted_energy[((size_t)b * K + sm.rank_tr[i]) * 2 + 1] = E[2 * i + 1];
        }
    }
    __syncthreads();
    // ---- 2./3. quaternions of the kept rotations
    for (int r = tid; r < keep; r += AGG_THREADS) {
        float v[6];
        for (int c = 0; c < 6; ++c) v[c] = P[9 * sm.ord_rot[r] + c];
        float q[4];
        rot6_to_quat(v, q);
        const float sg = q[0] > 0.f ? 1.f : -1.f;   // ((Q[..., 0:1] > 0).float() - 0.5) * 2
        for (int c = 0; c < 4; ++c) {
            sm.q[r][c] = q[c];
            sm.qo[r][c] = sg * q[c];
        }
    }
    __syncthreads();
    if (tid == 0) {
        // average_quaternion_batch with uniform weights: A = sum_r w qo qo^T / sum w
        const float w = 1.0f / (float)keep;
        float wsum = 0.f;
        for (int r = 0; r < keep; ++r) wsum += w;
        double A[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                float acc = 0.f;
                for (int r = 0; r < keep; ++r) acc += (sm.qo[r][i] * sm.qo[r][j]) * w;
                A[i][j] = (double)(acc / wsum);
            }
        top_eigvec4(A, sm.qavg);
    }
    // ---- 4. DBSCAN over rows of D = 1 - <qi, qj>^2
    if (clustering) {
        for (int e = tid; e < keep * keep; e += AGG_THREADS) {
            const int i = e / keep, j = e - i * keep;
            const float dot = ((sm.q[i][0] * sm.q[j][0] + sm.q[i][1] * sm.q[j][1]) + sm.q[i][2] * sm.q[j][2]) +
                              sm.q[i][3] * sm.q[j][3];
            sm.D[i][j] = 1.f - dot * dot;
        }
        __syncthreads();
        for (int e = tid; e < keep * keep; e += AGG_THREADS) {
            const int i = e / keep, j = e - i * keep;
            double d2 = 0.0;
            for (int c = 0; c < keep; ++c) {
                const double df = (double)sm.D[i][c] - (double)sm.D[j][c];
                d2 += df * df;
            }
            sm.adj[i][j] = sqrt(d2) <= (double)eps;
        }
        __syncthreads();
        for (int i = tid; i < keep; i += AGG_THREADS) {
            int cnt = 0;
            for (int j = 0; j < keep; ++j) cnt += sm.adj[i][j];
            sm.ncount[i] = cnt;
            sm.label[i] = -1;
        }
        __syncthreads();
        if (tid == 0) {
            // -1 unvisited, -2 queued; membership does not depend on the expansion order
            int nlab = 0;
            for (int i = 0; i < keep; ++i) {
                if (sm.label[i] != -1 || sm.ncount[i] < min_samples) continue;
                int top = 0;
                sm.stack[top++] = i;
                sm.label[i] = -2;
                while (top > 0) {
                    const int p = sm.stack[--top];
                    sm.label[p] = nlab;
                    if (sm.ncount[p] < min_samples) continue;   // border point: not expanded
                    for (int j = 0; j < keep; ++j)
                        if (sm.label[j] == -1 && sm.adj[p][j]) {
                            sm.label[j] = -2;
                            sm.stack[top++] = j;
                        }
                }
                ++nlab;
            }
            if (nlab > 0) {
                int best = 0, bestc = -1;
                for (int l = 0; l < nlab; ++l) {
                    int c = 0;
                    for (int i = 0; i < keep; ++i) c += sm.label[i] == l;
                    if (c > bestc) { bestc = c; best = l; }
                }
                const float w = 1.0f / (float)bestc;
                float wsum = 0.f;
                for (int r = 0; r < bestc; ++r) wsum += w;
                double A[4][4];
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j) {
                        float acc = 0.f;
                        for (int r = 0; r < keep; ++r)
                            if (sm.label[r] == best) acc += (sm.qo[r][i] * sm.qo[r][j]) * w;
                        A[i][j] = (double)(acc / wsum);
                    }
                top_eigvec4(A, sm.qavg);
            }
        }
    }
    __syncthreads();
    // ---- 5. 4x4 [R t; 0 1]
    if (tid < 16) {
        const int r = tid >> 2, c = tid & 3;
        float v;
        if (r == 3) {
            v = c == 3 ? 1.f : 0.f;
        } else if (c == 3) {
            float acc = 0.f;
            for (int k = 0; k < keep; ++k) acc += P[9 * sm.ord_tr[k] + 6 + r];
            v = acc / (float)keep;
        } else {  // quaternion_to_matrix (rotation_conversions.py:41-70)
            const float qr = sm.qavg[0], qi = sm.qavg[1], qj = sm.qavg[2], qk = sm.qavg[3];
            const float two_s = 2.0f / (((qr * qr + qi * qi) + qj * qj) + qk * qk);
            const float m[9] = {1 - two_s * (qj * qj + qk * qk), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr),
                                two_s * (qi * qj + qk * qr), 1 - two_s * (qi * qi + qk * qk), two_s * (qj * qk - qi * qr),
                                two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi * qi + qj * qj)};
            v = 0.f;
#pragma unroll
            for (int e = 0; e < 9; ++e)
                if (e == r * 3 + c) v = m[e];
        }
        agg[(size_t)b * 16 + tid] = v;
    }
}

extern "C" int gp_rank_aggregate(const float* poses, const float* energy, int b, int k, int retain, int clustering,
                                 float eps, int min_samples, float* aggregated, float* sorted_pose,
                                 float* sorted_energy, hipStream_t stream) {
    GP_REQUIRE(b == 0 || (poses && energy && aggregated), "rank_aggregate: null pointer");
    GP_REQUIRE(b >= 0 && k >= 1 && k <= AGG_MAXK, "rank_aggregate: need 1 <= k <= %d (k=%d)", AGG_MAXK, k);
    GP_REQUIRE(retain >= 1 && retain <= k && retain <= AGG_MAXKEEP, "rank_aggregate: need 1 <= retain <= min(k, %d)",
               AGG_MAXKEEP);
    GP_REQUIRE(!clustering || min_samples >= 1, "rank_aggregate: DBSCAN needs min_samples >= 1");
    if (!b) return GP_OK;
    const size_t lds = sizeof(AggSmem);
    if (lds > 160 * 1024) {
        gp_set_error("rank_aggregate: LDS %zu", lds);
        return GP_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(rank_aggregate_kernel, dim3(b), dim3(AGG_THREADS), lds, stream, poses, energy, k, retain,
                       clustering, eps, min_samples, aggregated, sorted_pose, sorted_energy);
    return gp_check_launch("rank_aggregate_kernel");
}

// ============================================================================ stage glue
// process_batch's pts_center (datasets_omni6dpose.py:746-752: zero_mean = mean(pts[:, :, :3], 1)).
// One workgroup per object; per-thread strided sums over points, then a fixed-order tree.
__global__ __launch_bounds__(256) void points_mean_kernel(const float* __restrict__ pts, int n, int c,
                                                          float* __restrict__ out) {
    __shared__ float red[3][256];
    const int b = blockIdx.x, tid = threadIdx.x;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    const float* p = pts + (size_t)b * n * c;
    for (int i = tid; i < n; i += 256) {
        s0 += ld1(p + (size_t)i * c + 0);
        s1 += ld1(p + (size_t)i * c + 1);
        s2 += ld1(p + (size_t)i * c + 2);
    }
    red[0][tid] = s0;
    red[1][tid] = s1;
    red[2][tid] = s2;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            red[0][tid] += red[0][tid + st];
            red[1][tid] += red[1][tid + st];
            red[2][tid] += red[2][tid + st];
        }
        __syncthreads();
    }
    if (tid < 3) out[(size_t)b * 3 + tid] = fdiv(red[tid][0], (float)n);
}

extern "C" int gp_points_mean(const float* pts, int b, int n, int c, float* out, hipStream_t stream) {
    GP_REQUIRE(b >= 0 && n >= 1 && c >= 3 && (b == 0 || (pts && out)), "points_mean: bad arguments");
    if (!b) return GP_OK;
    hipLaunchKernelGGL(points_mean_kernel, dim3(b), dim3(256), 0, stream, pts, n, c, out);
    return gp_check_launch("points_mean_kernel");
}

// inference_scale without a ScaleNet checkpoint (evaluation_single.py:233-252): the points in the
// aggregated object frame, q = R^T (p - t), and length = 2 max_n |q| per axis. Max is
// order-independent, so the result depends only on the per-point arithmetic.
__global__ __launch_bounds__(256) void bbox_length_kernel(const float* __restrict__ pcl, int n, int c,
                                                          const float* __restrict__ pose, float* __restrict__ out) {
#pragma clang fp contract(off)
    __shared__ float red[3][256];
    const int b = blockIdx.x, tid = threadIdx.x;
    const float* P = pose + (size_t)b * 16;
    const float r00 = P[0], r01 = P[1], r02 = P[2], t0 = P[3];
    const float r10 = P[4], r11 = P[5], r12 = P[6], t1 = P[7];
    const float r20 = P[8], r21 = P[9], r22 = P[10], t2 = P[11];
    float m0 = 0.f, m1 = 0.f, m2 = 0.f;
    const float* p = pcl + (size_t)b * n * c;
    for (int i = tid; i < n; i += 256) {
        const float d0 = ld1(p + (size_t)i * c) - t0, d1 = ld1(p + (size_t)i * c + 1) - t1, d2 = ld1(p + (size_t)i * c + 2) - t2;
        // bmm(R^T, d): row j of R^T is column j of R
        m0 = fmaxf(m0, fabsf((r00 * d0 + r10 * d1) + r20 * d2));
        m1 = fmaxf(m1, fabsf((r01 * d0 + r11 * d1) + r21 * d2));
        m2 = fmaxf(m2, fabsf((r02 * d0 + r12 * d1) + r22 * d2));
    }
    red[0][tid] = m0;
    red[1][tid] = m1;
    red[2][tid] = m2;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            red[0][tid] = fmaxf(red[0][tid], red[0][tid + st]);
            red[1][tid] = fmaxf(red[1][tid], red[1][tid + st]);
            red[2][tid] = fmaxf(red[2][tid], red[2][tid + st]);
        }
        __syncthreads();
    }
    if (tid < 3) out[(size_t)b * 3 + tid] = red[tid][0] * 2.0f;
}

extern "C" int gp_bbox_length(const float* pcl, int b, int n, int c, const float* pose, float* length,
                              hipStream_t stream) {
    GP_REQUIRE(b >= 0 && n >= 1 && c >= 3 && (b == 0 || (pcl && pose && length)), "bbox_length: bad arguments");
    if (!b) return GP_OK;
    hipLaunchKernelGGL(bbox_length_kernel, dim3(b), dim3(256), 0, stream, pcl, n, c, pose, length);
    return gp_check_launch("bbox_length_kernel");
}
