/*
 * ORACLE — test infrastructure only. Never linked into the product path.
 *
 * Plain-C restatement of the reference's PointNet++ CUDA point ops, serialised thread by
 * thread so that tie rules and comparison semantics are reproduced exactly:
 *
 *   fps          <- networks/pts_encoder/pointnet2_utils/pointnet2/src/sampling_gpu.cu:86-209
 *                   (+ launcher :211-253, opt_n_threads cuda_utils.h:9-13, temp=1e10
 *                    pointnet2_utils.py:32-34)
 *   ball_query   <- src/ball_query_gpu.cu:9-45 (idx zero-initialised, pointnet2_utils.py:246)
 *
 * Distances are evaluated as separately rounded fp32 operations in the reference's textual
 * order ((dx*dx + dy*dy) + dz*dz); build with -ffp-contract=off (see oracle/Makefile).
 * The reference has no CPU implementation of these ops and its CUDA sources
 * cannot be built here, so this restatement is pinned by hand-computed known-answer tests
 * (tests/test_oracle_pointops.py) rather than by reference outputs.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

static int opt_n_threads(int work_size) {
    const int pow_2 = (int)(log((double)work_size) / log(2.0));
    int v = 1 << pow_2;
    if (v > 1024) v = 1024;
    if (v < 1) v = 1;
    return v;
}

int oracle_fps_block_size(int n) { return opt_n_threads(n); }

/* xyz (B,N,3) fp32, idx (B,M) int32 */
void oracle_fps(const float *xyz, int b, int n, int m, int *idx) {
    if (m <= 0) return;
    const int bs = opt_n_threads(n);
    float *temp = (float *)malloc(sizeof(float) * (size_t)n);
    float *dists = (float *)malloc(sizeof(float) * (size_t)bs);
    int *dists_i = (int *)malloc(sizeof(int) * (size_t)bs);
    for (int bi = 0; bi < b; ++bi) {
        const float *ds = xyz + (size_t)bi * n * 3;
        int *out = idx + (size_t)bi * m;
        for (int k = 0; k < n; ++k) temp[k] = 1e10f;
        int old = 0;
        out[0] = old;
        for (int j = 1; j < m; ++j) {
            const float x1 = ds[old * 3 + 0], y1 = ds[old * 3 + 1], z1 = ds[old * 3 + 2];
            for (int tid = 0; tid < bs; ++tid) {
                int besti = 0;
                float best = -1.f;
                for (int k = tid; k < n; k += bs) {
                    const float x2 = ds[k * 3 + 0], y2 = ds[k * 3 + 1], z2 = ds[k * 3 + 2];
                    const float dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
                    const float d = dx * dx + dy * dy + dz * dz;
                    const float d2 = d < temp[k] ? d : temp[k];
                    temp[k] = d2;
                    besti = d2 > best ? k : besti;
                    best = d2 > best ? d2 : best;
                }
                dists[tid] = best;
                dists_i[tid] = besti;
            }
            /* shared-memory tree: slot t keeps slot t+h unless v2 > v1 (sampling_gpu.cu:86-91) */
            for (int h = bs / 2; h >= 1; h /= 2) {
                for (int t = 0; t < h; ++t) {
                    const float v1 = dists[t], v2 = dists[t + h];
                    const int i1 = dists_i[t], i2 = dists_i[t + h];
                    dists[t] = v1 > v2 ? v1 : v2;
                    dists_i[t] = v2 > v1 ? i2 : i1;
                }
            }
            old = dists_i[0];
            out[j] = old;
        }
    }
    free(temp);
    free(dists);
    free(dists_i);
}

/* new_xyz (B,M,3), xyz (B,N,3), idx (B,M,nsample) int32, caller zero-initialised */
void oracle_ball_query(int b, int n, int m, float radius, int nsample, const float *new_xyz,
                       const float *xyz, int *idx) {
    const float radius2 = radius * radius;
    for (int bi = 0; bi < b; ++bi) {
        for (int p = 0; p < m; ++p) {
            const float *c = new_xyz + ((size_t)bi * m + p) * 3;
            const float *pts = xyz + (size_t)bi * n * 3;
            int *o = idx + ((size_t)bi * m + p) * nsample;
            const float nx = c[0], ny = c[1], nz = c[2];
            int cnt = 0;
            for (int k = 0; k < n; ++k) {
                const float dx = nx - pts[k * 3 + 0], dy = ny - pts[k * 3 + 1],
                            dz = nz - pts[k * 3 + 2];
                const float d2 = dx * dx + dy * dy + dz * dz;
                if (d2 < radius2) {
                    if (cnt == 0)
                        for (int l = 0; l < nsample; ++l) o[l] = k;
                    o[cnt] = k;
                    ++cnt;
                    if (cnt >= nsample) break;
                }
            }
        }
    }
}
