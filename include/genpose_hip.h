/*
 * genpose_hip.h -- C ABI of libgenpose_hip.so, the MI355X (gfx950) implementation of the
 * GenPose++ pose-candidate path.
 *
 * Conventions (replacing the reference's pybind module `pointnet2_cuda`,
 * networks/pts_encoder/pointnet2_utils/pointnet2/src/pointnet2_api.cpp:10-24):
 *   - every pointer argument is caller-owned DEVICE memory unless marked "host";
 *     the library never allocates inside a call (workspaces are sized by *_workspace_size);
 *   - every call is enqueued on `stream` and returns immediately (no device sync);
 *   - every call returns 0 (GP_OK) or a negative status; gp_last_error() (thread-local)
 *     describes the failure. Nothing calls exit() (the reference launchers do, e.g.
 *     src/ball_query_gpu.cu:61-65);
 *   - calls are stateless and re-entrant across distinct streams.
 * Layouts are row-major; "packed" weights are produced by genpose2_amd/pack.py.
 */
#ifndef GENPOSE_HIP_H
#define GENPOSE_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GP_OK = 0, GP_ERR_INVALID = -1, GP_ERR_LAUNCH = -2, GP_ERR_UNSUPPORTED = -3 };

/* Thread-local description of the last failure (empty string if none). */
const char *gp_last_error(void);
/* ABI version of this header. */
int gp_abi_version(void);
#define GP_ABI_VERSION 7

/* ===================================================================== operator level
 * Drop-in forward ops of `pointnet2_cuda` (same argument meaning and layouts). */

/* furthest_point_sampling_wrapper(b, n, m, points, temp, idx)  src/sampling.cpp / sampling_gpu.cu:94-253
 * xyz (b,n,3) fp32, idx (b,m) int32. `temp` (b,n) is accepted for signature parity and may be
 * NULL: the kernel keeps the running min-distance on chip. Tie rule identical to the reference
 * (strict > within a thread, lower reduction slot on ties, block size min(2^floor(log2 n),1024)). */
int gp_furthest_point_sampling(int b, int n, int m, const float *xyz, float *temp, int *idx,
                               hipStream_t stream);

/* gather_points_wrapper(b, c, n, npoints, points, idx, out)  src/sampling_gpu.cu:8-44
 * points (b,c,n), idx (b,npoints) int32 -> out (b,c,npoints). */
int gp_gather_points(int b, int c, int n, int npoints, const float *points, const int *idx,
                     float *out, hipStream_t stream);

/* ball_query_wrapper(b, n, m, radius, nsample, new_xyz, xyz, idx)  src/ball_query_gpu.cu:9-66
 * new_xyz (b,m,3), xyz (b,n,3) -> idx (b,m,nsample) int32: first nsample points with
 * d^2 < radius^2 in index order, padded with the first hit, 0 when there is no hit. */
int gp_ball_query(int b, int n, int m, float radius, int nsample, const float *new_xyz,
                  const float *xyz, int *idx, hipStream_t stream);

/* group_points_wrapper(b, c, n, npoints, nsample, points, idx, out)  src/group_points_gpu.cu:47-85
 * points (b,c,n), idx (b,npoints,nsample) -> out (b,c,npoints,nsample). */
int gp_group_points(int b, int c, int n, int npoints, int nsample, const float *points,
                    const int *idx, float *out, hipStream_t stream);

/* ===================================================================== fused encoder
 * Pointnet2ClsMSG(0) with the Light config (networks/pts_encoder/pointnet2.py:211-252).
 * `wbuf` holds all packed, BN-folded layers; `layer_off` (HOST, int64 [5][2][3][4]) gives, for
 * layer i of branch b of level l, {float offset of the fp32 A fragments, float offset of the bias
 * (padded to 32), float offset of the split-f16 hi/lo planes or -1, their power-of-two exponent}
 * (-1 = absent). Levels 2-3 run as split-f16 MFMA (per-column activation scaling) when all four of
 * their layer-1/2 plane offsets are given, exact fp32 MFMA otherwise. ABI 5: the [..][4] table;
 * a [5][2][3][2] table of ABI <= 3 is no longer accepted. The exponents are weight-derived state: a
 * host that receives the weights from another rank must receive this table too. */
size_t gp_encoder_workspace_size(int b, int n);
/* HOST out: byte offsets in the workspace of, per level l<4: fps idx (b,M_l) int32,
 * new_xyz (b,M_l,3) fp32, ball idx branch0/1 (b,M_l,ns) int32; and per level l<5 the level
 * features (b,M_l,C_l) point-major fp32.  offsets[l*5 + {0..4}] = {fps, new_xyz, ball0, ball1, feat}. */
int gp_encoder_workspace_layout(int b, int n, int64_t *offsets);
/* pts (b,n,3) un-centred points -> feat (b,1024). */
int gp_encoder_forward(const float *wbuf, const int64_t *layer_off, const float *pts, int b, int n,
                       void *workspace, size_t workspace_bytes, float *feat, hipStream_t stream);
/* Two models over the same points (the ScoreNet and EnergyNet encoders of one batch) share the geometry
 * -- FPS indices, centroids and ball lists depend only on the points. gp_encoder_geometry runs the FPS
 * chain of all four levels and the ball lists of every level into `workspace`; gp_encoder_forward_geom
 * is gp_encoder_forward with that geometry read from `geometry` (a workspace of the same (b, n) layout
 * that gp_encoder_geometry filled, possibly `workspace` itself) and only the per-level MLPs run, their
 * scratch in `workspace`. Same results as gp_encoder_forward, bit for bit. */
int gp_encoder_geometry(const float *pts, int b, int n, void *workspace, size_t workspace_bytes,
                        hipStream_t stream);
int gp_encoder_forward_geom(const float *wbuf, const int64_t *layer_off, const float *pts, int b, int n,
                            const void *geometry, void *workspace, size_t workspace_bytes, float *feat,
                            hipStream_t stream);
/* The same two calls over a range of levels, so that level 0's MLPs can start while the FPS chain and ball
 * lists of levels 1-3 are still being computed (on another stream): gp_encoder_geometry_levels fills the
 * geometry of levels [first, last) (first > 0 reads level first-1's centroids from the workspace);
 * gp_encoder_forward_geom_levels runs SA levels [first, last) of 5 (level l reads level l-1's features from
 * `workspace`; level 4 writes `feat`). geometry_levels(0, 4) == gp_encoder_geometry and
 * forward_geom_levels(0, 5) == gp_encoder_forward_geom; any split gives the same bits. */
int gp_encoder_geometry_levels(const float *pts, int b, int n, void *workspace, size_t workspace_bytes,
                               int first, int last, hipStream_t stream);
int gp_encoder_forward_geom_levels(const float *wbuf, const int64_t *layer_off, const float *pts, int b, int n,
                                   const void *geometry, void *workspace, size_t workspace_bytes, float *feat,
                                   int first, int last, hipStream_t stream);
/* Level-by-level form (the fused encoders, whose levels take features computed between levels):
 * gp_encoder_fps runs the FPS chain of all four levels into the workspace (fps idx + new_xyz, as
 * gp_encoder_workspace_layout places them); gp_sa_level then runs SA level `level`
 * (PointnetSAModuleMSG.forward, pointnet2_modules.py:19-124: ball query of both radii, group, the
 * BN-folded SharedMLPs, max-pool) on its input features feat_prev (b, n_prev, c_prev) point-major
 * (NULL with c_prev = 0 at level 0) -> out (b, M_level, C_level) point-major (level 4: (b, 1024)).
 * c_prev: level 0 any multiple of 16 (Pointnet2ClsMSGFus: 384, pointnet2.py:281-285), level l > 0
 * the previous level's channels. `wbuf`/`layer_off` as gp_encoder_forward, packed for those widths. */
int gp_encoder_fps(const float *pts, int b, int n, void *workspace, size_t workspace_bytes,
                   hipStream_t stream);
int gp_sa_level(const float *wbuf, const int64_t *layer_off, int level, int c_prev, const float *pts,
                int b, int n, const float *feat_prev, void *workspace, size_t workspace_bytes,
                float *out, hipStream_t stream);
/* gp_sa_level over geometry that gp_encoder_geometry left in `geometry` (a workspace of the same (b, n) layout,
 * possibly `workspace` itself): no ball query; the level's scratch goes to `workspace`. The ScoreNet and
 * EnergyNet fused encoders of one batch share one geometry pass this way. Same bits as gp_sa_level. */
int gp_sa_level_geom(const float *wbuf, const int64_t *layer_off, int level, int c_prev, const float *pts,
                     int b, int n, const float *feat_prev, const void *geometry, void *workspace,
                     size_t workspace_bytes, float *out, hipStream_t stream);

/* ===================================================================== fused-encoder blocks
 * The DINO-pointwise encoder Pointnet2ClsMSGFus (pointnet2.py:255-388) between SA levels:
 * TransformerBlockWithRelativePE (attention.py:491-533) with the EfficientRelativePositionalEncoding
 * bias (attention.py:648-735), and GatedAttentionFusion (attention.py:224-325). Token tensors are
 * point-major (b, n, C) fp32, i.e. the reference's (b, C, n) transposed. */
/* y[r, :] = act(x[r, :k] . w^T + bias), r < m; w (n, k) row-major (nn.Linear / Conv1d k=1 layout),
 * k and n multiples of 16; ldx / ldy = row strides of x / y (>= k / n). act: 0 none, 1 ReLU,
 * 2 sigmoid. Exact fp32 MFMA (v_mfma_f32_16x16x4_f32). */
int gp_linear(const float *x, int ldx, int m, int k, const float *w, const float *bias, int n,
              int act, float *y, int ldy, hipStream_t stream);
/* The same linear in split-f16 arithmetic (three v_mfma_f32_16x16x32_f16 products of hi / lo f16
 * planes, fp32 accumulation; x scaled per row by a power of two from its max |x|). wpk: int32 words
 * [e, 0, 0, 0] + the planes of W * 2^e, rows zero-padded to a multiple of 128, in
 * genpose2_amd/fus_encoder.py pack_split_linear's layout (gp_linear_split_words(n, k) words).
 * k % 32 == 0, n % 16 == 0. rmax: m floats, x's row maxima max_k |x| -- computed here, or given
 * by the caller with flags |= GP_LINEAR_RMAX_GIVEN (e.g. the ymax of the linear that produced x).
 * ymax: NULL, or m floats that receive max |y| per row. act 3 is GatedAttentionFusion's gate with its
 * mix (attention.py:316-320): x = [cur | att] (k = 2n), y = g * cur + (1 - g) * att with
 * g = sigmoid(x W^T + b). */
#define GP_LINEAR_RMAX_GIVEN 1
size_t gp_linear_split_words(int n, int k);
int gp_linear_split(const float *x, int ldx, int m, int k, const int32_t *wpk, const float *bias, int n,
                    int act, float *y, int ldy, float *rmax, int flags, float *ymax, hipStream_t stream);
/* y = LayerNorm(x + r) over the last dim d (gamma, beta, eps; d % 4 == 0), m rows; y may alias x.
 * ymax: NULL, or m floats that receive max |y| per row. */
int gp_add_layernorm(const float *x, const float *r, int m, int d, const float *gamma,
                     const float *beta, float eps, float *y, float *ymax, hipStream_t stream);
/* Relative-PE bias of EfficientRelativePositionalEncoding (8 heads): xyz (b, n, 3) ->
 * bias (b, 8, n, n) = the reference's relative_bias[b, h, i, j] (query i, key j,
 * rel = xyz[j] - xyz[i]). pe (host-packed, 1024 floats):
 * [0:16) dist.0.w, [16:32) dist.0.b, [32:160) dist.2.w (8x16), [160:168) dist.2.b,
 * [168:216) dir.0.w (16x3), [216:232) dir.0.b, [232:360) dir.2.w, [360:368) dir.2.b,
 * [368:496) fusion.w (8x16), [496:504) fusion.b; then the fusion layer composed with the second
 * layers: [512:640) A[h][u] = (fusion.w[:, :8] dist.2.w)[h][u], [640:768) B[h][u] likewise with
 * dir.2.w, [768:776) c = fusion.w [dist.2.b; dir.2.b] + fusion.b, [776:824) dir.0.w as [axis][u]. */
size_t gp_relpe_bias_bytes(int b, int n);
int gp_relpe_bias(const float *pe, const float *xyz, int b, int n, float *bias, hipStream_t stream);
/* Multi-head attention with an additive bias (MultiheadAttentionWithRelativePE core,
 * attention.py:436-488, eval): qkv (b, n, 3d) rows [q | k | v] (heads of d/8 channels),
 * bias (b, 8, n, n) [b][h][query][key] as gp_relpe_bias writes it, or NULL ->
 * out (b, n, d) = softmax(q k^T / sqrt(d/8) + bias) v per head. ymax: NULL, or b * n floats that
 * receive max |out| per token. */
int gp_mha_attention(const float *qkv, const float *bias, int b, int n, int d, float *out,
                     float *ymax, hipStream_t stream);
/* gp_relpe_bias + gp_mha_attention in one kernel, the bias evaluated per (query, key) pair in registers
 * (no (b, 8, n, n) buffer): qkv as gp_mha_attention, xyz (b, n, 3), pe as gp_relpe_bias. Head dims
 * d / 8 <= 32 (the fused encoder's levels 0 and 1). ymax: NULL or b * n floats (max |out| per token). */
int gp_mha_relpe_attention(const float *qkv, const float *xyz, const float *pe, int b, int n, int d,
                           float *out, float *ymax, hipStream_t stream);
/* F.interpolate(mode="linear", align_corners=False) along the point index: x (b, n_in, c) ->
 * y (b, n_out, c) (pointnet2.py:344-350); c % 4 == 0. ymax: NULL, or b * n_out floats (max |y| per row). */
int gp_interp_points(const float *x, int b, int n_in, int c, int n_out, float *y, float *ymax,
                     hipStream_t stream);
/* GatedAttentionFusion's attention stage (attention.py:298-313) per object: cur (b, n, c), ot (b, n, c)
 * (original_transform output) -> gcat (b, n, 2c) = [cur | ot * ca * sp] with ca = channel attention
 * of mean_n [cur | ot] (ca1: (2c/4, 2c) + bias, ReLU, ca3: (c, 2c/4) + bias, sigmoid) and sp =
 * sigmoid(conv1d_7([max_c cur ; mean_c cur])) (sp_w: (2, 7), zero padding 3). c % 32 == 0.
 * ws: gp_fusion_attend_workspace_size(b, n, c) bytes of device scratch (the per-object statistics).
 * gmax: NULL, or b * n floats that receive max |gcat| per token. */
size_t gp_fusion_attend_workspace_size(int b, int n, int c);
int gp_fusion_attend(const float *cur, const float *ot, int b, int n, int c, const float *ca1_w,
                     const float *ca1_b, const float *ca3_w, const float *ca3_b, const float *sp_w,
                     float *gcat, float *gmax, void *ws, size_t ws_bytes, hipStream_t stream);
/* fused = g * cur + (1 - g) * att with cur = gcat[:, :c], att = gcat[:, c:] (attention.py:318-320):
 * g (rows, c), gcat (rows, 2c) -> out (rows, c). */
int gp_fusion_mix(const float *g, const float *gcat, int rows, int c, float *out, hipStream_t stream);

/* ===================================================================== score / energy heads
 * PoseScoreNet / PoseEnergyNet with Rx_Ry_and_T heads (scorenet.py:109-275, energynet.py:32-208),
 * split into per-object (pts), per-step (t) and per-candidate (pose) column blocks of the first
 * head layer. All "packed" tensors come from genpose2_amd/pack.py. */
typedef struct {
    const float *pe0_w; /* pose_encoder.0: packed 256x16 */
    const float *pe0_b; /* 256 */
    const float *pe2_w; /* pose_encoder.2: packed 256x256 */
    const float *pe2_b; /* 256 */
    const float *h1p_w; /* head layer 1, pose columns: packed 768x256 */
    const float *h2_w;  /* head layer 2: [3 heads][3][256] */
    const float *h2_b;  /* [9] */
    const float *h1pts_t; /* head layer 1, pts columns, transposed (1024, 768) */
    const float *h1_b;    /* head layer 1 bias (768) */
    const float *gfp_w;   /* t_encoder.0.W (64) */
    const float *te_w_t;  /* t_encoder.1.weight transposed (128,128) */
    const float *te_b;    /* (128) */
    const float *h1t_t;   /* head layer 1, t columns, transposed (128, 768) */
    /* f16x3 form of pe2_w / h1p_w (pack.py pack_h16_fragments(w, e, 3), ABI 7): three f16 planes
     * hi, mid, lo of W * 2^e (6 bytes per weight). hsc = {A0, B0, A2, B2, e_pe2, e_h1p, 0, 0}: max row
     * L1 norm and max |bias| of pose_encoder.0 / .2 (activation bounds) and the two weight exponents.
     * Used by every per-candidate head kernel (PC step, score/energy eval, ODE stages): six f16 MFMA
     * products per 32-deep chunk over three planes of each operand, fp32 accumulation. All three NULL:
     * those GEMMs run in exact fp32 MFMA instead. */
    const void *pe2_h;
    const void *h1p_h;
    const float *hsc;
} gp_head_weights;

/* Per-object projection P[b] = W1_pts . pts_feat[b] + b1 -> pobj (b,768). */
int gp_head_object_proj(const gp_head_weights *w, const float *pts_feat, int b, float *pobj,
                        hipStream_t stream);
/* Per-time projection tproj[k] = W1_t . relu(W_t . GFP(t_k) + b_t) for t (nt) -> (nt,768). */
int gp_head_time_proj(const gp_head_weights *w, const float *t, int nt, float *tproj,
                      hipStream_t stream);

/* Score evaluation s = heads(x, t) / (sigma + 1e-7) for R rows, rows r -> object r / k.
 * `tproj_row` (768) and `sigma` are those of the single time value of this call. */
int gp_score_eval(const gp_head_weights *w, const float *pobj, const float *tproj_row,
                  float sigma, const float *x, int rows, int k, float *score, hipStream_t stream);

/* Energy (IP / score / identical, decoupled rot-trans): pose rows (R,9) with translation
 * already relative to pts_center -> energy (R,2). t is a single value with its tproj row. */
int gp_energy_eval(const gp_head_weights *w, const float *pobj, const float *tproj_row,
                   float sigma, const float *pose, int rows, int k, float *energy,
                   hipStream_t stream);

/* ===================================================================== PC sampler
 * cond_pc_sampler (samplers.py:113-177) for R = b*k rows over T steps, fused per step:
 * [finish step i-1: Langevin corrector with the batch-mean score norm, renormalise,
 *  reverse-SDE Euler-Maruyama predictor, Gram-Schmidt] + [score at step i].
 * step_tab (HOST, T x 5 fp32): {t, sigma, g, dt, sqrt_dt} exactly as the reference forms them.
 * x (R,9) holds the initial state (prior sample or init_x) and is overwritten.
 * noise: z1/z2 (T,R,9) injected draws, or both NULL to use device Philox4x32 seeded by `seed`.
 * Outputs: res (R,9) = mean_x of the last step (+pts_center, GS), q (R,7) = [quat_wxyz, trans]
 * (posenet_agent.py:554-556), xs (R,T,9) trajectory or NULL. */
size_t gp_pc_workspace_size(int rows);
/* Candidates per PC-step workgroup gp_pc_sample uses for `rows` (split != 0: head weights carry the
 * f16x3 planes). For accounting only (the per-workgroup weight stream). */
int gp_pc_tile_rows(int rows, int split);
int gp_pc_sample(const gp_head_weights *w, const float *pobj, const float *tproj,
                 const float *step_tab, int steps, float *x, int rows, int k,
                 const float *pts_center, const float *z1, const float *z2, uint64_t seed,
                 float snr, float *res, float *q, float *xs, void *workspace,
                 size_t workspace_bytes, hipStream_t stream);

/* Global-batch PC sampling over shards (SURVEY 8e's optional mode; replaces nothing in the reference,
 * whose single cond_pc_sampler call (samplers.py:113-177) couples every row of the batch through the
 * Langevin grad_norm mean at :143-144). Each shard samples its contiguous block of rows
 * [row_off, row_off + rows) of a batch of rows_total rows with the tiling one call on rows_total rows
 * would use: its workgroups' partial sums of ||s_r|| go to entries [shard * per, shard * per + nwg) of
 * `part` (2 x gp_pc_global_partials(...) floats, zero-filled by the caller, per = that count / shards),
 * and after every scoring launch `exchange(ctx, step, slot, n, stream)` must make the slot's n entries
 * hold every shard's partials (an all-gather of `per`-entry chunks, enqueued on `stream`) before the
 * next launch reads them; grad_norm is their sum (in the fixed order) over rows_total, and the Philox
 * draws are keyed by the global row. With every shard but the last holding shard_rows_max rows, a
 * multiple of the tile (gp_pc_tile_rows(rows_total)), the result equals one gp_pc_sample call on the
 * whole batch bit for bit. exchange returns 0 on success. */
typedef int (*gp_pc_exchange_fn)(void *ctx, int step, float *slot, int n, hipStream_t stream);
int gp_pc_global_partials(int rows_total, int shard_rows_max, int shards, int split);
int gp_pc_sample_global(const gp_head_weights *w, const float *pobj, const float *tproj,
                        const float *step_tab, int steps, float *x, int rows, int k,
                        const float *pts_center, uint64_t seed, float snr, float *res, float *q,
                        float *xs, int rows_total, int row_off, int shard, int shards,
                        int shard_rows_max, float *part, gp_pc_exchange_fn exchange, void *ctx,
                        void *workspace, size_t workspace_bytes, hipStream_t stream);

/* The step table of cond_pc_sampler (samplers.py:129-130, sde.py:15-27) for hosts without Python:
 * out (HOST, steps x 5 fp32) = {t, sigma(t), g(t), dt, sqrt(dt)} with t = torch.linspace(1, eps,
 * steps) in float32 (bit-identical to torch's CPU rounding), sigma = f32(0.01) * 5000^t (power
 * correctly rounded; torch's Sleef pow is within 1 ulp of it, so sigma / g within 2 / 3 ulp of
 * sde.py's), g = sigma * f32(sqrt(2 ln 5000)), dt, sqrt(dt) (correctly rounded, torch's within 1 ulp).
 * Replaces genpose2_amd/sde.py pc_step_table; feeds gp_head_time_proj (column 0) and gp_pc_sample. */
int gp_pc_step_table(int steps, float eps, float *out);

/* Standard normals (Philox4x32-10 keyed by seed, counter {row, col/4, stream, 0x5EED}, Box-Muller)
 * -> out (rows, cols). The replacement of torch.randn_like in cond_pc_sampler (samplers.py:147,165):
 * gp_pc_sample with z1 = z2 = NULL draws step j's corrector / predictor noise as streams 2j / 2j+1
 * with cols = 9, identical to gp_randn(seed, 2j (+1), rows, 9, ...). */
int gp_randn(uint64_t seed, uint32_t stream, int rows, int cols, float *out, hipStream_t hs);

/* Quaternion / GS epilogue used by the ODE path: rows (R,9) fp64 -> in-place GS of [:6],
 * + pts_center on [6:], and q (R,7) fp64. */
int gp_pose_epilogue_f64(double *pose, int rows, int k, const float *pts_center, double *q,
                         hipStream_t stream);

/* ===================================================================== ODE sampler
 * cond_ode_sampler (samplers.py:180-258): the probability-flow ODE dx/dt = -0.5 g(t)^2 score
 * integrated by a Dormand-Prince 5(4) pair whose controller restates scipy solve_ivp RK45
 * (samplers.py:226-234; the controller's scalars run on the host, genpose2_amd/ode.py).
 * The state y, the stage derivatives K_0..K_6 and y_new are fp64 (R,9) device arrays; the score
 * model sees float(y) (samplers.py:210) at t32 = float(t) with sigma = sigma(t32) in fp32, and a
 * derivative is K = coef * double(score) with coef = -(0.5 g(t)^2) formed on the host.
 * Every call needs gp_ode_workspace_size(rows) bytes of workspace (time rows + error partials). */
size_t gp_ode_workspace_size(int rows);
/* One right-hand side: kout = coef * score(float(y + (sum_{j<nk} acoef[j] kin[j]) * h), t32).
 * kin (HOST array of nk device pointers) and acoef (HOST, nk) may be NULL when nk == 0. */
int gp_ode_rhs(const gp_head_weights *w, const float *pobj, float t32, float sigma, double coef,
               const double *y, const double *const *kin, const double *acoef, int nk, double h,
               int rows, int k, double *kout, void *workspace, size_t workspace_bytes,
               hipStream_t stream);
/* One attempted step (scipy rk.py rk_step + _estimate_error_norm): for s = 1..5
 * K_s = f(t_s, y + (sum_{j<s} A[s][j] K_j) h); y_new = y + (sum_{j<6} B_j K_j) h;
 * K_6 = f(t + h, y_new); err_out[0] = rms((sum_j E_j K_j) h / (atol + max(|y|,|y_new|) rtol)).
 * t32_6 / sigma_6 / coef_6 (HOST, 6 each): stage times 1..5 and t + h. kslots (HOST, 7 device
 * pointers) holds K_0 = f(t, y) on entry. tableau_a (HOST 6x6 row-major), b (HOST 6), e (HOST 7). */
int gp_ode_attempt(const gp_head_weights *w, const float *pobj, const float *t32_6,
                   const float *sigma_6, const double *coef_6, const double *y,
                   double *const *kslots, const double *tableau_a, const double *b, const double *e,
                   double h, double rtol, double atol, int rows, int k, double *ynew, double *err_out,
                   void *workspace, size_t workspace_bytes, hipStream_t stream);
/* select_initial_step norms (scipy _ivp/common.py) over n elements, scale = atol + |y0| rtol:
 * f1 == NULL -> out[0] = rms(y0/scale), out[1] = rms(f0/scale); else out[2] = rms((f1-f0)/scale). */
int gp_ode_init_norms(const double *y0, const double *f0, const double *f1, long long n,
                      double atol, double rtol, double *out, hipStream_t stream);
/* Dense output of an accepted step (scipy RkDenseOutput): for i in [i0, i1),
 * x = (t_eval[i] - t_old)/h, out[row] = h * (K^T P) cumprod([x,x,x,x]) + y_old with
 * row = reverse ? i_base - i : i - i_base. P7x4 (HOST 7x4), kslots (HOST, 7 device pointers). */
int gp_ode_dense(const double *const *kslots, const double *P7x4, const double *y_old,
                 const double *t_eval, int i0, int i1, int i_base, int reverse, double t_old,
                 double h, long long n, double *out, hipStream_t stream);
/* Device-controlled RK45 (the default pred_func path): the step controller itself runs on the
 * device. gp_ode_auto_attempt(n, what): what & 1 launches the control kernel of attempt n -- it
 * decides attempt n-1 from its error norm (scipy _step_impl accept/reject and step-size update)
 * and prepares attempt n (min_step check, h, t_new, the 6 stage times with their scalars and time
 * rows); what & 2 launches attempt n's 6 stage kernels, which return at once if no attempt was
 * prepared. State: two OdeCtl records (gp_ode_ctl_size() bytes each, layout mirrored in
 * genpose2_amd/ode.py) at the start of the workspace; attempt n reads record n & 1 and writes
 * record (n + 1) & 1 (the host writes record 0 after select_initial_step). The status field of a
 * record reads 0 running, 1 finished, -1 step size below the spacing of t. y0/y1: the two fp64
 * state buffers; kslots (HOST, 7 device pointers), tableau_a (HOST 6x6), b (HOST 6), e (HOST 7). */
size_t gp_ode_ctl_size(void);
size_t gp_ode_auto_workspace_size(int rows);
int gp_ode_auto_attempt(const gp_head_weights *w, const float *pobj, int n, int what,
                        double t_bound, double direction, double rtol, double atol,
                        double sig_min, double base, double diff_scale, double *y0, double *y1,
                        double *const *kslots, const double *tableau_a, const double *b,
                        const double *e, int rows, int k, void *workspace, size_t workspace_bytes,
                        hipStream_t stream);
/* gp_ode_auto_attempt whose control kernel also reports to the host without a copy: host_status (4 ints of
 * host memory the device can write, e.g. hipHostMalloc'd) word n & 3 becomes 4 n + (status + 1) once attempt n
 * is decided and prepared, so the host can keep attempts enqueued and poll, with no event or copy between a
 * control launch and its stage launch. */
int gp_ode_auto_attempt_hs(const gp_head_weights *w, const float *pobj, int n, int what,
                           double t_bound, double direction, double rtol, double atol,
                           double sig_min, double base, double diff_scale, double *y0, double *y1,
                           double *const *kslots, const double *tableau_a, const double *b,
                           const double *e, int rows, int k, void *workspace, size_t workspace_bytes,
                           int *host_status, hipStream_t stream);
/* Global-batch RK45 over shards (SURVEY 8e's optional mode for the ODE; replaces nothing in the reference,
 * whose single solve_ivp call (samplers.py:226-234) takes one error norm over the whole batch's state per
 * attempt). Each shard integrates its contiguous rows [row_off, row_off + rows) of rows_total with the
 * tiling of one call on rows_total rows: its workgroups' error partials go to entries
 * [shard * per, shard * per + nwg) of the workspace's gp_ode_global_partials(...) partials (per = that
 * count / shards), and after each attempt's stage launch `exchange(ctx, attempt, part, n, stream)` must
 * make all n entries hold every shard's partials (an all-gather of `per`-entry fp64 chunks enqueued on
 * `stream`) before the next control kernel sums them in the fixed order over rows_total * 9 elements.
 * Every rank then takes the same accept / reject decisions. The caller runs select_initial_step on the
 * WHOLE batch's y0, f0 and f1 (gp_ode_init_norms over all rows_total rows, e.g. after all-gathering the
 * shards' vectors). With every shard but the last holding shard_rows_max rows, a multiple of the tile, the
 * result equals one solve on the whole batch bit for bit. Workspace: gp_ode_global_workspace_size(n)
 * bytes; host_status as gp_ode_auto_attempt_hs, or NULL. */
typedef int (*gp_ode_exchange_fn)(void *ctx, int attempt, double *part, int n, hipStream_t stream);
int gp_ode_global_partials(int rows_total, int shard_rows_max, int shards, int split);
size_t gp_ode_global_workspace_size(int part_n);
/* Byte offset of the error partials (fp64) in a device-controlled workspace: a global-batch host zero-fills
 * the gp_ode_global_partials(...) entries there before the first attempt and all-gathers them in exchange. */
size_t gp_ode_auto_partials_offset(void);
int gp_ode_auto_attempt_global(const gp_head_weights *w, const float *pobj, int n, int what,
                               double t_bound, double direction, double rtol, double atol,
                               double sig_min, double base, double diff_scale, double *y0, double *y1,
                               double *const *kslots, const double *tableau_a, const double *b,
                               const double *e, int rows, int k, int rows_total, int row_off, int shard,
                               int shards, int shard_rows_max, gp_ode_exchange_fn exchange, void *ctx,
                               void *workspace, size_t workspace_bytes, int *host_status,
                               hipStream_t stream);
/* The whole ODE sampler in one call (cond_ode_sampler, samplers.py:180-258, with scipy solve_ivp
 * RK45, samplers.py:226-234) for hosts without Python: x0 (R,9) fp32 device = the prior sample
 * [+ init_x] at T0; select_initial_step on the host from two RHS norms, then device-controlled
 * attempts (gp_ode_auto_attempt), the dense output at eps when steps > 0 (t_eval = linspace(T0, eps,
 * steps); steps = 0: t_eval unset), the final denoise and epilogue (gp_ode_denoise) -> pose (R,9),
 * q (R,7) fp64 device. HOST outs: nfev (scipy's count, including the two select_initial_step
 * evaluations), status (1 done, -1 step size below the spacing of t: with steps > 0 that returns an
 * error, since the t_eval outputs collected before the failure need the host controller).
 * Workspace: gp_ode_sample_workspace_size(rows) bytes. Synchronises `stream` once per attempt (a
 * 4-byte status read, one attempt kept enqueued ahead). Replaces genpose2_amd/ode.py rk45_device +
 * PoseNet._ode (agent.py). */
size_t gp_ode_sample_workspace_size(int rows);
int gp_ode_sample(const gp_head_weights *w, const float *pobj, const float *x0, int rows, int k,
                  double T0, double eps, int steps, double rtol, double atol,
                  const float *pts_center, double *pose, double *q, int *nfev, int *status,
                  void *workspace, size_t workspace_bytes, hipStream_t stream);
/* Final denoise (samplers.py:240-249) + epilogue: grad = score(float(x), t32) fp32,
 * x + (0 - g2 * grad) * step (fp32 product, fp64 sum), GS of [:6], + pts_center, quaternion
 * (posenet_agent.py:554-556) -> pose (R,9) fp64, q (R,7) fp64. */
int gp_ode_denoise(const gp_head_weights *w, const float *pobj, float t32, float sigma, float g2,
                   float step, const double *x, int rows, int k, const float *pts_center,
                   double *pose, double *q, void *workspace, size_t workspace_bytes,
                   hipStream_t stream);

/* ===================================================================== ImgEncoder (--dino pointwise)
 * ImgEncoder.forward (networks/img_encoder/img_encoder.py:48-100) over the three DINOv3 intermediate
 * layers l0, l1, l2 (b, np, d), patch-major as get_intermediate_layers(n=[2, 6, 11], norm=True) returns
 * them (np = g*g patches, d = 384): layer attention (la_w1 (d/2, d), la_b1, la_w2 (d/2), la_b2 a host
 * scalar), geometric attention with the (np, np) position table geo_table (gp_img_geo_table), the 3x3
 * edge conv (conv_w (d/4, d, 3, 3) as stored, conv_b), and the final mix with geo_gate =
 * relu(geo_weight), edge_gate = relu(edge_weight) (host scalars) -> out (b, np, d). Optional outputs
 * (NULL to skip): layer_w (b*np, 3) layer-attention weights, edge_out (b, d/4) edge weights.
 * Workspace: gp_img_encoder_workspace_size(b, np, d) bytes. */
size_t gp_img_encoder_workspace_size(int b, int np, int d);
int gp_img_encoder(const float *l0, const float *l1, const float *l2, int b, int np, int d,
                   const float *la_w1, const float *la_b1, const float *la_w2, float la_b2,
                   const float *geo_table, const float *conv_w, const float *conv_b, float geo_gate,
                   float edge_gate, float *out, float *layer_w, float *edge_out, void *workspace,
                   size_t workspace_bytes, hipStream_t stream);
/* gp_img_encoder with the layer-attention Linear and the edge conv as split-f16 GEMMs (gp_linear_split's
 * arithmetic): la_w1_h / conv_w_h are those weights in fus_encoder.pack_split_linear's layout (conv_w as its
 * (d/4, 9d) rows); NULL runs that GEMM in exact fp32 (gp_img_encoder passes NULL for both). */
int gp_img_encoder2(const float *l0, const float *l1, const float *l2, int b, int np, int d,
                    const float *la_w1, const float *la_b1, const float *la_w2, float la_b2,
                    const float *geo_table, const float *conv_w, const float *conv_b, float geo_gate,
                    float edge_gate, const int32_t *la_w1_h, const int32_t *conv_w_h, float *out,
                    float *layer_w, float *edge_out, void *workspace, size_t workspace_bytes,
                    hipStream_t stream);
/* gp_img_encoder2 with the edge conv's split-f16 GEMM gathering its im2col rows from the fused feature map
 * itself (implicit GEMM: no (b np, 9d) column buffer, ~906 MB at b = 256, np = 256, d = 384). conv_w_hp are the
 * planes of conv_w in POSITION-major order: fus_encoder.pack_split_linear of conv_w.permute(0, 2, 3, 1) as its
 * (d/4, 9d) rows (k index (ky * 3 + kx) * d + channel). The products are the same, summed in that order: within
 * rounding of gp_img_encoder2. conv_w_hp == NULL runs the edge conv in exact fp32 (as gp_img_encoder2 does).
 * Workspace: gp_img_encoder3_workspace_size(b, np, d, conv_w_hp != NULL). */
size_t gp_img_encoder3_workspace_size(int b, int np, int d, int split_conv);
int gp_img_encoder3(const float *l0, const float *l1, const float *l2, int b, int np, int d,
                    const float *la_w1, const float *la_b1, const float *la_w2, float la_b2,
                    const float *geo_table, const float *conv_w, const float *conv_b, float geo_gate,
                    float edge_gate, const int32_t *la_w1_h, const int32_t *conv_w_hp, float *out,
                    float *layer_w, float *edge_out, void *workspace, size_t workspace_bytes,
                    hipStream_t stream);
/* HOST: the geometric attention's position table rel_pos_emb(rel_pos_idx).sum(-1) (img_encoder.py:
 * 68-76): table[i][j] = sum_k E[clamp((r_j - r_i + g - 1)(2g - 1) + (c_j - c_i + g - 1), 0, num_emb - 1)][k]
 * for patches i, j at (row, col) = (p / g, p % g). rel_pos_emb (num_emb, edim) host -> table (g^2, g^2)
 * host (the sum runs in order; torch's vector sum may differ from it in the last bit). */
int gp_img_geo_table(const float *rel_pos_emb, int num_emb, int edim, int grid, float *table);
/* The patch -> point gather of GFObjectPose.extract_pts_feature (posenet.py:146-192): out[b][i] =
 * feat[b][clamp((xs[b][i] // patch_px) * grid + ys[b][i] // patch_px, 0, np - 1)] (floor division;
 * the reference's patch_px = 14, grid = 16). feat (b, np, d), xs/ys (b, n) int32 -> out (b, n, d). */
int gp_gather_patch_points(const float *feat, int b, int np, int d, const int *xs, const int *ys, int n,
                           int patch_px, int grid, float *out, hipStream_t stream);

/* ===================================================================== ScaleNet
 * ScaleNet.forward (scalenet.py:33-49): axes (b,3,3), pts_feat (b,1024) -> length (b,3). */
typedef struct {
    const float *ae0_w; /* (256,180) */
    const float *ae0_b;
    const float *ae2_w; /* (256,256) */
    const float *ae2_b;
    const float *ft0_w; /* (256,1280) */
    const float *ft0_b;
    const float *ft2_w; /* (3,256) */
    const float *ft2_b;
} gp_scale_weights;
int gp_scale_forward(const gp_scale_weights *w, const float *axes, const float *pts_feat, int b,
                     float *length, hipStream_t stream);

/* ===================================================================== ranking / aggregation
 * sort_poses_by_energy (networks/reward.py:131-155) + aggregate_pose
 * (runners/evaluation_single.py:160-219) for b objects of k candidates, one launch.
 * poses (b,k,9) fp32 [rot6 | trans], energy (b,k,2) fp32 [rot, trans] -> aggregated (b,4,4).
 * retain = int(k * retain_ratio) (1..min(k,128)); clustering != 0 runs DBSCAN(eps, min_samples)
 * on the rows of D = 1 - <q_i,q_j>^2 of the retained quaternions and re-averages the largest
 * cluster (min_samples = int(clustering_minpts * retain) as the reference passes it).
 * sorted_pose (b,k,9) / sorted_energy (b,k,2) may be NULL; when given they receive the
 * reference's sort_poses_by_energy outputs (descending, ties by lower index). */
int gp_rank_aggregate(const float *poses, const float *energy, int b, int k, int retain,
                      int clustering, float eps, int min_samples, float *aggregated,
                      float *sorted_pose, float *sorted_energy, hipStream_t stream);

/* ===================================================================== stage glue
 * process_batch's pts_center (datasets_omni6dpose.py:746-752): out (b,3) = mean over n of
 * pts (b,n,c)[:, :, :3], c >= 3. */
int gp_points_mean(const float *pts, int b, int n, int c, float *out, hipStream_t stream);
/* inference_scale without a ScaleNet checkpoint (runners/evaluation_single.py:233-252):
 * pcl (b,n,c) raw points, pose (b,4,4) aggregated [R t; 0 1] -> length (b,3) =
 * 2 * max_n |R^T (p_n - t)| per axis. */
int gp_bbox_length(const float *pcl, int b, int n, int c, const float *pose, float *length,
                   hipStream_t stream);

/* ===================================================================== weight packing
 * The load path of PoseNet.load_ckpt -> load_state_dict (posenet_agent.py:171-203) for the --dino none
 * models, without Python: a model's state-dict tensors (HOST float32 arrays named by the reference's
 * model_state_dict keys; a "module." prefix is stripped; num_batches_tracked and unknown keys are ignored)
 * -> every packed layout the kernels read (BN folded in float64, MFMA fragment order, split-f16 planes and
 * bounds), byte-identical to genpose2_amd/pack.py.
 * gp_weights_pack uploads them into ONE device allocation (the only allocating call of the library; not a
 * hot call) and returns an opaque handle; gp_weights_heads / gp_weights_scale / gp_weights_encoder give
 * the structs and pointers the other entry points take (valid until gp_weights_free).
 * gp_weights_pack_host writes the same packed buffer to host memory instead (out == NULL: size query):
 * fields[GP_PACK_NFIELDS] = float offsets of the encoder buffer (GP_PACK_ENC), the 16 gp_head_weights
 * fields in struct order (GP_PACK_HEADS + i) or the 8 gp_scale_weights fields (GP_PACK_SCALE + i), -1 if
 * absent; enc_table (120 int64) = gp_encoder_forward's layer_off relative to the encoder buffer. */
enum { GP_MODEL_SCORE = 0, GP_MODEL_ENERGY = 1, GP_MODEL_SCALE = 2 };
enum { GP_PACK_ENC = 0, GP_PACK_HEADS = 1, GP_PACK_SCALE = 17, GP_PACK_NFIELDS = 25 };
typedef struct gp_weights gp_weights;
int gp_weights_pack(int kind, int n, const char *const *names, const float *const *data,
                    const int64_t *numel, gp_weights **out);
void gp_weights_free(gp_weights *w);
const gp_head_weights *gp_weights_heads(const gp_weights *w);
const gp_scale_weights *gp_weights_scale(const gp_weights *w);
const float *gp_weights_encoder(const gp_weights *w, const int64_t **layer_off);
int gp_weights_pack_host(int kind, int n, const char *const *names, const float *const *data,
                         const int64_t *numel, float *out, size_t out_floats, size_t *need_floats,
                         int64_t *fields, int64_t *enc_table);

#ifdef __cplusplus
}
#endif
#endif /* GENPOSE_HIP_H */
