/*
 * mvreg — MI355X-native pairwise registration hot path of LMPCR
 * (zgojcic/3D_multiview_reg).  C ABI of libmvreg_hip.so.
 *
 * Conventions (every entry point):
 *   - returns 0 (MVR_OK) or a negative error code; never throws across the ABI;
 *   - all pointers are DEVICE pointers allocated by the caller (no hidden
 *     allocation); workspaces are sized by the paired *_workspace_bytes() query;
 *   - calls are stream-ordered on `stream` (a hipStream_t; 0 = legacy default),
 *     re-entrant, and thread-safe across distinct streams/devices;
 *   - strides are in ELEMENTS;
 *   - empty work: when the count that sizes an array is 0 (no rows, pairs, points or fragments), the entry point
 *     returns MVR_OK after validating its scalar arguments and never reads the pointers of the empty arrays, which
 *     may be NULL (a zero-element torch tensor's data_ptr() is 0).  Outputs whose size does not depend on that
 *     count (per-fragment counts, offsets, hash tables that are cleared) are still written, so their pointers stay
 *     required.
 *
 * Process-wide settings: exactly two entry points, mvr_set_math (operand arithmetic) and mvr_debug_force (tests:
 * fallback paths), write process-global values of the library, read by the host side of each later call when it
 * builds its launches.  They are not per stream, per thread or per call.  Set them once, before any thread issues
 * work: two threads selecting different settings race, and a change never affects launches already enqueued.  The
 * defaults are the fp32-equivalent paths the parity tests pin; the Python mirror sets the arithmetic only through
 * lib._native.set_math, before the first forward.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repo).
 */
#ifndef MVREG_H
#define MVREG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mvr_stream_t; /* == hipStream_t */

#define MVR_OK 0
#define MVR_EINVAL -1
#define MVR_ELAUNCH -2

/* ------------------------------------------------------------------------
 * Weighted Procrustes / Kabsch.
 * Replaces lib/utils.py:164-237 kabsch_transformation_estimation (+ residuals
 * lib/utils.py:240-256), and — when guard_pos != NULL — the batch-coupled
 * zero-weight guard of lib/filtering/oanet.py:177-178 (if any pair q has
 * guard_pos[q]==0, every pair's weights get +1/N; w and w_copy are rewritten).
 * guard_group > 0 evaluates the guard per group of that many consecutive pairs (the reference
 * evaluation batch of 32 when a batch is split across ranks); 0 = the whole batch.
 *   x1(p,n,:) = x1[p*x_pstride + n*x_nstride + 0..2], x2 likewise.
 *   w may be NULL (all ones).  R [P,3,3] row-major, t [P,3], res [P, res_pstride],
 *   status[P]: 0 ok, 1 non-finite covariance (reference's SVD-exception branch:
 *   R=I, t=0).  res/res_copy/w_copy/status may be NULL.
 * ---------------------------------------------------------------------- */
int mvr_procrustes(const float* x1, const float* x2, int64_t x_pstride, int64_t x_nstride, float* w,
                   int64_t w_pstride, const int32_t* guard_pos, float* w_copy, int64_t wc_pstride, int P, int N,
                   int normalize, float eps, float* R, float* t, float* res, int64_t res_pstride, float* res_copy,
                   int64_t rc_pstride, int32_t* status, int guard_group, mvr_stream_t stream);
/* fp64 variant (fp64 inputs compute in fp64 in the reference, utils.py:164). */
int mvr_procrustes_f64(const double* x1, const double* x2, int64_t x_pstride, int64_t x_nstride, double* w,
                       int64_t w_pstride, const int32_t* guard_pos, double* w_copy, int64_t wc_pstride, int P, int N,
                       int normalize, double eps, double* R, double* t, double* res, int64_t res_pstride,
                       double* res_copy, int64_t rc_pstride, int32_t* status, int guard_group,
                       mvr_stream_t stream);

/* ------------------------------------------------------------------------
 * RANSAC over given correspondences, batched over pairs.
 * Replaces lib/utils.py:671-709 run_ransac (Open3D 0.9
 * registration_ransac_based_on_correspondence, point-to-point estimation without
 * scaling, ransac_n = 4, max distance 0.05, RANSACConvergenceCriteria(50000, 2500):
 * 2500 iterations) as called at scripts/benchmark_pairwise_registration.py:100,212.
 *   x1(p,i,:) = x1[p*x_pstride + 3i + 0..2] (fp64), x2 likewise; n[p] correspondences of pair p.
 *   Outputs: T [P,4,4] row-major (x2 ~ T x1; identity when no hypothesis has an inlier or
 *   n[p] < ransac_n), fitness [P], rmse [P], best_iter [P] (-1: none).
 *   Draw j of iteration i for pair p: splitmix64(seed + ((p<<40)|(i<<8)|j) * 0x9E3779B97F4A7C15) % n[p]
 *   (Open3D draws std::rand() % n from a clock seed).  hyp_out [P,iters,12] (R row-major, t) may be
 *   NULL; workspace >= mvr_ransac_workspace_bytes(P, iters).
 * ---------------------------------------------------------------------- */
size_t mvr_ransac_workspace_bytes(int P, int iters);
int mvr_ransac(const double* x1, const double* x2, int64_t x_pstride, const int32_t* n, int P, int ransac_n,
               int iters, double max_dist, uint64_t seed, double* T, double* fitness, double* rmse,
               int32_t* best_iter, double* hyp_out, void* workspace, size_t workspace_bytes, mvr_stream_t stream);

/* ------------------------------------------------------------------------
 * Process-wide selections (the only two; every other choice a launch makes is a function of its arguments).
 * mvr_set_math: the operand arithmetic of every kernel that has a choice.  0 (default) f32eq: every fp32 product on
 *   the three-term bf16 split (h + m + l, 6 MFMAs: fp32-equivalent operands).  1 split16: the two-term fp16 split
 *   (h + l, 3 MFMAs per product, 22-bit operands) in the generic GEMM, the point convs, diff_pool / the 4-wave
 *   diff_unpool, the sparse convs with > 64 output channels and the feature-NN distances, wherever the launch has a
 *   range flag: weight rows range-scaled, activations range-checked, and a guarded split-bf16 re-run of any launch
 *   whose operands left the fp16 window; split-bf16 directly where the output overwrites an input.  Returns the
 *   previous mode.
 * mvr_debug_force (tests): force one of the fallback paths the library keeps for shapes its fast kernels do not
 *   cover — 0 the feature NN's online softmax only, 1 point convs and OAFilter conv2 on the generic GEMM, 2 diff_pool
 *   / diff_unpool unfused (embedding GEMM + softmax + pooling GEMM), 3 the block's conv1 stored instead of folded
 *   into the first PointCN, 4 diff_pool without key splits, 5 the 8-wave diff_unpool at <= 512 clusters, 6 the
 *   OANet block's point activations row-major instead of chunk-major (bit-identical).  value 0 restores the
 *   default.  Returns the previous value (MVR_EINVAL for an unknown path).
 * ---------------------------------------------------------------------- */
int mvr_set_math(int mode);
int mvr_debug_force(int what, int value);

/* ------------------------------------------------------------------------
 * One fused MFMA batched GEMM of the OANet schedule (exposed for tests):
 *   C[b](m,n) = sum_k pro_A(A(m,k)) pro_B(B(k,n)) + bias + R[b](m,n)
 * pro: 0 none, 1 relu(A*sc[k]+sh[k]), 2 relu(B*sc[k]+sh[k]) (sc/sh at [b*sPb + k]),
 *      3 B(k,n) * f[b*sPb + (k/128)*pld + n] (per-tile softmax factor).
 * bias_mode: 0 none, 1 per m, 2 per n.  stats_mode: 0 none, 1 row sum/sumsq,
 * 2 row softmax (C <- exp(v - tile row max), partials (tile max, sum)), 3 the same per column,
 * 4 column sum/sumsq (float2 partials, see csrc/gemm.hpp).
 * Layout: 16-byte aligned pointers, all strides multiples of 4 floats, rows padded to
 * round_up(K|N, 4) floats holding finite values (MVR_EINVAL otherwise).
 * math: must be 1, the three-term bf16 split (x = h+m+l, products hh+hm+mh+mm+hl+lh on
 * v_mfma_f32_32x32x16_bf16, fp32 accumulation: fp32-level accuracy); other values return MVR_EINVAL (the exact
 * fp32-MFMA variant of round 2 was removed: 2.7x slower at the same accuracy class).
 * Replaces the nn.Conv2d(k=1) / torch.matmul calls of lib/filtering/oanet.py.
 * ---------------------------------------------------------------------- */
int mvr_gemm_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* B,
                 int64_t sBb, int64_t ldb, int b_kcontig, float* C, int64_t sCb, int64_t ldc, const float* R,
                 int64_t sRb, const float* bias, int bias_mode, const float* psc, const float* psh, int64_t sPb,
                 int64_t pld, int pro, float* stats, int64_t st_ld, int st_off, int stats_mode, int math,
                 int32_t* range_flag, mvr_stream_t stream);
/* OAFilter conv2 (oanet.py:72-81: the 1x1 conv over the clusters on the transpose, W2 [K][K] shared by every pair):
 * C[b](m, n) = sum_k relu(A[b](m, k) psc[b*sPb + k] + psh[b*sPb + k]) W(n, k) + bias[n] + R[b](m, n), M = 128, row
 * statistics per 128-column tile as mvr_gemm_f32's stats_mode 1 (st_off 0), on the split-once kernel (gemm.hip
 * oaf_conv2_kernel: W split into an image once per launch, each A element folded and split once per workgroup,
 * 128 x 256 tiles).  img: >= mvr_oaf_conv2_image_bytes(N, K) bytes of 16-byte aligned device scratch, written by the
 * call.  Layout as mvr_gemm_f32; K % 4 == 0 and 32 < K <= 512.  MVR_EINVAL when the shape is not the kernel's
 * (mvr_oan_block_forward then runs the generic GEMM). */
int mvr_oaf_conv2_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* W,
                      int64_t ldw, float* C, int64_t sCb, int64_t ldc, const float* R, int64_t sRb, const float* bias,
                      const float* psc, const float* psh, int64_t sPb, float* stats, int64_t st_ld, void* img,
                      int64_t img_bytes, mvr_stream_t stream);
size_t mvr_oaf_conv2_image_bytes(int N, int K);

/* ------------------------------------------------------------------------
 * OANet block (lib/filtering/oanet.py:132-185 OANBlock.forward) — parameters
 * are the reference module's tensors (conv weights [Cout][Cin] row-major =
 * the Conv2d weight with its 1x1 tail dropped).
 * ---------------------------------------------------------------------- */
typedef struct { const float* weight; const float* bias; } mvr_conv_p;
typedef struct { const float* gamma; const float* beta; const float* mean; const float* var; } mvr_bn_p;
typedef struct { mvr_bn_p bn1; mvr_conv_p conv3; mvr_bn_p bn5; mvr_conv_p conv7; mvr_conv_p shortcut; } mvr_pointcn_p;
typedef struct {
  mvr_bn_p bn1; mvr_conv_p conv1; /* conv1: IN(1e-3) BN ReLU Conv          (oanet.py:64-69) */
  mvr_bn_p bn2; mvr_conv_p conv2; /* conv2: BN(points) ReLU Conv(points)  (oanet.py:72-76) */
  mvr_bn_p bn3; mvr_conv_p conv3; /* conv3: IN(1e-3) BN ReLU Conv          (oanet.py:77-83) */
} mvr_oafilter_p;

#define MVR_OAN_MAX_HALF 8
typedef struct {
  int in_channels;  /* 6 (reg_init) or 8 (reg_iter) */
  int channels;     /* net_channel (128) */
  int clusters;     /* clusters (500) */
  int half_layers;  /* (net_depth / (iter_num+1)) / 2  (3) */
  mvr_conv_p conv1;
  mvr_pointcn_p l1_1[MVR_OAN_MAX_HALF];
  mvr_bn_p down_bn; mvr_conv_p down_conv;
  mvr_oafilter_p l2[MVR_OAN_MAX_HALF];
  mvr_bn_p up_bn; mvr_conv_p up_conv;
  mvr_pointcn_p l1_2[MVR_OAN_MAX_HALF]; /* l1_2[0] has a shortcut conv (2C -> C) */
  mvr_conv_p output;
} mvr_oan_block_p;

size_t mvr_oan_block_workspace_bytes(int channels, int clusters, int in_channels, int P, int N);

/* input(p,c,n) = input[p*in_pstride + c*ld + n]  (Cin = blk->in_channels); ld >= round_up(N, 4),
 * a multiple of 4, input 16-byte aligned, padding columns [N, ld) finite (zero).
 * xs(p,n,0..5) = xs[p*xs_pstride + n*xs_nstride + 0..5]  (x1 | x2 for Kabsch)
 * Outputs: logits/scores [P,N] (contiguous), R [P,3,3], t [P,3], res [P,N];
 * latent(p,c,n) = latent[p*C*ld + c*ld + n] (may be NULL); res_row/score_row: optional copies written at
 * row pointers with pair stride row_pstride (the next block's input rows 6,7).
 * guard_pos: int32 [P]: per-pair counts of positive weights (zeroed here).  status: int32 [P] (may be NULL).
 * guard_group: scope of the zero-row guard (see mvr_procrustes): 0 the whole batch, > 0 groups of that many
 * pairs; < 0 the block stops after its output head — scores hold relu(tanh(logits)) unguarded, guard_pos the
 * counts, and R, t, res, res_row, score_row are left to the caller's mvr_procrustes (a guard evaluated over
 * pairs on other devices: lib/distributed.py scene mode).
 * bn_train: 0 BatchNorm with running statistics (module.eval()); 1 batch statistics over all P pairs
 * (module.train(): the reference's forward batch); G > 1 batch statistics per group of G consecutive pairs (the
 * last group may be smaller) — G forwards of the reference's loader batches in one call (pair it with
 * guard_group = G). */
/* Diagnostics: how many split-bf16 re-runs of split-fp16 attention launches ran on the current device since
   the last reset (synchronises the device); -1 on error. */
int mvr_attn_reruns(int reset);
/* Debugging: while buf is non-NULL, every mvr_oan_block_forward launch sequence adds a position-weighted
 * 64-bit hash of each stage's activation to the next of cap device slots (zeroed by the caller);
 * NULL disables.  Not for concurrent use from two streams. */
int mvr_debug_stage_hash(unsigned long long* buf, int cap);
/* Debugging: copy the statistics partials hashed as stage `stage` into dst (bytes); NULL disables. */
int mvr_debug_stage_dump(int stage, void* dst, size_t bytes);
/* Diagnostics: the point-activation layout the latest mvr_oan_block_forward chose — 1 chunk-major (every 32-point
 * chunk of a pair one contiguous block), 0 row-major, -1 no forward yet (bench.py records it in its config). */
int mvr_oan_last_layout(void);
int mvr_oan_block_forward(const mvr_oan_block_p* blk, const float* input, int64_t in_pstride, int64_t ld,
                          const float* xs, int64_t xs_pstride, int64_t xs_nstride, int P, int N, int bn_train,
                          float* logits,
                          float* scores, float* R, float* t, float* res, float* latent, float* res_row,
                          float* score_row, int64_t row_pstride, int32_t* guard_pos, int32_t* status, int guard_group,
                          void* workspace,
                          size_t workspace_bytes, mvr_stream_t stream);

/* Fused diff_pool (lib/filtering/oanet.py:96-110), channels == 128, clusters <= 1024:
 *   x_down(p,c,j) = sum_n x(p,c,n) softmax_n(e(p,j,n)),  e = W . relu(x * sc + sh) + b
 * x(p,c,n) = x[p*x_pstride + c*x_ld + n] (x_ld >= round_up(N,4), multiple of 4, 16-byte aligned);
 * sc/sh(p,c) = sc[p*s_pstride + c] (the embedding conv's InstanceNorm+BatchNorm folded to an affine);
 * weight [clusters][128] (16-byte aligned), bias [clusters] (may be NULL);
 * out(p,c,j) = out[p*out_pstride + c*out_ld + j], out_ld >= round_up(clusters,4), columns [clusters,
 * round_up(clusters,4)) written 0.  stats (may be NULL): float pairs (sum, squared deviations from the
 * tile mean) of row c over the 128-column tile t at stats[2*((p*ceil(clusters/128) + t)*st_ld + st_off + c)].
 * The [clusters x N] embedding never leaves the chip (flash-style online softmax). */
int mvr_oan_diff_pool(const float* x, int64_t x_pstride, int64_t x_ld, const float* sc, const float* sh,
                      int64_t s_pstride, const float* weight, const float* bias, int P, int channels, int N,
                      int clusters, float* out, int64_t out_pstride, int64_t out_ld, float* stats, int64_t st_ld,
                      int st_off, mvr_stream_t stream);
/* The same with a workspace (mvr_oan_diff_pool_workspace_bytes(P, 128, clusters) bytes, 16-byte aligned):
 * when one workgroup per (pair, 256-cluster block) leaves the last dispatch round partly idle, the
 * points of each block are split over 2 or 4 workgroups whose partial (output, running max, sum) the
 * last one to finish merges.  Same results up to fp32 summation order. */
size_t mvr_oan_diff_pool_workspace_bytes(int P, int channels, int clusters);
int mvr_oan_diff_pool_ws(const float* x, int64_t x_pstride, int64_t x_ld, const float* sc, const float* sh,
                         int64_t s_pstride, const float* weight, const float* bias, int P, int channels, int N,
                         int clusters, float* out, int64_t out_pstride, int64_t out_ld, float* stats, int64_t st_ld,
                         int st_off, void* workspace, size_t workspace_bytes, mvr_stream_t stream);

/* Fused diff_unpool (lib/filtering/oanet.py:113-129), channels == 128, clusters <= 1024:
 *   out(p,c,n) = sum_j x_down(p,c,j) softmax_j(e(p,j,n)),  e = W . relu(x_up * sc + sh) + b
 * x_up as x above; x_down(p,c,j) = x_down[p*xd_pstride + c*xd_ld + j]; out like x (columns [N,
 * round_up(N,4)) written 0); stats per 128-column tile of N as above (ceil(N/128) tiles per pair).
 * workspace: mvr_oan_diff_unpool_workspace_bytes(P, 128, clusters) bytes, 16-byte aligned (the
 * split-bf16 images of W and x_down). */
size_t mvr_oan_diff_unpool_workspace_bytes(int P, int channels, int clusters);
int mvr_oan_diff_unpool(const float* x_up, int64_t x_pstride, int64_t x_ld, const float* sc, const float* sh,
                        int64_t s_pstride, const float* weight, const float* bias, const float* x_down,
                        int64_t xd_pstride, int64_t xd_ld, int P, int channels, int N, int clusters, float* out,
                        int64_t out_pstride, int64_t out_ld, float* stats, int64_t st_ld, int st_off,
                        void* workspace, size_t workspace_bytes, mvr_stream_t stream);

/* Correspondences [P][N][C] (strided) -> channel-major network input out[p*out_pstride + c*out_ld + n]
 * (the transpose of lib/filtering/oanet.py:234). */
int mvr_xs_to_channels(const float* xs, int64_t xs_pstride, int64_t xs_nstride, int C, int P, int N, float* out,
                       int64_t out_pstride, int64_t out_ld, mvr_stream_t stream);

/* ------------------------------------------------------------------------
 * Overlap gate (lib/utils.py:713-786 compute_overlap_ratio; benchmark:219-220).
 * Open3D VoxelDownSample restated: per fragment b (xyz float32 [n,3], frag_off [B+1] device int64),
 * voxel index floor((p - (min_b - v/2)) / v) in fp64, centroid = fp64 sum of the voxel's points in input
 * order / count.  out_xyz fp64 [n,3] capacity (voxels of a fragment contiguous, fragments in order),
 * out_off [B+1] (device).  Voxel coordinates must stay below 65536 per axis; B <= 4096.
 * ---------------------------------------------------------------------- */
size_t mvr_voxel_centroids_workspace_bytes(int64_t n);
int mvr_voxel_centroids(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel, void* workspace,
                        size_t workspace_bytes, double* out_xyz, int64_t* out_off, mvr_stream_t stream);
/* Radius index over fp64 points [M,3] in fragments off [B+1] (device): points sorted by (fragment, cell of
 * size r) + a hash of the occupied cells.  `index` holds mvr_radius_index_bytes(M) bytes and stays valid
 * for mvr_radius_overlap_count calls on the same points. */
size_t mvr_radius_index_bytes(int64_t M);
int mvr_radius_index_build(const double* xyz, const int64_t* off, int B, int64_t M, double r, void* index,
                           size_t bytes, mvr_stream_t stream);
/* counts[2p + d] = number of points q of fragment pairs[2p + d] whose image T[p][d] q (3x4 row-major fp64,
 * T [P][2][12]) lies at Euclidean distance < r from some point of fragment pairs[2p + 1 - d].
 * With trans the reference's argument: T[p][0] = inv(trans) (pc_i side), T[p][1] = trans (pc_j side).
 * max_points >= the largest fragment. */
int mvr_radius_overlap_count(const void* index, size_t bytes, const double* xyz, const int64_t* off, int B,
                             int64_t M, const int64_t* pairs, const double* T, int P, int64_t max_points, double r,
                             int32_t* counts, mvr_stream_t stream);

/* Farthest point sampling per fragment (Sampler 'fps', lib/layers.py:134-141 — pointnet2
 * furthest_point_sample semantics of oracle/fps.py: seed = first point, running min of squared
 * distances, first maximum on ties).  xyz [sum n][3] with fragment row offsets (device `offsets`
 * and the same values on the host, B+1 entries); idx_out [B][m] int64 global rows.  n >= m for
 * every fragment, n <= 81920. */
int mvr_fps(const float* xyz, const int64_t* offsets, const int64_t* offsets_host, int B, int m, int64_t* idx_out,
            mvr_stream_t stream);

/* Coordinate-space nearest neighbour, knn_point(k=1, pos1, pos2) (lib/utils.py:274-299): for batch row b and
 * query i of pos2 ([B][M] rows of 3 floats at pos2 + b*p2_bstride + i*p2_rstride), the nearest of the N rows of
 * pos1 under the reference's fp32 squared distance ((dx^2 + dy^2) + dz^2, no contraction); first index on equal
 * distances.  dist_out [B][M] (may be NULL), idx_out [B][M] int64 (may be NULL, not both).  Row strides >= 3. */
int mvr_knn1(const float* pos1, int64_t p1_bstride, int64_t p1_rstride, const float* pos2, int64_t p2_bstride,
             int64_t p2_rstride, int B, int N, int M, float* dist_out, int64_t* idx_out, mvr_stream_t stream);

/* Mutual nearest-neighbour flag of the soft matches, extract_mutuals (lib/utils.py:822-848): j = knn1 of x1m[b,i]
 * among x2[b, 0..N), flag_out[b*N + i] = |x1[b,i] - x2m[b,j]|^2 < thr2 ? 1 : 0 (thr2 = threshold^2 rounded to
 * fp32, as the reference's float32 comparison does).  idx_out [B][N] (may be NULL) receives j. */
int mvr_mutuals(const float* x1, int64_t x1_bstride, int64_t x1_rstride, const float* x2, int64_t x2_bstride,
                int64_t x2_rstride, const float* x1m, int64_t x1m_bstride, int64_t x1m_rstride, const float* x2m,
                int64_t x2m_bstride, int64_t x2m_rstride, int B, int N, float thr2, float* flag_out, int64_t* idx_out,
                mvr_stream_t stream);

/* ------------------------------------------------------------------------
 * Feature-space (soft) nearest neighbour for a batch of fragment pairs.
 * Replaces lib/layers.py:44-88 Soft_NN.forward (+ pairwise_distance
 * lib/utils.py:968-992, the pair gather lib/utils.py:850-885 and the xs
 * assembly lib/utils.py:915).  For pair p = (s, t) = pairs[2p], pairs[2p+1]:
 *   queries Fq[s*fq_fstride + n*32 + c], targets Ft[t*ft_fstride + m*32 + c],
 *   target coords Xt[t*xt_fstride + m*3 + k]  (n < Nq, m < Mt, C must be 32);
 * mode 0: x_corr = softmax_m((2 fq.ft - |ft|^2) * inv_tau2) . Xt   ('soft')
 * mode 1: x_corr = Xt[argmax_m(fq.ft*2 - |ft|^2)]                   ('soft'+st, 'hard')
 * out(p,n,:) = [Xq(s,n,0..2) (if Xq != NULL) | x_corr(0..2)] at
 * out[p*out_pstride + n*out_nstride]; idx_out [P][Nq] argmax (mode 1, may be NULL).
 * ---------------------------------------------------------------------- */
int mvr_feat_nn(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const float* Xq,
                int64_t xq_fstride, const float* Xt, int64_t xt_fstride, const int64_t* pairs, int P, int Nq, int Mt,
                int C, float inv_tau2, int mode, float* out, int64_t out_pstride, int64_t out_nstride,
                int32_t* idx_out, mvr_stream_t stream);
/* mvr_feat_nn with a workspace (mvr_feat_nn_workspace_bytes(n_frag, Mt), 16-byte aligned): the soft fast path then
 * splits the target fragments' features once per call into an image of its LDS stages (Ft holds n_frag fragments of
 * Mt targets; every pair's target index < n_frag) and stages them by LDS-DMA.  Results identical to mvr_feat_nn. */
size_t mvr_feat_nn_workspace_bytes(int n_frag, int Mt);
int mvr_feat_nn_ws(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const float* Xq,
                   int64_t xq_fstride, const float* Xt, int64_t xt_fstride, const int64_t* pairs, int P, int Nq,
                   int Mt, int C, float inv_tau2, int mode, float* out, int64_t out_pstride, int64_t out_nstride,
                   int32_t* idx_out, int n_frag, void* workspace, size_t workspace_bytes, mvr_stream_t stream);

/* soft_gumbel correspondences (lib/layers.py:72-78: F.gumbel_softmax(-dist, tau, hard) . y_c): mvr_feat_nn's pairs
 * and layouts, x_corr = softmax((2 fq.ft - |ft|^2 + g) * inv_tau) . Xt (hard = 0) or Xt[argmax of the same noisy
 * logits] (hard = 1: the straight-through forward value; idx_out receives the index), with g = -ln(-ln u) per (query,
 * target) and u a counter-based hash of (seed, pairs[2p], pairs[2p+1], query, target) — reproducible across batch
 * shapes (oracle/soft_nn.py restates it); not torch's Philox stream. */
int mvr_feat_nn_gumbel(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const float* Xq,
                       int64_t xq_fstride, const float* Xt, int64_t xt_fstride, const int64_t* pairs, int P, int Nq,
                       int Mt, int C, float inv_tau, int hard, uint64_t seed, float* out, int64_t out_pstride,
                       int64_t out_nstride, int32_t* idx_out, mvr_stream_t stream);

/* Two nearest neighbours in feature space (scripts/extract_data.py:178-184, sklearn NearestNeighbors
 * kneighbors(n_neighbors=2), Euclidean): for pair p and query j of fragment pairs[2p] (Fq rows, fragment stride
 * fq_fstride), idx2_out[(p*Nq + j)*2 + k] = k-th nearest row of fragment pairs[2p+1] (Ft, Mt >= 2 rows),
 * smallest distance first, first index on ties (split-bf16 MFMA distances; fp32-level near-ties may order
 * differently from fp64).  dist2_out (may be NULL): the fp64 distances of those two rows.  C == 32. */
int mvr_feat_knn2(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const int64_t* pairs,
                  int P, int Nq, int Mt, int C, int32_t* idx2_out, double* dist2_out, mvr_stream_t stream);

/* Row gather dst[i][:] = src[idx[i]][:] (C floats per row): the Sampler's
 * index_select (lib/layers.py:151-152) with host-drawn (np.random) indices. */
int mvr_gather_rows(const float* src, int C, const int64_t* idx, int n, float* dst, mvr_stream_t stream);

/* ------------------------------------------------------------------------
 * Sparse-voxel primitives of the FCGF descriptor (MinkowskiEngine 0.4 calls in
 * lib/descriptor/fcgf.py, scripts/pairwise_demo.py:79-93, scripts/utils.py:102-120).
 * coords are int32 [M][4] = (batch, x, y, z); hash tables are opaque device
 * buffers of mvr_hash_table_bytes(M) bytes.
 * ---------------------------------------------------------------------- */
size_t mvr_hash_table_bytes(int64_t M);
size_t mvr_voxelize_workspace_bytes(int64_t n);
/* ME.utils.sparse_quantize(floor(xyz/voxel), return_index=True) per fragment, batched:
 * fragment b owns points [frag_off[b], frag_off[b+1]).  floor((double)x / voxel) in float64 with a correctly
 * rounded division — the reference's numpy arithmetic on Open3D's float64 points (scripts/utils.py:108-109).  Writes the unique voxels in
 * first-occurrence order: coords_out [n][4] (first count rows valid), sel_out [n]
 * (source point index), counts_out int64 [1+B] = {total, per-fragment}. */
int mvr_voxelize(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel, void* workspace,
                 size_t workspace_bytes, int32_t* coords_out, int64_t* sel_out, int64_t* counts_out,
                 mvr_stream_t stream);
/* mvr_voxelize over float64 points (the caller's float64 array floored as it is: scripts/utils.py:108-109 applies
 * np.floor to Open3D's float64 points; no float32 rounding first).  Same workspace size, outputs and order. */
int mvr_voxelize_f64(const double* xyz, const int64_t* frag_off, int B, int64_t n, double voxel, void* workspace,
                     size_t workspace_bytes, int32_t* coords_out, int64_t* sel_out, int64_t* counts_out,
                     mvr_stream_t stream);
/* mvr_voxelize for a hinted voxel count (distinct_hint: the expected voxels of the whole batch).  Each fragment's
 * keys are split into hash buckets sized so that the mean fragment's share of the hint fills half of a workgroup's
 * LDS table; a bucket with more voxels than its table takes, or a coordinate outside the keys' 17-bit range, sets
 * counts_out[B + 1] (counts_out has B + 2 entries): the caller then re-runs mvr_voxelize.  Otherwise the same
 * outputs as mvr_voxelize. */
size_t mvr_voxelize_hint_workspace_bytes(int64_t n, int64_t distinct_hint);
int mvr_voxelize_hint(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel,
                      int64_t distinct_hint, void* ws, size_t ws_bytes, int32_t* coords_out, int64_t* sel_out,
                      int64_t* counts_out, mvr_stream_t stream);
size_t mvr_coords_downsample_workspace_bytes(int64_t M);
/* strided coordinate set floor(c/s)*s (first-occurrence order); counts_out as above */
int mvr_coords_downsample(const int32_t* coords, int64_t M, int B, int stride_out, void* workspace,
                          size_t workspace_bytes, int32_t* coords_out, int64_t* counts_out, mvr_stream_t stream);
int mvr_hash_build(const int32_t* coords, int64_t M, void* table, size_t table_bytes, mvr_stream_t stream);
/* the same for a coordinate set on the lattice of `stride` (a power of two: every coordinate a multiple of it, the
 * tensor stride of an FCGF level): the 2x2x2 cells of that lattice share one 8-slot bucket of the table, so a kernel
 * map's stencil probes read a few runs instead of scattered slots (MinkowskiEngine's CoordinateManager keeps one map
 * per tensor stride likewise, fcgf.py:118-227).  Same lookups and results as mvr_hash_build. */
int mvr_hash_build_lattice(const int32_t* coords, int64_t M, int stride, void* table, size_t table_bytes,
                           mvr_stream_t stream);
/* kernel map as a neighbour table nbr[o][k] (k = (dx+r) + ks(dy+r) + ks^2(dz+r)):
 * row of out_coords[o] + sign*off_k*step in the input table (sign -1 if transposed), or -1 */
int mvr_kernel_map(const int32_t* out_coords, int64_t Mout, const void* in_table, size_t in_table_bytes, int ksize,
                   int step, int transposed, int32_t* nbr, mvr_stream_t stream);
/* mvr_kernel_map visiting the output rows in row_order (int32 [Mout], a permutation; NULL: row order) — the same
 * table; a spatial order (mvr_kernel_map_orders with nbr NULL) makes the workgroups that run together probe
 * neighbouring cells of the input table */
int mvr_kernel_map_x(const int32_t* out_coords, int64_t Mout, const void* in_table, size_t in_table_bytes, int ksize,
                     int step, int transposed, int32_t* nbr, const int32_t* row_order, mvr_stream_t stream);
/* 3^3 map of a set onto itself (out set == the table's set in row order: FCGF's stride-1 convs), equal to
 * mvr_kernel_map(coords, M, table, ..., 3, step, 0, nbr): half the offsets are probed, each hit also writes its mirror
 * entry (neighbour 26 - k of i is o when neighbour k of o is i), the centre is the row itself. */
int mvr_kernel_map_sym(const int32_t* coords, int64_t M, const void* table, size_t table_bytes, int step, int32_t* nbr,
                       mvr_stream_t stream);
/* dst [Md][K] = the transpose of src [Ms][K]: dst[i][k] = o where src[o][k] = i, else -1.  The transposed stride-2
 * conv's map between two sets (mvr_kernel_map(..., transposed = 1)) is the transpose of the strided conv's map between
 * them (FCGF's up maps from its down maps). */
int mvr_kernel_map_transpose(const int32_t* src, int64_t Ms, int K, int32_t* dst, int64_t Md, mvr_stream_t stream);
/* Row order of a kernel map: output rows sorted by their active-offset mask (K <= 27), so that a
 * tile of consecutive rows shares its active offsets; with out_coords (int32 [Mout][4], the map's output
 * coordinates, multiples of step) rows of one mask are further ordered by fragment and Morton code of
 * coordinates / step (spatially compact tiles: L2 reuse of the gathered rows).  Stable: ties keep row order.
 * A hand-written onesweep LSD radix sort (csrc/radix.hip: a control-block clear, one histogram launch, one launch
 * per 8-bit digit).  Workspace: mvr_kernel_map_order_bytes(Mout). */
size_t mvr_kernel_map_order_bytes(int64_t Mout);
int mvr_kernel_map_order(const int32_t* nbr, const int32_t* out_coords, int step, int64_t Mout, int K, int32_t* perm,
                         void* workspace, size_t workspace_bytes, mvr_stream_t stream);
/* The row orders of n_maps (<= 16) kernel maps in ONE sort (the map index in the top key bits): host arrays
 * nbr[j] (int32 [Mo[j]][K]), out_coords[j] (or out_coords NULL: masks only) with steps[j]; perm_out int32
 * [sum Mo]: map j's order (local row indices, exactly mvr_kernel_map_order's) at offset Mo[0] + ... + Mo[j-1].
 * Workspace: mvr_kernel_map_orders_bytes(sum Mo).  (FCGF: all ten 3^3 maps of a scene, lib/sparse.py
 * CoordinateManager.prepare_orders.)  nbr NULL with K = 0: coordinate sets only (out_coords required) — each
 * set's rows in (fragment, Morton code of coordinates / step) order, stable (the kernel maps' visiting order). */
size_t mvr_kernel_map_orders_bytes(int64_t total);
int mvr_kernel_map_orders(int n_maps, const int32_t* const* nbr, const int32_t* const* out_coords, const int* steps,
                          const int64_t* Mo, int K, int32_t* perm_out, void* workspace, size_t workspace_bytes,
                          mvr_stream_t stream);
/* The same stable radix sort on its own: values int32 [n] (NULL: 0..n-1) in ascending order of the key bits
 * [0, bits) of keys uint64 [n] -> vals_out.  Workspace: mvr_radix_sort_pairs_bytes(n). */
size_t mvr_radix_sort_pairs_bytes(int64_t n);
int mvr_radix_sort_pairs(const uint64_t* keys, const int32_t* vals, int64_t n, int bits, int32_t* vals_out,
                         void* workspace, size_t workspace_bytes, mvr_stream_t stream);
/* MinkowskiConvolution forward, gather-GEMM over the neighbour table (nbr NULL & K==1:
 * identity map, i.e. a 1x1x1 conv); W [K][Cin][Cout]; epilogue (+bias[Cout]) ->
 * BatchNorm eval (bn.gamma NULL: none) -> (+res[o*ldres+c]) -> ReLU if relu.
 * perm (optional): order in which output rows are tiled (mvr_kernel_map_order); results are
 * written to their own rows either way.
 * wimg (required, 16-byte aligned): the weights pre-split by mvr_spconv_wimage -> split-bf16 MFMA path
 * (fp32-level accuracy, ~2.7x the exact-fp32 MFMA rate).  Cin a multiple of 32 (every FCGF conv), Cout and ldin
 * multiples of 4, in and W 16-byte aligned; MVR_EINVAL otherwise.
 * range_flag (optional, device int32 owned by the stream's call sequence): enables the split-fp16 pass when
 * mvr_set_math(1) (the flag is cleared by the call, set by a split-fp16 pass whose operands left the fp16
 * window, and read by its guarded split-bf16 re-run); NULL -> split-bf16 only.  out is either disjoint from res
 * or equal to it (in place). */
int mvr_spconv(const float* in, int64_t ldin, int Cin, const int32_t* nbr, const int32_t* perm, int K, int64_t Mout,
               const float* W, int Cout, const float* bias, mvr_bn_p bn, float bn_eps, const float* res,
               int64_t ldres, int relu, float* out, int64_t ldout, const void* wimg, int32_t* range_flag,
               mvr_stream_t stream);
/* mvr_spconv with split-bf16 planes beside the fp32 buffers (FCGF: every conv's output feeds the next conv's
 * gathers).  in_planes (optional, 16-byte aligned, ldin % 8 == 0): the input's (h, m, l) bf16 planes, row r plane p
 * at in_planes + (3 r + p) ldin — the split the kernel would otherwise repeat for each of a row's ~14 gathers; the
 * split-bf16 pass gathers them instead of `in` (bit-identical results; a split-fp16 pass still reads `in`).
 * out_planes (optional): also write the output's planes, row r plane p at out_planes + (3 r + p) ldout. */
int mvr_spconv_x(const float* in, int64_t ldin, int Cin, const int32_t* nbr, const int32_t* perm, int K, int64_t Mout,
                 const float* W, int Cout, const float* bias, mvr_bn_p bn, float bn_eps, const float* res,
                 int64_t ldres, int relu, float* out, int64_t ldout, const void* wimg, int32_t* range_flag,
                 const uint16_t* in_planes, uint16_t* out_planes, mvr_stream_t stream);
/* Weight image of mvr_spconv's split paths: W [K][Cin][Cout] fp32 -> three bf16 planes in
 * [K][ceil(Cin/32)][plane][round_up(Cout,128)][40] rows (80-byte rows, zero padded), then the same rows as two
 * fp16 planes of W[.][.][c] s_c (s_c: a power of two bringing output channel c's weights to <= 2^14), then
 * s_c and 1 / (s_c 2^6) per channel. */
size_t mvr_spconv_wimage_bytes(int K, int Cin, int Cout);
int mvr_spconv_wimage(const float* W, int K, int Cin, int Cout, void* img, size_t bytes, mvr_stream_t stream);
/* Brick map of a coordinate set (4x4x4 bricks: hash of brick coordinates -> 64 row slots), the
 * neighbourhood structure of the large-stencil conv below.  Workspace:
 * mvr_brick_map_bytes(M).  _stride: a set at tensor stride `stride` (a power of two, coordinates multiples of it):
 * cells are coordinates / stride; mvr_brick_map_build = stride 1. */
size_t mvr_brick_map_bytes(int64_t M);
int mvr_brick_map_build(const int32_t* coords, int64_t M, void* workspace, size_t workspace_bytes,
                        mvr_stream_t stream);
int mvr_brick_map_build_stride(const int32_t* coords, int64_t M, int stride, void* workspace, size_t workspace_bytes,
                               mvr_stream_t stream);
/* single-input-channel conv with a large stencil (FCGF conv1, 7^3) over the input set's brick map
 * (in_bricks built from the Min input coordinates; input cell = coordinate / step).
 * out_coords NULL: the output set is the input set itself (Mout == Min, step 1, ksize 7; output row o =
 * input row o) — computed brick by brick as dense 7^3 windows on split-bf16 MFMA. */
int mvr_spconv_c1(const int32_t* out_coords, int64_t Mout, const void* in_bricks, int64_t Min, size_t in_bricks_bytes,
                  const float* feat, int ksize, int step, const float* W, int Cout, mvr_bn_p bn, float bn_eps,
                  int relu, float* out, int64_t ldout, mvr_stream_t stream);
/* mvr_spconv_c1 (brick path, out_coords NULL) also writing the output's split-bf16 planes (mvr_spconv_x's layout) */
int mvr_spconv_c1_x(const int32_t* out_coords, int64_t Mout, const void* in_bricks, int64_t Min,
                    size_t in_bricks_bytes, const float* feat, int ksize, int step, const float* W, int Cout,
                    mvr_bn_p bn, float bn_eps, int relu, float* out, int64_t ldout, uint16_t* out_planes,
                    mvr_stream_t stream);
/* x[o][:C] /= ||x[o][:C]||  (fcgf.py:274-278) */
int mvr_l2norm_rows(float* x, int64_t M, int C, int64_t ld, mvr_stream_t stream);

/* Sampler 'rand' (lib/layers.py:145-148) on the host: for each fragment b in order,
 * np.random.choice(arange(start_b, start_b + counts[b]), tgt, replace=False) drawn from numpy's
 * legacy MT19937 RandomState (key uint32[624] and *pos as np.random.get_state() gives them; advanced
 * in place for np.random.set_state()).  out int64 [B][tgt]; ws int64 scratch of max(counts).
 * Requires tgt <= counts[b].  Host-only (no device work, no stream). */
int mvr_sample_rand_mt19937(uint32_t* key, int32_t* pos, const int64_t* counts, int B, int tgt, int64_t* out,
                            int64_t* ws);

/* Opt-in per-kernel-class device timing (hipEvents on the launching stream).
 * mvr_prof_set(1) resets and enables; mvr_prof_get(kind, ...) synchronises the
 * recorded events and returns totals since then (kinds: csrc/prof.hpp ProfKind). */
int mvr_prof_set(int on);
/* kinds that get event records while enabled: bit k = kind k (default: all) */
int mvr_prof_mask(unsigned mask);
int mvr_prof_get(int kind, double* ms, long long* launches, double* flops, double* bytes);
/* launch order since mvr_prof_set(1): kind and algorithmic bytes per profiled launch (<= cap);
 * returns the count (joins rocprofv3 PMC dispatch rows to kernel classes) */
int mvr_prof_seq(int* kinds, double* bytes, int cap);
/* the library's source identity (sha256 prefix of its sources + variant flags) as a NUL-terminated string: MVR_OK,
 * or the buffer size needed when cap is too small (bench.py uses the PMC counters only of this same build) */
int mvr_source_hash(char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
