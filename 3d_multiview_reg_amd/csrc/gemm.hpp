// Batched fp32 MFMA GEMM with fused prologue transforms and epilogue statistics.
// Used for every 1x1 convolution / pooling matmul of the OANet filter
// (lib/filtering/oanet.py) — see gemm.hip.
#pragma once
#include "knobs.hpp"
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mvreg.h"

namespace mvr {

enum Pro : int {
  PRO_NONE = 0,   // operands used as stored
  PRO_A_K = 1,    // A(m,k) <- relu(A*sc[k] + sh[k])           (BN+ReLU on the reduction axis of A)
  PRO_B_K = 2,    // B(k,n) <- relu(B*sc[k] + sh[k])           (IN+BN+ReLU folded, per input channel)
  PRO_B_SMX = 3,  // B(k,n) <- B(k,n) * f[k/128][n]            (softmax: B holds exp(x - tile max) as
                  //                                            written by an ST_*SMX epilogue, f the
                  //                                            per-tile factor exp(tile max - max)/sum)
};
enum Bias : int { BIAS_NONE = 0, BIAS_M = 1, BIAS_N = 2 };
enum Stats : int {
  ST_NONE = 0,
  ST_ROW = 1,     // per (b, n-tile, m): (sum, sum of squared deviations from the tile mean) over
                  // the tile's columns                                          -> InstanceNorm stats
  ST_ROWSMX = 2,  // C <- exp(v - mt), mt = max of row m over the tile's columns;
                  // per (b, n-tile, m): (mt, sum exp(v - mt))                 -> softmax over n
  ST_COLSMX = 3,  // C <- exp(v - mt), mt = max of column n over the tile's rows;
                  // per (b, m-tile, n): (mt, sum exp(v - mt))                 -> softmax over m
  ST_COL = 4,     // per (b, m-tile, n): (sum, squared deviations) over the tile's rows
                  //                                                           -> train-mode BN over m
};

// Arithmetic of the MFMA main loop.  MATH_BF16X3 (the only value a caller passes): each fp32 operand split into three bf16 terms (x = h + m + l to 2^-25 |x|) and the
// six products hh, hm, mh, mm, hl, lh accumulated in fp32 by v_mfma_f32_32x32x16_bf16 — fp32-level
// accuracy (the dropped ml, lm, ll terms are <= 2^-23 relative) at 6/16 of the fp32 MFMA cycles.
// MATH_F16X2 (internal): two-term split-fp16 (mfma_bf16.hpp) of A x 2^6 and B x 2^6, 3 MFMAs per product; what a
// MATH_BF16X3 launch runs first under mvr_set_math(1), with a guarded MATH_BF16X3 re-run when an operand
// left the split-fp16 window (gemm.hip launch_t).
enum Math : int { MATH_BF16X3 = 1, MATH_F16X2 = 2 };

constexpr int GEMM_BM = 128, GEMM_BN = 128, GEMM_BK = 32;

struct GemmArgs {
  int M, N, K, batch;
  const float* A; int64_t sAb; int64_t lda;            // A(m,k) = A[b*sAb + m*lda + k]
  const float* B; int64_t sBb; int64_t ldb; int bkc;   // bkc=0: B[b*sBb + k*ldb + n]; bkc=1: B[b*sBb + n*ldb + k]
  float* C; int64_t sCb; int64_t ldc;                  // C(m,n) = C[b*sCb + m*ldc + n]
  const float* R; int64_t sRb;                         // residual, same ldc as C
  const float* bias;                                   // [M] (BIAS_M) or [N] (BIAS_N)
  const float* psc; const float* psh; int64_t sPb;     // PRO_A_K/PRO_B_K: per-k vectors psc/psh [b*sPb + k];
  int64_t pld;                                         // PRO_B_SMX: factors psc[b*sPb + (k/128)*pld + n]
  float2* stats; int64_t st_ld; int st_off;            // partial statistics (see Stats)
  int pro, bias_mode, stats_mode, has_res;
  int prof_kind;                                       // ProfKind tag (prof.hpp); 0 by default
  int math;                                            // Math: MATH_BF16X3 (anything else is MVR_EINVAL)
  int no_store;                                        // 1: statistics only, C is not written (may be null)
  // output head fused into the epilogue (pconv only, M = 128): logits[b*N + n] = head_w . C(:, n) + head_bp[0] (nullable),
  // scores = relu(tanh(logits)), pos[b] += #positive scores (oanet.py:163,174-178)
  const float* head_w; const float* head_bp; float* logits; float* scores; int32_t* pos;
  // the block's conv1 folded into its first PointCN (pconv only, M = K = 128): xin = 1, the B operand
  // rows are x(k, n) = xb[k] + xw[k][:xci] . B(:xci, n) (B then holds the block input, xci <= 8 rows);
  // xin = 2, the residual is x(m, n) recomputed the same way from R (the block input).  xw [128][8]
  // (columns >= xci zero), xb [128] (nullable)
  int xin; int xci; const float* xw; const float* xb;
  int64_t xld;   // row stride of the block input (xin = 2: R's rows; xin = 1 uses ldb)
  // MATH_BF16X3 under mvr_set_math(1): a zeroed int in device memory owned by this launch
  // (stream-ordered); the split-fp16 pass sets it when an operand leaves the fp16 window and the guarded split-bf16
  // pass then recomputes every output.  Null: split-bf16 only.
  int* flag;
  // InstanceNorm fold of the output fused into the producer (pconv only, stats_mode ST_ROW, split-bf16 launches):
  // the workgroup that completes a pair's statistics (a per-pair arrival counter, fin_cnt[b], zeroed by the
  // caller) merges them like in_finalize_kernel and writes the fold for the next conv's prologue:
  // fin_sc/fin_sh [b*fin_ld + m] (eval; fin_sc2/fin_sh2 with fin_bn2 / fin_eps2 when set: a second fold of the
  // same statistics) or (mean, var) into fin_mv [b*M + m] (fin_train).  launch_gemm sets *fin_done when it did.
  int* fin_cnt; float fin_eps; mvr_bn_p fin_bn; float* fin_sc; float* fin_sh; int64_t fin_ld;
  float fin_eps2; mvr_bn_p fin_bn2; float* fin_sc2; float* fin_sh2;
  int fin_train; float2* fin_mv; int* fin_done;
  // OAFilter conv2 shape (M = 128, PRO_A_K, B = weights [N][K] shared by every pair, BIAS_N, ST_ROW, residual) with
  // the split-once OAFilter conv2 kernel: scratch for the weights' split-bf16 image (oaf_conv2_image_bytes(N, K) bytes, written
  // by the launch), which routes it to the split-once kernel (gemm.hip oaf_conv2_kernel).  Null: generic kernel.
  uint16_t* wimg; int64_t wimg_bytes;
  // chunk-major point activations (point-conv kernel only, bkc = 0): element (row, n) of B / C / R at
  // row ld + (n >> 5) cs + (n & 31) with the operand's chunk stride cs (0: row-major, row ld + n); ldr: the
  // residual's row stride (0: ldc)
  int64_t bcs, ccs, rcs, ldr;
};

// Layout contract — operands are staged by 16-byte LDS-DMA with every address clamped into the
// padded rows, so: all pointers 16-byte aligned; lda, ldb, ldc, pld and every batch stride a
// multiple of 4; A rows (and B rows when bkc) readable up to round_up(K, 4) floats, B rows
// (bkc = 0), C/R rows and factor rows up to round_up(N, 4) floats, all of them finite there.
// Padding columns of C in [N, round_up(N, 4)) are written (finite values: 0 after a softmax
// epilogue) and never enter results, statistics or the K tail.  PRO_A_K / PRO_B_K need K % 4 == 0
// and K <= 512.  Launch on `stream`; returns 0 or a negative error (MVR_EINVAL on a violated
// contract).  The output (C) is either disjoint from A, B and R or equal to R (in place, residual); it never
// partially overlaps an input.
int launch_gemm(const GemmArgs& g, hipStream_t stream);

// 128 -> 128 point convolutions (pconv.hip): launch_gemm routes the shapes pconv_covers() accepts there
bool pconv_covers(const GemmArgs& g);   // head fields set: only pconv can run it
int launch_pconv(const GemmArgs& g, hipStream_t stream);

// diff_pool / diff_unpool (oan_attn.hip) over point activations in either layout (chunk stride cs, GemmArgs
// bcs): the C-ABI mvr_oan_diff_pool_ws / mvr_oan_diff_unpool with cs = 32 (row-major)
int oan_diff_pool_cm(const float* x, int64_t x_pstride, int64_t x_ld, int64_t x_cs, const float* sc, const float* sh,
                     int64_t s_pstride, const float* weight, const float* bias, int P, int channels, int N, int clusters,
                     float* out, int64_t out_pstride, int64_t out_ld, float* stats, int64_t st_ld, int st_off,
                     void* workspace, size_t workspace_bytes, hipStream_t stream);
int oan_diff_unpool_cm(const float* x_up, int64_t x_pstride, int64_t x_ld, int64_t x_cs, const float* sc,
                       const float* sh, int64_t s_pstride, const float* weight, const float* bias, const float* x_down,
                       int64_t xd_pstride, int64_t xd_ld, int P, int channels, int N, int clusters, float* out,
                       int64_t out_pstride, int64_t out_ld, int64_t out_cs, float* stats, int64_t st_ld, int st_off,
                       void* workspace, size_t workspace_bytes, hipStream_t stream);

// bytes of the weights' split-bf16 image the OAFilter conv2 kernel reads (GemmArgs.wimg)
int64_t oaf_conv2_image_bytes(int N, int K);

inline int gemm_ntiles(int N){ return (N + GEMM_BN - 1) / GEMM_BN; }
inline int gemm_mtiles(int M) { return (M + GEMM_BM - 1) / GEMM_BM; }
inline int64_t round4(int64_t x) { return (x + 3) & ~(int64_t)3; }
inline int64_t round32(int64_t x) { return (x + 31) & ~(int64_t)31; }

}  // namespace mvr
