// Batched fp32 MFMA GEMM with fused prologue transforms and epilogue statistics.
// Used for every 1x1 convolution / pooling matmul of the OANet filter
// (lib/filtering/oanet.py) — see gemm.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mvr {

enum Pro : int {
  PRO_NONE = 0,   // operands used as stored
  PRO_A_K = 1,    // A(m,k) <- relu(A*sc[k] + sh[k])           (BN+ReLU on the reduction axis of A)
  PRO_B_K = 2,    // B(k,n) <- relu(B*sc[k] + sh[k])           (IN+BN+ReLU folded, per input channel)
  PRO_B_SMX = 3,  // B(k,n) <- exp(B - mx[n]) * rs[n]           (softmax normalised by column)
};
enum Bias : int { BIAS_NONE = 0, BIAS_M = 1, BIAS_N = 2 };
enum Stats : int {
  ST_NONE = 0,
  ST_ROW = 1,     // per (b, n-tile, m): (sum, sumsq) over the tile's columns  -> InstanceNorm stats
  ST_ROWSMX = 2,  // per (b, n-tile, m): (max, sum exp(v-max))                 -> softmax over n
  ST_COLSMX = 3,  // per (b, m-tile, n): (max, sum exp(v-max))                 -> softmax over m
  ST_COL = 4,     // per (b, m-tile, n): (sum, sumsq) over the tile's rows     -> train-mode BN over m
};

constexpr int GEMM_BM = 128, GEMM_BN = 128, GEMM_BK = 16;

struct GemmArgs {
  int M, N, K, batch;
  const float* A; int64_t sAb; int64_t lda;            // A(m,k) = A[b*sAb + m*lda + k]
  const float* B; int64_t sBb; int64_t ldb; int bkc;   // bkc=0: B[b*sBb + k*ldb + n]; bkc=1: B[b*sBb + n*ldb + k]
  float* C; int64_t sCb; int64_t ldc;                  // C(m,n) = C[b*sCb + m*ldc + n]
  const float* R; int64_t sRb;                         // residual, same ldc as C
  const float* bias;                                   // [M] (BIAS_M) or [N] (BIAS_N)
  const float* psc; const float* psh; int64_t sPb;     // prologue vectors (batch stride sPb, may be 0)
  float2* stats; int64_t st_ld; int st_off;            // partial statistics (see Stats)
  int pro, bias_mode, stats_mode, has_res;
  int prof_kind;                                       // ProfKind tag (prof.hpp); 0 by default
  int use_v1;                                          // force the register-staged kernel (tests)
};

// Launch on `stream`; returns 0 or a negative error.
int launch_gemm(const GemmArgs& g, hipStream_t stream);

inline int gemm_ntiles(int N) { return (N + GEMM_BN - 1) / GEMM_BN; }
inline int gemm_mtiles(int M) { return (M + GEMM_BM - 1) / GEMM_BM; }

}  // namespace mvr
