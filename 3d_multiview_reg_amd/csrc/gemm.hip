// Batched fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32,
// exact fp32 fma chains — no reduced-precision path, so OANet inlier masks match
// the fp32 reference).
//
//   C[b](m,n) = sum_k  pro_A(A[b](m,k)) * pro_B(B[b](k,n))  (+ bias) (+ R[b](m,n))
//
// with the OANet elementwise work fused in:
//   * prologue (applied while staging the tile global -> registers -> LDS):
//       InstanceNorm+BatchNorm+ReLU folded to relu(x*sc[k]+sh[k]) on the reduction axis, or the
//       column softmax exp(x-mx[n])*rs[n] of diff_pool / diff_unpool (oanet.py:106-128);
//   * epilogue: bias, residual add (PointCN / OAFilter shortcuts, oanet.py:39-42,87-92),
//       and the partial statistics the NEXT layer needs (InstanceNorm sum/sumsq per row,
//       softmax max/sum-exp per row or per column), reduced across the 32-lane half by a
//       register-transposing butterfly (16 shuffles for 16 rows instead of 80).
//
// Tile: 128x128 per 256-thread workgroup (4 waves in 2x2, each 64x64 = 2x2 MFMA 32x32
// blocks), BK=16, register-staged double-buffered LDS, one barrier per K step.
// Roofline: 2*M*N*K flops per GEMM against the 157.3 TF/s fp32 MFMA peak.
#include "common.hpp"
#include "gemm.hpp"
#include "prof.hpp"

namespace mvr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = GEMM_BM, BN = GEMM_BN, BK = GEMM_BK;
constexpr int LDA_S = BM + 4, LDB_S = BN + 4;
constexpr float NEG_BIG = -3.0e38f;

struct KArgs {
  GemmArgs g;
  int vecA, vecB;
};

__device__ __forceinline__ float4 ld4(const float* p, bool vec, int valid) {
  // valid: number of in-range elements (0..4) starting at p
  if (vec && valid == 4) return *reinterpret_cast<const float4*>(p);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid > 0) r.x = p[0];
  if (valid > 1) r.y = p[1];
  if (valid > 2) r.z = p[2];
  if (valid > 3) r.w = p[3];
  return r;
}

__device__ __forceinline__ float& f4(float4& v, int i) { return reinterpret_cast<float*>(&v)[i]; }

__device__ __forceinline__ void smx_combine(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  s = s * expf(m - M) + s2 * expf(m2 - M);
  m = M;
}

// Butterfly over the 32 lanes of a half-wave for 16 per-lane values (one per MFMA row
// register).  On return lane l holds in v[0] the reduction of register
// rho(l) = 8*b4 + 4*b3 + 2*b2 + b1 (bits of l), lanes l and l^1 identical.
template <bool SMX>
__device__ __forceinline__ void butterfly16(float (&v)[16], float (&s)[16], int lane) {
#pragma unroll
  for (int step = 0; step < 4; ++step) {
    const int half = 8 >> step;             // 8,4,2,1 registers kept
    const int mask = 16 >> step;            // xor 16,8,4,2
    const bool hi = (lane & mask) != 0;
#pragma unroll
    for (int r = 0; r < half; ++r) {
      const float send_v = hi ? v[r] : v[r + half];
      const float send_s = hi ? s[r] : s[r + half];
      const float rv = __shfl_xor(send_v, mask, 64);
      const float rs = __shfl_xor(send_s, mask, 64);
      float kv = hi ? v[r + half] : v[r];
      float ks = hi ? s[r + half] : s[r];
      if (SMX) {
        smx_combine(kv, ks, rv, rs);
      } else {
        kv += rv;
        ks += rs;
      }
      v[r] = kv;
      s[r] = ks;
    }
  }
  const float rv = __shfl_xor(v[0], 1, 64);
  const float rs = __shfl_xor(s[0], 1, 64);
  if (SMX) {
    smx_combine(v[0], s[0], rv, rs);
  } else {
    v[0] += rv;
    s[0] += rs;
  }
}

template <int PRO, int BKC, int BIAS, int STATS, int RES>
__global__ __launch_bounds__(256) void gemm_kernel(KArgs ka) {
  const GemmArgs& g = ka.g;
  __shared__ float As[2][BK][LDA_S];
  __shared__ float Bs[2][BK][LDB_S];
  __shared__ float2 red[2][BM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = g.M, N = g.N, K = g.K;

  const float* A = g.A + (int64_t)b * g.sAb;
  const float* B = g.B + (int64_t)b * g.sBb;
  const float* psc = g.psc ? g.psc + (int64_t)b * g.sPb : nullptr;
  const float* psh = g.psh ? g.psh + (int64_t)b * g.sPb : nullptr;
  const bool vecA = ka.vecA, vecB = ka.vecB;

  float4 ra[2], rb[2];

  auto load = [&](int k0) {
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      // ---- A tile: 128 (m) x 16 (k), k-contiguous in memory
      {
        const int m = (tid >> 2) + 64 * rep, kq = (tid & 3) * 4;
        const int gm = m0 + m, gk = k0 + kq;
        const int valid = (gm < M) ? min(4, max(0, K - gk)) : 0;
        float4 v = ld4(A + (int64_t)gm * g.lda + gk, vecA, valid);
        if (PRO == PRO_A_K) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            f4(v, i) = (gk + i < K) ? fmaxf(fmaf(f4(v, i), psc[gk + i], psh[gk + i]), 0.f) : 0.f;
        }
        ra[rep] = v;
      }
      // ---- B tile: 16 (k) x 128 (n)
      if (!BKC) {
        const int k = (tid >> 5) + 8 * rep, nq = (tid & 31) * 4;
        const int gk = k0 + k, gn = n0 + nq;
        const int valid = (gk < K) ? min(4, max(0, N - gn)) : 0;
        float4 v = ld4(B + (int64_t)gk * g.ldb + gn, vecB, valid);
        if (PRO == PRO_B_K) {
          if (gk < K) {
            const float sc = psc[gk], sh = psh[gk];
#pragma unroll
            for (int i = 0; i < 4; ++i) f4(v, i) = fmaxf(fmaf(f4(v, i), sc, sh), 0.f);
          }
        } else if (PRO == PRO_B_SMX) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            f4(v, i) = (i < valid) ? expf(f4(v, i) - psc[gn + i]) * psh[gn + i] : 0.f;
        }
        rb[rep] = v;
      } else {
        const int n = (tid >> 2) + 64 * rep, kq = (tid & 3) * 4;
        const int gn = n0 + n, gk = k0 + kq;
        const int valid = (gn < N) ? min(4, max(0, K - gk)) : 0;
        float4 v = ld4(B + (int64_t)gn * g.ldb + gk, vecB, valid);
        if (PRO == PRO_B_K) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            f4(v, i) = (i < valid) ? fmaxf(fmaf(f4(v, i), psc[gk + i], psh[gk + i]), 0.f) : 0.f;
        } else if (PRO == PRO_B_SMX) {
          if (valid > 0) {
            const float mx = psc[gn], rs = psh[gn];
#pragma unroll
            for (int i = 0; i < 4; ++i) f4(v, i) = (i < valid) ? expf(f4(v, i) - mx) * rs : 0.f;
          }
        }
        rb[rep] = v;
      }
    }
  };

  auto store = [&](int buf) {
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      {
        const int m = (tid >> 2) + 64 * rep, kq = (tid & 3) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) As[buf][kq + i][m] = f4(ra[rep], i);
      }
      if (!BKC) {
        const int k = (tid >> 5) + 8 * rep, nq = (tid & 31) * 4;
        *reinterpret_cast<float4*>(&Bs[buf][k][nq]) = rb[rep];
      } else {
        const int n = (tid >> 2) + 64 * rep, kq = (tid & 3) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) Bs[buf][kq + i][n] = f4(rb[rep], i);
      }
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  const int khalf = lane >> 5, l32 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a0 = As[cur][kk + khalf][wm * 64 + l32];
      const float a1 = As[cur][kk + khalf][wm * 64 + 32 + l32];
      const float b0 = Bs[cur][kk + khalf][wn * 64 + l32];
      const float b1 = Bs[cur][kk + khalf][wn * 64 + 32 + l32];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ------------------------------------------------------------------ epilogue
  float* C = g.C + (int64_t)b * g.sCb;
  const float* Rr = RES ? g.R + (int64_t)b * g.sRb : nullptr;
  float colm[2], cols[2];  // COLSMX running (max, sum) / COL (sum, sumsq) for this lane's two columns
  colm[0] = colm[1] = (STATS == ST_COLSMX) ? NEG_BIG : 0.f;
  cols[0] = cols[1] = 0.f;

#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float sv[16], ss[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sv[r] = (STATS == ST_ROWSMX) ? NEG_BIG : 0.f;
      ss[r] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn * 64 + j * 32 + l32;
      const bool nok = gn < N;
      float bn_ = 0.f;
      if (BIAS == BIAS_N && nok) bn_ = g.bias[gn];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        const bool ok = nok && gm < M;
        float v = acc[i][j][r];
        if (BIAS == BIAS_M) v += (gm < M) ? g.bias[gm] : 0.f;
        if (BIAS == BIAS_N) v += bn_;
        if (RES && ok) v += Rr[(int64_t)gm * g.ldc + gn];
        if (ok) C[(int64_t)gm * g.ldc + gn] = v;
        if (STATS == ST_ROW) {
          if (ok) { sv[r] += v; ss[r] = fmaf(v, v, ss[r]); }
        } else if (STATS == ST_ROWSMX) {
          if (ok) smx_combine(sv[r], ss[r], v, 1.f);
        } else if (STATS == ST_COLSMX) {
          if (ok) smx_combine(colm[j], cols[j], v, 1.f);
        } else if (STATS == ST_COL) {
          if (ok) { colm[j] += v; cols[j] = fmaf(v, v, cols[j]); }
        }
      }
    }
    if (STATS == ST_ROW || STATS == ST_ROWSMX) {
      butterfly16<STATS == ST_ROWSMX>(sv, ss, lane);
      const int rho = ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
      const int row = wm * 64 + i * 32 + (rho & 3) + 8 * (rho >> 2) + 4 * khalf;
      if ((lane & 1) == 0) red[wn][row] = make_float2(sv[0], ss[0]);
    }
  }
  if (STATS == ST_ROW || STATS == ST_ROWSMX) {
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      float2 a = red[0][tid], c = red[1][tid];
      if (STATS == ST_ROW) {
        a.x += c.x;
        a.y += c.y;
      } else {
        smx_combine(a.x, a.y, c.x, c.y);
      }
      g.stats[((int64_t)b * gridDim.x + blockIdx.x) * g.st_ld + g.st_off + m0 + tid] = a;
    }
  }
  if (STATS == ST_COLSMX || STATS == ST_COL) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float om = __shfl_xor(colm[j], 32, 64), os = __shfl_xor(cols[j], 32, 64);
      if (STATS == ST_COLSMX) {
        smx_combine(colm[j], cols[j], om, os);
      } else {
        colm[j] += om;
        cols[j] += os;
      }
      if (khalf == 0) red[wm][wn * 64 + j * 32 + l32] = make_float2(colm[j], cols[j]);
    }
    __syncthreads();
    if (tid < BN && n0 + tid < N) {
      float2 a = red[0][tid], c = red[1][tid];
      if (STATS == ST_COLSMX) {
        smx_combine(a.x, a.y, c.x, c.y);
      } else {
        a.x += c.x;
        a.y += c.y;
      }
      g.stats[((int64_t)b * gridDim.y + blockIdx.y) * g.st_ld + g.st_off + n0 + tid] = a;
    }
  }
}

template <int PRO, int BKC, int BIAS, int STATS, int RES>
static void launch_t(const KArgs& ka, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm_kernel<PRO, BKC, BIAS, STATS, RES>), grid, dim3(256), 0, s, ka);
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int launch_gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return MVR_OK;
  if (!g.A || !g.B || !g.C) return MVR_EINVAL;
  if (g.K < 0) return MVR_EINVAL;
  if (g.pro != PRO_NONE && (!g.psc || !g.psh)) return MVR_EINVAL;
  if (g.stats_mode != ST_NONE && !g.stats) return MVR_EINVAL;
  if (g.bias_mode != BIAS_NONE && !g.bias) return MVR_EINVAL;
  if (g.has_res && !g.R) return MVR_EINVAL;
  KArgs ka;
  ka.g = g;
  ka.vecA = al16(g.A) && (g.lda % 4 == 0) && (g.sAb % 4 == 0);
  ka.vecB = al16(g.B) && (g.ldb % 4 == 0) && (g.sBb % 4 == 0);
  dim3 grid(gemm_ntiles(g.N), gemm_mtiles(g.M), g.batch);
  if (grid.y > 65535 || grid.z > 65535) return MVR_EINVAL;
  const double fl = 2.0 * g.M * g.N * (double)g.K * g.batch;
  const double by = 4.0 * ((double)g.M * g.K * (g.sAb ? g.batch : 1) + (double)g.K * g.N * (g.sBb ? g.batch : 1) +
                           (double)g.M * g.N * g.batch * (g.has_res ? 2 : 1));
  ProfScope prof(g.prof_kind, fl, by, s);
  // Dispatch only the combinations the OANet schedule uses (oanet.hip).
#define MVR_CASE(P, BKC_, BI, ST, RS)                                                                     \
  if (g.pro == P && g.bkc == BKC_ && g.bias_mode == BI && g.stats_mode == ST && (g.has_res != 0) == RS) { \
    launch_t<P, BKC_, BI, ST, RS>(ka, grid, s);                                                         \
    MVR_CHECK_LAUNCH();                                                                                  \
    return MVR_OK;                                                                                       \
  }
  MVR_CASE(PRO_NONE, 0, BIAS_M, ST_ROW, 0)      // conv1 (input -> 128)
  MVR_CASE(PRO_NONE, 0, BIAS_M, ST_NONE, 0)     // PointCN shortcut conv
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_ROW, 0)       // PointCN conv.3 / OAFilter conv1.3 (+stats)
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_NONE, 0)      // OAFilter conv1.3
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_COL, 0)       // OAFilter conv1.3, train-mode BN(points) stats
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_ROW, 1)       // PointCN conv.7 / OAFilter conv3.4 (+residual)
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_ROWSMX, 0)    // diff_pool embedding (softmax over points)
  MVR_CASE(PRO_B_K, 0, BIAS_M, ST_COLSMX, 0)    // diff_unpool embedding (softmax over clusters)
  MVR_CASE(PRO_B_SMX, 1, BIAS_NONE, ST_ROW, 0)  // diff_pool matmul  x . S^T
  MVR_CASE(PRO_B_SMX, 0, BIAS_NONE, ST_ROW, 0)  // diff_unpool matmul x_down . S
  MVR_CASE(PRO_A_K, 1, BIAS_N, ST_ROW, 1)       // OAFilter conv2 (spatial, on the transpose)
  MVR_CASE(PRO_NONE, 0, BIAS_NONE, ST_NONE, 0)  // plain batched GEMM (tests)
  MVR_CASE(PRO_NONE, 1, BIAS_NONE, ST_NONE, 0)
#undef MVR_CASE
  return MVR_EINVAL;
}

}  // namespace mvr

// C-ABI: one fused GEMM (exposed for unit tests and host-side composition).
extern "C" int mvr_gemm_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* B,
                            int64_t sBb, int64_t ldb, int b_kcontig, float* C, int64_t sCb, int64_t ldc,
                            const float* R, int64_t sRb, const float* bias, int bias_mode, const float* psc,
                            const float* psh, int64_t sPb, int pro, float* stats, int64_t st_ld, int st_off,
                            int stats_mode, hipStream_t stream) {
  mvr::GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.batch = batch;
  g.A = A; g.sAb = sAb; g.lda = lda;
  g.B = B; g.sBb = sBb; g.ldb = ldb; g.bkc = b_kcontig;
  g.C = C; g.sCb = sCb; g.ldc = ldc;
  g.R = R; g.sRb = sRb; g.has_res = R != nullptr;
  g.bias = bias; g.bias_mode = bias_mode;
  g.psc = psc; g.psh = psh; g.sPb = sPb; g.pro = pro;
  g.stats = reinterpret_cast<float2*>(stats); g.st_ld = st_ld; g.st_off = st_off; g.stats_mode = stats_mode;
  return mvr::launch_gemm(g, stream);
}
