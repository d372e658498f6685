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
  long long persist;  // v2: number of persistent workgroups
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
__device__ __forceinline__ float f4(const float4& v, int i) { return reinterpret_cast<const float*>(&v)[i]; }

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

// ============================================================================================
// v2: LDS-DMA staged variant (global_load_lds_dwordx4, no register staging), BK = 32.
//   * A is always row-major [M][K] ("x-major": k contiguous); B is [K][N] (k-major) or [N][K].
//   * x-major tiles land in LDS as [row][32] with the 16-byte chunks XOR-swizzled by (row & 7)
//     through the per-lane SOURCE address (the LDS write stays lane-linear), read back with
//     ds_read_b128 = 4 consecutive k.  The MFMA k order inside a BK step is permuted
//     (step s, lane half h -> k = 8*(s>>2) + 4h + (s&3)) identically for A and B, so every
//     k-major B value is read at its permuted row with ds_read_b32.
//   * prologue transforms (IN/BN/ReLU, softmax) are applied to the operand right after the
//     LDS read; the K tail is zeroed there (clamped loads keep every address in bounds).
//   * 2-stage ring: stage t+1 is in flight while stage t is multiplied; one barrier per stage.
// ============================================================================================
constexpr int G2_BK = 32;
constexpr int G2_KV = 512;  // max K with a per-k prologue vector held in LDS
constexpr int G2_STAGE = 128 * G2_BK;  // floats per operand per stage

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at lds_base + 16*l.
// Inline asm so that hipcc does not track it: the compiler otherwise drains every LDS-DMA in flight
// (s_waitcnt vmcnt(0)) before the next ds_read, which serialises the stage ring.  Completion is
// waited for explicitly (vmcnt) before the barrier that publishes the stage.
__device__ __forceinline__ void glds16(const float* src, float* lds_base) {
  const uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)lds_base;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
__device__ __forceinline__ void glds_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int PRO, int BKC, int BIAS, int STATS, int RES>
__global__ __launch_bounds__(256, 2) void gemm2_kernel(KArgs ka) {
  // Persistent: workgroup w owns tiles w, w + grid, ...; the 2-stage LDS-DMA ring runs across
  // tile boundaries, so the next tile's first stage (and its prologue vectors) is in flight while
  // the current tile finishes and runs its epilogue.
  const GemmArgs& g = ka.g;
  constexpr int VEC = G2_KV + 32;
  __shared__ __attribute__((aligned(16))) float smem[4 * G2_STAGE + 4 * VEC + 4 * BM];
  float* Asm = smem;                         // [2][128][32]
  float* Bsm = smem + 2 * G2_STAGE;          // [2][...]
  float* vec = smem + 4 * G2_STAGE;          // [2 tile parities][2 (scale|max), (shift|1/sum)][VEC]
  float2* red = reinterpret_cast<float2*>(vec + 4 * VEC);   // [2][128]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int kh = lane >> 5, l32 = lane & 31;
  const int M = g.M, N = g.N, K = g.K;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int ntiles = ntn * ntm * g.batch;
  const int nk = (K + G2_BK - 1) / G2_BK;
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int S = my_tiles * nk;
  if (S <= 0) return;

  auto tile_of = [&](int i, int& b, int& tm, int& tn) {
    const int t = blockIdx.x + i * gridDim.x;
    tn = t % ntn;
    const int r = t / ntn;
    tm = r % ntm;
    b = r / ntm;
  };

  // per-tile prologue vectors -> LDS (wave 0, LDS-DMA): per-k scale/shift (IN/BN) or per-column
  // softmax max / reciprocal sum
  auto issue_vec = [&](int par, int b, int n0) {
    if (wid != 0) return;
    if (PRO == PRO_A_K || PRO == PRO_B_K) {
      const float* ps = g.psc + (int64_t)b * g.sPb;
      const float* ph = g.psh + (int64_t)b * g.sPb;
      for (int c0 = 0; c0 < K / 4; c0 += 64) {
        if (c0 + lane < K / 4) {
          glds16(ps + 4 * (c0 + lane), vec + (2 * par) * VEC + 4 * c0);
          glds16(ph + 4 * (c0 + lane), vec + (2 * par + 1) * VEC + 4 * c0);
        }
      }
    } else if (PRO == PRO_B_SMX) {
      const int n = min(n0 + 4 * l32, N - 4);
      const float* src = (kh == 0 ? g.psc : g.psh) + (int64_t)b * g.sPb + n;
      glds16(src, vec + (2 * par) * VEC);   // lanes 0-31 -> max[128], lanes 32-63 -> rsum[128]
    }
  };

  auto issue = [&](int gs) {
    const int i = gs / nk, ks = gs - (gs / nk) * nk;
    int b, tm, tn;
    tile_of(i, b, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN, k0 = ks * G2_BK;
    if (ks == 0) issue_vec(i & 1, b, n0);
    float* As = Asm + (gs & 1) * G2_STAGE;
    float* Bs = Bsm + (gs & 1) * G2_STAGE;
    const float* A = g.A + (int64_t)b * g.sAb;
    const float* B = g.B + (int64_t)b * g.sBb;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int r = 32 * wid + 8 * ii + (lane >> 3);          // tile row
      const int c = (lane & 7) ^ (r & 7);                      // logical chunk held by this lane
      const int gm = min(m0 + r, M - 1);
      const int gk = min(k0 + 4 * c, K - 4);
      glds16(A + (int64_t)gm * g.lda + gk, As + (32 * wid + 8 * ii) * G2_BK);
    }
    if (!BKC) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int kr = 8 * wid + 2 * ii + (lane >> 5);
        const int gk = min(k0 + kr, K - 1);
        const int gn = min(n0 + 4 * (lane & 31), N - 4);
        glds16(B + (int64_t)gk * g.ldb + gn, Bs + (8 * wid + 2 * ii) * BN);
      }
    } else {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int r = 32 * wid + 8 * ii + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        const int gn = min(n0 + r, N - 1);
        const int gk = min(k0 + 4 * c, K - 4);
        glds16(B + (int64_t)gn * g.ldb + gk, Bs + (32 * wid + 8 * ii) * G2_BK);
      }
    }
  };

  floatx16 acc[2][2];
  float cmx[2] = {0.f, 0.f}, crs[2] = {0.f, 0.f};   // per-column softmax constants (PRO_B_SMX)

  issue(0);
  glds_wait_all();
  __syncthreads();
  if (S > 1) issue(1);
  for (int gs = 0; gs < S; ++gs) {
    const int i = gs / nk, ks = gs - (gs / nk) * nk;
    const int par = i & 1;
    const float* vsc = vec + (2 * par) * VEC;
    const float* vsh = vec + (2 * par + 1) * VEC;
    if (ks == 0) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ii][j][r] = 0.f;
      if (PRO == PRO_B_SMX) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          cmx[j] = vsc[wn * 64 + j * 32 + l32];
          crs[j] = vsc[BN + wn * 64 + j * 32 + l32];
        }
      }
    }
    const float* As = Asm + (gs & 1) * G2_STAGE;
    const float* Bs = Bsm + (gs & 1) * G2_STAGE;
    const int k0 = ks * G2_BK;
    const bool tail = k0 + G2_BK > K;
    // all operands of the stage -> registers (one LDS wait), transforms, then 64 MFMAs back to back
    float4 a4[2][4], b4[2][4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int q = 2 * s4 + kh;   // 16-byte chunk (4 consecutive k) of this lane half
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int x = wm * 64 + ii * 32 + l32;
        a4[ii][s4] = *reinterpret_cast<const float4*>(As + x * G2_BK + 4 * (q ^ (x & 7)));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int x = wn * 64 + j * 32 + l32;
        if (BKC) {
          b4[j][s4] = *reinterpret_cast<const float4*>(Bs + x * G2_BK + 4 * (q ^ (x & 7)));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) f4(b4[j][s4], e) = Bs[(4 * q + e) * BN + x];
        }
      }
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int kb = k0 + 4 * (2 * s4 + kh);
      if (PRO == PRO_A_K || PRO == PRO_B_K) {
        const float4 sc4 = *reinterpret_cast<const float4*>(vsc + kb);
        const float4 sh4 = *reinterpret_cast<const float4*>(vsh + kb);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = kb + e < K;
          if (PRO == PRO_A_K) {
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
              f4(a4[ii][s4], e) = ok ? fmaxf(fmaf(f4(a4[ii][s4], e), f4(sc4, e), f4(sh4, e)), 0.f) : 0.f;
          } else {
#pragma unroll
            for (int j = 0; j < 2; ++j)
              f4(b4[j][s4], e) = ok ? fmaxf(fmaf(f4(b4[j][s4], e), f4(sc4, e), f4(sh4, e)), 0.f) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = f4(b4[j][s4], e);
            if (PRO == PRO_B_SMX) v = expf(v - cmx[j]) * crs[j];
            if (tail && kb + e >= K) v = 0.f;
            f4(b4[j][s4], e) = v;
          }
      }
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4(a4[ii][s4], e), f4(b4[j][s4], e), acc[ii][j], 0, 0,
                                                              0);
    glds_wait_all();                                  // stage gs+1 (issued one stage ago) landed
    __syncthreads();                                  // ... for every wave; stage gs fully read
    if (gs + 2 < S) issue(gs + 2);
    if (ks != nk - 1) continue;

    // -------------------------------------------------------------- epilogue of tile i
    int b, tm, tn;
    tile_of(i, b, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    float* C = g.C + (int64_t)b * g.sCb;
    const float* Rr = RES ? g.R + (int64_t)b * g.sRb : nullptr;
    float colm[2], cols[2];
    colm[0] = colm[1] = (STATS == ST_COLSMX) ? NEG_BIG : 0.f;
    cols[0] = cols[1] = 0.f;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
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
          const int gm = m0 + wm * 64 + ii * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
          const bool ok = nok && gm < M;
          float v = acc[ii][j][r];
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
        const int row = wm * 64 + ii * 32 + (rho & 3) + 8 * (rho >> 2) + 4 * kh;
        if ((lane & 1) == 0) red[wn * BM + row] = make_float2(sv[0], ss[0]);
      }
    }
    if (STATS == ST_ROW || STATS == ST_ROWSMX) {
      __syncthreads();
      if (tid < BM && m0 + tid < M) {
        float2 a = red[tid], c = red[BM + tid];
        if (STATS == ST_ROW) {
          a.x += c.x;
          a.y += c.y;
        } else {
          smx_combine(a.x, a.y, c.x, c.y);
        }
        g.stats[((int64_t)b * ntn + tn) * g.st_ld + g.st_off + m0 + tid] = a;
      }
      __syncthreads();   // red reusable by the next tile
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
        if (kh == 0) red[wm * BN + wn * 64 + j * 32 + l32] = make_float2(colm[j], cols[j]);
      }
      __syncthreads();
      if (tid < BN && n0 + tid < N) {
        float2 a = red[tid], c = red[BN + tid];
        if (STATS == ST_COLSMX) {
          smx_combine(a.x, a.y, c.x, c.y);
        } else {
          a.x += c.x;
          a.y += c.y;
        }
        g.stats[((int64_t)b * ntm + tm) * g.st_ld + g.st_off + n0 + tid] = a;
      }
      __syncthreads();
    }
  }
}

template <int PRO, int BKC, int BIAS, int STATS, int RES>
static void launch_t2(const KArgs& ka, dim3 grid, hipStream_t s) {
  const long long tiles = (long long)grid.x * grid.y * grid.z;
  const unsigned wgs = (unsigned)(tiles < ka.persist ? tiles : ka.persist);
  hipLaunchKernelGGL((gemm2_kernel<PRO, BKC, BIAS, STATS, RES>), dim3(wgs), dim3(256), 0, s, ka);
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
  ka.persist = 2 * 256;  // 2 workgroups per CU (LDS-bound), 256 CUs
  dim3 grid(gemm_ntiles(g.N), gemm_mtiles(g.M), g.batch);
  if (grid.y > 65535 || grid.z > 65535) return MVR_EINVAL;
  const double fl = 2.0 * g.M * g.N * (double)g.K * g.batch;
  const double by = 4.0 * ((double)g.M * g.K * (g.sAb ? g.batch : 1) + (double)g.K * g.N * (g.sBb ? g.batch : 1) +
                           (double)g.M * g.N * g.batch * (g.has_res ? 2 : 1));
  ProfScope prof(g.prof_kind, fl, by, s);
  // v2 (LDS-DMA) needs 16-byte aligned rows everywhere it loads and K >= 4
  const bool vec_ok = (g.pro == PRO_NONE) ||
                      (al16(g.psc) && al16(g.psh) && (g.sPb % 4 == 0) && (g.pro != PRO_B_SMX || g.N % 4 == 0));
  const bool v2 = g.use_v1 == 0 && ka.vecA && ka.vecB && vec_ok && (g.K % 4 == 0) && g.K >= 4 &&
                  (g.N % 4 == 0 || g.bkc) && g.N >= 4 && ((g.pro != PRO_A_K && g.pro != PRO_B_K) || g.K <= G2_KV);
  // Dispatch only the combinations the OANet schedule uses (oanet.hip).
#define MVR_CASE(P, BKC_, BI, ST, RS)                                                                     \
  if (g.pro == P && g.bkc == BKC_ && g.bias_mode == BI && g.stats_mode == ST && (g.has_res != 0) == RS) { \
    if (v2) launch_t2<P, BKC_, BI, ST, RS>(ka, grid, s);                                                \
    else launch_t<P, BKC_, BI, ST, RS>(ka, grid, s);                                                    \
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
extern "C" int mvr_gemm_f32_variant(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* B,
                            int64_t sBb, int64_t ldb, int b_kcontig, float* C, int64_t sCb, int64_t ldc,
                            const float* R, int64_t sRb, const float* bias, int bias_mode, const float* psc,
                            const float* psh, int64_t sPb, int pro, float* stats, int64_t st_ld, int st_off,
                            int stats_mode, int use_v1, hipStream_t stream) {
  mvr::GemmArgs g{};
  g.use_v1 = use_v1;
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

extern "C" int mvr_gemm_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* B,
                            int64_t sBb, int64_t ldb, int b_kcontig, float* C, int64_t sCb, int64_t ldc,
                            const float* R, int64_t sRb, const float* bias, int bias_mode, const float* psc,
                            const float* psh, int64_t sPb, int pro, float* stats, int64_t st_ld, int st_off,
                            int stats_mode, hipStream_t stream) {
  return mvr_gemm_f32_variant(M, N, K, batch, A, sAb, lda, B, sBb, ldb, b_kcontig, C, sCb, ldc, R, sRb, bias,
                              bias_mode, psc, psh, sPb, pro, stats, st_ld, st_off, stats_mode, 0, stream);
}
