// Batched fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32,
// exact fp32 fma chains — no reduced-precision path, so OANet inlier masks match
// the fp32 reference).
//
//   C[b](m,n) = sum_k  pro_A(A[b](m,k)) * pro_B(B[b](k,n))  (+ bias) (+ R[b](m,n))
//
// with the OANet elementwise work fused in:
//   * prologue, applied to the operand right after its LDS read: InstanceNorm+BatchNorm+ReLU
//     folded to relu(x*sc[k]+sh[k]) on the reduction axis, or the per-tile softmax factor of
//     diff_pool / diff_unpool (oanet.py:106-128, see ST_ROWSMX / PRO_B_SMX in gemm.hpp);
//   * epilogue: bias, residual (PointCN / OAFilter shortcuts, oanet.py:39-42,87-92), the softmax
//     exponentials (one exp per element, normalised later by the consumer's factor) and the
//     partial statistics the NEXT layer needs.
//
// Schedule: persistent grid (2 workgroups per CU), 128x128 tile per 256-thread workgroup
// (4 waves in 2x2, each 64x64 = 2x2 MFMA 32x32 blocks), BK = 32, operands staged by
// global_load_lds_dwordx4 (no register staging) into a 2-stage LDS ring that runs across tile
// boundaries, so the next tile's loads overlap the current tile's epilogue.
//   * x-major tiles (k contiguous) land in LDS as [row][32] with the 16-byte chunks XOR-swizzled
//     by (row & 7) through the per-lane SOURCE address (the LDS write stays lane-linear), read
//     back with ds_read_b128 = 4 consecutive k.  The MFMA k order inside a stage is permuted
//     (step s, lane half h -> k = 8*(s>>2) + 4h + (s&3)) identically for A and B, so a k-major B
//     value is read at its permuted row with ds_read_b32.
//   * epilogue: each 4x4 quad of an accumulator block is transposed across its 4 lanes (DPP) so a
//     lane owns 4 consecutive columns of a row: float4 residual loads and stores, row statistics
//     reduced with 3 swizzles, column statistics with 2 DPP moves and one cross-half shuffle.
// Roofline: 2*M*N*K flops per GEMM against the 157.3 TF/s fp32 MFMA peak.
#include <atomic>
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "knobs.hpp"
#include "gemm.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"

#ifndef GEMM_EARLY
#define GEMM_EARLY 0   // 1: refill a stage's slot before its MFMAs (slower on the OAFilter shapes, the GEMM's only
                       // OANet users now: K = 128 0.085 vs 0.090 ms, K = 500 0.284 vs 0.297 ms per 435 pairs)
#endif

#ifndef GEMM_TRACE
#define GEMM_TRACE 0   // 1: per-phase cycle totals per wave (s_memtime), tools only
#endif

namespace mvr {

#if GEMM_TRACE
__device__ unsigned long long g_gemm_trace[8];
#define TSTAMP(slot)                                                   \
  do {                                                                 \
    unsigned long long t_;                                             \
    __builtin_amdgcn_sched_barrier(0);                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));  \
    __builtin_amdgcn_sched_barrier(0);                                 \
    tr[prev_slot] += t_ - t_last;                                      \
    t_last = t_;                                                       \
    prev_slot = (slot);                                                \
  } while (0)
#else
#define TSTAMP(slot) do {} while (0)
#endif


typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Which 16-byte chunk q (4 consecutive k of the 32-k stage) lane half h reads as its s4-th
// register: the 32x32x16 MFMA step st takes k = 16 st + 8h + j, i.e. chunks 4st + 2h and 4st + 2h + 1 as
// registers 2st, 2st + 1.
__device__ __forceinline__ int chunk_of(int s4, int h) { return 4 * (s4 >> 1) + 2 * h + (s4 & 1); }

constexpr int BM = GEMM_BM, BN = GEMM_BN, BK = GEMM_BK;
constexpr int KV_MAX = 512;        // max K with a per-k prologue vector held in LDS
constexpr int KV = KV_MAX + BK;    // vector slots: a stage may read up to 31 past K (zeros there)
constexpr int STAGE = 128 * BK;    // floats per operand per stage
constexpr float NEG_BIG = -3.0e38f;

struct KArgs {
  GemmArgs g;
  int persist;  // number of persistent workgroups
  int m_fast;   // tile order: m-tiles fastest (see tile_of)
  int* range; const int* guard; int epoch;   // MATH_F16X2 flag slot / MATH_BF16X3 re-run guard (pconv.hip scheme)
};

__device__ __forceinline__ float& f4(float4& v, int i) { return reinterpret_cast<float*>(&v)[i]; }
__device__ __forceinline__ float f4(const float4& v, int i) { return reinterpret_cast<const float*>(&v)[i]; }

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
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
// two LDS floats 128 floats (one k-major tile row) apart.  Inline asm: the compiler pairs the
// k-major reads across the wrong axis and shuffles registers; completion is awaited explicitly
// (lds_wait_all) before the values are used.
__device__ __forceinline__ f32x2 ds_read2_rows(uint32_t addr) {
  f32x2 r;
  asm volatile("ds_read2_b32 %0, %1 offset1:128" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
// lgkmcnt(0) with the 16 register pairs of the k-major reads as operands, so that the compiler
// cannot schedule any use of them before the wait (an asm output is "ready" at the asm otherwise)
__device__ __forceinline__ void lds_wait_regs(f32x2 (&r)[2][4][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(r[0][0][0]), "+v"(r[0][0][1]), "+v"(r[0][1][0]), "+v"(r[0][1][1]), "+v"(r[0][2][0]),
                 "+v"(r[0][2][1]), "+v"(r[0][3][0]), "+v"(r[0][3][1]), "+v"(r[1][0][0]), "+v"(r[1][0][1]),
                 "+v"(r[1][1][0]), "+v"(r[1][1][1]), "+v"(r[1][2][0]), "+v"(r[1][2][1]), "+v"(r[1][3][0]),
                 "+v"(r[1][3][1])
               :
               : "memory");
}
// workgroup barrier publishing LDS writes only (leaves LDS-DMA / global traffic in flight)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// cross-lane moves: DPP inside a quad of lanes, ds_swizzle (xor) inside a 32-lane half
__device__ __forceinline__ float dpp_x1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_x2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // quad_perm 2,3,0,1
}
template <int X>
__device__ __forceinline__ float swz(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (X << 10)));
}
// sum over the 8 lanes of a 32-lane half that share (lane & 3): two DPP row rotations (by 4 and 8
// lanes inside a 16-lane row, no LDS round trip) and one swizzle across the two rows
template <int R>
__device__ __forceinline__ float dpp_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8_p8(float v) {
  v += dpp_ror<4>(v);
  v += dpp_ror<8>(v);
  return v + swz<16>(v);
}

// 4x4 transpose across the 4 lanes t of a quad: on return register u of lane t holds what
// register t of lane u held.
__device__ __forceinline__ void quad_transpose(float& a0, float& a1, float& a2, float& a3, bool h1, bool h2) {
  {
    const float r = dpp_x1(h1 ? a0 : a1);
    if (h1) a0 = r; else a1 = r;
  }
  {
    const float r = dpp_x1(h1 ? a2 : a3);
    if (h1) a2 = r; else a3 = r;
  }
  {
    const float r = dpp_x2(h2 ? a0 : a2);
    if (h2) a0 = r; else a2 = r;
  }
  {
    const float r = dpp_x2(h2 ? a1 : a3);
    if (h2) a1 = r; else a3 = r;
  }
}

// 3-way bf16 split of 8 fp32 values (two float4 = 8 consecutive k) into MFMA fragments:
// x = h + m + l to 2^-25 |x| (RNE at each step; x - h and r - m are exact in fp32).  Works on
// packed pairs: v_cvt_pk_bf16_f32, shift/and unpack, v_pk_add_f32 — 4.5 VALU ops per value.
__device__ __forceinline__ unsigned cvt_pk_bf16(f32x2 x) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
}
__device__ __forceinline__ f32x2 unpack_bf16(unsigned p) {
  f32x2 r;
  r.x = __uint_as_float(p << 16);
  r.y = __uint_as_float(p & 0xffff0000u);
  return r;
}
__device__ __forceinline__ void split8(const float4& a, const float4& b, u32x4& H, u32x4& Mm, u32x4& L) {
  const f32x2 x[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned hp = cvt_pk_bf16(x[i]);
    const f32x2 r = bx::sub2(x[i], unpack_bf16(hp));
    const unsigned mp = cvt_pk_bf16(r);
    H[i] = hp;
    Mm[i] = mp;
    L[i] = cvt_pk_bf16(bx::sub2(r, unpack_bf16(mp)));
  }
}
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf16x8& h, bf16x8& m, bf16x8& l) {
  u32x4 H, Mm, L;
  split8(a, b, H, Mm, L);
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, Mm);
  l = __builtin_bit_cast(bf16x8, L);
}

// exp(x) for the softmax epilogues on v_exp_f32 (relative error ~1e-6 for |x| <= 20, against the
// ~1e-4 tolerance of the scores; the argument is <= 0 here)
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// Persistent-grid slot of this workgroup, XCD-aware: workgroups are dispatched round-robin over the
// 8 XCDs (each with its own L2), so consecutive tile indices (which share an operand: the n-tiles
// of one pair reuse its A rows, the m-tiles its B columns) are given to workgroups of one XCD.
__device__ __forceinline__ int xcd_slot() {
  const int G = gridDim.x, w = blockIdx.x;
  return (G & 7) ? w : (w & 7) * (G >> 3) + (w >> 3);
}

// Epilogue of one 128x128 tile from the 2x2-wave accumulator layout (MFMA 32x32 C map): bias,
// residual, softmax exponentials, stores and partial statistics (see gemm.hpp Stats).  After the
// quad transpose, value v[ii][j][q] (float4) of this lane is
//   C(m0 + 64wm + 32ii + 8q + 4kh + t4,  n0 + 64wn + 32j + 4p8 + u),  u = 0..3
// red / redm: LDS scratch ([2][128] float2 / float); the caller guarantees a workgroup barrier
// between two epilogues.
template <int BIAS, int STATS, int RES>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& g, floatx16 (&acc)[2][2], int b, int tm, int tn,
                                              float2* red, float* redm) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int kh = lane >> 5, l32 = lane & 31;
  const int t4 = lane & 3, p8 = l32 >> 2;
  const bool h1 = (t4 & 1) != 0, h2 = (t4 & 2) != 0;
  const int M = g.M, N = g.N;
  const int N4 = (N + 3) & ~3;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int m0 = tm * BM, n0 = tn * BN;
  float* C = g.C + (int64_t)b * g.sCb;
  if (STATS == ST_NONE || STATS == ST_ROW) {
    // row-local work: one 32-row block at a time (half the live registers of the general path)
    const int nw = min(max(N - (n0 + wn * 64), 0), 64);   // valid columns of this wave
    const float rnw = nw > 0 ? 1.f / (float)nw : 0.f;
    bool cok[2][4], sok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn * 64 + j * 32 + 4 * p8;
      sok[j] = gn < N4;
#pragma unroll
      for (int u = 0; u < 4; ++u) cok[j][u] = gn + u < N;
    }
    float bn[2][4];
    if (BIAS == BIAS_N) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) bn[j][u] = cok[j][u] ? g.bias[n0 + wn * 64 + j * 32 + 4 * p8 + u] : 0.f;
    }
    // all global loads of the epilogue up front (one latency): row biases and both blocks' residuals
    float bm[2][4];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bm[ii][q] = BIAS == BIAS_M ? g.bias[min(m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4, M - 1)] : 0.f;
    float4 w[2][2][4];
    if (RES) {
      const float* Rr = g.R + (int64_t)b * g.sRb;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gm = min(m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4, M - 1);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int gn = min(n0 + wn * 64 + j * 32 + 4 * p8, N4 - 4);
            w[ii][j][q] = *reinterpret_cast<const float4*>(Rr + (int64_t)gm * g.ldc + gn);
          }
        }
    }
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gm = m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
        const bool rok = gm < M;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float a0 = acc[ii][j][4 * q], a1 = acc[ii][j][4 * q + 1], a2 = acc[ii][j][4 * q + 2],
                a3 = acc[ii][j][4 * q + 3];
          quad_transpose(a0, a1, a2, a3, h1, h2);
          const float bq = bm[ii][q];
          float4 x = make_float4(a0 + bq, a1 + bq, a2 + bq, a3 + bq);
          if (BIAS == BIAS_N) { x.x += bn[j][0]; x.y += bn[j][1]; x.z += bn[j][2]; x.w += bn[j][3]; }
          if (RES) { x.x += w[ii][j][q].x; x.y += w[ii][j][q].y; x.z += w[ii][j][q].z; x.w += w[ii][j][q].w; }
          w[ii][j][q] = x;
          if (rok && sok[j] && !g.no_store)
            *reinterpret_cast<float4*>(C + (int64_t)gm * g.ldc + n0 + wn * 64 + j * 32 + 4 * p8) = x;
        }
      }
      if (STATS == ST_ROW) {   // (sum, squared deviations from the wave-local mean) of each row
        float sm[4], s2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sm[q] = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) sm[q] += cok[j][u] ? f4(w[ii][j][q], u) : 0.f;
          sm[q] = sum8_p8(sm[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float mu = sm[q] * rnw;
          s2[q] = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float d = cok[j][u] ? f4(w[ii][j][q], u) - mu : 0.f;
              s2[q] = fmaf(d, d, s2[q]);
            }
          s2[q] = sum8_p8(s2[q]);
        }
        if (p8 == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) red[wn * BM + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4] = make_float2(sm[q], s2[q]);
        }
      }
    }
    if (STATS == ST_ROW) {
      lds_barrier();
      if (tid < BM && m0 + tid < M) {
        const float2 x = red[tid], c = red[BM + tid];
        const int na = min(N - n0, 64), nb = min(max(N - n0 - 64, 0), 64);
        float2 o = x;
        if (nb > 0) {
          const float d = c.x / (float)nb - x.x / (float)na;
          o = make_float2(x.x + c.x, x.y + c.y + d * d * ((float)na * (float)nb / (float)(na + nb)));
        }
        g.stats[((int64_t)b * ntn + tn) * g.st_ld + g.st_off + m0 + tid] = o;
      }
    }
    return;
  }
  float4 v[2][2][4];
#pragma unroll
  for (int ii = 0; ii < 2; ++ii) {
    asm volatile("" ::: "memory");   // keep each block's residual loads in its own iteration (VGPRs)
    if (RES) {   // residual rows of this 32-row block (loads issued before the transposes)
      const float* Rr = g.R + (int64_t)b * g.sRb;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gm = min(m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4, M - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int gn = min(n0 + wn * 64 + j * 32 + 4 * p8, N4 - 4);
          v[ii][j][q] = *reinterpret_cast<const float4*>(Rr + (int64_t)gm * g.ldc + gn);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a0 = acc[ii][j][4 * q], a1 = acc[ii][j][4 * q + 1], a2 = acc[ii][j][4 * q + 2],
              a3 = acc[ii][j][4 * q + 3];
        quad_transpose(a0, a1, a2, a3, h1, h2);
        if (RES) {
          v[ii][j][q].x += a0; v[ii][j][q].y += a1; v[ii][j][q].z += a2; v[ii][j][q].w += a3;
        } else {
          v[ii][j][q] = make_float4(a0, a1, a2, a3);
        }
      }
  }
  // validity: rows, columns (per component), float4 stores inside the padded row
  bool rok[2][4];
  bool cok[2][4];
  bool sok[2];
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int q = 0; q < 4; ++q) rok[ii][q] = m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4 < M;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int gn = n0 + wn * 64 + j * 32 + 4 * p8;
    sok[j] = gn < N4;
#pragma unroll
    for (int u = 0; u < 4; ++u) cok[j][u] = gn + u < N;
  }
  if (BIAS == BIAS_M) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float bm = g.bias[min(m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4, M - 1)];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          v[ii][j][q].x += bm; v[ii][j][q].y += bm; v[ii][j][q].z += bm; v[ii][j][q].w += bm;
        }
      }
  } else if (BIAS == BIAS_N) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn * 64 + j * 32 + 4 * p8;
      float bn[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) bn[u] = cok[j][u] ? g.bias[gn + u] : 0.f;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) f4(v[ii][j][q], u) += bn[u];
    }
  }

  if (STATS == ST_ROWSMX) {
    // tile row maxima -> exp(v - max) in place
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float mx = NEG_BIG;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (cok[j][u]) mx = fmaxf(mx, f4(v[ii][j][q], u));
        mx = fmaxf(mx, swz<4>(mx));
        mx = fmaxf(mx, swz<8>(mx));
        mx = fmaxf(mx, swz<16>(mx));
        if (p8 == 0) redm[wn * BM + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4] = mx;
      }
    lds_barrier();
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
        const float mx = fmaxf(redm[rl], redm[BM + rl]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u)
            f4(v[ii][j][q], u) = (rok[ii][q] && cok[j][u]) ? fast_exp(f4(v[ii][j][q], u) - mx) : 0.f;
      }
  } else if (STATS == ST_COLSMX) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float4 cm = make_float4(NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG);
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (rok[ii][q]) {
#pragma unroll
            for (int u = 0; u < 4; ++u) f4(cm, u) = fmaxf(f4(cm, u), f4(v[ii][j][q], u));
          }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float x = f4(cm, u);
        x = fmaxf(x, dpp_x1(x));
        x = fmaxf(x, dpp_x2(x));
        x = fmaxf(x, __shfl_xor(x, 32, 64));
        f4(cm, u) = x;
      }
      const float mine = t4 == 0 ? cm.x : t4 == 1 ? cm.y : t4 == 2 ? cm.z : cm.w;
      if (kh == 0) redm[wm * BN + wn * 64 + j * 32 + 4 * p8 + t4] = mine;
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = wn * 64 + j * 32 + 4 * p8;
      const float4 c0 = *reinterpret_cast<const float4*>(redm + cl);
      const float4 c1 = *reinterpret_cast<const float4*>(redm + BN + cl);
      float mx[4] = {fmaxf(c0.x, c1.x), fmaxf(c0.y, c1.y), fmaxf(c0.z, c1.z), fmaxf(c0.w, c1.w)};
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u)
            f4(v[ii][j][q], u) = (rok[ii][q] && cok[j][u]) ? fast_exp(f4(v[ii][j][q], u) - mx[u]) : 0.f;
    }
  }

  // stores (full float4 inside the padded row)
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!rok[ii][q]) continue;
      const int gm = m0 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int gn = n0 + wn * 64 + j * 32 + 4 * p8;
        if (sok[j]) *reinterpret_cast<float4*>(C + (int64_t)gm * g.ldc + gn) = v[ii][j][q];
      }
    }

  // Statistics.  ST_ROW / ST_COL: per wave (64 columns / rows) the sum and the sum of squared
  // deviations from the wave-local mean, merged across the two waves with Chan's formula — a
  // two-pass variance per tile (sum-of-squares minus squared mean cancels catastrophically for
  // InstanceNorm inputs whose mean is large against their spread).
  if (STATS == ST_ROW || STATS == ST_ROWSMX) {
    const int nw = min(max(N - (n0 + wn * 64), 0), 64);   // valid columns of this wave
    const float rnw = nw > 0 ? 1.f / (float)nw : 0.f;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) s += cok[j][u] ? f4(v[ii][j][q], u) : 0.f;
        s += swz<4>(s);
        s += swz<8>(s);
        s += swz<16>(s);
        if (STATS == ST_ROW) {
          const float mu = s * rnw;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float d = cok[j][u] ? f4(v[ii][j][q], u) - mu : 0.f;
              s2 = fmaf(d, d, s2);
            }
          s2 += swz<4>(s2);
          s2 += swz<8>(s2);
          s2 += swz<16>(s2);
        }
        if (p8 == 0) red[wn * BM + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4] = make_float2(s, s2);
      }
    lds_barrier();
    if (tid < BM && m0 + tid < M) {
      const float2 a = red[tid], c = red[BM + tid];
      float2 o;
      if (STATS == ST_ROW) {
        const int na = min(N - n0, 64), nb = min(max(N - n0 - 64, 0), 64);
        o = a;
        if (nb > 0) {
          const float d = c.x / (float)nb - a.x / (float)na;
          o = make_float2(a.x + c.x, a.y + c.y + d * d * ((float)na * (float)nb / (float)(na + nb)));
        }
      } else {
        o = make_float2(fmaxf(redm[tid], redm[BM + tid]), a.x + c.x);
      }
      g.stats[((int64_t)b * ntn + tn) * g.st_ld + g.st_off + m0 + tid] = o;
    }
  } else if (STATS == ST_COL || STATS == ST_COLSMX) {
    const int nw = min(max(M - (m0 + wm * 64), 0), 64);   // valid rows of this wave
    const float rnw = nw > 0 ? 1.f / (float)nw : 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float s[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) s[u] += rok[ii][q] ? f4(v[ii][j][q], u) : 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s[u] += dpp_x1(s[u]);
        s[u] += dpp_x2(s[u]);
        s[u] += __shfl_xor(s[u], 32, 64);
      }
      if (STATS == ST_COL) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float mu = s[u] * rnw;
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float d = rok[ii][q] ? f4(v[ii][j][q], u) - mu : 0.f;
              s2[u] = fmaf(d, d, s2[u]);
            }
          s2[u] += dpp_x1(s2[u]);
          s2[u] += dpp_x2(s2[u]);
          s2[u] += __shfl_xor(s2[u], 32, 64);
        }
      }
      const float ms = t4 == 0 ? s[0] : t4 == 1 ? s[1] : t4 == 2 ? s[2] : s[3];
      const float ms2 = t4 == 0 ? s2[0] : t4 == 1 ? s2[1] : t4 == 2 ? s2[2] : s2[3];
      if (kh == 0) red[wm * BN + wn * 64 + j * 32 + 4 * p8 + t4] = make_float2(ms, ms2);
    }
    lds_barrier();
    if (tid < BN && n0 + tid < N) {
      const float2 a = red[tid], c = red[BN + tid];
      float2 o;
      if (STATS == ST_COL) {
        const int na = min(M - m0, 64), nb = min(max(M - m0 - 64, 0), 64);
        o = a;
        if (nb > 0) {
          const float d = c.x / (float)nb - a.x / (float)na;
          o = make_float2(a.x + c.x, a.y + c.y + d * d * ((float)na * (float)nb / (float)(na + nb)));
        }
      } else {
        o = make_float2(fmaxf(redm[tid], redm[BN + tid]), a.x + c.x);
      }
      g.stats[((int64_t)b * ntm + tm) * g.st_ld + g.st_off + n0 + tid] = o;
    }
  }
}

template <int MATH, int PRO, int BKC, int BIAS, int STATS, int RES>
__global__ __launch_bounds__(256, 2) void gemm_kernel(KArgs ka) {
  // Persistent: workgroup w owns tiles w, w + grid, ...
  const GemmArgs& g = ka.g;
  __shared__ __attribute__((aligned(16))) float smem[4 * STAGE + 4 * KV + 2 * BN + 4 * BM + 2 * BM];
  float* Asm = smem;                          // [2][128][32]
  float* Bsm = smem + 2 * STAGE;              // [2][...]
  float* vec = smem + 4 * STAGE;              // [2 tile parities][scale | shift][KV]
  float* fac = vec + 4 * KV;                  // [2 stages][128] softmax factors (PRO_B_SMX)
  float2* red = reinterpret_cast<float2*>(fac + 2 * BN);    // [2][128] partial statistics
  float* redm = fac + 2 * BN + 4 * BM;                      // [2][128] tile maxima (softmax)
  if (ka.guard && *ka.guard != ka.epoch) return;   // uniform: the split-fp16 launch stayed in its window
  float amx = 0.f, bmx = 0.f;   // MATH_F16X2: max |A| x 2^6, |B| x 2^6 this lane split

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int kh = lane >> 5, l32 = lane & 31;
  const int M = g.M, N = g.N, K = g.K;
  const int N4 = (N + 3) & ~3, K4 = (K + 3) & ~3;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int ntiles = ntn * ntm * g.batch;
  const int nk = (K + BK - 1) / BK;
  const int my_tiles = (ntiles - xcd_slot() + (int)gridDim.x - 1) / (int)gridDim.x;
  const int S = my_tiles * nk;
  if (S <= 0) return;

  // tile order: consecutive tiles share the operand that is re-read from HBM — the m-tiles of one
  // B column block when A is batch-shared weights (L2-resident), else the n-tiles of one A row block
  auto tile_of = [&](int i, int& b, int& tm, int& tn) {
    const int t = xcd_slot() + i * gridDim.x;
    if (ka.m_fast) {
      tm = t % ntm;
      const int r = t / ntm;
      tn = r % ntn;
      b = r / ntn;
    } else {
      tn = t % ntn;
      const int r = t / ntn;
      tm = r % ntm;
      b = r / ntm;
    }
  };

  // per-tile prologue vectors -> LDS (wave 0): per-k scale/shift (IN/BN)
  auto issue_vec = [&](int par, int b) {
    if (wid != 0) return;
    const float* ps = g.psc + (int64_t)b * g.sPb;
    const float* ph = g.psh + (int64_t)b * g.sPb;
    for (int c0 = 0; c0 < K / 4; c0 += 64) {
      if (c0 + lane < K / 4) {
        glds16(ps + 4 * (c0 + lane), vec + (2 * par) * KV + 4 * c0);
        glds16(ph + 4 * (c0 + lane), vec + (2 * par + 1) * KV + 4 * c0);
      }
    }
  };

  // stage issue: stages run tile-major (tile i of this workgroup, k step ks), tracked incrementally
  int is_i = 0, is_ks = 0, is_b = 0, is_m0 = 0, is_n0 = 0;
  // per-tile int32 element offsets of this lane's LDS-DMA sources (k0 = 0); x-major tiles put
  // logical 16-byte chunk lc of row (lane >> 3) into LDS slot (lane & 7)
  const int lc = (lane & 7) ^ ((lane >> 3) & 7);
  int a_off[4], b_off[4];
  const float* Ab = g.A;
  const float* Bb = g.B;
  auto issue = [&](int gs) {
    if (is_ks == 0) {
      int tm, tn;
      tile_of(is_i, is_b, tm, tn);
      is_m0 = tm * BM;
      is_n0 = tn * BN;
      if (PRO == PRO_A_K || PRO == PRO_B_K) issue_vec(is_i & 1, is_b);
      Ab = g.A + (int64_t)is_b * g.sAb;
      Bb = g.B + (int64_t)is_b * g.sBb;
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int r = 32 * wid + 8 * ii + (lane >> 3);
        a_off[ii] = min(is_m0 + r, M - 1) * (int)g.lda + 4 * lc;
        if (!BKC)
          b_off[ii] = (8 * wid + 2 * ii + (lane >> 5)) * (int)g.ldb + min(is_n0 + 4 * (lane & 31), N4 - 4);
        else
          b_off[ii] = min(is_n0 + r, N - 1) * (int)g.ldb + 4 * lc;
      }
    }
    const int b = is_b, n0 = is_n0, k0 = is_ks * BK;
    if (++is_ks == nk) {
      is_ks = 0;
      ++is_i;
    }
    if (PRO == PRO_B_SMX && wid == 0 && lane < 32) {
      const int n = min(n0 + 4 * lane, N4 - 4);
      glds16(g.psc + (int64_t)b * g.sPb + (int64_t)(k0 / 128) * g.pld + n, fac + (gs & 1) * BN);
    }
    float* As = Asm + (gs & 1) * STAGE;
    float* Bs = Bsm + (gs & 1) * STAGE;
    if (k0 + BK <= K) {   // full stage: no clamping
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) glds16(Ab + a_off[ii] + k0, As + (32 * wid + 8 * ii) * BK);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        if (!BKC)
          glds16(Bb + (b_off[ii] + (int64_t)k0 * g.ldb), Bs + (8 * wid + 2 * ii) * BN);
        else
          glds16(Bb + b_off[ii] + k0, Bs + (32 * wid + 8 * ii) * BK);
      }
    } else {              // K tail: clamp every source into the padded rows
      const int gk = min(k0 + 4 * lc, K4 - 4) - 4 * lc;
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) glds16(Ab + a_off[ii] + gk, As + (32 * wid + 8 * ii) * BK);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        if (!BKC) {
          const int kr = 8 * wid + 2 * ii + (lane >> 5);
          const int64_t o = b_off[ii] + (int64_t)(min(k0 + kr, K - 1) - kr) * g.ldb;
          glds16(Bb + o, Bs + (8 * wid + 2 * ii) * BN);
        } else {
          glds16(Bb + b_off[ii] + gk, Bs + (32 * wid + 8 * ii) * BK);
        }
      }
    }
  };

  floatx16 acc[2][2];

  if (PRO == PRO_A_K || PRO == PRO_B_K) {   // zero scale/shift past K (see the K-tail note below)
    for (int e = tid; e < 4 * KV; e += 256) vec[e] = 0.f;
    lds_barrier();
  }
  // Stage ring (2 LDS slots).  Early issue: once every wave holds stage gs in registers, slot gs&1
  // is refilled with stage gs + 2, so two stages are in flight during stage gs's MFMAs.  A per-tile
  // prologue vector issued with stage gs + 2 may then belong to tile i + 2 (same parity slot as the
  // tile being multiplied) when a tile has a single stage: those GEMMs refill after the MFMAs.
  const bool early = GEMM_EARLY && !((PRO == PRO_A_K || PRO == PRO_B_K) && nk < 2);
#if GEMM_TRACE
  unsigned long long tr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = __builtin_amdgcn_s_memtime();
  int prev_slot = 7;
#endif
  issue(0);
  glds_wait_all();
  __syncthreads();
  if (S > 1) issue(1);
  int i = 0, ks = -1;   // tile / k step of the stage being multiplied
  for (int gs = 0; gs < S; ++gs) {
    if (++ks == nk) {
      ks = 0;
      ++i;
    }
    TSTAMP(0);
    if (early && gs > 0) {
      // stage gs landed: loads complete in order, and stage gs + 1 (if issued) put at least 8
      // younger LDS-DMAs per lane behind it (4 A + 4 B chunks)
      if (gs + 1 < S) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    }
    const int par = i & 1;
    const float* vsc = vec + (2 * par) * KV;
    const float* vsh = vec + (2 * par + 1) * KV;
    if (ks == 0) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ii][j][r] = 0.f;
    }
    const float* As = Asm + (gs & 1) * STAGE;
    const float* Bs = Bsm + (gs & 1) * STAGE;
    const int k0 = ks * BK;
    // K tail: rows k >= K of the stage must contribute nothing.  Prologue transforms see zero
    // scale/shift there (the vector area is zero-filled past K); untransformed / softmax-scaled
    // B operands are zeroed in LDS.
    if ((PRO == PRO_NONE || PRO == PRO_B_SMX) && k0 + BK > K) {
      float* Bz = Bsm + (gs & 1) * STAGE;
      const int kv = K - k0;   // valid k of this stage (1..31)
      for (int e = tid; e < STAGE; e += 256) {
        const int k = BKC ? 4 * ((e & 31) >> 2 ^ ((e >> 5) & 7)) + (e & 3) : e / BN;
        if (k >= kv) Bz[e] = 0.f;
      }
      lds_barrier();
    }
    // all operands of the stage -> registers (one LDS wait), transforms, then 64 MFMAs back to back
    float4 a4[2][4], b4[2][4];
    f32x2 bkr[2][4][2];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int q = chunk_of(s4, kh);   // 16-byte chunk (4 consecutive k) of this lane half
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int x = wm * 64 + ii * 32 + l32;
        a4[ii][s4] = *reinterpret_cast<const float4*>(As + x * BK + 4 * (q ^ (x & 7)));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int x = wn * 64 + j * 32 + l32;
        if (BKC) {
          b4[j][s4] = *reinterpret_cast<const float4*>(Bs + x * BK + 4 * (q ^ (x & 7)));
        } else {
          // rows 4q..4q+3 of the k-major tile: two ds_read2_b32 (row pairs 128 floats apart)
          const uint32_t la = lds_addr(Bs + (4 * q) * BN + x);
          bkr[j][s4][0] = ds_read2_rows(la);
          bkr[j][s4][1] = ds_read2_rows(la + 2 * BN * 4);
        }
      }
    }
    float fm[2] = {1.f, 1.f};
    if (PRO == PRO_B_SMX) {
#pragma unroll
      for (int j = 0; j < 2; ++j) fm[j] = fac[(gs & 1) * BN + wn * 64 + j * 32 + l32];
    }
    if (!BKC) {
      lds_wait_regs(bkr);   // the asm reads' registers are tied to the wait: no use can move above it
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          b4[j][s4] = make_float4(bkr[j][s4][0].x, bkr[j][s4][0].y, bkr[j][s4][1].x, bkr[j][s4][1].y);
    }
    TSTAMP(2);
    if (early) {
      lds_barrier();                                  // every wave holds stage gs: refill its slot
      if (gs + 2 < S) issue(gs + 2);
    }
    TSTAMP(3);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int kb = k0 + 4 * chunk_of(s4, kh);
      if (PRO == PRO_A_K || PRO == PRO_B_K) {
        const float4 sc4 = *reinterpret_cast<const float4*>(vsc + kb);
        const float4 sh4 = *reinterpret_cast<const float4*>(vsh + kb);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (PRO == PRO_A_K) {
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
              f4(a4[ii][s4], e) = fmaxf(fmaf(f4(a4[ii][s4], e), f4(sc4, e), f4(sh4, e)), 0.f);
          } else {
#pragma unroll
            for (int j = 0; j < 2; ++j)
              f4(b4[j][s4], e) = fmaxf(fmaf(f4(b4[j][s4], e), f4(sc4, e), f4(sh4, e)), 0.f);
          }
        }
      } else if (PRO == PRO_B_SMX) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) f4(b4[j][s4], e) *= fm[j];
      }
    }
    if (MATH == MATH_F16X2) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bx::FragT<1> fa[2], fb[2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const float4 u0 = a4[ii][2 * st], u1 = a4[ii][2 * st + 1];
          float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] *= 64.f;
            amx = fmaxf(amx, fabsf(v[e]));
          }
          fa[ii] = bx::split8t<1>(v);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 u0 = b4[j][2 * st], u1 = b4[j][2 * st + 1];
          float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] *= 64.f;
            bmx = fmaxf(bmx, fabsf(v[e]));
          }
          fb[j] = bx::split8t<1>(v);
        }
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[ii][j] = bx::mma<1>(fa[ii], fb[j], acc[ii][j]);
      }
    } else {
      // two k16 steps; lane half h holds k = 16s + 8h + (0..7) = chunks (2s, 2s+1) of its registers
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) split8(a4[ii][2 * st], a4[ii][2 * st + 1], ah[ii], am[ii], al[ii]);
#pragma unroll
        for (int j = 0; j < 2; ++j) split8(b4[j][2 * st], b4[j][2 * st + 1], bh[j], bm[j], bl[j]);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // small terms first
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[ii], bh[j], acc[ii][j], 0, 0, 0);
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ii], bl[j], acc[ii][j], 0, 0, 0);
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[ii], bm[j], acc[ii][j], 0, 0, 0);
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[ii], bh[j], acc[ii][j], 0, 0, 0);
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ii], bm[j], acc[ii][j], 0, 0, 0);
            acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ii], bh[j], acc[ii][j], 0, 0, 0);
          }
      }
    }
    TSTAMP(4);
    if (!early) {
      glds_wait_all();                                // stage gs+1 (issued one stage ago) landed
      __syncthreads();                                // ... for every wave; stage gs fully read
      if (gs + 2 < S) issue(gs + 2);
    }
    if (ks != nk - 1) continue;

    // -------------------------------------------------------------- epilogue of tile i
    // after the quad transpose, value v[ii][j][q] (float4) of this lane is
    //   C(m0 + 64wm + 32ii + 8q + 4kh + t4,  n0 + 64wn + 32j + 4p8 + u),  u = 0..3
    int b, tm, tn;
    tile_of(i, b, tm, tn);
    TSTAMP(5);
    if (MATH == MATH_F16X2) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[ii][j] *= 1.f / 4096.f;   // the operands' 2^6 x 2^6
    }
    tile_epilogue<BIAS, STATS, RES>(g, acc, b, tm, tn, red, redm);
    TSTAMP(6);
    // (red / redm are next written in the next tile's epilogue, after at least one stage barrier)
  }
#if GEMM_TRACE
  TSTAMP(7);
  if (lane == 0)
    for (int q = 0; q < 8; ++q) atomicAdd(&g_gemm_trace[q], tr[q]);
#endif
  if (MATH == MATH_F16X2) {   // outside the window: past 65504 (1023.5 unscaled), or nonzero but all below 2^-9
    const bool bad = !(amx < bx::F16_RANGE) || !(bmx < bx::F16_RANGE) || (amx > 0.f && amx < 0.125f) ||
                     (bmx > 0.f && bmx < 0.125f);
    if (__any(bad) && lane == 0) atomicExch(ka.range, ka.epoch);
  }
}

// ------------------------------------------------------------------------------------------------------------
// OAFilter conv2 (oanet.py:72-81, the 1x1 conv over clusters run on the transpose, oanet.hip oafilter):
//   C[b](m, n) = sum_k relu(A[b](m, k) sc[b][k] + sh[b][k]) W(n, k) + bias[n] + R[b](m, n),   m < 128
// with W [N][K] shared by every pair and per-128-column row statistics (ST_ROW).  Split once: the generic kernel
// above re-splits every A element in the two waves that share its rows and every B element in the two that share
// its columns, per stage; here
//   * W is split into its three bf16 planes once per launch (oaf_w_image_kernel, 1.5 MB for 500 x 500), in the
//     exact LDS image order, and staged by LDS-DMA;
//   * the A slab of a stage is loaded into registers one stage ahead (fp32, 32 B per thread), folded (BN + ReLU)
//     and split by the whole workgroup, each element once, into three LDS planes — in the middle of the previous
//     stage's MFMAs;
//   * one 512-thread workgroup per CU computes a 128 x 256 tile (8 waves of 64 x 64): A is read once per 256
//     columns, and the MFMA fragments come straight from the planes by ds_read_b128.
// Planes are [rows][32 k] bf16 (64-byte rows) with the 16-byte chunk c of row r stored at c ^ ((r >> 2) & 3):
// every ds_read_b128 lane group (MI355X_MICROARCH §LDS) then covers 16 distinct 16-byte slots of the 256-byte
// bank row.  K % 4 == 0 (the PRO_A_K contract); M == 128.
constexpr int C2_BN = 256, C2_BK = 32, C2_THREADS = 512;
constexpr int C2_APL = 128 * C2_BK;                  // bf16 per A plane and stage (8 KB)
constexpr int C2_BPL = C2_BN * C2_BK;                // bf16 per B plane and stage (16 KB)
constexpr int C2_SLOT = 3 * (C2_APL + C2_BPL);       // bf16 per stage slot (72 KB)
constexpr int C2_KMAX = 512;                         // largest K (the per-tile fold vectors live in LDS)
#ifndef C2_RPRE
#define C2_RPRE 0     // 1: a tile's residual loaded at the start of its last stage (64 VGPRs across that stage)
#endif
#ifndef C2_AISSUE
#define C2_AISSUE 3   // MFMA slot of the first k16 step after which the next A loads issue (21: round-4 first version)
#endif

__host__ __device__ inline int c2_npad(int N) { return (N + C2_BN - 1) / C2_BN * C2_BN; }
__host__ __device__ inline int c2_nks(int K) { return (K + C2_BK - 1) / C2_BK; }

int64_t oaf_conv2_image_bytes(int N, int K) {
  if (N <= 0 || K <= 0) return 0;
  return (int64_t)3 * c2_nks(K) * c2_npad(N) * C2_BK * 2;
}

// img[p][ks][n][32]: plane p (h, m, l) of W(n, 32 ks + 8c + e) at chunk position c ^ ((n >> 2) & 3), element e;
// zero past N and K.  One thread per (ks, n, c).
__global__ void oaf_w_image_kernel(const float* __restrict__ W, int N, int K, int64_t ldw, int Npad, int nks,
                                   uint16_t* __restrict__ img) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)nks * Npad * 4) return;
  const int c = (int)(i & 3);
  const int n = (int)((i >> 2) % Npad), ks = (int)((i >> 2) / Npad);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 32 * ks + 8 * c + e;
    v[e] = (n < N && k < K) ? W[(int64_t)n * ldw + k] : 0.f;
  }
  u32x4 H, Mm, L;
  split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), H, Mm, L);
  const int64_t plane = (int64_t)nks * Npad * C2_BK;
  const int64_t o = ((int64_t)ks * Npad + n) * C2_BK + 8 * (c ^ ((n >> 2) & 3));
  *reinterpret_cast<u32x4*>(img + o) = H;
  *reinterpret_cast<u32x4*>(img + plane + o) = Mm;
  *reinterpret_cast<u32x4*>(img + 2 * plane + o) = L;
}

__global__ __launch_bounds__(C2_THREADS, 1) void oaf_conv2_kernel(GemmArgs g, const uint16_t* __restrict__ img) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[2 * C2_SLOT];
  __shared__ float2 red[4 * 128];
  __shared__ __attribute__((aligned(16))) float fsv[2][2][C2_KMAX + C2_BK];   // [tile parity][scale | shift][k]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;             // 64-row half, 64-column quarter of the tile
  const int l32 = lane & 31, kh = lane >> 5;
  const int N = g.N, K = g.K;
  const int N4 = (N + 3) & ~3;
  const int ntn = (N + C2_BN - 1) / C2_BN, ntn128 = (N + 127) / 128;
  const int Npad = ntn * C2_BN, nks = c2_nks(K);
  const int ntiles = ntn * g.batch;
  const int G = gridDim.x, slot = xcd_slot();
  const int my_tiles = (ntiles - slot + G - 1) / G;
  const int S = my_tiles * nks;
  if (S <= 0) return;

  // A staging: thread -> row am, 8 k from 8 ac (32 bytes of fp32 per stage)
  const int am = tid >> 2, ac = tid & 3;
  const int apos = am * C2_BK + 8 * (ac ^ ((am >> 2) & 3));
  // A registers: two sets, stage s in set s & 1 (selected at compile time: the stage loop is unrolled by two), so a
  // stage's loads are issued two stages before its split
  f32x4 ra[2][2];
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto issue_a = [&](auto SET, int gs) {   // 2 loads
    constexpr int s_ = decltype(SET)::value;
    const int t = slot + (gs / nks) * G, ks = gs % nks;
    const int b = t / ntn;
    const int k = ks * C2_BK + 8 * ac;
    const int k0 = min(k, K - 4), k1 = min(k + 4, K - 4);   // clamped into the row; zeroed past K at the fold
    const float* Ar = g.A + (int64_t)b * g.sAb + (int64_t)am * g.lda;
    ra[s_][0] = *reinterpret_cast<const f32x4*>(Ar + k0);
    ra[s_][1] = *reinterpret_cast<const f32x4*>(Ar + k1);
  };
  // the fold vectors (scale, shift per k) of this workgroup's tile i -> LDS parity i & 1: one float4 per thread
  // (2 K / 4 <= 256 threads), loaded a stage before it is stored
  const int q4 = K / 4;
  f32x4 fv;
  auto load_fold = [&](int i) {
    const int b = (slot + min(i, my_tiles - 1) * G) / ntn;
    if (tid < 2 * q4)
      fv = *reinterpret_cast<const f32x4*>((tid < q4 ? g.psc : g.psh) + (int64_t)b * g.sPb + 4 * (tid < q4 ? tid : tid - q4));
  };
  auto store_fold = [&](int i) {
    if (tid < 2 * q4) *reinterpret_cast<f32x4*>(&fsv[i & 1][tid < q4 ? 0 : 1][4 * (tid < q4 ? tid : tid - q4)]) = fv;
  };
  auto store_a = [&](auto SET, int gs, int sl) {   // fold + split the registers of stage gs into slot sl's A planes
    constexpr int s_ = decltype(SET)::value;
    const f32x4 ra0 = ra[s_][0], ra1 = ra[s_][1];
    const int k = (gs % nks) * C2_BK + 8 * ac;
    const float* fs = fsv[(gs / nks) & 1][0] + k;
    const float* fh = fsv[(gs / nks) & 1][1] + k;
    const f32x4 rs0 = *reinterpret_cast<const f32x4*>(fs), rs1 = *reinterpret_cast<const f32x4*>(fs + 4);
    const f32x4 rh0 = *reinterpret_cast<const f32x4*>(fh), rh1 = *reinterpret_cast<const f32x4*>(fh + 4);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = k + e < K ? fmaxf(fmaf(ra0[e], rs0[e], rh0[e]), 0.f) : 0.f;
      v[4 + e] = k + 4 + e < K ? fmaxf(fmaf(ra1[e], rs1[e], rh1[e]), 0.f) : 0.f;
    }
    u32x4 H, Mm, L;
    split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), H, Mm, L);
    uint16_t* As = sm + sl * C2_SLOT;
    *reinterpret_cast<u32x4*>(As + apos) = H;
    *reinterpret_cast<u32x4*>(As + C2_APL + apos) = Mm;
    *reinterpret_cast<u32x4*>(As + 2 * C2_APL + apos) = L;
  };
  // B staging: the 3 planes x 16 KB of a stage are 48 one-KB LDS-DMA pieces, 6 per wave
  auto issue_b = [&](int gs, int sl) {
    const int t = slot + (gs / nks) * G, ks = gs % nks;
    const int tn = t % ntn;
    uint16_t* Bs = sm + sl * C2_SLOT + 3 * C2_APL;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int idx = 6 * wid + q, p = idx >> 4, seg = idx & 15;
      const uint32_t off =
          (uint32_t)((((int64_t)p * nks + ks) * Npad + (int64_t)tn * C2_BN) * C2_BK * 2) + 1024u * seg + 16u * lane;
      glds16s(img, off, lds_addr(Bs + p * C2_BPL + 512 * seg));
    }
  };

  floatx16 acc[2][2];
  const int t4 = lane & 3, p8 = l32 >> 2;
  const bool h1 = (t4 & 1) != 0, h2 = (t4 & 2) != 0;

  // Per stage gs (one barrier): right after the barrier B(gs + 1) goes by DMA into the other slot (a whole stage to
  // land); the A registers of gs + 1 (loaded a stage ago) are folded and split into that slot interleaved with the
  // first k16 step's MFMAs, then the A loads of gs + 2 are issued.  The last stage does the same with clamped
  // indices into the unused slot (branch-free: one scheduling region for the split and the MFMAs).  Loads retire in
  // order: vmcnt(2) at the end of a stage = B(gs + 1) landed, the 2 younger A loads still in flight.
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ii][j][r] = 0.f;
#if GEMM_TRACE   // phases: 0 barrier, 1 A wait + DMA issue, 2 first k16 step (+ split), 3 second, 4 epilogue, 5 stage-end wait
  unsigned long long tr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = __builtin_amdgcn_s_memtime();
  int prev_slot = 7;
#endif
  load_fold(0);
  store_fold(0);
  issue_a(I0{}, 0);
  issue_a(I1{}, min(1, S - 1));
  __syncthreads();
  store_a(I0{}, 0, 0);
  issue_b(0, 0);
  issue_a(I0{}, min(2, S - 1));
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // B(0) (and A(1), older) landed; A(2) in flight
  float4 w[2][2][4];   // the residual of the tile's output, loaded at the start of its last stage
  // stage gs: splits A(gs + 1) from set (gs + 1) & 1 and reloads that set with A(gs + 3)
  auto stage = [&](auto SET, const int gs) {
    constexpr int s_ = decltype(SET)::value;
    const int ks = gs % nks, ti = gs / nks;
    const int gn = min(gs + 1, S - 1), so = (gs + 1) & 1;
    TSTAMP(0);
    lds_barrier();   // stage gs's A planes written and its B planes landed (each wave waited its own DMA);
                     // every wave has finished reading slot so (stage gs - 1); fold vectors stored a stage ago visible
    TSTAMP(1);
    // the next tile's fold vectors: loaded in its predecessor's first stage, stored in the second (published by the
    // next barrier, read from the predecessor's last stage on); with two stages per tile, stored at once
    if (ks == 0) {
      load_fold(ti + 1);
      if (nks < 3) store_fold(ti + 1);
    } else if (ks == 1 && nks >= 3) {
      store_fold(ti + 1);
    }
    // the A registers of gs + 1 ready before the DMA is issued (a use here makes the compiler's wait precede it)
    asm volatile("" ::"v"(ra[s_][0]), "v"(ra[s_][1]));
    issue_b(gn, so);
    if (C2_RPRE && ks == nks - 1) {   // the tile's residual, in flight during its last stage's MFMAs
      const int t = slot + ti * G;
      const int b = t / ntn, nb0 = (t % ntn) * C2_BN + wn * 64;
      const float* Rb = g.R + (int64_t)b * g.sRb;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gm = wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int gnc = min(nb0 + j * 32 + 4 * p8, N4 - 4);
            w[ii][j][q] = *reinterpret_cast<const float4*>(Rb + (int64_t)gm * g.ldc + gnc);
          }
        }
    }
    TSTAMP(2);
    const uint16_t* As = sm + (gs & 1) * C2_SLOT;
    const uint16_t* Bs = As + 3 * C2_APL;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int cc = 2 * st + kh;   // 16-byte chunk of k 16 st + 8 kh .. + 7
      bx::Frag fa[2], fb[2];
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int r = wm * 64 + ii * 32 + l32;
        const int o = r * C2_BK + 8 * (cc ^ ((r >> 2) & 3));
        fa[ii].h = *reinterpret_cast<const bf16x8*>(As + o);
        fa[ii].m = *reinterpret_cast<const bf16x8*>(As + C2_APL + o);
        fa[ii].l = *reinterpret_cast<const bf16x8*>(As + 2 * C2_APL + o);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 64 + j * 32 + l32;
        const int o = r * C2_BK + 8 * (cc ^ ((r >> 2) & 3));
        fb[j].h = *reinterpret_cast<const bf16x8*>(Bs + o);
        fb[j].m = *reinterpret_cast<const bf16x8*>(Bs + C2_BPL + o);
        fb[j].l = *reinterpret_cast<const bf16x8*>(Bs + 2 * C2_BPL + o);
      }
      if (st == 0) store_a(SET, gn, so);
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[ii][j] = bx::mfma6(fa[ii], fb[j], acc[ii][j]);
      if (st == 0) {
        issue_a(SET, min(gs + 3, S - 1));
        // 12 fragment reads, then the 24 MFMAs each followed by a share of the split (VALU, its 3 LDS writes)
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);   // (+ the 4 fold-vector reads of the split)
#pragma unroll
        for (int u = 0; u < 24; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          if (u == C2_AISSUE) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);   // once the fold has read ra
          if (u == 20) __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        TSTAMP(3);
      }
    }
    TSTAMP(4);
    if (ks == nks - 1) {
      // ------------------------------------------------------------ epilogue of the tile (row path of tile_epilogue)
      const int t = slot + (gs / nks) * G;
      const int b = t / ntn, tn = t % ntn;
      const int n0 = tn * C2_BN, nb0 = n0 + wn * 64;
      const int nw = min(max(N - nb0, 0), 64);
      const float rnw = nw > 0 ? 1.f / (float)nw : 0.f;
      bool cok[2][4], sok[2];
      float bn[2][4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int gn = nb0 + j * 32 + 4 * p8;
        sok[j] = gn < N4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          cok[j][u] = gn + u < N;
          bn[j][u] = cok[j][u] ? g.bias[gn + u] : 0.f;
        }
      }
      float* Cb = g.C + (int64_t)b * g.sCb;
      if (!C2_RPRE) {   // the residual loaded here (no prefetch during the last stage)
        const float* Rb = g.R + (int64_t)b * g.sRb;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int gm = wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int gnc = min(nb0 + j * 32 + 4 * p8, N4 - 4);
              w[ii][j][q] = *reinterpret_cast<const float4*>(Rb + (int64_t)gm * g.ldc + gnc);
            }
          }
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gm = wm * 64 + ii * 32 + 8 * q + 4 * kh + t4;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float a0 = acc[ii][j][4 * q], a1 = acc[ii][j][4 * q + 1], a2 = acc[ii][j][4 * q + 2],
                  a3 = acc[ii][j][4 * q + 3];
            quad_transpose(a0, a1, a2, a3, h1, h2);
            const float4 x = make_float4(a0 + bn[j][0] + w[ii][j][q].x, a1 + bn[j][1] + w[ii][j][q].y,
                                         a2 + bn[j][2] + w[ii][j][q].z, a3 + bn[j][3] + w[ii][j][q].w);
            w[ii][j][q] = x;
            if (sok[j]) *reinterpret_cast<float4*>(Cb + (int64_t)gm * g.ldc + nb0 + j * 32 + 4 * p8) = x;
          }
        }
        float s1[4], s2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s1[q] = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) s1[q] += cok[j][u] ? f4(w[ii][j][q], u) : 0.f;
          s1[q] = sum8_p8(s1[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float mu = s1[q] * rnw;
          s2[q] = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float d = cok[j][u] ? f4(w[ii][j][q], u) - mu : 0.f;
              s2[q] = fmaf(d, d, s2[q]);
            }
          s2[q] = sum8_p8(s2[q]);
        }
        if (p8 == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            red[wn * 128 + wm * 64 + ii * 32 + 8 * q + 4 * kh + t4] = make_float2(s1[q], s2[q]);
        }
      }
      lds_barrier();
      if (tid < 256) {   // merge the two 64-column waves of each 128-column statistics tile (Chan)
        const int half = tid >> 7, row = tid & 127;
        const int n0h = n0 + 128 * half;
        if (n0h < N) {
          const float2 x = red[(2 * half) * 128 + row], c = red[(2 * half + 1) * 128 + row];
          const int na = min(N - n0h, 64), nb = min(max(N - n0h - 64, 0), 64);
          float2 o = x;
          if (nb > 0) {
            const float d = c.x / (float)nb - x.x / (float)na;
            o = make_float2(x.x + c.x, x.y + c.y + d * d * ((float)na * (float)nb / (float)(na + nb)));
          }
          g.stats[((int64_t)b * ntn128 + 2 * tn + half) * g.st_ld + g.st_off + row] = o;
        }
      }
      // (red is next written in the next tile's epilogue, after at least one stage barrier)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ii][j][r] = 0.f;   // the next tile's accumulators
    }
    TSTAMP(5);
    // B(gs + 1) landed (and A(gs + 2), older), A(gs + 3) (2 loads, younger) in flight.  After an epilogue its stores
    // are outstanding too (not ordered with the loads): drain everything.
    if (ks != nks - 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  for (int gs = 0; gs < S; gs += 2) {
    stage(I1{}, gs);
    if (gs + 1 < S) stage(I0{}, gs + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup
#if GEMM_TRACE
  TSTAMP(7);
  if (lane == 0)
    for (int q = 0; q < 8; ++q) atomicAdd(&g_gemm_trace[q], tr[q]);
#endif
}


static bool oaf_conv2_covers(const GemmArgs& g) {
  return g.wimg && g.M == 128 && g.pro == PRO_A_K && g.bkc == 1 && g.sBb == 0 && g.bias_mode == BIAS_N &&
         g.stats_mode == ST_ROW && g.has_res && !g.no_store && !g.head_w && !g.xin && g.K % 4 == 0 &&
         g.K > C2_BK && g.K <= C2_KMAX &&
         g.wimg_bytes >= oaf_conv2_image_bytes(g.N, g.K) && (reinterpret_cast<uintptr_t>(g.wimg) & 15) == 0 &&
         (int64_t)c2_nks(g.K) * c2_npad(g.N) * C2_BK * 2 * 3 < ((int64_t)1 << 31);
}

static int launch_oaf_conv2(const GemmArgs& g, hipStream_t s) {
  const int Npad = c2_npad(g.N), nks = c2_nks(g.K);
  const int64_t nthr = (int64_t)nks * Npad * 4;
  hipLaunchKernelGGL(oaf_w_image_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, g.B, g.N, g.K, g.ldb,
                     Npad, nks, g.wimg);
  MVR_CHECK_LAUNCH();
  const long long tiles = (long long)(Npad / C2_BN) * g.batch;
  const unsigned wgs = (unsigned)(tiles < GPU_CUS ? tiles : GPU_CUS);   // one 144-KB-LDS workgroup per CU
  hipLaunchKernelGGL(oaf_conv2_kernel, dim3(wgs), dim3(C2_THREADS), 0, s, g, (const uint16_t*)g.wimg);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

#ifndef GEMM_F16_DEFAULT
#define GEMM_F16_DEFAULT 0
#endif
int g_gemm_h = GEMM_F16_DEFAULT;   // mvr_set_math: MATH_BF16X3 launches run split-fp16 first

template <int PRO, int BKC, int BIAS, int STATS, int RES>
static void launch_t(const KArgs& ka0, long long tiles, hipStream_t s) {
  KArgs ka = ka0;
  const unsigned wgs = (unsigned)(tiles < ka.persist ? tiles : ka.persist);
  // split-fp16 first when the caller provides a zeroed flag word, unless the output is an operand or the residual
  // (in place: the re-run reads them).  Outputs never partially overlap inputs (launch_gemm contract), so the test is
  // pointer equality — a property of the call, not of where the allocator placed the buffers.
  const GemmArgs& g = ka.g;
  const bool alias = g.C && (g.C == g.A || g.C == g.B || (g.has_res && g.C == g.R));
  if (g_gemm_h && g.flag && !alias) {
    ka.range = g.flag;
    ka.epoch = 1;
    hipLaunchKernelGGL((gemm_kernel<MATH_F16X2, PRO, BKC, BIAS, STATS, RES>), dim3(wgs), dim3(256), 0, s, ka);
    ka.guard = ka.range;
    ka.range = nullptr;
  }
  hipLaunchKernelGGL((gemm_kernel<MATH_BF16X3, PRO, BKC, BIAS, STATS, RES>), dim3(wgs), dim3(256), 0, s, ka);
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

static int launch_gemm_impl(const GemmArgs& g, hipStream_t s, bool conv2) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return MVR_OK;
  if (!g.A || !g.B || (!g.C && !g.no_store) || g.K <= 0) return MVR_EINVAL;
  // no_store: statistics only (row statistics), or the output head only (point-conv kernel)
  if (g.no_store && !g.head_w && (g.stats_mode != ST_ROW || g.has_res)) return MVR_EINVAL;
  if (g.pro != PRO_NONE && !g.psc) return MVR_EINVAL;
  if ((g.pro == PRO_A_K || g.pro == PRO_B_K) && !g.psh) return MVR_EINVAL;
  if (g.stats_mode != ST_NONE && !g.stats) return MVR_EINVAL;
  if (g.bias_mode != BIAS_NONE && !g.bias) return MVR_EINVAL;
  if (g.has_res && !g.R) return MVR_EINVAL;
  if (g.math != MATH_BF16X3) return MVR_EINVAL;
  // layout contract (gemm.hpp)
  const int64_t K4 = round4(g.K), N4 = round4(g.N);
  // a chunk-major operand: rows 32 floats apart inside each chunk, the chunks past all its rows
  const bool cm = g.bcs || g.ccs || (g.has_res && (g.rcs || (g.ldr && g.ldr != g.ldc)));
  const int64_t ldr = g.ldr ? g.ldr : g.ldc;
  bool ok = al16(g.A) && al16(g.B) && al16(g.C) && g.lda % 4 == 0 && g.ldb % 4 == 0 && g.ldc % 4 == 0 &&
            g.sAb % 4 == 0 && g.sBb % 4 == 0 && g.sCb % 4 == 0 && g.lda >= K4 && g.ldc >= (g.ccs ? 32 : N4) &&
            g.ldb >= (g.bkc ? K4 : (g.bcs ? 32 : N4));
  if (g.bcs) ok = ok && !g.bkc && g.ldb == 32 && g.bcs % 4 == 0 && g.bcs >= 32LL * g.K;
  if (g.ccs) ok = ok && g.ldc == 32 && g.ccs % 4 == 0 && g.ccs >= 32LL * g.M;
  if (g.has_res) {
    ok = ok && al16(g.R) && g.sRb % 4 == 0;
    if (g.xin != 2)   // (xin = 2: R is the block input, rows xld apart: pconv_covers)
      ok = ok && ldr % 4 == 0 && (g.rcs ? ldr == 32 && g.rcs % 4 == 0 && g.rcs >= 32LL * g.M : ldr >= N4);
  }
  if (cm && !pconv_covers(g)) return MVR_EINVAL;   // only the point-conv kernel addresses chunk-major operands
  if (g.pro == PRO_A_K || g.pro == PRO_B_K)
    ok = ok && al16(g.psc) && al16(g.psh) && g.sPb % 4 == 0 && g.K % 4 == 0 && g.K <= KV_MAX;
  if (g.pro == PRO_B_SMX) ok = ok && al16(g.psc) && g.sPb % 4 == 0 && g.pld % 4 == 0 && g.pld >= N4;
  if (!ok) return MVR_EINVAL;
  KArgs ka{};
  ka.g = g;
  ka.persist = 2 * GPU_CUS;  // 2 workgroups per CU (LDS-bound)
  ka.m_fast = (g.sAb == 0 && gemm_mtiles(g.M) > 1) ? 1 : 0;
  const long long tiles = (long long)gemm_ntiles(g.N) * gemm_mtiles(g.M) * g.batch;
  if (tiles > 0x7fffffffLL) return MVR_EINVAL;
  const double fl = 2.0 * g.M * g.N * (double)g.K * g.batch;
  double by = 4.0 * ((double)g.M * g.K * (g.sAb ? g.batch : 1) + (double)g.K * g.N * (g.sBb ? g.batch : 1) +
                     (double)g.M * g.N * g.batch * ((g.has_res ? 2 : 1) - (g.no_store ? 1 : 0)));
  if (g.xin) {   // folded conv1 (pconv): the block input's xci rows replace B (xin 1) or the residual (xin 2)
    if (!pconv_covers(g)) return MVR_EINVAL;
    by = 4.0 * ((double)g.M * g.K + (double)g.N * g.batch * (g.xin == 1 ? g.xci + g.M : g.K + g.xci + g.M));
  }
  ProfScope prof(g.prof_kind, fl, by, s);
  if (pconv_covers(g)) return launch_pconv(g, s);
  if (conv2 && oaf_conv2_covers(g)) return launch_oaf_conv2(g, s);   // (not under FORCE_GENERIC_GEMM)
  if (g.head_w) return MVR_EINVAL;   // the fused head exists on the point-conv kernel only
  // Dispatch only the combinations the OANet schedule uses (oanet.hip).
#define MVR_CASE(P, BKC_, BI, ST, RS)                                                                     \
  if (g.pro == P && g.bkc == BKC_ && g.bias_mode == BI && g.stats_mode == ST && (g.has_res != 0) == RS) { \
    launch_t<P, BKC_, BI, ST, RS>(ka, tiles, s);                                                        \
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

int launch_gemm(const GemmArgs& g, hipStream_t s) { return launch_gemm_impl(g, s, !g_force[FORCE_GENERIC_GEMM]); }

}  // namespace mvr

// C-ABI: one fused GEMM (exposed for unit tests and host-side composition).
extern "C" int mvr_gemm_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda, const float* B,
                            int64_t sBb, int64_t ldb, int b_kcontig, float* C, int64_t sCb, int64_t ldc,
                            const float* R, int64_t sRb, const float* bias, int bias_mode, const float* psc,
                            const float* psh, int64_t sPb, int64_t pld, int pro, float* stats, int64_t st_ld,
                            int st_off, int stats_mode, int math, int32_t* range_flag, hipStream_t stream) {
  mvr::GemmArgs g{};
  if (range_flag && math == mvr::MATH_BF16X3 && (mvr::g_gemm_h || mvr::g_pconv_h)) {
    if (hipMemsetAsync(range_flag, 0, sizeof(int32_t), stream) != hipSuccess) return MVR_ELAUNCH;
    g.flag = range_flag;
  }
  g.math = math;
  g.M = M; g.N = N; g.K = K; g.batch = batch;
  g.A = A; g.sAb = sAb; g.lda = lda;
  g.B = B; g.sBb = sBb; g.ldb = ldb; g.bkc = b_kcontig;
  g.C = C; g.sCb = sCb; g.ldc = ldc;
  g.R = R; g.sRb = sRb; g.has_res = R != nullptr;
  g.bias = bias; g.bias_mode = bias_mode;
  g.psc = psc; g.psh = psh; g.sPb = sPb; g.pld = pld; g.pro = pro;
  g.stats = reinterpret_cast<float2*>(stats); g.st_ld = st_ld; g.st_off = st_off; g.stats_mode = stats_mode;
  return mvr::launch_gemm(g, stream);
}

#if GEMM_TRACE
extern "C" int mvr_gemm_trace(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mvr::g_gemm_trace), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mvr::g_gemm_trace), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// C-ABI: the OAFilter conv2 launch on the split-once kernel (tests; also under FORCE_GENERIC_GEMM): W [N][K]
// (row stride ldw) shared by every pair, A folded by (psc, psh) per k, bias per n, residual R, row statistics per
// 128-column tile; img: img_bytes >= mvr_oaf_conv2_image_bytes(N, K) of scratch.  MVR_EINVAL when the shape is not
// the kernel's (M != 128, K % 4 != 0, a null operand).
extern "C" int mvr_oaf_conv2_f32(int M, int N, int K, int batch, const float* A, int64_t sAb, int64_t lda,
                                 const float* W, int64_t ldw, float* C, int64_t sCb, int64_t ldc, const float* R,
                                 int64_t sRb, const float* bias, const float* psc, const float* psh, int64_t sPb,
                                 float* stats, int64_t st_ld, void* img, int64_t img_bytes, hipStream_t stream) {
  mvr::GemmArgs g{};
  g.math = mvr::MATH_BF16X3;
  g.M = M; g.N = N; g.K = K; g.batch = batch;
  g.A = A; g.sAb = sAb; g.lda = lda;
  g.B = W; g.sBb = 0; g.ldb = ldw; g.bkc = 1;
  g.C = C; g.sCb = sCb; g.ldc = ldc;
  g.R = R; g.sRb = sRb; g.has_res = 1;
  g.bias = bias; g.bias_mode = mvr::BIAS_N;
  g.psc = psc; g.psh = psh; g.sPb = sPb; g.pro = mvr::PRO_A_K;
  g.stats = reinterpret_cast<float2*>(stats); g.st_ld = st_ld; g.stats_mode = mvr::ST_ROW;
  g.wimg = static_cast<uint16_t*>(img); g.wimg_bytes = img_bytes;
  if (M != 128 || K % 4 || N < 0 || batch < 0) return MVR_EINVAL;
  if (N == 0 || batch == 0) return MVR_OK;   // empty: NULL pointers allowed
  if (!R || !bias || !psc || !psh || !stats || !img) return MVR_EINVAL;
  if (!mvr::oaf_conv2_covers(g)) return MVR_EINVAL;
  return mvr::launch_gemm_impl(g, stream, true);
}

extern "C" size_t mvr_oaf_conv2_image_bytes(int N, int K) { return (size_t)mvr::oaf_conv2_image_bytes(N, K); }


