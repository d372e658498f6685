// Fused PointCN (lib/filtering/oanet.py:18-43) for channels == out_channels == 128 (identity
// shortcut):
//     y = W7 . relu(IN_BN_t(t)) + b7 + x,   t = W3 . relu(IN_BN_x(x)) + b3
// The InstanceNorm statistics of t come from a statistics-only pass of the conv3 GEMM (gemm.hip,
// no_store), so t never reaches HBM: per PointCN the activations cross HBM three times (x for
// the statistics, x here, y) instead of five (x, t written, t and x read, y).
//
// Persistent kernel, one 512-thread workgroup per CU streaming a contiguous range of 32-point
// chunks (pair-major).  Per chunk, in a three-step software pipeline with one barrier per step:
//   * LDS-DMA of the raw x chunk [128 c][32 n] (two steps ahead),
//   * all 8 waves: normalise (IN+BN+ReLU folded to relu(x*sc1+sh1)) and split into the bf16
//     B-fragment image of the conv3 GEMM (one fragment per thread),
//   * waves 0-3 ("A"): t = W3[32-row block] . xn with W3 held split in registers, then
//     relu(t*sc2+sh2) split straight from the accumulator registers into the B-fragment image
//     of the conv7 GEMM (k in the C-register order, see mfma_bf16.hpp),
//   * waves 4-7 ("B"): y = W7[32-row block] . tn + b7 (W7 split in registers, k permuted to
//     match), transposed through a per-wave LDS scratch, + residual, stored, and the per-chunk
//     (sum, squared deviations) partials of y for the next InstanceNorm.
// Each SIMD hosts one A and one B wave (48 split MFMAs each per chunk).
// Roofline: 2 GEMMs x 2 x 128 x 128 flops per point (split MFMA) against 8 + 8 bytes per
// channel-point (x in, y out): AI = 64 flop/B -> HBM-bound on the split-MFMA ridge (52).
#include "common.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"
#include "mvreg.h"

namespace mvr {
namespace {

using namespace bx;

constexpr int PC = 128;              // channels
constexpr int PCH = 32;              // points per chunk
constexpr int RAWB = PC * PCH * 4;   // raw fp32 chunk [128 c][32 n] (16 KB)
constexpr int FRB = 3 * 64 * 16;     // one fragment set: h, m, l planes x 64 lanes x 16 B (3 KB)
constexpr int XNB = 8 * FRB;         // xn image: 8 k-steps of 16 channels (24 KB)
constexpr int TNB = 8 * FRB;         // tn image: 4 o-blocks x 2 k-steps (24 KB)
constexpr int YLD = 33;              // row stride (floats) of a B wave's transpose scratch

#define PCN_FENCE() __builtin_amdgcn_sched_barrier(0)
// ablation switches for tools/pcn_micro.py experiments (0 in the product build): 1 no MFMA,
// 2 no split, 4 no B epilogue, 8 no DMA
#ifndef PCN_ABL
#define PCN_ABL 0
#endif

struct PcnArgs {
  const float* X; int64_t xps, xld;     // x [P][128][xld]
  float* Y; int64_t yps, yld;           // y [P][128][yld] (may alias x)
  const float* sc1; const float* sh1;   // [P][128]: relu(x * sc1 + sh1) is conv3's input
  const float* sc2; const float* sh2;   // [P][128]: relu(t * sc2 + sh2) is conv7's input
  const float* W3; const float* b3;     // [128][128], [128]
  const float* W7; const float* b7;
  float2* stats; int64_t st_ld; int st_off;   // [P][nch][st_ld] (+ st_off + c) per 32-point chunk, nullable
  int P, N, nch;                        // nch = ceil(N / 32)
  int64_t total;                        // P * nch
};

__device__ __forceinline__ void glds16c(const char* src, char* lds_base) {
  const uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_base;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}

__device__ __forceinline__ Frag read_frag(const char* base, int k) {
  Frag f;
  f.h = *reinterpret_cast<const bf16x8*>(base + k * FRB);
  f.m = *reinterpret_cast<const bf16x8*>(base + k * FRB + 1024);
  f.l = *reinterpret_cast<const bf16x8*>(base + k * FRB + 2048);
  return f;
}
__device__ __forceinline__ void write_frag(char* base, const Frag& f) {
  *reinterpret_cast<bf16x8*>(base) = f.h;
  *reinterpret_cast<bf16x8*>(base + 1024) = f.m;
  *reinterpret_cast<bf16x8*>(base + 2048) = f.l;
}

__global__ __launch_bounds__(512) void pointcn_chain_kernel(PcnArgs a) {
  __shared__ __attribute__((aligned(16))) char raw[2][RAWB];
  __shared__ __attribute__((aligned(16))) char xnI[2][XNB];
  __shared__ __attribute__((aligned(16))) char tnI[2][TNB];
  __shared__ __attribute__((aligned(16))) float ybuf[4][32 * YLD];
  __shared__ __attribute__((aligned(16))) float f2s[2][2][PC];   // (sc2, sh2) of pairs by parity
  __shared__ __attribute__((aligned(16))) float f1s[2][2][PC];   // (sc1, sh1) of pairs by parity
  __shared__ __attribute__((aligned(16))) float bsh[2][PC];       // (b3, b7), read at each GEMM start
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t per = (a.total + gridDim.x - 1) / gridDim.x;
  const int64_t g0 = min(a.total, (int64_t)blockIdx.x * per), g1 = min(a.total, g0 + per);
  const int nloc = (int)(g1 - g0);
  if (nloc <= 0) return;   // uniform
  const bool isA = w < 4;
  const int blk = w & 3;
  const int N = a.N, N4 = (N + 3) & ~3, nlast = N4 - 4;

  // weights as split A fragments (loaded once): A waves W3 rows 32 blk + l32 over k = c;
  // B waves W7 rows 32 blk + l32 over k-step q = 2 ab + s: o = 32 ab + 16 s + 8 (i >> 2) + 4h + (i & 3)
  Frag wf[8];
  {
    const float* W = isA ? a.W3 : a.W7;
    const float* wr = W + (int64_t)(32 * blk + l32) * PC;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int o0 = isA ? 16 * q + 8 * h : 32 * (q >> 1) + 16 * (q & 1) + 4 * h;
      const int o1 = isA ? o0 + 4 : o0 + 8;
      const float4 u0 = *reinterpret_cast<const float4*>(wr + o0);
      const float4 u1 = *reinterpret_cast<const float4*>(wr + o1);
      const float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      split8(v, wf[q].h, wf[q].m, wf[q].l);
    }
    if (tid < PC) {
      bsh[0][tid] = a.b3 ? a.b3[tid] : 0.f;
      bsh[1][tid] = a.b7 ? a.b7[tid] : 0.f;
    }
  }
  // accumulator initialised with this wave's bias rows 32 blk + 8 q + 4h + 0..3
  auto bias_init = [&](floatx16& S) {
    const float* bv = bsh[isA ? 0 : 1] + 32 * blk + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 u = *reinterpret_cast<const float4*>(bv + 8 * q);
      S[4 * q + 0] = u.x; S[4 * q + 1] = u.y; S[4 * q + 2] = u.z; S[4 * q + 3] = u.w;
    }
  };

  // raw chunk g -> raw[slot], by the A waves only (their only vector-memory traffic, so vmcnt(0)
  // before the step barrier waits for exactly this); wave w: rows 32 w .. 32 w + 31
  auto dma = [&](int p, int kc, int slot) {
    if (PCN_ABL & 8) return;
    const int n = min(kc * PCH + 4 * (lane & 7), nlast);
    const float* src = a.X + (int64_t)p * a.xps + n;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r0 = 32 * w + 8 * i;
      glds16c(reinterpret_cast<const char*>(src + (int64_t)(r0 + (lane >> 3)) * a.xld), raw[slot] + r0 * 128);
    }
  };

  // Per-pair folds through LDS slots by pair parity (consecutive pairs use different slots), so the
  // steady loop issues no global loads besides the DMA and the residual prefetch:
  //   (sc1, sh1) of chunk k + 1's pair are staged at step k (read by the split at step k + 1),
  //   (sc2, sh2) of chunk k's pair are staged at step k (read by the A waves at step k + 1).
  auto stage_fold = [&](float (*f)[PC], const float* sc, const float* sh, int p) {
    if (tid < PC) {
      f[0][tid] = sc[(int64_t)p * PC + tid];
      f[1][tid] = sh[(int64_t)p * PC + tid];
    }
  };

  // split: thread -> fragment (k-step w, lane): xn[16 w + 8h + i][n = lane row].  Two halves so that
  // they can be interleaved with a GEMM's MFMA groups: split_load issues the LDS reads, split_finish
  // normalises, splits and writes the fragment.
  float sv[8];
  auto split_load = [&](int p, int kc, int slot, bool first, bool next_new) {
    if (PCN_ABL & 2) return;
    if (first) stage_fold(f2s[p & 1], a.sc2, a.sh2, p);
    if (next_new) stage_fold(f1s[(p + 1) & 1], a.sc1, a.sh1, p + 1);
    const float* rw = reinterpret_cast<const float*>(raw[slot]);
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = rw[(16 * w + 8 * h + i) * PCH + l32];
  };
  auto split_finish = [&](int p, int kc, int slot) {
    if (PCN_ABL & 2) return;
    const bool nok = kc * PCH + l32 < N;
    const float* f1 = &f1s[p & 1][0][16 * w + 8 * h];
    const float4 sa = *reinterpret_cast<const float4*>(f1), sb = *reinterpret_cast<const float4*>(f1 + 4);
    const float4 ha = *reinterpret_cast<const float4*>(f1 + PC), hb = *reinterpret_cast<const float4*>(f1 + PC + 4);
    const float s1[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float h1[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float y = fmaxf(fmaf(sv[i], s1[i], h1[i]), 0.f);
      sv[i] = nok ? y : 0.f;
    }
    Frag f;
    split8(sv, f.h, f.m, f.l);
    write_frag(xnI[slot] + w * FRB + lane * 16, f);
  };

  // A: t = W3 . xn + b3 -> relu(t * sc2 + sh2) -> conv7 B fragments; hook(ks) runs after the ks-th
  // MFMA group (independent work interleaved with the matrix pipe)
  auto gemm1 = [&](int p, int slot, auto&& hook) {
    floatx16 S;
    bias_init(S);
    const char* xi = xnI[slot] + lane * 16;
    Frag cur = read_frag(xi, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      Frag nxt;
      if (ks < 7) nxt = read_frag(xi, ks + 1);
      PCN_FENCE();
      if (PCN_ABL & 1) asm volatile("" ::"v"(cur.h), "v"(cur.m), "v"(cur.l), "v"(wf[ks].h));
      else S = mfma6(wf[ks], cur, S);
      hook(ks);
      PCN_FENCE();
      if (ks < 7) cur = nxt;
    }
    float t[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // rows o = 32 blk + 8 q + 4h + 0..3
      const float4 sc = *reinterpret_cast<const float4*>(&f2s[p & 1][0][32 * blk + 8 * q + 4 * h]);
      const float4 sh = *reinterpret_cast<const float4*>(&f2s[p & 1][1][32 * blk + 8 * q + 4 * h]);
      t[4 * q + 0] = fmaxf(fmaf(S[4 * q + 0], sc.x, sh.x), 0.f);
      t[4 * q + 1] = fmaxf(fmaf(S[4 * q + 1], sc.y, sh.y), 0.f);
      t[4 * q + 2] = fmaxf(fmaf(S[4 * q + 2], sc.z, sh.z), 0.f);
      t[4 * q + 3] = fmaxf(fmaf(S[4 * q + 3], sc.w, sh.w), 0.f);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Frag f;
      split8(t + 8 * s, f.h, f.m, f.l);
      write_frag(tnI[slot] + (2 * blk + s) * FRB + lane * 16, f);
    }
  };

  // B: y = W7 . tn + b7 + x, stored, with per-chunk statistics.  The residual x of the wave's 32 rows
  // of the next chunk is DMA'd one step ahead into the wave's scratch ([32 rows][32] fp32) — asm
  // loads the compiler does not track, waited for explicitly — which then doubles as the transpose
  // buffer ([32][YLD]).  The epilogue of chunk k - 3 (still in acc) runs before GEMM2 of chunk k - 2,
  // whose MFMA groups carry the split of chunk k.
  auto dma_res = [&](int p, int kc) {
    if (PCN_ABL & 8) return;
    const int n = min(kc * PCH + 4 * (lane & 7), nlast);
    const float* src = a.X + (int64_t)p * a.xps + (int64_t)(32 * blk) * a.xld + n;
    char* dst = reinterpret_cast<char*>(ybuf[blk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16c(reinterpret_cast<const char*>(src + (int64_t)(8 * i + (lane >> 3)) * a.xld), dst + i * 1024);
  };
  floatx16 acc;
  auto gemm2 = [&](int slot, auto&& hook) {
    bias_init(acc);
    const char* ti = tnI[slot] + lane * 16;
    Frag cur = read_frag(ti, 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      Frag nxt;
      if (q < 7) nxt = read_frag(ti, q + 1);
      PCN_FENCE();
      if (PCN_ABL & 1) asm volatile("" ::"v"(cur.h), "v"(cur.m), "v"(cur.l), "v"(wf[q].h));
      else acc = mfma6(wf[q], cur, acc);
      hook(q);
      PCN_FENCE();
      if (q < 7) cur = nxt;
    }
  };
  // epilogue (chunk (ep, ekc), accumulator acc)
  const int erow = lane >> 1, ec0 = 16 * (lane & 1);
  float4 eres[4];
  float ev[16];
  float* yb = ybuf[blk];
  auto ep_read_res = [&]() {
    if (!(PCN_ABL & 32)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this chunk's residual DMA (one step old)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) eres[i4] = *reinterpret_cast<const float4*>(yb + erow * PCH + ec0 + 4 * i4);
  };
  auto ep_transpose = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // residual read before the transpose overwrites it
#pragma unroll
    for (int r = 0; r < 16; ++r) yb[((r & 3) + 8 * (r >> 2) + 4 * h) * YLD + l32] = acc[r];
  };
  auto ep_read_y = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i) ev[i] = yb[erow * YLD + ec0 + i];
  };
  auto ep_finish = [&](int p, int kc, bool has_next) {
    const int n0 = kc * PCH + ec0;
    const int o = 32 * blk + erow;
    const int nv = min(max(N - n0, 0), 16);
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float x = i < 4 ? (&eres[0].x)[i] : (i < 8 ? (&eres[1].x)[i - 4] : (i < 12 ? (&eres[2].x)[i - 8] : (&eres[3].x)[i - 12]));
      const float y = ev[i] + x;
      ev[i] = i < nv ? y : 0.f;
      sm += ev[i];
    }
    sm += __shfl_xor(sm, 1, 64);
    const int cnt = min(max(N - kc * PCH, 0), PCH);
    const float mu = sm / (float)cnt;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float d = i < nv ? ev[i] - mu : 0.f;
      m2 = fmaf(d, d, m2);
    }
    m2 += __shfl_xor(m2, 1, 64);
    if (!(PCN_ABL & 16) && a.stats && (lane & 1) == 0) a.stats[((int64_t)p * a.nch + kc) * a.st_ld + a.st_off + o] = make_float2(sm, m2);
    float* yr = a.Y + (int64_t)p * a.yps + (int64_t)o * a.yld + n0;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4)
      if (!(PCN_ABL & 16) && n0 + 4 * i4 < N4)
        *reinterpret_cast<float4*>(yr + 4 * i4) = make_float4(ev[4 * i4], ev[4 * i4 + 1], ev[4 * i4 + 2], ev[4 * i4 + 3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // transpose reads done before the DMA lands
    if (has_next) dma_res(kc + 1 == a.nch ? p + 1 : p, kc + 1 == a.nch ? 0 : kc + 1);
  };

  // step barrier: LDS writes published, no wait for the B waves' residual loads and y stores
  auto step_barrier = [&]() {
    if (isA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the raw-chunk DMA
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  // chunk cursors (pair, chunk-in-pair), advanced without divisions: DMA (k + 1), split (k), A (k - 1), B (k - 2)
  struct Cur {
    int p, kc;
  };
  const int nch = a.nch;
  auto adv = [&](Cur& c) {
    if (++c.kc == nch) { c.kc = 0; ++c.p; }
  };
  const Cur c0{(int)(g0 / nch), (int)(g0 - (g0 / nch) * nch)};
  Cur cn = c0, cs = c0, ca = c0;
  if (isA) dma(c0.p, c0.kc, 0);
  else dma_res(c0.p, c0.kc);
  stage_fold(f1s[c0.p & 1], a.sc1, a.sh1, c0.p);
  adv(cn);
  step_barrier();
  // Step k: DMA chunk k + 1 (A), split chunk k (all), GEMM1 chunk k - 1 (A), GEMM2 chunk k - 2 (B),
  // epilogue chunk k - 3 (B).  The two waves of a SIMD run complementary phases: A starts with its
  // MFMAs and ends with VALU/LDS work, B starts with the previous chunk's epilogue and the split and
  // ends with its MFMAs.
  Cur ce = c0;
  for (int k = 0; k < nloc + 3; ++k) {
    const bool do_split = k < nloc;
    const bool split_first = k == 0 || cs.kc == 0, split_next_new = k + 1 < nloc && cs.kc == nch - 1;
    const int slot = k & 1;
    if (isA) {
      if (k + 1 < nloc) dma(cn.p, cn.kc, (k + 1) & 1);
      if (k >= 1 && k <= nloc) {
        gemm1(ca.p, (k - 1) & 1, [&](int ks) {
          if (!do_split) return;
          if (ks == 1) split_load(cs.p, cs.kc, slot, split_first, split_next_new);
          if (ks == 4) split_finish(cs.p, cs.kc, slot);
        });
        adv(ca);
      } else if (do_split) {
        split_load(cs.p, cs.kc, slot, split_first, split_next_new);
        split_finish(cs.p, cs.kc, slot);
      }
    } else {
      const bool do_ep = k >= 3 && k - 3 < nloc;
      const bool ep_next = k - 2 < nloc;
      if (do_ep && !(PCN_ABL & 4)) {
        ep_read_res();
        ep_transpose();
        ep_read_y();
        ep_finish(ce.p, ce.kc, ep_next);
      }
      if (k >= 2 && k - 2 < nloc) {
        gemm2(k & 1, [&](int q) {
          if (!do_split) return;
          if (q == 1) split_load(cs.p, cs.kc, slot, split_first, split_next_new);
          if (q == 4) split_finish(cs.p, cs.kc, slot);
        });
      } else if (do_split) {
        split_load(cs.p, cs.kc, slot, split_first, split_next_new);
        split_finish(cs.p, cs.kc, slot);
      }
      if (do_ep) adv(ce);
    }
    if (k + 1 < nloc) adv(cn);
    if (do_split) adv(cs);
    step_barrier();
  }
}

}  // namespace
}  // namespace mvr

using namespace mvr;

extern "C" int mvr_pointcn_fused(const float* x, int64_t x_pstride, int64_t x_ld, float* y, int64_t y_pstride,
                                 int64_t y_ld, const float* sc1, const float* sh1, const float* sc2, const float* sh2,
                                 const float* w3, const float* b3, const float* w7, const float* b7, int P,
                                 int channels, int N, float* stats, int64_t st_ld, int st_off, hipStream_t stream) {
  if (!x || !y || !sc1 || !sh1 || !sc2 || !sh2 || !w3 || !w7 || P < 0 || N <= 0 || channels != PC) return MVR_EINVAL;
  if (stats && (st_off < 0 || st_ld < st_off + PC)) return MVR_EINVAL;
  const int64_t N4 = ((int64_t)N + 3) & ~(int64_t)3;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (x_ld < N4 || y_ld < N4 || (x_ld & 3) || (y_ld & 3) || (x_pstride & 3) || (y_pstride & 3) || !al16(x) ||
      !al16(y) || !al16(w3) || !al16(w7))
    return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  PcnArgs a{};
  a.X = x; a.xps = x_pstride; a.xld = x_ld;
  a.Y = y; a.yps = y_pstride; a.yld = y_ld;
  a.sc1 = sc1; a.sh1 = sh1; a.sc2 = sc2; a.sh2 = sh2;
  a.W3 = w3; a.b3 = b3; a.W7 = w7; a.b7 = b7;
  a.stats = reinterpret_cast<float2*>(stats); a.st_ld = st_ld; a.st_off = st_off;
  a.P = P; a.N = N; a.nch = (N + PCH - 1) / PCH;
  a.total = (int64_t)P * a.nch;
  const double fl = 4.0 * PC * PC * (double)N * P;
  const double by = 2.0 * 4.0 * PC * (double)N * P;
  ProfScope prof(PK_POINTCN, fl, by, stream);
  const int grid = (int)(a.total < 256 ? a.total : 256);
  hipLaunchKernelGGL(pointcn_chain_kernel, dim3(grid), dim3(512), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}
