// Point convolution of the OANet filter, 128 -> 128 channels over points (the PointCN convs,
// lib/filtering/oanet.py:18-43, and OAFilter conv3 on clusters, :86-92):
//
//   Y[b](m, n) = sum_k W(m, k) * pro(X[b](k, n)) + bias(m) (+ R[b](m, n)),   m, k < 128
//   pro(x) = relu(x * sc[b][k] + sh[b][k])   (InstanceNorm + BatchNorm + ReLU folded) or identity
//
// with the per-(pair, channel, 128-point tile) partial statistics of Y (sum, squared deviations
// from the tile mean) the next InstanceNorm needs — the same contract as gemm_kernel's ST_ROW
// epilogue (gemm.hpp), so the two are interchangeable per launch.
//
// Why a separate kernel: the generic GEMM stages both operands through LDS-DMA, splits the weights
// into bf16 terms again for every tile and splits every activation value in two waves (2x2 wave
// grid).  Here
//   * the weights are split once per workgroup and held as MFMA A-fragments in VGPRs (wave w owns
//     output rows 32w .. 32w+31 over all 128 k: 8 k-steps x 3 terms x 4 VGPRs),
//   * each activation value is loaded by exactly one lane, straight into MFMA B-fragment order
//     (lane l of wave w: column n0 + (l & 31), rows k = 32w + 16t + 8(l >> 5) + i — two 128-byte row
//     segments per load instruction), normalised, split once, and published to the other waves as
//     fragment planes in LDS (lane-linear 16-byte writes and reads, conflict-free),
//   * two 32-point chunks are in flight in registers while one is multiplied,
//   * the accumulator goes through a per-wave LDS scratch so that each lane owns 16 consecutive
//     columns of one row: float4 residual loads / stores and lane-local statistics.
// Workgroups own contiguous ranges of 128-point statistics groups (pair-major), so the partials of
// a group come from one workgroup and consecutive chunks of a workgroup share cache lines.
// Roofline: 2*128*128 flops per point-pair column against (128 + 128 (+128 residual)) * 4 bytes:
// AI = 32 (21 with the residual) flop/B < the split-MFMA ridge -> HBM-bound.
#include "common.hpp"
#include "gemm.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"

namespace mvr {

int g_pconv = 1;   // mvr_set_pconv: 0 routes these convs to gemm_kernel (A/B timing)

namespace {

using namespace bx;

constexpr int PC = 128;              // input = output channels
constexpr int CH = 32;               // points per chunk (one MFMA column block)
constexpr int GRP = 4;               // chunks per statistics group (128 points, gemm.hpp GEMM_BN)
constexpr int FRB = 3 * 64 * 16;     // one k-step's fragment set: h, m, l planes x 64 lanes x 16 B
constexpr int XIB = 8 * FRB;         // one chunk's B-fragment image (8 k-steps): 24 KB
constexpr int YLD = 33;              // row stride (floats) of the per-wave transpose scratch

struct PcArgs {
  const float* X; int64_t xps, xld;     // input [P][128][xld]
  float* Y; int64_t yps, yld;           // output [P][128][yld]
  const float* R; int64_t rps;          // residual [P][128][yld] (RES)
  const float* W; int64_t wld;          // weight [128][wld]
  const float* bias;                    // [128] or null
  const float* sc; const float* sh; int64_t sPb;   // prologue fold [P][sPb] (PRO)
  float2* stats; int64_t st_ld; int st_off;        // [P][ngrp][st_ld] (+ st_off + m) (STATS)
  int N, nch, ngrp;
  int64_t groups;                       // P * ngrp
};

template <int PRO, int RES, int STATS>
__global__ __launch_bounds__(256, 2) void pconv_kernel(PcArgs a) {
  __shared__ __attribute__((aligned(16))) char xi[2][XIB];
  __shared__ __attribute__((aligned(16))) float ys[4][32 * YLD];
  __shared__ __attribute__((aligned(16))) float fold[2][2][PC];   // (sc, sh) by pair parity

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.N, N4 = (N + 3) & ~3, nch = a.nch;

  // contiguous range of statistics groups -> chunk range [c0, c1) in (pair, chunk) order
  const int64_t G = a.groups;
  const int64_t g0 = G * blockIdx.x / gridDim.x, g1 = G * (blockIdx.x + 1) / gridDim.x;
  if (g0 >= g1) return;   // uniform
  const int p0 = (int)(g0 / a.ngrp), p1 = (int)(g1 / a.ngrp);
  const int64_t c0 = (int64_t)p0 * nch + GRP * (int)(g0 - (int64_t)p0 * a.ngrp);
  const int64_t c1 = (int64_t)p1 * nch + min(GRP * (int)(g1 - (int64_t)p1 * a.ngrp), nch);
  const int nloc = (int)(c1 - c0);

  // weights -> split A fragments: row 32w + l32, k = 16q + 8h + 0..7
  Frag wf[8];
  {
    const float* wr = a.W + (int64_t)(32 * w + l32) * a.wld + 8 * h;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 u0 = *reinterpret_cast<const float4*>(wr + 16 * q);
      const float4 u1 = *reinterpret_cast<const float4*>(wr + 16 * q + 4);
      const float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      split8(v, wf[q].h, wf[q].m, wf[q].l);
    }
  }
  // epilogue ownership: row 32w + erow, columns ec0 .. ec0 + 15 of the chunk
  const int erow = lane >> 1, ec0 = 16 * (lane & 1);
  const int orow = 32 * w + erow;
  const float bias = a.bias ? a.bias[orow] : 0.f;

  struct Cur {
    int p, kc;
  };
  auto adv = [&](Cur& c) {
    if (++c.kc == nch) { c.kc = 0; ++c.p; }
  };
  const Cur cstart{p0, (int)(c0 - (int64_t)p0 * nch)};

  auto stage_fold = [&](int p) {
    if (PRO && tid < PC) {
      fold[p & 1][0][tid] = a.sc[(int64_t)p * a.sPb + tid];
      fold[p & 1][1][tid] = a.sh[(int64_t)p * a.sPb + tid];
    }
  };
  // chunk c -> 16 registers in B-fragment order: k = 32w + 16t + 8h + i -> r[8t + i]
  auto issue_x = [&](const Cur& c, float (&r)[16]) {
    const int n = min(c.kc * CH + l32, N - 1);
    const float* src = a.X + (int64_t)c.p * a.xps + (int64_t)(32 * w + 8 * h) * a.xld + n;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 8; ++i) r[8 * t + i] = src[(int64_t)(16 * t + i) * a.xld];
  };
  // normalise + split chunk registers -> fragment image slot
  auto split_x = [&](const Cur& c, const float (&r)[16], int slot) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float v[8];
      if (PRO) {
        const float* f = &fold[c.p & 1][0][32 * w + 16 * t + 8 * h];
        const float4 sa = *reinterpret_cast<const float4*>(f), sb = *reinterpret_cast<const float4*>(f + 4);
        const float4 ha = *reinterpret_cast<const float4*>(f + PC), hb = *reinterpret_cast<const float4*>(f + PC + 4);
        const float s1[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
        const float h1[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaxf(fmaf(r[8 * t + i], s1[i], h1[i]), 0.f);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = r[8 * t + i];
      }
      Frag f;
      split8(v, f.h, f.m, f.l);
      char* dst = xi[slot] + (2 * w + t) * FRB + lane * 16;
      *reinterpret_cast<bf16x8*>(dst) = f.h;
      *reinterpret_cast<bf16x8*>(dst + 1024) = f.m;
      *reinterpret_cast<bf16x8*>(dst + 2048) = f.l;
    }
  };

  float rn = 0.f, rs = 0.f, rm2 = 0.f;   // running statistics of row orow over the current group
  float* yb = ys[w];
  // residual of chunk c (rows orow, columns ec0 .. ec0 + 15), addresses clamped into the padded row:
  // issued unconditionally one step ahead so that the compiler's vmcnt bookkeeping stays exact
  float4 rr[4];
  auto issue_r = [&](const Cur& c) {
    if (!RES) return;
    const float* rsrc = a.R + (int64_t)c.p * a.rps + (int64_t)orow * a.yld;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4)
      rr[i4] = *reinterpret_cast<const float4*>(rsrc + min(c.kc * CH + ec0 + 4 * i4, N4 - 4));
  };
  auto compute = [&](const Cur& c, int slot) {
    const int n0 = c.kc * CH;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const char* img = xi[slot] + lane * 16;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      Frag b;
      b.h = *reinterpret_cast<const bf16x8*>(img + ks * FRB);
      b.m = *reinterpret_cast<const bf16x8*>(img + ks * FRB + 1024);
      b.l = *reinterpret_cast<const bf16x8*>(img + ks * FRB + 2048);
      acc = mfma6(wf[ks], b, acc);
    }
    // transpose through the wave's scratch: register q = row (q & 3) + 8 (q >> 2) + 4h, column l32
#pragma unroll
    for (int q = 0; q < 16; ++q) yb[((q & 3) + 8 * (q >> 2) + 4 * h) * YLD + l32] = acc[q];
    float ev[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ev[i] = yb[erow * YLD + ec0 + i] + bias;
    if (RES) {
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        ev[4 * i4] += rr[i4].x; ev[4 * i4 + 1] += rr[i4].y; ev[4 * i4 + 2] += rr[i4].z; ev[4 * i4 + 3] += rr[i4].w;
      }
    }
    float* ydst = a.Y + (int64_t)c.p * a.yps + (int64_t)orow * a.yld + n0 + ec0;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4)
      if (n0 + ec0 + 4 * i4 < N4)
        reinterpret_cast<float4*>(ydst)[i4] = make_float4(ev[4 * i4], ev[4 * i4 + 1], ev[4 * i4 + 2], ev[4 * i4 + 3]);
    if (STATS) {
      const int nv = min(max(N - n0 - ec0, 0), 16);      // valid columns of this lane
      const int cnt = min(N - n0, CH);                    // ... of the chunk (>= 1)
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) s += i < nv ? ev[i] : 0.f;
      s += __shfl_xor(s, 1, 64);
      const float mu = s / (float)cnt;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float d = i < nv ? ev[i] - mu : 0.f;
        m2 = fmaf(d, d, m2);
      }
      m2 += __shfl_xor(m2, 1, 64);
      const float fc = (float)cnt;
      if (rn == 0.f) {
        rn = fc; rs = s; rm2 = m2;
      } else {   // Chan's merge
        const float d = mu - rs / rn;
        rm2 += m2 + d * d * (rn * fc / (rn + fc));
        rs += s;
        rn += fc;
      }
      if ((c.kc % GRP) == GRP - 1 || c.kc == nch - 1) {
        if ((lane & 1) == 0)
          a.stats[((int64_t)c.p * a.ngrp + c.kc / GRP) * a.st_ld + a.st_off + orow] = make_float2(rs, rm2);
        rn = 0.f;
      }
    }
  };

  // Step j: split chunk j (registers -> image j & 1), refill the registers with chunk j + 2, stage the
  // fold of chunk j + 1's pair when it starts one, barrier, multiply + epilogue of chunk j, then the
  // residual of chunk j + 1.  Loads past the range re-read the last chunk (unconditional issue keeps
  // every s_waitcnt the compiler derives a partial one: two chunks stay in flight).
  float xa[16], xb[16];
  Cur cs = cstart, cc = cstart, ci = cstart, cr = cstart;   // split, compute, x-issue, residual cursors
  stage_fold(cstart.p);
  issue_x(ci, xa);
  if (1 < nloc) adv(ci);
  issue_x(ci, xb);
  if (2 < nloc) adv(ci);
  issue_r(cr);
  if (1 < nloc) adv(cr);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  auto step = [&](int j, float (&xr)[16]) {
    split_x(cs, xr, j & 1);
    issue_x(ci, xr);
    if (j + 3 < nloc) adv(ci);
    adv(cs);
    if (j + 1 < nloc && cs.kc == 0) stage_fold(cs.p);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    compute(cc, j & 1);
    adv(cc);
    issue_r(cr);
    if (j + 2 < nloc) adv(cr);
  };
  int j = 0;
  for (; j + 1 < nloc; j += 2) {
    step(j, xa);
    step(j + 1, xb);
  }
  if (j < nloc) step(j, xa);
}

}  // namespace

// Dispatched by launch_gemm for the shapes it covers; the caller has checked the common contract.
bool pconv_covers(const GemmArgs& g) {
  return g_pconv && g.math == MATH_BF16X3 && g.M == PC && g.K == PC && !g.bkc && g.sAb == 0 && !g.no_store &&
         (g.pro == PRO_NONE || g.pro == PRO_B_K) && (g.stats_mode == ST_NONE || g.stats_mode == ST_ROW) &&
         g.bias_mode != BIAS_N && g.N > 0;
}

int launch_pconv(const GemmArgs& g, hipStream_t s) {
  PcArgs a{};
  a.X = g.B; a.xps = g.sBb; a.xld = g.ldb;
  a.Y = g.C; a.yps = g.sCb; a.yld = g.ldc;
  a.R = g.R; a.rps = g.sRb;
  a.W = g.A; a.wld = g.lda;
  a.bias = g.bias_mode == BIAS_M ? g.bias : nullptr;
  a.sc = g.psc; a.sh = g.psh; a.sPb = g.sPb;
  a.stats = g.stats; a.st_ld = g.st_ld; a.st_off = g.st_off;
  a.N = g.N;
  a.nch = (g.N + CH - 1) / CH;
  a.ngrp = (a.nch + GRP - 1) / GRP;
  a.groups = (int64_t)g.batch * a.ngrp;
  const int grid = (int)(a.groups < 512 ? a.groups : 512);
  const int pro = g.pro == PRO_B_K, res = g.has_res != 0, st = g.stats_mode == ST_ROW;
#define MVR_PC(P_, R_, S_)                                                                  \
  if (pro == P_ && res == R_ && st == S_) {                                                 \
    hipLaunchKernelGGL((pconv_kernel<P_, R_, S_>), dim3(grid), dim3(256), 0, s, a);         \
    MVR_CHECK_LAUNCH();                                                                     \
    return MVR_OK;                                                                          \
  }
  MVR_PC(1, 0, 1)
  MVR_PC(1, 1, 1)
  MVR_PC(1, 0, 0)
  MVR_PC(1, 1, 0)
  MVR_PC(0, 0, 1)
  MVR_PC(0, 1, 1)
  MVR_PC(0, 0, 0)
  MVR_PC(0, 1, 0)
#undef MVR_PC
  return MVR_EINVAL;
}

}  // namespace mvr

extern "C" int mvr_set_pconv(int on) {
  const int prev = mvr::g_pconv;
  mvr::g_pconv = on ? 1 : 0;
  return prev;
}
