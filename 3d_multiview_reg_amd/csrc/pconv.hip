// Point convolution of the OANet filter, 128 (or 256) -> 128 channels over points (the PointCN convs,
// lib/filtering/oanet.py:18-43, the 256-channel first PointCN after diff_unpool, :155, and OAFilter
// conv3 on clusters, :86-92):
//
//   Y[b](m, n) = sum_k W(m, k) * pro(X[b](k, n)) + bias(m) (+ R[b](m, n)),   m < 128, k < 128 (256)
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

#ifndef PCONV_POISON
#define PCONV_POISON 0
#endif
#ifndef PCONV_NTS
#define PCONV_NTS 1   // nontemporal output stores (-2 % per launch, tools/jobs A/B)
#endif
#ifndef PCONV_NTR
#define PCONV_NTR 0   // experiment: nontemporal residual loads
#endif
#ifndef PCONV_NTL
#define PCONV_NTL 2   // cache-policy bits of the activation buffer loads: nt (streamed once; -3 % per step's point convs)
#endif

#ifndef PCONV_TRACE
#define PCONV_TRACE 0   // 1: per-phase cycle totals per wave (s_memtime) of the KS = 8 kernels, tools only (mvr_pconv_trace)
#endif
#if PCONV_TRACE
__device__ unsigned long long g_pconv_trace[8];   // 0 MFMAs (+ splits, load issue), 1 epilogue, 2 step bookkeeping,
                                                  // 3 step barrier, 4 prologue, 5 tail
#define PCSTAMP(slot)                                                  \
  do {                                                                 \
    unsigned long long t_;                                             \
    __builtin_amdgcn_sched_barrier(0);                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));  \
    __builtin_amdgcn_sched_barrier(0);                                 \
    ptr_[pprev_] += t_ - plast_;                                       \
    plast_ = t_;                                                       \
    pprev_ = (slot);                                                   \
  } while (0)
#else
#define PCSTAMP(slot) do {} while (0)
#endif

#ifndef PCONV_BUF
#define PCONV_BUF 1   // the residual loads and the output stores through a per-pair buffer resource with 32-bit lane offsets
                      // (0: 64-bit per-lane addresses; conv7 then held 256 VGPRs with 2 spilled and 42 register copies
                      // per step pair: bit-identical, -0.2 ms per step, profiles/r06/ab_r6s22_pconv_buffer.txt)
#endif

#ifndef PCONV_GRID
#define PCONV_GRID 1   // workgroups per resident slot (1: one persistent round; >1 / <0: the round-4 grid experiments)
#endif
#ifndef PCONV_MATH_DEFAULT
#define PCONV_MATH_DEFAULT 0
#endif
int g_pconv_h = PCONV_MATH_DEFAULT;   // mvr_set_math: 0 split-bf16 (fp32-equivalent, default), 1 split-fp16
                                      // (re-run in split-bf16 when out of range)

namespace {

using namespace bx;

constexpr int PC = 128;              // output channels (input channels: 16 KS, KS = 8 or 16 k-steps)
constexpr int CH = 32;               // points per chunk (one MFMA column block)
constexpr int GRP = 4;               // chunks per statistics group (128 points, gemm.hpp GEMM_BN)
constexpr int YLD = 32;              // row stride (floats) of the per-wave transpose scratch

// Activation layouts (per operand): element (row k, point n) at k ld + (n >> 5) cs + (n & 31) — row-major
// [rows][ld] with cs = 32, or chunk-major [N / 32][rows][32] with ld = 32, cs = 32 rows (oanet.hip: every 32-point
// chunk of a pair one contiguous block, so a chunk's loads and stores are whole 16 KB blocks instead of 128 row
// segments 128 bytes long)
struct PcArgs {
  const float* X; int64_t xps, xld, xcs;   // input [P][128][xld]
  float* Y; int64_t yps, yld, ycs;         // output [P][128][yld]
  const float* R; int64_t rps, rrs, rcs;   // residual (RES): rows rrs apart
  const float* W; int64_t wld;          // weight [128][wld]
  const float* bias;                    // [128] or null
  const float* sc; const float* sh; int64_t sPb;   // prologue fold [P][sPb] (PRO)
  float2* stats; int64_t st_ld; int st_off;        // [P][ngrp][st_ld] (+ st_off + m) (STATS)
  int N, nch, ngrp;
  int64_t groups;                       // P * ngrp
  const float* hw; const float* hb;     // HEAD: output conv 128 -> 1 (oanet.py:163)
  float* logits; float* scores; int32_t* pos;   // [P][N], [P][N], [P]
  int xci; const float* xw; const float* xb;    // XI: x(k, n) = xb[k] + xw[k][:xci] . in(:, n) (xw [128][8])
  int64_t rld;                                  // XI & 2: row stride of the block input R
  int* range; const int* guard; int epoch;      // split-fp16: the caller's zeroed flag word, set to epoch (1) when an
                                                // activation is out of range; split-bf16 re-run: return unless *guard == epoch
  // the output's InstanceNorm fold, finished by the workgroup that completes a pair's statistics (GemmArgs fin_*)
  int* fcnt; float feps; mvr_bn_p fbn; float* fsc; float* fsh; int64_t fld;
  float feps2; mvr_bn_p fbn2; float* fsc2; float* fsh2; int ftrain; float2* fmv;
};

// (sc, sh) of IN(eps) + BN(eval) from the pooled (mean, var): in_finalize_kernel's arithmetic
__device__ __forceinline__ void fold_write(const mvr_bn_p& bn, float eps, double mean, double var, float* sc, float* sh,
                                           int64_t at, int c) {
  const float rin = (float)(1.0 / sqrt(var + (double)eps));
  float g = 1.f, b = 0.f, rm = 0.f, rs = 1.f;
  if (bn.gamma) {
    g = bn.gamma[c];
    b = bn.beta[c];
    rm = bn.mean[c];
    rs = 1.f / sqrtf(bn.var[c] + 1e-5f);
  }
  const float gs = g * rs;
  sc[at] = rin * gs;
  sh[at] = (float)((double)b - (mean * (double)rin + (double)rm) * (double)gs);
}

// Fused InstanceNorm finalize of pair p (the caller is the workgroup whose counter arrival completed the pair's
// statistics): the 128 channels' partials of its T = ngrp 128-point tiles (read with device-coherent loads: the
// producers wrote them with device-coherent stores, so no L2 write-back or invalidation is needed) merged
// exactly as in_finalize_kernel does for 128 channels (4 tile groups t = g, g + 4, ..., their double partials
// combined in group order; Chan's merge), so the fold is bit-identical to the separate launch's.
// red: 4 x 128 doubles of LDS scratch; threads 0..255 take part, every thread of the workgroup reaches the barriers.
__device__ __forceinline__ float2 ld_coherent(const float2* q) {
  return __builtin_bit_cast(float2, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(q), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
__device__ void fin_pair(const PcArgs& a, int p, double* red, int tid) {
  const int T = a.ngrp, L = a.N, c = tid & 127, g0 = 2 * ((tid >> 7) & 1);
  const bool act = tid < 256;
  const float2* sp = a.stats + (int64_t)p * T * a.st_ld + a.st_off + c;
  if (act) {
    double t0 = 0.0, t1 = 0.0;
#pragma unroll 4
    for (int t = g0; t < T; t += 4) t0 += (double)ld_coherent(sp + (int64_t)t * a.st_ld).x;
#pragma unroll 4
    for (int t = g0 + 1; t < T; t += 4) t1 += (double)ld_coherent(sp + (int64_t)t * a.st_ld).x;
    red[g0 * 128 + c] = t0;
    red[(g0 + 1) * 128 + c] = t1;
  }
  __syncthreads();
  double tot = 0.0;
  for (int j = 0; j < 4; ++j) tot += red[j * 128 + c];
  const double mean = tot / L, rtw = 1.0 / 128;
  double m2[2] = {0.0, 0.0};
  if (act) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll 4
      for (int t = g0 + u; t < T; t += 4) {
        const float2 v = ld_coherent(sp + (int64_t)t * a.st_ld);
        const int nv = min(128, L - 128 * t);
        const double d = (double)v.x * (nv == 128 ? rtw : 1.0 / nv) - mean;
        m2[u] += (double)v.y + d * d * nv;
      }
    }
  }
  __syncthreads();   // every group has read the sums
  if (act) {
    red[g0 * 128 + c] = m2[0];
    red[(g0 + 1) * 128 + c] = m2[1];
  }
  __syncthreads();
  if (tid < 128) {
    double m = 0.0;
    for (int j = 0; j < 4; ++j) m += red[j * 128 + c];
    const double var = fmax(m / L, 0.0);
    if (a.ftrain) {
      a.fmv[(int64_t)p * PC + c] = make_float2((float)mean, (float)var);
    } else {
      fold_write(a.fbn, a.feps, mean, var, a.fsc, a.fsh, (int64_t)p * a.fld + c, c);
      if (a.fsc2) fold_write(a.fbn2, a.feps2, mean, var, a.fsc2, a.fsh2, (int64_t)p * a.fld + c, c);
    }
  }
  __syncthreads();   // red is reused by the next pair
}

// lastp: 32 x YLD ints of LDS scratch ([0] count, [1..] the pairs this workgroup completes), red: fin_pair's
__device__ void fin_tail(const PcArgs& a, int* lastp, double* red, int tid) {
  const int64_t G = a.groups;
  const int64_t g0 = G * blockIdx.x / gridDim.x, g1 = G * (blockIdx.x + 1) / gridDim.x;
  if (g0 >= g1) return;   // uniform (such a workgroup returned before its main loop anyway)
  // every lane's statistics stores (device-coherent) complete before the arrival: no agent-scope release fence,
  // whose L2 write-back (buffer_wbl2) and, on the acquire side, L2 invalidation (buffer_inv) cost every workgroup
  // of the launch and every other kernel on the XCD their cached lines
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int nl = 0;
    const int pfirst = (int)(g0 / a.ngrp), plast = (int)((g1 - 1) / a.ngrp);
    for (int p = pfirst; p <= plast; ++p) {
      const int64_t lo = g0 > (int64_t)p * a.ngrp ? g0 : (int64_t)p * a.ngrp;
      const int64_t hi = g1 < (int64_t)(p + 1) * a.ngrp ? g1 : (int64_t)(p + 1) * a.ngrp;
      const int n = (int)(hi - lo);
      const int old = __hip_atomic_fetch_add(a.fcnt + p, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + n == a.ngrp && nl < 32 * YLD - 1) lastp[1 + nl++] = p;
    }
    lastp[0] = nl;
  }
  __syncthreads();
  const int nl = lastp[0];
  for (int i = 0; i < nl; ++i) fin_pair(a, lastp[1 + i], red, tid);
}

#define PC_FENCE() __builtin_amdgcn_sched_barrier(0)

// sum over the 8 lanes 8g .. 8g+7 (all of them receive it): quad butterflies, then the half-row mirror
__device__ __forceinline__ float sum8(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));  // row_half_mirror
  return v;
}

// KS = 8: 128 input channels, two workgroups per CU (weights 96 VGPRs per lane).  KS = 16: the
// 256 -> 128 convs of the first PointCN after diff_unpool (oanet.py:155), one workgroup per CU
// (weights 192 VGPRs, chunk images 2 x 48 KB).  HEAD = 2: output head only, Y not stored (the
// block's last conv when its activation is not returned).
// XI: the block's conv1 (oanet.py:144-145, Cin = 6 or 8 -> 128) folded into its first PointCN, so its
// 128-channel output x is never stored: XI = 1, the B operand rows are recomputed from the block input
// (8 loads per point instead of 128 rows); XI = 2, the residual (RES) is recomputed from it.  Both use
// the same fma order, so the two recomputations of x are bit-identical.
// KW = 2 (KS = 16 only): 8 waves, the reduction split in two halves — wave w multiplies row block
// w & 3 over input channels 128 (w >> 2) .. +127 (96 weight VGPRs, two waves per SIMD, where the 4-wave
// KS = 16 form has one wave per SIMD and cannot overlap its MFMA chain with its own memory waits); the
// upper half's partial sums reach the lower half's waves through LDS one step later, which then run the
// epilogue for both (no residual / head there).
// H = 1: split-fp16 operands (mfma_bf16.hpp: 3 MFMAs per product instead of 6, 2-plane images).  Each
// weight row is scaled by a power of two to <= 2^14 and the activations by XS = 2^6 as they are split
// (activations are O(1) — IN + BN + ReLU outputs, or the block's residual stream —: 22-bit precision down to
// 2^-9, below 65504 up to 1023); the epilogue undoes both per row.  A lane that splits an activation of
// 1023.5 or more, or whose activations (8 input rows over all its chunks) are all below 2^-9 without being
// all zero, marks the launch, whose split-bf16 re-run then replaces every output.
template <int KS, int PRO, int RES, int STATS, int HEAD, int XI = 0, int KW = 1, int H = 0>
__global__ __launch_bounds__(256 * KW, KS == 8 ? 2 : 1) void pconv_kernel(PcArgs a) {
  constexpr int CIN = 16 * KS;   // input channels
  constexpr int FRBT = planes<H>() * 1024;     // one k-step's fragment set: planes x 64 lanes x 16 B
  constexpr float XS = H ? 64.f : 1.f;
  static_assert(!H || HEAD == 0, "the head's positive counts are not re-runnable");
  if (a.guard && *a.guard != a.epoch) return;   // uniform: the split-fp16 launch stayed in range
  constexpr int NWV = 4 * KW;    // waves
  constexpr int KSW = KS / KW;   // k-steps each wave multiplies
  constexpr int NT = KS / NWV;   // 16-row k-steps each wave loads and splits per chunk
  constexpr int RW = CIN / NWV;  // input rows per wave
  constexpr int NX = (XI & 1) ? 8 : 8 * NT;   // activation registers per chunk
  static_assert(!XI || KS == 8, "conv1 folding: 128-channel convs");
  static_assert(KW == 1 || (KS == 16 && KW == 2 && !RES && !HEAD && !XI), "k-split: the 256 -> 128 convs");
  __shared__ __attribute__((aligned(16))) char xi[2][KS * FRBT];     // chunk images (B fragments)
  __shared__ float srisc[H ? PC : 1];                                // H = 1: 1 / (row scale XS)
  __shared__ __attribute__((aligned(16))) float ys[4][32 * YLD];   // per wave: residual DMA / transpose
  __shared__ __attribute__((aligned(16))) float fold[2][2][CIN];   // (sc, sh) by pair parity
  __shared__ float sbias[PC];
  __shared__ float shw[HEAD ? PC : 1];
  __shared__ __attribute__((aligned(16))) float hpart[HEAD ? 2 : 1][4][CH];   // HEAD: per-wave partial logits by step parity
  __shared__ __attribute__((aligned(16))) float xws[XI ? PC : 1][8];   // XI: conv1 weights, bias
  __shared__ float xbs[XI ? PC : 1];
  // XI & 2: the same weights as float4 over an epilogue lane's 4 rows 32w + erow + 8q: [ci][w][erow][q], bias [w][erow][q]
  __shared__ __attribute__((aligned(16))) float xwe[(XI & 2) ? 8 : 1][(XI & 2) ? PC : 4];
  __shared__ __attribute__((aligned(16))) float xbe[(XI & 2) ? PC : 4];
  __shared__ __attribute__((aligned(16))) float xib[(XI & 2) ? 4 : 1][(XI & 2) ? 256 : 4];   // per wave: input chunk
  // KW = 2: the upper half's partial accumulators by chunk parity, [slot][row block][q][lane] float4 planes
  __shared__ __attribute__((aligned(16))) float4 xch[KW == 2 ? 2 : 1][KW == 2 ? 4 : 1][KW == 2 ? 4 : 1][KW == 2 ? 64 : 1];

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
#if PCONV_TRACE
  unsigned long long ptr_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, plast_ = __builtin_amdgcn_s_memtime();
  int pprev_ = 4;
#endif
#if PCONV_POISON   // debugging: NaN in every LDS array before use (finds reads of data never written)
  {
    auto poison = [&](void* p, size_t bytes) {
      float* f = reinterpret_cast<float*>(p);
      for (size_t i = tid; i < bytes / 4; i += blockDim.x) f[i] = __builtin_nanf("");
    };
    poison(xi, sizeof(xi)); poison(ys, sizeof(ys)); poison(fold, sizeof(fold)); poison(sbias, sizeof(sbias));
    poison(shw, sizeof(shw)); poison(hpart, sizeof(hpart)); poison(xws, sizeof(xws));
    poison(xbs, sizeof(xbs)); poison(xwe, sizeof(xwe)); poison(xbe, sizeof(xbe)); poison(xib, sizeof(xib));
    poison(xch, sizeof(xch));
    __syncthreads();
  }
#endif
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave (loads / splits input rows RW wv ..)
  const int w = wv & 3;                                      // output row block
  const int kh = wv >> 2;                                    // KW = 2: reduction half
  const int N = a.N, N4 = (N + 3) & ~3, nch = a.nch;

  // contiguous range of statistics groups -> chunk range [c0, c1) in (pair, chunk) order
  const int64_t G = a.groups;
  const int64_t g0 = G * blockIdx.x / gridDim.x, g1 = G * (blockIdx.x + 1) / gridDim.x;
  if (g0 >= g1) return;   // uniform
  const int p0 = (int)(g0 / a.ngrp), p1 = (int)(g1 / a.ngrp);
  const int64_t c0 = (int64_t)p0 * nch + GRP * (int)(g0 - (int64_t)p0 * a.ngrp);
  const int64_t c1 = (int64_t)p1 * nch + min(GRP * (int)(g1 - (int64_t)p1 * a.ngrp), nch);
  const int nloc = (int)(c1 - c0);

  // weights -> split A fragments: row 32w + l32, k = 128 kh + 16q + 8h + 0..7 (H = 1: the row scaled)
  FragT<H> wf[KSW];
  {
    const float* wrow = a.W + (int64_t)(32 * w + l32) * a.wld;
    float wsc = 1.f;
    if (H) {   // the whole row (every lane of the row's waves / halves derives the same scale)
      float amax = 0.f;
      for (int k = 0; k < CIN; k += 4) {
        const float4 u = *reinterpret_cast<const float4*>(wrow + k);
        amax = fmaxf(fmaxf(amax, fmaxf(fabsf(u.x), fabsf(u.y))), fmaxf(fabsf(u.z), fabsf(u.w)));
      }
      wsc = range_scale(amax);
      if (kh == 0 && h == 0) srisc[32 * w + l32] = 1.f / (wsc * XS);   // published by the prologue barriers
    }
    const float* wr = wrow + 128 * kh * (KW - 1) + 8 * h;
#pragma unroll
    for (int q = 0; q < KSW; ++q) {
      const float4 u0 = *reinterpret_cast<const float4*>(wr + 16 * q);
      const float4 u1 = *reinterpret_cast<const float4*>(wr + 16 * q + 4);
      const float v[8] = {u0.x * wsc, u0.y * wsc, u0.z * wsc, u0.w * wsc, u1.x * wsc, u1.y * wsc, u1.z * wsc, u1.w * wsc};
      wf[q] = split8t<H>(v);
    }
  }
  bool xbad = false;   // H = 1: an activation of this lane's splits past the fp16 range
  float xmx = 0.f;     // H = 1: max |activation| x XS of this lane's splits
  // epilogue ownership: rows 32w + erow + 8q (q = 0..3), columns ec0 .. ec0 + 3 of the chunk — each
  // float4 store instruction of the wave then writes 8 whole 128-byte row segments
  const int erow = lane >> 3, ec0 = 4 * (lane & 7);
  if (tid < PC) sbias[tid] = a.bias ? a.bias[tid] : 0.f;   // published by the prologue barriers
  if (HEAD && tid < PC) shw[tid] = a.hw[tid];
  if (XI && tid < PC) {
    const int k = tid, ke = (k & ~31) + 4 * (k & 7) + ((k >> 3) & 3);   // (w, erow, q) slot of row k
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      xws[k][c] = a.xw[k * 8 + c];
      if (XI & 2) xwe[c][ke] = a.xw[k * 8 + c];
    }
    xbs[k] = a.xb ? a.xb[k] : 0.f;
    if (XI & 2) xbe[ke] = xbs[k];
  }

  // chunk cursor (pair, chunk in pair); cursors past the range stay on the last chunk (clamped
  // re-reads keep the issue unconditional, hence every s_waitcnt the compiler derives exact)
  struct Cur {
    int p, kc, j;
  };
  auto adv = [&](Cur& c) {
    if (c.j + 1 >= nloc) return;
    ++c.j;
    if (++c.kc == nch) { c.kc = 0; ++c.p; }
  };
  const Cur cstart{p0, (int)(c0 - (int64_t)p0 * nch), 0};

  auto stage_fold = [&](int p) {
    if (PRO && tid < CIN) {
      fold[p & 1][0][tid] = a.sc[(int64_t)p * a.sPb + tid];
      fold[p & 1][1][tid] = a.sh[(int64_t)p * a.sPb + tid];
    }
  };
  // chunk c -> NX registers in B-fragment order: k = RW w + 16t + 8h + i -> r[8t + i].  Buffer loads on
  // a per-(pair, wave) descriptor: the row offsets (16t + i) ld are wave-uniform (soffset), the lane's
  // (8h rows, column) part one voffset per chunk — no per-load 64-bit address arithmetic.
  const int xld4 = (int)a.xld * 4;
  auto issue_x = [&](const Cur& c, float (&r)[NX]) {
    const int n = min(c.kc * CH + l32, N - 1);
    const float* base = a.X + (int64_t)c.p * a.xps + (int64_t)(RW * wv) * a.xld;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
    if (XI & 1) {   // the block input's rows 0 .. xci-1 (clamped: weight columns past xci are zero)
      const float* ib = a.X + (int64_t)c.p * a.xps;
      const __amdgpu_buffer_rsrc_t ri =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ib), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int i = 0; i < NX; ++i)
        r[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, 4 * n, min(i, a.xci - 1) * xld4, 0));
      return;
    }
    const int vo = 8 * h * xld4 + 4 * ((n >> 5) * (int)a.xcs + (n & 31));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        r[8 * t + i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, (16 * t + i) * xld4,
                                                                                      PCONV_NTL));
  };
  // normalise + split half t of a chunk's registers -> its k-step fragment in image slot
  auto split_half = [&](const Cur& c, const float (&r)[NX], int slot, int t) {
    float v[8];
    float xr[8];   // the B rows of this half as loaded, or (XI & 1) recomputed from the block input
    if (XI & 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = RW * w + 16 * t + 8 * h + i;
        const float4 w0 = *reinterpret_cast<const float4*>(&xws[k][0]), w1 = *reinterpret_cast<const float4*>(&xws[k][4]);
        float acc = xbs[k];
        acc = fmaf(w0.x, r[0], acc); acc = fmaf(w0.y, r[1], acc); acc = fmaf(w0.z, r[2], acc); acc = fmaf(w0.w, r[3], acc);
        acc = fmaf(w1.x, r[4], acc); acc = fmaf(w1.y, r[5], acc); acc = fmaf(w1.z, r[6], acc); acc = fmaf(w1.w, r[7], acc);
        xr[i] = acc;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xr[i] = r[8 * t + i];
    }
    if (PRO) {
      const float* f = &fold[c.p & 1][0][RW * wv + 16 * t + 8 * h];
      const float4 sa = *reinterpret_cast<const float4*>(f), sb = *reinterpret_cast<const float4*>(f + 4);
      const float4 ha = *reinterpret_cast<const float4*>(f + CIN), hb = *reinterpret_cast<const float4*>(f + CIN + 4);
      const float s1[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
      const float h1[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaxf(fmaf(xr[i], s1[i], h1[i]), 0.f);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = xr[i];
    }
    char* dst = xi[slot] + (NT * wv + t) * FRBT + lane * 16;
    if (H) {
      float mx = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[i] *= XS;
        mx = fmaxf(mx, fabsf(v[i]));
      }
      xbad |= !(mx < F16_RANGE);
      xmx = fmaxf(xmx, mx);
      const FragT<H> f = split8t<H>(v);
#pragma unroll
      for (int pl = 0; pl < planes<H>(); ++pl) *reinterpret_cast<typename FragT<H>::V*>(dst + 1024 * pl) = f.p[pl];
      return;
    }
    Frag f;
    split8(v, f.h, f.m, f.l);
    *reinterpret_cast<bf16x8*>(dst) = f.h;
    *reinterpret_cast<bf16x8*>(dst + 1024) = f.m;
    *reinterpret_cast<bf16x8*>(dst + 2048) = f.l;
  };

  // residual of chunk c, loaded one step ahead into registers: this lane's rows 32w + erow + 8q (q = 0..3)
  // x columns ec0 .. ec0 + 3 of the chunk, exactly the values its epilogue owns (no LDS trip); XI & 2: the
  // lane's 16 bytes of the block input's 8 rows x 32 columns (row lane / 8, columns 4 (lane & 7)), which
  // the epilogue publishes to the wave's xib for the recomputation.  Columns clamped into the padded row.
  // (These were LDS-DMAs once: an LDS-DMA does not complete in order with loads into registers, so the
  // vmcnt counts that were meant to cover it did not — run-to-run differences under load.)
  float* yb = ys[w];
  float4 rres[(RES && !(XI & 2)) ? 4 : 1];
  float4 rxi;
  auto load_r = [&](const Cur& c) {
    if (!RES) return;
    const int n = min(c.kc * CH + ec0, N4 - 4);
    if (XI & 2) {
      rxi = *reinterpret_cast<const float4*>(a.R + (int64_t)c.p * a.rps + (int64_t)min(lane >> 3, a.xci - 1) * a.rld + n);
      return;
    }
    if (PCONV_BUF) {   // the pair's residual as a buffer (wave-uniform base), 32-bit lane offsets
      const __amdgpu_buffer_rsrc_t rr =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.R + (int64_t)c.p * a.rps), (short)0, 0x7fffffff, 0x00020000);
      const int ro = 4 * ((32 * w + erow) * (int)a.rrs + (n >> 5) * (int)a.rcs + (n & 31));
#pragma unroll
      for (int q = 0; q < 4; ++q)
        rres[(RES && !(XI & 2)) ? q : 0] = __builtin_bit_cast(
            float4, __builtin_amdgcn_raw_buffer_load_b128(rr, ro + 4 * 8 * q * (int)a.rrs, 0, 0));
      return;
    }
    const float* src = a.R + (int64_t)c.p * a.rps + (int64_t)(32 * w + erow) * a.rrs + (int64_t)(n >> 5) * a.rcs + (n & 31);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (PCONV_NTR) {
        const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (int64_t)(8 * q) * a.rrs));
        rres[(RES && !(XI & 2)) ? q : 0] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                                                       __uint_as_float(u.w));
      } else {
        rres[(RES && !(XI & 2)) ? q : 0] = *reinterpret_cast<const float4*>(src + (int64_t)(8 * q) * a.rrs);
      }
    }
  };

  // running statistics of the current 128-point group, per lane (its 4 rows x 4 columns of each chunk):
  // sums of d = y - K and d^2 with the row shift K = the mean of the group's first chunk (8-lane sums);
  // the lanes of a row meet once per group
  int rn = 0;
  float ls[4], lss[4];
  // multiply chunk c (image slot) with hook(ks) after each k-step's MFMA group, then the epilogue
  // multiply chunk (image slot) with hook(ks) after each k-step's MFMA group
  auto mfma = [&](int slot, auto&& hook) {
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const char* img = xi[slot] + KSW * kh * (KW - 1) * FRBT + lane * 16;
    FragT<H> cur = ld_frag<H>(img, 1024);
#pragma unroll
    for (int ks = 0; ks < KSW; ++ks) {
      FragT<H> nxt;
      if (ks < KSW - 1) nxt = ld_frag<H>(img + (ks + 1) * FRBT, 1024);
      PC_FENCE();
      acc = mma<H>(wf[ks], cur, acc);
      hook(ks);
      PC_FENCE();
      if (ks < KSW - 1) cur = nxt;
    }
    return acc;
  };
  // epilogue of chunk c (accumulator acc): bias (+ residual), stores, head, statistics
  auto epilogue = [&](const Cur& c, const floatx16& acc) {
    const int n0 = c.kc * CH;
    // value (q, e) of this lane: row erow + 8q of the wave's 32, column n0 + ec0 + e
    float4 ev[4];
    if (RES && !(XI & 2)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) ev[q] = rres[(RES && !(XI & 2)) ? q : 0];
    } else {
      if (XI & 2) *reinterpret_cast<float4*>(xib[w] + 32 * (lane >> 3) + 4 * (lane & 7)) = rxi;   // read below by this wave
#pragma unroll
      for (int q = 0; q < 4; ++q) ev[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // transpose through the wave's scratch: accumulator register r = row (r & 3) + 8 (r >> 2) + 4h, column l32
#pragma unroll
    for (int r = 0; r < 16; ++r) yb[((r & 3) + 8 * (r >> 2) + 4 * h) * YLD + l32] = acc[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 v = *reinterpret_cast<const float4*>(yb + (erow + 8 * q) * YLD + ec0);
      if (H) {
        const float is = srisc[32 * w + erow + 8 * q];
        v.x *= is; v.y *= is; v.z *= is; v.w *= is;
      }
      const float bq = sbias[32 * w + erow + 8 * q];
      ev[q].x += v.x + bq; ev[q].y += v.y + bq; ev[q].z += v.z + bq; ev[q].w += v.w + bq;
    }
    if (XI & 2) {   // + x, recomputed for the lane's 4 rows x 4 columns in split_half's fma order
      int e0 = 32 * w + 4 * erow;   // this lane's (w, erow) slot of xwe / xbe
      asm volatile("" : "+v"(e0));   // opaque per chunk: the weight reads stay here (hoisted out of the chunk
                                     // loop they would occupy registers across it and spill)
      const float* xi = xib[w];
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // one row at a time (register pressure)
        const float b = xbe[e0 + q];
        float4 xq = make_float4(b, b, b, b);
#pragma unroll
        for (int ci = 0; ci < 8; ++ci) {
          const float4 v = *reinterpret_cast<const float4*>(xi + ci * 32 + ec0);
          const float wq = xwe[ci][e0 + q];
          xq.x = fmaf(wq, v.x, xq.x); xq.y = fmaf(wq, v.y, xq.y); xq.z = fmaf(wq, v.z, xq.z); xq.w = fmaf(wq, v.w, xq.w);
        }
        // x + conv7 output (fp32 addition commutes: the reference's x + out)
        ev[q].x += xq.x; ev[q].y += xq.y; ev[q].z += xq.z; ev[q].w += xq.w;
        PC_FENCE();
      }
    }
    float* ydst = a.Y + (int64_t)c.p * a.yps + (int64_t)(32 * w + erow) * a.yld + (int64_t)c.kc * a.ycs + ec0;
    const bool full = n0 + CH <= N;   // uniform: every column of the chunk is valid
    if (PCONV_BUF && HEAD != 2 && a.Y) {   // the pair's output as a buffer, 32-bit lane offsets
      const __amdgpu_buffer_rsrc_t ry =
          __builtin_amdgcn_make_buffer_rsrc(a.Y + (int64_t)c.p * a.yps, (short)0, 0x7fffffff, 0x00020000);
      const int yo = 4 * ((32 * w + erow) * (int)a.yld + c.kc * (int)a.ycs + ec0);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (full || n0 + ec0 < N4) {
          const u32x4 u = {__float_as_uint(ev[q].x), __float_as_uint(ev[q].y), __float_as_uint(ev[q].z),
                           __float_as_uint(ev[q].w)};
          __builtin_amdgcn_raw_buffer_store_b128(u, ry, yo + 4 * 8 * q * (int)a.yld, 0, PCONV_NTS ? 2 : 0);
        }
    } else if (HEAD != 2 && a.Y) {   // (a.Y null: a statistics-only pass)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (full || n0 + ec0 < N4) {
          if (PCONV_NTS) {
            const u32x4 u = {__float_as_uint(ev[q].x), __float_as_uint(ev[q].y), __float_as_uint(ev[q].z),
                             __float_as_uint(ev[q].w)};
            __builtin_nontemporal_store(u, reinterpret_cast<u32x4*>(ydst + (int64_t)(8 * q) * a.yld));
          } else {
            *reinterpret_cast<float4*>(ydst + (int64_t)(8 * q) * a.yld) = ev[q];
          }
        }
    }
    if (HEAD) {   // partial logits of the wave's 32 rows for the chunk's columns, summed over lanes l ^ 8, 16, 32
      float hp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float wq = shw[32 * w + erow + 8 * q];
        hp[0] = fmaf(wq, ev[q].x, hp[0]); hp[1] = fmaf(wq, ev[q].y, hp[1]);
        hp[2] = fmaf(wq, ev[q].z, hp[2]); hp[3] = fmaf(wq, ev[q].w, hp[3]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hp[e] += __shfl_xor(hp[e], 8, 64);
        hp[e] += __shfl_xor(hp[e], 16, 64);
        hp[e] += __shfl_xor(hp[e], 32, 64);
      }
      if (lane < 8) *reinterpret_cast<float4*>(&hpart[c.j & 1][w][ec0]) = make_float4(hp[0], hp[1], hp[2], hp[3]);
    }
    if (STATS) {
      const int cnt = min(N - n0, CH);   // valid columns of the chunk (>= 1)
      const int nv = full ? 4 : min(max(N - n0 - ec0, 0), 4);
      if (!full) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (nv < 4) ev[q].w = 0.f;
          if (nv < 3) ev[q].z = 0.f;
          if (nv < 2) ev[q].y = 0.f;
          if (nv < 1) ev[q].x = 0.f;
        }
      }
      // row shift of the running sums: the row's bias (a constant, so no state crosses chunks — a shift kept
      // in LDS from the group's first chunk gave run-to-run differences; y - bias is the conv (+ residual)
      // term, O(its spread), so SS - S^2 / n keeps fp32 accuracy)
      float sK[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) sK[q] = sbias[32 * w + erow + 8 * q];
      if (c.kc % GRP == 0) {   // the group's first chunk
#pragma unroll
        for (int q = 0; q < 4; ++q) ls[q] = lss[q] = 0.f;
        rn = 0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float d0 = ev[q].x - sK[q], d1 = ev[q].y - sK[q], d2 = ev[q].z - sK[q], d3 = ev[q].w - sK[q];
        if (!full) {
          if (nv < 4) d3 = 0.f;
          if (nv < 3) d2 = 0.f;
          if (nv < 2) d1 = 0.f;
          if (nv < 1) d0 = 0.f;
        }
        ls[q] += (d0 + d1) + (d2 + d3);
        lss[q] = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, lss[q]))));
      }
      rn += cnt;
      if ((c.kc % GRP) == GRP - 1 || c.kc == nch - 1) {
        // (sum, squared deviations from the group mean) = (n K + S, SS - S^2 / n) over the row's 8 lanes
        const float fn = (float)rn, rinv = __builtin_amdgcn_rcpf(fn);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float S = sum8(ls[q]), SS = sum8(lss[q]);
          ls[q] = fmaf(fn, sK[q], S);
          lss[q] = fmaxf(SS - S * S * rinv, 0.f);
        }
        if ((lane & 7) == 0) {
          float2* st = a.stats + ((int64_t)c.p * a.ngrp + c.kc / GRP) * a.st_ld + a.st_off + 32 * w + erow;
          if (a.fcnt) {   // read back in this launch by the pair's last arriver (fin_pair): device-coherent stores
#pragma unroll
            for (int q = 0; q < 4; ++q)
              __hip_atomic_store(reinterpret_cast<unsigned long long*>(st + 8 * q),
                                 __builtin_bit_cast(unsigned long long, make_float2(ls[q], lss[q])), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) st[8 * q] = make_float2(ls[q], lss[q]);
          }
        }
      }
    }
  };

  // Software pipeline (chunk j of this workgroup's range; register set (j % 3)):
  //   step j: MFMAs of chunk j from image slot j & 1, with the split of chunk j + 1 (registers ->
  //   slot (j + 1) & 1) and the load of chunk j + 4 into the freed registers interleaved between
  //   the MFMA groups; epilogue of chunk j; residual DMA of chunk j + 1; fold of chunk j + 2's pair
  //   when it starts one; one barrier.
  // NSET register sets (3; 2 where the residual's registers or the k-split take the room): a chunk's loads
  // are issued NSET steps before its MFMAs
  constexpr int NSET = (RES || KW == 2) ? 2 : 3;
  float x0[NX], x1[NX], x2[NSET == 3 ? NX : 1];
  Cur cc = cstart, cs = cstart, ci = cstart, cf = cstart, cr = cstart;   // compute, split, issue, fold, residual
  stage_fold(cf.p);
  adv(cf);
  if (cf.p != cstart.p) stage_fold(cf.p);
  issue_x(ci, x0);
  adv(ci);
  issue_x(ci, x1);
  adv(ci);
  if constexpr (NSET == 3) {
    issue_x(ci, x2);
    adv(ci);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int t = 0; t < NT; ++t) split_half(cs, x0, 0, t);
  adv(cs);
  issue_x(ci, x0);
  adv(ci);
  load_r(cr);
  adv(cr);
  {
    const Cur prev = cf;
    adv(cf);
    if (cf.p != prev.p) stage_fold(cf.p);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // HEAD: wave 0 completes the logits of the chunk computed one step ago (its partials are published
  // by the step barrier): sum of the 4 waves' rows + bias, scores, positive count for the guard
  auto head_finish = [&](const Cur& c) {
    if (!HEAD || w != 0) return;
    const int col = c.kc * CH + l32;
    float lg = a.hb ? a.hb[0] : 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) lg += hpart[c.j & 1][ww][l32];
    const float sc = fmaxf(tanhf(lg), 0.f);
    const bool ok = lane < 32 && col < N;
    if (ok) {
      a.logits[(int64_t)c.p * N + col] = lg;
      a.scores[(int64_t)c.p * N + col] = sc;
    }
    const int np = __popcll(__ballot(ok && sc > 0.f));
    if (lane == 0 && np) atomicAdd(a.pos + c.p, np);
  };
  Cur ch = cstart;   // head cursor (one step behind compute)
  Cur cp = cstart;     // KW = 2: chunk whose epilogue is pending (lower half), one step behind
  floatx16 accp;       // ... and its lower-half accumulator
  auto step = [&](int j, auto& xs) {
    PCSTAMP(0);
    if (HEAD && j > 0) {
      head_finish(ch);
      adv(ch);
    }
    floatx16 acc = mfma(j & 1, [&](int ks) {
      if ((ks & 1) && ks < 2 * NT) split_half(cs, xs, (j + 1) & 1, ks >> 1);
      if (ks == 2 * NT) issue_x(ci, xs);
    });
    PCSTAMP(1);
    if constexpr (KW == 1) {
      epilogue(cc, acc);
    } else if (kh) {   // upper half: publish the partial sums (read by the lower half after the step barrier)
#pragma unroll
      for (int q = 0; q < 4; ++q) xch[j & 1][w][q][lane] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
    } else {
      if (j > 0) {   // the previous chunk: its upper-half partials were published by the last step barrier
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 u = xch[(j - 1) & 1][w][q][lane];
          accp[4 * q] += u.x; accp[4 * q + 1] += u.y; accp[4 * q + 2] += u.z; accp[4 * q + 3] += u.w;
        }
        epilogue(cp, accp);
        adv(cp);
      }
      accp = acc;
    }
    PCSTAMP(2);
    adv(cc);
    adv(cs);
    adv(ci);
    load_r(cr);
    adv(cr);
    const Cur prev = cf;
    adv(cf);
    if (cf.p != prev.p) stage_fold(cf.p);
    PCSTAMP(3);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  int j = 0;
  if constexpr (NSET == 3) {
    for (; j + 2 < nloc; j += 3) {
      step(j, x1);
      step(j + 1, x2);
      step(j + 2, x0);
    }
    if (j < nloc) step(j, x1);
    if (j + 1 < nloc) step(j + 1, x2);
  } else {
    for (; j + 1 < nloc; j += 2) {
      step(j, x1);
      step(j + 1, x0);
    }
    if (j < nloc) step(j, x1);
  }
  PCSTAMP(5);
  if (HEAD) head_finish(ch);   // the last chunk (published by the last step's barrier)
  if constexpr (KW == 2) {
    if (!kh) {   // the last chunk's epilogue (its upper-half partials: published by the last step barrier)
      const int jl = nloc - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 u = xch[jl & 1][w][q][lane];
        accp[4 * q] += u.x; accp[4 * q + 1] += u.y; accp[4 * q + 2] += u.z; accp[4 * q + 3] += u.w;
      }
      epilogue(cp, accp);
    }
  }
  if (H && __any(xbad || (xmx > 0.f && xmx < 0.125f)) && lane == 0) atomicExch(a.range, a.epoch);
#if PCONV_TRACE
  PCSTAMP(5);
  if (lane == 0 && KS == 8)
    for (int q_ = 0; q_ < 8; ++q_) atomicAdd(&g_pconv_trace[q_], ptr_[q_]);
#endif
  if constexpr (STATS && !H) {
    // Fused finalize (a.fcnt): publish this workgroup's statistics partials (every wave drains its stores, one
    // agent-scope release), add its tile count to each of its pairs' arrival counters; the workgroup completing
    // a pair acquires and merges that pair's partials (the in-launch reduction recipe of
    // cdna_hip_programming.md: correct for any spread of a pair's tiles over XCDs).  The arguments are re-read
    // here through an opaque kernarg pointer and the range recomputed, so none of it stays live (in SGPRs)
    // across the main loop.  Scratch: ys (free now).
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const PcArgs& A = *reinterpret_cast<const PcArgs*>(ka);
    if (A.fcnt) fin_tail(A, reinterpret_cast<int*>(&ys[0][0]), reinterpret_cast<double*>(&ys[1][0]), tid);
  }
}

}  // namespace

// Dispatched by launch_gemm for the shapes it covers; the caller has checked the common contract.
// N > CH: with one chunk per pair the fold of chunk j + 3's pair (staged at the end of step j) could
// land in the slot another wave still reads while splitting chunk j + 1 (pairs j + 1 and j + 3 then
// differ by 2, same parity); with >= 2 chunks per pair consecutive staged pairs always alternate.
#ifndef PCONV_OFF
#define PCONV_OFF 0   // diagnosis builds: route classes of convs to gemm_kernel (1 plain 128-channel, 8 the 256 ->
                      // 128 k-split, 16 head epilogue)
#endif

bool pconv_covers(const GemmArgs& g) {
  if ((PCONV_OFF & 16) && g.head_w) return false;
  if ((PCONV_OFF & 8) && g.K == 2 * PC) return false;
  if ((PCONV_OFF & 1) && !g.xin && !g.head_w && g.K == PC) return false;
  if (g.xin) {   // folded conv1: only the two shapes the OANet schedule uses
    const bool ok = !g_force[FORCE_GENERIC_GEMM] && g.math == MATH_BF16X3 && g.M == PC && g.K == PC && !g.bkc && g.sAb == 0 &&
                    g.pro == PRO_B_K && g.stats_mode == ST_ROW && !g.head_w && !g.no_store && g.bias_mode != BIAS_N &&
                    g.N > CH && g.xw && g.xci >= 1 && g.xci <= 8 && (g.xin != 2 || (g.xld % 4 == 0 && g.xld >= round4(g.N)));
    return ok && ((g.xin == 1 && !g.has_res) || (g.xin == 2 && g.has_res));
  }
  if (g.head_w && g.stats_mode != ST_NONE) return false;
  // statistics-only passes (the fused PointCN's conv3 pass): 128 -> 128 with the prologue, no residual
  if (g.no_store && !g.head_w && !(g.stats_mode == ST_ROW && !g.has_res && g.K == PC && g.pro == PRO_B_K)) return false;
  if (g.K == 2 * PC && (g.has_res || g.head_w)) return false;   // KS = 16 runs the 256 -> 128 convs only
  return !g_force[FORCE_GENERIC_GEMM] && g.math == MATH_BF16X3 && g.M == PC && (g.K == PC || g.K == 2 * PC) && !g.bkc && g.sAb == 0 &&
         (g.pro == PRO_NONE || g.pro == PRO_B_K) && (g.stats_mode == ST_NONE || g.stats_mode == ST_ROW) &&
         g.bias_mode != BIAS_N && g.N > CH;
}

int launch_pconv(const GemmArgs& g, hipStream_t s) {
  PcArgs a{};
  a.X = g.B; a.xps = g.sBb; a.xld = g.ldb; a.xcs = g.bcs ? g.bcs : CH;
  a.Y = g.C; a.yps = g.sCb; a.yld = g.ldc; a.ycs = g.ccs ? g.ccs : CH;
  a.R = g.R; a.rps = g.sRb; a.rrs = g.ldr ? g.ldr : g.ldc; a.rcs = g.rcs ? g.rcs : CH;
  a.W = g.A; a.wld = g.lda;
  a.bias = g.bias_mode == BIAS_M ? g.bias : nullptr;
  a.sc = g.psc; a.sh = g.psh; a.sPb = g.sPb;
  a.stats = g.stats; a.st_ld = g.st_ld; a.st_off = g.st_off;
  a.N = g.N;
  a.nch = (g.N + CH - 1) / CH;
  a.ngrp = (a.nch + GRP - 1) / GRP;
  a.groups = (int64_t)g.batch * a.ngrp;
  a.hw = g.head_w; a.hb = g.head_bp; a.logits = g.logits; a.scores = g.scores; a.pos = g.pos;
  a.xci = g.xci; a.xw = g.xw; a.xb = g.xb; a.rld = g.xld;
  const int ks = g.K / 16;
  // resident workgroups (2 / 1 per CU), one persistent round (PCONV_GRID > 1: that many contiguous group ranges per
  // slot; < 0: 1 / |PCONV_GRID| of the slots — both measured slower in the pipeline)
  const int64_t res_slots = (ks == 8 ? 2 : 1) * (int64_t)GPU_CUS;
  const int64_t slots = PCONV_GRID > 0 ? res_slots * PCONV_GRID : res_slots / -PCONV_GRID;
  const int grid = (int)(a.groups < slots ? a.groups : slots);
  const int pro = g.pro == PRO_B_K, res = g.has_res != 0, st = g.stats_mode == ST_ROW;
  const int head = g.head_w ? (g.no_store ? 2 : 1) : 0;
  if (head && (!g.logits || !g.scores || !g.pos)) return MVR_EINVAL;
  // split-fp16, then its guarded split-bf16 re-run — only with a caller-provided (zeroed) flag word, not for the
  // head launches (their positive counts are atomics) nor where the output overwrites the residual in place
  // (the re-run needs the residual intact).  Which arithmetic a launch takes depends on its arguments and
  // operand values only (no process state: no launch counters, no address-range tests).
  // (the same alias test as gemm.hip's launch_t: the re-run needs every input intact)
  const bool h1 = g_pconv_h && g.flag && !head && !(g.C == g.A || g.C == g.B || (g.has_res && g.R == g.C));
  if (h1) {
    a.range = g.flag;
    a.epoch = 1;
  }
  // the output's InstanceNorm fold in the last-arriving workgroup of each pair (split-bf16 launches only: the
  // split-fp16 pass and its guarded re-run would both arrive)
  if (g.fin_cnt && st && !h1 && !head) {
    if (!g.fin_train && (!g.fin_sc || !g.fin_sh)) return MVR_EINVAL;
    if (g.fin_train && !g.fin_mv) return MVR_EINVAL;
    a.fcnt = g.fin_cnt; a.feps = g.fin_eps; a.fbn = g.fin_bn; a.fsc = g.fin_sc; a.fsh = g.fin_sh; a.fld = g.fin_ld;
    a.feps2 = g.fin_eps2; a.fbn2 = g.fin_bn2; a.fsc2 = g.fin_sc2; a.fsh2 = g.fin_sh2;
    a.ftrain = g.fin_train; a.fmv = g.fin_mv;
    if (g.fin_done) *g.fin_done = 1;
  }
#define MVR_PCL(THREADS, ...)                                                   \
  do {                                                                          \
    if (h1) {                                                                   \
      hipLaunchKernelGGL((__VA_ARGS__, 1>), dim3(grid), dim3(THREADS), 0, s, a); \
      MVR_CHECK_LAUNCH();                                                       \
      a.guard = a.range;                                                        \
      a.range = nullptr;                                                        \
    }                                                                           \
    hipLaunchKernelGGL((__VA_ARGS__, 0>), dim3(grid), dim3(THREADS), 0, s, a);   \
    MVR_CHECK_LAUNCH();                                                         \
    return MVR_OK;                                                              \
  } while (0)
  if (g.xin == 1) MVR_PCL(256, pconv_kernel<8, 1, 0, 1, 0, 1, 1);   // folded conv1 -> conv3 of the block's first PointCN
  if (g.xin == 2) MVR_PCL(256, pconv_kernel<8, 1, 1, 1, 0, 2, 1);   // ... and its conv7 with the residual x recomputed
#define MVR_PC(K_, P_, R_, S_, H_) \
  if (ks == K_ && pro == P_ && res == R_ && st == S_ && head == H_) MVR_PCL(256, pconv_kernel<K_, P_, R_, S_, H_, 0, 1);
  MVR_PC(8, 1, 0, 1, 0)
  MVR_PC(8, 1, 1, 1, 0)
  MVR_PC(8, 1, 0, 0, 0)
  MVR_PC(8, 1, 1, 0, 0)
  MVR_PC(8, 0, 0, 1, 0)
  MVR_PC(8, 0, 1, 1, 0)
  MVR_PC(8, 0, 0, 0, 0)
  MVR_PC(8, 0, 1, 0, 0)
#undef MVR_PC
  // the last PointCN conv of a block with the output head (oanet.py:174-175), and the same when the block's
  // output activation is not returned (head only): split-bf16 only
  if (ks == 8 && pro == 1 && res == 1 && st == 0 && head == 1) {
    hipLaunchKernelGGL((pconv_kernel<8, 1, 1, 0, 1>), dim3(grid), dim3(256), 0, s, a);
    MVR_CHECK_LAUNCH();
    return MVR_OK;
  }
  if (ks == 8 && pro == 1 && res == 1 && st == 0 && head == 2) {
    hipLaunchKernelGGL((pconv_kernel<8, 1, 1, 0, 2>), dim3(grid), dim3(256), 0, s, a);
    MVR_CHECK_LAUNCH();
    return MVR_OK;
  }
  // 256 -> 128 (PointCN(2C -> C) after diff_unpool, oanet.py:155): the k-split 8-wave form, one workgroup per CU
#define MVR_PC16(P_, S_) \
  if (ks == 16 && pro == P_ && res == 0 && st == S_ && head == 0) MVR_PCL(512, pconv_kernel<16, P_, 0, S_, 0, 0, 2);
  MVR_PC16(1, 1)   // conv3 (IN/BN/ReLU prologue, statistics)
  MVR_PC16(0, 0)   // shortcut (raw input)
  MVR_PC16(1, 0)
  MVR_PC16(0, 1)
#undef MVR_PC16
#undef MVR_PCL
  return MVR_EINVAL;
}

}  // namespace mvr

#if PCONV_TRACE
// tools only (library built with -DPCONV_TRACE=1): the phase totals of every KS = 8 point-conv wave since the last reset
extern "C" int mvr_pconv_trace(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mvr::g_pconv_trace), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mvr::g_pconv_trace), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
