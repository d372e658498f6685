// Fused diff_pool / diff_unpool of the OANet block (lib/filtering/oanet.py:96-129) as flash-style
// attention on the split-bf16 matrix cores (mfma_bf16.hpp).
//
// diff_pool (oanet.py:96-110), per pair:   x_down[c][j] = sum_n x[c][n] softmax_n(e[j][n])
// diff_unpool (oanet.py:113-129), per pair: out[c][n]   = sum_j x_down[c][j] softmax_j(e[j][n])
// with e = W . relu(x * sc + sh) + b (the InstanceNorm + BatchNorm + ReLU of the embedding conv
// folded per (pair, channel) by in_finalize_kernel).  The reference materialises the [clusters x
// points] embedding and softmax (10 MB per pair, written and re-read twice per block); here it
// never leaves registers: each 512-thread workgroup owns 256 queries (8 waves x 32, one query per
// lane column, two waves per SIMD) and streams the keys through a double-buffered LDS ring shared
// by the 8 waves, with an online softmax (running max / sum per query, base 2).
//
//   pool:   queries j (clusters, W rows held split in registers), keys n (points, 32 per stage).
//           S^T[n][j] = xn^T . W^T  -> softmax over n is over the rows of a lane's column
//           O[c][j]  += x[c][n] . P[n][j]   (P taken from the S^T registers, no LDS trip)
//           The x tile of a stage is split on its way into LDS twice: normalised (K image, read
//           transposed with ds_read_b64_tr_b16) and raw (V image, n in the C-register k order).
//   unpool: queries n (points, xn split in registers), keys j (clusters, 32 per stage) from
//           images pre-split in HBM by split_w_kernel / split_xd_kernel and staged by LDS-DMA.
// Inside a stage the operand fragments are software-pipelined one MFMA group ahead
// (sched_barrier fences keep the compiler from sinking the reads to their uses).
//
// Channels are fixed at 128 (OANet net_channels, RegBlock.yaml).  Epilogue: the output tile goes
// through LDS for coalesced row stores and the per-(pair, channel, 128-column tile) (sum, squared
// deviations) partials that the next InstanceNorm needs (gemm.hpp ST_ROW).
//
// Roofline: 4 * C * clusters * points flops per pair on the split MFMA (6 bf16 MFMAs per fp32
// product: 16 * 157.3 / 6 = 419 TF/s fp32-equivalent); HBM traffic ~ x once + the output.
#include <algorithm>
#include <functional>
#include <vector>

#include "common.hpp"
#include "gemm.hpp"
#include "knobs.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"
#include "mvreg.h"

namespace mvr {

using namespace bx;

constexpr int AC = 128;                  // channels
constexpr int AKB = 32;                  // keys per stage
constexpr int AQ = 256;                  // queries per workgroup (8 waves x 32)
constexpr int ATHREADS = 512;
constexpr int ATL = AQ + 4;              // fp32 row stride of the epilogue tile in LDS
constexpr int PLANE = AC * AKB * 2;      // bytes of one bf16 plane of a stage image (8 KB)
constexpr int IMG = 3 * PLANE;           // h, m, l planes (24 KB)
constexpr int STAGE_B = 2 * IMG;         // one stage: two images (48 KB)
constexpr int MAX_CLUSTERS = 1024;
// unpool W image: [32 j][128 c] bf16 rows padded to 272 bytes (row r starts 17 r bank quads in, so
// the 16 rows of a ds_read_b128 lane group are conflict-free and a k-step is an immediate offset),
// image padded to 27 KB so that a stage (W image + x_down image) is a whole number of 1 KB DMAs
constexpr int WROW = 272;
constexpr int WPLANE = 32 * WROW;
constexpr int WIMG = 27 * 1024;
constexpr int USTAGE = WIMG + IMG;       // 51 KB
static_assert(3 * WPLANE <= WIMG, "W image padding");
constexpr float LOG2E = 1.4426950408889634f;
constexpr float A_NEG = -3.0e38f;
static_assert(64 * ATL * 4 <= 2 * STAGE_B, "epilogue half tile must fit the stage ring");

// ---------------------------------------------------------------------------------------------
// Operand math.  H = 0: split-bf16, three bf16 terms per fp32 operand, 6 MFMAs per product (mfma_bf16.hpp).
// H = 1: split-fp16, x = h + l with h = fp16(x), l = fp16(x - h) (RNE; x - h exact in fp32): 22 significant
// bits, |x - h - l| <= 2^-22 |x| for |x| >= 2^-3 and <= 2^-25 absolute below; the products hh, hl, lh on
// v_mfma_f32_32x32x16_f16 (3 MFMAs; the dropped ll <= 2^-22 relative).  The H = 1 kernels keep every
// operand where that holds, or hand the launch to H = 0:
//  * weight rows are scaled by a power of two to <= 2^14 (undone on the logits): relative 2^-22 per term;
//  * probabilities are formed as exp2(v - m + 7) <= 2^15 (the same factor is in the softmax sum);
//  * the logit side's activations (K / query operand) are checked against the fp16 range (< 65504); their
//    absolute floor (2^-25 per term below 2^-3) bounds the logit error by 2^-25 sum_c |W[j][c] log2 e|,
//    so a weight row with that sum > 128 (a floor above 2^-18 in log2 units) sends the launch to H = 0;
//  * the value side (V operand: pool's raw x, unpool's x_down) is checked per row (channel), whose
//    relative precision the next InstanceNorm exposes: a row with max |v| >= 65504 or in (0, 2^-3) too.
// A launch that trips a check sets its flag word and is re-run with H = 0 (guarded launches that return
// at once when the flag is clear), so results are within ~4x fp32 rounding of exact or are split-bf16's.
// ---------------------------------------------------------------------------------------------

__device__ int g_attn_reruns;           // guarded split-bf16 re-runs that ran (mvr_attn_reruns, diagnostics)
constexpr float F16_FLOOR = 0.125f;     // below: the low term is subnormal (absolute 2^-25)
constexpr float W_SUM_MAX = 128.f;      // max sum_c |W[j][c] log2 e| of a weight row (logit floor <= 2^-18)
// value-side row check: out of range, or nonzero and below the full-precision floor
__device__ __forceinline__ bool v_row_bad(float rmax) { return !(rmax < F16_RANGE) || (rmax > 0.f && rmax < F16_FLOOR); }

#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

#ifndef ATTN_TRACE
#define ATTN_TRACE 0   // 1: per-phase cycle totals per wave (s_memtime) of the pool / 4-wave unpool kernels, tools only
#endif
#if ATTN_TRACE
__device__ unsigned long long g_attn_trace[16];   // [0, 8) pool, [8, 16) unpool
#define ATSTAMP(slot)                                                  \
  do {                                                                 \
    unsigned long long t_;                                             \
    __builtin_amdgcn_sched_barrier(0);                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));  \
    __builtin_amdgcn_sched_barrier(0);                                 \
    tr_[prev_] += t_ - tlast_;                                         \
    tlast_ = t_;                                                       \
    prev_ = (slot);                                                    \
  } while (0)
#define ATSTART() unsigned long long tr_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast_ = __builtin_amdgcn_s_memtime(); int prev_ = 7
#define ATEND(base)                                                                  \
  do {                                                                               \
    ATSTAMP(7);                                                                      \
    if ((threadIdx.x & 63) == 0)                                                     \
      for (int q_ = 0; q_ < 8; ++q_) atomicAdd(&g_attn_trace[(base) + q_], tr_[q_]); \
  } while (0)
#else
#define ATSTAMP(slot) do {} while (0)
#define ATSTART() do {} while (0)
#define ATEND(base) do {} while (0)
#endif
// one MFMA, then a share of the VALU and LDS writes placed in the same scheduling region, six times
#define ATTN_INTERLEAVE6()                          \
  do {                                              \
    _Pragma("unroll") for (int u_ = 0; u_ < 6; ++u_) { \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); \
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0); \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0); \
    }                                               \
  } while (0)
// the same for the 3 MFMAs of a split-fp16 product (the split itself is shorter: ~2/3 of the VALU)
#define ATTN_INTERLEAVE3()                          \
  do {                                              \
    _Pragma("unroll") for (int u_ = 0; u_ < 3; ++u_) { \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); \
      __builtin_amdgcn_sched_group_barrier(0x002, 7, 0); \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0); \
    }                                               \
  } while (0)

// Byte offset of the 4 keys 4q .. 4q+3 (q = 0..7) of row `row` in a [row][32 keys] bf16 image
// whose 16-byte chunk (s, h) holds the 8 keys of k-step s, lane half h in the C-register k order
// (keys 16s + 4h + 0..3 and 16s + 8 + 4h + 0..3), chunk slot XOR-swizzled by (row >> 2) & 3 so
// that the 32 rows of an A-fragment read are conflict-free.
__device__ __forceinline__ int kord_off(int row, int q) {
  const int s = q >> 2, a = (q >> 1) & 1, h = q & 1;
  return row * 64 + 16 * ((2 * s + h) ^ ((row >> 2) & 3)) + 8 * a;
}
// A fragment (row = 32 cb + lane row, k-step s) of such an image
__device__ __forceinline__ Frag kord_frag(const char* img, int row, int s, int h) {
  const int off = row * 64 + 16 * ((2 * s + h) ^ ((row >> 2) & 3));
  Frag f;
  f.h = *reinterpret_cast<const bf16x8*>(img + off);
  f.m = *reinterpret_cast<const bf16x8*>(img + PLANE + off);
  f.l = *reinterpret_cast<const bf16x8*>(img + 2 * PLANE + off);
  return f;
}

template <int X>
__device__ __forceinline__ float swz_x(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (X << 10)));
}
__device__ __forceinline__ float half_sum(float v) {   // sum over the 32 lanes of a wave half
  v += swz_x<1>(v);
  v += swz_x<2>(v);
  v += swz_x<4>(v);
  v += swz_x<8>(v);
  v += swz_x<16>(v);
  return v;
}

// Workgroup -> (pair, block): the blocks of 8 consecutive pairs are interleaved so that all
// blocks of one pair are dealt to the same XCD (round-robin dispatch: b and b + 8 share one),
// where they share the pair's operands in L2.
__device__ __forceinline__ void pair_block(int nblk, int& p, int& blk) {
  const int b = blockIdx.x, x = b & 7, t = b >> 3;
  blk = t % nblk;
  p = (t / nblk) * 8 + x;
}

// Online softmax over the 16 rows of a lane column (+ the partner half): v holds logits * log2e.
// Lazy rescaling: the running max m moves only when a block exceeds it by more than RESCALE (log2
// units), so the probabilities exp2(v - m) stay <= 2^RESCALE and O, l are rescaled a few times per
// query instead of every block; O / l is the softmax-weighted sum whichever m was used.
// Leaves the probabilities in v, times 2^PSH (the sum l carries the same factor).
constexpr float RESCALE = 8.f;
template <int PSH = 0>
__device__ __forceinline__ void online_softmax(float (&v)[16], float& m, float& l, floatx16 (&O)[4]) {
  float bm = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), v[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) bm = __builtin_fmaxf(__builtin_fmaxf(bm, v[r]), v[r + 1]);
  bm = fmaxf(bm, v[15]);
  bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
  if (__any(bm > m + RESCALE)) {
    const float mn = fmaxf(m, bm);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) O[cb] *= alpha;
  }
  const float ms = m - (float)PSH;
  float ps = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r] = __builtin_amdgcn_exp2f(v[r] - ms);
    ps += v[r];
  }
  l += ps;
}

// column n of a row in the point activations' layout (oanet.hip): row-major (cs = 32: the row's element n) or
// chunk-major (rows 32 floats apart inside each 32-point chunk, chunks cs apart)
__device__ __forceinline__ int64_t cm_off(int n, int64_t cs) { return (int64_t)(n >> 5) * cs + (n & 31); }

// O (rows c = 32 cb + (q & 3) + 8 (q >> 2) + 4h, column = 32 w + lane row) * inv -> out[c][col0 + col]
// for columns < L (zeros in [L, round4(L))), and, per 128-column tile t of the 256 (tile index
// col0 / 128 + t), st[t * st_tile + c] = (sum, squared deviations) over the tile's valid columns.
// T: LDS scratch of 64 x ATL floats (two passes of 64 rows); the caller has synchronised.
__device__ __forceinline__ void tile_out(float* T, const floatx16 (&O)[4], float inv, bool colok, float* out,
                                         int64_t ld, int64_t cs, int col0, int L, float2* st, int64_t st_tile) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int col = 32 * w + l32;
  const int Lp = (L + 3) & ~3;
  const int nv = min(max(L - col0 - 128 * h, 0), 128);   // valid columns of this lane half's tile
  const float rnv = nv > 0 ? 1.f / (float)nv : 0.f;
  bool ok[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ok[u] = 4 * l32 + u < nv;
  const bool sok = col0 + 4 * lane < Lp;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = 32 * cc + (q & 3) + 8 * (q >> 2) + 4 * h;
        T[c * ATL + col] = colok ? O[2 * hf + cc][q] * inv : 0.f;
      }
    __syncthreads();
    for (int it = 0; it < 8; ++it) {
      const int cl = 8 * w + it, c = 64 * hf + cl;
      float4 x = *reinterpret_cast<const float4*>(T + cl * ATL + 4 * lane);
      if (!ok[0]) x.x = 0.f;
      if (!ok[1]) x.y = 0.f;
      if (!ok[2]) x.z = 0.f;
      if (!ok[3]) x.w = 0.f;
      if (st) {
        const float sm = half_sum((x.x + x.y) + (x.z + x.w));
        const float mu = sm * rnv;
        const float d0 = ok[0] ? x.x - mu : 0.f, d1 = ok[1] ? x.y - mu : 0.f, d2 = ok[2] ? x.z - mu : 0.f,
                    d3 = ok[3] ? x.w - mu : 0.f;
        const float m2 = half_sum((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
        if (l32 == 0 && nv > 0) st[h * st_tile + c] = make_float2(sm, m2);
      }
      if (sok) *reinterpret_cast<float4*>(out + (int64_t)c * ld + cm_off(col0 + 4 * lane, cs)) = x;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// diff_pool
// ---------------------------------------------------------------------------------------------
struct PoolArgs {
  const float* X; int64_t xps, xld, xcs;           // x [P][128][xld] (raw; xcs: chunk stride, cm_off)
  const float* sc; const float* sh; int64_t sps;   // folded IN+BN: xn = relu(x * sc[c] + sh[c])
  const float* W; const float* bias;               // embedding conv [Kc][128], [Kc]
  int P, N, Kc, nqb;                               // nqb = ceil(Kc / 256) query blocks
  float* out; int64_t ops, old;                    // x_down [P][128][old]
  float2* stats; int64_t st_ld; int st_off;        // [P][ceil(Kc/128)][st_ld] (+ st_off + c), nullable
  int nks;                                         // key splits per (pair, query block) of the split tail; 1: none
  int g0;                                          // nks > 1: pair octets [0, g0) unsplit, the rest split (the tail)
  float* part; int* cnt;                           // nks > 1: per-split (O, m, l) slabs, arrival tickets
  int* range;                                      // H = 1: set when an operand is outside the fp16 range
  const int* guard;                                // H = 0 re-run: return unless *guard is set
};

constexpr int PSLAB = 66 * ATHREADS;               // floats of one split's slab: O (64 / thread), m, l

__device__ __forceinline__ void glds16b(const char* src, char* lds_base) {
  const uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_base;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}

// (glds16s: the same from a wave-uniform base + 32-bit lane offset, common.hpp)

constexpr int XT = AC * AKB * 4;   // raw fp32 key tile [128 c][32 n] (16 KB)
constexpr int PRAW = 3;            // raw key tiles in the LDS-DMA ring: a tile's DMA has two stages to land
template <int H> constexpr int pool_smem() {
  return 4 * planes<H>() * PLANE > 64 * ATL * 4 ? 4 * planes<H>() * PLANE : 64 * ATL * 4;
}

template <int H>
__global__ __launch_bounds__(ATHREADS) void oan_pool_kernel(PoolArgs a) {
  constexpr int NP = planes<H>();
  constexpr int IMGT = NP * PLANE;         // one stage image (K or V)
  constexpr int STAGET = 2 * IMGT;         // one stage: K image, V image
  __shared__ __attribute__((aligned(16))) char smem[pool_smem<H>()];   // stage ring; epilogue tile
  __shared__ __attribute__((aligned(16))) char xraw[PRAW * XT];        // LDS-DMA ring of raw key tiles
  __shared__ float2 ssh[AC];                                          // (sc, sh) of this pair
  if (a.guard) {
    if (*a.guard == 0) return;   // uniform: the fp16 launch before this one stayed in range
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_attn_reruns, 1);
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  int p, jb, ks = 0, nks = 1;
  const int nb0 = 8 * a.nqb * a.g0;   // blocks of the unsplit pair octets (nks > 1)
  if (a.nks > 1 && (int)blockIdx.x >= nb0) {
    // the split tail: the splits of one (pair, query block) are blocks b, b + 8, ..: one XCD, adjacent
    const int b = blockIdx.x - nb0, x = b & 7;
    int t = b >> 3;
    nks = a.nks;
    ks = t % nks;
    t /= nks;
    jb = t % a.nqb;
    p = (a.g0 + t / a.nqb) * 8 + x;
  } else {
    pair_block(a.nqb, p, jb);
  }
  if (p >= a.P) return;   // uniform over the workgroup
  ATSTART();   // pool phases: 0 prologue, 1 S MFMAs (+ V split), 2 softmax + P split, 3 O MFMAs (+ K split),
               // 4 stage-end wait + barrier, 5 split merge, 6 epilogue
  ATSTAMP(0);
  const float* X = a.X + (int64_t)p * a.xps;
  const int N = a.N;
  const int nkb = (N + AKB - 1) / AKB;
  const int kb0 = nkb * ks / nks, kb1 = nkb * (ks + 1) / nks;   // this split's key blocks
  const int nlast = ((N + 3) & ~3) - 4;   // last readable 4-key group of a row

  // raw tile kb -> xraw[kb & 1] as [c][32] fp32 rows: wave w moves rows 16 w .. 16 w + 15 in two
  // 1 KB DMAs (lane: row + lane / 8, keys 4 (lane & 7)); keys past the end read a clamped column
  // and are zeroed when the tile is split
  // (uniform pair base + 32-bit lane offsets: 64-bit per-lane pointers held across the key loop spilled to scratch,
  // and each reload's vmcnt(0) also waited for the tile DMA just issued)
  const uint32_t xraw_lds = lds_addr(xraw);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t xld4 = (uint32_t)a.xld * 4u;
  auto dma_tile = [&](int kb) {
    const int n = min(kb * AKB + 4 * (lane & 7), nlast);
    const uint32_t dst = xraw_lds + (uint32_t)((kb % PRAW) * XT);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = 16 * wu + 8 * i;
      glds16s(X, (uint32_t)(r0 + (lane >> 3)) * xld4 + 4u * (uint32_t)cm_off(n, a.xcs), dst + (uint32_t)(r0 * 128));
    }
  };
  dma_tile(kb0);
  if (tid < AC) ssh[tid] = make_float2(a.sc[(int64_t)p * a.sps + tid], a.sh[(int64_t)p * a.sps + tid]);

  // queries: this lane's W row (column j of S^T) as split B fragments, one per 16-channel k-step
  // (H = 1: the row scaled to <= 2^14, the scale undone on the logits)
  const int j = jb * AQ + 32 * w + l32;
  const bool jok = j < a.Kc;
  const float* wr = a.W + (int64_t)min(j, a.Kc - 1) * AC + 8 * h;
  FragT<H> q[8];
  float wsc = 1.f;
  bool wbad = false;
  {
    float v[8][8];
    float amax = 0.f, asum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const float4 u0 = *reinterpret_cast<const float4*>(wr + 16 * ks);
      const float4 u1 = *reinterpret_cast<const float4*>(wr + 16 * ks + 4);
      const float t[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[ks][i] = jok ? t[i] * LOG2E : 0.f;   // logits in log2 units
        amax = fmaxf(amax, fabsf(v[ks][i]));
        asum += fabsf(v[ks][i]);
      }
    }
    if (H) {
      wbad = asum + __shfl_xor(asum, 32, 64) > W_SUM_MAX;
      wsc = range_scale(fmaxf(amax, __shfl_xor(amax, 32, 64)));
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[ks][i] *= wsc;
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) q[ks] = split8t<H>(v[ks]);
  }
  const float wisc = 1.f / wsc;   // exact: a power of two
  const float bj = ((jok && a.bias) ? a.bias[j] * LOG2E : 0.f) * wsc;
  float kmax = 0.f;               // H = 1: max xn split so far (K operand range check)
  float vmax[2] = {0.f, 0.f};     // H = 1: max |x| of this thread's two channel rows so far (V operand)

  const int sq = tid & 7;
  // the split of raw tile kb + 1 in four parts placed between the MFMAs of a stage (the 8 waves run
  // their stages in step, so a split phase of its own leaves the matrix pipes idle): load_x reads a
  // thread's two raw key groups (thread -> channel c = tid / 8 + 64 i, keys 4 (tid & 7) .. +3),
  // store_v / store_k write one of them to the V / K image of stage st
  auto load_x = [&](int kb, int i) {
    const int c = (tid >> 3) + 64 * i;
    float4 x = *reinterpret_cast<const float4*>(xraw + (kb % PRAW) * XT + c * 128 + 16 * sq);
    if (kb * AKB + 4 * sq >= N) x = make_float4(0.f, 0.f, 0.f, 0.f);
    return x;
  };
  auto store_v = [&](int st, int i, float4 x) {
    asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w));   // keep the split at its placement
    char* V = smem + st * STAGET + IMGT;
    const int c = (tid >> 3) + 64 * i;
    u32x2 o[3];
    split4t<H>(x, o);
    const int vo = kord_off(c, sq);
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<u32x2*>(V + pl * PLANE + vo) = o[pl];
    if (H) vmax[i] = fmaxf(fmaxf(vmax[i], fmaxf(fabsf(x.x), fabsf(x.y))), fmaxf(fabsf(x.z), fabsf(x.w)));
  };
  auto store_k = [&](int st, int i, float4 x, const float2& f) {
    asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w));
    char* K = smem + st * STAGET;
    const int c = (tid >> 3) + 64 * i;
    const float4 xn = make_float4(fmaxf(fmaf(x.x, f.x, f.y), 0.f), fmaxf(fmaf(x.y, f.x, f.y), 0.f),
                                  fmaxf(fmaf(x.z, f.x, f.y), 0.f), fmaxf(fmaf(x.w, f.x, f.y), 0.f));
    u32x2 o[3];
    split4t<H>(xn, o);
    const int ko = c * 64 + 8 * sq;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<u32x2*>(K + pl * PLANE + ko) = o[pl];
    if (H) kmax = fmaxf(fmaxf(kmax, fmaxf(xn.x, xn.y)), fmaxf(xn.z, xn.w));
  };

  floatx16 O[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[cb][r] = 0.f;
  float m = A_NEG, l = 0.f;

  // transposed-read address of the K image: row c0 + (lane & 15) / 4, keys 16 (g & 1) + 4 (lane & 3)
  const int g = lane >> 4;
  const int tr_off = ((lane & 15) >> 2) * 64 + 32 * (g & 1) + 8 * (lane & 3);
  auto read_k = [&](const char* K, int ks) {
    const int o0 = (16 * ks + 8 * h) * 64 + tr_off, o1 = o0 + 4 * 64;
    FragT<H> f;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      const u32x2 t0 = ds_read_tr(K + pl * PLANE + o0), t1 = ds_read_tr(K + pl * PLANE + o1);
      f.p[pl] = __builtin_bit_cast(typename FragT<H>::V, u32x4{t0[0], t0[1], t1[0], t1[1]});
    }
    return f;
  };
  // A fragment (row = 32 cb + lane row, k-step s) of a V image
  auto v_frag = [&](const char* V, int row, int s) {
    return ld_frag<H>(V + row * 64 + 16 * ((2 * s + h) ^ ((row >> 2) & 3)), PLANE);
  };

  // ring: raw tile kb + 3 lands while stage kb & 1 is consumed and tile kb + 1 is split into the other (two DMA
  // instructions per lane and tile, nothing else in flight: vmcnt(2) = all but the youngest tile)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  dma_tile(kb0 + 1);
  dma_tile(kb0 + 2);
  {
    const float4 x0 = load_x(kb0, 0), x1 = load_x(kb0, 1);
    store_v(kb0 & 1, 0, x0);
    store_k(kb0 & 1, 0, x0, ssh[tid >> 3]);
    store_v(kb0 & 1, 1, x1);
    store_k(kb0 & 1, 1, x1, ssh[(tid >> 3) + 64]);
  }
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // tile kb0 + 1 landed, kb0 + 2 in flight
  __syncthreads();
  for (int kb = kb0; kb < kb1; ++kb) {
    ATSTAMP(1);
    const int st = kb & 1;
    // tile kb + 1 (zeros past the end) -> stage st ^ 1, split between the MFMAs below
    const float4 x0 = load_x(kb + 1, 0);
    float4 x1;
    dma_tile(kb + 3);             // into the buffer of tile kb, split one iteration ago
    const char* K = smem + st * STAGET;
    const char* V = K + IMGT;
    // S^T[n][j] = b[j] + sum_c xn[c][n] W[j][c] (log2 units; H = 1: times wsc), fragments one k-step ahead
    floatx16 S;
    float bjl = bj;
    asm volatile("" : "+v"(bjl));   // a per-stage splat: hoisted, the 16-register splat of bj stayed live (spills)
#pragma unroll
    for (int r = 0; r < 16; ++r) S[r] = bjl;
    FragT<H> cur = read_k(K, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      FragT<H> nxt;
      if (ks < 7) nxt = read_k(K, ks + 1);
      SCHED_FENCE();
      if (ks == 2) store_v(st ^ 1, 0, x0);
      if (ks == 5) store_k(st ^ 1, 0, x0, ssh[tid >> 3]);
      if (ks == 6) x1 = load_x(kb + 1, 1);
      S = mma<H>(cur, q[ks], S);
      if (ks == 2 || ks == 5) {
        if (H) ATTN_INTERLEAVE3(); else ATTN_INTERLEAVE6();
      }
      SCHED_FENCE();
      if (ks < 7) cur = nxt;
    }
    ATSTAMP(2);
    FragT<H> vf = v_frag(V, l32, 0);   // first V fragment, in flight during the softmax
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = H ? S[r] * wisc : S[r];
    if (kb * AKB + AKB > N) {   // ragged last block
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb * AKB + (r & 3) + 8 * (r >> 2) + 4 * h >= N) v[r] = -__builtin_inff();
    }
    online_softmax<H ? 7 : 0>(v, m, l, O);
    FragT<H> pf[2] = {split8t<H>(v), split8t<H>(v + 8)};
    ATSTAMP(3);
    // O[c][j] += sum_n x[c][n] P[n][j]
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int s = i >> 2, cb = i & 3;
      FragT<H> nxt;
      if (i < 7) nxt = v_frag(V, 32 * ((i + 1) & 3) + l32, (i + 1) >> 2);
      SCHED_FENCE();
      if (i == 2) store_v(st ^ 1, 1, x1);
      if (i == 5) store_k(st ^ 1, 1, x1, ssh[(tid >> 3) + 64]);
      O[cb] = mma<H>(vf, pf[s], O[cb]);
      if (i == 2 || i == 5) {
        if (H) ATTN_INTERLEAVE3(); else ATTN_INTERLEAVE6();
      }
      SCHED_FENCE();
      if (i < 7) vf = nxt;
    }
    ATSTAMP(4);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // tile kb + 2 landed, kb + 3 in flight
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // no tile DMA outlives the loop
  ATSTAMP(5);
  if (H) {
    // rows: the 8 threads of a channel (tid & 7) saw all of this split's keys of it
    bool bad = wbad || !(kmax < F16_RANGE);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float r = vmax[i];
      r = fmaxf(r, __shfl_xor(r, 1, 64));
      r = fmaxf(r, __shfl_xor(r, 2, 64));
      r = fmaxf(r, __shfl_xor(r, 4, 64));
      bad |= v_row_bad(r);
    }
    if (__any(bad) && lane == 0) atomicOr(a.range, 1);
  }
  if (nks > 1) {
    // publish this split's (O, m, l); the last split to arrive merges all of them (counter hand-off:
    // device-coherent stores, each lane's complete before the ticket, device-coherent loads by the reducer — no
    // agent-scope fences, whose L2 write-back / invalidation cost every workgroup on the XCD its cached lines)
    const int64_t slot = (int64_t)p * a.nqb + jb;
    float* mine = a.part + (slot * nks + ks) * PSLAB + tid;
    auto st_c = [](float* q, float v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) st_c(mine + (16 * cb + r) * ATHREADS, O[cb][r]);
    st_c(mine + 64 * ATHREADS, m);
    st_c(mine + 65 * ATHREADS, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(xraw);   // the raw-tile ring is drained
    if (tid == 0) {
      const int tk = __hip_atomic_fetch_add(a.cnt + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // tickets are not reset between the fp16 launch and its guarded re-run: the last split of a slot
      // draws nks - 1 modulo nks
      flag[0] = tk % nks == nks - 1;
    }
    __syncthreads();
    if (!flag[0]) {   // uniform
      ATEND(0);
      return;
    }
    // merge the splits in split order (whichever arrived last: the result does not depend on arrival order)
    const floatx16 own[4] = {O[0], O[1], O[2], O[3]};
    const float mown = m, lown = l;
    auto ld_c = [](const float* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int o = 0; o < nks; ++o) {
      const float* th = a.part + (slot * nks + o) * PSLAB + tid;
      const float m2 = o == ks ? mown : ld_c(th + 64 * ATHREADS), l2 = o == ks ? lown : ld_c(th + 65 * ATHREADS);
      if (o == 0) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int r = 0; r < 16; ++r) O[cb][r] = o == ks ? own[cb][r] : ld_c(th + (16 * cb + r) * ATHREADS);
        m = m2;
        l = l2;
        continue;
      }
      const float mn = fmaxf(m, m2);
      const float f1 = __builtin_amdgcn_exp2f(m - mn), f2 = __builtin_amdgcn_exp2f(m2 - mn);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          O[cb][r] = O[cb][r] * f1 + (o == ks ? own[cb][r] : ld_c(th + (16 * cb + r) * ATHREADS)) * f2;
      l = l * f1 + l2 * f2;
      m = mn;
    }
  }
  ATSTAMP(6);
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  const int ntile = (a.Kc + 127) / 128;
  tile_out(reinterpret_cast<float*>(smem), O, inv, jok, a.out + (int64_t)p * a.ops, a.old, 32, jb * AQ, a.Kc,
           a.stats ? a.stats + ((int64_t)p * ntile + 2 * jb) * a.st_ld + a.st_off : nullptr, a.st_ld);
  ATEND(0);
}

// ---------------------------------------------------------------------------------------------
// diff_unpool
// ---------------------------------------------------------------------------------------------
// W [Kc][128] -> image [nkb][planes][32 j][WROW bytes] (wimg_stride<H> bytes per block); rows j >= Kc zero.
// A row is 16 adjacent threads (8 channels each).  bs[j] = (b[j] log2e, 1) with H = 0; with H = 1 the row is
// scaled by s = range_scale(max |row|) and bs[j] = (b[j] log2e s, 1 / s); rows j >= Kc: (-inf, 1).
template <int H> constexpr int wimg_stride() { return H ? 17 * 1024 : WIMG; }
template <int H> constexpr int ximg_bytes() { return planes<H>() * PLANE; }
static_assert(2 * WPLANE <= 17 * 1024, "fp16 W image block");

template <int H>
__global__ void split_w_kernel(const float* __restrict__ W, const float* __restrict__ bias, int Kc, int nkb, char* img,
                               float2* bs, int* range, const int* guard) {
  if (guard && *guard == 0) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // nkb * 512 threads: a multiple of 16
  if (i >= nkb * 512) return;
  const int ch = i & 15, jj = (i >> 4) & 31, kb = i >> 9;
  const int j = kb * AKB + jj;
  float v[8];
  float amax = 0.f, asum = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = j < Kc ? W[(int64_t)j * AC + 8 * ch + e] * LOG2E : 0.f;   // log2 units
    amax = fmaxf(amax, fabsf(v[e]));
    asum += fabsf(v[e]);
  }
  float s = 1.f;
  if (H) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      amax = fmaxf(amax, __shfl_xor(amax, o, 64));
      asum += __shfl_xor(asum, o, 64);
    }
    if (__any(asum > W_SUM_MAX) && (threadIdx.x & 63) == 0) atomicOr(range, 1);
    s = range_scale(amax);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= s;
  }
  const FragT<H> f = split8t<H>(v);
  char* base = img + (int64_t)kb * wimg_stride<H>() + jj * WROW + 16 * ch;
#pragma unroll
  for (int pl = 0; pl < planes<H>(); ++pl) *reinterpret_cast<typename FragT<H>::V*>(base + pl * WPLANE) = f.p[pl];
  if (ch == 0)
    bs[j] = j < Kc ? make_float2((bias ? bias[j] * LOG2E : 0.f) * s, 1.f / s) : make_float2(-__builtin_inff(), 1.f);
}

// x_down [P][128][ld] (Kc valid columns) -> split-bf16 image [P][nkb][3 planes][128 c][32 j] (kord_off order)
__global__ void split_xd_kernel(const float* __restrict__ XD, int64_t ps, int64_t ld, int P, int Kc, int nkb,
                                char* img, const int* guard) {
  if (guard && *guard == 0) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)P * nkb * 1024) return;
  const int q = (int)(i & 7), c = (int)((i >> 3) & 127);
  const int64_t pk = i >> 10;   // p * nkb + kb
  const int kb = (int)(pk % nkb);
  const int64_t p = pk / nkb;
  const int j0 = kb * AKB + 4 * q;
  const float* src = XD + p * ps + (int64_t)c * ld;
  const float4 x = make_float4(j0 < Kc ? src[j0] : 0.f, j0 + 1 < Kc ? src[j0 + 1] : 0.f,
                               j0 + 2 < Kc ? src[j0 + 2] : 0.f, j0 + 3 < Kc ? src[j0 + 3] : 0.f);
  u32x2 o[3];
  split4t<0>(x, o);
  char* base = img + pk * ximg_bytes<0>() + kord_off(c, q);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x2*>(base + pl * PLANE) = o[pl];
}

// the split-fp16 image [P][nkb][2 planes][128 c][32 j], one wave per row (p, c) of x_down (Kc <= 512: lane l
// holds clusters 8 l .. 8 l + 7), with the value-side row check
__global__ void split_xd16_kernel(const float* __restrict__ XD, int64_t ps, int64_t ld, int P, int Kc, int nkb,
                                  char* img, int* range) {
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;   // p * 128 + c
  const int lane = threadIdx.x & 63;
  if (row >= (int64_t)P * AC) return;   // whole waves
  const int c = (int)(row & 127);
  const int64_t p = row >> 7;
  const float* src = XD + p * ps + (int64_t)c * ld;
  float v[8];
  float rmax = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int j = 8 * lane + e;
    v[e] = j < Kc ? src[j] : 0.f;
    rmax = fmaxf(rmax, fabsf(v[e]));
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, o, 64));
  if (lane == 0 && v_row_bad(rmax)) atomicOr(range, 1);
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int j0 = 8 * lane + 4 * g, kb = j0 >> 5, q = (j0 & 31) >> 2;
    if (kb >= nkb) break;
    u32x2 o[3];
    split4t<1>(make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]), o);
    char* base = img + (p * nkb + kb) * ximg_bytes<1>() + kord_off(c, q);
    *reinterpret_cast<u32x2*>(base) = o[0];
    *reinterpret_cast<u32x2*>(base + PLANE) = o[1];
  }
}

struct UnpoolArgs {
  const float* X; int64_t xps, xld, xcs;           // x_up [P][128][xld] (raw; xcs: chunk stride, cm_off)
  const float* sc; const float* sh; int64_t sps;   // folded IN+BN of the embedding input
  const char* wimg;                                // split_w_kernel image [nkb][wimg_stride]
  const float* bias;                               // [Kc], nullable (the 8-wave kernel)
  const float2* bs;                                // split_w_kernel (bias, 1 / row scale) [nkb * 32]
  const char* dimg;                                // split_xd_kernel image [P][nkb][ximg_bytes]
  int P, N, Kc, nkb, nqb;                          // nqb = ceil(N / queries per workgroup)
  float* out; int64_t ops, old, ocs;               // [P][128][old] (ocs: chunk stride, cm_off)
  float2* stats; int64_t st_ld; int st_off;        // [P][ceil(N/128)][st_ld] (+ st_off + c), nullable
  int* range;                                      // H = 1: set when an operand is outside the fp16 range
  const int* guard;                                // H = 0 re-run: return unless *guard is set
};


__global__ __launch_bounds__(ATHREADS) void oan_unpool_kernel(UnpoolArgs a) {
  // stage ring; the query prologue double-buffers 32 KB quarters at [USTAGE, USTAGE + 64 KB)
  __shared__ __attribute__((aligned(16))) char smem[USTAGE + 64 * 1024];
  __shared__ __attribute__((aligned(16))) float bsh[MAX_CLUSTERS];
  __shared__ float2 ssh[AC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  int p, nb;
  pair_block(a.nqb, p, nb);
  if (p >= a.P) return;
  const int N = a.N, nkb = a.nkb;
  const char* dimg = a.dimg + (int64_t)p * nkb * IMG;

  // a 51 KB stage (W image block, then x_down image block) as 1 KB LDS-DMAs dealt over the 8 waves
  auto issue = [&](int kb, int st) {
    char* dst = smem + st * USTAGE;
    for (int off = w * 1024; off < USTAGE; off += 8 * 1024) {
      const char* src = off < WIMG ? a.wimg + (int64_t)kb * WIMG + off : dimg + (int64_t)kb * IMG + (off - WIMG);
      glds16b(src + 16 * lane, dst + off);
    }
  };
  issue(0, 0);

  for (int i = tid; i < nkb * AKB; i += ATHREADS)
    bsh[i] = i < a.Kc ? (a.bias ? a.bias[i] * LOG2E : 0.f) : -__builtin_inff();
  if (tid < AC) ssh[tid] = make_float2(a.sc[(int64_t)p * a.sps + tid], a.sh[(int64_t)p * a.sps + tid]);

  // queries: this lane's point n (column), xn[c][n] for c = 16 ks + 8h + i as split B fragments.
  // The workgroup's x_up rows (128 channels x 256 points) are staged through LDS in quarters of 32
  // channels (whole 1 KB row segments by LDS-DMA, double-buffered behind stage 0) and read back as
  // columns; points past the end read a clamped column and are zeroed.
  const int n = nb * AQ + 32 * w + l32;
  const bool nok = n < N;
  const int nlast = ((N + 3) & ~3) - 4;
  const float* xb = a.X + (int64_t)p * a.xps + cm_off(min(nb * AQ + 4 * lane, nlast), a.xcs);
  auto qdma = [&](int qt) {
    char* dst = smem + USTAGE + (qt & 1) * 32768;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * w + i;
      glds16b(reinterpret_cast<const char*>(xb + (int64_t)(32 * qt + r) * a.xld), dst + r * 1024);
    }
  };
  qdma(0);
  Frag q[8];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    if (qt < 3) {
      qdma(qt + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // all but quarter qt + 1 landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const float* xt = reinterpret_cast<const float*>(smem + USTAGE + (qt & 1) * 32768) + 32 * w + l32;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ks = 2 * qt + kk;
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 16 * ks + 8 * h + i;
        const float2 f = ssh[c];
        const float x = fmaxf(fmaf(xt[(c - 32 * qt) * 256], f.x, f.y), 0.f);
        v[i] = nok ? x : 0.f;
      }
      split8(v, q[ks].h, q[ks].m, q[ks].l);
    }
    __syncthreads();
  }

  floatx16 O[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[cb][r] = 0.f;
  float m = A_NEG, l = 0.f;

  const int wbase = l32 * WROW + 16 * h;
  auto read_w = [&](const char* Wi, int ks) {
    const int off = wbase + 32 * ks;
    Frag f;
    f.h = *reinterpret_cast<const bf16x8*>(Wi + off);
    f.m = *reinterpret_cast<const bf16x8*>(Wi + WPLANE + off);
    f.l = *reinterpret_cast<const bf16x8*>(Wi + 2 * WPLANE + off);
    return f;
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const int st = kb & 1;
    if (kb + 1 < nkb) issue(kb + 1, st ^ 1);
    const char* Wi = smem + st * USTAGE;
    const char* D = Wi + WIMG;
    // S[j][n] = b[j] + sum_c W[j][c] xn[c][n] (log2 units; -inf rows past the clusters), fragments
    // one k-step ahead
    floatx16 S;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const float4 b = *reinterpret_cast<const float4*>(bsh + kb * AKB + 8 * r4 + 4 * h);
      S[4 * r4 + 0] = b.x;
      S[4 * r4 + 1] = b.y;
      S[4 * r4 + 2] = b.z;
      S[4 * r4 + 3] = b.w;
    }
    Frag cur = read_w(Wi, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      Frag nxt;
      if (ks < 7) nxt = read_w(Wi, ks + 1);
      SCHED_FENCE();
      S = mfma6(cur, q[ks], S);
      SCHED_FENCE();
      if (ks < 7) cur = nxt;
    }
    Frag df = kord_frag(D, l32, 0, h);
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = S[r];
    online_softmax(v, m, l, O);
    Frag pf[2];
    split8(v, pf[0].h, pf[0].m, pf[0].l);
    split8(v + 8, pf[1].h, pf[1].m, pf[1].l);
    // O[c][n] += sum_j x_down[c][j] P[j][n]
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int s = i >> 2, cb = i & 3;
      Frag nxt;
      if (i < 7) nxt = kord_frag(D, 32 * ((i + 1) & 3) + l32, (i + 1) >> 2, h);
      SCHED_FENCE();
      O[cb] = mfma6(df, pf[s], O[cb]);
      SCHED_FENCE();
      if (i < 7) df = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  const int ntile = (N + 127) / 128;
  tile_out(reinterpret_cast<float*>(smem), O, inv, nok, a.out + (int64_t)p * a.ops, a.old, a.ocs, nb * AQ, N,
           a.stats ? a.stats + ((int64_t)p * ntile + 2 * nb) * a.st_ld + a.st_off : nullptr, a.st_ld);
}

// ---------------------------------------------------------------------------------------------
// diff_unpool, 4-wave form: 128 queries per 256-thread workgroup, two workgroups per CU.  The 8-wave
// kernel above owns a CU alone, so its per-workgroup prologue (x_up columns in) and epilogue (output
// and statistics out) leave the matrix pipes idle; here the two co-resident workgroups drift out of
// phase and cover each other's prologue, epilogue and LDS-DMA waits.  LDS (76.8 KB + 2.5 KB): the W
// image double-buffered (26112 B each, unpadded) and one x_down image (24 KB): W(kb+1) lands during
// stage kb, x_down(kb+1) during the S MFMAs of stage kb+1.  Requires clusters <= 512.
// ---------------------------------------------------------------------------------------------
constexpr int U4T = 256;                 // threads
constexpr int U4Q = 128;                 // queries per workgroup
constexpr int U4QB = 32 * U4Q * 4;       // a prologue quarter: 32 channels x 128 points fp32 (16 KB)
constexpr int U4TL = U4Q + 4;            // fp32 row stride of the epilogue tile
template <int H> constexpr int u4_wimg() { return planes<H>() * WPLANE; }   // W image block as it lands in LDS
template <int H> constexpr int u4_lds() { return 2 * u4_wimg<H>() + ximg_bytes<H>(); }   // 76800 / 51200 B
static_assert(u4_wimg<0>() + 2 * U4QB <= u4_lds<0>() && u4_wimg<1>() + 2 * U4QB <= u4_lds<1>(),
              "prologue quarters (at the second W buffer) fit");
static_assert(64 * U4TL * 4 <= u4_lds<1>(), "epilogue half tile fits");

template <int H>
__global__ __launch_bounds__(U4T, 2) void oan_unpool4_kernel(UnpoolArgs a) {
  constexpr int WI4 = u4_wimg<H>();
  constexpr int XDO = 2 * WI4;             // x_down image offset
  constexpr int XIMG = ximg_bytes<H>();
  constexpr int WSTR = wimg_stride<H>();
  __shared__ __attribute__((aligned(16))) char smem[u4_lds<H>()];
  __shared__ __attribute__((aligned(16))) float bsh[512];
  __shared__ __attribute__((aligned(16))) float ish[H ? 512 : 4];
  __shared__ float2 ssh[AC];
  if (a.guard) {
    if (*a.guard == 0) return;   // uniform: the fp16 launch before this one stayed in range
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_attn_reruns, 1);
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  int p, nb;
  pair_block(a.nqb, p, nb);
  if (p >= a.P) return;   // uniform over the workgroup
  ATSTART();   // unpool phases: 0 prologue, 1 S MFMAs, 2 softmax + split, 3 x_down wait + barrier, 4 O MFMAs,
               // 5 barrier + DMA issue, 6 epilogue
  ATSTAMP(0);
  const int N = a.N, nkb = a.nkb;
  const char* dimg = a.dimg + (int64_t)p * nkb * XIMG;

  // W image block kb -> smem + (kb & 1) WI4 (1 KB DMAs dealt over the 4 waves; the last may be partial);
  // x_down image block kb -> smem + XDO
  // (uniform bases + 32-bit lane offsets, fixed trip counts: the per-stage DMA issue stays a few scalar ops)
  const uint32_t smem_lds = lds_addr(smem);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto issue_w = [&](int kb) {
    const uint32_t dst = smem_lds + (uint32_t)((kb & 1) * WI4);
    const char* src = a.wimg + (int64_t)kb * WSTR;
#pragma unroll
    for (int i = 0; i < (WI4 + 4095) / 4096; ++i) {
      const int off = wu * 1024 + 4096 * i;
      if (off < WI4 && off + 16 * lane < WI4) glds16s(src, (uint32_t)(off + 16 * lane), dst + (uint32_t)off);
    }
  };
  auto issue_xd = [&](int kb) {
    const char* src = dimg + (int64_t)kb * XIMG;
#pragma unroll
    for (int i = 0; i < (XIMG + 4095) / 4096; ++i) {
      const int off = wu * 1024 + 4096 * i;
      if (off < XIMG) glds16s(src, (uint32_t)(off + 16 * lane), smem_lds + (uint32_t)(XDO + off));
    }
  };
  issue_w(0);

  for (int i = tid; i < nkb * AKB; i += U4T) {
    const float2 b = a.bs[i];
    bsh[i] = b.x;
    if (H) ish[i] = b.y;
  }
  if (tid < AC) ssh[tid] = make_float2(a.sc[(int64_t)p * a.sps + tid], a.sh[(int64_t)p * a.sps + tid]);

  // queries: this lane's point n = nb 128 + 32 w + l32; xn[c][n] for c = 16 ks + 8h + i as split B
  // fragments.  The 128 x 128 x_up block comes through LDS in quarters of 32 channels (a DMA moves two
  // 512-byte row segments: lane -> row 2i + h, points 4 l32 .. +3), double-buffered at [WI4, WI4 +
  // 32 KB); points past the end read a clamped column and are zeroed.
  const int n = nb * U4Q + 32 * w + l32;
  const bool nok = n < N;
  const int nlast = ((N + 3) & ~3) - 4;
  const float* xb = a.X + (int64_t)p * a.xps + cm_off(min(nb * U4Q + 4 * l32, nlast), a.xcs);
  auto qdma = [&](int qt) {
    char* dst = smem + WI4 + (qt & 1) * U4QB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r2 = 4 * w + i;   // row pair (2 r2, 2 r2 + 1) of the quarter
      glds16b(reinterpret_cast<const char*>(xb + (int64_t)(32 * qt + 2 * r2 + h) * a.xld), dst + r2 * 1024);
    }
  };
  qdma(0);
  FragT<H> q[8];
  float xmax = 0.f;
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    if (qt < 3) {   // (the W(0) DMAs are older: waited with quarter 0)
      qdma(qt + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // all but quarter qt + 1 landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const float* xt = reinterpret_cast<const float*>(smem + WI4 + (qt & 1) * U4QB) + 32 * w + l32;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ks = 2 * qt + kk;
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 16 * ks + 8 * h + i;
        const float2 f = ssh[c];
        const float x = fmaxf(fmaf(xt[(c - 32 * qt) * U4Q], f.x, f.y), 0.f);
        v[i] = nok ? x : 0.f;
        if (H) xmax = fmaxf(xmax, v[i]);
      }
      q[ks] = split8t<H>(v);
    }
    __syncthreads();
  }
  if (H && __any(!(xmax < F16_RANGE)) && lane == 0) atomicOr(a.range, 1);
  issue_xd(0);

  floatx16 O[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[cb][r] = 0.f;
  float m = A_NEG, l = 0.f;

  const int wbase = l32 * WROW + 16 * h;
  auto read_w = [&](const char* Wi, int ks) { return ld_frag<H>(Wi + wbase + 32 * ks, WPLANE); };
  auto d_frag = [&](const char* D, int row, int s) {
    return ld_frag<H>(D + row * 64 + 16 * ((2 * s + h) ^ ((row >> 2) & 3)), PLANE);
  };

  // stage kb: W(kb) landed (waited before the barrier that ended stage kb - 1 / the prologue);
  // x_down(kb) in flight
  for (int kb = 0; kb < nkb; ++kb) {
    ATSTAMP(1);
    if (kb + 1 < nkb) issue_w(kb + 1);   // the other W buffer: last read by stage kb - 1
    const char* Wi = smem + (kb & 1) * WI4;
    const char* D = smem + XDO;
    // S[j][n] = b[j] + sum_c W[j][c] xn[c][n] (log2 units, H = 1: row j times its scale; -inf rows past
    // the clusters)
    floatx16 S;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const float4 b = *reinterpret_cast<const float4*>(bsh + kb * AKB + 8 * r4 + 4 * h);
      S[4 * r4 + 0] = b.x;
      S[4 * r4 + 1] = b.y;
      S[4 * r4 + 2] = b.z;
      S[4 * r4 + 3] = b.w;
    }
    FragT<H> cur = read_w(Wi, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      FragT<H> nxt;
      if (ks < 7) nxt = read_w(Wi, ks + 1);
      SCHED_FENCE();
      S = mma<H>(cur, q[ks], S);
      SCHED_FENCE();
      if (ks < 7) cur = nxt;
    }
    ATSTAMP(2);
    float v[16];
    if (H) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 is = *reinterpret_cast<const float4*>(ish + kb * AKB + 8 * r4 + 4 * h);
        v[4 * r4 + 0] = S[4 * r4 + 0] * is.x;
        v[4 * r4 + 1] = S[4 * r4 + 1] * is.y;
        v[4 * r4 + 2] = S[4 * r4 + 2] * is.z;
        v[4 * r4 + 3] = S[4 * r4 + 3] * is.w;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = S[r];
    }
    online_softmax<H ? 7 : 0>(v, m, l, O);
    FragT<H> pf[2] = {split8t<H>(v), split8t<H>(v + 8)};
    ATSTAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // x_down(kb) (and W(kb + 1))
    __syncthreads();
    ATSTAMP(4);
    FragT<H> df = d_frag(D, l32, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int s = i >> 2, cb = i & 3;
      FragT<H> nxt;
      if (i < 7) nxt = d_frag(D, 32 * ((i + 1) & 3) + l32, (i + 1) >> 2);
      SCHED_FENCE();
      O[cb] = mma<H>(df, pf[s], O[cb]);
      SCHED_FENCE();
      if (i < 7) df = nxt;
    }
    ATSTAMP(5);
    __syncthreads();   // every wave is done with x_down(kb) and W(kb)
    if (kb + 1 < nkb) issue_xd(kb + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATSTAMP(6);

  // epilogue: O (rows c = 32 cb + (q & 3) + 8 (q >> 2) + 4h, column 32 w + l32) / l -> out[c][nb 128 + col]
  // through an LDS tile in two passes of 64 rows; a wave stores two rows per step (lane half h: row
  // 2 it + h, columns 4 l32 .. +3) and forms the rows' (sum, squared deviations) over the tile's valid
  // columns (the workgroup's 128 columns are one statistics tile)
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  float* T = reinterpret_cast<float*>(smem);
  const int col0 = nb * U4Q;
  const int nv = min(max(N - col0, 0), U4Q);
  const float rnv = nv > 0 ? 1.f / (float)nv : 0.f;
  bool ok[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ok[u] = 4 * l32 + u < nv;
  const int Lp = (N + 3) & ~3;
  const bool sok = col0 + 4 * l32 < Lp;
  float* out = a.out + (int64_t)p * a.ops;
  float2* st = a.stats ? a.stats + ((int64_t)p * ((N + 127) / 128) + nb) * a.st_ld + a.st_off : nullptr;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) {
        const int c = 32 * cc + (q2 & 3) + 8 * (q2 >> 2) + 4 * h;
        T[c * U4TL + 32 * w + l32] = nok ? O[2 * hf + cc][q2] * inv : 0.f;
      }
    __syncthreads();
    for (int it = 0; it < 8; ++it) {
      const int cl = 16 * w + 2 * it + h, c = 64 * hf + cl;
      float4 x = *reinterpret_cast<const float4*>(T + cl * U4TL + 4 * l32);
      if (!ok[0]) x.x = 0.f;
      if (!ok[1]) x.y = 0.f;
      if (!ok[2]) x.z = 0.f;
      if (!ok[3]) x.w = 0.f;
      if (st) {
        const float sm = half_sum((x.x + x.y) + (x.z + x.w));
        const float mu = sm * rnv;
        const float d0 = ok[0] ? x.x - mu : 0.f, d1 = ok[1] ? x.y - mu : 0.f, d2 = ok[2] ? x.z - mu : 0.f,
                    d3 = ok[3] ? x.w - mu : 0.f;
        const float m2 = half_sum((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
        if (l32 == 0 && nv > 0) st[c] = make_float2(sm, m2);
      }
      if (sok) *reinterpret_cast<float4*>(out + (int64_t)c * a.old + cm_off(col0 + 4 * l32, a.ocs)) = x;
    }
    __syncthreads();
  }
  ATEND(8);
}

#ifndef ATTN_MATH_DEFAULT
#define ATTN_MATH_DEFAULT 0
#endif
int g_attn_h = ATTN_MATH_DEFAULT;  // mvr_set_math: split-fp16 (1) or split-bf16 (0) pool / 4-wave unpool

}  // namespace mvr

using namespace mvr;

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static int64_t round_up4(int64_t x) { return (x + 3) & ~(int64_t)3; }

#if ATTN_TRACE
extern "C" int mvr_attn_trace(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mvr::g_attn_trace), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mvr::g_attn_trace), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

extern "C" size_t mvr_oan_diff_unpool_workspace_bytes(int P, int channels, int clusters) {
  if (P <= 0 || channels != AC || clusters <= 0 || clusters > MAX_CLUSTERS) return 0;
  const size_t nkb = (size_t)(clusters + AKB - 1) / AKB;
  return nkb * (WIMG + (size_t)P * IMG + AKB * sizeof(float2)) + 512;   // W image, x_down images, bs, flag
}

// Key splits of the pool launch: with one 512-thread workgroup per CU, P x ceil(Kc / 256) workgroups
// leave a partial last round (435 pairs: 880 workgroups = 3.44 rounds of 256).  Splitting the keys (points) of
// a (pair, query block) into k parts shortens the rounds, but every split unit writes an (O, m, l) slab that the
// last one reads back (135 KB each), and the split changes a unit's summation order.
//  * default: every unit in 2 parts at N >= 16 key blocks (3.5 rounds instead of 4 at 435 pairs), a function of N
//    alone, so a pair's result does not depend on the batch it came in (pair-sharded runs over any number of ranks
//    give the one-process records bit for bit at the default f32eq maths, tests/test_gpu_distributed.py; under
//    split16 a guarded launch re-runs in split-bf16 when ANY of its pairs leaves the fp16 window, so there the
//    precision a pair gets depends on which pairs share its launch);
//  * POOL_TAIL builds (round 4, not kept): only a TAIL is split: the pair octets [0, g0) run whole, the rest in k parts,
//    dispatched after them.  Candidates (k in {1, 2, 4} with >= 8 key blocks per part; g0 = every octet, no octet,
//    or the most octets whose whole units fill complete rounds) are ranked by the makespan of the dispatch order
//    on `cus` slots (a unit = 1, a part = 1 / k), ties to fewer slabs: fewer slabs (224 instead of 1760 at 435
//    pairs), but the split of a pair then depends on the batch size and the device's CU count.
struct PoolSplit { int nks, g0; };
#ifndef POOL_TAIL
#define POOL_TAIL 0
#endif
static double pool_makespan(int64_t full, int64_t parts, int k, int cus) {
  // greedy in dispatch order: the whole units first, then the parts, each to the earliest free slot
  std::vector<double> slot((size_t)cus, 0.0);
  std::make_heap(slot.begin(), slot.end(), std::greater<double>());
  auto put = [&](double d) {
    std::pop_heap(slot.begin(), slot.end(), std::greater<double>());
    slot.back() += d;
    std::push_heap(slot.begin(), slot.end(), std::greater<double>());
  };
  for (int64_t i = 0; i < full; ++i) put(1.0);
  for (int64_t i = 0; i < parts; ++i) put(1.0 / k);
  return *std::max_element(slot.begin(), slot.end());
}
static PoolSplit pool_splits(int P, int nqb, int N) {
  const int nkb = (N + AKB - 1) / AKB;
  if (!POOL_TAIL) return nkb >= 16 ? PoolSplit{2, 0} : PoolSplit{1, (P + 7) / 8};
  int dev = 0, cus = 0;   // the current device's CU count (an attribute query, no process state)
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int G = (P + 7) / 8;                 // pair octets
  const int64_t per = 8LL * nqb;             // workgroups of one octet, unsplit
  PoolSplit best{1, G};
  double tbest = pool_makespan(per * G, 0, 1, cus);
  int64_t slabs_best = 0;
  for (int k = 2; k <= 4; k *= 2) {
    if (nkb < 8 * k) break;
    const int gfill = (int)(((per * G) / cus) * cus / per);   // most whole octets in complete rounds
    const int cands[3] = {0, gfill, G};
    for (int g0 : cands) {
      if (g0 >= G) continue;
      const int64_t parts = per * k * (G - g0);
      const double t = pool_makespan(per * g0, parts, k, cus);
      if (t < tbest - 1e-9 || (t < tbest + 1e-9 && parts < slabs_best)) {
        tbest = t;
        best = PoolSplit{k, g0};
        slabs_best = parts;
      }
    }
  }
  return best;
}

// pool workspace: [nks > 1: per-split slabs, slot tickets] [range flag]
static size_t pool_ws_bytes(int P, int clusters, int nks) {
  const size_t slots = (size_t)P * ((clusters + AQ - 1) / AQ);
  return (nks > 1 ? slots * ((size_t)nks * PSLAB * 4 + 4) : 0) + 512;
}


extern "C" size_t mvr_oan_diff_pool_workspace_bytes(int P, int channels, int clusters) {
  if (P <= 0 || channels != AC || clusters <= 0 || clusters > MAX_CLUSTERS) return 0;
  return pool_ws_bytes(P, clusters, 4);
}

extern "C" int mvr_oan_diff_pool_ws(const float* x, int64_t x_pstride, int64_t x_ld, const float* sc,
                                    const float* sh, int64_t s_pstride, const float* weight, const float* bias, int P,
                                    int channels, int N, int clusters, float* out, int64_t out_pstride, int64_t out_ld,
                                    float* stats, int64_t st_ld, int st_off, void* workspace, size_t workspace_bytes,
                                    hipStream_t stream);

extern "C" int mvr_oan_diff_pool(const float* x, int64_t x_pstride, int64_t x_ld, const float* sc, const float* sh,
                                 int64_t s_pstride, const float* weight, const float* bias, int P, int channels, int N,
                                 int clusters, float* out, int64_t out_pstride, int64_t out_ld, float* stats,
                                 int64_t st_ld, int st_off, hipStream_t stream) {
  return mvr_oan_diff_pool_ws(x, x_pstride, x_ld, sc, sh, s_pstride, weight, bias, P, channels, N, clusters, out,
                              out_pstride, out_ld, stats, st_ld, st_off, nullptr, 0, stream);
}

extern "C" int mvr_oan_diff_pool_ws(const float* x, int64_t x_pstride, int64_t x_ld, const float* sc,
                                    const float* sh, int64_t s_pstride, const float* weight, const float* bias, int P,
                                    int channels, int N, int clusters, float* out, int64_t out_pstride, int64_t out_ld,
                                    float* stats, int64_t st_ld, int st_off, void* workspace, size_t workspace_bytes,
                                    hipStream_t stream) {
  return mvr::oan_diff_pool_cm(x, x_pstride, x_ld, 32, sc, sh, s_pstride, weight, bias, P, channels, N, clusters, out,
                               out_pstride, out_ld, stats, st_ld, st_off, workspace, workspace_bytes, stream);
}

// x row-major (x_cs = 32) or chunk-major (x_ld = 32, chunks x_cs >= 32 x 128 floats apart: oanet.hip's point
// activations)
int mvr::oan_diff_pool_cm(const float* x, int64_t x_pstride, int64_t x_ld, int64_t x_cs, const float* sc,
                          const float* sh, int64_t s_pstride, const float* weight, const float* bias, int P,
                          int channels, int N, int clusters, float* out, int64_t out_pstride, int64_t out_ld,
                          float* stats, int64_t st_ld, int st_off, void* workspace, size_t workspace_bytes,
                          hipStream_t stream) {
  if (P < 0 || N <= 0 || channels != AC || clusters <= 0 || clusters > MAX_CLUSTERS) return MVR_EINVAL;
  if (P == 0) return MVR_OK;   // no pairs: NULL pointers allowed
  if (!x || !sc || !sh || !weight || !out) return MVR_EINVAL;
  const bool xcm = x_cs != 32;
  if ((xcm ? (x_ld != 32 || (x_cs & 3) || x_cs < 32 * AC) : x_ld < round_up4(N)) || (x_ld & 3) || (x_pstride & 3) ||
      !al16(x) || !al16(weight) || !al16(out) || out_ld < round_up4(clusters) || (out_ld & 3) || (out_pstride & 3) ||
      (stats && (st_ld < channels + st_off)))
    return MVR_EINVAL;
  // 32-bit lane offsets of the tile DMAs
  if ((xcm ? (int64_t)((N + 31) / 32) * x_cs : (int64_t)AC * x_ld) * 4 >= ((int64_t)1 << 31)) return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  PoolArgs a{};
  a.X = x; a.xps = x_pstride; a.xld = x_ld; a.xcs = x_cs;
  a.sc = sc; a.sh = sh; a.sps = s_pstride;
  a.W = weight; a.bias = bias;
  a.P = P; a.N = N; a.Kc = clusters; a.nqb = (clusters + AQ - 1) / AQ;
  a.out = out; a.ops = out_pstride; a.old = out_ld;
  a.stats = reinterpret_cast<float2*>(stats); a.st_ld = st_ld; a.st_off = st_off;
  a.nks = 1;
  const size_t slots = (size_t)P * a.nqb;
  int* range = nullptr;   // split-fp16 needs the workspace's flag word
  // with a workspace the key-split count is a function of the shape alone (pool_splits); a workspace smaller than
  // mvr_oan_diff_pool_workspace_bytes is an error rather than a silently different split (and summation order)
  if (workspace) {
    if (!al16(workspace) || workspace_bytes < pool_ws_bytes(P, clusters, 4)) return MVR_EINVAL;
    const PoolSplit ps = pool_splits(P, a.nqb, N);
    const int k = ps.nks;
    if (k > 1) {
      a.nks = k;
      a.g0 = ps.g0;
      a.part = reinterpret_cast<float*>(workspace);
      a.cnt = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + slots * (size_t)k * PSLAB * 4);
    }
    if (g_attn_h)
      range = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                     (a.nks > 1 ? slots * ((size_t)a.nks * PSLAB * 4 + 4) : 0));
  }
  // the tickets and the flag word are adjacent: one memset
  if (a.nks > 1 || range) {
    void* z = a.nks > 1 ? (void*)a.cnt : (void*)range;
    const size_t zb = (a.nks > 1 ? slots * sizeof(int) : 0) + (range ? sizeof(int) : 0);
    if (hipMemsetAsync(z, 0, zb, stream) != hipSuccess) return MVR_ELAUNCH;
  }
  const double fl = 4.0 * AC * clusters * (double)N * P;
  const double by = 4.0 * AC * ((double)N + clusters) * P;
  ProfScope prof(PK_POOL, fl, by, stream);
  const int G = (P + 7) / 8;
  const int grid = a.nks > 1 ? 8 * a.nqb * (a.g0 + a.nks * (G - a.g0)) : G * 8 * a.nqb;
  if (range) {   // split-fp16, then the split-bf16 re-run that returns at once unless an operand was out of range
    a.range = range;
    hipLaunchKernelGGL(oan_pool_kernel<1>, dim3(grid), dim3(ATHREADS), 0, stream, a);
    MVR_CHECK_LAUNCH();
    a.range = nullptr;
    a.guard = range;
  }
  hipLaunchKernelGGL(oan_pool_kernel<0>, dim3(grid), dim3(ATHREADS), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_oan_diff_unpool(const float* x_up, int64_t x_pstride, int64_t x_ld, const float* sc,
                                   const float* sh, int64_t s_pstride, const float* weight, const float* bias,
                                   const float* x_down, int64_t xd_pstride, int64_t xd_ld, int P, int channels,
                                   int N, int clusters, float* out, int64_t out_pstride, int64_t out_ld, float* stats,
                                   int64_t st_ld, int st_off, void* workspace, size_t workspace_bytes,
                                   hipStream_t stream) {
  return mvr::oan_diff_unpool_cm(x_up, x_pstride, x_ld, 32, sc, sh, s_pstride, weight, bias, x_down, xd_pstride,
                                 xd_ld, P, channels, N, clusters, out, out_pstride, out_ld, 32, stats, st_ld, st_off,
                                 workspace, workspace_bytes, stream);
}

// x_up and out row-major (cs = 32) or chunk-major (ld = 32, chunks cs >= 32 x 128 floats apart)
int mvr::oan_diff_unpool_cm(const float* x_up, int64_t x_pstride, int64_t x_ld, int64_t x_cs, const float* sc,
                            const float* sh, int64_t s_pstride, const float* weight, const float* bias,
                            const float* x_down, int64_t xd_pstride, int64_t xd_ld, int P, int channels, int N,
                            int clusters, float* out, int64_t out_pstride, int64_t out_ld, int64_t out_cs,
                            float* stats, int64_t st_ld, int st_off, void* workspace, size_t workspace_bytes,
                            hipStream_t stream) {
  if (P < 0 || N <= 0 || channels != AC || clusters <= 0 || clusters > MAX_CLUSTERS) return MVR_EINVAL;
  if (P == 0) return MVR_OK;   // no pairs: NULL pointers allowed
  if (!x_up || !sc || !sh || !weight || !x_down || !out || !workspace) return MVR_EINVAL;
  auto bad_layout = [&](int64_t ld, int64_t cs) {
    return cs != 32 ? (ld != 32 || (cs & 3) || cs < 32 * AC) : ld < round_up4(N);
  };
  if (bad_layout(x_ld, x_cs) || (x_ld & 3) || (x_pstride & 3) || xd_ld < clusters || bad_layout(out_ld, out_cs) ||
      (out_ld & 3) || (out_pstride & 3) || !al16(out) || !al16(workspace) || (stats && (st_ld < channels + st_off)))
    return MVR_EINVAL;
  if (P == 0) return MVR_OK;
  if (workspace_bytes < mvr_oan_diff_unpool_workspace_bytes(P, channels, clusters)) return MVR_EINVAL;
  const int nkb = (clusters + AKB - 1) / AKB;
  char* wimg = reinterpret_cast<char*>(workspace);
  char* dimg = wimg + (size_t)nkb * WIMG;
  float2* bs = reinterpret_cast<float2*>(dimg + (size_t)P * nkb * IMG);
  int* range = reinterpret_cast<int*>(bs + (size_t)nkb * AKB);
  const double fl = 4.0 * AC * clusters * (double)N * P;
  const double by = 4.0 * AC * (2.0 * N + clusters) * P;
  ProfScope prof(PK_UNPOOL, fl, by, stream);
  UnpoolArgs a{};
  a.X = x_up; a.xps = x_pstride; a.xld = x_ld; a.xcs = x_cs;
  a.sc = sc; a.sh = sh; a.sps = s_pstride;
  a.wimg = wimg; a.bias = bias; a.bs = bs; a.dimg = dimg;
  a.P = P; a.N = N; a.Kc = clusters; a.nkb = nkb; a.nqb = (N + AQ - 1) / AQ;
  a.out = out; a.ops = out_pstride; a.old = out_ld; a.ocs = out_cs;
  a.stats = reinterpret_cast<float2*>(stats); a.st_ld = st_ld; a.st_off = st_off;
  const int64_t nx = (int64_t)P * nkb * 1024;
  const dim3 gw((nkb * 512 + 255) / 256), gx((unsigned)((nx + 255) / 256));
  if (!g_force[FORCE_UNPOOL8] && clusters <= 512) {
    a.nqb = (N + U4Q - 1) / U4Q;
    const int grid = ((P + 7) / 8) * 8 * a.nqb;
    const int* guard = nullptr;
    if (g_attn_h) {   // split-fp16, then the split-bf16 re-run that returns at once unless an operand was out of range
      if (hipMemsetAsync(range, 0, sizeof(int), stream) != hipSuccess) return MVR_ELAUNCH;
      hipLaunchKernelGGL(split_w_kernel<1>, gw, dim3(256), 0, stream, weight, bias, clusters, nkb, wimg, bs, range,
                         nullptr);
      MVR_CHECK_LAUNCH();
      hipLaunchKernelGGL(split_xd16_kernel, dim3((unsigned)(((int64_t)P * AC * 64 + 255) / 256)), dim3(256), 0, stream,
                         x_down, xd_pstride, xd_ld, P, clusters, nkb, dimg, range);
      MVR_CHECK_LAUNCH();
      a.range = range;
      hipLaunchKernelGGL(oan_unpool4_kernel<1>, dim3(grid), dim3(U4T), 0, stream, a);
      MVR_CHECK_LAUNCH();
      a.range = nullptr;
      a.guard = guard = range;
    }
    hipLaunchKernelGGL(split_w_kernel<0>, gw, dim3(256), 0, stream, weight, bias, clusters, nkb, wimg, bs, nullptr,
                       guard);
    MVR_CHECK_LAUNCH();
    hipLaunchKernelGGL(split_xd_kernel, gx, dim3(256), 0, stream, x_down, xd_pstride, xd_ld, P, clusters, nkb, dimg,
                       guard);
    MVR_CHECK_LAUNCH();
    hipLaunchKernelGGL(oan_unpool4_kernel<0>, dim3(grid), dim3(U4T), 0, stream, a);
  } else {
    hipLaunchKernelGGL(split_w_kernel<0>, gw, dim3(256), 0, stream, weight, bias, clusters, nkb, wimg, bs, nullptr,
                       nullptr);
    MVR_CHECK_LAUNCH();
    hipLaunchKernelGGL(split_xd_kernel, gx, dim3(256), 0, stream, x_down, xd_pstride, xd_ld, P, clusters, nkb, dimg,
                       nullptr);
    MVR_CHECK_LAUNCH();
    const int grid = ((P + 7) / 8) * 8 * a.nqb;
    hipLaunchKernelGGL(oan_unpool_kernel, dim3(grid), dim3(ATHREADS), 0, stream, a);
  }
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_attn_reruns(int reset) {
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_attn_reruns), sizeof(int)) != hipSuccess)
    return -1;
  if (reset) {
    const int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_attn_reruns), &z, sizeof(int)) != hipSuccess) return -1;
  }
  return v;
}

