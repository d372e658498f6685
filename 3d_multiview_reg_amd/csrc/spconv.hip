// Sparse 3-D convolution (MinkowskiConvolution / MinkowskiConvolutionTranspose forward,
// used throughout lib/descriptor/fcgf.py:118-227) as an output-stationary gather-GEMM:
//
//   out[o][c] = epi( sum_k sum_ci in[nbr[o][k]][ci] * W[k][ci][c] )
//   epi = (+bias) -> BatchNorm (eval: running stats) -> (+residual) -> (ReLU)
//
// nbr is the kernel map as a neighbour table (csrc/sparse.hip); -1 entries contribute
// nothing.  Output rows are visited in the order `perm` (mvr_kernel_map_order: rows sorted by
// their active-offset mask, then spatially), so a tile's rows share their active offsets and the union the tile
// iterates stays small (a transposed stride-2 conv has <= 8 of 27 per row, by coordinate parity).  Per 128-row
// output tile the workgroup first lists the stencil offsets that have at least one neighbour in the tile and
// skips the empty ones; each step gathers 32 input channels of the tile's neighbour rows straight into registers
// and multiplies them with the pre-split weights on the bf16 MFMAs (below).  No atomics: every output row is
// owned by exactly one workgroup (deterministic results).

#include "common.hpp"
#include "knobs.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"
#include "sparse.hpp"

namespace mvr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct SpArgs {
  const float* in; int64_t ldin; int Cin;
  const int32_t* nbr; int K; int64_t Mout;
  const int32_t* perm;   // optional output row order (tile t covers rows perm[64t .. 64t+63])
  const float* W; int Cout;
  const float* bias;
  mvr_bn_p bn; float bn_eps;
  const float* res; int64_t ldres;
  int relu;
  float* out; int64_t ldout;
  int* range; const int* guard; int epoch;   // split-fp16 flag word (set to epoch 1) / split-bf16 re-run guard
  const uint16_t* inp;   // optional: the input as split-bf16 planes, row r plane p at inp + (3 r + p) ldin (bf16)
  uint16_t* outp;        // optional: the output's planes too, row r plane p at outp + (3 r + p) ldout
};

constexpr int SP_KMAX = 32;
__device__ __attribute__((aligned(16))) float g_sp_zero[4];   // what an absent neighbour gathers


#ifndef SP_TRACE
#define SP_TRACE 0   // 1: spconv_bx per-phase cycle totals per wave (s_memtime), tools only (mvr_spconv_trace)
#endif
#if SP_TRACE
__device__ unsigned long long g_sp_trace[8];
#define SPSTAMP(slot)                                                  \
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
#define SPSTAMP(slot) do {} while (0)
#endif

// ---------------------------------------------------------------------------------------------
// The gather-GEMM on v_mfma_f32_32x32x16_bf16 with both operands as three bf16 terms (fp32-level accuracy, see
// mfma_bf16.hpp) — 2.7x the fp32 MFMA rate.
// 128 output rows per workgroup, one 32-row slab per wave over all TN output channels (NJ = TN / 32
// accumulator tiles), so a wave's gathered rows are its own A operand: each lane gathers its row's 8
// channels of each k-step straight into registers (three steps in flight), splits them itself — no LDS
// for A, no duplicated gathers.  A step is 32 input channels of one active stencil offset.  The weights
// come pre-split (mvr_spconv_wimage: [k][32-channel block][plane][Cout][32 + 8 pad] bf16, 80-byte rows)
// and reach LDS through registers one step ahead (shared by the 4 waves).  All loads are compiler-tracked:
// the gathers of step s + 3 stay in flight while step s + 1's weights are awaited.
constexpr int SB_K = 32;     // input channels per step
constexpr int SB_BST = 40;   // bf16 row stride of the weight image (80 B)
constexpr int SB_CP = 128;   // output-channel padding of the weight image (largest TN)
#ifndef SPBX_WBUF
#define SPBX_WBUF 1   // the weight-stage loads through a buffer resource (wave-uniform base) with 32-bit lane offsets
                      // (0: 64-bit per-lane addresses; spconv<128,3,0,0> then held 256 VGPRs with 4 spilled:
                      // bit-identical, the FCGF convs -2 %, profiles/r06/ab_r6s24_spconv_wbuf.txt)
#endif
#ifndef SPBX_NS32   // gathered steps in flight per output-channel tile width (register budget)
#define SPBX_NS32 3
#endif
#ifndef SPBX_NS64
#define SPBX_NS64 3
#endif
#ifndef SPBX_NS128
#define SPBX_NS128 3
#endif
// the same for the pre-split gathers (PS = 1: 24 VGPRs per set of gathered planes instead of 16 of fp32)
#ifndef SPBX_PS_NS32
#define SPBX_PS_NS32 3
#endif
#ifndef SPBX_PS_NS64
#define SPBX_PS_NS64 3
#endif
#ifndef SPBX_PS_NS128
#define SPBX_PS_NS128 2
#endif

// H = 1: split-fp16 (mfma_bf16.hpp, 3 MFMAs per product): the image's fp16 section (each output channel's
// weights scaled by a power of two to <= 2^14), the gathered features x XS = 2^6 as they are split, both undone
// per column in the epilogue (isc); a lane that splits a value of 1023.5 or more, or whose values are all below
// 2^-9 without being zero, marks the launch (the caller's flag word) for its guarded split-bf16 re-run.
// PS = 1 (H = 0 only): the input arrives pre-split — its producer's epilogue wrote the (h, m, l) bf16 planes of
// every value (a.outp below, the same RNE split as split8t) — so a step gathers the three planes of its 8 channels
// (three 16-byte loads per half instead of two of fp32) and splits nothing: the ~5 VALU per gathered value that
// every one of a row's ~14 uses repeated are gone.  Bit-identical to PS = 0.
template <int TN, int NS, int H, int PS>
__global__ __launch_bounds__(256, 2) void spconv_bx_kernel(SpArgs a, const uint16_t* __restrict__ wimg, int64_t CoutP,
                                                           const float* __restrict__ isc) {
  using namespace bx;
  // NS: steps in flight (register sets: gathered rows + weights)
  constexpr int NPL = planes<H>();
  constexpr float XS = H ? 64.f : 1.f;
  constexpr int TM = 128;                       // output rows per workgroup (4 waves x 32)
  constexpr int NJ = TN / 32;                   // accumulator tiles per wave
  constexpr int BPL = TN * SB_BST;              // 16-bit elements of one plane of a weight stage
  constexpr int BG = NPL * BPL * 2 / 16;        // 16-byte granules of a weight stage
  constexpr int GPT = (BG + 255) / 256;         // ... per thread
  if (a.guard && *a.guard != a.epoch) return;   // uniform: the split-fp16 launch stayed in range
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][NPL * BPL];
  __shared__ int32_t nb[TM][SP_KMAX + 1];
  __shared__ int klist[SP_KMAX];
  __shared__ int orow_s[TM];     // the tile's output rows (perm applied; -1 past Mout)
  __shared__ unsigned wmask[4];  // per-wave OR of the rows' active-offset masks

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
#if SP_TRACE   // phases: 0 tile setup, 1 weight store (+ wait), 2 A split, 3 gather issue, 4 MFMAs, 5 barrier, 6 epilogue
  unsigned long long tr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = __builtin_amdgcn_s_memtime();
  int prev_slot = 0;
#endif
  // 1-D grid of (row tile, column tile) in dispatch order (round robin over the XCDs: an XCD-contiguous tile order
  // was measured slower, DESIGN §4.1 — one XCD then gets all the expensive tiles of a mask class)
  const int gy = (a.Cout + TN - 1) / TN;
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t o0 = (t / gy) * TM;
  const int c0 = (int)(t % gy) * TN;
  const int K = a.K;

  // tile setup in two dependent rounds of loads (the rows' perm entries, then every neighbour entry of the tile at
  // once, coalesced along the rows of the map) instead of one round per 256 entries
  if (tid < TM) {
    const int64_t o = o0 + tid;
    orow_s[tid] = o < a.Mout ? (int)(a.perm ? a.perm[o] : o) : -1;
  }
  __syncthreads();
  {
    constexpr int EMAX = (TM * SP_KMAX + 255) / 256;
    const int dq = 256 / K, dr = 256 - dq * K;   // entry e + 256 = (row + dq, k + dr), carried
    int row = tid / K, k = tid - row * K;
    int vv[EMAX], ks[EMAX], rs[EMAX];
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      ks[i] = k;
      rs[i] = row;
      vv[i] = -1;
      if (row < TM) {
        const int orow = orow_s[row];
        if (orow >= 0) vv[i] = a.nbr ? a.nbr[(int64_t)orow * K + k] : orow;
      }
      row += dq;
      k += dr;
      if (k >= K) {
        k -= K;
        ++row;
      }
    }
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (rs[i] < TM) {
        nb[rs[i]][ks[i]] = vv[i];
        if (vv[i] >= 0) m |= 1u << ks[i];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m |= (unsigned)__shfl_xor((int)m, off, 64);
    if (lane == 0) wmask[w] = m;
  }
  __syncthreads();
  const unsigned kmask = wmask[0] | wmask[1] | wmask[2] | wmask[3];
  if (tid < K && ((kmask >> tid) & 1u)) klist[__popc(kmask & ((1u << tid) - 1u))] = tid;
  const int nk = __popc(kmask);
  __syncthreads();

  const int nci = (a.Cin + SB_K - 1) / SB_K;
  const int steps = nk * nci;
  const int row = 32 * w + l32;   // this lane's tile row

  // gathered A of one step: k-step st, channels ci0 + 16 st + 8h + (0..7) of the lane's row, as two
  // float4 each (clamped addresses; validity bits applied at the split)
  typedef float f32x4 __attribute__((ext_vector_type(4)));   // (a HIP float4 copy becomes a memcpy through scratch)
  static_assert(!(PS && H), "pre-split planes are split-bf16");
  struct ASet {
    float4 v[PS ? 1 : 4];                  // fp32 gathers (PS = 0)
    bf16x8 pv[PS ? 2 : 1][PS ? 3 : 1];     // pre-split gathers (PS = 1): [k16 half][plane]
    f32x4 bq[GPT];   // the step's weight stage granules (this thread's share)
  };
  auto load_a = [&](int s, ASet& A) {
    if (s >= steps) s = steps - 1;   // clamped re-read past the end
    const int k = klist[s / nci];
    const int ci0 = (s % nci) * SB_K;
    const int src = nb[row][k];
    if (PS) {
      const uint16_t* base = a.inp + (int64_t)(src >= 0 ? src : 0) * 3 * a.ldin;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {   // an absent neighbour reads zero planes
          const uint16_t* pq = base + pl * a.ldin + ci0 + 16 * st + 8 * h;
          A.pv[st % (PS ? 2 : 1)][pl % (PS ? 3 : 1)] =
              *reinterpret_cast<const bf16x8*>(src >= 0 ? (const void*)pq : (const void*)g_sp_zero);
        }
    } else {
      const float* base = a.in + (int64_t)(src >= 0 ? src : 0) * a.ldin;
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // an absent neighbour reads zeros (no masking at the split; Cin % 32 == 0)
        const int ci = ci0 + 16 * (q >> 1) + 8 * h + 4 * (q & 1);
        const float* pq = src >= 0 ? base + ci : g_sp_zero;
        A.v[q % (PS ? 1 : 4)] = *reinterpret_cast<const float4*>(pq);
      }
    }
    const int cb = s % nci;
    const char* wb = reinterpret_cast<const char*>(wimg) + ((int64_t)(k * nci + cb) * NPL * CoutP + c0) * SB_BST * 2;
#if SPBX_WBUF
    // the step's weight stage as a buffer (wave-uniform base), 32-bit lane offsets
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, 0x7fffffff,
                                                                        0x00020000);
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int g = min(tid + 256 * i, BG - 1);
      const int pl = g / (TN * 5), wi = g - pl * (TN * 5);
      A.bq[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rw, pl * (int)CoutP * SB_BST * 2 + wi * 16, 0, 0));
    }
#else
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int g = min(tid + 256 * i, BG - 1);
      const int pl = g / (TN * 5), wi = g - pl * (TN * 5);
      A.bq[i] = *reinterpret_cast<const f32x4*>(wb + (int64_t)pl * CoutP * SB_BST * 2 + wi * 16);
    }
#endif
  };
  bool xbad = false;   // H = 1: a gathered value past the fp16 window
  float xmx = 0.f;     // H = 1: max |value| x XS of this lane's splits
  auto frag_a = [&](const ASet& A, int st) {
    if (PS) {
      FragT<H> f;
#pragma unroll
      for (int pl = 0; pl < planes<H>(); ++pl)
        f.p[pl] = __builtin_bit_cast(typename FragT<H>::V, A.pv[st % (PS ? 2 : 1)][pl % (PS ? 3 : 1)]);
      return f;
    }
    float v[8];
    const float4 x0 = A.v[(2 * st) % (PS ? 1 : 4)], x1 = A.v[(2 * st + 1) % (PS ? 1 : 4)];
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    if (H) {
      float mx = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[i] *= XS;
        mx = fmaxf(mx, fabsf(v[i]));
      }
      xbad |= !(mx < F16_RANGE);
      xmx = fmaxf(xmx, mx);
    }
    return split8t<H>(v);
  };
  // weight stage of a step: granule g of [plane][TN rows][80 B] <- image rows (k, channel block) at column c0
  auto store_b = [&](const ASet& A, int buf) {
    char* dst = reinterpret_cast<char*>(Bs[buf]);
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int g = tid + 256 * i;
      if (g < BG) *reinterpret_cast<f32x4*>(dst + g * 16) = A.bq[i];
    }
  };

  floatx16 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  if (steps > 0) {
    // step s: the weights of step s + 1 (loaded NS steps ago) -> the other LDS stage, the split of step s's
    // gathered rows, its set refilled with step s + NS, the MFMAs; one barrier
    ASet A[NS];
    SPSTAMP(7);
#pragma unroll
    for (int u = 0; u < NS; ++u) load_a(u, A[u]);
    store_b(A[0], 0);
    __syncthreads();
    auto step = [&](int s, ASet& A, const ASet& An) {
      const int cur = s & 1;
      SPSTAMP(1);
      if (s + 1 < steps) store_b(An, cur ^ 1);
      SPSTAMP(2);
      const FragT<H> fa0 = frag_a(A, 0), fa1 = frag_a(A, 1);
      SPSTAMP(3);
      load_a(s + NS, A);
      SPSTAMP(4);
      const uint16_t* Bq = Bs[cur];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const FragT<H>& fa = st ? fa1 : fa0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint16_t* bp = Bq + (32 * j + l32) * SB_BST + 16 * st + 8 * h;
          const FragT<H> fb = ld_frag<H>(reinterpret_cast<const char*>(bp), 2 * BPL);
          acc[j] = mma<H>(fa, fb, acc[j]);
        }
      }
      SPSTAMP(5);
      __syncthreads();
    };
    int s = 0;
    for (; s + NS - 1 < steps; s += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) step(s + u, A[u], A[(u + 1) % NS]);
    }
#pragma unroll
    for (int u = 0; u < NS - 1; ++u)
      if (s + u < steps) step(s + u, A[u], A[(u + 1) % NS]);
  }

  SPSTAMP(6);
  // epilogue: the rows from LDS, every residual of a column tile loaded before its stores (out may be res)
  int orr[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) orr[r] = orow_s[32 * w + (r & 3) + 8 * (r >> 2) + 4 * h];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = c0 + j * 32 + l32;
    if (c >= a.Cout) continue;
    float bsc = 1.f, bsh = 0.f;
    if (a.bn.gamma) {
      bsc = a.bn.gamma[c] / sqrtf(a.bn.var[c] + a.bn_eps);
      bsh = a.bn.beta[c] - a.bn.mean[c] * bsc;
    }
    const float bias = a.bias ? a.bias[c] : 0.f;
    const float is = H ? isc[c] : 1.f;
    float rv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rv[r] = a.res && orr[r] >= 0 ? a.res[(int64_t)orr[r] * a.ldres + c] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (orr[r] < 0) continue;
      float v = (H ? acc[j][r] * is : acc[j][r]) + bias;
      v = fmaf(v, bsc, bsh);
      if (a.res) v += rv[r];
      if (a.relu) v = fmaxf(v, 0.f);
      a.out[(int64_t)orr[r] * a.ldout + c] = v;
      if (a.outp) bx::store_planes(a.outp + (int64_t)orr[r] * 3 * a.ldout + c, a.ldout, v);
    }
  }
  if (H && __any(xbad || (xmx > 0.f && xmx < 0.125f)) && lane == 0) atomicExch(a.range, a.epoch);
#if SP_TRACE
  SPSTAMP(0);
  if (lane == 0)
    for (int q = 0; q < 8; ++q) atomicAdd(&g_sp_trace[q], tr[q]);
#endif
}

// per output channel c: s_c = range_scale(max_{k, ci} |W[k][ci][c]|) -> wsc[c], isc[c] = 1 / (s_c 2^6); one wave
// per channel
__global__ void spconv_wscale_kernel(const float* __restrict__ W, int K, int Cin, int Cout, int64_t CoutP, float* wsc,
                                     float* isc) {
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (c >= CoutP) return;   // whole waves
  float amax = 0.f;
  if (c < Cout)
    for (int64_t e = lane; e < (int64_t)K * Cin; e += 64) amax = fmaxf(amax, fabsf(W[e * Cout + c]));
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if (lane == 0) {
    const float s = bx::range_scale(amax);
    wsc[c] = s;
    isc[c] = 1.f / (s * 64.f);
  }
}

// W [K][Cin][Cout] fp32 -> image: [K][nci][3][CoutP][40] bf16 (h, m, l planes; zero padding), then
// [K][nci][2][CoutP][40] fp16 (h, l of W[.][.][c] wsc[c]), then wsc[CoutP], isc[CoutP]
__global__ void spconv_wimage_kernel(const float* __restrict__ W, int K, int Cin, int Cout, int nci, int64_t CoutP,
                                     uint16_t* img, uint16_t* img16, const float* __restrict__ wsc) {
  using namespace bx;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (k, cb, c, 4 groups of 8 channels)
  const int64_t total = (int64_t)K * nci * CoutP * 4;
  if (e >= total) return;
  const int q = (int)(e & 3);
  const int64_t t = e >> 2;
  const int c = (int)(t % CoutP);
  const int64_t kb = t / CoutP;   // k * nci + cb
  const int cb = (int)(kb % nci), k = (int)(kb / nci);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ci = cb * SB_K + 8 * q + i;
    v[i] = (ci < Cin && c < Cout) ? W[((int64_t)k * Cin + ci) * Cout + c] : 0.f;
  }
  Frag f;
  split8(v, f.h, f.m, f.l);
  uint16_t* row = img + ((kb * 3) * CoutP + c) * SB_BST + 8 * q;
  *reinterpret_cast<bf16x8*>(row) = f.h;
  *reinterpret_cast<bf16x8*>(row + CoutP * SB_BST) = f.m;
  *reinterpret_cast<bf16x8*>(row + 2 * CoutP * SB_BST) = f.l;
  const float sc = wsc[c];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= sc;
  const FragT<1> g = split8t<1>(v);
  uint16_t* row16 = img16 + ((kb * 2) * CoutP + c) * SB_BST + 8 * q;
  *reinterpret_cast<f16x8*>(row16) = g.p[0];
  *reinterpret_cast<f16x8*>(row16 + CoutP * SB_BST) = g.p[1];
}

#ifndef SPCONV_MATH_DEFAULT
#define SPCONV_MATH_DEFAULT 0
#endif
int g_spconv_h = SPCONV_MATH_DEFAULT;   // mvr_set_math: split-fp16 (1) where a range flag is passed

}  // namespace mvr

using namespace mvr;

static int64_t sp_coutp(int Cout) { return ((int64_t)Cout + SB_CP - 1) / SB_CP * SB_CP; }

// image sections (bytes): bf16 planes, fp16 planes, wsc, isc
static size_t sp_bf16_bytes(int K, int Cin, int Cout) {
  return (size_t)K * ((Cin + SB_K - 1) / SB_K) * 3 * sp_coutp(Cout) * SB_BST * 2;
}
static size_t sp_f16_bytes(int K, int Cin, int Cout) { return sp_bf16_bytes(K, Cin, Cout) / 3 * 2; }

extern "C" size_t mvr_spconv_wimage_bytes(int K, int Cin, int Cout) {
  if (K <= 0 || Cin <= 0 || Cout <= 0) return 0;
  return sp_bf16_bytes(K, Cin, Cout) + sp_f16_bytes(K, Cin, Cout) + 2 * sp_coutp(Cout) * sizeof(float);
}

extern "C" int mvr_spconv_wimage(const float* W, int K, int Cin, int Cout, void* img, size_t bytes, hipStream_t s) {
  if (!W || !img || K <= 0 || K > SP_KMAX || Cin <= 0 || Cout <= 0 || bytes < mvr_spconv_wimage_bytes(K, Cin, Cout) ||
      (reinterpret_cast<uintptr_t>(img) & 15))
    return MVR_EINVAL;
  const int nci = (Cin + SB_K - 1) / SB_K;
  const int64_t CoutP = sp_coutp(Cout);
  const int64_t total = (int64_t)K * nci * CoutP * 4;
  char* base = reinterpret_cast<char*>(img);
  uint16_t* img16 = reinterpret_cast<uint16_t*>(base + sp_bf16_bytes(K, Cin, Cout));
  float* wsc = reinterpret_cast<float*>(base + sp_bf16_bytes(K, Cin, Cout) + sp_f16_bytes(K, Cin, Cout));
  hipLaunchKernelGGL(spconv_wscale_kernel, dim3((unsigned)((CoutP * 64 + 255) / 256)), dim3(256), 0, s, W, K, Cin, Cout,
                     CoutP, wsc, wsc + CoutP);
  MVR_CHECK_LAUNCH();
  hipLaunchKernelGGL(spconv_wimage_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, W, K, Cin, Cout, nci,
                     CoutP, reinterpret_cast<uint16_t*>(img), img16, wsc);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_spconv_x(const float* in, int64_t ldin, int Cin, const int32_t* nbr, const int32_t* perm, int K,
                            int64_t Mout, const float* W, int Cout, const float* bias, mvr_bn_p bn, float bn_eps,
                            const float* res, int64_t ldres, int relu, float* out, int64_t ldout, const void* wimg,
                            int32_t* range_flag, const uint16_t* in_planes, uint16_t* out_planes, hipStream_t s) {
  if (Cin <= 0 || Cout <= 0 || K <= 0 || K > SP_KMAX || Mout < 0) return MVR_EINVAL;
  if (Mout == 0) return MVR_OK;   // no output rows: NULL pointers allowed (mvreg.h conventions)
  if (!in || !W || !out || !wimg) return MVR_EINVAL;
  if ((in_planes && ((ldin & 7) || (reinterpret_cast<uintptr_t>(in_planes) & 15))) ||
      (out_planes && (reinterpret_cast<uintptr_t>(out_planes) & 1)))
    return MVR_EINVAL;
  if (reinterpret_cast<uintptr_t>(wimg) & 15) return MVR_EINVAL;
  if (!nbr && K != 1) return MVR_EINVAL;
  if ((Cin % SB_K) || (Cout & 3) || (ldin & 3) || (reinterpret_cast<uintptr_t>(in) & 15) ||
      (reinterpret_cast<uintptr_t>(W) & 15))
    return MVR_EINVAL;
  SpArgs a{in, ldin, Cin, nbr, K, Mout, perm, W, Cout, bias, bn, bn_eps, res, ldres, relu, out, ldout,
           nullptr, nullptr, 0, in_planes, out_planes};
  // the launch cannot see how many kernel-map entries are present (no host sync): FLOPs as if every offset were,
  // bytes compulsory (input rows ~ output rows, the neighbour table, the weights); bench.py replaces both class
  // totals with counts from the kernel maps
  ProfScope prof(PK_SPCONV, 2.0 * Mout * (double)K * Cin * Cout,
                 (double)Mout * (Cin + Cout) * 4.0 + (nbr ? (double)Mout * K * 4.0 : 0.0) + 4.0 * K * Cin * Cout, s);
  const char* base = reinterpret_cast<const char*>(wimg);
  const uint16_t* wi = reinterpret_cast<const uint16_t*>(wimg);
  const uint16_t* wi16 = reinterpret_cast<const uint16_t*>(base + sp_bf16_bytes(K, Cin, Cout));
  const int64_t CoutP = sp_coutp(Cout);
  const float* isc = reinterpret_cast<const float*>(base + sp_bf16_bytes(K, Cin, Cout) + sp_f16_bytes(K, Cin, Cout)) +
                     CoutP;
  const unsigned gx = (unsigned)((Mout + 127) / 128);
  // split-fp16 then its guarded split-bf16 re-run: only with the caller's flag word (cleared here, stream-ordered)
  // and not where the output is the residual (in place: the re-run reads it).  Output tiles of 32 / 64 channels
  // stay split-bf16: there the split-fp16 kernel holds more VGPRs (155 vs 125 at TN = 32), one workgroup per CU
  // fewer for a gather-latency bound loop — measured slower (tools/spconv_micro.py: s1:1:32:32 0.378 -> 0.384 ms,
  // up:1:128:64 0.403 -> 0.453), where the 128-channel tiles gain (s1:4:128:128 0.304 -> 0.217, s1:8:256:256
  // 0.437 -> 0.346).  (in / out never alias: rows are gathered.)
  const bool h1 = g_spconv_h && range_flag && Cout > 64 && res != out;
  if (h1) {
    if (hipMemsetAsync(range_flag, 0, sizeof(int32_t), s) != hipSuccess) return MVR_ELAUNCH;
    a.range = range_flag;
    a.epoch = 1;
  }
#define MVR_SPL(TN_, NS_, PNS_, GY)                                                                             \
  do {                                                                                                         \
    if (h1) {                                                                                                  \
      hipLaunchKernelGGL((spconv_bx_kernel<TN_, NS_, 1, 0>), dim3(gx * (GY)), dim3(256), 0, s, a, wi16, CoutP, isc); \
      MVR_CHECK_LAUNCH();                                                                                      \
      a.guard = a.range;                                                                                       \
      a.range = nullptr;                                                                                       \
    }                                                                                                          \
    if (in_planes)                                                                                             \
      hipLaunchKernelGGL((spconv_bx_kernel<TN_, PNS_, 0, 1>), dim3(gx * (GY)), dim3(256), 0, s, a, wi, CoutP, isc); \
    else                                                                                                       \
      hipLaunchKernelGGL((spconv_bx_kernel<TN_, NS_, 0, 0>), dim3(gx * (GY)), dim3(256), 0, s, a, wi, CoutP, isc); \
  } while (0)
  if (Cout <= 32)
    MVR_SPL(32, SPBX_NS32, SPBX_PS_NS32, 1);
  else if (Cout <= 64)
    MVR_SPL(64, SPBX_NS64, SPBX_PS_NS64, (Cout + 63) / 64);
  else
    MVR_SPL(128, SPBX_NS128, SPBX_PS_NS128, (Cout + 127) / 128);
#undef MVR_SPL
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_spconv(const float* in, int64_t ldin, int Cin, const int32_t* nbr, const int32_t* perm, int K,
                          int64_t Mout, const float* W, int Cout, const float* bias, mvr_bn_p bn, float bn_eps,
                          const float* res, int64_t ldres, int relu, float* out, int64_t ldout, const void* wimg,
                          int32_t* range_flag, hipStream_t s) {
  return mvr_spconv_x(in, ldin, Cin, nbr, perm, K, Mout, W, Cout, bias, bn, bn_eps, res, ldres, relu, out, ldout, wimg,
                      range_flag, nullptr, nullptr, s);
}

#if SP_TRACE
// tools only (library built with -DSP_TRACE=1): the phase totals of every spconv_bx wave since the last reset
extern "C" int mvr_spconv_trace(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mvr::g_sp_trace), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mvr::g_sp_trace), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
