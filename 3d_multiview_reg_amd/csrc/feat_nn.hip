// Feature-space nearest neighbour (Soft_NN) for a batch of fragment pairs.
//
// Replaces lib/layers.py:44-88 (Soft_NN.forward) + lib/utils.py:968-992
// (pairwise_distance) + the pair gather of lib/utils.py:850-885 and the xs
// assembly of lib/utils.py:915.  The reference materialises the [P,N,M]
// distance and softmax matrices (100 MB per pair); here they never leave
// registers:
//   * S^T = Ft . Fs^T on v_mfma_f32_32x32x16_bf16 with both operands split into three bf16
//     terms (fp32-level accuracy, see gemm.hpp MATH_BF16X3); the QUERY index is the lane column,
//     so each lane owns one query's running softmax state;
//   * logits (2 fs.ft - |ft|^2) / tau^2 (|fs|^2 is constant per query and cancels in the
//     softmax / argmax);
//   * flash-style online softmax in base 2 over 32-target chunks, the 3-wide weighted
//     coordinate sum accumulated in packed fp32 (v_pk_fma_f32) registers;
//   * argmax tracking for the straight-through ('st') and 'hard' modes.
// Targets stream through double-buffered LDS in 128-row stages shared by the 4 waves (128
// queries) of a workgroup: the next stage is loaded into registers during the current one, then
// split into bf16 planes once per workgroup (not per wave) on its way into LDS.
//
// FLOPs per pair ~ 2*N*M*C (MFMA) + N*M*(exp + ~6 VALU); HBM: features/coords of the two
// fragments (L2/MALL-resident across the pairs that share them).
#include "common.hpp"
#include "knobs.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"

namespace mvr {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

#ifndef NN_STAGE_ROWS
#define NN_STAGE_ROWS 128
#endif
constexpr int NN_STAGE = NN_STAGE_ROWS;   // targets per LDS stage
constexpr int NN_TPR = 256 / NN_STAGE;    // staging threads per target row
constexpr int NN_FPT = 32 / NN_TPR;       // ... and the feature dims each of them loads (multiple of 8)
static_assert(NN_STAGE % 32 == 0 && NN_FPT % 8 == 0, "stage: whole 32-target chunks, 8-dim split groups");
constexpr int NN_ROW = 32;         // bf16 per LDS plane row; 16-byte chunk c of row r sits at slot
                                   // c ^ ((r >> 2) & 3): conflict-free ds_read_b128 down 16 rows
constexpr float NN_NEG = -3.0e38f;

struct NNArgs {
  const float* Fq; int64_t fq_fs;    // query features [*][Nq][32], fragment stride (elements)
  const float* Ft; int64_t ft_fs;    // target features [*][Mt][32]
  const float* Xq; int64_t xq_fs;    // query coords (optional: output then holds [x_q | x_corr])
  const float* Xt; int64_t xt_fs;    // target coords [*][Mt][3]
  const int64_t* pairs;              // [P][2] (query fragment, target fragment)
  int P, Nq, Mt;
  float k2;                          // log2(e) / tau^2
  int mode;                          // 0 soft, 1 argmax (soft+st / hard)
  float* out; int64_t o_ps, o_ns;    // out(p,n,:) = [x_q(0..2) |] x_corr(0..2)
  int32_t* idx;                      // optional argmax index [P][Nq]
  int fast;                          // soft mode: try the bounded-shift path first (feat_nn_fast)
  const char* timg; int64_t timg_fs; // optional: targets pre-split per stage (nn_presplit_kernel), bytes per fragment
  unsigned seed_lo, seed_hi;         // MODE 3 / 4 (soft_gumbel): the noise's seed
  float itau;                        // MODE 3 / 4: 1 / tau (the noise's scale in the logit)
};

// soft_gumbel (lib/layers.py:72-78, F.gumbel_softmax(-dist, tau, hard)): y = softmax((-dist + g) / tau) with
// g = -log(e), e ~ Exp(1) per (query, target).  The noise is counter-based — a 32-bit hash of (seed, query fragment,
// target fragment, query, target), so it does not depend on the batch a pair runs in and oracle/soft_nn.py
// reproduces it — instead of torch's Philox stream (the reference's draws cannot be replayed: SURVEY §8a6, parity by
// restatement).  u = (hash >> 9 + 1/2) 2^-23 in (0, 1) — 24 significant bits, exact in fp32, so u never rounds to
// 1 (g = inf) and the oracle's float64 u is the same number — e = -ln u.
__device__ __host__ __forceinline__ unsigned nn_mix32(unsigned x) {   // lowbias32 finalizer
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ unsigned nn_gumbel_query(const NNArgs& a, int64_t src, int64_t tgt, int j) {
  const unsigned k = nn_mix32(a.seed_lo ^ nn_mix32(a.seed_hi + 0x9E3779B9u * (unsigned)tgt) ^
                              (0x85EBCA77u * (unsigned)src));
  return nn_mix32(k ^ (unsigned)j);
}
// the noise's contribution to a logit in log2 units (z = log2(e) (2 fs.ft - |ft|^2) / tau): log2(e) g / tau
__device__ __forceinline__ float nn_gumbel_z(unsigned hq, int i, float itau) {
  const unsigned x = nn_mix32(hq + 0x9E3779B9u * (unsigned)i);
  const float u = ((float)(x >> 9) + 0.5f) * 1.1920928955078125e-7f;          // (0, 1), exact in fp32
  const float w = ((float)(0x7FFFFFu - (x >> 9)) + 0.5f) * 1.1920928955078125e-7f;   // 1 - u, exact
  // -ln u > 0; near u = 1 (w < 2^-6) the series of -ln(1 - w), so e keeps its relative precision where the noise
  // is largest (g = -ln e) and that element dominates the softmax
  const float e = w < 0.015625f ? w * fmaf(w, fmaf(w, fmaf(w, 0.25f, 0.33333334f), 0.5f), 1.f)
                                : -0.69314718055994531f * __builtin_amdgcn_logf(u);
  return -itau * __builtin_amdgcn_logf(e);                                     // log2(e) g / tau, g = -ln e
}

// Pre-split target image (mvr_feat_nn_ws): per target fragment and 128-target stage, the bytes the fast path's LDS
// stage holds — the three bf16 planes of the features in the swizzled [row][32] layout, then (x, y, z, k2 |ft|^2)
// per target — so that a stage is two LDS-DMA copies instead of loads, splits and LDS stores in every workgroup
// (each target fragment is staged by 40 query blocks x 29 pairs).
constexpr int NN_IMG_PLANES = 3 * NN_STAGE * NN_ROW * 2;   // 24 KB
constexpr int NN_IMG_STAGE = NN_IMG_PLANES + NN_STAGE * 16 + NN_STAGE * 4;   // + 2 KB of (x, y, z, w hm) + 512 B of w l

__device__ __forceinline__ unsigned nn_cvt_pk(f32x2 x) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
}
__device__ __forceinline__ f32x2 nn_unpack(unsigned p) {
  f32x2 r;
  r.x = __uint_as_float(p << 16);
  r.y = __uint_as_float(p & 0xffff0000u);
  return r;
}
// 8 fp32 -> three bf16x8 terms (x = h + m + l to 2^-25 |x|), as u32x4 (packed pairs)
__device__ __forceinline__ void nn_split8(const float4& a, const float4& b, u32x4& H, u32x4& Mm, u32x4& L) {
  const f32x2 x[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned hp = nn_cvt_pk(x[i]);
    const f32x2 r = bx::sub2(x[i], nn_unpack(hp));
    const unsigned mp = nn_cvt_pk(r);
    H[i] = hp;
    Mm[i] = mp;
    L[i] = nn_cvt_pk(bx::sub2(r, nn_unpack(mp)));
  }
}
// 8 fp32 -> two fp16x8 terms of 2^8 x (x 2^8 = h + l to 2^-22 relative, 2^-25 absolute), as u32x4; the
// fp16 form of the fast path (feat_nn_fast<1>): |x| < 2^7 keeps x 2^8 inside the fp16 range
__device__ __forceinline__ void nn_split8h(const float4& a, const float4& b, u32x4& H, u32x4& L) {
  const f32x2 x[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 v = x[i] * 256.f;
    const f16x2 hh = __builtin_convertvector(v, f16x2);
    H[i] = __builtin_bit_cast(unsigned, hh);
    L[i] = __builtin_bit_cast(unsigned, __builtin_convertvector(v - __builtin_convertvector(hh, f32x2), f16x2));
  }
}
// The split-bf16 fast path folds the target term -k2 |ft|^2 of the logit into the distance MFMAs (one more MFMA per
// 32-target chunk against a constant operand of ones, instead of one fma per (query, target)): -w as three bf16
// terms, (h | m << 16) in the .w slot of the target's (x, y, z, .) entry and l in a second word.  Invalid targets
// (past Mt): h = -inf, m = l = 0 (weight 0).
__device__ __forceinline__ void nn_wsplit(float w, bool ok, unsigned& hm, unsigned& l) {
  if (!ok) {
    hm = 0xFF80u;   // bf16 -inf
    l = 0u;
    return;
  }
  const float v = -w;
  const unsigned hp = nn_cvt_pk((f32x2){v, 0.f}) & 0xFFFFu;
  const float r = v - __uint_as_float(hp << 16);
  const unsigned mp = nn_cvt_pk((f32x2){r, 0.f}) & 0xFFFFu;
  hm = hp | (mp << 16);
  l = nn_cvt_pk((f32x2){r - __uint_as_float(mp << 16), 0.f}) & 0xFFFFu;
}
__device__ __forceinline__ float nn_max3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }
// |f|^2 over a stage thread's 16 dims in one fixed fma order (the stage split and the pre-split image share it:
// identical stages)
__device__ __forceinline__ float nn_norm16(const float4 (&fr)[4]) {
  float n2 = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    n2 = fmaf(fr[v].x, fr[v].x, n2);
    n2 = fmaf(fr[v].y, fr[v].y, n2);
    n2 = fmaf(fr[v].z, fr[v].z, n2);
    n2 = fmaf(fr[v].w, fr[v].w, n2);
  }
  return n2;
}

struct NNSmem {
  unsigned short Fp[2][3][NN_STAGE][NN_ROW];   // bf16 planes h, m, l of the target features
  union {
    float Xs[2][4][NN_STAGE];                  // online path: x, y, z, |ft|^2 k2 (SoA)
    float4 Xf[2][NN_STAGE];                    // fast path: (x, y, z, |ft|^2 k2) per target (split-bf16: .w = hm
  };                                           // bits of nn_wsplit)
  unsigned Wl[2][NN_STAGE];                    // split-bf16 fast path: the l term of nn_wsplit
  int flag;
};

// Workgroup -> (pair, 128-query block): XCD-contiguous (common.hpp xcd_tile), so the query blocks of a pair, which
// all stream the same target fragment, run on one XCD and share its L2 instead of each XCD fetching the targets
__device__ __forceinline__ void nn_block(int& p, int& qb) {
  const int64_t nb = (int64_t)gridDim.x * gridDim.y;
  const int64_t t = xcd_tile((int64_t)blockIdx.y * gridDim.x + blockIdx.x, nb);
  p = (int)(t / gridDim.x);
  qb = (int)(t % gridDim.x);
}

// Online-softmax path (any temperature / feature scale; argmax modes).
template <int MODE>
__device__ __forceinline__ void feat_nn_online(const NNArgs& a, NNSmem& sm) {
  auto& Fp = sm.Fp;
  auto& Xs = sm.Xs;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;
  int p, qb;
  nn_block(p, qb);
  const int64_t src = a.pairs[2 * p], tgt = a.pairs[2 * p + 1];
  const float* Fq = a.Fq + src * a.fq_fs;
  const float* Ft = a.Ft + tgt * a.ft_fs;
  const float* Xt = a.Xt + tgt * a.xt_fs;
  const int j = qb * 128 + wid * 32 + l32;  // this lane's query
  const bool jok = j < a.Nq;
  const int Mt = a.Mt;

  // query = B operand of k16 step s: lane half kh holds dims 16s + 8kh + (0..7)
  bf16x8 qh[2], qm[2], ql[2];
  {
    const float4* qp = reinterpret_cast<const float4*>(Fq + (int64_t)(jok ? j : 0) * 32);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 H, Mm, L;
      nn_split8(qp[4 * s + 2 * kh], qp[4 * s + 2 * kh + 1], H, Mm, L);
      qh[s] = __builtin_bit_cast(bf16x8, H);
      qm[s] = __builtin_bit_cast(bf16x8, Mm);
      ql[s] = __builtin_bit_cast(bf16x8, L);
    }
  }

  // stage staging: thread -> target row (tid >> 1), dims 16 (tid & 1) .. +15; coords by tid < 128
  const int srow = tid / NN_TPR, spart = tid % NN_TPR;
  float4 fr[NN_FPT / 4];
  float xr0 = 0.f, xr1 = 0.f, xr2 = 0.f;
  auto load_regs = [&](int t0) {
    const int gi = t0 + srow;
    const float4* fp = reinterpret_cast<const float4*>(Ft + (int64_t)(gi < Mt ? gi : 0) * 32 + NN_FPT * spart);
#pragma unroll
    for (int v = 0; v < NN_FPT / 4; ++v) fr[v] = gi < Mt ? fp[v] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE != 2 && tid < NN_STAGE) {
      const int gc = t0 + tid;
      if (gc < Mt) {
        const float* xp = Xt + (int64_t)gc * 3;
        xr0 = xp[0]; xr1 = xp[1]; xr2 = xp[2];
      }
    }
  };
  auto store_lds = [&](int buf, int t0) {
#pragma unroll
    for (int g = 0; g < NN_FPT / 8; ++g) {   // dims NN_FPT spart + 8g .. +7
      u32x4 H, Mm, L;
      nn_split8(fr[2 * g], fr[2 * g + 1], H, Mm, L);
      const int c = 8 * (((NN_FPT / 8) * spart + g) ^ ((srow >> 2) & 3));
      *reinterpret_cast<u32x4*>(&Fp[buf][0][srow][c]) = H;
      *reinterpret_cast<u32x4*>(&Fp[buf][1][srow][c]) = Mm;
      *reinterpret_cast<u32x4*>(&Fp[buf][2][srow][c]) = L;
    }
    float n2 = 0.f;
#pragma unroll
    for (int v = 0; v < NN_FPT / 4; ++v) n2 += fr[v].x * fr[v].x + fr[v].y * fr[v].y + fr[v].z * fr[v].z + fr[v].w * fr[v].w;
#pragma unroll
    for (int o = 1; o < NN_TPR; o <<= 1) n2 += __shfl_xor(n2, o, 64);
    // invalid targets: +inf -> logit -inf -> weight 0, never the argmax
    if (spart == 0) Xs[buf][3][srow] = (t0 + srow < Mt) ? n2 * a.k2 : __builtin_inff();
    if (MODE != 2 && tid < NN_STAGE) {
      Xs[buf][0][tid] = xr0;
      Xs[buf][1][tid] = xr1;
      Xs[buf][2][tid] = xr2;
    }
  };

  float run_m = NN_NEG;
  f32x2 s2 = {0.f, 0.f}, ax2 = {0.f, 0.f}, ay2 = {0.f, 0.f}, az2 = {0.f, 0.f};
  float best = NN_NEG, second = NN_NEG;
  int besti = 0x7fffffff, secondi = 0x7fffffff;
  const float kk2 = 2.f * a.k2;
  constexpr bool GUM = MODE == 3 || MODE == 4;   // soft_gumbel: soft / hard (straight-through)
  const unsigned hq = GUM ? nn_gumbel_query(a, src, tgt, j) : 0u;

  const int nst = (Mt + NN_STAGE - 1) / NN_STAGE;
  load_regs(0);
  store_lds(0, 0);
  __syncthreads();
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    const int t0 = st * NN_STAGE;
    if (st + 1 < nst) load_regs(t0 + NN_STAGE);
    // 4 chunks of 32 targets; the MFMAs of chunk c+1 are issued before the softmax of chunk c so
    // the two streams interleave within the wave (invalid targets carry |ft|^2 k2 = +inf)
    auto mfma_chunk = [&](int i0) {
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int row = i0 + l32;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 8 * ((2 * s + kh) ^ ((row >> 2) & 3));
        const bf16x8 th = *reinterpret_cast<const bf16x8*>(&Fp[cur][0][row][c]);
        const bf16x8 tm = *reinterpret_cast<const bf16x8*>(&Fp[cur][1][row][c]);
        const bf16x8 tl = *reinterpret_cast<const bf16x8*>(&Fp[cur][2][row][c]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, qh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, ql[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qm[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qh[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qm[s], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qh[s], acc, 0, 0, 0);
      }
      return acc;
    };
    // acc[r] = ft[i] . fs[j],  i = i0 + 8 (r >> 2) + 4 kh + (r & 3)
    auto consume = [&](const floatx16& acc, int i0) {
      f32x2 z[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 T = *reinterpret_cast<const float4*>(&Xs[cur][3][i0 + 8 * g + 4 * kh]);
        const f32x2 a0 = {acc[4 * g], acc[4 * g + 1]}, a1 = {acc[4 * g + 2], acc[4 * g + 3]};
        const f32x2 t0v = {T.x, T.y}, t1v = {T.z, T.w};
        z[2 * g] = a0 * kk2 - t0v;
        z[2 * g + 1] = a1 * kk2 - t1v;
      }
      if (GUM) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          z[r >> 1][r & 1] += nn_gumbel_z(hq, t0 + i0 + 8 * (r >> 2) + 4 * kh + (r & 3), a.itau);
      }
      if (MODE == 1 || MODE == 4) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {   // increasing r = increasing target index: '>' keeps the first
          const float v = z[r >> 1][r & 1];
          if (v > best) {
            best = v;
            besti = t0 + i0 + 8 * (r >> 2) + 4 * kh + (r & 3);
          }
        }
      } else if (MODE == 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {   // two best (smallest distance), first index on ties
          const float v = z[r >> 1][r & 1];
          const int i = t0 + i0 + 8 * (r >> 2) + 4 * kh + (r & 3);
          if (v > best) {
            second = best; secondi = besti;
            best = v; besti = i;
          } else if (v > second) {
            second = v; secondi = i;
          }
        }
      } else {
        float cm = nn_max3(z[0].x, z[0].y, z[1].x);
        cm = nn_max3(cm, z[1].y, z[2].x);
        cm = nn_max3(cm, z[2].y, z[3].x);
        cm = nn_max3(cm, z[3].y, z[4].x);
        cm = nn_max3(cm, z[4].y, z[5].x);
        cm = nn_max3(cm, z[5].y, z[6].x);
        cm = nn_max3(cm, z[6].y, z[7].x);
        cm = __builtin_fmaxf(cm, z[7].y);
        cm = __builtin_fmaxf(cm, __shfl_xor(cm, 32, 64));
        const float nm = __builtin_fmaxf(run_m, cm);
        const float sc = __builtin_amdgcn_exp2f(run_m - nm);   // 1 unless the maximum moved
        s2 *= sc; ax2 *= sc; ay2 *= sc; az2 *= sc;
        run_m = nm;
        const f32x2 nm2 = {nm, nm};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int il = i0 + 8 * g + 4 * kh;
          const float4 X = *reinterpret_cast<const float4*>(&Xs[cur][0][il]);
          const float4 Y = *reinterpret_cast<const float4*>(&Xs[cur][1][il]);
          const float4 Z = *reinterpret_cast<const float4*>(&Xs[cur][2][il]);
          const f32x2 d0 = z[2 * g] - nm2, d1 = z[2 * g + 1] - nm2;
          const f32x2 p0 = {__builtin_amdgcn_exp2f(d0.x), __builtin_amdgcn_exp2f(d0.y)};
          const f32x2 p1 = {__builtin_amdgcn_exp2f(d1.x), __builtin_amdgcn_exp2f(d1.y)};
          s2 += p0 + p1;
          ax2 = __builtin_elementwise_fma(p0, (f32x2){X.x, X.y}, ax2);
          ax2 = __builtin_elementwise_fma(p1, (f32x2){X.z, X.w}, ax2);
          ay2 = __builtin_elementwise_fma(p0, (f32x2){Y.x, Y.y}, ay2);
          ay2 = __builtin_elementwise_fma(p1, (f32x2){Y.z, Y.w}, ay2);
          az2 = __builtin_elementwise_fma(p0, (f32x2){Z.x, Z.y}, az2);
          az2 = __builtin_elementwise_fma(p1, (f32x2){Z.z, Z.w}, az2);
        }
      }
    };
    floatx16 acc = mfma_chunk(0);
#pragma unroll 1
    for (int i0 = 0; i0 < NN_STAGE - 32; i0 += 32) {
      const floatx16 nxt = mfma_chunk(i0 + 32);
      consume(acc, i0);
      acc = nxt;
    }
    consume(acc, NN_STAGE - 32);
    if (st + 1 < nst) store_lds(cur ^ 1, t0 + NN_STAGE);   // buffer last read in stage st-1
    __syncthreads();
    cur ^= 1;
  }

  if (MODE == 2) {   // merge the two lane halves' disjoint candidate sets
    const float ob = __shfl_xor(best, 32, 64), os = __shfl_xor(second, 32, 64);
    const int oi = __shfl_xor(besti, 32, 64), osi = __shfl_xor(secondi, 32, 64);
    auto better = [](float v, int i, float w, int k) { return v > w || (v == w && i < k); };
    float v1 = best, v2 = second;
    int i1 = besti, i2 = secondi;
    if (better(ob, oi, v1, i1)) {
      // other's best leads: second is the better of (mine best, other's second)
      if (better(v1, i1, os, osi)) { v2 = v1; i2 = i1; } else { v2 = os; i2 = osi; }
      v1 = ob; i1 = oi;
    } else if (better(ob, oi, v2, i2)) {
      v2 = ob; i2 = oi;
    }
    if (jok && kh == 0) {
      a.idx[((int64_t)p * a.Nq + j) * 2] = i1;
      a.idx[((int64_t)p * a.Nq + j) * 2 + 1] = i2;
    }
    return;
  }
  (void)Fp;
  float ox, oy, oz;
  if (MODE == 0 || MODE == 3) {
    const float run_s = s2.x + s2.y, ax = ax2.x + ax2.y, ay = ay2.x + ay2.y, az = az2.x + az2.y;
    const float s = run_s + __shfl_xor(run_s, 32, 64);
    ox = (ax + __shfl_xor(ax, 32, 64)) / s;
    oy = (ay + __shfl_xor(ay, 32, 64)) / s;
    oz = (az + __shfl_xor(az, 32, 64)) / s;
  } else {
    const float ob = __shfl_xor(best, 32, 64);
    const int oi = __shfl_xor(besti, 32, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
    const float* xp = Xt + (int64_t)(besti < Mt ? besti : 0) * 3;
    ox = xp[0]; oy = xp[1]; oz = xp[2];
  }
  if (jok && kh == 0) {
    float* o = a.out + (int64_t)p * a.o_ps + (int64_t)j * a.o_ns;
    if (a.Xq) {
      const float* xq = a.Xq + src * a.xq_fs + (int64_t)j * 3;
      o[0] = xq[0]; o[1] = xq[1]; o[2] = xq[2];
      o += 3;
    }
    o[0] = ox; o[1] = oy; o[2] = oz;
    if (a.idx && (MODE == 1 || MODE == 4)) a.idx[(int64_t)p * a.Nq + j] = besti;
  }
}


// Fast soft path.  Two changes against the online path:
//  * the softmax shift is the per-query bound k2 |fs|^2 instead of a running maximum: the
//    accumulator starts at -|fs|^2 / 2, so logit = 2 k2 acc - k2 |ft|^2 = -k2 |fs - ft|^2 <= 0 (log2
//    units) — exp2 never overflows, no maximum is tracked, nothing is rescaled.  Valid while a query's
//    softmax sum stays >= 2^-60 (its nearest target within sqrt(60 / k2) in feature space; unit-norm
//    descriptors at tau = 0.3 always are); the kernel re-runs a workgroup on the online path otherwise;
//  * S = Fs . Ft^T with the TARGET as the lane column: a lane's 16 accumulator registers are 16
//    queries against one target, so the target's (x, y, z, k2 |ft|^2) is one LDS read per 32-target
//    chunk, and each lane keeps per-query partial sums over the targets it saw (4 x 16 registers),
//    reduced across the 32 lanes once at the end.
// Per (query, target): one fma, one exp2, one add, three fmas.
// H = 0: the distance MFMAs on three-term split-bf16 (6 per k-step); H = 1: on two-term split-fp16 of the
// features scaled by 2^8 (3 per k-step; the accumulator is in 2^16 units, undone in the logit's fma).  H = 1
// needs |f|^2 < 2^14 for every query and target (|f_i| < 2^7: in range); a workgroup that sees a larger norm
// falls back to the online path like an underflowed one.  Unit-norm descriptors: |f_i| <= 1, so the
// absolute floor of the low term (2^-25 of the scaled value) is 2^-33 of a component.
template <int H>
__device__ __forceinline__ bool feat_nn_fast(const NNArgs& a, NNSmem& sm) {
  auto& Fp = sm.Fp;
  auto& Xf = sm.Xf;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;
  int p, qb;
  nn_block(p, qb);
  const int64_t src = a.pairs[2 * p], tgt = a.pairs[2 * p + 1];
  const float* Fq = a.Fq + src * a.fq_fs;
  const float* Ft = a.Ft + tgt * a.ft_fs;
  const float* Xt = a.Xt + tgt * a.xt_fs;
  const int q0 = qb * 128 + wid * 32;   // this wave's 32 queries
  const int Mt = a.Mt;

  // queries = A operand rows: lane row l32, dims 16s + 8kh + (0..7)
  bf16x8 qh[2], qm[2], ql[2];
  f16x8 q16h[2], q16l[2];
  float q2 = 0.f;
  {
    const int jq = q0 + l32;
    const float4* qp = reinterpret_cast<const float4*>(Fq + (int64_t)(jq < a.Nq ? jq : 0) * 32);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float4 u = qp[v];
      q2 += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 Hh, Mm, L;
      if (H) {
        nn_split8h(qp[4 * s + 2 * kh], qp[4 * s + 2 * kh + 1], Hh, L);
        q16h[s] = __builtin_bit_cast(f16x8, Hh);
        q16l[s] = __builtin_bit_cast(f16x8, L);
      } else {   // the logit's scale 2 k2 folded into the query operand
        const float kq = 2.f * a.k2;
        const float4 u0 = qp[4 * s + 2 * kh], u1 = qp[4 * s + 2 * kh + 1];
        nn_split8(make_float4(u0.x * kq, u0.y * kq, u0.z * kq, u0.w * kq),
                  make_float4(u1.x * kq, u1.y * kq, u1.z * kq, u1.w * kq), Hh, Mm, L);
        qh[s] = __builtin_bit_cast(bf16x8, Hh);
        qm[s] = __builtin_bit_cast(bf16x8, Mm);
        ql[s] = __builtin_bit_cast(bf16x8, L);
      }
    }
  }
  constexpr float ACC_UNIT = H ? 65536.f : 1.f;   // accumulator units (2^8 x 2^8 with H = 1)
  bool bad = H && !(q2 < 16384.f);                 // H = 1 range (NaN included)
  // accumulator register r holds query row 8 (r >> 2) + 4 kh + (r & 3): its start value -|fs|^2 / 2 (H = 1), or
  // -k2 |fs|^2 (split-bf16: the accumulator is the logit itself, 2 k2 fs.ft - k2 |fs|^2 - k2 |ft|^2, the last term
  // from the ones MFMA below)
  floatx16 init;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    init[r] = (H ? -0.5f * ACC_UNIT : -a.k2) * __shfl(q2, 8 * (r >> 2) + 4 * kh + (r & 3), 64);
  // the ones operand: k-slots 0, 1 of the low lane half and slot 8 of the high one (the target's h, m | l words)
  const bf16x8 ones = __builtin_bit_cast(bf16x8, (u32x4){kh ? 0x3F80u : 0x3F803F80u, 0u, 0u, 0u});

  const int srow = tid / NN_TPR, spart = tid % NN_TPR;
  float4 fr[NN_FPT / 4];
  float xr0 = 0.f, xr1 = 0.f, xr2 = 0.f;
  auto load_regs = [&](int t0) {
    const int gi = t0 + srow;
    const float4* fp = reinterpret_cast<const float4*>(Ft + (int64_t)(gi < Mt ? gi : 0) * 32 + NN_FPT * spart);
#pragma unroll
    for (int v = 0; v < NN_FPT / 4; ++v) fr[v] = gi < Mt ? fp[v] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < NN_STAGE) {
      const int gc = t0 + tid;
      if (gc < Mt) {
        const float* xp = Xt + (int64_t)gc * 3;
        xr0 = xp[0]; xr1 = xp[1]; xr2 = xp[2];
      }
    }
  };
  auto store_lds = [&](int buf, int t0) {
#pragma unroll
    for (int g = 0; g < NN_FPT / 8; ++g) {
      u32x4 Hh, Mm, L;
      const int c = 8 * (((NN_FPT / 8) * spart + g) ^ ((srow >> 2) & 3));
      if (H) {
        nn_split8h(fr[2 * g], fr[2 * g + 1], Hh, L);
        *reinterpret_cast<u32x4*>(&Fp[buf][0][srow][c]) = Hh;
        *reinterpret_cast<u32x4*>(&Fp[buf][1][srow][c]) = L;
      } else {
        nn_split8(fr[2 * g], fr[2 * g + 1], Hh, Mm, L);
        *reinterpret_cast<u32x4*>(&Fp[buf][0][srow][c]) = Hh;
        *reinterpret_cast<u32x4*>(&Fp[buf][1][srow][c]) = Mm;
        *reinterpret_cast<u32x4*>(&Fp[buf][2][srow][c]) = L;
      }
    }
    static_assert(NN_FPT == 16, "nn_norm16");
    float n2 = nn_norm16(fr);
#pragma unroll
    for (int o = 1; o < NN_TPR; o <<= 1) n2 += __shfl_xor(n2, o, 64);
    if (H) bad |= !(n2 < 16384.f);   // rows past Mt are zeros
    if (tid < NN_STAGE) {
      Xf[buf][tid].x = xr0;
      Xf[buf][tid].y = xr1;
      Xf[buf][tid].z = xr2;
    }
    // invalid targets: +inf -> logit -inf -> weight 0 (their coordinates stay finite)
    if (spart == 0) {
      if (H) {
        Xf[buf][srow].w = (t0 + srow < Mt) ? n2 * a.k2 : __builtin_inff();
      } else {
        unsigned hm, wl;
        nn_wsplit(n2 * a.k2, t0 + srow < Mt, hm, wl);
        Xf[buf][srow].w = __uint_as_float(hm);
        sm.Wl[buf][srow] = wl;
      }
    }
  };

  // pre-split image: stage st -> buffer buf by LDS-DMA (each wave copies its 1 KB slices; completion awaited before
  // the barrier that publishes the buffer)
  const bool dma = !H && a.timg;
  const char* timg = dma ? a.timg + tgt * a.timg_fs : nullptr;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  auto dma_stage = [&](int buf, int st) {
    const char* src = timg + (int64_t)st * NN_IMG_STAGE;
    const uint32_t fp = lds_addr(&Fp[buf][0][0][0]), xf = lds_addr(&Xf[buf][0]);
#pragma unroll
    for (int i = 0; i < NN_IMG_PLANES / 4096; ++i)
      glds16s(src, (uint32_t)(i * 4096 + wu * 1024 + lane * 16), fp + (uint32_t)(i * 4096 + wu * 1024));
    if (wu < NN_STAGE * 16 / 1024)
      glds16s(src, (uint32_t)(NN_IMG_PLANES + wu * 1024 + lane * 16), xf + (uint32_t)(wu * 1024));
    static_assert(NN_STAGE * 4 == 512 && NN_STAGE * 16 / 1024 == 2, "the w l words: half a DMA of wave 2");
    if (wu == 2 && lane < 32)
      glds16s(src, (uint32_t)(NN_IMG_PLANES + NN_STAGE * 16 + lane * 16), lds_addr(&sm.Wl[buf][0]));
  };

  float S[16], AX[16], AY[16], AZ[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) S[r] = AX[r] = AY[r] = AZ[r] = 0.f;
  const float kk2 = 2.f * a.k2 / ACC_UNIT;
  const int nst = (Mt + NN_STAGE - 1) / NN_STAGE;
  if (dma) {
    dma_stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load_regs(0);
    store_lds(0, 0);
  }
  __syncthreads();
  int cur = 0;
  auto mfma_chunk = [&](int i0) {
    floatx16 acc = init;
    const int row = i0 + l32;
    if (!H) {   // -k2 |ft|^2 of target row (h + m in the low lane half, l in the high one)
      const unsigned wv = kh ? sm.Wl[cur][row] : __float_as_uint(Xf[cur][row].w);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, __builtin_bit_cast(bf16x8, (u32x4){wv, 0u, 0u, 0u}), acc, 0,
                                                    0, 0);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 8 * ((2 * s + kh) ^ ((row >> 2) & 3));
      if (H) {
        const f16x8 th = *reinterpret_cast<const f16x8*>(&Fp[cur][0][row][c]);
        const f16x8 tl = *reinterpret_cast<const f16x8*>(&Fp[cur][1][row][c]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(q16l[s], th, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(q16h[s], tl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(q16h[s], th, acc, 0, 0, 0);
        continue;
      }
      const bf16x8 th = *reinterpret_cast<const bf16x8*>(&Fp[cur][0][row][c]);
      const bf16x8 tm = *reinterpret_cast<const bf16x8*>(&Fp[cur][1][row][c]);
      const bf16x8 tl = *reinterpret_cast<const bf16x8*>(&Fp[cur][2][row][c]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql[s], th, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh[s], tl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm[s], tm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh[s], tm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm[s], th, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh[s], th, acc, 0, 0, 0);
    }
    return acc;
  };
  // acc[r] = fs[query row(r)] . ft[i0 + l32] - |fs|^2 / 2
  auto consume = [&](const floatx16& acc, int i0) {
    const float4 X = Xf[cur][i0 + l32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pw = __builtin_amdgcn_exp2f(H ? fmaf(acc[r], kk2, -X.w) : acc[r]);
      S[r] += pw;
      AX[r] = fmaf(pw, X.x, AX[r]);
      AY[r] = fmaf(pw, X.y, AY[r]);
      AZ[r] = fmaf(pw, X.z, AZ[r]);
    }
  };
  for (int st = 0; st < nst; ++st) {
    const int t0 = st * NN_STAGE;
    if (st + 1 < nst) {
      if (dma) dma_stage(cur ^ 1, st + 1);   // buffer last read in stage st - 1
      else load_regs(t0 + NN_STAGE);
    }
    floatx16 acc = mfma_chunk(0);
#pragma unroll 1
    for (int i0 = 0; i0 < NN_STAGE - 32; i0 += 32) {
      const floatx16 nxt = mfma_chunk(i0 + 32);
      consume(acc, i0);
      acc = nxt;
    }
    consume(acc, NN_STAGE - 32);
    if (st + 1 < nst) {
      if (dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else store_lds(cur ^ 1, t0 + NN_STAGE);
    }
    __syncthreads();
    cur ^= 1;
  }
  // reduce the per-lane partial sums over the 32 targets-lanes of each half
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      S[r] += __shfl_xor(S[r], o, 64);
      AX[r] += __shfl_xor(AX[r], o, 64);
      AY[r] += __shfl_xor(AY[r], o, 64);
      AZ[r] += __shfl_xor(AZ[r], o, 64);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int jq = q0 + 8 * (r >> 2) + 4 * kh + (r & 3);
    bad |= jq < a.Nq && !(S[r] >= 0x1p-60f);   // underflowed (or non-finite) softmax sum
  }
  if (tid == 0) sm.flag = 0;
  __syncthreads();
  if (bad) sm.flag = 1;
  __syncthreads();
  if (sm.flag) return false;
  // lane l32 = r of each half writes register r's query
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int jq = q0 + 8 * (r >> 2) + 4 * kh + (r & 3);
    if (l32 == r && jq < a.Nq) {
      float* o = a.out + (int64_t)p * a.o_ps + (int64_t)jq * a.o_ns;
      if (a.Xq) {
        const float* xq = a.Xq + src * a.xq_fs + (int64_t)jq * 3;
        o[0] = xq[0]; o[1] = xq[1]; o[2] = xq[2];
        o += 3;
      }
      o[0] = AX[r] / S[r]; o[1] = AY[r] / S[r]; o[2] = AZ[r] / S[r];
    }
  }
  return true;
}

// two threads per (fragment, padded target row), 16 dims each — the split and the norm in exactly store_lds's
// order (bit-identical stages): the row's three bf16 planes (swizzled as the LDS stage) and, from the first thread,
// (x, y, z, k2 |ft|^2) (+inf past Mt: weight 0)
__global__ void nn_presplit_kernel(const float* __restrict__ Ft, int64_t ft_fs, const float* __restrict__ Xt,
                                   int64_t xt_fs, int nfrag, int Mt, int nst, float k2, char* img, int64_t img_fs) {
  static_assert(NN_TPR == 2 && NN_FPT == 16, "presplit mirrors the 2-threads-per-row stage");
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int spart = (int)(e & 1);
  const int64_t rr = e >> 1;
  const int rows = nst * NN_STAGE;
  const bool in = rr < (int64_t)nfrag * rows;   // (whole shuffle pairs stay active)
  const int f = in ? (int)(rr / rows) : 0, r = in ? (int)(rr - (int64_t)f * rows) : 0;
  const int st = r / NN_STAGE, srow = r - st * NN_STAGE;
  const bool ok = in && r < Mt;
  float4 fr[4];
  const float4* fp = reinterpret_cast<const float4*>(Ft + f * ft_fs + (int64_t)(ok ? r : 0) * 32 + NN_FPT * spart);
#pragma unroll
  for (int v = 0; v < 4; ++v) fr[v] = ok ? fp[v] : make_float4(0.f, 0.f, 0.f, 0.f);
  char* base = img + f * img_fs + (int64_t)st * NN_IMG_STAGE;
  constexpr int plane = NN_STAGE * NN_ROW * 2;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    u32x4 H, Mm, L;
    nn_split8(fr[2 * g], fr[2 * g + 1], H, Mm, L);
    const int c = 8 * ((2 * spart + g) ^ ((srow >> 2) & 3));
    if (in) {
      *reinterpret_cast<u32x4*>(base + (srow * NN_ROW + c) * 2) = H;
      *reinterpret_cast<u32x4*>(base + plane + (srow * NN_ROW + c) * 2) = Mm;
      *reinterpret_cast<u32x4*>(base + 2 * plane + (srow * NN_ROW + c) * 2) = L;
    }
  }
  float n2 = nn_norm16(fr);
  n2 += __shfl_xor(n2, 1, 64);
  if (in && spart == 0) {
    unsigned hm, wl;
    nn_wsplit(n2 * k2, ok, hm, wl);
    float4 x = make_float4(0.f, 0.f, 0.f, __uint_as_float(hm));
    if (ok) {
      const float* xp = Xt + f * xt_fs + (int64_t)r * 3;
      x = make_float4(xp[0], xp[1], xp[2], __uint_as_float(hm));
    }
    *reinterpret_cast<float4*>(base + NN_IMG_PLANES + srow * 16) = x;
    *reinterpret_cast<unsigned*>(base + NN_IMG_PLANES + NN_STAGE * 16 + srow * 4) = wl;
  }
}

int g_feat_nn_fast = 1;   // knobs.hpp: 0 online path only, 1 fast path split-bf16 (default), 2 fast path split-fp16

// MODE 0 (soft) with a.fast: the bounded-shift path, falling back to the online path for a workgroup
// whose softmax sums underflowed; otherwise the online path (MODE 1 argmax, 2 two nearest).
template <int MODE>
#ifndef NN_OCC
#define NN_OCC 2
#endif
__global__ __launch_bounds__(256, MODE == 0 ? NN_OCC : 3) void feat_nn_kernel(NNArgs a) {
  __shared__ __attribute__((aligned(16))) NNSmem sm;
  if (MODE == 0 && a.fast) {
    if (a.fast == 2 ? feat_nn_fast<1>(a, sm) : feat_nn_fast<0>(a, sm)) return;
    __syncthreads();
  }
  feat_nn_online<MODE>(a, sm);
}

// exact fp64 distances of the two neighbours: d[p][j][k] = |Fq(src, j) - Ft(tgt, idx[p][j][k])|
__global__ void knn2_dist_kernel(const float* __restrict__ Fq, int64_t fq_fs, const float* __restrict__ Ft,
                                 int64_t ft_fs, const int64_t* __restrict__ pairs, int P, int Nq, int Mt,
                                 const int32_t* __restrict__ idx, double* dist) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)P * Nq * 2) return;
  const int64_t pj = e >> 1;
  const int p = (int)(pj / Nq), j = (int)(pj - (int64_t)p * Nq);
  const int t = idx[e];
  if (t < 0 || t >= Mt) { dist[e] = __builtin_inf(); return; }
  const float* q = Fq + pairs[2 * p] * fq_fs + (int64_t)j * 32;
  const float* f = Ft + pairs[2 * p + 1] * ft_fs + (int64_t)t * 32;
  double s = 0.0;
  for (int c = 0; c < 32; ++c) {
    const double d = (double)q[c] - (double)f[c];
    s += d * d;
  }
  dist[e] = sqrt(s);
}

// rows gather: dst[i][:] = src[idx[i]][:]  (Sampler.forward, lib/layers.py:151-152)
__global__ void gather_rows_kernel(const float* __restrict__ src, int C, const int64_t* __restrict__ idx, int n,
                                   float* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * C) return;
  const int64_t i = e / C, c = e - i * C;
  dst[e] = src[idx[i] * C + c];
}

}  // namespace mvr

static int64_t nn_img_fs(int Mt) { return (int64_t)((Mt + mvr::NN_STAGE - 1) / mvr::NN_STAGE) * mvr::NN_IMG_STAGE; }

extern "C" size_t mvr_feat_nn_workspace_bytes(int n_frag, int Mt) {
  if (n_frag <= 0 || Mt <= 0) return 0;
  return (size_t)n_frag * nn_img_fs(Mt);
}

extern "C" int mvr_feat_nn_ws(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride,
                              const float* Xq, int64_t xq_fstride, const float* Xt, int64_t xt_fstride,
                              const int64_t* pairs, int P, int Nq, int Mt, int C, float inv_tau2, int mode, float* out,
                              int64_t out_pstride, int64_t out_nstride, int32_t* idx_out, int n_frag, void* workspace,
                              size_t workspace_bytes, hipStream_t stream);

extern "C" int mvr_feat_nn(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride, const float* Xq,
                           int64_t xq_fstride, const float* Xt, int64_t xt_fstride, const int64_t* pairs, int P,
                           int Nq, int Mt, int C, float inv_tau2, int mode, float* out, int64_t out_pstride,
                           int64_t out_nstride, int32_t* idx_out, hipStream_t stream) {
  return mvr_feat_nn_ws(Fq, fq_fstride, Ft, ft_fstride, Xq, xq_fstride, Xt, xt_fstride, pairs, P, Nq, Mt, C, inv_tau2,
                        mode, out, out_pstride, out_nstride, idx_out, 0, nullptr, 0, stream);
}

extern "C" int mvr_feat_nn_ws(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride,
                              const float* Xq, int64_t xq_fstride, const float* Xt, int64_t xt_fstride,
                              const int64_t* pairs, int P, int Nq, int Mt, int C, float inv_tau2, int mode, float* out,
                              int64_t out_pstride, int64_t out_nstride, int32_t* idx_out, int n_frag, void* workspace,
                              size_t workspace_bytes, hipStream_t stream) {
  if (P < 0 || Nq < 0 || Mt <= 0 || C != 32 || (mode != 0 && mode != 1)) return MVR_EINVAL;
  if (P == 0 || Nq == 0) return MVR_OK;   // empty batch: NULL pointers allowed (mvreg.h conventions)
  if (!Fq || !Ft || !Xt || !pairs || !out) return MVR_EINVAL;
  if (workspace && (n_frag <= 0 || workspace_bytes < mvr_feat_nn_workspace_bytes(n_frag, Mt) ||
                    (reinterpret_cast<uintptr_t>(workspace) & 15)))
    return MVR_EINVAL;
  if (C != 32) return MVR_EINVAL;  // FCGF descriptor width (fcgf.py:108 out_channels=32)
  if ((reinterpret_cast<uintptr_t>(Fq) & 15) || (reinterpret_cast<uintptr_t>(Ft) & 15) || (fq_fstride & 3) ||
      (ft_fstride & 3))
    return MVR_EINVAL;
  mvr::NNArgs a{Fq, fq_fstride, Ft, ft_fstride, Xq, xq_fstride, Xt, xt_fstride, pairs, P, Nq, Mt,
                inv_tau2 * 1.4426950408889634f, mode, out, out_pstride, out_nstride, idx_out, mvr::g_feat_nn_fast,
                nullptr, 0};
  // the split-bf16 fast path stages its targets from a pre-split image when the caller gives the workspace (the
  // pair list's target fragments must be < n_frag)
  if (workspace && mode == 0 && mvr::g_feat_nn_fast == 1) {
    const int nst = (Mt + mvr::NN_STAGE - 1) / mvr::NN_STAGE;
    const int64_t n = (int64_t)n_frag * nst * mvr::NN_STAGE * 2;
    hipLaunchKernelGGL(mvr::nn_presplit_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, Ft, ft_fstride,
                       Xt, xt_fstride, n_frag, Mt, nst, a.k2, reinterpret_cast<char*>(workspace), nn_img_fs(Mt));
    MVR_CHECK_LAUNCH();
    a.timg = reinterpret_cast<const char*>(workspace);
    a.timg_fs = nn_img_fs(Mt);
  }
  mvr::ProfScope prof(mvr::PK_FEAT_NN, 2.0 * P * (double)Nq * Mt * C, (double)P * (Nq + Mt) * (C + 3) * 4 + P * Nq * 24.0,
                      stream);
  const dim3 grid((Nq + 127) / 128, P);
  if (mode == 0)
    hipLaunchKernelGGL(mvr::feat_nn_kernel<0>, grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(mvr::feat_nn_kernel<1>, grid, dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

// soft_gumbel (lib/layers.py:72-78): the online path with counter-based Gumbel noise (nn_gumbel_z), hard = 0 the
// soft weights, 1 the straight-through forward value (the one-hot of the noisy argmax).  Same layouts as mvr_feat_nn.
extern "C" int mvr_feat_nn_gumbel(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride,
                                  const float* Xq, int64_t xq_fstride, const float* Xt, int64_t xt_fstride,
                                  const int64_t* pairs, int P, int Nq, int Mt, int C, float inv_tau, int hard,
                                  uint64_t seed, float* out, int64_t out_pstride, int64_t out_nstride, int32_t* idx_out,
                                  hipStream_t stream) {
  if (P < 0 || Nq < 0 || Mt <= 0 || C != 32 || (hard != 0 && hard != 1) || !(inv_tau > 0.f)) return MVR_EINVAL;
  if (P == 0 || Nq == 0) return MVR_OK;
  if (!Fq || !Ft || !Xt || !pairs || !out) return MVR_EINVAL;
  if ((reinterpret_cast<uintptr_t>(Fq) & 15) || (reinterpret_cast<uintptr_t>(Ft) & 15) || (fq_fstride & 3) ||
      (ft_fstride & 3))
    return MVR_EINVAL;
  mvr::NNArgs a{Fq, fq_fstride, Ft, ft_fstride, Xq, xq_fstride, Xt, xt_fstride, pairs, P, Nq, Mt,
                inv_tau * 1.4426950408889634f, hard ? 4 : 3, out, out_pstride, out_nstride, idx_out, 0, nullptr, 0,
                (unsigned)seed, (unsigned)(seed >> 32), inv_tau};
  mvr::ProfScope prof(mvr::PK_FEAT_NN, 2.0 * P * (double)Nq * Mt * C, (double)P * (Nq + Mt) * (C + 3) * 4 + P * Nq * 24.0,
                      stream);
  const dim3 grid((Nq + 127) / 128, P);
  if (hard)
    hipLaunchKernelGGL(mvr::feat_nn_kernel<4>, grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(mvr::feat_nn_kernel<3>, grid, dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_feat_knn2(const float* Fq, int64_t fq_fstride, const float* Ft, int64_t ft_fstride,
                             const int64_t* pairs, int P, int Nq, int Mt, int C, int32_t* idx2_out, double* dist2_out,
                             hipStream_t stream) {
  if (P < 0 || Nq < 0 || Mt < 2 || C != 32) return MVR_EINVAL;
  if (P == 0 || Nq == 0) return MVR_OK;
  if (!Fq || !Ft || !pairs || !idx2_out) return MVR_EINVAL;
  if ((reinterpret_cast<uintptr_t>(Fq) & 15) || (reinterpret_cast<uintptr_t>(Ft) & 15) || (fq_fstride & 3) ||
      (ft_fstride & 3))
    return MVR_EINVAL;
  mvr::NNArgs a{Fq, fq_fstride, Ft, ft_fstride, nullptr, 0, Ft, 0, pairs, P, Nq, Mt, 1.4426950408889634f, 2,
                nullptr, 0, 0, idx2_out, 0, nullptr, 0};
  mvr::ProfScope prof(mvr::PK_FEAT_NN, 2.0 * P * (double)Nq * Mt * C, (double)P * (Nq + Mt) * C * 4 + P * Nq * 8.0,
                      stream);
  hipLaunchKernelGGL(mvr::feat_nn_kernel<2>, dim3((Nq + 127) / 128, P), dim3(256), 0, stream, a);
  MVR_CHECK_LAUNCH();
  if (dist2_out) {
    const int64_t n = (int64_t)P * Nq * 2;
    hipLaunchKernelGGL(mvr::knn2_dist_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, Fq, fq_fstride,
                       Ft, ft_fstride, pairs, P, Nq, Mt, idx2_out, dist2_out);
    MVR_CHECK_LAUNCH();
  }
  return MVR_OK;
}

extern "C" int mvr_gather_rows(const float* src, int C, const int64_t* idx, int n, float* dst, hipStream_t stream) {
  if (C <= 0 || n < 0) return MVR_EINVAL;
  if (n == 0) return MVR_OK;
  if (!src || !idx || !dst) return MVR_EINVAL;
  const int64_t tot = (int64_t)n * C;
  hipLaunchKernelGGL(mvr::gather_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, src, C, idx, n,
                     dst);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

