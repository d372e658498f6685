// Split-bf16 matrix-core helpers shared by the fused kernels (gfx950, v_mfma_f32_32x32x16_bf16).
//
// fp32 operands are split into three bf16 terms, x = h + m + l to 2^-25 |x| (RNE at each step;
// x - h and r - m are exact in fp32), and the products hh, hm, mh, mm, hl, lh are accumulated in
// fp32 — fp32-level accuracy (the dropped ml, lm, ll terms are <= 2^-23 relative), see gemm.hpp
// MATH_BF16X3.
//
// Operand maps of v_mfma_f32_32x32x16_bf16 (lane l, r = l & 31, h = l >> 5): A[row r][k = 8h + i],
// B[k = 8h + i][col r] in element i = 0..7; C[row (q & 3) + 8 (q >> 2) + 4h][col r] in register q.
// Registers 8s .. 8s+7 of a C tile are, as a B (or A) fragment of k-step s, its rows
// 16s + 8(i >> 2) + 4h + (i & 3): the other operand must supply that same k order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mvr {
namespace bx {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned cvt_pk(f32x2 x) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
}
__device__ __forceinline__ f32x2 unpack(unsigned p) {
  f32x2 r;
  r.x = __uint_as_float(p << 16);
  r.y = __uint_as_float(p & 0xffff0000u);
  return r;
}
// x - y of a pair.  MVR_PK_SPLIT 0: two v_sub_f32 instead of one v_pk_add_f32, which costs more issue than its two
// halves beside the MFMAs (MI355X_MICROARCH.md, per-instruction constants); the same RNE subtraction, bit-identical.
// (The files are built without the SLP vectorizer, which would pair them again.)
#ifndef MVR_PK_SPLIT
#define MVR_PK_SPLIT 1
#endif
__device__ __forceinline__ f32x2 sub2(f32x2 x, f32x2 y) {
#if MVR_PK_SPLIT
  return x - y;
#else
  f32x2 r;
  r.x = x.x - y.x;
  r.y = x.y - y.y;
  return r;
#endif
}
// two fp32 -> packed (h, m, l) bf16 pairs
__device__ __forceinline__ void split2(f32x2 x, unsigned& H, unsigned& M, unsigned& L) {
  H = cvt_pk(x);
  const f32x2 r = sub2(x, unpack(H));
  M = cvt_pk(r);
  L = cvt_pk(sub2(r, unpack(M)));
}
__device__ __forceinline__ void split4(const float4& a, u32x2& H, u32x2& M, u32x2& L) {
  unsigned h0, m0, l0, h1, m1, l1;
  split2(f32x2{a.x, a.y}, h0, m0, l0);
  split2(f32x2{a.z, a.w}, h1, m1, l1);
  H = u32x2{h0, h1};
  M = u32x2{m0, m1};
  L = u32x2{l0, l1};
}
__device__ __forceinline__ void split8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
  unsigned hh[4], mm[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split2(f32x2{v[2 * i], v[2 * i + 1]}, hh[i], mm[i], ll[i]);
  const u32x4 H{hh[0], hh[1], hh[2], hh[3]}, M{mm[0], mm[1], mm[2], mm[3]}, L{ll[0], ll[1], ll[2], ll[3]};
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}

struct Frag {
  bf16x8 h, m, l;
};

// acc += A . B over the six significant split products, small terms first
__device__ __forceinline__ floatx16 mfma6(const Frag& a, const Frag& b, floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
  return acc;
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, columns 4p..4p+3 of a 4x16
// block of 16-bit elements; lane i of the group receives column i (rows 0..3 in elements 0..3).
// EXEC must be all ones.
__device__ __forceinline__ u32x2 ds_read_tr(const char* lds) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_i16x4*)(const __attribute__((address_space(3))) char*)lds);
  return __builtin_bit_cast(u32x2, r);
}

// ---------------------------------------------------------------------------------------------
// Split-math generic forms.  H = 0: the three-term split-bf16 above (6 MFMAs per product); H = 1: two-term
// split-fp16, x = h + l, h = fp16(x), l = fp16(x - h) (RNE, x - h exact in fp32): 22 significant bits
// (2^-22 relative for |x| >= 2^-3, 2^-25 absolute below, overflow at 65504), products hh, hl, lh on
// v_mfma_f32_32x32x16_f16 (3 MFMAs).  Callers keep operands inside that window (see oan_attn.hip, pconv.hip).
// ---------------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
constexpr float F16_RANGE = 65504.f;

template <int H> struct FragT;
template <> struct FragT<0> { typedef bf16x8 V; V p[3]; };
template <> struct FragT<1> { typedef f16x8 V; V p[2]; };
template <int H> constexpr int planes() { return H ? 2 : 3; }

template <int H> __device__ __forceinline__ void split_pair(f32x2 x, unsigned* o);
template <> __device__ __forceinline__ void split_pair<0>(f32x2 x, unsigned* o) {
  o[0] = cvt_pk(x);
  const f32x2 r = sub2(x, unpack(o[0]));
  o[1] = cvt_pk(r);
  o[2] = cvt_pk(sub2(r, unpack(o[1])));
}
template <> __device__ __forceinline__ void split_pair<1>(f32x2 x, unsigned* o) {
  const f16x2 hh = __builtin_convertvector(x, f16x2);
  o[0] = __builtin_bit_cast(unsigned, hh);
  const f32x2 r = sub2(x, __builtin_convertvector(hh, f32x2));
  o[1] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, f16x2));
}
// 4 fp32 -> one u32x2 (4 packed 16-bit terms) per plane
template <int H> __device__ __forceinline__ void split4t(const float4& a, u32x2* o) {
  unsigned lo[3], hi[3];
  split_pair<H>(f32x2{a.x, a.y}, lo);
  split_pair<H>(f32x2{a.z, a.w}, hi);
#pragma unroll
  for (int i = 0; i < planes<H>(); ++i) o[i] = u32x2{lo[i], hi[i]};
}
template <int H> __device__ __forceinline__ FragT<H> split8t(const float* v) {
  unsigned t[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) split_pair<H>(f32x2{v[2 * i], v[2 * i + 1]}, t[i]);
  FragT<H> f;
#pragma unroll
  for (int pl = 0; pl < planes<H>(); ++pl)
    f.p[pl] = __builtin_bit_cast(typename FragT<H>::V, u32x4{t[0][pl], t[1][pl], t[2][pl], t[3][pl]});
  return f;
}
// acc += A . B, small terms first
template <int H> __device__ __forceinline__ floatx16 mma(const FragT<H>& a, const FragT<H>& b, floatx16 acc);
template <> __device__ __forceinline__ floatx16 mma<0>(const FragT<0>& a, const FragT<0>& b, floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
  return acc;
}
template <> __device__ __forceinline__ floatx16 mma<1>(const FragT<1>& a, const FragT<1>& b, floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.p[0], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.p[0], b.p[0], acc, 0, 0, 0);
  return acc;
}
// a fragment whose planes sit `ps` bytes apart
template <int H> __device__ __forceinline__ FragT<H> ld_frag(const char* p, int ps) {
  FragT<H> f;
#pragma unroll
  for (int pl = 0; pl < planes<H>(); ++pl) f.p[pl] = *reinterpret_cast<const typename FragT<H>::V*>(p + pl * ps);
  return f;
}
// the (h, m, l) split-bf16 planes of one value (split_pair<0>, element for element) at p, p + ld, p + 2 ld: a
// producer's epilogue writes them beside its fp32 output for the next sparse conv (spconv.hip PS = 1)
__device__ __forceinline__ void store_planes(uint16_t* p, int64_t ld, float v) {
  unsigned o[3];
  split_pair<0>(f32x2{v, 0.f}, o);
  p[0] = (uint16_t)o[0];
  p[ld] = (uint16_t)o[1];
  p[2 * ld] = (uint16_t)o[2];
}
// power-of-two scale bringing |x| <= amax to <= 2^14 (amax = 0: 2^14)
__device__ __forceinline__ float range_scale(float amax) {
  int e;
  (void)frexpf(amax, &e);   // amax < 2^e
  return ldexpf(1.f, min(max(14 - e, -64), 64));
}

}  // namespace bx
}  // namespace mvr
