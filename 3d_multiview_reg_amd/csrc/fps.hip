// Farthest point sampling per fragment (Sampler 'fps', lib/layers.py:128-141; pointnet2_ops
// furthest_point_sample semantics as fixed in oracle/fps.py: seed index 0, squared-Euclidean
// running minimum, first maximum on ties, no origin skip).
//
// m dependent steps per fragment, so one 1024-thread workgroup owns a fragment and keeps its
// points and running distances in registers (PER points per thread); each step is a local
// update + a block argmax (64-bit (distance bits, ~index) max: ties -> lowest index) through
// DPP/swizzle wave reductions and one LDS exchange.  Fragments run concurrently on separate CUs.
// Distances use explicitly rounded fp32 ops (no FMA contraction) so the indices match the
// oracle bit for bit.
#include "common.hpp"
#include "prof.hpp"

namespace mvr {


__device__ __forceinline__ uint64_t fps_key(float d, int i) {
  return ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)(~i);   // d >= 0: bit order = value order
}
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ float fps_d2(float px, float py, float pz, float lx, float ly, float lz) {
  const float dx = __fsub_rn(px, lx), dy = __fsub_rn(py, ly), dz = __fsub_rn(pz, lz);
  return __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
}

// FPS_T threads x PER points per thread; XYZ_REG: coordinates held in registers (4 VGPRs per
// point: 1024 threads up to 16 points, 512 threads up to 48), else re-read from L2 each step.
template <int FPS_T, int PER, bool XYZ_REG>
__global__ __launch_bounds__(FPS_T) void fps_kernel(const float* __restrict__ xyz, const int64_t* __restrict__ off,
                                                    int m, int64_t* __restrict__ idx_out) {
  __shared__ uint64_t wbest[FPS_T / 64];
  __shared__ float last[3];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t s0 = off[f];
  const int n = (int)(off[f + 1] - s0);
  const float* p = xyz + s0 * 3;
  float px[XYZ_REG ? PER : 1], py[XYZ_REG ? PER : 1], pz[XYZ_REG ? PER : 1], d[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int k = tid + j * FPS_T;
    const bool ok = k < n;
    if (XYZ_REG) {
      px[j] = ok ? p[3 * k] : 0.f;
      py[j] = ok ? p[3 * k + 1] : 0.f;
      pz[j] = ok ? p[3 * k + 2] : 0.f;
    }
    d[j] = ok ? __builtin_inff() : -1.f;   // absent points never win
  }
  int64_t* out = idx_out + (int64_t)f * m;
  if (tid == 0) {
    out[0] = s0;
    last[0] = p[0]; last[1] = p[1]; last[2] = p[2];
  }
  __syncthreads();
  for (int it = 1; it < m; ++it) {
    const float lx = last[0], ly = last[1], lz = last[2];
    uint64_t best = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (!XYZ_REG && (j & 7) == 0) asm volatile("" ::: "memory");   // bound the loads in flight (VGPRs)
      if (d[j] >= 0.f) {
        const int k = tid + j * FPS_T;
        const float qx = XYZ_REG ? px[j] : p[3 * k], qy = XYZ_REG ? py[j] : p[3 * k + 1],
                    qz = XYZ_REG ? pz[j] : p[3 * k + 2];
        d[j] = fminf(d[j], fps_d2(qx, qy, qz, lx, ly, lz));
        best = umax64(best, fps_key(d[j], tid + j * FPS_T));
      }
    }
#pragma unroll
    for (int msk = 32; msk >= 1; msk >>= 1) best = umax64(best, shfl_xor64(best, msk));
    if (lane == 0) wbest[wid] = best;
    __syncthreads();   // also: every thread has read last[] of this step
    if (wid == 0) {
      uint64_t b = lane < FPS_T / 64 ? wbest[lane] : 0;
#pragma unroll
      for (int msk = FPS_T / 128; msk >= 1; msk >>= 1) b = umax64(b, shfl_xor64(b, msk));
      if (lane == 0) {
        const int k = (int)(~(uint32_t)b);
        out[it] = s0 + k;
        last[0] = p[3 * k]; last[1] = p[3 * k + 1]; last[2] = p[3 * k + 2];
      }
    }
    __syncthreads();
  }
}

// One-barrier form for fragments of up to 1024 * PER points, all held in registers (4 VGPRs per point).
// Step: every thread updates its points' running minimum and keeps its own best (first maximum in its index
// order: strict '>' over ascending j, so the lowest index among equal distances); each wave finds its best by a
// float max (DPP within rows, lane reads across them) and, only when several lanes tie on it, a min over their
// indices; the winning lane writes (d, index, coordinates) of its point to its wave's slot; ONE barrier; every
// thread then reads the 16 slots and picks the block's best (ties -> lowest index) with its coordinates, so the
// next step starts without a global load on the critical path.  Slots alternate by step parity (a wave can only
// reach step i + 2's writes after every wave passed step i + 1's barrier, i.e. finished reading step i's slots).
// Same arithmetic and tie rule as fps_kernel (explicitly rounded fp32 distances): identical indices.
__device__ __forceinline__ float row_max16(float v) {   // max over the 16 lanes of a DPP row, in every lane
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true)));    // quad 1,0,3,2
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true)));    // quad 2,3,0,1
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true)));   // half mirror
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, true)));   // row mirror
  return v;
}
__device__ __forceinline__ float wave_max_uniform(float v) {
  v = row_max16(v);
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(a, b), fmaxf(c, d));
}

struct FpsSlot {
  float d, x, y, z;
  int k, pad0, pad1, pad2;
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

// squared distances of two points at once on packed fp32 (v_pk_add_f32 / v_pk_mul_f32: two lanes of IEEE
// round-to-nearest arithmetic per instruction; contraction off, so each op rounds exactly like fps_d2's)
__device__ __forceinline__ f32x2 fps_d2x2(f32x2 px, f32x2 py, f32x2 pz, f32x2 lx, f32x2 ly, f32x2 lz) {
#pragma clang fp contract(off)
  const f32x2 dx = px - lx, dy = py - ly, dz = pz - lz;
  return (dx * dx + dy * dy) + dz * dz;
}

template <int T, int PER>
__global__ __launch_bounds__(T) void fps_reg_kernel(const float* __restrict__ xyz, const int64_t* __restrict__ off,
                                                    int m, int64_t* __restrict__ idx_out) {
  static_assert(PER % 2 == 0, "points are processed in pairs");
  constexpr int NW = T / 64, P2 = PER / 2;
  static_assert(NW <= 16, "the slot reduction runs in one DPP row");
  __shared__ FpsSlot slot[2][NW];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t s0 = off[f];
  const int n = (int)(off[f + 1] - s0);
  const float* p = xyz + s0 * 3;
  // point j of this thread: index tid + j T, held in pair j / 2, component j % 2
  f32x2 px[P2], py[P2], pz[P2], d[P2];
#pragma unroll
  for (int j2 = 0; j2 < P2; ++j2) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int k = tid + (2 * j2 + e) * T;
      const bool ok = k < n;
      px[j2][e] = ok ? p[3 * k] : 0.f;
      py[j2][e] = ok ? p[3 * k + 1] : 0.f;
      pz[j2][e] = ok ? p[3 * k + 2] : 0.f;
      d[j2][e] = ok ? __builtin_inff() : -1.f;   // absent points: min(-1, distance) stays -1, never the best
    }
  }
  int64_t* out = idx_out + (int64_t)f * m;
  if (tid == 0) out[0] = s0;
  f32x2 lx = {p[0], p[0]}, ly = {p[1], p[1]}, lz = {p[2], p[2]};
  for (int it = 1; it < m; ++it) {
    float bd = -2.f;
    int bj = 0;
#pragma unroll
    for (int j2 = 0; j2 < P2; ++j2) {
      const f32x2 dd = fps_d2x2(px[j2], py[j2], pz[j2], lx, ly, lz);
      d[j2][0] = fminf(d[j2][0], dd[0]);
      d[j2][1] = fminf(d[j2][1], dd[1]);
      if (d[j2][0] > bd) { bd = d[j2][0]; bj = 2 * j2; }
      if (d[j2][1] > bd) { bd = d[j2][1]; bj = 2 * j2 + 1; }
    }
    const float wm = wave_max_uniform(bd);
    uint64_t cand = __ballot(bd == wm);
    const int mk = tid + bj * T;
    if (__popcll(cand) > 1) {   // several lanes hold the wave's best distance: the lowest index wins
      int km = (bd == wm) ? mk : 0x7fffffff;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) km = min(km, __shfl_xor(km, o, 64));
      cand = __ballot(bd == wm && mk == km);
    }
    const int wl = __ffsll((unsigned long long)cand) - 1;
    if (lane == wl) {   // the winner's point: a select over its registers (one lane: the rest are masked)
      f32x2 x2 = px[0], y2 = py[0], z2 = pz[0];
#pragma unroll
      for (int j2 = 1; j2 < P2; ++j2)
        if ((bj >> 1) == j2) { x2 = px[j2]; y2 = py[j2]; z2 = pz[j2]; }
      const int e = bj & 1;
      FpsSlot& sl = slot[it & 1][wid];
      sl.d = wm; sl.k = mk; sl.x = e ? x2[1] : x2[0]; sl.y = e ? y2[1] : y2[0]; sl.z = e ? z2[1] : z2[0];
    }
    __syncthreads();
    // every wave reduces the NW slots itself, lane-parallel: lane i (< NW) reads slot i; max distance over the
    // lanes, then the lowest index among the lanes holding it; the winner's coordinates: three uniform reads
    const bool sv = lane < NW;
    const float dw = sv ? slot[it & 1][lane].d : -3.f;
    const int kw = sv ? slot[it & 1][lane].k : 0x7fffffff;
    const float gm = row_max16(dw);   // NW <= 16: the slots sit in lanes 0..15 (one DPP row)
    const float gd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gm), 0));
    int kk = (sv && dw == gd) ? kw : 0x7fffffff;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) kk = min(kk, __shfl_xor(kk, o, 64));
    const int gk = __builtin_amdgcn_readlane(kk, 0);
    const int gw = __ffsll((unsigned long long)__ballot(sv && dw == gd && kw == gk)) - 1;
    const float nx = slot[it & 1][gw].x, ny = slot[it & 1][gw].y, nz = slot[it & 1][gw].z;
    lx = f32x2{nx, nx}; ly = f32x2{ny, ny}; lz = f32x2{nz, nz};
    if (tid == 0) out[it] = s0 + gk;
  }
}

}  // namespace mvr

// xyz [sum n, 3] fp32 (fragments back to back, offsets off[B+1]); idx_out [B][m] int64 global rows
extern "C" int mvr_fps(const float* xyz, const int64_t* offsets, const int64_t* offsets_host, int B, int m,
                       int64_t* idx_out, hipStream_t stream) {
  if (B < 0 || m <= 0) return MVR_EINVAL;
  if (B == 0) return MVR_OK;
  if (!xyz || !offsets || !offsets_host || !idx_out) return MVR_EINVAL;
  int64_t nmax = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t n = offsets_host[b + 1] - offsets_host[b];
    if (n < m) return MVR_EINVAL;   // FPS draws m distinct points
    nmax = n > nmax ? n : nmax;
  }
  if (B == 0) return MVR_OK;
  mvr::ProfScope prof(mvr::PK_SMALL, 9.0 * (double)nmax * m * B, (double)nmax * 12 * B, stream);
  const dim3 g(B);
#define MVR_FPS(T, PER, REG)                                                                                \
  if (nmax <= (int64_t)(T) * (PER)) {                                                                    \
    hipLaunchKernelGGL((mvr::fps_kernel<T, PER, REG>), g, dim3(T), 0, stream, xyz, offsets, m, idx_out); \
    MVR_CHECK_LAUNCH();                                                                                 \
    return MVR_OK;                                                                                      \
  }
#define MVR_FPSR(T, PER)                                                                                  \
  if (nmax <= (int64_t)(T) * (PER)) {                                                                  \
    hipLaunchKernelGGL((mvr::fps_reg_kernel<T, PER>), g, dim3(T), 0, stream, xyz, offsets, m, idx_out); \
    MVR_CHECK_LAUNCH();                                                                                \
    return MVR_OK;                                                                                     \
  }
  // 1024 threads: 4 VGPRs per point within the 128 a 1024-thread workgroup allows; 512 threads: 256
  MVR_FPSR(1024, 4)
  MVR_FPSR(1024, 8)
  MVR_FPSR(1024, 16)
  MVR_FPSR(1024, 20)
  MVR_FPSR(1024, 24)
  MVR_FPSR(768, 32)
  MVR_FPSR(512, 48)
#undef MVR_FPSR
  MVR_FPS(1024, 64, false)
  MVR_FPS(512, 160, false)
#undef MVR_FPS
  return MVR_EINVAL;   // > 81920 points per fragment
}
