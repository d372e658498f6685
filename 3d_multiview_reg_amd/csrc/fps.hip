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

}  // namespace mvr

// xyz [sum n, 3] fp32 (fragments back to back, offsets off[B+1]); idx_out [B][m] int64 global rows
extern "C" int mvr_fps(const float* xyz, const int64_t* offsets, const int64_t* offsets_host, int B, int m,
                       int64_t* idx_out, hipStream_t stream) {
  if (!xyz || !offsets || !offsets_host || !idx_out || B < 0 || m <= 0) return MVR_EINVAL;
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
  MVR_FPS(1024, 8, true)
  MVR_FPS(1024, 16, true)
  MVR_FPS(512, 40, true)
  MVR_FPS(1024, 64, false)
  MVR_FPS(512, 160, false)
#undef MVR_FPS
  return MVR_EINVAL;   // > 81920 points per fragment
}
