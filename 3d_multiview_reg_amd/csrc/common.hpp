// Shared device helpers for the mvreg HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MVR_OK 0
#define MVR_EINVAL -1
#define MVR_ELAUNCH -2

#define MVR_CHECK_LAUNCH()                                  \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return MVR_ELAUNCH;               \
  } while (0)

namespace mvr {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of NV doubles; result valid in every thread.  `red` must hold
// NV * (blockDim/64) doubles of LDS.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[w * NV + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += red[j * NV + i];
    v[i] = s;
  }
  __syncthreads();
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4): lane l's bytes from base + off land at LDS byte address
// lds + 16 l.  base and lds wave-uniform (SGPRs), off a 32-bit lane offset: no 64-bit per-lane pointers or
// generic-to-LDS casts stay live in a loop.  Inline asm: the compiler does not count it, so the caller waits
// (s_waitcnt vmcnt) before the data is read.
__device__ __forceinline__ void glds16s(const void* base, uint32_t off, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(off), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {   // byte address of a __shared__ object
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// XCD-aware workgroup -> tile map.  Workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share one, each
// XCD with its own L2): this bijection on [0, nb) gives XCD b % 8 a contiguous range of tiles instead, so the
// workgroups one XCD runs together work on neighbouring tiles and share what they read in its L2.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8;
  return x * q + (x < r ? x : r) + b / 8;
}

}  // namespace mvr
