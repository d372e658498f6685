// Does a pair-chunked OANet schedule get its activations served by the 256 MiB Infinity Cache?
// Emulates the point-conv traffic of one PointCN on a chunk of P pairs (128 channels x 5024 points fp32 =
// 2.57 MB per pair per tensor): conv3 reads X, writes T; conv7 reads T and X, writes X (in place) — repeated, so
// every buffer is re-read right after it was written.  Reports the achieved (read + write) GB/s per chunk size,
// with default-policy and nontemporal loads / stores.  No arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mall_micro tools/mall_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ f4v ld(const f4v* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <int NT>
__device__ __forceinline__ void st(f4v* p, f4v v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Y = X (+ R when R): one pass, float4 per lane, 4 in flight
template <int NTL, int NTS>
__global__ __launch_bounds__(256) void pass_kernel(const f4v* __restrict__ X, const f4v* R, f4v* Y, long n4) {
  const long stride = (long)gridDim.x * 256 * 4;
  for (long i = (long)blockIdx.x * 1024 + threadIdx.x; i < n4; i += stride) {
    f4v v[4], r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long k = i + 256L * u;
      v[u] = k < n4 ? ld<NTL>(X + k) : f4v{0.f, 0.f, 0.f, 0.f};
      r[u] = (R && k < n4) ? ld<NTL>(R + k) : f4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long k = i + 256L * u;
      if (k < n4) st<NTS>(Y + k, v[u] * 1.0001f + r[u]);
    }
  }
}

template <int NTL, int NTS>
static int run(long pairs, int total_pairs, f4v* X, f4v* T, int iters, double* gbs) {
  const long n4 = pairs * 128L * 5024 / 4;
  const int chunks = (int)(total_pairs / pairs);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto body = [&]() {
    for (int c = 0; c < chunks; ++c) {
      f4v* x = X + (long)c * n4;
      f4v* t = T + (long)c * n4;
      for (int l = 0; l < 6; ++l) {   // 6 PointCN of one chunk, back to back
        hipLaunchKernelGGL((pass_kernel<NTL, NTS>), dim3(2048), dim3(256), 0, 0, x, nullptr, t, n4);   // conv3
        hipLaunchKernelGGL((pass_kernel<NTL, NTS>), dim3(2048), dim3(256), 0, 0, t, x, x, n4);         // conv7 + res
      }
    }
  };
  body();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) body();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)chunks * 6 * (2.0 + 3.0) * n4 * 16;   // conv3: r+w, conv7: 2r+w
  *gbs = bytes * iters / (ms * 1e-3) / 1e9;
  return 0;
}

int main() {
  const int total = 432;   // divisible by 8, 12, 16, 24, 36, 48, 72, 108, 144, 216, 432
  const long n = (long)total * 128 * 5024;
  f4v *X, *T;
  CK(hipMalloc(&X, n * 4));
  CK(hipMalloc(&T, n * 4));
  CK(hipMemset(X, 0, n * 4));
  CK(hipMemset(T, 0, n * 4));
  printf("pairs/chunk  MB/tensor   default GB/s   ntload GB/s   ntstore GB/s   nt both GB/s\n");
  for (int pc : {8, 12, 16, 24, 36, 48, 72, 144, 432}) {
    double g0, g1, g2, g3;
    if (run<0, 0>(pc, total, X, T, 3, &g0) || run<2, 0>(pc, total, X, T, 3, &g1) || run<0, 1>(pc, total, X, T, 3, &g2) ||
        run<2, 1>(pc, total, X, T, 3, &g3))
      return 1;
    printf("%5d %12.1f %14.0f %13.0f %14.0f %14.0f\n", pc, pc * 128.0 * 5024 * 4 / 1e6, g0, g1, g2, g3);
    fflush(stdout);
  }
  return 0;
}
