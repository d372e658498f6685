// Streaming ceilings of MI355X HBM for the point-conv traffic shape: read-only, write-only and copy
// (read + write) of a 1.1 GB fp32 buffer (435 pairs x 128 channels x 5024 points), float4 per lane,
// with default-policy or nontemporal stores, at several grid sizes.  No arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_micro tools/bw_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                    \
    }                                                              \
  } while (0)

// MODE 0 read only (sum into sink), 1 write only, 2 copy; NT: nontemporal stores; UNR: float4 per lane in flight
template <int MODE, int NT, int UNR>
__global__ __launch_bounds__(256) void bw_kernel(const float4* __restrict__ X, float4* __restrict__ Y, long n4,
                                                 float* sink) {
  const long stride = (long)gridDim.x * 256 * UNR;
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 * UNR + threadIdx.x; i < n4; i += stride) {
    float4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long k = i + 256L * u;
      if (MODE != 1) v[u] = k < n4 ? X[k] : make_float4(0.f, 0.f, 0.f, 0.f);
      else v[u] = make_float4((float)k, 1.f, 2.f, 3.f);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long k = i + 256L * u;
      if (MODE == 0) {
        acc += v[u].x + v[u].y + v[u].z + v[u].w;
      } else if (k < n4) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        if (NT) __builtin_nontemporal_store(f4v{v[u].x, v[u].y, v[u].z, v[u].w}, reinterpret_cast<f4v*>(&Y[k]));
        else Y[k] = v[u];
      }
    }
  }
  if (MODE == 0 && acc == 12345.f) sink[0] = acc;
}

template <int MODE, int NT, int UNR>
static float run(const float4* X, float4* Y, long n4, float* sink, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((bw_kernel<MODE, NT, UNR>), dim3(grid), dim3(256), 0, 0, X, Y, n4, sink);
  (void)hipEventRecord(a, 0);
  const int it = 10;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((bw_kernel<MODE, NT, UNR>), dim3(grid), dim3(256), 0, 0, X, Y, n4, sink);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / it;
}

int main() {
  const long n = 435L * 128 * 5024;   // floats
  const long n4 = n / 4;
  float4 *X, *Y;
  float* sink;
  CK(hipMalloc(&X, n * 4));
  CK(hipMalloc(&Y, n * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(X, 0, n * 4));
  const double gb = n * 4.0 / 1e9;
  for (int grid : {1024, 2048, 4096, 16384}) {
    const float r4 = run<0, 0, 4>(X, Y, n4, sink, grid), r8 = run<0, 0, 8>(X, Y, n4, sink, grid);
    const float w4 = run<1, 0, 4>(X, Y, n4, sink, grid), w4n = run<1, 1, 4>(X, Y, n4, sink, grid);
    const float c4 = run<2, 0, 4>(X, Y, n4, sink, grid), c4n = run<2, 1, 4>(X, Y, n4, sink, grid);
    const float c8 = run<2, 0, 8>(X, Y, n4, sink, grid), c8n = run<2, 1, 8>(X, Y, n4, sink, grid);
    printf("grid %5d  read U4 %.0f U8 %.0f GB/s | write %.0f nt %.0f | copy U4 %.0f nt %.0f  U8 %.0f nt %.0f GB/s\n", grid,
           gb / r4 * 1e3, gb / r8 * 1e3, gb / w4 * 1e3, gb / w4n * 1e3, 2 * gb / c4 * 1e3, 2 * gb / c4n * 1e3,
           2 * gb / c8 * 1e3, 2 * gb / c8n * 1e3);
  }
  return 0;
}
