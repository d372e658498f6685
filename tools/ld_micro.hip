// Load-pattern micro-benchmark for the point convolution (csrc/pconv.hip): how fast can 256-thread
// workgroups stream [P][128][ld] fp32 activations when every step reads 128 rows x (128 V) bytes
// (V consecutive floats per lane, rows strided by ld) and writes the same amount, two steps in
// flight in registers — no arithmetic.  Build: hipcc --offload-arch=gfx950 -O3 -o ld_micro ld_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int V>
struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef float2 T; };
template <> struct Vec<4> { typedef float4 T; };

template <int V, int STORE, int TILED = 0>
__global__ __launch_bounds__(256, 2) void stream_kernel(const float* X, float* Y, int P, int N, int ld, float* sink) {
  typedef typename Vec<V>::T T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int PTS = 32 * V;                       // points per step
  const int nst = (N + PTS - 1) / PTS;          // steps per pair
  const long total = (long)P * nst;
  const long s0 = total * blockIdx.x / gridDim.x, s1 = total * (blockIdx.x + 1) / gridDim.x;
  const int nloc = (int)(s1 - s0);
  auto addr = [&](long s, int t, int i) -> long {
    const long p = s / nst;
    const int n = min((int)(s - p * nst) * PTS + V * l32, N - V);
    if (TILED)   // chunk-major [P][N / 32][128][32]: a step's 128 rows x 128 B are one contiguous 16 KB block
      return p * 128L * ld + (long)(n >> 5) * 4096 + (long)(32 * w + 8 * h + 16 * t + i) * 32 + (n & 31);
    return p * 128L * ld + (long)(32 * w + 8 * h + 16 * t + i) * ld + n;
  };
  T xa[16], xb[16];
  float acc = 0.f;
  auto issue = [&](long s, T (&r)[16]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 8; ++i) r[8 * t + i] = *reinterpret_cast<const T*>(X + addr(s, t, i));
  };
  auto consume = [&](long s, T (&r)[16]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float* f = reinterpret_cast<const float*>(&r[q]);
#pragma unroll
      for (int e = 0; e < V; ++e) acc += f[e];
      if (STORE == 1) *reinterpret_cast<T*>(Y + addr(s, q >> 3, q & 7)) = r[q];
    }
    if (STORE == 2) {   // pconv's epilogue pattern: lane -> row (lane >> 1) of the wave's 32, 16 columns
      const long p = s / nst;
      const int n0 = (int)(s - p * nst) * PTS;
      const int nn = min(n0 + 16 * (lane & 1), N - 16);
      float* dst = TILED ? Y + p * 128L * ld + (long)(nn >> 5) * 4096 + (long)(32 * w + (lane >> 1)) * 32 + (nn & 31)
                         : Y + p * 128L * ld + (long)(32 * w + (lane >> 1)) * ld + nn;
      const float* f = reinterpret_cast<const float*>(&r[0]);
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) reinterpret_cast<float4*>(dst)[i4] = make_float4(f[0], f[1], acc, f[0]);
    }
  };
  issue(s0, xa);
  issue(min(s0 + 1, s1 - 1), xb);
  int j = 0;
  for (; j + 1 < nloc; j += 2) {
    consume(s0 + j, xa);
    issue(min(s0 + j + 2, s1 - 1), xa);
    asm volatile("s_barrier" ::: "memory");
    consume(s0 + j + 1, xb);
    issue(min(s0 + j + 3, s1 - 1), xb);
    asm volatile("s_barrier" ::: "memory");
  }
  if (j < nloc) consume(s0 + j, xa);
  if (acc == 12345.f) sink[0] = acc;
}

// reference: the same bytes as one contiguous stream (a point-major [P][N][128] layout), 16 B per lane,
// 4 KB per wave-instruction group, UNR loads in flight per lane
template <int UNR>
__global__ __launch_bounds__(256, 2) void copy_kernel(const float4* X, float4* Y, long n4) {
  const long stride = (long)gridDim.x * 256 * UNR;
  for (long base = (long)blockIdx.x * 256 * UNR + threadIdx.x; base < n4; base += stride) {
    float4 r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) r[u] = base + 256L * u < n4 ? X[base + 256L * u] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (base + 256L * u < n4) Y[base + 256L * u] = r[u];
  }
}

template <int UNR>
static float run_copy(const float* X, float* Y, long n4, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int it = 0; it < 2; ++it)
    hipLaunchKernelGGL((copy_kernel<UNR>), dim3(grid), dim3(256), 0, 0, (const float4*)X, (float4*)Y, n4);
  hipEventRecord(e0);
  for (int it = 0; it < 10; ++it)
    hipLaunchKernelGGL((copy_kernel<UNR>), dim3(grid), dim3(256), 0, 0, (const float4*)X, (float4*)Y, n4);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

template <int V, int STORE, int TILED = 0>
static float run(const float* X, float* Y, int P, int N, int ld, float* sink, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int it = 0; it < 2; ++it) hipLaunchKernelGGL((stream_kernel<V, STORE, TILED>), dim3(grid), dim3(256), 0, 0, X, Y, P, N, ld, sink);
  hipEventRecord(e0);
  const int iters = 10;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((stream_kernel<V, STORE, TILED>), dim3(grid), dim3(256), 0, 0, X, Y, P, N, ld, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / iters;
}

int main() {
  const int P = 435, N = 5000;
  float *X, *Y, *sink;
  const size_t bytes = (size_t)P * 128 * 5024 * 4;
  hipMalloc(&X, bytes);
  hipMalloc(&Y, bytes);
  hipMalloc(&sink, 64);
  hipMemset(X, 0, bytes);
  {
    const long n4 = (long)P * 128 * N / 4;
    const double gb = 2.0 * P * 128.0 * N * 4 / 1e9;
    for (int grid : {512, 1024, 2048}) {
      const float a = run_copy<4>(X, Y, n4, grid), b = run_copy<8>(X, Y, n4, grid);
      printf("contiguous copy grid %4d: UNR4 %.3f ms (%.0f GB/s)  UNR8 %.3f ms (%.0f GB/s)\n", grid, a, gb / a * 1e3, b,
             gb / b * 1e3);
    }
  }
  for (int ld : {5000, 5024}) {
    const double gb = 2.0 * P * 128.0 * N * 4 / 1e9;
    for (int grid : {512, 1024}) {
      float t1 = run<1, 1>(X, Y, P, N, ld, sink, grid);
      float t2 = run<2, 1>(X, Y, P, N, ld, sink, grid);
      float t4 = run<4, 1>(X, Y, P, N, ld, sink, grid);
      float e1 = run<1, 2>(X, Y, P, N, ld, sink, grid);
      float r1 = run<1, 0>(X, Y, P, N, ld, sink, grid);
      float r4 = run<4, 0>(X, Y, P, N, ld, sink, grid);
      printf("ld %d grid %4d  read+write: V1 %.3f ms (%.0f GB/s)  V2 %.3f (%.0f)  V4 %.3f (%.0f) | pconv-store V1 %.3f (%.0f) | read only: V1 %.3f (%.0f) V4 %.3f (%.0f)\n",
             ld, grid, t1, gb / t1 * 1e3, t2, gb / t2 * 1e3, t4, gb / t4 * 1e3, e1, gb / e1 * 1e3, r1, gb / 2 / r1 * 1e3, r4,
             gb / 2 / r4 * 1e3);
    }
  }
  {   // chunk-major layout (N a multiple of 32 per pair, ld = N): pconv's loads and epilogue stores
    const int N = 4992, ld = 4992;
    const double gb = 2.0 * P * 128.0 * N * 4 / 1e9;
    for (int grid : {512, 1024}) {
      const float rw = run<1, 1>(X, Y, P, N, ld, sink, grid), rwt = run<1, 1, 1>(X, Y, P, N, ld, sink, grid);
      const float e = run<1, 2>(X, Y, P, N, ld, sink, grid), et = run<1, 2, 1>(X, Y, P, N, ld, sink, grid);
      const float r = run<1, 0>(X, Y, P, N, ld, sink, grid), rt = run<1, 0, 1>(X, Y, P, N, ld, sink, grid);
      printf("N %d grid %4d  rows vs chunk-major: read+write %.3f (%.0f GB/s) / %.3f (%.0f) | pconv-store %.3f (%.0f) / "
             "%.3f (%.0f) | read only %.3f (%.0f) / %.3f (%.0f)\n",
             N, grid, rw, gb / rw * 1e3, rwt, gb / rwt * 1e3, e, gb / e * 1e3, et, gb / et * 1e3, r, gb / 2 / r * 1e3,
             rt, gb / 2 / rt * 1e3);
    }
  }
  return 0;
}
