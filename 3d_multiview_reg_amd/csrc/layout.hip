// Layout helpers on the hot path (no reference counterpart beyond tensor views).
#include "common.hpp"

namespace mvr {
// out(p,c,n) = xs(p,n,c): correspondences [P][N][C] -> channel-major network input
// (the reference's data['xs'].transpose(1,3), lib/filtering/oanet.py:234).
__global__ void xs_to_channels_kernel(const float* __restrict__ xs, int64_t ps, int64_t ns, int C, int N,
                                      float* __restrict__ out, int64_t ops, int64_t ld) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (n >= N) return;
  const float* src = xs + (int64_t)p * ps + (int64_t)n * ns;
  float* dst = out + (int64_t)p * ops + n;
  for (int c = 0; c < C; ++c) dst[(int64_t)c * ld] = src[c];
}
}  // namespace mvr

extern "C" int mvr_xs_to_channels(const float* xs, int64_t xs_pstride, int64_t xs_nstride, int C, int P, int N,
                                  float* out, int64_t out_pstride, int64_t out_ld, hipStream_t stream) {
  if (C < 0 || P < 0 || N < 0 || out_ld < N) return MVR_EINVAL;
  if (P == 0 || N == 0 || C == 0) return MVR_OK;
  if (!xs || !out) return MVR_EINVAL;
  hipLaunchKernelGGL(mvr::xs_to_channels_kernel, dim3((N + 255) / 256, P), dim3(256), 0, stream, xs, xs_pstride,
                     xs_nstride, C, N, out, out_pstride, out_ld);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}
