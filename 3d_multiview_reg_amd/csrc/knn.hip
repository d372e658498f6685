// Coordinate-space nearest neighbour and the mutual-NN flag of the soft matches:
//
//   knn_point(k=1, pos1, pos2)      lib/utils.py:274-299   squared L2 sum(-(pos1 - pos2)^2, -1), topk(1) of -d
//   extract_mutuals(x1, x2, m1, m2) lib/utils.py:822-848   j = NN of m1[i] among x2; mutual = |x1[i] - m2[j]|^2 < thr^2
//
// The reference materialises [b, m, n, 3] repeats of both clouds (5000 x 5000 x 3 per pair); here one workgroup
// takes 1024 queries of one batch row (4 per thread, two packed-fp32 pairs) and streams the targets through LDS in
// tiles of 1024 (16 KB, broadcast reads).  Per (query, target): packed sub / mul / add (no contraction: the sum is
// ((dx^2 + dy^2) + dz^2) in fp32, the reference's reduction order) and a strict-less compare, so the first index
// wins on equal distances.  Padding targets are NaN (never selected).  VALU-bound: ~7 issue slots per
// (query, target); HBM traffic is the two clouds once per workgroup.
#include <math.h>
#include <stdint.h>

#include "common.hpp"
#include "mvreg.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int KT = 1024;        // targets per LDS tile
constexpr int KQ = 4;           // queries per thread
constexpr int KB = 256;         // threads per workgroup

struct Pts {
  const float* p;
  int64_t bs, rs;               // batch and row stride (floats); 3 contiguous coordinates per row
  __device__ __forceinline__ const float* row(int b, int64_t i) const { return p + b * bs + i * rs; }
};

struct KnnArgs {
  Pts tgt, qry;                 // targets [B][Nt], queries [B][Nq]
  int Nt, Nq;
  float* dist;                  // [B][Nq] squared distance of the nearest target (may be null)
  int64_t* idx;                 // [B][Nq] its index (may be null)
  Pts x1, m2;                   // mutuals: source points, soft matches of the targets (indexed by target row)
  float thr2;
  float* flag;                  // [B][Nq] 1.0 mutual, 0.0 otherwise (null: plain knn)
};

__device__ __forceinline__ float sq3(float dx, float dy, float dz) {
#pragma clang fp contract(off)
  return (dx * dx + dy * dy) + dz * dz;
}

__global__ __launch_bounds__(KB) void knn1_kernel(KnnArgs a) {
#pragma clang fp contract(off)
  __shared__ float4 st[KT];
  const int b = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * (KB * KQ) + threadIdx.x;
  f2 qx[KQ / 2], qy[KQ / 2], qz[KQ / 2];
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    const int64_t q = q0 + (int64_t)k * KB;
    float x = 0.f, y = 0.f, z = 0.f;
    if (q < a.Nq) {
      const float* r = a.qry.row(b, q);
      x = r[0];
      y = r[1];
      z = r[2];
    }
    qx[k >> 1][k & 1] = x;
    qy[k >> 1][k & 1] = y;
    qz[k >> 1][k & 1] = z;
  }
  float bd[KQ];
  int bi[KQ];
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    bd[k] = INFINITY;
    bi[k] = 0;
  }
  for (int t0 = 0; t0 < a.Nt; t0 += KT) {
    const int cnt = min(KT, a.Nt - t0);
    const int cnt8 = (cnt + 7) & ~7;
    __syncthreads();
    for (int j = threadIdx.x; j < cnt8; j += KB) {
      float4 v = make_float4(NAN, NAN, NAN, 0.f);
      if (j < cnt) {
        const float* r = a.tgt.row(b, t0 + j);
        v = make_float4(r[0], r[1], r[2], 0.f);
      }
      st[j] = v;
    }
    __syncthreads();
    for (int j = 0; j < cnt8; j += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 t = st[j + u];
        const f2 tx = {t.x, t.x}, ty = {t.y, t.y}, tz = {t.z, t.z};
#pragma unroll
        for (int h = 0; h < KQ / 2; ++h) {
          const f2 dx = qx[h] - tx, dy = qy[h] - ty, dz = qz[h] - tz;
          const f2 d = (dx * dx + dy * dy) + dz * dz;
          const int id = t0 + j + u;
          if (d.x < bd[2 * h]) {
            bd[2 * h] = d.x;
            bi[2 * h] = id;
          }
          if (d.y < bd[2 * h + 1]) {
            bd[2 * h + 1] = d.y;
            bi[2 * h + 1] = id;
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    const int64_t q = q0 + (int64_t)k * KB;
    if (q >= a.Nq) continue;
    const int64_t o = (int64_t)b * a.Nq + q;
    if (a.dist) a.dist[o] = bd[k];
    if (a.idx) a.idx[o] = bi[k];
    if (a.flag) {
      const float* p = a.x1.row(b, q);
      const float* m = a.m2.row(b, bi[k]);
      a.flag[o] = sq3(p[0] - m[0], p[1] - m[1], p[2] - m[2]) < a.thr2 ? 1.f : 0.f;
    }
  }
}

bool pts_ok(const float* p, int64_t bs, int64_t rs) { return p && bs >= 0 && rs >= 3; }

int launch(const KnnArgs& a, int B, hipStream_t s) {
  if (B <= 0 || a.Nq <= 0) return MVR_OK;
  const dim3 grid((unsigned)((a.Nq + KB * KQ - 1) / (KB * KQ)), (unsigned)B);
  knn1_kernel<<<grid, KB, 0, s>>>(a);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

}  // namespace

extern "C" int mvr_knn1(const float* pos1, int64_t p1_bstride, int64_t p1_rstride, const float* pos2,
                        int64_t p2_bstride, int64_t p2_rstride, int B, int N, int M, float* dist_out, int64_t* idx_out,
                        mvr_stream_t stream) {
  if (B < 0 || N <= 0 || M < 0 || N > (1 << 30)) return MVR_EINVAL;
  if (B == 0 || M == 0) return MVR_OK;   // no queries: NULL pointers allowed
  if (!pts_ok(pos1, p1_bstride, p1_rstride) || !pts_ok(pos2, p2_bstride, p2_rstride) || (!dist_out && !idx_out))
    return MVR_EINVAL;
  KnnArgs a{};
  a.tgt = Pts{pos1, p1_bstride, p1_rstride};
  a.qry = Pts{pos2, p2_bstride, p2_rstride};
  a.Nt = N;
  a.Nq = M;
  a.dist = dist_out;
  a.idx = idx_out;
  return launch(a, B, (hipStream_t)stream);
}

extern "C" int mvr_mutuals(const float* x1, int64_t x1_bstride, int64_t x1_rstride, const float* x2,
                           int64_t x2_bstride, int64_t x2_rstride, const float* x1m, int64_t x1m_bstride,
                           int64_t x1m_rstride, const float* x2m, int64_t x2m_bstride, int64_t x2m_rstride, int B, int N,
                           float thr2, float* flag_out, int64_t* idx_out, mvr_stream_t stream) {
  if (B < 0 || N <= 0 || N > (1 << 30)) return MVR_EINVAL;
  if (B == 0) return MVR_OK;
  if (!flag_out || !pts_ok(x1, x1_bstride, x1_rstride) ||
      !pts_ok(x2, x2_bstride, x2_rstride) || !pts_ok(x1m, x1m_bstride, x1m_rstride) ||
      !pts_ok(x2m, x2m_bstride, x2m_rstride))
    return MVR_EINVAL;
  KnnArgs a{};
  a.tgt = Pts{x2, x2_bstride, x2_rstride};
  a.qry = Pts{x1m, x1m_bstride, x1m_rstride};
  a.Nt = N;
  a.Nq = N;
  a.idx = idx_out;
  a.x1 = Pts{x1, x1_bstride, x1_rstride};
  a.m2 = Pts{x2m, x2m_bstride, x2m_rstride};
  a.thr2 = thr2;
  a.flag = flag_out;
  return launch(a, B, (hipStream_t)stream);
}
