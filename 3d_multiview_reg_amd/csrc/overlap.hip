// Overlap gate of the pairwise benchmark (lib/utils.py:713-786 compute_overlap_ratio) on the GPU,
// batched over the pairs of a scene:
//   * 'FCGF' method: Open3D VoxelDownSample (voxel grid anchored at min_bound - v/2, centroid =
//     fp64 sum of the voxel's points in input order / count) of every fragment, once per scene;
//   * radius index per fragment: points sorted by (fragment, cell of size r), occupied cells in an
//     open-addressing hash (cell -> [start, end) of the sorted order);
//   * per pair and direction, every query point is mapped by the rigid transform in fp64 and
//     counts as matched when some point of the other fragment lies at distance < r (the
//     reference's 1-NN distance test, sklearn NearestNeighbors in fp64) — a 27-cell probe with
//     early exit instead of a KD-tree.
// All geometry is fp64 (the reference works on float64 arrays).  Latency / hash-probe bound.  The sorts are the
// in-tree onesweep radix sort and the scan its reduce-then-scan sibling (radix.hip): no library kernels.
#include "common.hpp"
#include "prof.hpp"
#include "radix.hpp"
#include "mvreg.h"

namespace mvr {
namespace {

constexpr uint64_t OV_EMPTY = ~0ull;
constexpr int OV_BITS = 16;                 // bits per cell / voxel coordinate
constexpr int64_t OV_BIAS = 1 << 15;        // signed cell coordinates are biased by 2^15

__device__ __forceinline__ int frag_of(const int64_t* off, int B, int64_t i) {
  int lo = 0, hi = B;   // off[lo] <= i < off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint64_t pack_key(int b, int64_t x, int64_t y, int64_t z) {
  const uint64_t m = (1ull << OV_BITS) - 1;
  return ((uint64_t)b << (3 * OV_BITS)) | (((uint64_t)x & m) << (2 * OV_BITS)) | (((uint64_t)y & m) << OV_BITS) |
         ((uint64_t)z & m);
}
__device__ __forceinline__ uint64_t hash64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// ---------------------------------------------------------------------------- voxel centroids
__global__ void frag_min_kernel(const float* __restrict__ xyz, const int64_t* __restrict__ off, double* minb) {
  __shared__ double red[3][256];
  const int b = blockIdx.x;
  double m[3] = {1e300, 1e300, 1e300};
  for (int64_t i = off[b] + threadIdx.x; i < off[b + 1]; i += blockDim.x)
    for (int d = 0; d < 3; ++d) m[d] = fmin(m[d], (double)xyz[3 * i + d]);
  for (int d = 0; d < 3; ++d) red[d][threadIdx.x] = m[d];
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int d = 0; d < 3; ++d) red[d][threadIdx.x] = fmin(red[d][threadIdx.x], red[d][threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x < 3) minb[3 * b + threadIdx.x] = red[threadIdx.x][0];
}

// Open3D: ref = (p - (min_bound - v/2)) / v; index = floor(ref)   (fp64)
__global__ void voxel_key_kernel(const float* __restrict__ xyz, const int64_t* __restrict__ off, int B, int64_t n,
                                 const double* __restrict__ minb, double v, uint64_t* keys, uint64_t* keys2,
                                 int32_t* idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int b = frag_of(off, B, i);
  int64_t c[3];
  for (int d = 0; d < 3; ++d) c[d] = (int64_t)floor(((double)xyz[3 * i + d] - (minb[3 * b + d] - v * 0.5)) / v);
  const uint64_t k = pack_key(b, c[0], c[1], c[2]);
  keys[i] = k;
  keys2[i] = k;
  idx[i] = (int32_t)i;
}

// sorted keys from the sort's permutation (the sort itself returns the values only)
__global__ void gather_keys_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ perm, int64_t n,
                                   uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = k[perm[i]];
}

__global__ void head_flag_kernel(const uint64_t* __restrict__ k, int64_t n, int32_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// one thread per voxel: sequential fp64 sum of its points in input order (the stable sort keeps it)
__global__ void centroid_kernel(const float* __restrict__ xyz, const uint64_t* __restrict__ k,
                                const int32_t* __restrict__ sidx, const int32_t* __restrict__ head,
                                const int32_t* __restrict__ pos, int64_t n, int B, double* out, int64_t* out_off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  double s[3] = {0.0, 0.0, 0.0};
  int64_t j = i;
  do {
    const int64_t q = sidx[j];
    for (int d = 0; d < 3; ++d) s[d] += (double)xyz[3 * q + d];
    ++j;
  } while (j < n && k[j] == k[i]);
  const double cnt = (double)(j - i);
  const int64_t o = pos[i];
  for (int d = 0; d < 3; ++d) out[3 * o + d] = s[d] / cnt;
  const int b = (int)(k[i] >> (3 * OV_BITS));
  if (i == 0 || (int)(k[i - 1] >> (3 * OV_BITS)) != b) out_off[b] = o;   // first voxel of fragment b
}

__global__ void fix_offsets_kernel(int64_t* out_off, int B, const int32_t* head, const int32_t* pos, int64_t n) {
  out_off[B] = n > 0 ? (int64_t)pos[n - 1] + head[n - 1] : 0;
  for (int b = B - 1; b >= 0; --b)
    if (out_off[b] < 0) out_off[b] = out_off[b + 1];   // fragments without points
}

__global__ void fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ---------------------------------------------------------------------------- radius index
struct RIndex {
  int32_t* sidx;      // [M] point ids in (fragment, cell) order
  uint64_t* skey;     // [M]
  uint64_t* hkeys;    // [cap]
  int2* hval;         // [cap] (start, end) of the cell in the sorted order
  uint64_t cap;
};

__global__ void cell_key_kernel(const double* __restrict__ xyz, const int64_t* __restrict__ off, int B, int64_t M,
                                double r, uint64_t* keys, uint64_t* keys2, int32_t* idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int b = frag_of(off, B, i);
  int64_t c[3];
  for (int d = 0; d < 3; ++d) c[d] = (int64_t)floor(xyz[3 * i + d] / r) + OV_BIAS;
  const uint64_t k = pack_key(b, c[0], c[1], c[2]);
  keys[i] = k;
  keys2[i] = k;
  idx[i] = (int32_t)i;
}

__global__ void hash_clear64_kernel(uint64_t* k, uint64_t cap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) k[i] = OV_EMPTY;
}

__global__ void cell_insert_kernel(RIndex ix, int64_t M) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint64_t k = ix.skey[i];
  const bool first = i == 0 || ix.skey[i - 1] != k, last = i == M - 1 || ix.skey[i + 1] != k;
  if (!first && !last) return;
  uint64_t h = hash64(k) & (ix.cap - 1);
  while (true) {
    const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(ix.hkeys + h), OV_EMPTY, k);
    if (prev == OV_EMPTY || prev == k) break;
    h = (h + 1) & (ix.cap - 1);
  }
  if (first) ix.hval[h].x = (int)i;
  if (last) ix.hval[h].y = (int)i + 1;
}

__device__ __forceinline__ int2 cell_find(const RIndex& ix, uint64_t k) {
  uint64_t h = hash64(k) & (ix.cap - 1);
  while (true) {
    const uint64_t s = ix.hkeys[h];
    if (s == k) return ix.hval[h];
    if (s == OV_EMPTY) return make_int2(0, 0);
    h = (h + 1) & (ix.cap - 1);
  }
}

// blockIdx.y = 2 p + d: queries of fragment pairs[p][d] mapped by T[p][d] (3x4 row-major) against the
// points of fragment pairs[p][1 - d]
__global__ void overlap_count_kernel(RIndex ix, const double* __restrict__ xyz, const int64_t* __restrict__ off,
                                     const int64_t* __restrict__ pairs, const double* __restrict__ T, double r,
                                     int32_t* counts) {
  const int pd = blockIdx.y, p = pd >> 1, d = pd & 1;
  const int qf = (int)pairs[2 * p + d], tf = (int)pairs[2 * p + 1 - d];
  const int64_t i = off[qf] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool hit = false;
  if (i < off[qf + 1]) {
    const double* M = T + 12 * pd;
    const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    const double q[3] = {M[0] * x + M[1] * y + M[2] * z + M[3], M[4] * x + M[5] * y + M[6] * z + M[7],
                         M[8] * x + M[9] * y + M[10] * z + M[11]};
    int64_t c[3];
    for (int e = 0; e < 3; ++e) c[e] = (int64_t)floor(q[e] / r) + OV_BIAS;
    for (int dz = -1; dz <= 1 && !hit; ++dz)
      for (int dy = -1; dy <= 1 && !hit; ++dy)
        for (int dx = -1; dx <= 1 && !hit; ++dx) {
          const int2 se = cell_find(ix, pack_key(tf, c[0] + dx, c[1] + dy, c[2] + dz));
          for (int j = se.x; j < se.y; ++j) {
            const int64_t t = ix.sidx[j];
            const double ex = q[0] - xyz[3 * t], ey = q[1] - xyz[3 * t + 1], ez = q[2] - xyz[3 * t + 2];
            if (sqrt(ex * ex + ey * ey + ez * ez) < r) {
              hit = true;
              break;
            }
          }
        }
  }
  const unsigned long long bal = __ballot(hit);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(counts + pd, (int)__popcll(bal));
}

// ---------------------------------------------------------------------------- host helpers
inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }
inline char* take(char*& p, size_t b) {
  p = reinterpret_cast<char*>(((uintptr_t)p + 255) & ~(uintptr_t)255);
  char* r = p;
  p += b;
  return r;
}
size_t sort_bytes(int64_t n) { return radix_ws_bytes(n > 0 ? n : 1); }
size_t scan_bytes(int64_t n) { return scan_ws_bytes(n > 0 ? n : 1); }
// key bits of pack_key for fragments [0, B): 48 coordinate bits + the fragment index
int key_bits(int B) { return 3 * OV_BITS + (B > 1 ? 32 - __builtin_clz((unsigned)(B - 1)) : 1); }
uint64_t cap_for(int64_t M) {
  uint64_t c = 1024;
  while (c < (uint64_t)(2 * (M > 0 ? M : 1))) c <<= 1;
  return c;
}
RIndex index_view(void* base, int64_t M) {
  char* p = reinterpret_cast<char*>(base);
  RIndex ix{};
  ix.cap = cap_for(M);
  ix.sidx = reinterpret_cast<int32_t*>(take(p, (size_t)(M > 0 ? M : 1) * 4));
  ix.skey = reinterpret_cast<uint64_t*>(take(p, (size_t)(M > 0 ? M : 1) * 8));
  ix.hkeys = reinterpret_cast<uint64_t*>(take(p, ix.cap * 8));
  ix.hval = reinterpret_cast<int2*>(take(p, ix.cap * 8));
  return ix;
}
size_t index_bytes(int64_t M) {
  const size_t m = (size_t)(M > 0 ? M : 1);
  return m * 12 + cap_for(M) * 16 + 5 * 256;
}
// scratch of the index build (after the index itself)
size_t build_scratch_bytes(int64_t M) {
  const size_t m = (size_t)(M > 0 ? M : 1);
  return m * 8 + sort_bytes(M) + 3 * 256;
}

}  // namespace
}  // namespace mvr

using namespace mvr;

extern "C" size_t mvr_voxel_centroids_workspace_bytes(int64_t n) {
  const size_t m = (size_t)(n > 0 ? n : 1);
  return m * (8 + 8 + 4 + 4 + 4) + sort_bytes(n) + scan_bytes(n) + 4096 * 24 + 10 * 256;
}

extern "C" int mvr_voxel_centroids(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel,
                                   void* ws, size_t ws_bytes, double* out_xyz, int64_t* out_off, hipStream_t s) {
  if (!frag_off || !out_off || B <= 0 || B > 4096 || n < 0 || n > 0x7fffffff || !(voxel > 0.0)) return MVR_EINVAL;
  if (n > 0 && (!xyz || !ws || !out_xyz || ws_bytes < mvr_voxel_centroids_workspace_bytes(n))) return MVR_EINVAL;
  if (n == 0) {   // every fragment empty: offsets all 0 (NULL point / workspace pointers allowed)
    hipLaunchKernelGGL(fill_i64_kernel, dim3(nb(B + 1)), dim3(256), 0, s, out_off, (int64_t)B + 1, (int64_t)0);
    MVR_CHECK_LAUNCH();
    return MVR_OK;
  }
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)n * 40.0, s);
  char* p = reinterpret_cast<char*>(ws);
  const size_t m = (size_t)(n > 0 ? n : 1);
  uint64_t* kin = reinterpret_cast<uint64_t*>(take(p, m * 8));
  uint64_t* kout = reinterpret_cast<uint64_t*>(take(p, m * 8));
  int32_t* vout = reinterpret_cast<int32_t*>(take(p, m * 4));
  int32_t* head = reinterpret_cast<int32_t*>(take(p, m * 4));
  int32_t* pos = reinterpret_cast<int32_t*>(take(p, m * 4));
  double* minb = reinterpret_cast<double*>(take(p, 4096 * 24));
  size_t st = sort_bytes(n), sc = scan_bytes(n);
  void* tsort = take(p, st);
  void* tscan = take(p, sc);
  RadixWs rw = radix_ws(tsort, n);
  hipLaunchKernelGGL(fill_i64_kernel, dim3(nb(B + 1)), dim3(256), 0, s, out_off, (int64_t)B + 1, (int64_t)-1);
  hipLaunchKernelGGL(frag_min_kernel, dim3(B), dim3(256), 0, s, xyz, frag_off, minb);
  hipLaunchKernelGGL(voxel_key_kernel, dim3(nb(n)), dim3(256), 0, s, xyz, frag_off, B, n, minb, voxel, rw.ka, kin,
                     rw.va);
  int rc = radix_sort(rw, key_bits(B), vout, s);   // stable: a voxel's points stay in input order
  if (rc != MVR_OK) return rc;
  hipLaunchKernelGGL(gather_keys_kernel, dim3(nb(n)), dim3(256), 0, s, kin, vout, n, kout);
  hipLaunchKernelGGL(head_flag_kernel, dim3(nb(n)), dim3(256), 0, s, kout, n, head);
  if ((rc = excl_scan_i32(head, pos, n, tscan, sc, s)) != MVR_OK) return rc;
  hipLaunchKernelGGL(centroid_kernel, dim3(nb(n)), dim3(256), 0, s, xyz, kout, vout, head, pos, n, B, out_xyz,
                     out_off);
  hipLaunchKernelGGL(fix_offsets_kernel, dim3(1), dim3(1), 0, s, out_off, B, head, pos, n);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" size_t mvr_radius_index_bytes(int64_t M) { return index_bytes(M) + build_scratch_bytes(M); }

extern "C" int mvr_radius_index_build(const double* xyz, const int64_t* off, int B, int64_t M, double r, void* index,
                                      size_t bytes, hipStream_t s) {
  if (!off || !index || B <= 0 || B >= (1 << 15) || M < 0 || M > 0x7fffffff || !(r > 0.0) ||
      bytes < mvr_radius_index_bytes(M) || (M > 0 && !xyz))
    return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)M * 60.0, s);
  RIndex ix = index_view(index, M);
  char* p = reinterpret_cast<char*>(index) + index_bytes(M);
  const size_t m = (size_t)(M > 0 ? M : 1);
  uint64_t* kin = reinterpret_cast<uint64_t*>(take(p, m * 8));
  size_t st = sort_bytes(M);
  void* tsort = take(p, st);
  hipLaunchKernelGGL(hash_clear64_kernel, dim3(nb((int64_t)ix.cap)), dim3(256), 0, s, ix.hkeys, ix.cap);
  if (M == 0) {
    MVR_CHECK_LAUNCH();
    return MVR_OK;
  }
  RadixWs rw = radix_ws(tsort, M);
  hipLaunchKernelGGL(cell_key_kernel, dim3(nb(M)), dim3(256), 0, s, xyz, off, B, M, r, rw.ka, kin, rw.va);
  const int rc = radix_sort(rw, key_bits(B), ix.sidx, s);
  if (rc != MVR_OK) return rc;
  hipLaunchKernelGGL(gather_keys_kernel, dim3(nb(M)), dim3(256), 0, s, kin, ix.sidx, M, ix.skey);
  hipLaunchKernelGGL(cell_insert_kernel, dim3(nb(M)), dim3(256), 0, s, ix, M);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_radius_overlap_count(const void* index, size_t bytes, const double* xyz, const int64_t* off, int B,
                                        int64_t M, const int64_t* pairs, const double* T, int P, int64_t max_points,
                                        double r, int32_t* counts, hipStream_t s) {
  if (B <= 0 || M < 0 || P < 0 || max_points < 0 || !(r > 0.0) || P > 32767) return MVR_EINVAL;
  if (P == 0) return MVR_OK;   // no pairs: NULL pointers allowed
  if (!counts) return MVR_EINVAL;
  if (max_points > 0 && (!index || !xyz || !off || !pairs || !T || bytes < mvr_radius_index_bytes(M)))
    return MVR_EINVAL;
  if (hipMemsetAsync(counts, 0, sizeof(int32_t) * 2 * (size_t)P, s) != hipSuccess) return MVR_ELAUNCH;
  if (max_points == 0) return hipGetLastError() == hipSuccess ? MVR_OK : MVR_ELAUNCH;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)P * 2.0 * (double)max_points * 200.0, s);
  RIndex ix = index_view(const_cast<void*>(index), M);
  hipLaunchKernelGGL(overlap_count_kernel, dim3(nb(max_points), 2 * P), dim3(256), 0, s, ix, xyz, off, pairs, T, r,
                     counts);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}
