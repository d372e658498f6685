// Sparse-voxel machinery of the FCGF descriptor (the MinkowskiEngine 0.4
// primitives used by lib/descriptor/fcgf.py), written for MI355X:
//
//   * voxelisation  floor(xyz / voxel) + first-occurrence dedup  (ME.utils.sparse_quantize,
//                   scripts/pairwise_demo.py:79, scripts/utils.py:108-113)
//   * coordinate hash: open addressing on 64-bit (batch, x, y, z) keys, linear probing,
//                   inserts by 64-bit CAS + atomicMin of the first source row
//   * strided coordinate sets  floor(c / s) * s, first-occurrence order
//   * kernel maps as output-stationary neighbour tables nbr[o][k] (-1 = absent)
//                   for the 3^3 / 7^3 stencils, strided and transposed
//   * the sparse convolution itself (gather -> fp32 MFMA -> fused BN/residual/ReLU
//                   epilogue), csrc/spconv.hip
//
// Conventions the reference never pins (MinkowskiEngine is not vendored):
//   offset index k = (dx+r) + ks*(dy+r) + ks^2*(dz+r) (x fastest); strided output
//   coordinates floor(c/s)*s; transposed conv: in = out - off*s_out; output rows of
//   every dedup in first-occurrence order of the input rows.

#include <algorithm>

#include "common.hpp"
#include "mfma_bf16.hpp"
#include "prof.hpp"
#include "radix.hpp"
#include "sparse.hpp"

namespace mvr {

// ------------------------------------------------------------------ hashing
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ uint64_t pack_key(int b, int x, int y, int z) {
  return ((uint64_t)(uint32_t)b << 51) | ((uint64_t)((uint32_t)(x + KEY_BIAS) & KEY_MASK) << 34) |
         ((uint64_t)((uint32_t)(y + KEY_BIAS) & KEY_MASK) << 17) | (uint64_t)((uint32_t)(z + KEY_BIAS) & KEY_MASK);
}

// Home slot of a key.  t < 0: a hashed slot.  t >= 0 (coordinate tables of a level whose coordinates are
// multiples of 2^t): every voxel of a 2x2x2 cell of that lattice has the first slot of the cell's hashed 8-slot
// bucket (64 bytes of keys) as its home, so the cell's voxels sit side by side and a 3^3 stencil's 27 probes scan
// the buckets of <= 8 cells (shared by the neighbouring outputs) instead of 27 scattered lines.  (A slot per cell
// bit triple inside the bucket was slower: buckets hold ~2.3 keys at the tables' load, cells ~3 of their 8 voxels,
// so per-voxel slots made the buckets overflow into long probe chains.)  Linear probing from the home either way.
__device__ __forceinline__ uint64_t hash_home(const HashView& h, uint64_t key, int t) {
  if (t < 0) return mix64(key) & (h.cap - 1);
  const uint64_t cell = key & ~((1ULL << t) | (1ULL << (17 + t)) | (1ULL << (34 + t)));
  return (mix64(cell) << 3) & (h.cap - 1);
}
// where an insert into a lattice table starts probing: the voxel's cell bit triple inside its bucket (the voxels of
// one cell, inserted side by side by neighbouring threads, then do not all race for the bucket's first slot)
__device__ __forceinline__ int lattice_sub(uint64_t key, int t) {
  return (int)(((key >> t) & 1) | (((key >> (17 + t)) & 1) << 1) | (((key >> (34 + t)) & 1) << 2));
}

// lookup in a lattice table (t >= 0): the home bucket's 8 keys in one round trip (4 x 16-byte loads).  The insert
// probed from slot lattice_sub of the home bucket onwards, so an empty slot at or after it in the home bucket, or
// anywhere in a later bucket, that the key is not before proves it absent (slots never empty again).  This relies on
// no insert wrapping all the way round the table back into its home bucket's lower slots: hash_table_bytes sizes
// every table at >= 2 slots per key (load <= 1/2), so a probe run never spans the table.
__device__ __forceinline__ int64_t hash_find_bucket(const HashView& h, uint64_t key, int t) {
  uint64_t b = hash_home(h, key, t);
  int from = lattice_sub(key, t);
  for (uint64_t n = 0; n < h.cap; n += 8) {
    const uint4* kp = reinterpret_cast<const uint4*>(h.keys + b);
    uint64_t k[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 u = kp[q];
      k[2 * q] = ((uint64_t)u.y << 32) | u.x;
      k[2 * q + 1] = ((uint64_t)u.w << 32) | u.z;
    }
    int hit = -1;
    bool empty = false;
#pragma unroll
    for (int j = 7; j >= 0; --j) {
      if (k[j] == key) hit = j;
      empty |= j >= from && k[j] == EMPTY_KEY;
    }
    if (hit >= 0) return h.vals[b + hit];
    if (empty) return -1;
    b = (b + 8) & (h.cap - 1);
    from = 0;
  }
  return -1;
}

__device__ __forceinline__ int64_t hash_find(const HashView& h, uint64_t key, int t = -1) {
  if (t >= 0) return hash_find_bucket(h, key, t);
  uint64_t s = hash_home(h, key, t);
  for (uint64_t probe = 0; probe < h.cap; ++probe) {
    const uint64_t k = h.keys[s];
    if (k == key) return h.vals[s];
    if (k == EMPTY_KEY) return -1;
    s = (s + 1) & (h.cap - 1);
  }
  return -1;
}

// insert `key` with value candidate v; keeps the minimum v per key.  Plain reads first: a slot's key
// never changes once set and its value only decreases, so a (possibly stale) read that already shows
// the key with a value <= v proves the atomic unnecessary — duplicate keys (raw points of one voxel)
// then skip the contended CAS / atomicMin on their slot.
__device__ __forceinline__ void hash_insert_min(HashView h, uint64_t key, int32_t v, int t = -1) {
  uint64_t s = hash_home(h, key, t) + (t >= 0 ? lattice_sub(key, t) : 0);
  for (uint64_t probe = 0; probe < h.cap; ++probe) {
    unsigned long long cur = h.keys[s];
    if (cur == EMPTY_KEY)
      cur = atomicCAS(reinterpret_cast<unsigned long long*>(&h.keys[s]), (unsigned long long)EMPTY_KEY,
                      (unsigned long long)key);
    if (cur == EMPTY_KEY || cur == key) {
      if (h.vals[s] > v) atomicMin(&h.vals[s], v);
      return;
    }
    s = (s + 1) & (h.cap - 1);
  }
}

// the same with at most `maxp` probes; a key that finds no slot sets *overflow (the caller re-runs with a
// table sized for every key)
__device__ __forceinline__ void hash_insert_min_bounded(HashView h, uint64_t key, int32_t v, int maxp, int* overflow) {
  uint64_t s = mix64(key) & (h.cap - 1);
  for (int probe = 0; probe < maxp; ++probe) {
    unsigned long long cur = h.keys[s];
    if (cur == EMPTY_KEY)
      cur = atomicCAS(reinterpret_cast<unsigned long long*>(&h.keys[s]), (unsigned long long)EMPTY_KEY,
                      (unsigned long long)key);
    if (cur == EMPTY_KEY || cur == key) {
      if (h.vals[s] > v) atomicMin(&h.vals[s], v);
      return;
    }
    s = (s + 1) & (h.cap - 1);
  }
  atomicOr(overflow, 1);
}

__device__ __forceinline__ int64_t hash_slot(const HashView& h, uint64_t key) {
  uint64_t s = mix64(key) & (h.cap - 1);
  for (uint64_t probe = 0; probe < h.cap; ++probe) {
    const uint64_t k = h.keys[s];
    if (k == key) return (int64_t)s;
    if (k == EMPTY_KEY) return -1;
    s = (s + 1) & (h.cap - 1);
  }
  return -1;
}

__global__ void hash_clear_kernel(HashView h, int t = -1) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && h.hdr) h.hdr[0] = t;   // the home mode of the table (read by its lookups)
  if (i < h.cap) {
    h.keys[i] = EMPTY_KEY;
    h.vals[i] = 0x7fffffff;
  }
}

// ------------------------------------------------------------------ key generation
__device__ __forceinline__ int floor_div(int a, int s) { return (a >= 0) ? a / s : -((-a + s - 1) / s); }

// voxel keys of raw points: coords = floor(xyz / voxel) with the reference's arithmetic: the float32 PLY values
// widened to float64 (Open3D's points), divided (correctly rounded fp64 division, not a multiply by 1 / voxel)
// by the float64 voxel size, floored (scripts/utils.py:108-109, scripts/pairwise_demo.py:75-79); batch index from
// the fragment offsets.  T = double: the caller's float64 points as they are (scripts/utils.py extract_features
// floors Open3D's float64 array), no float32 rounding first.
// vcoords may be null (the partitioned path decodes the coordinates from the keys); range_bad (optional) is set when
// a coordinate falls outside the key's 17-bit field (keys would alias: the caller falls back to the global path).
// The fragment offsets are staged in LDS first (B <= VK_MAXB; more: read from memory): the binary search's dependent
// steps are then LDS round trips instead of memory ones.
constexpr int VK_MAXB = 1024;
template <typename T>
__global__ void vox_keys_kernel(const T* __restrict__ xyz, const int64_t* __restrict__ off, int B, int64_t n,
                                double voxel, uint64_t* keys, int4* vcoords, int* range_bad = nullptr) {
  __shared__ int64_t soff[VK_MAXB];
  const bool lds = B <= VK_MAXB;
  if (lds)
    for (int b = threadIdx.x; b < B; b += blockDim.x) soff[b] = off[b];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = B - 1;
  while (lo < hi) {  // last fragment with off[b] <= i
    const int mid = (lo + hi + 1) >> 1;
    if ((lds ? soff[mid] : off[mid]) <= i) lo = mid; else hi = mid - 1;
  }
  const int x = (int)floor((double)xyz[3 * i] / voxel);
  const int y = (int)floor((double)xyz[3 * i + 1] / voxel);
  const int z = (int)floor((double)xyz[3 * i + 2] / voxel);
  keys[i] = pack_key(lo, x, y, z);
  if (vcoords) vcoords[i] = make_int4(lo, x, y, z);
  if (range_bad && ((uint32_t)(x + KEY_BIAS) > KEY_MASK || (uint32_t)(y + KEY_BIAS) > KEY_MASK ||
                    (uint32_t)(z + KEY_BIAS) > KEY_MASK))
    atomicOr(range_bad, 1);
}

// coarse keys of a level: (b, floor(c/s)*s)
__global__ void coarse_keys_kernel(const int4* __restrict__ c, int64_t M, int s, uint64_t* keys, int4* cc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int4 v = c[i];
  const int4 o = make_int4(v.x, floor_div(v.y, s) * s, floor_div(v.z, s) * s, floor_div(v.w, s) * s);
  keys[i] = pack_key(o.x, o.y, o.z, o.w);
  cc[i] = o;
}

__global__ void insert_min_kernel(const uint64_t* __restrict__ keys, int64_t n, HashView h) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hash_insert_min(h, keys[i], (int32_t)i);
}

__global__ void insert_min_bounded_kernel(const uint64_t* __restrict__ keys, int64_t n, HashView h, int* overflow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hash_insert_min_bounded(h, keys[i], (int32_t)i, 64, overflow);
}

// first occurrences from the table instead of a lookup per key: every occupied slot holds its key's smallest source
// row (insert_min), so flag that row (flags zeroed before).  One pass over the table's slots (~2 per distinct key)
// with a scattered 4-byte store per distinct key, instead of a probe per source row (raw points: ~12 per voxel).
__global__ void slot_flag_kernel(HashView h, int32_t* flags) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < h.cap && h.keys[s] != EMPTY_KEY) flags[h.vals[s]] = 1;
}

// compact selected rows (first occurrences) in source order
__global__ void compact_kernel(const int32_t* __restrict__ flags, const int32_t* __restrict__ pos, int64_t n,
                               const int4* __restrict__ cc, int4* coords_out, int64_t* sel_out, int64_t* total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (total && i == n - 1) *total = (int64_t)pos[i] + flags[i];   // the count (exclusive scan + last flag)
  if (i < n && flags[i]) {
    const int p = pos[i];
    coords_out[p] = cc[i];
    if (sel_out) sel_out[p] = i;
  }
}

// the same with the coordinates decoded from the packed keys (exact for in-range coordinates: vox_keys_kernel
// flags the others)
__global__ void compact_keys_kernel(const int32_t* __restrict__ flags, const int32_t* __restrict__ pos, int64_t n,
                                    const uint64_t* __restrict__ keys, int4* coords_out, int64_t* sel_out,
                                    int64_t* total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (total && i == n - 1) *total = (int64_t)pos[i] + flags[i];
  if (i < n && flags[i]) {
    const int p = pos[i];
    const uint64_t k = keys[i];
    coords_out[p] = make_int4((int)(k >> 51), (int)((k >> 34) & KEY_MASK) - KEY_BIAS,
                              (int)((k >> 17) & KEY_MASK) - KEY_BIAS, (int)(k & KEY_MASK) - KEY_BIAS);
    if (sel_out) sel_out[p] = i;
  }
}

// Partitioned first occurrences of raw fragments (mvr_voxelize_hint).  Workgroup (fragment b, bucket q) scans the
// fragment's keys, keeps the ones whose bucket hash is q in an LDS hash table (key -> smallest source row, LDS CAS +
// min), then flags each kept key's smallest row: the global table's memory-side atomics and its clear / slot passes
// are gone, and the ~12 raw points per voxel meet in LDS.  The P buckets of a fragment run on one XCD (dispatch is
// round robin over the 8 XCDs: workgroups g, g + 8, ... share one), so its keys come from HBM once and from that
// XCD's L2 P - 1 times.  A key that finds no slot within VP_MAXP probes (a fragment with more voxels than the hint
// sized the buckets for) sets *overflow and the caller re-runs with the global table.  Same flags as insert_min +
// slot_flag_kernel: the smallest row of each distinct key.
#ifndef VP_LGTS
#define VP_LGTS 13   // LDS slots per workgroup 2^13 (64 KB of keys, 32 KB of rows)
#endif
#ifndef VP_NT
#define VP_NT 1024
#endif
#ifndef VP_UU
#define VP_UU 8
#endif
#ifndef VP_MODE
#define VP_MODE 0    // experiments: 1 scan + bucket test only (no inserts; results invalid)
#endif
constexpr int VP_TS = 1 << VP_LGTS;
constexpr int VP_THREADS = VP_NT;
constexpr int VP_MAXP = 64;
constexpr int VP_U = VP_UU;      // keys per thread in flight
constexpr int VP_Q = 128;        // per-wave member queue (entries)
__device__ __forceinline__ uint32_t vp_bucket(uint64_t key, int lgP) {   // Fibonacci hash of the folded key
  const uint32_t f = (uint32_t)key ^ (uint32_t)(key >> 32);
  return lgP ? (f * 0x9E3779B1u) >> (32 - lgP) : 0u;
}
__global__ __launch_bounds__(VP_THREADS) void vox_part_kernel(const uint64_t* __restrict__ keys,
                                                              const int64_t* __restrict__ off, int B, int lgP,
                                                              int32_t* flags, int* overflow) {
  __shared__ unsigned long long sk[VP_TS];
  __shared__ int sv[VP_TS];
  __shared__ int sovf;
  __shared__ unsigned long long vq_key[VP_THREADS / 64][VP_Q];   // per-wave queues of member keys and their rows
  __shared__ int vq_row[VP_THREADS / 64][VP_Q];
  const int tid = threadIdx.x;
  const int xcd = blockIdx.x & 7, r = blockIdx.x >> 3;
  const int b = xcd + 8 * (r >> lgP), q = r & ((1 << lgP) - 1);
  if (b >= B) return;   // uniform
  for (int s = tid; s < VP_TS; s += VP_THREADS) {
    sk[s] = EMPTY_KEY;
    sv[s] = 0x7fffffff;
  }
  if (tid == 0) sovf = 0;
  __syncthreads();
  const int64_t i1 = off[b + 1];
  // VP_U keys per thread in flight, the next batch loaded while this one is inserted (the LDS round trips of the
  // inserts would otherwise leave each wave one memory latency per batch)
  const int64_t ib = off[b] + tid, ilast = i1 - 1;
  constexpr int64_t VB = (int64_t)VP_U * VP_THREADS;   // rows per batch
  uint64_t ka[VP_U], kb[VP_U];
  auto load = [&](int64_t i0, uint64_t (&k)[VP_U]) {   // unconditional (clamped) loads: exact vmcnt waits
#pragma unroll
    for (int u = 0; u < VP_U; ++u) k[u] = keys[min(i0 + (int64_t)u * VP_THREADS, ilast)];
  };
  // Members (keys of this bucket, ~1 in P) go to a per-wave LDS queue, compacted by ballot; the queue is inserted 64
  // entries per pass when the next key position could overflow it, so a wave runs ~1 insert pass per 64 members
  // instead of one pass per key position with a few member lanes (the LDS atomics' latency is paid per pass):
  // 82 us per scene at 30 fragments x 250 k points (96 with a plain read before each CAS), against 156 for the
  // uncompacted loop and 520 for the global table's memory-side atomics (tools/vox_ab.sh).
  const int lane = tid & 63, wv = tid >> 6;
  unsigned long long* qk = vq_key[wv];
  int* qr = vq_row[wv];
  int qn = 0;   // wave-uniform queue fill
  auto insert1 = [&](uint64_t key, int row) {
    uint32_t s = (uint32_t)mix64(key) & (VP_TS - 1);
    for (int p = 0; p < VP_MAXP; ++p) {   // in LDS the CAS itself is the probe (a plain read first measured slower)
      const unsigned long long cur = atomicCAS(&sk[s], (unsigned long long)EMPTY_KEY, (unsigned long long)key);
      if (cur == EMPTY_KEY || cur == key) {
        atomicMin(&sv[s], row);
        return;
      }
      s = (s + 1) & (VP_TS - 1);
    }
    sovf = 1;
  };
  auto flush = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the queue writes of every lane of the wave
    if (VP_MODE != 1)
      for (int e = lane; e < qn; e += 64) insert1(qk[e], qr[e]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // queue reads done before it is refilled
    qn = 0;
  };
  auto enqueue = [&](int64_t i0, const uint64_t (&k)[VP_U]) {
#pragma unroll
    for (int u = 0; u < VP_U; ++u) {
      const int64_t i = i0 + (int64_t)u * VP_THREADS;
      const bool m = i <= ilast && vp_bucket(k[u], lgP) == (uint32_t)q;
      const uint64_t bal = __ballot(m);
      const int cnt = __popcll(bal);
      if (qn + cnt > VP_Q) flush();
      if (m) {
        const int pos = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        qk[pos] = k[u];
        qr[pos] = (int)i;
      }
      qn += cnt;
    }
  };
  // batches in wave-uniform steps (every lane of a wave runs the same iterations: the ballots need them all; rows past
  // the fragment are masked)
  const int64_t wb = off[b] + (tid & ~63);   // the wave's first row
  if (wb <= ilast) {
    load(ib, ka);
    for (int64_t w0 = wb; w0 <= ilast; w0 += 2 * VB) {
      const int64_t i0 = w0 + lane;
      load(i0 + VB, kb);
      enqueue(i0, ka);
      if (w0 + VB > ilast) break;
      load(i0 + 2 * VB, ka);
      enqueue(i0 + VB, kb);
    }
    flush();
  }
  __syncthreads();
  for (int s = tid; s < VP_TS; s += VP_THREADS)
    if (sk[s] != EMPTY_KEY) flags[sv[s]] = 1;
  if (tid == 0 && sovf) atomicOr(overflow, 1);
}

// per-batch row counts of the compacted set: a block-private LDS histogram over a contiguous run of
// output rows, then one global atomic per non-empty bin (batch-major rows: one or two per block, so
// no contention on the per-batch counters, whatever the input order)
__global__ void batch_count_kernel(const int4* __restrict__ coords, int B, int64_t* counts) {
  extern __shared__ int hist[];
  const int64_t total = counts[0];
  const int64_t per = (total + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(total, r0 + per);
  for (int b = threadIdx.x; b < B; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) atomicAdd(&hist[coords[r].x], 1);
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += blockDim.x)
    if (hist[b]) atomicAdd(reinterpret_cast<unsigned long long*>(&counts[1 + b]), (unsigned long long)hist[b]);
}

__global__ void build_table_kernel(const int4* __restrict__ c, int64_t M, HashView h, int t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) {
    const int4 v = c[i];
    hash_insert_min(h, pack_key(v.x, v.y, v.z, v.w), (int32_t)i, t);
  }
}

// ------------------------------------------------------------------ kernel maps
// nbr[o][k] = row of (coords[o] + sign*off_k*step) in the input table, or -1
// row_order (optional): thread block i / K handles output row row_order[i / K] — a spatial (fragment, Morton) order
// of the output set (mvr_kernel_map_orders without neighbour tables), so the workgroups that run together probe
// neighbouring lattice cells (L2 reuse) instead of the set's first-occurrence order (random in space)
__global__ void kernel_map_kernel(const int4* __restrict__ oc, int64_t Mo, HashView h, int ks, int step, int sign,
                                  int32_t* __restrict__ nbr, const int32_t* __restrict__ row_order) {
  const int K = ks * ks * ks;
  const int64_t e0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e0 >= Mo * K) return;
  const int64_t i = e0 / K;
  const int k = (int)(e0 - i * K);
  const int64_t o = row_order ? (int64_t)row_order[i] : i;
  const int64_t e = o * K + k;
  const int r = ks / 2;
  const int dx = k % ks - r, dy = (k / ks) % ks - r, dz = k / (ks * ks) - r;
  const int4 c = oc[o];
  int t = h.hdr[0];         // uniform: the table's home mode (-1 hashed, 0..15 lattice of stride 2^t)
  if (t < -1 || t > 15) {   // not a table hash_build wrote: no neighbour can be proven present
    nbr[e] = -1;
    return;
  }
  const int qx = c.y + sign * dx * step, qy = c.z + sign * dy * step, qz = c.w + sign * dz * step;
  // a lattice table (stride 2^t) holds only multiples of 2^t: a neighbour off the lattice (most offsets of a
  // transposed map, whose output stride is half the table's) is absent without a probe
  if (t >= 0 && ((qx | qy | qz) & ((1 << t) - 1)) != 0) {
    nbr[e] = -1;
    return;
  }
  nbr[e] = (int32_t)hash_find(h, pack_key(c.x, qx, qy, qz), t);
}

// A 3^3 map of a set onto ITSELF (out set == the table's set, row o = table value o; FCGF's stride-1 convs at every
// tensor stride) probes half the offsets: neighbour k of o is i exactly when neighbour 26 - k of i is o (offset 26 - k
// is -offset k), so thread (o, k < 13) writes both entries and the centre is o itself.  Entries no probe reaches stay
// -1 (the caller's fill).  Equal to kernel_map_kernel's map of the same table.
__global__ void kernel_map_sym_kernel(const int4* __restrict__ oc, int64_t Mo, HashView h, int step,
                                      int32_t* __restrict__ nbr) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= Mo * 14) return;
  const int64_t o = e / 14;
  const int k = (int)(e - o * 14);   // 0 .. 12 probed, 13 the centre
  if (k == 13) {
    nbr[o * 27 + 13] = (int32_t)o;
    return;
  }
  const int t = h.hdr[0];
  if (t < -1 || t > 15) return;   // not a table hash_build wrote: every entry stays -1
  const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
  const int4 c = oc[o];
  const int qx = c.y + dx * step, qy = c.z + dy * step, qz = c.w + dz * step;
  if (t >= 0 && ((qx | qy | qz) & ((1 << t) - 1)) != 0) return;   // off the table's lattice: absent
  const int64_t i = hash_find(h, pack_key(c.x, qx, qy, qz), t);
  if (i < 0) return;
  nbr[o * 27 + k] = (int32_t)i;
  nbr[i * 27 + (26 - k)] = (int32_t)o;
}

// the transpose of a map: dst[i][k] = o exactly where src[o][k] = i (entries no source reaches stay -1, the caller's
// fill).  A transposed stride-2 conv's map is the transpose of the strided conv's map between the same two sets:
// out(i) - off_k s = out(o)  <=>  out(o) + off_k s = out(i).
__global__ void kernel_map_transpose_kernel(const int32_t* __restrict__ src, int64_t Ms, int K, int32_t* __restrict__ dst,
                                            int64_t Md) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= Ms * K) return;
  const int32_t i = src[e];
  if (i < 0 || i >= Md) return;
  const int64_t o = e / K;
  const int k = (int)(e - o * K);
  dst[(int64_t)i * K + k] = (int32_t)o;
}

// ------------------------------------------------------------------ brick map
// Coordinates grouped in 4x4x4 bricks: a hash (batch, x>>2, y>>2, z>>2) -> brick id and a pool
// of 64 row indices per brick (-1 = empty cell).  A large stencil (FCGF conv1, 7^3) then costs
// <= 8 hash probes per output instead of 343, and neighbouring outputs read the same bricks
// (L1/L2 locality the per-voxel hash scatters away).
//   workspace: [16 B header: int32 brick counter] [keys u64 x cap] [rep/ids i32 x cap] [rows i32 x 64 x M]
//              [slot_of i32 x M] [brick coordinates int4 x M]
struct BrickView {
  HashView h;      // vals: representative row during the build, then the brick id
  int32_t* count;  // number of bricks
  int32_t* rows;   // [bricks][64]
  int4* bcoord;    // [bricks]: (batch, x >> 2, y >> 2, z >> 2)
};

__device__ __forceinline__ int brick_cell(int x, int y, int z) { return (x & 3) | ((y & 3) << 2) | ((z & 3) << 4); }

// A set at tensor stride 2^t (coordinates multiples of 2^t): cells are coordinates >> t, bricks 4 cells a side
// (brick coordinates >> (t + 2)); t = 0 for the voxel set itself.
__global__ void brick_insert_kernel(const int4* __restrict__ c, int64_t M, HashView h, int t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) {
    const int4 v = c[i];
    hash_insert_min(h, pack_key(v.x, v.y >> (t + 2), v.z >> (t + 2), v.w >> (t + 2)), (int32_t)i);
  }
}

// representatives (the minimum row of each brick) draw brick ids; workgroup-aggregated counter (one memory-side
// atomic per 256 rows: the ~10 k per-wave atomics on one address serialised at the memory side)
__global__ __launch_bounds__(256) void brick_ids_kernel(const int4* __restrict__ c, int64_t M, HashView h,
                                                        int32_t* count, int32_t* slot_of, int4* bcoord, int t) {
  __shared__ int wcnt[4];
  __shared__ int wbase;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t sl = -1;
  bool rep = false;
  int4 v = make_int4(0, 0, 0, 0);
  if (i < M) {
    v = c[i];
    sl = hash_slot(h, pack_key(v.x, v.y >> (t + 2), v.z >> (t + 2), v.w >> (t + 2)));
    rep = sl >= 0 && h.vals[sl] == (int32_t)i;
    slot_of[i] = (int32_t)sl;
  }
  const unsigned long long m = __ballot(rep);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wcnt[wv] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    wbase = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  int base = wbase;
  for (int w = 0; w < wv; ++w) base += wcnt[w];
  if (rep) {
    const int id = base + __popcll(m & ((1ULL << lane) - 1));
    h.vals[sl] = id;
    bcoord[id] = make_int4(v.x, v.y >> (t + 2), v.z >> (t + 2), v.w >> (t + 2));
  }
}

// the row slots of the bricks in use (count of them) to -1: the pool is sized for one brick per row, but a
// surface fills ~1/10 of that — clearing only the used bricks is ~10x fewer bytes than clearing the pool
__global__ void brick_rows_init_kernel(int32_t* rows, const int32_t* __restrict__ count) {
  const int64_t n = (int64_t)count[0] * 16;   // int4 granules
  int4* r = reinterpret_cast<int4*>(rows);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    r[i] = make_int4(-1, -1, -1, -1);
}

__global__ void brick_fill_kernel(const int4* __restrict__ c, int64_t M, HashView h, const int32_t* __restrict__ slot_of,
                                  int32_t* rows, int t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int4 v = c[i];
  const int sl = slot_of[i];
  if (sl < 0) return;
  rows[(int64_t)h.vals[sl] * 64 + brick_cell(v.y >> t, v.z >> t, v.w >> t)] = (int32_t)i;
}

// ------------------------------------------------------------------ conv1: Cin = 1, large stencil
// out[o][c] = sum_k feat[nbr(o,k)] * W[k][0][c] over the ks^3 window, gathered brick by brick;
// epilogue BN (eval, folded per column) / ReLU.  One thread per output row, W in LDS.
template <int CO>
__global__ __launch_bounds__(256) void spconv_c1_kernel(const int4* __restrict__ oc, int64_t Mo, BrickView bv,
                                                        const float* __restrict__ feat, int ks, int step,
                                                        const float* __restrict__ W, mvr_bn_p bn, float bn_eps,
                                                        int relu, float* __restrict__ out, int64_t ldout) {
  // [K][CO + 1]: lanes read different stencil rows k at the same channel — the odd row stride puts
  // them in different banks (a CO-float stride maps every lane of the wave to bank c)
  extern __shared__ float sW[];
  constexpr int WLD = CO + 1;
  const int K = ks * ks * ks;
  for (int e = threadIdx.x; e < K * CO; e += blockDim.x) sW[(e / CO) * WLD + e % CO] = W[e];
  __syncthreads();
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= Mo) return;
  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = 0.f;
  const int4 cc = oc[o];
  const int r = ks / 2;
  // the input set lives at tensor stride `step`: cell coordinates are c / step
  const int x = cc.y / step, y = cc.z / step, z = cc.w / step;
  for (int bz = (z - r) >> 2; bz <= (z + r) >> 2; ++bz)
    for (int by = (y - r) >> 2; by <= (y + r) >> 2; ++by)
      for (int bx = (x - r) >> 2; bx <= (x + r) >> 2; ++bx) {
        const int64_t sl = hash_slot(bv.h, pack_key(cc.x, bx, by, bz));
        if (sl < 0) continue;
        const int32_t* br = bv.rows + (int64_t)bv.h.vals[sl] * 64;
        const int x0 = max(x - r, 4 * bx), x1 = min(x + r, 4 * bx + 3);
        const int y0 = max(y - r, 4 * by), y1 = min(y + r, 4 * by + 3);
        const int z0 = max(z - r, 4 * bz), z1 = min(z + r, 4 * bz + 3);
        for (int cz = z0; cz <= z1; ++cz)
          for (int cy = y0; cy <= y1; ++cy)
            for (int cx = x0; cx <= x1; ++cx) {
              const int row = br[brick_cell(cx, cy, cz)];
              if (row < 0) continue;
              const float f = feat[row];
              const float* w = sW + ((cx - x + r) + ks * (cy - y + r) + ks * ks * (cz - z + r)) * WLD;
#pragma unroll
              for (int c = 0; c < CO; ++c) acc[c] = fmaf(f, w[c], acc[c]);
            }
      }
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    float v = acc[c];
    if (bn.gamma) {
      const float sc = bn.gamma[c] / sqrtf(bn.var[c] + bn_eps);
      v = (v - bn.mean[c]) * sc + bn.beta[c];
    }
    if (relu) v = fmaxf(v, 0.f);
    out[o * ldout + c] = v;
  }
}

// ------------------------------------------------------------------ conv1 over its own set, brick-tiled
// FCGF conv1 (fcgf.py:118-125: 7^3 stencil, 1 -> 32 channels, stride 1) maps the voxel set onto
// itself, so the output rows are the brick map's own rows.  One wave per 4x4x4 brick of output cells:
//   * the 10^3 window of input cells its 64 stencils read (cells 4b-3 .. 4b+6 per axis) is gathered
//     once into the wave's LDS grid (27 brick probes, then one row + one feature load per cell);
//   * out[64 cells][32] = im2col[64][343] . W[343][32] runs dense on v_mfma_f32_32x32x16_bf16 with
//     both operands split into three bf16 terms (mfma_bf16.hpp: fp32-level accuracy); the im2col
//     operand is read straight from the grid through a window-offset table, W is split once per
//     workgroup into B fragments in LDS; empty cells multiply zeros, empty output cells are skipped.
// Per brick: 22 k-steps x 2 row blocks x 6 MFMAs, instead of 343 dependent gathers per output row.
constexpr int C1_KSZ = 7, C1_K = 343, C1_NS = 22;   // 22 k-steps of 16 (343 padded with zero weights)
constexpr int C1_G = 10;                            // window edge (cells)
constexpr int C1_WAVES = 8;
constexpr int C1_GRID = 1024;                       // grid floats per wave (1000 used)

struct C1Smem {
  bx::bf16x8 wf[C1_NS][3][64];    // W as B fragments [k-step][term h, m, l][lane]   (66 KB)
  short off[C1_NS * 16];           // window offset of k: dx + 10 dy + 100 dz
  float grid[C1_WAVES][C1_GRID];   // per wave: the input window of its brick        (32 KB)
  float sc[32], sh[32];            // eval BatchNorm folded per channel
};

__global__ __launch_bounds__(512) void spconv_c1_brick_kernel(BrickView bv, const float* __restrict__ feat,
                                                              const float* __restrict__ W, mvr_bn_p bn,
                                                              float bn_eps, int relu, float* __restrict__ out,
                                                              int64_t ldout, uint16_t* __restrict__ outp) {
  using namespace bx;
  __shared__ __attribute__((aligned(16))) C1Smem sm;
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int w = tid >> 6;
  // B fragment of k-step s for lane ln: W[16 s + 8 (ln >> 5) + i][ln & 31], i = 0..7
  for (int e = tid; e < C1_NS * 64; e += blockDim.x) {
    const int s = e >> 6, ln = e & 63, k0 = 16 * s + 8 * (ln >> 5), c = ln & 31;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = k0 + i < C1_K ? W[(k0 + i) * 32 + c] : 0.f;
    Frag f;
    split8(v, f.h, f.m, f.l);
    sm.wf[s][0][ln] = f.h;
    sm.wf[s][1][ln] = f.m;
    sm.wf[s][2][ln] = f.l;
  }
  for (int k = tid; k < C1_NS * 16; k += blockDim.x)
    sm.off[k] = (short)(k < C1_K ? k % C1_KSZ + C1_G * ((k / C1_KSZ) % C1_KSZ) + C1_G * C1_G * (k / (C1_KSZ * C1_KSZ))
                                 : 0);
  if (tid < 32) {
    float sc = 1.f, sh = 0.f;
    if (bn.gamma) {
      sc = bn.gamma[tid] / sqrtf(bn.var[tid] + bn_eps);
      sh = bn.beta[tid] - bn.mean[tid] * sc;
    }
    sm.sc[tid] = sc;
    sm.sh[tid] = sh;
  }
  __syncthreads();
  const float csc = sm.sc[l32], csh = sm.sh[l32];
  // this lane's output cells 32 rb + l32 = (l32 & 3, (l32 >> 2) & 3, (l32 >> 4) + 2 rb) -> grid base
  const int base0 = (l32 & 3) + C1_G * ((l32 >> 2) & 3) + C1_G * C1_G * (l32 >> 4);
  const int base1 = base0 + 2 * C1_G * C1_G;
  float* g = sm.grid[w];
  const int nb = *bv.count;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  for (int b = blockIdx.x * C1_WAVES + w; b < nb; b += gridDim.x * C1_WAVES) {
    const int4 bc = bv.bcoord[b];
    int nid = -1;   // lane n < 27: id of the neighbour brick (n % 3, n / 3 % 3, n / 9) - 1
    if (lane < 27) {
      const int64_t sl =
          hash_slot(bv.h, pack_key(bc.x, bc.y + lane % 3 - 1, bc.z + (lane / 3) % 3 - 1, bc.w + lane / 9 - 1));
      nid = sl >= 0 ? bv.h.vals[sl] : -1;
    }
    // grid cell gi = lane + 64 i = (gx, gy, gz) sits at (gx + 1, gy + 1, gz + 1) from cell 4 (b - 1)
    int rw[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int gi = lane + 64 * i;
      const int ux = gi % C1_G + 1, uy = (gi / C1_G) % C1_G + 1, uz = gi / (C1_G * C1_G) + 1;
      const int id = __shfl(nid, (ux >> 2) + 3 * (uy >> 2) + 9 * min(uz >> 2, 2), 64);
      rw[i] = (gi < C1_G * C1_G * C1_G && id >= 0) ? bv.rows[(int64_t)id * 64 + brick_cell(ux, uy, uz)] : -1;
    }
    float fv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) fv[i] = rw[i] >= 0 ? feat[rw[i]] : 0.f;
    const int myrow = bv.rows[(int64_t)b * 64 + lane];   // output row of cell `lane` (-1: empty)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous brick's grid reads are done
#pragma unroll
    for (int i = 0; i < 16; ++i) g[lane + 64 * i] = fv[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    floatx16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
#pragma unroll 2
    for (int s = 0; s < C1_NS; ++s) {
      const s16x8 o = *reinterpret_cast<const s16x8*>(&sm.off[16 * s + 8 * hh]);
      Frag wf;
      wf.h = sm.wf[s][0][lane];
      wf.m = sm.wf[s][1][lane];
      wf.l = sm.wf[s][2][lane];
      float v0[8], v1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v0[i] = g[base0 + o[i]];
        v1[i] = g[base1 + o[i]];
      }
      Frag a0, a1;
      split8(v0, a0.h, a0.m, a0.l);
      split8(v1, a1.h, a1.m, a1.l);
      acc0 = mfma6(a0, wf, acc0);
      acc1 = mfma6(a1, wf, acc1);
    }
    // C[row (q & 3) + 8 (q >> 2) + 4 hh][column l32] of row block rb = cell 32 rb + row
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = (q & 3) + 8 * (q >> 2) + 4 * hh;
      const int r0 = __shfl(myrow, r, 64), r1 = __shfl(myrow, 32 + r, 64);
      float v0 = fmaf(acc0[q], csc, csh), v1 = fmaf(acc1[q], csc, csh);
      if (relu) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
      }
      if (r0 >= 0) out[(int64_t)r0 * ldout + l32] = v0;
      if (r1 >= 0) out[(int64_t)r1 * ldout + l32] = v1;
      if (outp) {   // the split-bf16 planes for the next sparse conv (spconv.hip PS = 1)
        if (r0 >= 0) store_planes(outp + (int64_t)r0 * 3 * ldout + l32, ldout, v0);
        if (r1 >= 0) store_planes(outp + (int64_t)r1 * 3 * ldout + l32, ldout, v1);
      }
    }
  }
}

__global__ void l2norm_rows_kernel(float* x, int64_t M, int C, int64_t ld) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= M) return;
  float* r = x + o * ld;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s = fmaf(r[c], r[c], s);
  const float inv = 1.f / sqrtf(s);
  for (int c = 0; c < C; ++c) r[c] *= inv;
}

// C = 32 (the FCGF descriptor width): 8 lanes per row, one float4 each — coalesced 128-byte rows
__global__ void l2norm_rows32_kernel(float* x, int64_t M, int64_t ld) {
  const int64_t o = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int part = threadIdx.x & 7;
  const bool ok = o < M;
  float4* r = reinterpret_cast<float4*>(x + (ok ? o : 0) * ld) + part;
  float4 v = ok ? *r : make_float4(0.f, 0.f, 0.f, 0.f);
  float s = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  const float inv = 1.f / sqrtf(s);
  if (ok) *r = make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
}

// ------------------------------------------------------------------ host helpers
static inline uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1024;
  while (p < v) p <<= 1;
  return p;
}

size_t hash_table_bytes(int64_t M) { return 16 + next_pow2((uint64_t)(2 * (M > 0 ? M : 1))) * 12; }

HashView hash_view(void* table, size_t bytes) {
  HashView h{};
  if (bytes < 16 + 1024 * 12) return h;
  uint64_t cap = 1024;
  while (16 + cap * 2 * 12 <= bytes) cap <<= 1;
  char* base = reinterpret_cast<char*>(table);
  h.cap = cap;
  h.keys = reinterpret_cast<uint64_t*>(base + 16);
  h.vals = reinterpret_cast<int32_t*>(base + 16 + cap * 8);
  h.hdr = reinterpret_cast<int32_t*>(base);
  return h;
}

static inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// dedup n keys (first occurrence, source order) -> coords_out [count], sel_out (optional), counts
struct DedupWs {
  uint64_t* keys; int4* cc; int32_t* flags; int32_t* pos; int32_t* bsum; void* table; size_t table_bytes;
};

// table sized for `keys` distinct keys (<= n)
static size_t dedup_scan_bytes(int64_t n) { return scan_ws_bytes(n > 0 ? n : 1); }
static size_t dedup_ws_bytes(int64_t n, int64_t keys = -1) {
  return (size_t)n * (8 + 16 + 4 + 4) + dedup_scan_bytes(n) + hash_table_bytes(keys < 0 ? n : keys) + 8 * 256;
}

static DedupWs dedup_ws(void* ws, int64_t n, int64_t keys = -1) {
  char* p = reinterpret_cast<char*>(ws);
  auto take = [&](size_t b) { p = reinterpret_cast<char*>(((uintptr_t)p + 255) & ~(uintptr_t)255); char* r = p; p += b; return r; };
  DedupWs d{};
  d.keys = reinterpret_cast<uint64_t*>(take((size_t)n * 8));
  d.cc = reinterpret_cast<int4*>(take((size_t)n * 16));
  d.flags = reinterpret_cast<int32_t*>(take((size_t)n * 4));
  d.pos = reinterpret_cast<int32_t*>(take((size_t)n * 4));
  d.bsum = reinterpret_cast<int32_t*>(take(dedup_scan_bytes(n)));
  d.table_bytes = hash_table_bytes(keys < 0 ? n : keys);
  d.table = take(d.table_bytes);
  return d;
}

static int dedup_run(const DedupWs& d, int64_t n, int4* coords_out, int64_t* sel_out, int64_t* counts, int B,
                     hipStream_t s, int* overflow = nullptr) {
  HashView h = hash_view(d.table, d.table_bytes);
  hipLaunchKernelGGL(hash_clear_kernel, dim3(nblk((int64_t)h.cap)), dim3(256), 0, s, h);
  if (overflow)
    hipLaunchKernelGGL(insert_min_bounded_kernel, dim3(nblk(n)), dim3(256), 0, s, d.keys, n, h, overflow);
  else
    hipLaunchKernelGGL(insert_min_kernel, dim3(nblk(n)), dim3(256), 0, s, d.keys, n, h);
  if (hipMemsetAsync(d.flags, 0, sizeof(int32_t) * (size_t)n, s) != hipSuccess) return MVR_ELAUNCH;
  hipLaunchKernelGGL(slot_flag_kernel, dim3(nblk((int64_t)h.cap)), dim3(256), 0, s, h, d.flags);
  if (hipMemsetAsync(counts, 0, sizeof(int64_t) * (1 + B), s) != hipSuccess) return MVR_ELAUNCH;
  const int rc = excl_scan_i32(d.flags, d.pos, n, d.bsum, dedup_scan_bytes(n), s);   // radix.hip
  if (rc != MVR_OK) return rc;
  hipLaunchKernelGGL(compact_kernel, dim3(nblk(n)), dim3(256), 0, s, d.flags, d.pos, n, d.cc, coords_out, sel_out,
                     counts);
  const int cb = (int)std::min<int64_t>(nblk(n), 512);
  hipLaunchKernelGGL(batch_count_kernel, dim3(cb), dim3(256), sizeof(int) * B, s, coords_out, B, counts);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

// ------------------------------------------------------------------ kernel-map row order
__device__ __forceinline__ uint32_t spread3(uint32_t v) {   // 8 bits -> every third bit of 24
  v &= 255u;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}
// sort key of an output row: its active-offset mask (the tile's offset union stays small), then — when the
// row's coordinates are given — its fragment and the Morton code of its coordinates / step (9 bits per axis,
// wrapped): rows of one mask class are tiled in spatial order, so the tiles an XCD runs together gather
// neighbour rows from one compact region (L2 reuse).  Only the tiling order changes: every output row is
// computed the same way wherever it sits.

// the sort keys of the kernel maps of one batched order call (mvr_kernel_map_orders): thread i = row o of map j
// (maps back to back in the combined key array); key = map index << 59 | offset mask << 32 | fragment and Morton
// code of c / step (9 bits per axis), value = o.  Sorted stably, map j's rows form the segment [start_j, start_j +
// M_j) of the result, in exactly mvr_kernel_map_order's order.
constexpr int ORDER_MAX_MAPS = 16;
struct OrderMaps {
  const int32_t* nbr[ORDER_MAX_MAPS];
  const int4* coords[ORDER_MAX_MAPS];
  int step[ORDER_MAX_MAPS];
  int64_t start[ORDER_MAX_MAPS + 1];
  int n, K;
  int jshift;   // key bit of the map index: 59 above the masks, 32 without neighbour tables (coordinate orders)
};
// A wave whose 64 rows lie in one map loads their neighbour rows (64 x K contiguous words) coalesced into LDS and
// each lane builds its mask there; a wave straddling two maps (at most n_maps - 1 of them) reads its rows directly.
__global__ __launch_bounds__(256) void order_keys_kernel(OrderMaps m, uint64_t* __restrict__ keys,
                                                         int32_t* __restrict__ vals) {
  __shared__ int32_t snb[4][64 * 27];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t total = m.start[m.n];
  const int64_t iw = i - lane;   // the wave's first row
  int j = 0;
  const int64_t ic = i < total ? i : total - 1;
  while (ic >= m.start[j + 1]) ++j;
  const int jf = __shfl(j, 0, 64), jl = __shfl(j, (int)min<int64_t>(63, total - 1 - iw), 64);
  const bool staged = iw < total && jf == jl && m.nbr[jf] != nullptr;   // wave-uniform
  if (staged) {
    const int64_t nrow = min<int64_t>(64, total - iw);
    const int32_t* src = m.nbr[jf] + (iw - m.start[jf]) * m.K;
    for (int e = lane; e < nrow * m.K; e += 64) snb[w][e] = src[e];
  }
  __syncthreads();
  if (i >= total) return;
  const int64_t o = i - m.start[j];
  uint32_t mask = 0;
  if (m.nbr[j]) {
    const int32_t* row = staged ? &snb[w][lane * m.K] : m.nbr[j] + o * m.K;
    for (int k = 0; k < m.K; ++k) mask |= (row[k] >= 0 ? 1u : 0u) << k;
  }
  uint32_t lo = 0;
  if (m.coords[j]) {
    const int4 c = m.coords[j][o];
    const int st = m.step[j];
    // fragment in 7 bits (<= 128 fragments stay apart: the Redwood scenes' ~50), then the Morton code of the low 8
    // bits per axis of coordinates / stride (256 cells: 6.4 m at 0.025 m)
    lo = ((uint32_t)c.x & 127u) << 25 | spread3((uint32_t)(c.y / st)) << 2 | spread3((uint32_t)(c.z / st)) << 1 |
         spread3((uint32_t)(c.w / st));
  }
  keys[i] = (uint64_t)j << m.jshift | (uint64_t)mask << 32 | lo;
  vals[i] = (int32_t)o;
}

}  // namespace mvr

using namespace mvr;

extern "C" size_t mvr_hash_table_bytes(int64_t M) { return hash_table_bytes(M); }

extern "C" size_t mvr_voxelize_workspace_bytes(int64_t n) { return dedup_ws_bytes(n); }

extern "C" int mvr_voxelize(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel, void* ws,
                            size_t ws_bytes, int32_t* coords_out, int64_t* sel_out, int64_t* counts_out,
                            hipStream_t s) {
  if (!frag_off || B <= 0 || B > MAX_BATCH || n < 0 || !(voxel > 0.0) || !counts_out) return MVR_EINVAL;
  if (n == 0) return hipMemsetAsync(counts_out, 0, sizeof(int64_t) * (1 + B), s) == hipSuccess ? MVR_OK : MVR_ELAUNCH;
  if (!xyz || !ws || !coords_out || ws_bytes < dedup_ws_bytes(n)) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)n * 40.0, s);
  DedupWs d = dedup_ws(ws, n);
  hipLaunchKernelGGL(vox_keys_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, xyz, frag_off, B, n, voxel,
                     d.keys, d.cc);
  return dedup_run(d, n, reinterpret_cast<int4*>(coords_out), sel_out, counts_out, B, s);
}

// mvr_voxelize over float64 points (same workspace, outputs and order)
extern "C" int mvr_voxelize_f64(const double* xyz, const int64_t* frag_off, int B, int64_t n, double voxel, void* ws,
                                size_t ws_bytes, int32_t* coords_out, int64_t* sel_out, int64_t* counts_out,
                                hipStream_t s) {
  if (!frag_off || B <= 0 || B > MAX_BATCH || n < 0 || !(voxel > 0.0) || !counts_out) return MVR_EINVAL;
  if (n == 0) return hipMemsetAsync(counts_out, 0, sizeof(int64_t) * (1 + B), s) == hipSuccess ? MVR_OK : MVR_ELAUNCH;
  if (!xyz || !ws || !coords_out || ws_bytes < dedup_ws_bytes(n)) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)n * 52.0, s);
  DedupWs d = dedup_ws(ws, n);
  hipLaunchKernelGGL(vox_keys_kernel<double>, dim3(nblk(n)), dim3(256), 0, s, xyz, frag_off, B, n, voxel,
                     d.keys, d.cc);
  return dedup_run(d, n, reinterpret_cast<int4*>(coords_out), sel_out, counts_out, B, s);
}

// The raw-point table sized for distinct_hint voxels instead of n points (the raw cloud holds ~12 points per
// voxel: a table for all of them is ~200 MB of clears and cache-missing probes per scene).  Inserts probe at most
// 64 slots; a key that finds none sets counts_out[B + 1] (counts_out: B + 2 entries), and the caller re-runs
// mvr_voxelize.  Same outputs as mvr_voxelize otherwise.
extern "C" size_t mvr_voxelize_hint_workspace_bytes(int64_t n, int64_t distinct_hint) {
  return dedup_ws_bytes(n, distinct_hint > 0 && distinct_hint < n ? distinct_hint : n);
}

extern "C" int mvr_voxelize_hint(const float* xyz, const int64_t* frag_off, int B, int64_t n, double voxel,
                                 int64_t distinct_hint, void* ws, size_t ws_bytes, int32_t* coords_out,
                                 int64_t* sel_out, int64_t* counts_out, hipStream_t s) {
  if (!frag_off || B <= 0 || B > MAX_BATCH || n < 0 || !(voxel > 0.0) || !counts_out || distinct_hint <= 0)
    return MVR_EINVAL;
  const int64_t keys = distinct_hint < n ? distinct_hint : n;
  if (n > 0 && (!xyz || !ws || !coords_out || ws_bytes < dedup_ws_bytes(n, keys))) return MVR_EINVAL;
  if (hipMemsetAsync(counts_out, 0, sizeof(int64_t) * (2 + B), s) != hipSuccess) return MVR_ELAUNCH;
  if (n == 0) return MVR_OK;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)n * 40.0, s);
  DedupWs d = dedup_ws(ws, n, keys);
  int* overflow = reinterpret_cast<int*>(counts_out + 1 + B);
  // buckets per fragment: the mean fragment's hinted voxels over half an LDS table each
  const int64_t per = (keys + B - 1) / B;
  int lgP = 0;
  while (lgP < 10 && ((int64_t)VP_TS / 2 << lgP) < per) ++lgP;
  hipLaunchKernelGGL(vox_keys_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, xyz, frag_off, B, n, voxel,
                     d.keys, (int4*)nullptr, overflow);
  if (hipMemsetAsync(d.flags, 0, sizeof(int32_t) * (size_t)n, s) != hipSuccess) return MVR_ELAUNCH;
  const unsigned grid = 8u * (unsigned)((B + 7) / 8) << lgP;
  hipLaunchKernelGGL(vox_part_kernel, dim3(grid), dim3(VP_THREADS), 0, s, d.keys, frag_off, B, lgP, d.flags, overflow);
  const int rc = excl_scan_i32(d.flags, d.pos, n, d.bsum, dedup_scan_bytes(n), s);   // radix.hip
  if (rc != MVR_OK) return rc;
  hipLaunchKernelGGL(compact_keys_kernel, dim3(nblk(n)), dim3(256), 0, s, d.flags, d.pos, n, d.keys,
                     reinterpret_cast<int4*>(coords_out), sel_out, counts_out);
  const int cb = (int)std::min<int64_t>(nblk(n), 512);
  hipLaunchKernelGGL(batch_count_kernel, dim3(cb), dim3(256), sizeof(int) * B, s, reinterpret_cast<int4*>(coords_out),
                     B, counts_out);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" size_t mvr_coords_downsample_workspace_bytes(int64_t M) { return dedup_ws_bytes(M); }

extern "C" int mvr_coords_downsample(const int32_t* coords, int64_t M, int B, int stride_out, void* ws,
                                     size_t ws_bytes, int32_t* coords_out, int64_t* counts_out, hipStream_t s) {
  if (M < 0 || B <= 0 || B > MAX_BATCH || stride_out <= 0 || !counts_out) return MVR_EINVAL;
  if (M == 0) return hipMemsetAsync(counts_out, 0, sizeof(int64_t) * (1 + B), s) == hipSuccess ? MVR_OK : MVR_ELAUNCH;
  if (!coords || !ws || !coords_out || ws_bytes < dedup_ws_bytes(M)) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)M * 40.0, s);
  DedupWs d = dedup_ws(ws, M);
  hipLaunchKernelGGL(coarse_keys_kernel, dim3(nblk(M)), dim3(256), 0, s, reinterpret_cast<const int4*>(coords), M,
                     stride_out, d.keys, d.cc);
  return dedup_run(d, M, reinterpret_cast<int4*>(coords_out), nullptr, counts_out, B, s);
}

static int hash_build(const int32_t* coords, int64_t M, int t, void* table, size_t table_bytes, hipStream_t s) {
  if (M < 0 || !table || (M > 0 && !coords)) return MVR_EINVAL;   // an empty set still clears its table
  if (table_bytes < hash_table_bytes(M)) return MVR_EINVAL;
  HashView h = hash_view(table, table_bytes);
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)h.cap * 12 + M * 28.0, s);
  hipLaunchKernelGGL(hash_clear_kernel, dim3(nblk((int64_t)h.cap)), dim3(256), 0, s, h, t);
  if (M > 0)
    hipLaunchKernelGGL(build_table_kernel, dim3(nblk(M)), dim3(256), 0, s, reinterpret_cast<const int4*>(coords), M,
                       h, t);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_hash_build(const int32_t* coords, int64_t M, void* table, size_t table_bytes, hipStream_t s) {
  return hash_build(coords, M, -1, table, table_bytes, s);
}

extern "C" int mvr_hash_build_lattice(const int32_t* coords, int64_t M, int stride, void* table, size_t table_bytes,
                                      hipStream_t s) {
  if (stride <= 0 || (stride & (stride - 1)) || stride > (1 << 15)) return MVR_EINVAL;
  return hash_build(coords, M, __builtin_ctz((unsigned)stride), table, table_bytes, s);
}

extern "C" int mvr_kernel_map_x(const int32_t* out_coords, int64_t Mout, const void* in_table, size_t in_table_bytes,
                                int ksize, int step, int transposed, int32_t* nbr, const int32_t* row_order,
                                hipStream_t s) {
  if (Mout < 0 || ksize <= 0 || (ksize & 1) == 0 || step <= 0) return MVR_EINVAL;
  if (Mout == 0) return MVR_OK;
  if (!out_coords || !in_table || !nbr) return MVR_EINVAL;
  HashView h = hash_view(const_cast<void*>(in_table), in_table_bytes);
  if (!h.cap) return MVR_EINVAL;
  const int64_t tot = Mout * (int64_t)ksize * ksize * ksize;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)tot * 4.0, s);
  hipLaunchKernelGGL(kernel_map_kernel, dim3(nblk(tot)), dim3(256), 0, s, reinterpret_cast<const int4*>(out_coords),
                     Mout, h, ksize, step, transposed ? -1 : 1, nbr, row_order);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_kernel_map_sym(const int32_t* coords, int64_t M, const void* table, size_t table_bytes, int step,
                                  int32_t* nbr, hipStream_t s) {
  if (M < 0 || step <= 0) return MVR_EINVAL;
  if (M == 0) return MVR_OK;
  if (!coords || !table || !nbr) return MVR_EINVAL;
  HashView h = hash_view(const_cast<void*>(table), table_bytes);
  if (!h.cap) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)M * 27 * 4.0, s);
  if (hipMemsetAsync(nbr, 0xFF, sizeof(int32_t) * 27 * (size_t)M, s) != hipSuccess) return MVR_ELAUNCH;
  hipLaunchKernelGGL(kernel_map_sym_kernel, dim3(nblk(M * 14)), dim3(256), 0, s, reinterpret_cast<const int4*>(coords), M,
                     h, step, nbr);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_kernel_map_transpose(const int32_t* src, int64_t Ms, int K, int32_t* dst, int64_t Md, hipStream_t s) {
  if (Ms < 0 || Md < 0 || K <= 0 || K > 343) return MVR_EINVAL;
  if (Md == 0) return MVR_OK;
  if (!dst || (Ms > 0 && !src)) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)(Ms + Md) * K * 4.0, s);
  if (hipMemsetAsync(dst, 0xFF, sizeof(int32_t) * (size_t)K * (size_t)Md, s) != hipSuccess) return MVR_ELAUNCH;
  if (Ms > 0)
    hipLaunchKernelGGL(kernel_map_transpose_kernel, dim3(nblk(Ms * K)), dim3(256), 0, s, src, Ms, K, dst, Md);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_kernel_map(const int32_t* out_coords, int64_t Mout, const void* in_table, size_t in_table_bytes,
                              int ksize, int step, int transposed, int32_t* nbr, hipStream_t s) {
  return mvr_kernel_map_x(out_coords, Mout, in_table, in_table_bytes, ksize, step, transposed, nbr, nullptr, s);
}

static size_t brick_slot_of_bytes(int64_t M) { return ((size_t)(M > 0 ? M : 1) * 4 + 15) & ~(size_t)15; }
static size_t brick_map_bytes(int64_t M) {
  const uint64_t cap = next_pow2((uint64_t)(2 * (M > 0 ? M : 1)));
  const size_t m = (size_t)(M > 0 ? M : 1);
  return 16 + cap * 12 + m * 64 * 4 + brick_slot_of_bytes(M) + m * 16;
}
static BrickView brick_view(void* ws, int64_t M) {
  BrickView v{};
  const uint64_t cap = next_pow2((uint64_t)(2 * (M > 0 ? M : 1)));
  const size_t m = (size_t)(M > 0 ? M : 1);
  char* base = reinterpret_cast<char*>(ws);
  v.count = reinterpret_cast<int32_t*>(base);
  v.h.cap = cap;
  v.h.keys = reinterpret_cast<uint64_t*>(base + 16);
  v.h.vals = reinterpret_cast<int32_t*>(base + 16 + cap * 8);
  v.rows = reinterpret_cast<int32_t*>(base + 16 + cap * 12);
  // after the rows and slot_of: 16-byte aligned (cap >= 1024)
  v.bcoord = reinterpret_cast<int4*>(base + 16 + cap * 12 + m * 64 * 4 + brick_slot_of_bytes(M));
  return v;
}

extern "C" size_t mvr_brick_map_bytes(int64_t M) { return brick_map_bytes(M); }

extern "C" int mvr_brick_map_build_stride(const int32_t* coords, int64_t M, int stride, void* ws, size_t ws_bytes,
                                          hipStream_t s) {
  if (M < 0 || !ws || ws_bytes < brick_map_bytes(M) || stride <= 0 || (stride & (stride - 1)) || stride > (1 << 12) ||
      (M > 0 && !coords))
    return MVR_EINVAL;
  const int t = __builtin_ctz((unsigned)stride);
  BrickView v = brick_view(ws, M);
  int32_t* slot_of = v.rows + (M > 0 ? M : 1) * 64;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)v.h.cap * 12 + M * 40.0, s);
  if (hipMemsetAsync(v.count, 0, 16, s) != hipSuccess) return MVR_ELAUNCH;
  hipLaunchKernelGGL(hash_clear_kernel, dim3(nblk((int64_t)v.h.cap)), dim3(256), 0, s, v.h, -1);
  if (M > 0) {
    const int4* c = reinterpret_cast<const int4*>(coords);
    hipLaunchKernelGGL(brick_insert_kernel, dim3(nblk(M)), dim3(256), 0, s, c, M, v.h, t);
    hipLaunchKernelGGL(brick_ids_kernel, dim3(nblk(M)), dim3(256), 0, s, c, M, v.h, v.count, slot_of, v.bcoord, t);
    hipLaunchKernelGGL(brick_rows_init_kernel, dim3((unsigned)std::min<int64_t>(1024, nblk(M * 16))), dim3(256), 0, s,
                       v.rows, v.count);
    hipLaunchKernelGGL(brick_fill_kernel, dim3(nblk(M)), dim3(256), 0, s, c, M, v.h, slot_of, v.rows, t);
  }
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_brick_map_build(const int32_t* coords, int64_t M, void* ws, size_t ws_bytes, hipStream_t s) {
  return mvr_brick_map_build_stride(coords, M, 1, ws, ws_bytes, s);
}

extern "C" int mvr_spconv_c1_x(const int32_t* out_coords, int64_t Mout, const void* in_bricks, int64_t Min,
                               size_t in_bricks_bytes, const float* feat, int ksize, int step, const float* W, int Cout,
                               mvr_bn_p bn, float bn_eps, int relu, float* out, int64_t ldout, uint16_t* out_planes,
                               hipStream_t s) {
  if (Mout < 0 || (ksize & 1) == 0 || step <= 0 || Min < 0) return MVR_EINVAL;
  if (Mout == 0 && (out_coords || Min == 0)) return MVR_OK;   // no output rows: NULL pointers allowed
  if (!in_bricks || !feat || !W || !out) return MVR_EINVAL;
  if (out_planes && (out_coords || (reinterpret_cast<uintptr_t>(out_planes) & 1))) return MVR_EINVAL;   // bricks only
  if (Cout != 32) return MVR_EINVAL;  // FCGF conv1: 1 -> CHANNELS[1] = 32 (fcgf.py:118-125)
  if (in_bricks_bytes < brick_map_bytes(Min)) return MVR_EINVAL;
  if (!out_coords) {   // the output set is the brick map's own set: output row o = input row o
    if (Mout != Min || step != 1 || ksize != C1_KSZ || ldout < 32) return MVR_EINVAL;
    if (Mout == 0) return MVR_OK;
    BrickView v = brick_view(const_cast<void*>(in_bricks), Min);
    ProfScope prof(PK_SPCONV, 2.0 * Mout * C1_K * Cout, (double)Mout * (16 + Cout * 4), s);
    const int grid = (int)std::min<int64_t>(256, (Mout + 63) / 64);
    hipLaunchKernelGGL(spconv_c1_brick_kernel, dim3(grid), dim3(512), 0, s, v, feat, W, bn, bn_eps, relu, out,
                       ldout, out_planes);
    MVR_CHECK_LAUNCH();
    return MVR_OK;
  }
  if (Mout == 0) return MVR_OK;
  BrickView v = brick_view(const_cast<void*>(in_bricks), Min);
  const int K = ksize * ksize * ksize;
  const size_t lds = (size_t)K * (Cout + 1) * sizeof(float);
  if (lds > 160 * 1024) return MVR_EINVAL;
  ProfScope prof(PK_SPCONV, 2.0 * Mout * K * Cout, (double)Mout * (16 + Cout * 4), s);
  hipLaunchKernelGGL(spconv_c1_kernel<32>, dim3(nblk(Mout)), dim3(256), lds, s,
                     reinterpret_cast<const int4*>(out_coords), Mout, v, feat, ksize, step, W, bn, bn_eps, relu, out,
                     ldout);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

extern "C" int mvr_spconv_c1(const int32_t* out_coords, int64_t Mout, const void* in_bricks, int64_t Min,
                             size_t in_bricks_bytes, const float* feat, int ksize, int step, const float* W, int Cout,
                             mvr_bn_p bn, float bn_eps, int relu, float* out, int64_t ldout, hipStream_t s) {
  return mvr_spconv_c1_x(out_coords, Mout, in_bricks, Min, in_bricks_bytes, feat, ksize, step, W, Cout, bn, bn_eps,
                         relu, out, ldout, nullptr, s);
}

extern "C" int mvr_l2norm_rows(float* x, int64_t M, int C, int64_t ld, hipStream_t s) {
  if (M < 0 || C <= 0 || ld < C) return MVR_EINVAL;
  if (M == 0) return MVR_OK;
  if (!x) return MVR_EINVAL;
  if (C == 32 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0)
    hipLaunchKernelGGL(l2norm_rows32_kernel, dim3((unsigned)((M * 8 + 255) / 256)), dim3(256), 0, s, x, M, ld);
  else
    hipLaunchKernelGGL(l2norm_rows_kernel, dim3(nblk(M)), dim3(256), 0, s, x, M, C, ld);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

// Order the output rows of kernel maps by their active-offset mask, then (out_coords given) fragment and Morton
// code: one stable LSD radix sort (radix.hip, hand-written onesweep) over the keys of ALL the maps of the call, the
// map index in the top key bits, so n maps cost one sort (a control-block clear, a histogram and 8 digit passes)
// instead of one each.  perm_out: int32 [sum M_j]; map j's order is perm_out[start_j : start_j + M_j) (start_j =
// M_0 + ... + M_{j-1}), local row indices.  Workspace: mvr_kernel_map_orders_bytes(total rows).
extern "C" size_t mvr_kernel_map_orders_bytes(int64_t total) { return radix_ws_bytes(total); }

extern "C" int mvr_kernel_map_orders(int n_maps, const int32_t* const* nbr, const int32_t* const* out_coords,
                                     const int* steps, const int64_t* Mo, int K, int32_t* perm_out, void* ws,
                                     size_t ws_bytes, hipStream_t s) {
  if (n_maps <= 0 || n_maps > ORDER_MAX_MAPS || !Mo || K < 0 || K > 27) return MVR_EINVAL;
  if ((!nbr) != (K == 0) || (!nbr && !out_coords)) return MVR_EINVAL;   // K = 0, nbr NULL: coordinate orders
  OrderMaps m{};
  m.n = n_maps;
  m.K = K;
  m.jshift = nbr ? 59 : 32;
  m.start[0] = 0;
  for (int j = 0; j < n_maps; ++j) {
    const int32_t* c = out_coords ? out_coords[j] : nullptr;
    if (Mo[j] < 0 || (Mo[j] > 0 && nbr && !nbr[j]) || (c && (!steps || steps[j] <= 0)) || (!nbr && Mo[j] > 0 && !c))
      return MVR_EINVAL;
    m.nbr[j] = nbr ? nbr[j] : nullptr;
    m.coords[j] = reinterpret_cast<const int4*>(c);
    m.step[j] = c ? steps[j] : 1;
    m.start[j + 1] = m.start[j] + Mo[j];
  }
  const int64_t total = m.start[n_maps];
  if (total > (int64_t)(1 << 30) - 1) return MVR_EINVAL;
  if (total == 0) return MVR_OK;   // every map empty: perm_out and ws may be NULL
  if (!perm_out || !ws || ws_bytes < radix_ws_bytes(total)) return MVR_EINVAL;
  ProfScope prof(PK_SPARSE_MISC, 0.0, (double)total * (4.0 * K + 16 + 8 * 24 + 4), s);
  RadixWs w = radix_ws(ws, total);
  hipLaunchKernelGGL(order_keys_kernel, dim3(nblk(total)), dim3(256), 0, s, m, w.ka, w.va);
  int bits = 32 + K;                                   // mask above bit 32, fragment + Morton below
  if (n_maps > 1) bits = m.jshift + (32 - __builtin_clz((unsigned)(n_maps - 1)));   // + the map index
  return radix_sort(w, bits, perm_out, s);
}

// one map (the same order as mvr_kernel_map_orders with n_maps = 1).  Workspace: mvr_kernel_map_order_bytes(Mo).
extern "C" size_t mvr_kernel_map_order_bytes(int64_t Mo) { return radix_ws_bytes(Mo); }

extern "C" int mvr_kernel_map_order(const int32_t* nbr, const int32_t* out_coords, int step, int64_t Mo, int K,
                                    int32_t* perm, void* ws, size_t ws_bytes, hipStream_t s) {
  if (Mo < 0 || K <= 0 || K > 27 || (out_coords && step <= 0)) return MVR_EINVAL;
  if (Mo == 0) return MVR_OK;
  if (!nbr || !perm) return MVR_EINVAL;
  return mvr_kernel_map_orders(1, &nbr, &out_coords, &step, &Mo, K, perm, ws, ws_bytes, s);
}
