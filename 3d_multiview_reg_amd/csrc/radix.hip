// Stable LSD radix sort of (uint64 key, int32 value) pairs, hand-written for gfx950 (wave64): the kernel-map row
// orders of the FCGF sparse convs (sparse.hip mvr_kernel_map_order[s]).  Onesweep structure:
//   * radix_hist_kernel   one pass over the keys: the digit histograms of EVERY pass (LDS, then global atomics);
//   * radix_pass_kernel   one launch per 8-bit digit.  A workgroup takes the next 4096-key tile (atomic ticket, so
//                         a tile only ever waits for tiles that started before it), loads it coalesced (wave w:
//                         keys [w * 1024, (w + 1) * 1024) of the tile, round r = 64 consecutive keys), ranks every
//                         key stably inside its wave (8 ballots give the lanes of the round that share its digit;
//                         one LDS atomic per digit group and round keeps the wave's running count), adds the
//                         counts of the waves before it, then finds the tile's global offset per digit by
//                         decoupled look-back over the tiles before it (a 32-bit word per (tile, digit): 2 status
//                         bits + count, device-coherent loads / stores, no fences) and scatters keys and values.
//                         The last pass writes the values only.
// Keys of equal value keep their input order, so the result equals any stable sort of the same keys.
#include "common.hpp"
#include "radix.hpp"

namespace mvr {

namespace {
constexpr uint32_t LB_AGG = 1u << 30;     // the tile's own count is published
constexpr uint32_t LB_INC = 2u << 30;     // the inclusive prefix (all tiles up to this one) is published
constexpr uint32_t LB_VAL = (1u << 30) - 1;
constexpr int CTRL_HIST = 0;                                      // [passes][bins]
constexpr int CTRL_TICKET = RADIX_MAX_PASSES * RADIX_BINS;        // [passes], padded to 64 words
constexpr int CTRL_LOOK = CTRL_TICKET + 64;                       // [passes][tiles][bins]

__device__ __forceinline__ uint32_t ld_coherent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coherent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive prefix sum over the 256 threads of the workgroup (one value each); `sh` = 4 words of LDS
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < w; ++i) off += sh[i];
  __syncthreads();
  return off + x - v;
}
}  // namespace

// digit mask of pass p of a `bits`-bit sort: the last pass of a bit count that is not a digit multiple keeps only the
// key bits below `bits` (key bits at or above it never decide the order)
__device__ __host__ __forceinline__ uint32_t radix_dmask(int bits, int p) {
  const int rem = bits - RADIX_BITS * p;
  return rem >= RADIX_BITS ? (uint32_t)(RADIX_BINS - 1) : ((1u << rem) - 1u);
}

__global__ __launch_bounds__(RADIX_THREADS) void radix_hist_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                                   int bits, uint32_t* __restrict__ hist) {
  const int npass = (bits + RADIX_BITS - 1) / RADIX_BITS;
  __shared__ uint32_t h[RADIX_MAX_PASSES * RADIX_BINS];
  for (int i = threadIdx.x; i < RADIX_MAX_PASSES * RADIX_BINS; i += RADIX_THREADS) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * RADIX_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * RADIX_THREADS) {
    const uint64_t k = keys[i];
    for (int p = 0; p < npass; ++p) atomicAdd(&h[p * RADIX_BINS + (int)((k >> (RADIX_BITS * p)) & radix_dmask(bits, p))], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < npass * RADIX_BINS; i += RADIX_THREADS)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

template <bool LAST>
__global__ __launch_bounds__(RADIX_THREADS) void radix_pass_kernel(const uint64_t* __restrict__ kin,
                                                                   const int32_t* __restrict__ vin,
                                                                   uint64_t* __restrict__ kout,
                                                                   int32_t* __restrict__ vout, int64_t n, int shift,
                                                                   uint32_t dmask, const uint32_t* __restrict__ hist,
                                                                   uint32_t* ticket, uint32_t* look) {
  __shared__ uint32_t wcnt[RADIX_THREADS / 64][RADIX_BINS];   // per wave: running digit counts, then offsets
  __shared__ uint32_t dbase[RADIX_BINS];                      // global offset of the tile's first key per digit
  __shared__ uint32_t sh_scan[4];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  for (int i = tid; i < (RADIX_THREADS / 64) * RADIX_BINS; i += RADIX_THREADS) (&wcnt[0][0])[i] = 0;
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t base = tile * RADIX_TILE + (int64_t)w * (64 * RADIX_KPT) + lane;

  uint64_t key[RADIX_KPT];
  int32_t val[RADIX_KPT];
#pragma unroll
  for (int r = 0; r < RADIX_KPT; ++r) {
    const int64_t i = base + r * 64;
    key[r] = i < n ? kin[i] : ~0ull;
    val[r] = i < n ? vin[i] : 0;
  }
  // stable rank of every key among the keys of its digit in this wave (round order = input order)
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t rank[RADIX_KPT];
#pragma unroll
  for (int r = 0; r < RADIX_KPT; ++r) {
    const bool valid = base + r * 64 < n;
    const uint32_t d = (uint32_t)(key[r] >> shift) & dmask;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RADIX_BITS; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    const uint32_t rk = (uint32_t)__popcll(peers & lt);
    const int leader = peers ? __builtin_ctzll(peers) : lane;
    uint32_t pre = 0;
    if (valid && rk == 0) pre = atomicAdd(&wcnt[w][d], (uint32_t)__popcll(peers));
    pre = __shfl(pre, leader, 64);
    rank[r] = pre + rk;
  }
  __syncthreads();
  // thread d: the waves' exclusive offsets for digit d, the tile's count, its global offset (look-back)
  const int d = tid;
  uint32_t tile_cnt = 0;
#pragma unroll
  for (int v = 0; v < RADIX_THREADS / 64; ++v) {
    const uint32_t c = wcnt[v][d];
    wcnt[v][d] = tile_cnt;
    tile_cnt += c;
  }
  uint32_t* lk = look + tile * RADIX_BINS + d;
  uint32_t prefix = 0;
  if (tile == 0) {
    st_coherent(lk, LB_INC | tile_cnt);
  } else {
    st_coherent(lk, LB_AGG | tile_cnt);
    for (int64_t j = tile - 1; j >= 0;) {
      const uint32_t e = ld_coherent(look + j * RADIX_BINS + d);
      if ((e & ~LB_VAL) == 0) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      prefix += e & LB_VAL;
      if (e & LB_INC) break;
      --j;
    }
    st_coherent(lk, LB_INC | (prefix + tile_cnt));
  }
  dbase[d] = block_excl_scan(hist[d], sh_scan) + prefix;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RADIX_KPT; ++r) {
    if (base + r * 64 < n) {
      const uint32_t dg = (uint32_t)(key[r] >> shift) & dmask;
      const uint32_t pos = dbase[dg] + wcnt[w][dg] + rank[r];
      if (!LAST) kout[pos] = key[r];
      vout[pos] = val[r];
    }
  }
}

// ---------------------------------------------------------------------------- exclusive scan (overlap gate)
namespace {
__global__ __launch_bounds__(RADIX_THREADS) void scan_tile_sum_kernel(const int32_t* __restrict__ in, int64_t n,
                                                                      int32_t* __restrict__ tsum) {
  __shared__ uint32_t sh[4];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  uint32_t v = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {   // coalesced: round r reads 256 consecutive values
    const int64_t i = base + r * RADIX_THREADS + threadIdx.x;
    if (i < n) v += (uint32_t)in[i];
  }
  const uint32_t ex = block_excl_scan(v, sh);
  if (threadIdx.x == RADIX_THREADS - 1) tsum[blockIdx.x] = (int32_t)(ex + v);
}

// one workgroup: tile sums -> their exclusive prefix, in place
__global__ __launch_bounds__(RADIX_THREADS) void scan_tile_prefix_kernel(int32_t* tsum, int64_t ntiles) {
  __shared__ uint32_t sh[4];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b = 0; b < ntiles; b += RADIX_THREADS) {
    const int64_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? (uint32_t)tsum[i] : 0u;
    const uint32_t c = carry;
    const uint32_t ex = block_excl_scan(v, sh);
    if (i < ntiles) tsum[i] = (int32_t)(c + ex);
    __syncthreads();
    if (threadIdx.x == RADIX_THREADS - 1) carry = c + ex + v;
    __syncthreads();
  }
}

// each thread scans 16 consecutive values of the tile (staged through LDS so the global reads stay coalesced)
__global__ __launch_bounds__(RADIX_THREADS) void scan_tile_kernel(const int32_t* in, int32_t* out, int64_t n,
                                                                  const int32_t* __restrict__ tpre) {
  __shared__ int32_t tile[SCAN_TILE + SCAN_TILE / 32];   // +1 word per 32: conflict-free column reads
  __shared__ uint32_t sh[4];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  auto at = [](int j) { return j + (j >> 5); };
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = r * RADIX_THREADS + threadIdx.x;
    tile[at(j)] = base + j < n ? in[base + j] : 0;
  }
  __syncthreads();
  uint32_t loc[16], s = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    loc[r] = s;
    s += (uint32_t)tile[at(threadIdx.x * 16 + r)];
  }
  const uint32_t off = (uint32_t)tpre[blockIdx.x] + block_excl_scan(s, sh);
#pragma unroll
  for (int r = 0; r < 16; ++r) tile[at(threadIdx.x * 16 + r)] = (int32_t)(off + loc[r]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = r * RADIX_THREADS + threadIdx.x;
    if (base + j < n) out[base + j] = tile[at(j)];
  }
}
}  // namespace

size_t scan_ws_bytes(int64_t n) { return ((size_t)((n + SCAN_TILE - 1) / SCAN_TILE + 1) * 4 + 255) & ~(size_t)255; }

int excl_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes, hipStream_t s) {
  if (n < 0) return MVR_EINVAL;
  if (n == 0) return MVR_OK;
  if (!in || !out || !ws || ws_bytes < scan_ws_bytes(n)) return MVR_EINVAL;
  const int64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  int32_t* tsum = reinterpret_cast<int32_t*>(ws);
  hipLaunchKernelGGL(scan_tile_sum_kernel, dim3((unsigned)nt), dim3(RADIX_THREADS), 0, s, in, n, tsum);
  hipLaunchKernelGGL(scan_tile_prefix_kernel, dim3(1), dim3(RADIX_THREADS), 0, s, tsum, nt);
  hipLaunchKernelGGL(scan_tile_kernel, dim3((unsigned)nt), dim3(RADIX_THREADS), 0, s, in, out, n, tsum);
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
static int64_t radix_tiles(int64_t n) { return (n + RADIX_TILE - 1) / RADIX_TILE; }
static size_t ctrl_words(int64_t n) {
  return (size_t)CTRL_LOOK + (size_t)RADIX_MAX_PASSES * (size_t)(radix_tiles(n) > 0 ? radix_tiles(n) : 1) * RADIX_BINS;
}

size_t radix_ws_bytes(int64_t n) {
  const size_t m = (size_t)(n > 0 ? n : 1);
  return 2 * align256(m * 8) + 2 * align256(m * 4) + align256(ctrl_words(n) * 4) + 256;
}

RadixWs radix_ws(void* ws, int64_t n) {
  const size_t m = (size_t)(n > 0 ? n : 1);
  char* p = reinterpret_cast<char*>(((uintptr_t)ws + 255) & ~(uintptr_t)255);
  RadixWs w;
  w.ka = reinterpret_cast<uint64_t*>(p); p += align256(m * 8);
  w.kb = reinterpret_cast<uint64_t*>(p); p += align256(m * 8);
  w.va = reinterpret_cast<int32_t*>(p); p += align256(m * 4);
  w.vb = reinterpret_cast<int32_t*>(p); p += align256(m * 4);
  w.ctrl = reinterpret_cast<uint32_t*>(p);
  w.ctrl_bytes = ctrl_words(n) * 4;
  w.n = n;
  w.tiles = radix_tiles(n);
  return w;
}

int radix_sort(const RadixWs& w, int bits, int32_t* vals_out, hipStream_t s) {
  if (w.n < 0 || w.n > (int64_t)LB_VAL || bits <= 0 || bits > 64) return MVR_EINVAL;
  if (w.n == 0) return MVR_OK;
  if (!vals_out) return MVR_EINVAL;
  const int npass = (bits + RADIX_BITS - 1) / RADIX_BITS;
  const size_t clear = ((size_t)CTRL_LOOK + (size_t)npass * w.tiles * RADIX_BINS) * 4;
  if (hipMemsetAsync(w.ctrl, 0, clear, s) != hipSuccess) return MVR_ELAUNCH;
  const int hgrid = (int)std::min<int64_t>(w.tiles, 512);
  hipLaunchKernelGGL(radix_hist_kernel, dim3(hgrid), dim3(RADIX_THREADS), 0, s, w.ka, w.n, bits, w.ctrl + CTRL_HIST);
  const uint64_t* kin = w.ka;
  const int32_t* vin = w.va;
  for (int p = 0; p < npass; ++p) {
    uint64_t* kout = (p & 1) ? w.ka : w.kb;
    int32_t* vout = (p & 1) ? w.va : w.vb;
    uint32_t* look = w.ctrl + CTRL_LOOK + (size_t)p * w.tiles * RADIX_BINS;
    if (p + 1 == npass)
      hipLaunchKernelGGL(radix_pass_kernel<true>, dim3((unsigned)w.tiles), dim3(RADIX_THREADS), 0, s, kin, vin,
                         nullptr, vals_out, w.n, RADIX_BITS * p, radix_dmask(bits, p), w.ctrl + CTRL_HIST + p * RADIX_BINS,
                         w.ctrl + CTRL_TICKET + p, look);
    else
      hipLaunchKernelGGL(radix_pass_kernel<false>, dim3((unsigned)w.tiles), dim3(RADIX_THREADS), 0, s, kin, vin,
                         kout, vout, w.n, RADIX_BITS * p, radix_dmask(bits, p), w.ctrl + CTRL_HIST + p * RADIX_BINS,
                         w.ctrl + CTRL_TICKET + p, look);
    kin = kout;
    vin = vout;
  }
  MVR_CHECK_LAUNCH();
  return MVR_OK;
}

}  // namespace mvr

// The sort on its own (any keys, any bit count; tests/test_gpu_radix.py against a stable CPU sort): keys uint64
// [n], values int32 [n] (NULL: the indices 0..n-1) -> vals_out int32 [n] = the values in stable ascending order of
// the keys' bits [0, bits).  Workspace: mvr_radix_sort_pairs_bytes(n).
namespace {
__global__ void radix_load_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ v, int64_t n,
                                  uint64_t* __restrict__ ka, int32_t* __restrict__ va) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ka[i] = k[i];
  va[i] = v ? v[i] : (int32_t)i;
}
}  // namespace

extern "C" size_t mvr_radix_sort_pairs_bytes(int64_t n) { return mvr::radix_ws_bytes(n); }

extern "C" int mvr_radix_sort_pairs(const uint64_t* keys, const int32_t* vals, int64_t n, int bits,
                                    int32_t* vals_out, void* ws, size_t ws_bytes, hipStream_t s) {
  if (n < 0 || bits <= 0 || bits > 64) return MVR_EINVAL;
  if (n == 0) return MVR_OK;   // pointers may be NULL with a zero count (mvreg.h conventions)
  if (!keys || !vals_out || !ws || ws_bytes < mvr::radix_ws_bytes(n)) return MVR_EINVAL;
  mvr::RadixWs w = mvr::radix_ws(ws, n);
  hipLaunchKernelGGL(radix_load_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, keys, vals, n, w.ka, w.va);
  return mvr::radix_sort(w, bits, vals_out, s);
}
