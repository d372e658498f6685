// Stable LSD radix sort of (uint64 key, int32 value) pairs on gfx950 (radix.hip): the row order of the sparse
// convs' kernel maps (mvr_kernel_map_order[s]).  Onesweep form: one histogram launch for every pass, then one
// launch per 8-bit digit that ranks each 4096-key tile in LDS (wave ballots, stable), finds the tile's global
// offsets by decoupled look-back over the tiles before it, and scatters.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mvr {

constexpr int RADIX_BITS = 8;
constexpr int RADIX_BINS = 1 << RADIX_BITS;
constexpr int RADIX_MAX_PASSES = 8;
constexpr int RADIX_THREADS = 256;                          // 4 waves; one digit per thread in the tile phases
constexpr int RADIX_KPT = 16;                               // keys per thread
constexpr int RADIX_TILE = RADIX_THREADS * RADIX_KPT;       // 4096 keys per tile

struct RadixWs {
  uint64_t* ka;      // keys (the caller writes them before radix_sort), ping
  uint64_t* kb;      // pong
  int32_t* va;       // values, ping (the caller writes them)
  int32_t* vb;       // pong
  uint32_t* ctrl;    // histograms [passes][bins], tile tickets [passes], look-back [passes][tiles][bins]
  size_t ctrl_bytes;
  int64_t n;
  int64_t tiles;
};

size_t radix_ws_bytes(int64_t n);
RadixWs radix_ws(void* ws, int64_t n);
// sort ws.ka / ws.va (n pairs) on key bits [0, bits) ascending, stable; the sorted values land in vals_out
// (which may not alias the workspace).  Launches: one control-block clear, one histogram, ceil(bits / 8) passes.
int radix_sort(const RadixWs& w, int bits, int32_t* vals_out, hipStream_t s);

// Exclusive prefix sum of n int32 values (the total must fit in int32): reduce-then-scan over 4096-value tiles, three
// launches (tile sums, one workgroup scanning them, the tiles' scans with their offsets).  in and out may alias.
// Workspace: scan_ws_bytes(n).
constexpr int SCAN_TILE = RADIX_THREADS * 16;
size_t scan_ws_bytes(int64_t n);
int excl_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace mvr
