// Host-side random interest-point sampling (lib/layers.py:145-148, Sampler 'rand'):
//
//   for each fragment b (in order):  idx_b = np.random.choice(np.arange(start_b, start_b + n_b), tgt,
//                                                             replace=False)
//
// on numpy's global legacy RandomState, reproduced draw for draw so that seeded runs select exactly the
// reference's points.  numpy implements choice(n, k, replace=False) as permutation(n)[:k], i.e. a
// Fisher-Yates shuffle of arange(n) (i = n-1 .. 1: j = random_interval(i), swap) whose bounded draws
// take 32-bit MT19937 outputs masked to the smallest 2^k - 1 >= i and rejected while > i.  numpy's own
// loop costs ~0.4 ms per 20k-point fragment (byte-wise swaps through memcpy); this one runs the same
// draws with 8-byte swaps.  The caller passes the RandomState's MT19937 key/pos (np.random.get_state())
// and writes the advanced state back (np.random.set_state()).  Not a GPU kernel: the draws are one
// sequential stream.
#include <stdint.h>

#include "common.hpp"
#include "mvreg.h"

namespace {

constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_A = 0x9908b0dfu, MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu;

struct Mt {
  uint32_t* key;
  int pos;
  void gen() {
    int i = 0;
    uint32_t y;
    for (; i < MT_N - MT_M; ++i) {
      y = (key[i] & MT_UPPER) | (key[i + 1] & MT_LOWER);
      key[i] = key[i + MT_M] ^ (y >> 1) ^ ((0u - (y & 1u)) & MT_A);
    }
    for (; i < MT_N - 1; ++i) {
      y = (key[i] & MT_UPPER) | (key[i + 1] & MT_LOWER);
      key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((0u - (y & 1u)) & MT_A);
    }
    y = (key[MT_N - 1] & MT_UPPER) | (key[0] & MT_LOWER);
    key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & MT_A);
    pos = 0;
  }
  uint32_t next32() {
    if (pos == MT_N) gen();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

}  // namespace

// key: uint32[624], *pos: the RandomState's MT19937 state (advanced in place).  counts[B]: points per
// fragment (fragment b's rows start at the sum of the previous counts); out: int64 [B][tgt] global row
// indices; ws: int64 scratch of max(counts) elements.  Requires tgt <= counts[b] (replace=False).
extern "C" int mvr_sample_rand_mt19937(uint32_t* key, int32_t* pos, const int64_t* counts, int B, int tgt,
                                       int64_t* out, int64_t* ws) {
  if (B < 0 || tgt < 0) return MVR_EINVAL;
  if (B == 0) return MVR_OK;   // no fragments: no draws (NULL pointers allowed)
  if (!key || !pos || !counts || !out || !ws || *pos < 0 || *pos > MT_N) return MVR_EINVAL;
  for (int b = 0; b < B; ++b)
    if (counts[b] < tgt || counts[b] > 0xffffffffLL) return MVR_EINVAL;
  Mt mt{key, *pos};
  int64_t start = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t n = counts[b];
    for (int64_t i = 0; i < n; ++i) ws[i] = i;
    // one draw per iteration, branch-free: a rejected draw (masked value > i) swaps ws[i] with itself and
    // keeps i; the mask (smallest all-ones value >= i) follows i
    int64_t i = n - 1;
    while (i >= 1) {
      const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)i);
      const int64_t j = (int64_t)(mt.next32() & mask);
      const int64_t acc = j <= i;
      const int64_t jj = acc ? j : i;
      const int64_t t = ws[jj];
      ws[jj] = ws[i];
      ws[i] = t;
      i -= acc;
    }
    int64_t* o = out + (int64_t)b * tgt;
    for (int k = 0; k < tgt; ++k) o[k] = start + ws[k];
    start += n;
  }
  *pos = mt.pos;
  return MVR_OK;
}
