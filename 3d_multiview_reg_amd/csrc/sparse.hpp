// Device hash-table view shared by sparse.hip / spconv.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mvreg.h"

namespace mvr {
constexpr uint64_t EMPTY_KEY = ~0ULL;
constexpr int KEY_BIAS = 1 << 16;           // coordinates in [-65536, 65535] (x, y, z: 17 bits each)
constexpr uint32_t KEY_MASK = (1u << 17) - 1;
constexpr int MAX_BATCH = 4095;             // batch index: 12 bits

struct HashView {
  uint64_t* keys;
  int32_t* vals;
  uint64_t cap;  // power of two
  int32_t* hdr;  // table header (plain tables: word 0 = the home mode, see hash_home); null for brick maps
};

size_t hash_table_bytes(int64_t M);
HashView hash_view(void* table, size_t bytes);
}  // namespace mvr
