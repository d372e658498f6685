// The library's two process-wide entry points (knobs.hpp): the operand arithmetic of every kernel that has a
// choice, and test-only forcing of fallback paths.
#include "common.hpp"
#include "knobs.hpp"
#include "mvreg.h"

namespace mvr {
int g_force[FORCE_COUNT] = {};
}

extern "C" int mvr_set_math(int mode) {
  using namespace mvr;
  const int prev = g_spconv_h ? 1 : 0;
  const int h = mode == 1 ? 1 : 0;
  g_gemm_h = g_pconv_h = g_attn_h = g_spconv_h = h;
  if (g_feat_nn_fast) g_feat_nn_fast = h ? 2 : 1;
  return prev;
}

extern "C" int mvr_debug_force(int what, int value) {
  using namespace mvr;
  if (what == FORCE_FEAT_NN_ONLINE) {   // kept with the arithmetic: 0 <-> the mode's fast path
    const int prev = g_feat_nn_fast ? 0 : 1;
    g_feat_nn_fast = value ? 0 : (g_spconv_h ? 2 : 1);
    return prev;
  }
  if (what < 0 || what >= FORCE_COUNT) return MVR_EINVAL;
  const int prev = g_force[what];
  g_force[what] = value ? 1 : 0;
  return prev;
}
