// Process-wide selections of libmvreg_hip.so (knobs.hip): the operand arithmetic (mvr_set_math) and, for tests,
// the forced use of the fallback paths the library keeps for shapes its fast kernels do not cover
// (mvr_debug_force).  Everything else about a launch is a function of its arguments.
#pragma once

namespace mvr {

constexpr int GPU_CUS = 256;   // MI355X: the CUs the persistent grids are sized for

// split-fp16 where a launch has a range flag (1) or split-bf16 everywhere (0); set together by mvr_set_math
extern int g_gemm_h;        // generic GEMM (gemm.hip)
extern int g_pconv_h;       // point convs (pconv.hip)
extern int g_attn_h;        // diff_pool / 4-wave diff_unpool (oan_attn.hip)
extern int g_spconv_h;      // sparse convs with > 64 output channels (spconv.hip)
extern int g_feat_nn_fast;  // feature NN: 1 bounded-shift softmax on split-bf16 distances, 2 on split-fp16, 0 online

// fallback paths forced by mvr_debug_force (tests compare them with the fast paths; all 0 by default)
enum ForcePath : int {
  FORCE_FEAT_NN_ONLINE = 0,   // feature NN: the online softmax only (the fast path's per-workgroup fallback)
  FORCE_GENERIC_GEMM = 1,     // point convs and OAFilter conv2 on the generic GEMM (their kernels' fallback)
  FORCE_UNFUSED_ATTN = 2,     // diff_pool / diff_unpool as embedding GEMM + softmax factors + pooling GEMM
  FORCE_NO_CONV1_FOLD = 3,    // the OANet block's conv1 stored instead of recomputed inside the first PointCN
  FORCE_POOL_NOSPLIT = 4,     // diff_pool without key splits (another fp32 summation order)
  FORCE_UNPOOL8 = 5,          // the 8-wave diff_unpool (clusters > 512) at <= 512 clusters too
  FORCE_ROW_LAYOUT = 6,       // the OANet block's point activations row-major instead of chunk-major
  FORCE_COUNT = 7
};
extern int g_force[FORCE_COUNT];

}  // namespace mvr
