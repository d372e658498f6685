// Opt-in per-kernel-class timing with HIP events on the launching stream
// (bench.py reads it to price the dominant kernel against its roofline).
#pragma once
#include <hip/hip_runtime.h>

namespace mvr {
enum ProfKind : int {
  PK_CONV_PTS = 0,   // OANet 1x1 conv over points (M=C, K=C or 2C, N=points)
  PK_EMBED = 1,      // diff_pool / diff_unpool embedding conv (M=clusters)
  PK_POOL = 2,       // diff_pool matmul (K=points)
  PK_UNPOOL = 3,     // diff_unpool matmul (K=clusters)
  PK_OAFILTER = 4,   // OAFilter GEMMs (N=clusters)
  PK_SMALL = 5,      // finalize / head / misc
  PK_PROCRUSTES = 6,
  PK_FEAT_NN = 7,
  PK_SPCONV = 8,     // FCGF sparse conv
  PK_SPARSE_MISC = 9,
  PK_POINTCN = 10,   // fused PointCN (pointcn.hip)
  PK_COUNT = 16
};
bool prof_on(int kind);
void prof_begin(int kind, double flops, double bytes, hipStream_t s);
void prof_end(int kind, hipStream_t s);
struct ProfScope {
  int k; hipStream_t s; bool on;
  ProfScope(int kind, double flops, double bytes, hipStream_t st) : k(kind), s(st), on(prof_on(kind)) {
    if (on) prof_begin(kind, flops, bytes, st);
  }
  ~ProfScope() { if (on) prof_end(k, s); }
};
}  // namespace mvr
