#include "prof.hpp"

#include <stdlib.h>

#include <mutex>
#include <vector>

#include "common.hpp"

namespace mvr {

// PMC attribution markers (MVR_PROF_MARK=1): an empty dispatch before and after every profiled
// region, so that rocprofv3's per-dispatch counters can be assigned to the launch sequence
// (tools/pmc_traffic.py) by position between markers rather than by kernel names.
__global__ void mvr_prof_mark_begin_kernel() {}
__global__ void mvr_prof_mark_end_kernel() {}

namespace {
struct Rec { int kind; hipEvent_t a, b; double flops, bytes; };
std::mutex mu;
bool enabled = false;
bool marks = false;
uint32_t kind_mask = ~0u;   // kinds that get events (mvr_prof_mask)
std::vector<Rec> recs;
std::vector<hipEvent_t> pool;
std::vector<int> open_idx;  // stack of records awaiting their end event
std::vector<int> seq_kind;  // launch order since mvr_prof_set (PMC attribution, tools/pmc_traffic.py)
std::vector<double> seq_bytes;
hipEvent_t get_ev() {
  if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}
double tot_ms[PK_COUNT], tot_fl[PK_COUNT], tot_by[PK_COUNT];
long long tot_n[PK_COUNT];
void drain() {
  for (auto& r : recs) {
    if (!r.b) continue;
    float ms = 0.f;
    (void)hipEventSynchronize(r.b);
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    tot_ms[r.kind] += ms; tot_fl[r.kind] += r.flops; tot_by[r.kind] += r.bytes; tot_n[r.kind] += 1;
    pool.push_back(r.a); pool.push_back(r.b);
  }
  recs.clear();
  open_idx.clear();
}
}  // namespace

bool prof_on(int kind) { return enabled && ((kind_mask >> kind) & 1u); }
void prof_begin(int kind, double flops, double bytes, hipStream_t s) {
  std::lock_guard<std::mutex> g(mu);
  Rec r{kind, get_ev(), nullptr, flops, bytes};
  if (marks) hipLaunchKernelGGL(mvr_prof_mark_begin_kernel, dim3(1), dim3(64), 0, s);
  (void)hipEventRecord(r.a, s);
  seq_kind.push_back(kind);
  seq_bytes.push_back(bytes);
  recs.push_back(r);
  open_idx.push_back((int)recs.size() - 1);
}
void prof_end(int kind, hipStream_t s) {
  std::lock_guard<std::mutex> g(mu);
  if (open_idx.empty()) return;
  Rec& r = recs[open_idx.back()];
  open_idx.pop_back();
  r.b = get_ev();
  (void)hipEventRecord(r.b, s);
  if (marks) hipLaunchKernelGGL(mvr_prof_mark_end_kernel, dim3(1), dim3(64), 0, s);
  (void)kind;
}
}  // namespace mvr

using namespace mvr;

#ifndef MVR_SRC_HASH
#define MVR_SRC_HASH "unknown"
#endif
// The build's source identity (csrc/Makefile: sha256 of csrc/*.hip, *.hpp, mvreg.h and the variant flags): recorded
// by tools/pmc_traffic.py with the counters it measured, so bench.py never prices this library with the counters of
// another build.
extern "C" int mvr_source_hash(char* buf, size_t cap) {
  const char* h = MVR_SRC_HASH;
  size_t n = 0;
  while (h[n]) ++n;
  if (!buf || cap <= n) return (int)n + 1;
  for (size_t i = 0; i <= n; ++i) buf[i] = h[i];
  return MVR_OK;
}

extern "C" int mvr_prof_set(int on) {
  std::lock_guard<std::mutex> g(mu);
  drain();
  for (int k = 0; k < PK_COUNT; ++k) { tot_ms[k] = tot_fl[k] = tot_by[k] = 0; tot_n[k] = 0; }
  seq_kind.clear();
  seq_bytes.clear();
  enabled = on != 0;
  const char* m = getenv("MVR_PROF_MARK");
  marks = enabled && m && m[0] == '1';
  return MVR_OK;
}

// Kinds recorded while enabled (bit k = kind k; default all): the bench times only the dominant
// class inside its timed region, so the other launches carry no event records.
extern "C" int mvr_prof_mask(unsigned mask) {
  std::lock_guard<std::mutex> g(mu);
  kind_mask = mask;
  return MVR_OK;
}

// Per-kind totals since mvr_prof_set: device milliseconds, launches, algorithmic flops and bytes.
extern "C" int mvr_prof_get(int kind, double* ms, long long* launches, double* flops, double* bytes) {
  if (kind < 0 || kind >= PK_COUNT) return MVR_EINVAL;
  std::lock_guard<std::mutex> g(mu);
  drain();
  if (ms) *ms = tot_ms[kind];
  if (launches) *launches = tot_n[kind];
  if (flops) *flops = tot_fl[kind];
  if (bytes) *bytes = tot_by[kind];
  return MVR_OK;
}

// Launch sequence since mvr_prof_set(1): kind and algorithmic bytes of each profiled launch, in
// order (up to cap entries); returns the number of launches recorded.
extern "C" int mvr_prof_seq(int* kinds, double* bytes, int cap) {
  std::lock_guard<std::mutex> g(mu);
  const int n = (int)seq_kind.size();
  for (int i = 0; i < n && i < cap; ++i) {
    if (kinds) kinds[i] = seq_kind[i];
    if (bytes) bytes[i] = seq_bytes[i];
  }
  return n;
}
