// Diagnostic helper (tools only, not the product library): a HIP stream restricted to a CU mask, for
// tools/diag_cumask.py.  hipcc --offload-arch=gfx950 -shared -fPIC tools/cumask.hip -o tools/vsp/libcumask.so
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

extern "C" int mvr_diag_stream_cu_mask(const uint32_t* mask, int words, void** out) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return -1;
  *out = (void*)s;
  return 0;
}
