// Internal helpers shared by the ftmi HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ftmi.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define FTMI_CHECK_LAUNCH()                         \
  do {                                              \
    hipError_t e__ = hipGetLastError();             \
    if (e__ != hipSuccess) return (int)e__;         \
  } while (0)

static inline bool ftmi_aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

static inline hipStream_t ftmi_hs(ftmi_stream_t s) { return (hipStream_t)s; }

// CUs a persistent grid may count on: the device's, or fewer when a test lowers it
// (ftmi_set_resident_cu_limit; defined in seq.hip)
__attribute__((visibility("hidden"))) int ftmi_resident_cus(void);

// Persistent-launch guard (rnn_bidir, rnn_gemv, highway_stack_spread, wavernn: workgroups
// that wait on each other).  Every workgroup of the grid must be resident at once, so the
// kernel's occupancy at this block size / LDS times the CU count must cover the grid;
// otherwise the caller returns FTMI_E_UNSUPPORTED before launching anything (instead of
// relying on a spin bound to turn the deadlock into a status bit).
static inline int ftmi_resident_ok(const void *kernel, int grid, int block, size_t smem) {
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, smem) != hipSuccess) {
    (void)hipGetLastError();  // a failed query must not surface in the caller's next HIP call
    return FTMI_E_UNSUPPORTED;
  }
  if (per <= 0) return FTMI_E_UNSUPPORTED;
  return (int64_t)per * ftmi_resident_cus() >= grid ? FTMI_OK : FTMI_E_UNSUPPORTED;
}

__device__ __forceinline__ float ftmi_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
