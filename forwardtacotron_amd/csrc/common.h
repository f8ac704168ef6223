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

__device__ __forceinline__ float ftmi_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
