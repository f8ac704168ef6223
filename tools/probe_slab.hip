// Prologue probe for the c2 prenet bank's one-launch kernel (conv_bank_halves_kernel): how long
// does each CU take to stage its 73 KB slab (143 rows x 128 channels of the 123 KB input,
// every block reading the same bytes) with and without the weight stream in flight?
//   hipcc -O3 --offload-arch=gfx950 tools/probe_slab.hip -o tools/probe_slab.bin
// us per launch, HIP events over 100 back-to-back launches (warm caches).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int SR = 143, CH = 128, ASL = (4 * SR * 8 + 511) / 512;  // 9 float4 per thread
constexpr int P = 48;  // halves per LDS row (the kernel's SL_P)

// MODE bit 0: slab loads; bit 1: weight loads (18 x 16 B per lane, 139 KB per block);
// bit 2: weights issued BEFORE the slab; bit 3: every block reads its own copy of x
template <int MODE>
__global__ __launch_bounds__(512, 1) void prologue(const float *x, const _Float16 *w, float *out,
                                                   long long *stamps) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[4 * 2 * (SR + 1) * P];
  const int tid = threadIdx.x, b = blockIdx.x, h = (b >> 3) & 1;
  const long long t0 = __builtin_amdgcn_s_memtime();
  const float *xb = x + ((MODE & 8) ? (size_t)b * 120 * 256 : 0);
  f16x8 r[18];
  auto wload = [&]() {
    const _Float16 *wb = w + (size_t)b * (139264 / 2) + (tid >> 6) * 1024 + (tid & 63) * 8;
#pragma unroll
    for (int i = 0; i < 18; ++i) r[i] = *(const f16x8 *)(wb + (size_t)i * 8 * 512);
  };
  if constexpr ((MODE & 2) && (MODE & 4)) wload();
  f32x4 av[ASL];
  if constexpr (MODE & 1) {
#pragma unroll
    for (int i = 0; i < ASL; ++i) {
      const int idx = tid + 512 * i, c = idx / (SR * 8), rem = idx - c * (SR * 8), sr = rem >> 3,
                seg = rem & 7;
      int m = sr - 8;
      m = m < 0 ? 0 : (m >= 120 ? 119 : m);
      av[i] = idx < 4 * SR * 8 ? *(const f32x4 *)(xb + m * 256 + h * 128 + c * 32 + seg * 4)
                               : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  if constexpr ((MODE & 2) && !(MODE & 4)) wload();
  if constexpr (MODE & 1) {
#pragma unroll
    for (int i = 0; i < ASL; ++i) {
      const int idx = tid + 512 * i;
      if (idx >= 4 * SR * 8) break;
      const int c = idx / (SR * 8), rem = idx - c * (SR * 8), sr = rem >> 3, seg = rem & 7;
      const f16x4 hh = __builtin_convertvector(av[i], f16x4);
      const f16x4 tt = __builtin_convertvector((av[i] - __builtin_convertvector(hh, f32x4)) * 2048.f, f16x4);
      _Float16 *dst = lds + c * 2 * (SR + 1) * P + sr * P + seg * 4;
      *(f16x4 *)dst = hh;
      *(f16x4 *)(dst + (SR + 1) * P) = tt;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = (float)lds[(tid * 7) % (4 * 2 * (SR + 1) * P)];
  if constexpr (MODE & 2) {
#pragma unroll
    for (int i = 0; i < 18; ++i) s += (float)r[i][i & 7];
  }
  const long long t2 = __builtin_amdgcn_s_memtime();
  out[b * 512 + tid] = s;
  if (tid == 0) {
    stamps[b * 2] = t1 - t0;
    stamps[b * 2 + 1] = t2 - t0;
  }
}

template <typename F>
static void timeit(const char *name, F launch, long long *dstamps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < 100; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  long long st[512];
  CK(hipMemcpy(st, dstamps, sizeof(st), hipMemcpyDeviceToHost));
  double s1 = 0, s2 = 0;
  long long m1 = 0, m2 = 0;
  for (int i = 0; i < 256; ++i) {
    s1 += st[2 * i];
    s2 += st[2 * i + 1];
    m1 = st[2 * i] > m1 ? st[2 * i] : m1;
    m2 = st[2 * i + 1] > m2 ? st[2 * i + 1] : m2;
  }
  printf("%-34s %7.2f us/launch | staged at %6.0f cyc (max %6lld), weights in at %6.0f (max %6lld)\n",
         name, ms * 1e3 / 100, s1 / 256, m1, s2 / 256, m2);
  fflush(stdout);
}

int main() {
  float *x, *out;
  _Float16 *w;
  long long *st;
  CK(hipMalloc(&x, (size_t)256 * 120 * 256 * 4));
  CK(hipMemset(x, 0, (size_t)256 * 120 * 256 * 4));
  CK(hipMalloc(&w, (size_t)256 * 139264 + 65536));
  CK(hipMemset(w, 0, (size_t)256 * 139264 + 65536));
  CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMalloc(&st, 4096));
  timeit("empty", [&] { prologue<0><<<256, 512>>>(x, w, out, st); }, st);
  timeit("slab (shared x)", [&] { prologue<1><<<256, 512>>>(x, w, out, st); }, st);
  timeit("slab (own x per block)", [&] { prologue<9><<<256, 512>>>(x, w, out, st); }, st);
  timeit("weights only", [&] { prologue<2><<<256, 512>>>(x, w, out, st); }, st);
  timeit("slab then weights (kernel order)", [&] { prologue<3><<<256, 512>>>(x, w, out, st); }, st);
  timeit("weights then slab", [&] { prologue<7><<<256, 512>>>(x, w, out, st); }, st);
  timeit("slab(own) then weights", [&] { prologue<11><<<256, 512>>>(x, w, out, st); }, st);
  return 0;
}
