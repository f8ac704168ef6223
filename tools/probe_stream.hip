// Weight-stream probe for the c2 prenet bank (B = 1, T = 120, K = 16, Cin = Cout = 256):
// how fast can 256 CUs pull the bank's 35.65 MB of f16 weight planes (2 planes x 4 B per
// weight) in the access pattern of a (group pair, 16-column set, channel half) schedule,
// against a contiguous per-block stream?  No compute: each lane sums what it loaded.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_stream.hip -o /tmp/probe_stream
// Prints per-variant us per launch (HIP events over back-to-back launches, warm Infinity
// Cache), per launch behind a 512 MiB overwrite (cold: the overwrite's dirty lines are
// still being written back while the launch reads), and per launch behind a 1 GiB streaming
// READ of another buffer (cold-read: the weights evicted from L2 and the Infinity Cache by
// clean lines, so the launch pays HBM reads only).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr int K = 16, C = 256, N = 256;
struct Planes {
  const _Float16 *g[K];  // group g: kernel size K - g, planes [2][N][Kpad]
};

__device__ __forceinline__ float hsum(f16x8 v) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (float)v[i];
  return s;
}

// bank pattern: block = (pair p, column set cs, channel half h); 68 (group, tap, chunk) steps,
// wave w takes steps w + NW i; lane (fr, fs) loads 16 B of column 16 cs + fr at channel
// 128 h + 32 chunk + 8 fs of tap j from both planes.  ALL = every load issued up front.
template <int NW, bool ALL>
__global__ __launch_bounds__(NW * 64, 1) void bank_pattern(Planes P, float *out) {
  const int b = blockIdx.x;
  // partners (h = 0 / 1) 8 blocks apart (one XCD under round-robin dispatch)
  const int h = (b >> 3) & 1, u = (b & 7) | ((b >> 4) << 3);  // u = 0..127
  const int p = u / 16, cs = u % 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fs = lane >> 4;
  const int kh = K - p, kl = p + 1, QH = 4 * kh, Q = QH + 4 * kl;  // Q = 68
  constexpr int NS = (68 + NW - 1) / NW;
  auto addr = [&](int q) {
    q = q < Q ? q : Q - 1;
    const bool hv = q < QH;
    const int g = hv ? p : K - 1 - p, k = hv ? kh : kl;
    const int qq = hv ? q : q - QH, j = qq >> 2, c = qq & 3;
    return P.g[g] + (size_t)(cs * 16 + fr) * (k * C) + j * C + 128 * h + 32 * c + 8 * fs;
  };
  float s = 0.f;
  if constexpr (ALL) {
    f16x8 r0[NS], r1[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int q = w + NW * i;
      const _Float16 *a = addr(q);
      const int k = (q < QH) ? kh : kl;
      r0[i] = *(const f16x8 *)a;
      r1[i] = *(const f16x8 *)(a + (size_t)N * k * C);
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) s += hsum(r0[i]) + hsum(r1[i]);
  } else {
    constexpr int PF = 4;
    f16x8 r0[PF], r1[PF];
    auto ld = [&](int i, f16x8 &x0, f16x8 &x1) {
      const int q = w + NW * i;
      const _Float16 *a = addr(q);
      const int k = (min(q, Q - 1) < QH) ? kh : kl;
      x0 = *(const f16x8 *)a;
      x1 = *(const f16x8 *)(a + (size_t)N * k * C);
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) ld(i, r0[i], r1[i]);
    for (int i0 = 0; i0 < NS; i0 += PF) {
#pragma unroll
      for (int v = 0; v < PF; ++v) {
        s += hsum(r0[v]) + hsum(r1[v]);
        ld(i0 + v + PF, r0[v], r1[v]);
      }
    }
  }
  out[b * NW * 64 + threadIdx.x] = s;
}

// contiguous: block b reads bytes [b, b + 1) * per of one flat buffer, 16 B per lane-load
template <int NT, int NB>
__global__ __launch_bounds__(NT, 1) void contig(const f32x4 *buf, size_t per16, float *out) {
  const f32x4 *a = buf + blockIdx.x * per16;
  const int L = (int)(per16 / NT);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 17;
  for (int i0 = 0; i0 < L; i0 += U) {
    f32x4 r[U];
#pragma unroll
    for (int i = 0; i < U; ++i) r[i] = i0 + i < L ? a[(i0 + i) * NT + threadIdx.x] : (f32x4){};
#pragma unroll
    for (int i = 0; i < U; ++i) s += r[i];
  }
  out[blockIdx.x * NT + threadIdx.x] = s.x + s.y + s.z + s.w;
}

// evicts every cache level by reading n16 x 16 B (clean lines); one float per block out
__global__ __launch_bounds__(256) void evict_read(const f32x4 *buf, size_t n16, float *out) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) s += buf[i];
  if (s.x == 12345.f) out[blockIdx.x] = s.y;  // never true for the zero buffer: keeps the loads
}

static f32x4 *g_rflush = nullptr;
static size_t g_rbytes = 0;
static float *g_rout = nullptr;

template <typename F>
static void timeit(const char *name, F launch, void *flush, size_t fbytes, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  const int reps = 100;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double warm = ms * 1e3 / reps;
  double cold = 0;
  for (int i = 0; i < 10; ++i) {
    CK(hipMemsetAsync(flush, i, fbytes));
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    cold += ms * 1e3 / 10;
  }
  double cold_r = 0;
  for (int i = 0; i < 10; ++i) {
    evict_read<<<4096, 256>>>(g_rflush, g_rbytes / 16, g_rout);
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    cold_r += ms * 1e3 / 10;
  }
  printf("%-28s warm %7.2f us (%5.2f TB/s) | cold %7.2f us (%5.2f TB/s) | cold-read %7.2f us (%5.2f TB/s)\n",
         name, warm, bytes / warm / 1e6, cold, bytes / cold / 1e6, cold_r, bytes / cold_r / 1e6);
  fflush(stdout);
}

int main() {
  Planes P;
  size_t total = 0;
  std::vector<_Float16 *> bufs;
  for (int g = 0; g < K; ++g) {
    const int k = K - g;
    const size_t n = (size_t)2 * N * k * C;
    _Float16 *d;
    CK(hipMalloc(&d, n * 2));
    CK(hipMemset(d, 0x11, n * 2));
    P.g[g] = d;
    total += n * 2;
  }
  f32x4 *flat;
  CK(hipMalloc(&flat, total));
  CK(hipMemset(flat, 0, total));
  float *out;
  CK(hipMalloc(&out, 1 << 22));
  const size_t fb = (size_t)512 << 20;
  void *flush;
  CK(hipMalloc(&flush, fb));
  g_rbytes = (size_t)1 << 30;
  CK(hipMalloc(&g_rflush, g_rbytes));
  CK(hipMemset(g_rflush, 0, g_rbytes));
  CK(hipMalloc(&g_rout, 1 << 16));
  printf("bank weight planes: %.2f MB\n", total / 1e6);
  const double B = (double)total;
  timeit("bank 8w ring4", [&] { bank_pattern<8, false><<<256, 512>>>(P, out); }, flush, fb, B);
  timeit("bank 8w all-upfront", [&] { bank_pattern<8, true><<<256, 512>>>(P, out); }, flush, fb, B);
  timeit("bank 16w all-upfront", [&] { bank_pattern<16, true><<<256, 1024>>>(P, out); }, flush, fb, B);
  timeit("bank 4w all-upfront", [&] { bank_pattern<4, true><<<256, 256>>>(P, out); }, flush, fb, B);
  const size_t per16 = total / 16 / 256;
  timeit("contig 256x512", [&] { contig<512, 256><<<256, 512>>>(flat, per16, out); }, flush, fb, B);
  timeit("contig 256x1024", [&] { contig<1024, 256><<<256, 1024>>>(flat, per16, out); }, flush, fb, B);
  const size_t per16b = total / 16 / 512;
  timeit("contig 512x256", [&] { contig<256, 512><<<512, 256>>>(flat, per16b, out); }, flush, fb, B);
  const size_t per16c = total / 16 / 1024;
  timeit("contig 1024x256", [&] { contig<256, 1024><<<1024, 256>>>(flat, per16c, out); }, flush, fb, B);
  timeit("empty 256x512", [&] { contig<512, 256><<<256, 512>>>(flat, 0, out); }, flush, fb, B);
  return 0;
}
