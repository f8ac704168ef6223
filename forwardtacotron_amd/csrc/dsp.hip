// Audio path of utils/dsp.py on gfx950: STFT / log-mel (wav_to_mel :71-87), ISTFT,
// fast Griffin-Lim (griffinlim :89-103 -> librosa 0.7.2 core.griffinlim) and the mel
// pseudo-inversion (feature.inverse.mel_to_stft -> util.nnls).
//
// Numerics follow librosa 0.7.2 on numpy 1.x: every FFT runs in float64 (numpy.fft
// upcasts), spectra are stored as complex64 and audio as float32.  Here each workgroup
// transforms TWO real frames with one fp64 complex FFT (z = a + i b) held in LDS
// (Stockham radix-2 autosort, twiddles from a host-built fp64 table), so the
// float32/complex64 results match the float64 reference up to its final rounding.
//
// Layouts (HBM): audio (B, L) rows with a stride; spectra FRAME-major (B, F, n_bins)
// complex64 (one frame's bins contiguous: coalesced), magnitudes (B, F, n_bins) float32,
// mel (B, n_mels, F) float32 (the reference's (n_mels, frames) per item).
#include "common.h"

// hipcc contracts a*b+c into FMA by default (-ffp-contract=fast; the __fmul_rn family is
// header-inlined and contracts too): the reference-order float32 roundings below need
// every multiply and add rounded on its own.
#pragma clang fp contract(off)

namespace {

struct FftPlan {
  int n, log2n, hop;
  const double *window;  // [n] periodic Hann, pad-centred
  const double2 *tw;     // [n/2] exp(-2 pi i k / n)
};

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// In-place (ping-pong) fp64 complex FFT of a[0..n) in LDS; returns the buffer holding the
// result.  Stockham autosort: stage s (= 1, 2, 4, ...) maps butterfly b = p*s + q to
// y[q + 2sp] = u + v, y[q + 2sp + s] = (u - v) w^(ps), u = a[b], v = a[b + n/2].
template <bool INV>
__device__ double2 *fft_lds(double2 *a, double2 *y, const FftPlan &P) {
  const int n = P.n, h = n >> 1;
  for (int ls = 0; ls < P.log2n; ++ls) {
    __syncthreads();
    const int s = 1 << ls;
    for (int b = threadIdx.x; b < h; b += blockDim.x) {
      const int p = b >> ls, q = b & (s - 1);
      const double2 u = a[b], v = a[b + h];
      double2 w = P.tw[p << ls];
      if (INV) w.y = -w.y;
      y[q + 2 * s * p] = cadd(u, v);
      y[q + 2 * s * p + s] = cmul(csub(u, v), w);
    }
    double2 *t = a;
    a = y;
    y = t;
  }
  __syncthreads();
  return a;
}

// numpy.pad(mode='reflect') index for any pad width (periodic reflection, period 2(L-1))
__device__ __forceinline__ int64_t reflect_index(int64_t j, int64_t L) {
  if (L <= 1) return 0;
  const int64_t per = 2 * (L - 1);
  j %= per;
  if (j < 0) j += per;
  return j >= L ? per - j : j;
}

// correctly rounded |re + i im| of a complex64 value
__device__ __forceinline__ float cabs_rn(float re, float im) {
  return (float)sqrt((double)re * (double)re + (double)im * (double)im);
}

enum { STFT_COMPLEX = 0, STFT_MEL = 1, STFT_GL = 2 };

struct StftParams {
  const float *y;
  int64_t y_stride;
  int B;
  int64_t L;
  const int32_t *lengths;  // samples per item (NULL: L)
  int F;
  const int32_t *frames;   // frames per item (NULL: F); frames beyond are skipped
  FftPlan P;
  // STFT_COMPLEX
  float2 *X;
  // STFT_MEL
  float *mel;
  const float *basis;  // [n_mels][n_bins]
  const int32_t *mlo, *mhi;
  int n_mels, log_norm;
  // STFT_GL
  const float *S;
  float2 *tprev;
  float c;
  int first;
};

template <int MODE>
__global__ __launch_bounds__(256) void stft_kernel(const StftParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double2 *buf0 = (double2 *)smem;
  double2 *buf1 = buf0 + p.P.n;
  const int b = blockIdx.y;
  const int f0 = 2 * blockIdx.x;
  const int Fb = p.frames ? min(p.frames[b], p.F) : p.F;
  if (f0 >= Fb) return;
  const bool two = f0 + 1 < Fb;
  const int64_t Lb = p.lengths ? (int64_t)p.lengths[b] : p.L;
  const float *yb = p.y + (int64_t)b * p.y_stride;
  const int n = p.P.n, half = n >> 1, nb = half + 1;

  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double w = p.P.window[i];
    const int64_t j0 = (int64_t)f0 * p.P.hop + i - half;
    const double a = w * (double)yb[reflect_index(j0, Lb)];
    const double c = two ? w * (double)yb[reflect_index(j0 + p.P.hop, Lb)] : 0.0;
    buf0[i] = make_double2(a, c);
  }
  const double2 *Z = fft_lds<false>(buf0, buf1, p.P);
  float *mag = (float *)(Z == buf0 ? buf1 : buf0);  // the free buffer

  for (int k = threadIdx.x; k < nb; k += blockDim.x) {
    const double2 zk = Z[k], zn = Z[(n - k) & (n - 1)];
    // A = (Z[k] + conj Z[n-k]) / 2,  B = (Z[k] - conj Z[n-k]) / 2i
    const float2 A = make_float2((float)(0.5 * (zk.x + zn.x)), (float)(0.5 * (zk.y - zn.y)));
    const float2 Bq = make_float2((float)(0.5 * (zk.y + zn.y)), (float)(-0.5 * (zk.x - zn.x)));
    for (int fr = 0; fr < 1 + two; ++fr) {
      const float2 v = fr ? Bq : A;
      const int64_t o = ((int64_t)b * p.F + f0 + fr) * nb + k;
      if constexpr (MODE == STFT_COMPLEX) {
        p.X[o] = v;
      } else if constexpr (MODE == STFT_MEL) {
        mag[fr * nb + k] = cabs_rn(v.x, v.y);
      } else {
        // fast GL update (librosa 0.7.2 griffinlim loop body, complex64 arithmetic):
        // angles = rebuilt - c * tprev; angles /= |angles| + 1e-16; X = S * angles
        float2 an = v;
        if (!p.first) {
          const float2 t = p.tprev[o];
          an.x = (v.x - (p.c * t.x));
          an.y = (v.y - (p.c * t.y));
        }
        const float d = (cabs_rn(an.x, an.y) + 1e-16f);
        const float scl = (1.0f / d);  // numpy complex / real: (a, b) * (1/d)
        an.x = (an.x * scl);
        an.y = (an.y * scl);
        const float s = p.S[o];
        p.tprev[o] = v;
        p.X[o] = make_float2((s * an.x), (s * an.y));
      }
    }
  }
  if constexpr (MODE == STFT_MEL) {
    __syncthreads();
    for (int t = threadIdx.x; t < (1 + two) * p.n_mels; t += blockDim.x) {
      const int fr = t / p.n_mels, i = t - fr * p.n_mels;
      const float *row = p.basis + (int64_t)i * nb;
      double acc = 0.0;
      for (int k = p.mlo[i]; k < p.mhi[i]; ++k) acc += (double)row[k] * (double)mag[fr * nb + k];
      float v = (float)acc;
      if (p.log_norm) v = (float)log((double)fmaxf(v, 1e-5f));
      p.mel[((int64_t)b * p.n_mels + i) * p.F + f0 + fr] = v;
    }
  }
}

// inverse rFFT of two frames per workgroup, times the window; frames written as fp64
// (B, F, n) so the overlap-add can round exactly like the float32 reference accumulation
__global__ __launch_bounds__(256) void istft_frames_kernel(const float2 *__restrict__ X, int F,
                                                           const int32_t *frames, FftPlan P,
                                                           double *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double2 *buf0 = (double2 *)smem;
  double2 *buf1 = buf0 + P.n;
  const int b = blockIdx.y;
  const int f0 = 2 * blockIdx.x;
  const int Fb = frames ? min(frames[b], F) : F;
  if (f0 >= Fb) return;
  const bool two = f0 + 1 < Fb;
  const int n = P.n, half = n >> 1, nb = half + 1;
  const float2 *X0 = X + ((int64_t)b * F + f0) * nb;
  const float2 *X1 = X0 + nb;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const bool mirror = k > half;
    const int kk = mirror ? n - k : k;
    const float2 a32 = X0[kk];
    const float2 b32 = two ? X1[kk] : make_float2(0.f, 0.f);
    double ar = a32.x, ai = a32.y, br = b32.x, bi = b32.y;
    if (kk == 0 || kk == half) ai = bi = 0.0;  // c2r ignores imag of DC / Nyquist
    if (mirror) {
      ai = -ai;
      bi = -bi;
    }
    buf0[k] = make_double2(ar - bi, ai + br);  // A_full + i B_full
  }
  const double2 *z = fft_lds<true>(buf0, buf1, P);
  const double scale = 1.0 / n;
  double *o = out + ((int64_t)b * F + f0) * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double2 v = z[i];
    o[i] = P.window[i] * (v.x * scale);
    if (two) o[n + i] = P.window[i] * (v.y * scale);
  }
}

// overlap-add in frame order with float32 rounding after every add, divide by the float32
// window sum-square where it exceeds FLT_MIN, crop n/2 on both sides (center=True)
__global__ void istft_ola_kernel(const double *__restrict__ fr, int F, const int32_t *frames,
                                 int n, int hop, const double *__restrict__ win_sq,
                                 float *__restrict__ y, int64_t y_stride, int64_t y_len, int B) {
  const int b = blockIdx.y;
  const int Fb = frames ? min(frames[b], F) : F;
  const int64_t Lb = Fb > 0 ? (int64_t)hop * (Fb - 1) : 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < y_len;
       s += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (s < Lb) {
      const int64_t sf = s + n / 2;
      const int64_t ihi = min((int64_t)Fb - 1, sf / hop);
      int64_t ilo = sf - n + 1 > 0 ? (sf - n + 1 + hop - 1) / hop : 0;
      float w2 = 0.f;
      for (int64_t i = ilo; i <= ihi; ++i) {
        const int64_t off = sf - i * hop;
        v = (float)((double)v + fr[((int64_t)b * F + i) * n + off]);
        w2 = (float)((double)w2 + win_sq[off]);
      }
      if (w2 > 1.17549435e-38f) v = (v / w2);
    }
    y[(int64_t)b * y_stride + s] = v;
  }
}

struct NnlsParams {
  const float *mel;  // (B, n_mels, F)
  int B, F, n_mels, nb;
  const int32_t *frames;
  int denorm;
  const float *rowvals;  // packed nonzeros of each mel row (contiguous support)
  const int32_t *rowptr, *rowlo;  // [n_mels + 1], [n_mels]
  const int32_t *bi;     // [nb][2] mel rows of each bin (-1: none)
  const float *bw;       // [nb][2] their weights
  const float *pinv;     // [nb][n_mels]
  float inv_L;
  int iters;
  float *S;  // (B, F, nb)
};

constexpr int NNLS_MAX_BINS = 64 * 33;  // n_fft <= 4096
constexpr int NNLS_MAX_MELS = 512;

// min ||A x - m||, x >= 0 for one frame per workgroup (one wave): FISTA on the sparse
// filterbank (each bin feeds at most two mel rows), started like librosa's nnls from the
// clipped minimum-norm least-squares solution pinv(A) m.  Everything stays in LDS /
// registers across the iterations; HBM sees only m in and x out.
// NR: mel rows per lane (n_mels <= 64 NR)
template <int NJ, int NR>
__global__ __launch_bounds__(64) void nnls_kernel(const NnlsParams p) {
  extern __shared__ float dyn[];  // m[n_mels] r[n_mels] y[nb] vals[nnz]
  float *m_s = dyn, *r_s = dyn + p.n_mels, *y_s = r_s + p.n_mels, *v_s = y_s + p.nb;
  const int frame = blockIdx.x;
  const int b = frame / p.F, f = frame - b * p.F;
  const int lane = threadIdx.x;
  const int Fb = p.frames ? min(p.frames[b], p.F) : p.F;
  float *Sout = p.S + (int64_t)frame * p.nb;
  if (f >= Fb) {
    for (int k = lane; k < p.nb; k += 64) Sout[k] = 0.f;
    return;
  }
  const int nnz = p.rowptr[p.n_mels];
  for (int i = lane; i < nnz; i += 64) v_s[i] = p.rowvals[i];
  for (int i = lane; i < p.n_mels; i += 64) {
    const float v = p.mel[((int64_t)b * p.n_mels + i) * p.F + f];
    m_s[i] = p.denorm ? (float)exp((double)v) : v;
  }
  __syncthreads();
  float x[NJ], yv[NJ], w0[NJ], w1[NJ];
  int i0[NJ], i1[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = lane + 64 * j;
    x[j] = 0.f;
    i0[j] = i1[j] = -1;
    w0[j] = w1[j] = 0.f;
    if (k < p.nb) {
      double acc = 0.0;
      const float *pr = p.pinv + (int64_t)k * p.n_mels;
      for (int i = 0; i < p.n_mels; ++i) acc += (double)pr[i] * (double)m_s[i];
      x[j] = fmaxf((float)acc, 0.f);
      i0[j] = p.bi[2 * k];
      i1[j] = p.bi[2 * k + 1];
      w0[j] = p.bw[2 * k];
      w1[j] = p.bw[2 * k + 1];
      y_s[k] = x[j];
    }
    yv[j] = x[j];
  }
  // the lane's mel rows (lane, lane + 64, ...: n_mels <= 512) and their sparse supports,
  // read once: inside the iteration loop they were three dependent global loads per row and
  // step.  The row sums keep their order (q ascending, one fmaf chain per row); the loop is
  // unrolled so a row's LDS reads issue back to back instead of one latency per term.
  int rlo[NR], ro[NR], rc[NR];
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int i = lane + 64 * u;
    rlo[u] = ro[u] = rc[u] = 0;
    if (i < p.n_mels) {
      rlo[u] = p.rowlo[i];
      ro[u] = p.rowptr[i];
      rc[u] = p.rowptr[i + 1] - ro[u];
    }
  }
  float t = 1.f;
  for (int it = 0; it < p.iters; ++it) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int i = lane + 64 * u;
      if (64 * u >= p.n_mels) break;  // uniform
      if (i < p.n_mels) {
        const float *vr = v_s + ro[u], *yr = y_s + rlo[u];
        const int cnt = rc[u];
        float acc = 0.f;
#pragma unroll 8
        for (int q = 0; q < cnt; ++q) acc = fmaf(vr[q], yr[q], acc);
        r_s[i] = acc - m_s[i];
      }
    }
    __syncthreads();
    const float tn = 0.5f * (1.f + sqrtf(1.f + 4.f * t * t));
    const float beta = (t - 1.f) / tn;
    t = tn;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = lane + 64 * j;
      if (k < p.nb) {
        float g = 0.f;
        if (i0[j] >= 0) g = w0[j] * r_s[i0[j]];
        if (i1[j] >= 0) g = fmaf(w1[j], r_s[i1[j]], g);
        const float xn = fmaxf(0.f, yv[j] - g * p.inv_L);
        yv[j] = xn + beta * (xn - x[j]);
        x[j] = xn;
        y_s[k] = yv[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = lane + 64 * j;
    if (k < p.nb) Sout[k] = x[j];
  }
}

int check_plan(int n, int hop, const double *window, const void *tw) {
  if (n < 16 || n > 4096 || (n & (n - 1)) || hop <= 0 || !window || !tw) return FTMI_E_ARG;
  return FTMI_OK;
}

int log2i(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return l;
}

size_t fft_smem(int n) { return (size_t)2 * n * sizeof(double2); }

template <int MODE>
int launch_stft(StftParams &p, hipStream_t s) {
  const size_t sm = fft_smem(p.P.n);
  if (sm > 64 * 1024)
    (void)hipFuncSetAttribute((const void *)stft_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)sm);
  dim3 grid((p.F + 1) / 2, p.B);
  hipLaunchKernelGGL(stft_kernel<MODE>, grid, dim3(256), sm, s, p);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

}  // namespace

extern "C" int ftmi_stft(const float *y, int64_t y_stride, int32_t B, int64_t L,
                         const int32_t *lengths, int32_t n_fft, int32_t hop,
                         const double *window, const void *twiddle, int32_t F,
                         const int32_t *frames, void *X, ftmi_stream_t stream) {
  if (!y || !X || B <= 0 || L <= 0 || F <= 0) return FTMI_E_ARG;
  if (int rc = check_plan(n_fft, hop, window, twiddle)) return rc;
  StftParams p = {};
  p.y = y, p.y_stride = y_stride, p.B = B, p.L = L, p.lengths = lengths, p.F = F, p.frames = frames;
  p.P = FftPlan{n_fft, log2i(n_fft), hop, window, (const double2 *)twiddle};
  p.X = (float2 *)X;
  return launch_stft<STFT_COMPLEX>(p, ftmi_hs(stream));
}

extern "C" int ftmi_mel_spectrogram(const float *y, int64_t y_stride, int32_t B, int64_t L,
                                    const int32_t *lengths, int32_t n_fft, int32_t hop,
                                    const double *window, const void *twiddle, int32_t F,
                                    const int32_t *frames, const float *basis,
                                    const int32_t *mel_lo, const int32_t *mel_hi, int32_t n_mels,
                                    int32_t log_norm, float *mel, ftmi_stream_t stream) {
  if (!y || !mel || !basis || !mel_lo || !mel_hi || B <= 0 || L <= 0 || F <= 0 || n_mels <= 0)
    return FTMI_E_ARG;
  if (int rc = check_plan(n_fft, hop, window, twiddle)) return rc;
  StftParams p = {};
  p.y = y, p.y_stride = y_stride, p.B = B, p.L = L, p.lengths = lengths, p.F = F, p.frames = frames;
  p.P = FftPlan{n_fft, log2i(n_fft), hop, window, (const double2 *)twiddle};
  p.mel = mel, p.basis = basis, p.mlo = mel_lo, p.mhi = mel_hi, p.n_mels = n_mels;
  p.log_norm = log_norm;
  return launch_stft<STFT_MEL>(p, ftmi_hs(stream));
}

extern "C" int ftmi_griffinlim_stft(const float *y, int64_t y_stride, int32_t B, int64_t L,
                                    const int32_t *lengths, int32_t n_fft, int32_t hop,
                                    const double *window, const void *twiddle, int32_t F,
                                    const int32_t *frames, const float *S, void *tprev,
                                    float c, int32_t first, void *X, ftmi_stream_t stream) {
  if (!y || !S || !tprev || !X || B <= 0 || L <= 0 || F <= 0) return FTMI_E_ARG;
  if (int rc = check_plan(n_fft, hop, window, twiddle)) return rc;
  StftParams p = {};
  p.y = y, p.y_stride = y_stride, p.B = B, p.L = L, p.lengths = lengths, p.F = F, p.frames = frames;
  p.P = FftPlan{n_fft, log2i(n_fft), hop, window, (const double2 *)twiddle};
  p.S = S, p.tprev = (float2 *)tprev, p.c = c, p.first = first, p.X = (float2 *)X;
  return launch_stft<STFT_GL>(p, ftmi_hs(stream));
}

extern "C" int64_t ftmi_istft_workspace_bytes(int32_t B, int32_t F, int32_t n_fft) {
  return (int64_t)B * F * n_fft * (int64_t)sizeof(double);
}

extern "C" int ftmi_istft(const void *X, int32_t B, int32_t F, const int32_t *frames,
                          int32_t n_fft, int32_t hop, const double *window, const double *win_sq,
                          const void *twiddle, void *work, float *y, int64_t y_stride,
                          int64_t y_len, ftmi_stream_t stream) {
  if (!X || !work || !y || !win_sq || B <= 0 || F <= 0 || y_len < 0) return FTMI_E_ARG;
  if (int rc = check_plan(n_fft, hop, window, twiddle)) return rc;
  const hipStream_t s = ftmi_hs(stream);
  FftPlan P{n_fft, log2i(n_fft), hop, window, (const double2 *)twiddle};
  const size_t sm = fft_smem(n_fft);
  if (sm > 64 * 1024)
    (void)hipFuncSetAttribute((const void *)istft_frames_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)sm);
  hipLaunchKernelGGL(istft_frames_kernel, dim3((F + 1) / 2, B), dim3(256), sm, s, (const float2 *)X,
                     F, frames, P, (double *)work);
  FTMI_CHECK_LAUNCH();
  if (y_len == 0) return FTMI_OK;
  const int64_t blocks = (y_len + 255) / 256;
  hipLaunchKernelGGL(istft_ola_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096), B), dim3(256), 0,
                     s, (const double *)work, F, frames, n_fft, hop, win_sq, y, y_stride, y_len, B);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_mel_nnls(const float *mel, int32_t B, int32_t F, const int32_t *frames,
                             int32_t n_mels, int32_t n_bins, int32_t denorm, int32_t nnz,
                             const float *rowvals,
                             const int32_t *rowptr, const int32_t *rowlo, const int32_t *bin_rows,
                             const float *bin_w, const float *pinv, float inv_L, int32_t iters,
                             float *S, ftmi_stream_t stream) {
  if (!mel || !S || !rowvals || !rowptr || !rowlo || !bin_rows || !bin_w || !pinv) return FTMI_E_ARG;
  if (B <= 0 || F <= 0 || n_mels <= 0 || n_mels > NNLS_MAX_MELS || n_bins <= 0 ||
      n_bins > NNLS_MAX_BINS || iters < 0)
    return FTMI_E_SHAPE;
  NnlsParams p{mel, B, F, n_mels, n_bins, frames, denorm, rowvals, rowptr, rowlo,
               bin_rows, bin_w, pinv, inv_L, iters, S};
  if (nnz <= 0 || nnz > 16384) return FTMI_E_SHAPE;
  const hipStream_t s = ftmi_hs(stream);
  const int nj = (n_bins + 63) / 64;
  const dim3 grid((unsigned)((int64_t)B * F)), block(64);
  const size_t sm = (size_t)(2 * n_mels + n_bins + nnz) * sizeof(float);
#define FTMI_NNLS_NJ(NR_)                                                       \
  if (nj <= 3)                                                                  \
    hipLaunchKernelGGL((nnls_kernel<3, NR_>), grid, block, sm, s, p);           \
  else if (nj <= 5)                                                             \
    hipLaunchKernelGGL((nnls_kernel<5, NR_>), grid, block, sm, s, p);           \
  else if (nj <= 9)                                                             \
    hipLaunchKernelGGL((nnls_kernel<9, NR_>), grid, block, sm, s, p);           \
  else if (nj <= 17)                                                            \
    hipLaunchKernelGGL((nnls_kernel<17, NR_>), grid, block, sm, s, p);          \
  else                                                                          \
    hipLaunchKernelGGL((nnls_kernel<33, NR_>), grid, block, sm, s, p);
  if (n_mels <= 128) {  // the model's 80 mels: two rows per lane
    FTMI_NNLS_NJ(2)
  } else {
    FTMI_NNLS_NJ(NNLS_MAX_MELS / 64)
  }
#undef FTMI_NNLS_NJ
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

namespace {
__global__ void spec_mul_kernel(const float *__restrict__ S, const float2 *__restrict__ A,
                                float2 *__restrict__ X, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float s = S[i];
    const float2 a = A[i];
    X[i] = make_float2((s * a.x), (s * a.y));
  }
}
}  // namespace

extern "C" int ftmi_spec_mul(const float *S, const void *angles, int64_t n, void *X,
                             ftmi_stream_t stream) {
  if (!S || !angles || !X || n < 0) return FTMI_E_ARG;
  if (n == 0) return FTMI_OK;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(spec_mul_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     ftmi_hs(stream), S, (const float2 *)angles, (float2 *)X, n);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

namespace {
// librosa 0.7.2 griffinlim's initial phases, np.exp(2j * np.pi * u) with u = np.random.rand
// (n_bins, T): float64 cos / sin of 6.283185307179586 * u (the imaginary part numpy forms),
// rounded to complex64, written frame-major (B, T, n_bins) from the bin-major draws
__global__ void unit_phase_kernel(const double *__restrict__ u, int32_t nb, int32_t T,
                                  int64_t n, float2 *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bt = i / nb;            // (item, frame)
    const int k = (int)(i - bt * nb);
    const int64_t b = bt / T, t = bt - b * T;
    const double y = 6.283185307179586 * u[(b * nb + k) * T + t];
    out[i] = make_float2((float)cos(y), (float)sin(y));
  }
}
}  // namespace

extern "C" int ftmi_unit_phases(const double *u, int32_t B, int32_t n_bins, int32_t T,
                                void *angles, ftmi_stream_t stream) {
  if (!u || !angles || B <= 0 || n_bins <= 0 || T <= 0) return FTMI_E_ARG;
  const int64_t n = (int64_t)B * n_bins * T;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(unit_phase_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     ftmi_hs(stream), u, n_bins, T, n, (float2 *)angles);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

// ==========================================================================================
// The fused Griffin-Lim iteration (round 6): one launch per iteration instead of the ISTFT
// frame kernel (fp64 frames through HBM: (B, F, 1024) x 8 B), the overlap-add kernel and the
// analysis kernel.  A workgroup owns a tile of TF consecutive frames of one item:
//   1. synthesis: the inverse rFFT of every frame whose support reaches the tile's analysis
//      windows (the tile +- GL_HALO frames: n_fft / hop = 4, plus the reflect padding at the
//      signal's ends), two real frames per complex fp64 FFT, each wave one pair;
//   2. overlap-add into a float32 segment in LDS in the reference's frame order (float32
//      rounding after every add, librosa 0.7.2 istft), then the division by the float32
//      window sum-square (its own frame-order accumulation) — the audio the tile's frames
//      analyse, never written to HBM;
//   3. analysis (center=True reflect padding) of the tile's frames, two per FFT, and the
//      fast-GL update (momentum, normalise, S * angles) — X to a second buffer (the halo
//      frames of the neighbouring tiles still read this iteration's X), tprev in place.
// The final ISTFT is the same kernel with the analysis replaced by the store of the tile's
// audio samples.  Specialised to the reference configuration n_fft = 1024, hop = 256
// (config.yaml); other sizes keep the three-kernel path.
//
// The FFT: 1024 points per wave, 16 per lane: a radix-16 DFT in registers over stride 64,
// twiddles, an LDS transpose, a radix-16 DFT in registers, twiddles, a radix-4 DFT across
// each quad of lanes (DPP quad permutes) — two LDS passes where the radix-2 Stockham
// kernels above make ten.  fp64 throughout, like numpy.fft under librosa.
namespace {

constexpr int GLN = 1024, GLHOP = 256, GLNB = GLN / 2 + 1;
constexpr int GL_HALO = 3;   // synthesis frames beyond the tile on each side (4 at the item's
                             // end when its last tile has one frame: reflect padding)
constexpr int gl_seg(int tf) { return (tf + 2 * GL_HALO) * GLHOP + GLN; }  // segment samples
constexpr int GL_ROW = 68;    // transpose row pitch (double2): rows 16 banks apart, conflict-free
constexpr int GL_BUF = 16 * GL_ROW;  // per-wave LDS buffer (double2)

// stage twiddles, laid out so a wave's 64 reads are consecutive (no bank conflicts):
// twA[(q - 1) * 64 + lane] = w^(lane q), q = 1..15; twB[l2 * 16 + k1] = w^(16 l2 k1)
constexpr int GL_TWA = 15 * 64, GL_TWB = 64;

// complex product with fused multiply-adds (the FFT's internal rounding: its outputs are
// rounded to float32, where a 1e-16-level change of the fp64 intermediates shows nowhere)
__device__ __forceinline__ double2 gl_cmul(double2 a, double2 b) {
  return make_double2(__fma_rn(a.x, b.x, -(a.y * b.y)), __fma_rn(a.x, b.y, a.y * b.x));
}

// 16-point DFT in registers: V[q] = sum_m v[m] w16^(mq) (radix-2 DIF, reordered)
__device__ __forceinline__ void gl_dft16(double2 (&v)[16]) {
  const double C1 = 0.92387953251128674, S1 = 0.38268343236508977, C2 = 0.70710678118654752;
  const double2 W[8] = {make_double2(1.0, 0.0),  make_double2(C1, -S1),  make_double2(C2, -C2),
                        make_double2(S1, -C1),   make_double2(0.0, -1.0), make_double2(-S1, -C1),
                        make_double2(-C2, -C2), make_double2(-C1, -S1)};
#pragma unroll
  for (int h = 8; h >= 1; h >>= 1) {
#pragma unroll
    for (int b = 0; b < 16; b += 2 * h) {
#pragma unroll
      for (int j = 0; j < h; ++j) {
        const double2 u = v[b + j], t = v[b + j + h];
        v[b + j] = cadd(u, t);
        const double2 d = csub(u, t);
        // W[4] = -i: 7 of the 17 products are a swap (the value gl_cmul rounds to)
        v[b + j + h] = (j == 0) ? d : (j * (8 / h) == 4) ? make_double2(d.y, -d.x) : gl_cmul(d, W[j * (8 / h)]);
      }
    }
  }
  constexpr int rev[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
  double2 r[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) r[k] = v[rev[k]];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = r[k];
}

template <int CTRL>
__device__ __forceinline__ double gl_dpp(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ double2 gl_dpp2(double2 v) {
  return make_double2(gl_dpp<CTRL>(v.x), gl_dpp<CTRL>(v.y));
}

// 1 / x in float64 to within ~2^-52 (v_rcp_f64 and two Newton steps; inf -> 0).  A float32
// quotient a / b of float32 values is never within 2^-49 (relative) of a float32 rounding
// midpoint — b * m for a 25-bit midpoint m differs from a by at least one unit of the
// product's 49-bit grid — so (float)(a * gl_rcp64(b)) IS the correctly rounded a / b that
// numpy computes.  The IEEE float32 division sequence reads VCC in v_div_fmas, which keeps
// independent divisions from overlapping.
// x is a float32 value at every call (|an| + 1e-16, the window sum-square), so the seed is
// the float32 reciprocal (~2^-22, the fast transcendental unit): two Newton steps reach
// ~2^-88.
__device__ __forceinline__ double gl_rcp64(double x) {
  double r = (double)__builtin_amdgcn_rcpf((float)x);
  double e = __fma_rn(-x, r, 1.0);
  r = __fma_rn(r, e, r);
  e = __fma_rn(-x, r, 1.0);
  r = __fma_rn(r, e, r);
  return __builtin_isinf(x) ? 0.0 : r;
}

// natural-order index k of the FFT output in a wave buffer (a 4-element gap every 256)
__device__ __forceinline__ int gl_pk(int k) { return k + ((k >> 8) << 2); }

__device__ __forceinline__ void gl_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// forward FFT of z[lane + 64 m] = v[m]; the result in buf (gl_pk order).  One wave, its own
// buffer: the exchanges are wave-local (no workgroup barrier), so the waves of a workgroup
// run their FFTs independently.
__device__ void gl_fft1024(double2 (&v)[16], double2 *buf, const double2 *twA, const double2 *twB) {
  const int lane = threadIdx.x & 63;
  gl_dft16(v);
#pragma unroll
  for (int q = 1; q < 16; ++q) v[q] = gl_cmul(v[q], twA[(q - 1) * 64 + lane]);
#pragma unroll
  for (int q = 0; q < 16; ++q) buf[q * GL_ROW + lane] = v[q];
  gl_wave_sync();
  const int q = lane >> 2, l2 = lane & 3;
#pragma unroll
  for (int l1 = 0; l1 < 16; ++l1) v[l1] = buf[q * GL_ROW + 4 * l1 + l2];
  gl_wave_sync();
  gl_dft16(v);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) v[k1] = gl_cmul(v[k1], twB[l2 * 16 + k1]);
  // 4-point DFT over l2 across the quad: lanes (0, 1, 2, 3) end with Y[0], Y[2], Y[1], Y[3].
  // Each step is partner +- own value: one fma per component with a per-lane sign.
  const double sg1 = (l2 < 2) ? 1.0 : -1.0, sg2 = (l2 & 1) ? -1.0 : 1.0;
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) {
    const double2 p = gl_dpp2<0x4E>(v[k1]);  // lane ^ 2
    double2 r = make_double2(__fma_rn(sg1, v[k1].x, p.x), __fma_rn(sg1, v[k1].y, p.y));
    if (l2 == 3) r = make_double2(r.y, -r.x);  // (-i) (x1 - x3)
    const double2 p2 = gl_dpp2<0xB1>(r);       // lane ^ 1
    v[k1] = make_double2(__fma_rn(sg2, r.x, p2.x), __fma_rn(sg2, r.y, p2.y));
  }
  const int k2 = ((l2 & 1) << 1) | (l2 >> 1);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) buf[gl_pk(q + 16 * k1 + 256 * k2)] = v[k1];
  gl_wave_sync();
}

struct GlParams {
  const float2 *Xin;
  float2 *Xout;
  const float *S;
  float2 *tprev;
  int B, F, tiles;
  const int32_t *frames;
  const double *window, *win_sq;
  const double2 *tw;
  float c;
  int first;
  float *y;
  int64_t y_stride, y_len;
};

#ifdef FTMI_GL_STAMPS
// diagnostic build only (libftmi_stamps.so): wave 0's s_memtime at the phase boundaries
__device__ unsigned long long ftmi_gl_stamps[4096 * 8];
#define GLSTAMP(i)                                                                 \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                   \
      __builtin_amdgcn_sched_barrier(0);                                           \
      ftmi_gl_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();         \
      __builtin_amdgcn_sched_barrier(0);                                           \
    }                                                                              \
  } while (0)
#else
#define GLSTAMP(i) \
  do {             \
  } while (0)
#endif

template <int W, int TF, bool FINAL>
__global__ __launch_bounds__(64 * W) void gl_fused_kernel(const GlParams p) {
  __shared__ float seg[gl_seg(TF)];
  __shared__ double2 bufs[W][GL_BUF];
  __shared__ double win[GLN];
  __shared__ double2 twA[GL_TWA], twB[GL_TWB];
  __shared__ float wss_int[GLHOP];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const double scale = 1.0 / GLN;
  double2 *buf = bufs[w];
  // the tables, once per workgroup (it walks tiles blockIdx.x, + gridDim.x, ...)
  for (int i = threadIdx.x; i < GLN; i += 64 * W) win[i] = p.window[i];
  for (int i = threadIdx.x; i < GL_TWA + GL_TWB; i += 64 * W) {
    const int j = i < GL_TWA ? (i & 63) * (i / 64 + 1) : 16 * ((i - GL_TWA) >> 4) * ((i - GL_TWA) & 15);
    const double2 t = p.tw[j & (GLN / 2 - 1)];  // w^(j + 512) = -w^j
    const double2 v = (j & (GLN / 2)) ? make_double2(-t.x, -t.y) : t;
    if (i < GL_TWA) twA[i] = v;
    else twB[i - GL_TWA] = v;
  }
  __syncthreads();
  // the window sum-square of a sample covered by four frames, accumulated in frame order
  // (offsets r + 768, r + 512, r + 256, r): the same for every interior sample
  for (int r = threadIdx.x; r < GLHOP; r += 64 * W) {
    float w2 = 0.f;
    for (int k = 3; k >= 0; --k) {
      const double wv = win[r + k * GLHOP];
      w2 = (float)((double)w2 + wv * wv);
    }
    wss_int[r] = w2;
  }
  static_assert(64 * W == GLHOP, "the overlap-add maps one thread to each sample of a hop");
  double wr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wr[j] = win[threadIdx.x + GLHOP * j];

  for (int tile = blockIdx.x; tile < p.B * p.tiles; tile += gridDim.x) {
  GLSTAMP(0);
  const int b = tile / p.tiles, t = tile - b * p.tiles;
  const int Fb = p.frames ? min(p.frames[b], p.F) : p.F;
  const int f0 = t * TF;
  if (f0 >= Fb) continue;
  const int f1 = min(f0 + TF, Fb);
  // synthesis frames whose support reaches the tile's analysis windows: [f0 - 3, f1 + 3);
  // the reflect padding at the item's end reaches frame Fb - 5 from the last frame
  const int a0 = max(0, f0 - GL_HALO - ((f1 == Fb && f1 - f0 < 2) ? 1 : 0));
  const int a1 = min(Fb, f1 + GL_HALO);
  const int sb = a0 * GLHOP;                  // segment start (uncropped samples)
  const int slen = (a1 - 1 - a0) * GLHOP + GLN;
  const int L = GLHOP * (Fb - 1);             // istft length of item b
  // the first round's spectra are requested before the segment is cleared
  const int nsyn = a1 - a0;
  float2 xa[16], xb[16];
  auto load_pair = [&](int r0) {
    const int fa = a0 + r0 + 2 * w, fb = fa + 1;
    const bool va = fa < a1, vb = fb < a1;
    const float2 *XA = p.Xin + ((int64_t)b * p.F + fa) * GLNB;
    const float2 *XB = XA + GLNB;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int k = lane + 64 * m;
      const int kk = k > GLN / 2 ? GLN - k : k;
      xa[m] = va ? XA[kk] : make_float2(0.f, 0.f);
      xb[m] = vb ? XB[kk] : make_float2(0.f, 0.f);
    }
  };
  load_pair(0);
  __syncthreads();  // the previous tile's last reads of seg and the wave buffers are done
  for (int i = threadIdx.x; i < slen; i += 64 * W) seg[i] = 0.f;
  GLSTAMP(1);

  // ---- 1 + 2: synthesis and overlap-add, W frame pairs per round.  The next round's spectra
  // are loaded (registers) while this round's frames are overlap-added.
  for (int r0 = 0; r0 < nsyn; r0 += 2 * W) {
    double2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int k = lane + 64 * m;
      const bool mirror = k > GLN / 2;
      const int kk = mirror ? GLN - k : k;
      double ar = xa[m].x, ai = xa[m].y, br = xb[m].x, bi = xb[m].y;
      if (kk == 0 || kk == GLN / 2) ai = bi = 0.0;  // c2r ignores imag of DC / Nyquist
      if (mirror) {
        ai = -ai;
        bi = -bi;
      }
      // conj(A_full + i B_full): the inverse FFT as conj(FFT(conj z))
      v[m] = make_double2(ar - bi, -(ai + br));
    }
    if (r0 == 0) GLSTAMP(2);
    gl_fft1024(v, buf, twA, twB);
    if (r0 == 0) GLSTAMP(3);
    __syncthreads();
    if (r0 + 2 * W < nsyn) load_pair(r0 + 2 * W);
    // overlap-add of this round's frames, each sample's frames in increasing order.  Thread
    // r (64 W = one hop of threads) owns the samples (rf0 + q) hop + r: frame rf0 + q - j
    // reaches them at offset r + j hop, so the thread's four window values sit in registers,
    // a frame's value is at r + 260 j of its wave's buffer (gl_pk), and which (q, j) pairs
    // exist depends only on the round's frame count — compile-time in a full round.  The
    // q's dependent float32-rounded chains are independent and interleave.
    const int rf0 = a0 + r0, nf = min(a1 - rf0, 2 * W);
    const int base = r0 * GLHOP + threadIdx.x;  // segment index of (q = 0, r)
    auto tap = [&](int fi, int j) -> double {
      const double *zc = (const double *)&bufs[fi >> 1][threadIdx.x + (GLHOP + 4) * j];
      return (fi & 1) ? -zc[1] : zc[0];
    };
    if (nf == 2 * W) {
#pragma unroll
      for (int q = 0; q < 2 * W + 3; ++q) {
        float acc = seg[base + q * GLHOP];
#pragma unroll
        for (int j = 3; j >= 0; --j) {
          const int fi = q - j;
          if (fi >= 0 && fi < 2 * W) acc = (float)((double)acc + wr[j] * (tap(fi, j) * scale));
        }
        seg[base + q * GLHOP] = acc;
      }
    } else {
      for (int q = 0; q < nf + 3; ++q) {
        float acc = seg[base + q * GLHOP];
#pragma unroll
        for (int j = 3; j >= 0; --j) {
          const int fi = q - j;
          if (fi >= 0 && fi < nf) acc = (float)((double)acc + wr[j] * (tap(fi, j) * scale));
        }
        seg[base + q * GLHOP] = acc;
      }
    }
    __syncthreads();
  }
  GLSTAMP(4);
  // window sum-square (float32, frame order over every frame of the item), division.  A
  // segment clear of the item's first 3 hops and its end has four frames at every sample:
  // the table, 4 samples per thread (independent divisions interleave); else per sample
  if (sb >= GLN - GLHOP && sb + slen <= Fb * GLHOP) {
    // thread r's samples all sit at hop offset r (sb is a multiple of the hop): one divisor
    const float w2 = wss_int[threadIdx.x];
    const double rw = gl_rcp64((double)w2);
    const bool div = w2 > 1.17549435e-38f;
    for (int i = threadIdx.x; i < slen; i += 64 * W) {
      const float v = seg[i];
      seg[i] = div ? (float)((double)v * rw) : v;  // == v / w2 (gl_rcp64)
    }
  } else {
    for (int i = threadIdx.x; i < slen; i += 64 * W) {
      const int s = sb + i;
      const int ihi = min(Fb - 1, s / GLHOP);
      const int ilo = max(0, (s - GLN + GLHOP) / GLHOP);
      float w2;
      if (ihi - ilo == 3) {
        w2 = wss_int[s & (GLHOP - 1)];
      } else {
        w2 = 0.f;
        for (int k = ilo; k <= ihi; ++k) {
          const double wv = win[s - k * GLHOP];
          w2 = (float)((double)w2 + wv * wv);
        }
      }
      const float v = seg[i];
      seg[i] = (w2 > 1.17549435e-38f) ? (float)((double)v * gl_rcp64((double)w2)) : v;
    }
  }
  __syncthreads();

  if constexpr (FINAL) {
    // the tile's audio samples (cropped by n/2), zeros past the item's length
    const int64_t j0 = (int64_t)f0 * GLHOP;
    const int64_t j1 = (f1 == Fb) ? p.y_len : min((int64_t)f1 * GLHOP, p.y_len);
    float *yb = p.y + (int64_t)b * p.y_stride;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 64 * W)
      yb[j] = (j < L) ? seg[j + GLN / 2 - sb] : 0.f;
  } else {
    // ---- 3: analysis of the tile's frames and the fast-GL update (each wave its own pairs)
    for (int r0 = 0; r0 < f1 - f0; r0 += 2 * W) {
      const int fa = f0 + r0 + 2 * w, fb = fa + 1;
      const bool va = fa < f1, vb = fb < f1;
      double2 v[16];
      const int ja = fa * GLHOP - GLN / 2;  // first sample of frame fa (cropped coordinates)
      const bool inner = ja >= 0 && ja + GLHOP + GLN - 1 < L;
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int i = lane + 64 * m;
        const double wi = win[i];
        double xa, xb;
        if (inner) {
          xa = (double)seg[ja + i + GLN / 2 - sb];
          xb = (double)seg[ja + GLHOP + i + GLN / 2 - sb];
        } else {
          xa = va ? (double)seg[reflect_index(ja + i, L) + GLN / 2 - sb] : 0.0;
          xb = vb ? (double)seg[reflect_index(ja + GLHOP + i, L) + GLN / 2 - sb] : 0.0;
        }
        v[m] = make_double2(va ? wi * xa : 0.0, vb ? wi * xb : 0.0);
      }
      // this pair's S and tprev (9 bins per lane per frame), loaded before the FFT so their
      // latency hides behind it
      float sv[2][9];
      float2 tp[2][9];
#pragma unroll
      for (int fr = 0; fr < 2; ++fr) {
        const bool vf = fr ? vb : va;
        const int64_t ob = ((int64_t)b * p.F + fa + fr) * GLNB;
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int k = lane + 64 * u;
          const bool ok = vf && k < GLNB;
          sv[fr][u] = ok ? p.S[ob + k] : 0.f;
          tp[fr][u] = (ok && !p.first) ? p.tprev[ob + k] : make_float2(0.f, 0.f);
        }
      }
      if (r0 == 0) GLSTAMP(5);
      gl_fft1024(v, buf, twA, twB);
      if (r0 == 0) GLSTAMP(6);
      // the update of all 18 bins straight-line (a clamped bin for the lanes past Nyquist),
      // then the stores: no branch between the bins' sqrt / division chains, so they
      // interleave (bin by bin behind the branches they ran ~500 cycles each)
      float2 xo[2][9];
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int k = min(lane + 64 * u, GLNB - 1);
        const double2 zk = buf[gl_pk(k)], zn = buf[gl_pk((GLN - k) & (GLN - 1))];
        const float2 A = make_float2((float)(0.5 * (zk.x + zn.x)), (float)(0.5 * (zk.y - zn.y)));
        const float2 Bq = make_float2((float)(0.5 * (zk.y + zn.y)), (float)(-0.5 * (zk.x - zn.x)));
#pragma unroll
        for (int fr = 0; fr < 2; ++fr) {
          const float2 vv = fr ? Bq : A;
          float2 an = vv;
          if (!p.first) {
            an.x = (vv.x - (p.c * tp[fr][u].x));
            an.y = (vv.y - (p.c * tp[fr][u].y));
          }
          const float d = (cabs_rn(an.x, an.y) + 1e-16f);
          const float scl = (float)gl_rcp64((double)d);  // == 1.0f / d (see gl_rcp64)
          an.x = (an.x * scl);
          an.y = (an.y * scl);
          tp[fr][u] = vv;
          xo[fr][u] = make_float2((sv[fr][u] * an.x), (sv[fr][u] * an.y));
        }
      }
      // every bin's result exists before the first store: vmcnt counts stores too, and with
      // both pending each wait becomes vmcnt(0) — one store acknowledgement per bin (the
      // empty asm takes the results as operands, so no computation sinks into a store's
      // branch)
#pragma unroll
      for (int u = 0; u < 9; ++u)
#pragma unroll
        for (int fr = 0; fr < 2; ++fr)
          asm volatile("" ::"v"(xo[fr][u].x), "v"(xo[fr][u].y), "v"(tp[fr][u].x), "v"(tp[fr][u].y));
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int k = lane + 64 * u;
#pragma unroll
        for (int fr = 0; fr < 2; ++fr) {
          if (k < GLNB && (fr ? vb : va)) {
            const int64_t o = ((int64_t)b * p.F + fa + fr) * GLNB + k;
            p.tprev[o] = tp[fr][u];
            p.Xout[o] = xo[fr][u];
          }
        }
      }
      gl_wave_sync();  // buf is this wave's next FFT buffer
    }
    GLSTAMP(7);
  }
  }  // tile
}

// the tile shape: W waves (one FFT pair each at a time), TF analysis frames per tile.  c5
// (B = 64, F = 1400) per iteration, tools/gl_bench.py: 4 x 16 1.34 ms before the
// conflict-free twiddle tables / fma quad stage, 1.10 after; 8 x 10 (162 KB of LDS, two waves
// per SIMD) 1.42; 4 x 32 (the halo 19 % of the synthesis instead of 38 %) 0.97-1.03 ms (the
// three-kernel path: 1.47).  What bounds it (PMC, profiles/r6_pmc_gl.txt): one wave per SIMD
// — every in-flight fp64 FFT holds a 17 KB LDS exchange buffer, so LDS, not VGPRs, caps the
// CU at four — and 33 % of wave cycles parked at waitcnt / barriers
#ifndef GL_IW
#define GL_IW 4
#define GL_ITF 32
#endif

// 32-frame tiles where the batch fills the chip (c5: 2,816 tiles), 8-frame tiles below one
// tile per CU (c2's 821-frame sentence: 26 tiles of 32 would leave 230 CUs idle; 103 of 8)
constexpr int GL_SMALL_TF = 8;

// workgroups that fit the chip at once (0: unknown); each walks tiles with a stride of the
// grid, so the tables are staged once per workgroup instead of once per tile
// (workgroups per CU from the kernel's static LDS, which is what limits it: one per CU)
template <int TF>
int gl_grid(int64_t tiles) {
  constexpr int lds = gl_seg(TF) * 4 + GL_IW * GL_BUF * 16 + GLN * 8 + (GL_TWA + GL_TWB) * 16 + GLHOP * 4;
  constexpr int per = (160 * 1024) / lds;
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      n = 0;
    }
    cus = n;
  }
  const int64_t cap = (int64_t)per * cus;
  return (int)((cap > 0 && tiles > cap) ? cap : tiles);
}

template <bool FINAL>
int gl_launch(GlParams p, hipStream_t s) {
  const int big = (p.F + GL_ITF - 1) / GL_ITF;
  if ((int64_t)p.B * big >= 256) {
    p.tiles = big;
    hipLaunchKernelGGL((gl_fused_kernel<GL_IW, GL_ITF, FINAL>), dim3(gl_grid<GL_ITF>((int64_t)p.B * p.tiles)),
                       dim3(64 * GL_IW), 0, s, p);
  } else {
    p.tiles = (p.F + GL_SMALL_TF - 1) / GL_SMALL_TF;
    hipLaunchKernelGGL((gl_fused_kernel<GL_IW, GL_SMALL_TF, FINAL>),
                       dim3(gl_grid<GL_SMALL_TF>((int64_t)p.B * p.tiles)), dim3(64 * GL_IW), 0, s, p);
  }
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

int gl_check(int32_t n_fft, int32_t hop, const double *window, const double *win_sq, const void *tw) {
  if (!window || !win_sq || !tw) return FTMI_E_ARG;
  if (n_fft != GLN || hop != GLHOP) return FTMI_E_UNSUPPORTED;
  return FTMI_OK;
}

}  // namespace

#ifdef FTMI_GL_STAMPS
extern "C" int ftmi_debug_gl_stamps(unsigned long long *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ftmi_gl_stamps),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" int ftmi_griffinlim_iter(const void *Xin, void *Xout, const float *S, void *tprev,
                                    int32_t B, int32_t F, const int32_t *frames, int32_t n_fft,
                                    int32_t hop, const double *window, const double *win_sq,
                                    const void *twiddle, float c, int32_t first,
                                    ftmi_stream_t stream) {
  if (!Xin || !Xout || !S || !tprev || B <= 0 || F <= 0 || Xin == Xout) return FTMI_E_ARG;
  if (int rc = gl_check(n_fft, hop, window, win_sq, twiddle)) return rc;
  GlParams p{};
  p.Xin = (const float2 *)Xin, p.Xout = (float2 *)Xout, p.S = S, p.tprev = (float2 *)tprev;
  p.B = B, p.F = F, p.frames = frames;
  p.window = window, p.win_sq = win_sq, p.tw = (const double2 *)twiddle;
  p.c = c, p.first = first;
  return gl_launch<false>(p, ftmi_hs(stream));
}

extern "C" int ftmi_istft_fused(const void *X, int32_t B, int32_t F, const int32_t *frames,
                                int32_t n_fft, int32_t hop, const double *window,
                                const double *win_sq, const void *twiddle, float *y,
                                int64_t y_stride, int64_t y_len, ftmi_stream_t stream) {
  if (!X || !y || B <= 0 || F <= 0 || y_len < 0 || y_stride < y_len) return FTMI_E_ARG;
  if (int rc = gl_check(n_fft, hop, window, win_sq, twiddle)) return rc;
  GlParams p{};
  p.Xin = (const float2 *)X;
  p.B = B, p.F = F, p.frames = frames;
  p.window = window, p.win_sq = win_sq, p.tw = (const double2 *)twiddle;
  p.y = y, p.y_stride = y_stride, p.y_len = y_len;
  return gl_launch<true>(p, ftmi_hs(stream));
}
