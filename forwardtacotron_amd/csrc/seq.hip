// Sequence-side kernels: embedding gather, duration -> LengthRegulator counts / index map,
// LengthRegulator expansion, pitch/energy conditioning, SeriesPredictor head.
// All are HBM/latency-bound integer or byte-moving work: coalesced float4 rows, no MFMA.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------------------
// nn.Embedding (models/forward_tacotron.py:125,304 ; :31,47)
__global__ void embedding_kernel(const int64_t *__restrict__ ids, int64_t n,
                                 const float *__restrict__ table, int64_t rows, int dim4,
                                 float *__restrict__ out, int32_t *err) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid / dim4;
  const int q = (int)(gid - r * dim4);
  if (r >= n) return;
  const int64_t id = ids[r];
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (id >= 0 && id < rows)
    v = ((const f32x4 *)(table + id * (int64_t)dim4 * 4))[q];
  else if (err && q == 0)
    *err = 1;
  ((f32x4 *)(out + r * (int64_t)dim4 * 4))[q] = v;
}

// ---------------------------------------------------------------------------------------
// generate()'s fill-2 rule (forward_tacotron.py:254-255) + LengthRegulator clip/count
// (common_layers.py:13,16) + per-row exclusive scan.  One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void duration_counts_kernel(float *dur, int B, int T,
                                                               int apply_fill, float fill,
                                                               int32_t *offsets, int32_t *totals,
                                                               int32_t *fill_flag,
                                                               const int64_t *ext_sum) {
  __shared__ long long s_part[16];
  __shared__ int s_fill;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t n = (int64_t)B * T;
  if (apply_fill && ext_sum) {  // batch-global decision (sharded batch): sum over all shards
    if (tid == 0) {
      s_fill = *ext_sum <= 0;
      if (fill_flag) *fill_flag = s_fill;
    }
    __syncthreads();
    if (s_fill)
      for (int64_t i = tid; i < n; i += 1024) dur[i] = fill;
    __syncthreads();
  } else if (apply_fill) {
    long long acc = 0;
    for (int64_t i = tid; i < n; i += 1024) acc += (long long)dur[i];  // trunc toward 0
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (lane == 0) s_part[wave] = acc;
    __syncthreads();
    if (tid == 0) {
      long long s = 0;
      for (int w = 0; w < 16; ++w) s += s_part[w];
      s_fill = s <= 0;
      if (fill_flag) *fill_flag = s_fill;
    }
    __syncthreads();
    if (s_fill)
      for (int64_t i = tid; i < n; i += 1024) dur[i] = fill;
    __syncthreads();
  } else if (fill_flag && tid == 0) {
    *fill_flag = 0;
  }
  // one wave per row: clip in place, count = int(fp32(dur + 0.5)), exclusive scan
  for (int b = wave; b < B; b += 16) {
    float *row = dur + (int64_t)b * T;
    int32_t *off = offsets + (int64_t)b * (T + 1);
    int carry = 0;
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + lane;
      int c = 0;
      if (t < T) {
        float d = row[t];
        if (d < 0.f) {
          d = 0.f;
          row[t] = d;
        }
        const float s = __fadd_rn(d, 0.5f);
        c = (int)s;  // truncation, as torch .long()
      }
      int incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      if (t < T) off[t] = carry + incl - c;
      carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) {
      off[T] = carry;
      totals[b] = carry;
    }
  }
}

// LengthRegulator frame -> phoneme map (repeat_interleave + pad_sequence, common_layers.py:15-18)
__global__ void lr_index_kernel(const int32_t *__restrict__ offsets, int B, int T, int T_mel,
                                int32_t *__restrict__ index) {
  const int b = blockIdx.y;
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= T_mel) return;
  const int32_t *off = offsets + (int64_t)b * (T + 1);
  int r = -1;
  if (f < off[T]) {
    int lo = 0, hi = T - 1;  // largest t with off[t] <= f
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= f)
        lo = mid;
      else
        hi = mid - 1;
    }
    r = lo;
  }
  index[(int64_t)b * T_mel + f] = r;
}

// y[b,f,:] = x[b,index[b,f],:] or 0 — one wave per frame row, float4 lanes
__global__ void length_regulate_kernel(const float *__restrict__ x, int64_t x_stride, int T,
                                       int C4, const int32_t *__restrict__ index, int64_t rows,
                                       int T_mel, float *__restrict__ y, int64_t y_stride) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int64_t b = r / T_mel;
  const int src = index[r];
  const f32x4 *xs = (const f32x4 *)(x + (b * T + (src < 0 ? 0 : src)) * x_stride);
  f32x4 *yd = (f32x4 *)(y + r * y_stride);
  for (int q = lane; q < C4; q += 64) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (src >= 0) v = xs[q];
    yd[q] = v;
  }
}

// the same on 4 channels per thread (C % 4 == 0, 16-B aligned rows) for a chunk of SP_ROWS
// rows: the 4 channels' weights (3 taps x 2 series + 2 biases) are loaded once into
// registers and reused for every row of the chunk (re-reading them per row moved 8x the x
// bytes through L2 in the folded form, where x is the (B, T, 4H) LSTM input projection)
constexpr int SP_ROWS = 32;
__global__ __launch_bounds__(256) void series_proj_add4_kernel(
    float *x, int64_t x_stride, int B, int T, int C, const float *__restrict__ pitch,
    const float *__restrict__ wp, const float *__restrict__ bp, float ps,
    const float *__restrict__ energy, const float *__restrict__ we,
    const float *__restrict__ be, float es) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= C) return;
  float wpa[12], wea[12];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const f32x4 a = *(const f32x4 *)(wp + 3 * c + 4 * q), d = *(const f32x4 *)(we + 3 * c + 4 * q);
    wpa[4 * q] = a.x; wpa[4 * q + 1] = a.y; wpa[4 * q + 2] = a.z; wpa[4 * q + 3] = a.w;
    wea[4 * q] = d.x; wea[4 * q + 1] = d.y; wea[4 * q + 2] = d.z; wea[4 * q + 3] = d.w;
  }
  const f32x4 bpv = *(const f32x4 *)(bp + c), bev = *(const f32x4 *)(be + c);
  const int64_t rows = (int64_t)B * T;
  const int64_t r0 = (int64_t)blockIdx.y * SP_ROWS;
  for (int64_t r = r0; r < r0 + SP_ROWS && r < rows; ++r) {
    const int b = (int)(r / T), t = (int)(r - (int64_t)b * T);
    const float *pr = pitch + (int64_t)b * T;
    const float *er = energy + (int64_t)b * T;
    const float p0 = t > 0 ? pr[t - 1] : 0.f, p1 = pr[t], p2 = t + 1 < T ? pr[t + 1] : 0.f;
    const float e0 = t > 0 ? er[t - 1] : 0.f, e1 = er[t], e2 = t + 1 < T ? er[t + 1] : 0.f;
    float *xr = x + r * x_stride + c;
    f32x4 v = *(f32x4 *)xr;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float P = bpv[e] + wpa[3 * e] * p0 + wpa[3 * e + 1] * p1 + wpa[3 * e + 2] * p2;
      const float E = bev[e] + wea[3 * e] * e0 + wea[3 * e + 1] * e1 + wea[3 * e + 2] * e2;
      float u = v[e];
      u = u + P * ps;
      u = u + E * es;
      v[e] = u;
    }
    *(f32x4 *)xr = v;
  }
}

// x += proj(pitch)*ps ; x += proj(energy)*es   (forward_tacotron.py:308-314)
__global__ void series_proj_add_kernel(float *x, int64_t x_stride, int B, int T, int C,
                                       const float *__restrict__ pitch,
                                       const float *__restrict__ wp, const float *__restrict__ bp,
                                       float ps, const float *__restrict__ energy,
                                       const float *__restrict__ we, const float *__restrict__ be,
                                       float es) {
  const int64_t r = blockIdx.x;  // (b, t) row
  const int b = (int)(r / T), t = (int)(r - (int64_t)b * T);
  const float *pr = pitch + (int64_t)b * T;
  const float *er = energy + (int64_t)b * T;
  const float p0 = t > 0 ? pr[t - 1] : 0.f, p1 = pr[t], p2 = t + 1 < T ? pr[t + 1] : 0.f;
  const float e0 = t > 0 ? er[t - 1] : 0.f, e1 = er[t], e2 = t + 1 < T ? er[t + 1] : 0.f;
  float *xr = x + r * x_stride;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float P = bp[c] + wp[3 * c] * p0 + wp[3 * c + 1] * p1 + wp[3 * c + 2] * p2;
    const float E = be[c] + we[3 * c] * e0 + we[3 * c + 1] * e1 + we[3 * c + 2] * e2;
    float v = xr[c];
    v = v + P * ps;
    v = v + E * es;
    xr[c] = v;
  }
}

// out[m] = (x[m,:] . w + bias) / alpha  — one wave per row
__global__ void rowdot_kernel(const float *__restrict__ x, int64_t x_stride, int64_t M, int C,
                              const float *__restrict__ w, const float *__restrict__ bias,
                              float alpha, float *__restrict__ out) {
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  const float *xr = x + m * x_stride;
  float acc = 0.f;
  for (int c = lane; c < C; c += 64) acc = fmaf(xr[c], w[c], acc);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) out[m] = (acc + (bias ? bias[0] : 0.f)) / alpha;
}

}  // namespace

extern "C" int ftmi_embedding(const int64_t *ids, int64_t n, const float *table,
                              int64_t num_rows, int64_t dim, float *out, int32_t *err,
                              ftmi_stream_t stream) {
  if (!ids || !table || !out || n < 0 || num_rows <= 0 || dim <= 0) return FTMI_E_ARG;
  if (dim % 4) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(table) || !ftmi_aligned16(out)) return FTMI_E_ALIGN;
  if (n == 0) return FTMI_OK;
  const int dim4 = (int)(dim / 4);
  const int64_t threads = n * dim4;
  hipLaunchKernelGGL(embedding_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     ftmi_hs(stream), ids, n, table, num_rows, dim4, out, err);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_duration_counts(float *dur, int32_t B, int32_t T, int32_t apply_fill,
                                    float fill_value, int32_t *offsets, int32_t *totals,
                                    int32_t *fill_flag, ftmi_stream_t stream) {
  if (!dur || !offsets || !totals || B <= 0 || T <= 0) return FTMI_E_ARG;
  hipLaunchKernelGGL(duration_counts_kernel, dim3(1), dim3(1024), 0, ftmi_hs(stream), dur, B, T,
                     apply_fill, fill_value, offsets, totals, fill_flag, (const int64_t *)nullptr);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

namespace {
__global__ __launch_bounds__(1024) void trunc_sum_kernel(const float *dur, int64_t n, int64_t *out) {
  __shared__ long long part[16];
  long long acc = 0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) acc += (long long)dur[i];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long s = 0;
    for (int w = 0; w < 16; ++w) s += part[w];
    *out = s;
  }
}
}  // namespace

extern "C" int ftmi_duration_trunc_sum(const float *dur, int32_t B, int32_t T, int64_t *out,
                                       ftmi_stream_t stream) {
  if (!dur || !out || B <= 0 || T <= 0) return FTMI_E_ARG;
  hipLaunchKernelGGL(trunc_sum_kernel, dim3(1), dim3(1024), 0, ftmi_hs(stream), dur, (int64_t)B * T, out);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_duration_counts_global(float *dur, int32_t B, int32_t T,
                                           const int64_t *global_sum, float fill_value,
                                           int32_t *offsets, int32_t *totals, int32_t *fill_flag,
                                           ftmi_stream_t stream) {
  if (!dur || !offsets || !totals || !global_sum || B <= 0 || T <= 0) return FTMI_E_ARG;
  hipLaunchKernelGGL(duration_counts_kernel, dim3(1), dim3(1024), 0, ftmi_hs(stream), dur, B, T, 1,
                     fill_value, offsets, totals, fill_flag, global_sum);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_lr_index(const int32_t *offsets, int32_t B, int32_t T, int32_t T_mel,
                             int32_t *index, ftmi_stream_t stream) {
  if (!offsets || !index || B <= 0 || T <= 0 || T_mel < 0) return FTMI_E_ARG;
  if (T_mel == 0) return FTMI_OK;
  hipLaunchKernelGGL(lr_index_kernel, dim3((T_mel + 255) / 256, B), dim3(256), 0,
                     ftmi_hs(stream), offsets, B, T, T_mel, index);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_length_regulate(const float *x, int64_t x_stride, int32_t B, int32_t T,
                                    int32_t C, const int32_t *index, int32_t T_mel, float *y,
                                    int64_t y_stride, ftmi_stream_t stream) {
  if (!x || !index || !y || B <= 0 || T <= 0 || C <= 0 || T_mel < 0) return FTMI_E_ARG;
  if (C % 4 || (x_stride & 3) || (y_stride & 3)) return FTMI_E_ALIGN;
  if (!ftmi_aligned16(x) || !ftmi_aligned16(y)) return FTMI_E_ALIGN;
  const int64_t rows = (int64_t)B * T_mel;
  if (rows == 0) return FTMI_OK;
  hipLaunchKernelGGL(length_regulate_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     ftmi_hs(stream), x, x_stride, T, C / 4, index, rows, T_mel, y, y_stride);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_series_proj_add(float *x, int64_t x_stride, int32_t B, int32_t T, int32_t C,
                                    const float *pitch, const float *wp, const float *bp,
                                    float pitch_strength, const float *energy, const float *we,
                                    const float *be, float energy_strength,
                                    ftmi_stream_t stream) {
  if (!x || !pitch || !wp || !bp || !energy || !we || !be) return FTMI_E_ARG;
  if (B <= 0 || T <= 0 || C <= 0) return FTMI_E_ARG;
  const bool vec = C % 4 == 0 && !(x_stride & 3) && ftmi_aligned16(x) && ftmi_aligned16(wp) &&
                   ftmi_aligned16(we) && ftmi_aligned16(bp) && ftmi_aligned16(be);
  if (vec) {
    const int64_t rows = (int64_t)B * T;
    hipLaunchKernelGGL(series_proj_add4_kernel,
                       dim3((unsigned)((C / 4 + 255) / 256), (unsigned)((rows + SP_ROWS - 1) / SP_ROWS)),
                       dim3(256), 0, ftmi_hs(stream), x, x_stride, B, T, C, pitch, wp, bp,
                       pitch_strength, energy, we, be, energy_strength);
    FTMI_CHECK_LAUNCH();
    return FTMI_OK;
  }
  hipLaunchKernelGGL(series_proj_add_kernel, dim3((unsigned)((int64_t)B * T)), dim3(256), 0,
                     ftmi_hs(stream), x, x_stride, B, T, C, pitch, wp, bp, pitch_strength,
                     energy, we, be, energy_strength);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_rowdot(const float *x, int64_t x_stride, int64_t M, int32_t C,
                           const float *w, const float *bias, float alpha, float *out,
                           ftmi_stream_t stream) {
  if (!x || !w || !out || M < 0 || C <= 0) return FTMI_E_ARG;
  if (M == 0) return FTMI_OK;
  hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     ftmi_hs(stream), x, x_stride, M, C, w, bias, alpha, out);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_abi_version(void) { return 19; }

static int g_cu_limit = 0;

extern "C" int32_t ftmi_set_resident_cu_limit(int32_t cus) {
  const int prev = g_cu_limit;
  g_cu_limit = cus > 0 ? cus : 0;
  return prev;
}

__attribute__((visibility("hidden"))) int ftmi_resident_cus(void) {
  static int dev_cus = 0;
  if (dev_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      dev_cus = n;
    else
      return 0;  // no device: nothing can be resident
  }
  return (g_cu_limit > 0 && g_cu_limit < dev_cus) ? g_cu_limit : dev_cus;
}

extern "C" const char *ftmi_strerror(int code) {
  switch (code) {
    case FTMI_OK: return "ok";
    case FTMI_E_ARG: return "ftmi: invalid argument (null pointer or non-positive size)";
    case FTMI_E_SHAPE: return "ftmi: unsupported shape";
    case FTMI_E_UNSUPPORTED: return "ftmi: configuration without a compiled kernel";
    case FTMI_E_ALIGN: return "ftmi: pointer or stride not 16-byte aligned";
    default: return hipGetErrorString((hipError_t)code);
  }
}
