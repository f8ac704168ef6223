// FastPitch transformer pieces (models/fast_pitch.py) on gfx950: token embedding +
// positional encoding (PositionalEncoding :16-33), LayerNorm (FFTBlock norm1/norm2,
// ForwardTransformer.norm), and fused multi-head self-attention (FFTBlock.self_attn =
// nn.MultiheadAttention, math path: softmax(q/sqrt(E) k^T + key_padding_mask) v) as one
// flash-style kernel on fp32 MFMA (v_mfma_f32_16x16x4_f32: products exact in fp32, only
// the summation order differs from the reference's bmm).  The projections (in_proj,
// out_proj, conv1 k9, conv2 k1) run on the GEMM family (gemm.hip).
#include "common.h"

// hipcc contracts a*b+c into FMA by default (-ffp-contract=fast; the __fmul_rn family is
// header-inlined and contracts too): the reference-order float32 roundings below need
// every multiply and add rounded on its own.
#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------- embedding + posenc
// out[b,t,:] = table[ids[b,t], :] + scale * pe[t, :]   (float32 mul, then add: torch order)
__global__ void embed_posenc_kernel(const int64_t *__restrict__ ids, int T, int64_t n,
                                    const float *__restrict__ table, int64_t rows, int dim,
                                    const float *__restrict__ pe, const float *__restrict__ scale,
                                    float *__restrict__ out, int32_t *err) {
  const float s = *scale;
  const int64_t total = n * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / dim;
    const int c = (int)(i - r * dim);
    const int t = (int)(r % T);
    const int64_t id = ids[r];
    float v = 0.f;
    if (id < 0 || id >= rows) {
      if (err) atomicOr(err, 1);
    } else {
      v = table[id * dim + c];
    }
    out[i] = v + s * pe[(int64_t)t * dim + c];
  }
}

// LengthRegulator expansion fused with the postnet's positional encoding:
// y[b,t,:] = (index[b,t] >= 0 ? x[b,index[b,t],:] : 0) + scale * pe[t,:]
__global__ void lr_posenc_kernel(const float *__restrict__ x, int64_t xs, int T, int C,
                                 const int32_t *__restrict__ index, int T_mel, int64_t n,
                                 const float *__restrict__ pe, const float *__restrict__ scale,
                                 float *__restrict__ y, int64_t ys) {
  const float s = *scale;
  const int64_t total = n * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C;
    const int c = (int)(i - r * C);
    const int b = (int)(r / T_mel), t = (int)(r - (int64_t)b * T_mel);
    const int src = index[r];
    const float v = src >= 0 ? x[((int64_t)b * T + src) * xs + c] : 0.f;
    y[r * ys + c] = v + s * pe[(int64_t)t * C + c];
  }
}

// ---------------------------------------------------------------- LayerNorm
// one wave per row; mean / variance accumulated in fp64 (biased variance, torch), then
// y = (x * rstd + (-rstd * mean)) * gamma + beta with the reference kernel's rounding order
template <int VPL>
__global__ __launch_bounds__(256) void layernorm_kernel(const float *__restrict__ x, int64_t xs,
                                                        int64_t M, int C, const float *__restrict__ g,
                                                        const float *__restrict__ bt, float eps,
                                                        float *__restrict__ y, int64_t ys) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float *xr = x + row * xs;
  float v[VPL];
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? xr[c] : 0.f;
    s += v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double mean = s / C;
  double q = 0.0;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    const double d = (double)v[j] - mean;
    if (c < C) q += d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = (float)(1.0 / sqrt(q / C + (double)eps));
  const float meanf = (float)mean;
  const float bias = -(rstd * meanf);
  float *yr = y + row * ys;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < C) yr[c] = (v[j] * rstd + bias) * g[c] + bt[c];
  }
}

// ---------------------------------------------------------------- attention
// grid (ceil(T/64), B*H), 256 threads: wave w owns query rows tile*64 + 16w .. +16.
// Key / value tiles of 32 keys are staged in LDS (fp32) and shared by the 4 waves;
// online softmax in registers (MFMA C layout: lane holds rows 4(lane>>4)+i, col lane&15).
constexpr int AT_KT = 32;

// max / sum over the 16 lanes of a DPP row (the 16 columns of an MFMA row group):
// rotations by 8, 4, 2, 1 within the row (row_ror), VALU only — the ds_bpermute of
// __shfl_xor is an LDS-pipe op with ~100 cycles of latency per step of the chain
template <int CTRL>
__device__ __forceinline__ float dpp_ror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                               __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}
#define FTMI_ROW16(OP, v)             \
  do {                                \
    v = OP(v, dpp_ror<0x128>(v));     \
    v = OP(v, dpp_ror<0x124>(v));     \
    v = OP(v, dpp_ror<0x122>(v));     \
    v = OP(v, dpp_ror<0x121>(v));     \
  } while (0)
__device__ __forceinline__ float add2(float a, float b) { return a + b; }

// PRE staging of the last key tile: 8 f16 keys key0 .. key0 + 7 of one plane row with the
// keys >= T zeroed.  The workspace's pad keys T..Tp-1 are never written by the producers and
// may hold a non-finite value left by an earlier, overflowing call (it reran on the exact
// path); a masked key has P = 0, and 0 * inf in the P V MFMA would be NaN.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t zero_keys_past(u32x4_t v, int key0, int T) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = key0 + 2 * i;  // word i = keys k (low half) and k + 1 (high half)
    v[i] &= k >= T ? 0u : (k + 1 >= T ? 0xFFFFu : 0xFFFFFFFFu);
  }
  return v;
}

template <int HD>
__global__ __launch_bounds__(256) void attention_kernel(const float *__restrict__ qkv, int64_t rs,
                                                        int B, int T, int H, int q_off, int k_off,
                                                        int v_off, const uint8_t *__restrict__ kpm,
                                                        float qscale, float *__restrict__ out,
                                                        int64_t os) {
  constexpr int KS = HD + 2;   // K row stride (floats): b32 B-operand reads conflict-free
  constexpr int VS = HD + 16;  // V row stride
  constexpr int PS = AT_KT + 2;
  constexpr int NT = HD / 16;  // output column tiles
  __shared__ float Ks[AT_KT * KS];
  __shared__ float Vs[AT_KT * VS];
  __shared__ float Ps[4][16 * PS];

  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int q0 = blockIdx.x * 64 + wave * 16;
  const float *base = qkv + (int64_t)b * T * rs;

  // A-operand fragments of this wave's 16 query rows, pre-scaled like the reference
  float qa[HD / 4];
  {
    const int qr = q0 + c16;
    const float *src = base + (int64_t)(qr < T ? qr : 0) * rs + q_off + h * HD;
#pragma unroll
    for (int ks = 0; ks < HD / 4; ++ks) qa[ks] = qr < T ? (src[4 * ks + g] * qscale) : 0.f;
  }
  f32x4 o[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
  }

  for (int k0 = 0; k0 < T; k0 += AT_KT) {
    __syncthreads();
    // stage K and V rows k0 .. k0+31 (zero past T)
    for (int e = threadIdx.x; e < AT_KT * HD / 4; e += 256) {
      const int r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4;
      const int key = k0 + r;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (key < T) {
        const float *row = base + (int64_t)key * rs + h * HD + c4;
        kv = *(const f32x4 *)(row + k_off);
        vv = *(const f32x4 *)(row + v_off);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Ks[r * KS + c4 + j] = kv[j];
        Vs[r * VS + c4 + j] = vv[j];
      }
    }
    __syncthreads();
    // S = (q c) K^T for 16 rows x 32 keys
    f32x4 s[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < HD / 4; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[ks], Ks[(n * 16 + c16) * KS + 4 * ks + g], acc,
                                                   0, 0, 0);
      s[n] = acc;
    }
    // mask: keys past T or flagged in key_padding_mask -> -inf (baddbmm with the float mask)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int key = k0 + n * 16 + c16;
      const bool dead = key >= T || (kpm && kpm[(int64_t)b * T + key]);
      if (dead)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[n][i] = -INFINITY;
    }
    // online softmax per row (rows 4g+i; the 16 lanes of group g hold its columns)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mx = fmaxf(s[0][i], s[1][i]);
#pragma unroll
      FTMI_ROW16(fmaxf, mx);
      const float mn = fmaxf(m[i], mx);
      const float alpha = mn == -INFINITY ? 1.f : expf(m[i] - mn);
      float ps = 0.f;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float pv = mn == -INFINITY ? 0.f : expf(s[n][i] - mn);
        s[n][i] = pv;
        ps += pv;
      }
#pragma unroll
      FTMI_ROW16(add2, ps);
      l[i] = l[i] * alpha + ps;
      m[i] = mn;
#pragma unroll
      for (int n = 0; n < NT; ++n) o[n][i] *= alpha;
    }
    // P (C layout) -> LDS -> A layout
    float *P = Ps[wave];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) P[(4 * g + i) * PS + n * 16 + c16] = s[n][i];
    __syncthreads();
    // O += P V
#pragma unroll
    for (int ks = 0; ks < AT_KT / 4; ++ks) {
      const float pa = P[c16 * PS + 4 * ks + g];
#pragma unroll
      for (int n = 0; n < NT; ++n)
        o[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, Vs[(4 * ks + g) * VS + n * 16 + c16], o[n],
                                                    0, 0, 0);
    }
  }
  // normalise and store
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qr = q0 + 4 * g + i;
    if (qr >= T) continue;
    float *dst = out + ((int64_t)b * T + qr) * os + h * HD;
    const float inv = l[i];
#pragma unroll
    for (int n = 0; n < NT; ++n) dst[n * 16 + c16] = o[n][i] / inv;
  }
}

// ---------------------------------------------------------------- attention, f16x3
// The same flash-style self-attention with both contractions on the f16x3 split (the GEMM
// family's default path, gemm.hip): every operand x = x_h + 2^-11 x_t (f16 head, scaled f16
// tail) and a product of two split operands = a_h b_h + 2^-11 (a_t b_h + a_h b_t) (dropped
// term < 2^-22 relative) — here the big term and the two small ones go to separate
// accumulators (no 2^11-scaled head, so any |x| < 65504 is in range), combined once.
// v_mfma_f32_16x16x32_f16.  Workgroup = 8 waves x 16 queries; key tiles of 64: per tile and
// wave S = (q c) K^T is 4 key blocks x HD/32 k-steps x 3 MFMAs and O += P V is 2 k-steps x
// HD/16 column tiles x 3 MFMAs.  The softmax stays fp32 (online; exponentials on v_exp_f32,
// |error| ~1 ulp of the argument's product with log2 e).  K is staged [key][d] and V
// transposed [d][key] in LDS as f16 head / tail planes with row pitches that keep the
// ds_read_b128 fragment reads conflict free.  An operand beyond the f16 range sets bit 0
// of *status (the caller reruns on the fp32 kernel).
constexpr int AH_W = 8;    // waves (x 16 queries) per workgroup of the f16x3 kernel
constexpr int AH_KT = 64;  // keys per tile
constexpr float AH_LAZY = 8.f;  // lazy running max: P <= e^8 between moves of the max

// PRE: K and V come pre-split from attn_split_kv_kernel (kv: f16 planes K head, K tail
// [B*H][Tp][HD] and V head, V tail transposed [B*H][HD][Tp]): the tile staging is a copy, the
// split VALU (which every query tile of a head repeated) is gone.
template <int HD, bool PRE>
__global__ __launch_bounds__(64 * AH_W) void attention_h3_kernel(
    const float *__restrict__ qkv, int64_t rs, int B, int T, int H, int q_off, int k_off,
    int v_off, const uint8_t *__restrict__ kpm, float qscale, float *__restrict__ out,
    int64_t os, unsigned *status, const _Float16 *__restrict__ kv, int Tp) {
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  constexpr int NTH = 64 * AH_W;
  constexpr float TS = 2048.f, TU = 1.f / 2048.f;  // tail scale 2^11
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr int KP = HD + 16;      // K row pitch (halves)
  constexpr int VP = AH_KT + 16;   // V^T row pitch (halves)
  constexpr int PP = AH_KT + 4;    // P row pitch (floats)
  constexpr int NT = HD / 16;      // output column tiles
  constexpr int KQ = HD / 32;      // k-steps of q k^T
  constexpr int NB = AH_KT / 16;   // key blocks per tile
  constexpr int KK = AH_KT / 32;   // k-steps of P V
  __shared__ __attribute__((aligned(16))) _Float16 Kh[AH_KT * KP], Kt[AH_KT * KP];
  __shared__ __attribute__((aligned(16))) _Float16 Vh[HD * VP], Vt[HD * VP];
  __shared__ __attribute__((aligned(16))) float Ps[AH_W][16 * PP];

  // XCD-aware order (1-D grid): the query tiles of one (batch, head) are consecutive blocks
  // of ONE XCD (blocks L and L + 8 share an XCD), so its K / V rows are fetched into that
  // XCD's L2 once and re-read from there by every query tile; with (B H) % 8 != 0 the plain
  // order (tile fastest).
  const int nq = (T + 16 * AH_W - 1) / (16 * AH_W), nbh = B * H;
  int bh, qtile;
  if (nbh % 8 == 0) {
    const int L = blockIdx.x, q8 = L >> 3;
    bh = (L & 7) + 8 * (q8 / nq);
    qtile = q8 % nq;
  } else {
    bh = blockIdx.x / nq;
    qtile = blockIdx.x % nq;
  }
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int q0 = qtile * 16 * AH_W + wave * 16;
  const float *base = qkv + (int64_t)b * T * rs;
  float amax = 0.f;  // range guard

  auto split8 = [&](const f32x4 a, const f32x4 c, f16x8 &hd, f16x8 &tl) {
    float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      amax = fmaxf(amax, fabsf(v[e]));
      const _Float16 hh = (_Float16)v[e];
      hd[e] = hh;
      tl[e] = (_Float16)((v[e] - (float)hh) * TS);
    }
  };

  // P in [0, e^AH_LAZY]: split without the range guard (packed conversions)
  auto split8p = [&](const f32x4 a, const f32x4 c, f16x8 &hd, f16x8 &tl) {
    typedef float f32x8 __attribute__((ext_vector_type(8)));
    const f32x8 v = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    hd = __builtin_convertvector(v, f16x8);
    tl = __builtin_convertvector((v - __builtin_convertvector(hd, f32x8)) * TS, f16x8);
  };

  // A fragments of this wave's 16 query rows (lane: row c16, d = 32 ks + 8 g + j), scaled by
  // qscale in fp32 first, like the reference
  f16x8 qh[KQ], qt[KQ];
  {
    const int qr = q0 + c16;
    const float *src = base + (int64_t)(qr < T ? qr : 0) * rs + q_off + h * HD;
#pragma unroll
    for (int ks = 0; ks < KQ; ++ks) {
      f32x4 a = *(const f32x4 *)(src + 32 * ks + 8 * g);
      f32x4 c = *(const f32x4 *)(src + 32 * ks + 8 * g + 4);
      if (qr >= T) a = c = (f32x4){0.f, 0.f, 0.f, 0.f};
      split8(a * qscale, c * qscale, qh[ks], qt[ks]);
    }
  }
  f32x4 ob[NT], osm[NT];  // P V: big term, small terms (x 2^11)
#pragma unroll
  for (int n = 0; n < NT; ++n) ob[n] = osm[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
  }

  // ---- K / V tile staging, software-pipelined: the global loads of tile k0 + AH_KT are in
  // flight (registers) while tile k0 is multiplied; after the next barrier they are split
  // (or, PRE, copied) into the LDS planes.  Without it every tile waited the full memory
  // latency (PMC: 53 % of wave cycles in waits, MFMA 17 % busy).
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int NKC = PRE ? 2 * AH_KT * HD / 8 / NTH : AH_KT * HD / 4 / NTH;  // K slots
  constexpr int NVC = PRE ? 2 * HD * AH_KT / 8 / NTH : HD * (AH_KT / 8) / NTH;  // V slots
  static_assert(NKC * NTH == (PRE ? 2 * AH_KT * HD / 8 : AH_KT * HD / 4) &&
                NVC * NTH == (PRE ? 2 * HD * AH_KT / 8 : HD * (AH_KT / 8)), "staging slots");
  u32x4 kr[NKC], vr[PRE ? NVC : 1];
  float vs[PRE ? 1 : NVC][8];
  const size_t plane = PRE ? (size_t)B * H * Tp * HD : 0;
  const int last0 = (T - 1) / AH_KT * AH_KT;  // start of the last tile
  auto load_tile = [&](int k0) {
    k0 = k0 < last0 ? k0 : last0;  // past the end: a clamped (unused) reload
    if constexpr (PRE) {
      const _Float16 *kb = kv + ((size_t)bh * Tp + k0) * HD;
      const _Float16 *vb = kv + 2 * plane + (size_t)bh * HD * Tp + k0;
#pragma unroll
      for (int i = 0; i < NKC; ++i) {
        const int e = tid + NTH * i, pl = e / (AH_KT * HD / 8), q = e - pl * (AH_KT * HD / 8);
        const int r = q / (HD / 8), c8 = (q - r * (HD / 8)) * 8;
        kr[i] = *(const u32x4 *)(kb + pl * plane + (size_t)r * HD + c8);
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {
        const int e = tid + NTH * i, pl = e / (HD * AH_KT / 8), q = e - pl * (HD * AH_KT / 8);
        const int d = q / (AH_KT / 8), c8 = (q - d * (AH_KT / 8)) * 8;
        vr[i] = *(const u32x4 *)(vb + pl * plane + (size_t)d * Tp + c8);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NKC; ++i) {  // K: one float4 of a key row (row clamped to T - 1)
        const int e = tid + NTH * i, r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4;
        const int key = min(k0 + r, T - 1);
        kr[i] = *(const u32x4 *)(base + (int64_t)key * rs + k_off + h * HD + c4);
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {  // V: 8 keys of one column d
        const int e = tid + NTH * i, d = e % HD, kg = e / HD;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int key = min(k0 + kg * 8 + j, T - 1);
          vs[i][j] = base[(int64_t)key * rs + v_off + h * HD + d];
        }
      }
    }
  };
  auto store_tile = [&](int k0) {
    if constexpr (PRE) {
      const bool tail = k0 + AH_KT > T;  // the last tile: pad keys are zeroed (uniform)
#pragma unroll
      for (int i = 0; i < NKC; ++i) {
        const int e = tid + NTH * i, pl = e / (AH_KT * HD / 8), q = e - pl * (AH_KT * HD / 8);
        const int r = q / (HD / 8), c8 = (q - r * (HD / 8)) * 8;
        u32x4 kk = kr[i];
        if (tail && k0 + r >= T) kk = (u32x4){0u, 0u, 0u, 0u};
        *(u32x4 *)&(pl ? Kt : Kh)[r * KP + c8] = kk;
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {
        const int e = tid + NTH * i, pl = e / (HD * AH_KT / 8), q = e - pl * (HD * AH_KT / 8);
        const int d = q / (AH_KT / 8), c8 = (q - d * (AH_KT / 8)) * 8;
        *(u32x4 *)&(pl ? Vt : Vh)[d * VP + c8] = tail ? zero_keys_past(vr[i], k0 + c8, T) : vr[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NKC; ++i) {
        const int e = tid + NTH * i, r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4;
        f32x4 kvv = __builtin_bit_cast(f32x4, kr[i]);
        if (k0 + r >= T) kvv = (f32x4){0.f, 0.f, 0.f, 0.f};
        f16x4 hh, tt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          amax = fmaxf(amax, fabsf(kvv[j]));
          hh[j] = (_Float16)kvv[j];
          tt[j] = (_Float16)((kvv[j] - (float)hh[j]) * TS);
        }
        *(f16x4 *)&Kh[r * KP + c4] = hh;
        *(f16x4 *)&Kt[r * KP + c4] = tt;
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {
        const int e = tid + NTH * i, d = e % HD, kg = e / HD;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = k0 + kg * 8 + j < T ? vs[i][j] : 0.f;
        f16x8 hh, tt;
        split8((f32x4){v[0], v[1], v[2], v[3]}, (f32x4){v[4], v[5], v[6], v[7]}, hh, tt);
        *(f16x8 *)&Vh[d * VP + kg * 8] = hh;
        *(f16x8 *)&Vt[d * VP + kg * 8] = tt;
      }
    }
  };
  load_tile(0);

  for (int k0 = 0; k0 < T; k0 += AH_KT) {
    __syncthreads();  // every wave is done with the previous tile's LDS planes
    store_tile(k0);
    __syncthreads();
    load_tile(k0 + AH_KT);
    // ---- S = (q c) K^T: 16 rows x AH_KT keys
    f32x4 s[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      f32x4 big = {0.f, 0.f, 0.f, 0.f}, sm = {0.f, 0.f, 0.f, 0.f};
      const int o = (n * 16 + c16) * KP + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KQ; ++ks) {
        const f16x8 kh = *(const f16x8 *)&Kh[o + 32 * ks];
        const f16x8 kt = *(const f16x8 *)&Kt[o + 32 * ks];
        sm = __builtin_amdgcn_mfma_f32_16x16x32_f16(qt[ks], kh, sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[ks], kt, sm, 0, 0, 0);
        big = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[ks], kh, big, 0, 0, 0);
      }
      s[n] = big + sm * TU;
      // mask: keys past T or flagged in key_padding_mask -> -inf (only a tile that reaches
      // past T, or with a mask, has any: a uniform branch)
      if (k0 + AH_KT > T || kpm) {
        const int key = k0 + n * 16 + c16;
        const bool dead = key >= T || (kpm && kpm[(int64_t)b * T + key]);
        if (dead)
#pragma unroll
          for (int i = 0; i < 4; ++i) s[n][i] = -INFINITY;
      }
    }
    // ---- online softmax per row (rows 4g+i; the 16 lanes of group g hold its columns) with
    // a lazy running max: m moves only when a row's tile max exceeds it by more than
    // AH_LAZY (so P = exp(s - m) <= e^AH_LAZY, far inside the f16 range of the P split), and
    // the O rescale runs only on tiles where some row of the wave moved it — the same
    // softmax, exp(s - m) / sum exp(s - m) for whichever m, up to rounding
    bool moved = false;
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mx = s[0][i];
#pragma unroll
      for (int n = 1; n < NB; ++n) mx = fmaxf(mx, s[n][i]);
#pragma unroll
      FTMI_ROW16(fmaxf, mx);
      const bool up = mx > m[i] + AH_LAZY;  // false while the row has only masked keys
      const float mn = up ? mx : m[i];
      alpha[i] = up ? __builtin_amdgcn_exp2f((m[i] - mn) * LOG2E) : 1.f;  // exp2(-inf) = 0
      moved |= up;
      // P = 2^(s log2e - m log2e): one FMA per score; a row without a live key yet has
      // m = -inf and only -inf scores: P = 0
      const float off = mn == -INFINITY ? 0.f : -mn * LOG2E;
      float ps = 0.f;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(s[n][i], LOG2E, off));
        s[n][i] = pv;
        ps += pv;
      }
#pragma unroll
      FTMI_ROW16(add2, ps);
      l[i] = l[i] * alpha[i] + ps;
      m[i] = mn;
    }
    if (__any(moved)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          ob[n][i] *= alpha[i];
          osm[n][i] *= alpha[i];
        }
    }
    // ---- P (C layout) -> this wave's LDS rows -> A layout (row c16, keys 32 kk + 8 g ..)
    float *P = Ps[wave];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) P[(4 * g + i) * PP + n * 16 + c16] = s[n][i];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      f16x8 ph, pt;
      const f32x4 a = *(const f32x4 *)&P[c16 * PP + 32 * kk + 8 * g];
      const f32x4 c = *(const f32x4 *)&P[c16 * PP + 32 * kk + 8 * g + 4];
      split8p(a, c, ph, pt);
      // ---- O += P V
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int o = (n * 16 + c16) * VP + 32 * kk + 8 * g;
        const f16x8 vh = *(const f16x8 *)&Vh[o];
        const f16x8 vt = *(const f16x8 *)&Vt[o];
        osm[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pt, vh, osm[n], 0, 0, 0);
        osm[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, vt, osm[n], 0, 0, 0);
        ob[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, vh, ob[n], 0, 0, 0);
      }
    }
  }
  if (!(amax <= 65504.f) && status) atomicOr(status, 1u);
  // normalise and store
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qr = q0 + 4 * g + i;
    if (qr >= T) continue;
    float *dst = out + ((int64_t)b * T + qr) * os + h * HD;
    const float inv = l[i];
#pragma unroll
    for (int n = 0; n < NT; ++n) dst[n * 16 + c16] = (ob[n][i] + osm[n][i] * TU) / inv;
  }
}

// ---- transposed form: S^T = K (q c)^T and O^T = V^T P^T ----------------------------------
// The same f16x3 flash attention with both MFMAs' operands swapped, so the C layout puts ONE
// query in each lane (column c16) and keys / head dims in its rows: a lane's 16 scores of a
// 64-key tile all belong to its query, so the softmax runs in-lane plus two cross-group
// shuffles (no 16-lane row reductions per row), the running max / sum are one value per
// lane, the O rescale multiplies whole accumulators by the lane's own alpha, and P needs no
// LDS round trip: the 8 scores a lane holds of a 32-key step (keys 4g .. 4g+3 of two 16-key
// blocks) ARE its B fragment for O^T = V^T P^T once V^T's keys are stored in the same order
// (position 8g + j of a 32-key group holds key 4g + j, j < 4, else 16 + 4g + j - 4).  K and V^T
// fragments are read at the same LDS addresses as attention_h3_kernel's; LDS drops the P
// buffers, which leaves room for two K / V tile buffers: one barrier per tile, and the tile
// stores overlap other waves' MFMAs instead of a phase where no wave multiplies.  PRE only (K / V from the split-plane workspace).  Numerically the same algorithm;
// the P V products sum in a permuted key order inside each MFMA.
template <int HD, bool PRE>
__global__ __launch_bounds__(64 * AH_W) void attention_t3_kernel(
    const float *__restrict__ qkv, int64_t rs, int B, int T, int H, int q_off, int k_off,
    int v_off, const uint8_t *__restrict__ kpm, float qscale, float *__restrict__ out,
    int64_t os, unsigned *status, const _Float16 *__restrict__ kv, int Tp) {
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  typedef float f32x8 __attribute__((ext_vector_type(8)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  constexpr int NTH = 64 * AH_W;
  constexpr float TS = 2048.f, TU = 1.f / 2048.f;
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr int KP = HD + 16, VP = AH_KT + 16;
  constexpr int NT = HD / 16, KQ = HD / 32, NB = AH_KT / 16, KK = AH_KT / 32;
  // two tile buffers (152 KB at HD = 128): tile t + 1 is stored while tile t is multiplied
  __shared__ __attribute__((aligned(16))) _Float16 Kh[2][AH_KT * KP], Kt[2][AH_KT * KP];
  __shared__ __attribute__((aligned(16))) _Float16 Vh[2][HD * VP], Vt[2][HD * VP];

  const int nq = (T + 16 * AH_W - 1) / (16 * AH_W), nbh = B * H;
  int bh, qtile;
  if (nbh % 8 == 0) {
    const int L = blockIdx.x, q8 = L >> 3;
    bh = (L & 7) + 8 * (q8 / nq);
    qtile = q8 % nq;
  } else {
    bh = blockIdx.x / nq;
    qtile = blockIdx.x % nq;
  }
  const int b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int q0 = qtile * 16 * AH_W + wave * 16;
  const float *base = qkv + (int64_t)b * T * rs;
  float amax = 0.f;

  // B fragments of this wave's 16 queries (lane: query c16, d = 32 ks + 8 g + j), q c in fp32
  f16x8 qh[KQ], qt[KQ];
  {
    const int qr = q0 + c16;
    const float *src = base + (int64_t)(qr < T ? qr : 0) * rs + q_off + h * HD;
#pragma unroll
    for (int ks = 0; ks < KQ; ++ks) {
      f32x4 a = *(const f32x4 *)(src + 32 * ks + 8 * g) * qscale;
      f32x4 c = *(const f32x4 *)(src + 32 * ks + 8 * g + 4) * qscale;
      if (qr >= T) a = c = (f32x4){0.f, 0.f, 0.f, 0.f};
      const f32x8 v = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
      qh[ks] = __builtin_convertvector(v, f16x8);
      qt[ks] = __builtin_convertvector((v - __builtin_convertvector(qh[ks], f32x8)) * TS, f16x8);
    }
  }
  f32x4 ob[NT], osm[NT];  // O^T: lane (query c16, d = 16 n + 4 g + i); big / small terms
#pragma unroll
  for (int n = 0; n < NT; ++n) ob[n] = osm[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  // PRE: K / V f16 planes from the workspace (16-B copies); else fp32 rows of qkv, split here
  // (attention_h3_kernel's loads: K a float4 of a key row, V 8 keys of one column)
  constexpr int NKC = PRE ? 2 * AH_KT * HD / 8 / NTH : AH_KT * HD / 4 / NTH;
  constexpr int NVC = PRE ? 2 * HD * AH_KT / 8 / NTH : HD * (AH_KT / 8) / NTH;
  static_assert(NKC * NTH == (PRE ? 2 * AH_KT * HD / 8 : AH_KT * HD / 4) &&
                NVC * NTH == (PRE ? 2 * HD * AH_KT / 8 : HD * (AH_KT / 8)), "slots");
  u32x4 kr[NKC], vr[PRE ? NVC : 1];
  float vs[PRE ? 1 : NVC][8];
  const size_t plane = PRE ? (size_t)B * H * Tp * HD : 0;
  const int last0 = (T - 1) / AH_KT * AH_KT;
  auto load_tile = [&](int k0) {
    k0 = k0 < last0 ? k0 : last0;  // past the end: a clamped (unused) reload
    if constexpr (!PRE) {
#pragma unroll
      for (int i = 0; i < NKC; ++i) {
        const int e = tid + NTH * i, r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4;
        const int key = min(k0 + r, T - 1);
        kr[i] = *(const u32x4 *)(base + (int64_t)key * rs + k_off + h * HD + c4);
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {
        const int e = tid + NTH * i, d = e % HD, kg = e / HD;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int key = min(k0 + kg * 8 + j, T - 1);
          vs[i][j] = base[(int64_t)key * rs + v_off + h * HD + d];
        }
      }
      return;
    }
    const _Float16 *kb = kv + ((size_t)bh * Tp + k0) * HD;
    const _Float16 *vb = kv + 2 * plane + (size_t)bh * HD * Tp + k0;
#pragma unroll
    for (int i = 0; i < NKC; ++i) {
      const int e = tid + NTH * i, pl = e / (AH_KT * HD / 8), q = e - pl * (AH_KT * HD / 8);
      const int r = q / (HD / 8), c8 = (q - r * (HD / 8)) * 8;
      kr[i] = *(const u32x4 *)(kb + pl * plane + (size_t)r * HD + c8);
    }
#pragma unroll
    for (int i = 0; i < NVC; ++i) {
      const int e = tid + NTH * i, pl = e / (HD * AH_KT / 8), q = e - pl * (HD * AH_KT / 8);
      const int d = q / (AH_KT / 8), c8 = (q - d * (AH_KT / 8)) * 8;
      vr[i] = *(const u32x4 *)(vb + pl * plane + (size_t)d * Tp + c8);
    }
  };
  // position of key w (0..31) of a 32-key group: the k order of the lanes' P fragments
  auto kpos = [](int w) { return w < 16 ? 2 * w : 2 * (w - 16) + 4; };
  auto store_tile = [&](int buf, int k0) {
    if constexpr (!PRE) {
#pragma unroll
      for (int i = 0; i < NKC; ++i) {
        const int e = tid + NTH * i, r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4;
        f32x4 kvv = __builtin_bit_cast(f32x4, kr[i]);
        if (k0 + r >= T) kvv = (f32x4){0.f, 0.f, 0.f, 0.f};
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        f16x4 hh, tt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          amax = fmaxf(amax, fabsf(kvv[j]));
          hh[j] = (_Float16)kvv[j];
          tt[j] = (_Float16)((kvv[j] - (float)hh[j]) * TS);
        }
        *(f16x4 *)&Kh[buf][r * KP + c4] = hh;
        *(f16x4 *)&Kt[buf][r * KP + c4] = tt;
      }
#pragma unroll
      for (int i = 0; i < NVC; ++i) {
        const int e = tid + NTH * i, d = e % HD, kg = e / HD;
        f32x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = k0 + kg * 8 + j < T ? vs[i][j] : 0.f;
          amax = fmaxf(amax, fabsf(v[j]));
        }
        const f16x8 hh = __builtin_convertvector(v, f16x8);
        const f16x8 tt = __builtin_convertvector((v - __builtin_convertvector(hh, f32x8)) * TS, f16x8);
        const u32x4 hb = __builtin_bit_cast(u32x4, hh), tb = __builtin_bit_cast(u32x4, tt);
        const int c8 = kg * 8, w = c8 & 31;
        _Float16 *rh = &Vh[buf][d * VP + (c8 & ~31)], *rt = &Vt[buf][d * VP + (c8 & ~31)];
        *(u32x2 *)(rh + kpos(w)) = (u32x2){hb.x, hb.y};
        *(u32x2 *)(rh + kpos(w + 4)) = (u32x2){hb.z, hb.w};
        *(u32x2 *)(rt + kpos(w)) = (u32x2){tb.x, tb.y};
        *(u32x2 *)(rt + kpos(w + 4)) = (u32x2){tb.z, tb.w};
      }
      return;
    }
    const bool tail = k0 + AH_KT > T;  // the last tile: pad keys are zeroed (uniform)
#pragma unroll
    for (int i = 0; i < NKC; ++i) {
      const int e = tid + NTH * i, pl = e / (AH_KT * HD / 8), q = e - pl * (AH_KT * HD / 8);
      const int r = q / (HD / 8), c8 = (q - r * (HD / 8)) * 8;
      u32x4 kk = kr[i];
      if (tail && k0 + r >= T) kk = (u32x4){0u, 0u, 0u, 0u};
      *(u32x4 *)&(pl ? Kt : Kh)[buf][r * KP + c8] = kk;
    }
#pragma unroll
    for (int i = 0; i < NVC; ++i) {
      const int e = tid + NTH * i, pl = e / (HD * AH_KT / 8), q = e - pl * (HD * AH_KT / 8);
      const int d = q / (AH_KT / 8), c8 = (q - d * (AH_KT / 8)) * 8;
      _Float16 *row = &(pl ? Vt : Vh)[buf][d * VP + (c8 & ~31)];
      const int w = c8 & 31;
      const u32x4 vv = tail ? zero_keys_past(vr[i], k0 + c8, T) : vr[i];
      *(u32x2 *)(row + kpos(w)) = (u32x2){vv.x, vv.y};
      *(u32x2 *)(row + kpos(w + 4)) = (u32x2){vv.z, vv.w};
    }
  };
  load_tile(0);
  store_tile(0, 0);
  load_tile(AH_KT);
  __syncthreads();

  for (int k0 = 0, cb = 0; k0 < T; k0 += AH_KT, cb ^= 1) {
    // dead keys of the tile (past T or flagged in key_padding_mask), one bit per key: lane l
    // reads key k0 + l's flag (issued here, under the S MFMAs)
    const bool masked = k0 + AH_KT > T || kpm;
    unsigned long long dm = 0;
    if (masked) {
      const int key = k0 + lane;
      dm = __ballot(key >= T || (kpm && kpm[(int64_t)b * T + key]));
    }
    // ---- S^T = K (q c)^T: lane (query c16, keys 16 n + 4 g + i)
    f32x4 s[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      f32x4 big = {0.f, 0.f, 0.f, 0.f}, sm = {0.f, 0.f, 0.f, 0.f};
      const int o = (n * 16 + c16) * KP + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KQ; ++ks) {
        const f16x8 kh = *(const f16x8 *)&Kh[cb][o + 32 * ks];
        const f16x8 kt = *(const f16x8 *)&Kt[cb][o + 32 * ks];
        sm = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qt[ks], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_16x16x32_f16(kt, qh[ks], sm, 0, 0, 0);
        big = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qh[ks], big, 0, 0, 0);
      }
      s[n] = big + sm * TU;
      if (masked) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((dm >> (n * 16 + 4 * g + i)) & 1ull) s[n][i] = -INFINITY;
      }
    }
    // ---- online softmax of the lane's query (lazy running max, as attention_h3_kernel)
    float mx = s[0][0];
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[n][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const bool up = mx > m + AH_LAZY;  // false while the query has only masked keys
    const float mn = up ? mx : m;
    const float alpha = up ? __builtin_amdgcn_exp2f((m - mn) * LOG2E) : 1.f;
    const float off = mn == -INFINITY ? 0.f : -mn * LOG2E;
    float ps = 0.f;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(s[n][i], LOG2E, off));
        s[n][i] = pv;
        ps += pv;
      }
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
    if (__any(up)) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        ob[n] *= alpha;
        osm[n] *= alpha;
      }
    }
    // ---- O^T += V^T P^T: the lane's 8 probabilities of key step kk are its B fragment
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const f32x4 a = s[2 * kk], c = s[2 * kk + 1];
      const f32x8 v = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      const f16x8 ph = __builtin_convertvector(v, f16x8);
      const f16x8 pt = __builtin_convertvector((v - __builtin_convertvector(ph, f32x8)) * TS, f16x8);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int o = (n * 16 + c16) * VP + 32 * kk + 8 * g;
        const f16x8 vh = *(const f16x8 *)&Vh[cb][o];
        const f16x8 vt = *(const f16x8 *)&Vt[cb][o];
        osm[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pt, osm[n], 0, 0, 0);
        osm[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vt, ph, osm[n], 0, 0, 0);
        ob[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph, ob[n], 0, 0, 0);
      }
    }
    // the next tile into the other buffer (every wave passed the barrier after its last read
    // of that buffer), then the loads of the one after
    if (k0 + AH_KT < T) {
      store_tile(cb ^ 1, k0 + AH_KT);
      load_tile(k0 + 2 * AH_KT);
    }
    __syncthreads();
  }
  if (!(amax <= 65504.f) && status) atomicOr(status, 1u);
  const int qr = q0 + c16;
  if (qr < T) {  // the lane's query row: 4 consecutive head dims per block, 16-B stores
    float *dst = out + ((int64_t)b * T + qr) * os + h * HD + 4 * g;
#pragma unroll
    for (int n = 0; n < NT; ++n) *(f32x4 *)(dst + 16 * n) = (ob[n] + osm[n] * TU) / l;
  }
}

// K and V of every (batch, head) split once into f16 head / scaled tail planes for the
// PRE attention kernel: K [B*H][Tp][HD], V transposed [B*H][HD][Tp] (keys >= T zero).  One
// workgroup per (64 keys, b*h): K rows straight through, V through an LDS tile.  A value
// beyond the f16 range sets bit 0 of *status.
template <int HD>
__global__ __launch_bounds__(256) void attn_split_kv_kernel(const float *__restrict__ qkv,
                                                            int64_t rs, int B, int T, int H,
                                                            int k_off, int v_off, int Tp,
                                                            _Float16 *__restrict__ kv,
                                                            unsigned *status) {
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  constexpr float TS = 2048.f;
  __shared__ float vt[64][HD + 1];
  const int k0 = blockIdx.x * 64, bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const size_t plane = (size_t)B * H * Tp * HD;
  const float *base = qkv + (size_t)b * T * rs;
  float amax = 0.f;
  for (int e = threadIdx.x; e < 64 * HD / 4; e += 256) {
    const int r = e / (HD / 4), c4 = (e - r * (HD / 4)) * 4, key = k0 + r;
    f32x4 kvv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
    if (key < T) {
      kvv = *(const f32x4 *)(base + (size_t)key * rs + k_off + h * HD + c4);
      vv = *(const f32x4 *)(base + (size_t)key * rs + v_off + h * HD + c4);
    }
    f16x4 hh, tt;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      amax = fmaxf(amax, fmaxf(fabsf(kvv[j]), fabsf(vv[j])));
      hh[j] = (_Float16)kvv[j];
      tt[j] = (_Float16)((kvv[j] - (float)hh[j]) * TS);
      vt[r][c4 + j] = vv[j];
    }
    const size_t o = ((size_t)bh * Tp + key) * HD + c4;
    *(f16x4 *)(kv + o) = hh;
    *(f16x4 *)(kv + plane + o) = tt;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HD * 16; e += 256) {  // V^T: row d, 4 keys per thread
    const int d = e / 16, kq = (e - d * 16) * 4;
    f16x4 hh, tt;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = vt[kq + j][d];
      hh[j] = (_Float16)v;
      tt[j] = (_Float16)((v - (float)hh[j]) * TS);
    }
    const size_t o = ((size_t)bh * HD + d) * Tp + k0 + kq;
    *(f16x4 *)(kv + 2 * plane + o) = hh;
    *(f16x4 *)(kv + 3 * plane + o) = tt;
  }
  if (!(amax <= 65504.f) && status) atomicOr(status, 1u);
}

}  // namespace

extern "C" int ftmi_embedding_posenc(const int64_t *ids, int32_t B, int32_t T, const float *table,
                                     int64_t rows, int32_t dim, const float *pe,
                                     const float *scale, float *out, int32_t *err,
                                     ftmi_stream_t stream) {
  if (!ids || !table || !pe || !scale || !out || B <= 0 || T <= 0 || dim <= 0) return FTMI_E_ARG;
  const int64_t n = (int64_t)B * T;
  const int64_t total = n * dim;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(embed_posenc_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     ftmi_hs(stream), ids, T, n, table, rows, dim, pe, scale, out, err);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_lr_posenc(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t C,
                              const int32_t *index, int32_t T_mel, const float *pe,
                              const float *scale, float *y, int64_t y_stride, ftmi_stream_t stream) {
  if (!x || !index || !pe || !scale || !y || B <= 0 || T <= 0 || C <= 0 || T_mel < 0) return FTMI_E_ARG;
  const int64_t n = (int64_t)B * T_mel;
  if (n == 0) return FTMI_OK;
  const int64_t blocks = (n * C + 255) / 256;
  hipLaunchKernelGGL(lr_posenc_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     ftmi_hs(stream), x, x_stride, T, C, index, T_mel, n, pe, scale, y, y_stride);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_layernorm(const float *x, int64_t x_stride, int64_t M, int32_t C,
                              const float *gamma, const float *beta, float eps, float *y,
                              int64_t y_stride, ftmi_stream_t stream) {
  if (!x || !gamma || !beta || !y || M <= 0 || C <= 0) return FTMI_E_ARG;
  if (C > 64 * 16) return FTMI_E_SHAPE;
  const dim3 grid((unsigned)((M + 3) / 4)), block(256);
  const hipStream_t s = ftmi_hs(stream);
  const int vpl = (C + 63) / 64;
  if (vpl <= 2)
    hipLaunchKernelGGL(layernorm_kernel<2>, grid, block, 0, s, x, x_stride, M, C, gamma, beta, eps, y, y_stride);
  else if (vpl <= 4)
    hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, s, x, x_stride, M, C, gamma, beta, eps, y, y_stride);
  else if (vpl <= 8)
    hipLaunchKernelGGL(layernorm_kernel<8>, grid, block, 0, s, x, x_stride, M, C, gamma, beta, eps, y, y_stride);
  else
    hipLaunchKernelGGL(layernorm_kernel<16>, grid, block, 0, s, x, x_stride, M, C, gamma, beta, eps, y, y_stride);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int64_t ftmi_attention_workspace_bytes(int32_t B, int32_t T, int32_t H,
                                                  int32_t head_dim) {
  if (B <= 0 || T <= 0 || H <= 0 || head_dim <= 0) return 0;
  const int64_t Tp = (T + 63) / 64 * 64;
  return 4 * (int64_t)B * H * Tp * head_dim * 2;
}

// the transposed kernel for the pre-split (K / V workspace) paths with 16-B aligned output
// rows; FTMI_ATTN_T=0 (read per call) keeps attention_h3_kernel
static bool attn_transposed() {
  const char *e = getenv("FTMI_ATTN_T");
  return !e || atoi(e) != 0;
}

extern "C" int ftmi_attention_kv(const float *q, int64_t row_stride, int32_t B, int32_t T,
                                 int32_t H, int32_t head_dim, const uint8_t *key_padding_mask,
                                 float qscale, float *out, int64_t out_stride, uint32_t *status,
                                 const void *kv_workspace, int64_t workspace_bytes,
                                 ftmi_stream_t stream) {
  if (!q || !out || !kv_workspace || B <= 0 || T <= 0 || H <= 0) return FTMI_E_ARG;
  if (head_dim != 64 && head_dim != 128) return FTMI_E_UNSUPPORTED;
  if (workspace_bytes < ftmi_attention_workspace_bytes(B, T, H, head_dim)) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(q) || (row_stride & 3) || !ftmi_aligned16(kv_workspace)) return FTMI_E_ALIGN;
  const int nq = (T + 16 * AH_W - 1) / (16 * AH_W), Tp = (T + 63) / 64 * 64;
  const dim3 g1((unsigned)(nq * B * H)), b1(64 * AH_W);
  const _Float16 *kv = (const _Float16 *)kv_workspace;
  const hipStream_t s = ftmi_hs(stream);
  if (attn_transposed() && (out_stride & 3) == 0 && ftmi_aligned16(out)) {
    if (head_dim == 64)
      hipLaunchKernelGGL((attention_t3_kernel<64, true>), g1, b1, 0, s, q, row_stride, B, T, H,
                         0, 0, 0, key_padding_mask, qscale, out, out_stride, status, kv, Tp);
    else
      hipLaunchKernelGGL((attention_t3_kernel<128, true>), g1, b1, 0, s, q, row_stride, B, T, H,
                         0, 0, 0, key_padding_mask, qscale, out, out_stride, status, kv, Tp);
  } else if (head_dim == 64)
    hipLaunchKernelGGL((attention_h3_kernel<64, true>), g1, b1, 0, s, q, row_stride, B, T, H, 0,
                       0, 0, key_padding_mask, qscale, out, out_stride, status, kv, Tp);
  else
    hipLaunchKernelGGL((attention_h3_kernel<128, true>), g1, b1, 0, s, q, row_stride, B, T, H, 0,
                       0, 0, key_padding_mask, qscale, out, out_stride, status, kv, Tp);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_attention(const float *qkv, int64_t row_stride, int32_t B, int32_t T,
                              int32_t H, int32_t head_dim, int32_t q_off, int32_t k_off,
                              int32_t v_off, const uint8_t *key_padding_mask, float qscale,
                              float *out, int64_t out_stride, int32_t mma, uint32_t *status,
                              void *workspace, int64_t workspace_bytes, ftmi_stream_t stream) {
  if (!qkv || !out || B <= 0 || T <= 0 || H <= 0) return FTMI_E_ARG;
  if (head_dim != 64 && head_dim != 128) return FTMI_E_UNSUPPORTED;
  if (mma != FTMI_MMA_F32 && mma != FTMI_MMA_F16X3) return FTMI_E_UNSUPPORTED;
  if (!ftmi_aligned16(qkv) || (row_stride & 3) || (q_off & 3) || (k_off & 3) || (v_off & 3))
    return FTMI_E_ALIGN;
  if (workspace && !ftmi_aligned16(workspace)) return FTMI_E_ALIGN;
  const dim3 grid((unsigned)((T + 63) / 64), (unsigned)(B * H)), block(256);
  const hipStream_t s = ftmi_hs(stream);
  if (mma == FTMI_MMA_F16X3) {
    const int nq = (T + 16 * AH_W - 1) / (16 * AH_W);
    const dim3 g1((unsigned)(nq * B * H)), b1(64 * AH_W);
    const int Tp = (T + 63) / 64 * 64;
    const bool pre = workspace && workspace_bytes >= ftmi_attention_workspace_bytes(B, T, H, head_dim);
    _Float16 *kv = (_Float16 *)workspace;
#define FTMI_ATTN_H3(HD_)                                                                       \
  if (pre) {                                                                                     \
    hipLaunchKernelGGL(attn_split_kv_kernel<HD_>, dim3((unsigned)(Tp / 64), (unsigned)(B * H)),  \
                       dim3(256), 0, s, qkv, row_stride, B, T, H, k_off, v_off, Tp, kv, status); \
    if (attn_transposed() && (out_stride & 3) == 0 && ftmi_aligned16(out))                      \
      hipLaunchKernelGGL((attention_t3_kernel<HD_, true>), g1, b1, 0, s, qkv, row_stride, B, T,  \
                         H, q_off, 0, 0, key_padding_mask, qscale, out, out_stride, status,       \
                         (const _Float16 *)kv, Tp);                                               \
    else                                                                                          \
      hipLaunchKernelGGL((attention_h3_kernel<HD_, true>), g1, b1, 0, s, qkv, row_stride, B, T,  \
                         H, q_off, k_off, v_off, key_padding_mask, qscale, out, out_stride,       \
                         status, (const _Float16 *)kv, Tp);                                       \
  } else if (attn_transposed() && (out_stride & 3) == 0 && ftmi_aligned16(out)) {                 \
    hipLaunchKernelGGL((attention_t3_kernel<HD_, false>), g1, b1, 0, s, qkv, row_stride, B, T,  \
                       H, q_off, k_off, v_off, key_padding_mask, qscale, out, out_stride, status,\
                       (const _Float16 *)nullptr, 0);                                            \
  } else {                                                                                       \
    hipLaunchKernelGGL((attention_h3_kernel<HD_, false>), g1, b1, 0, s, qkv, row_stride, B, T,  \
                       H, q_off, k_off, v_off, key_padding_mask, qscale, out, out_stride,       \
                       status, (const _Float16 *)nullptr, 0);                                   \
  }
    if (head_dim == 64) {
      FTMI_ATTN_H3(64)
    } else {
      FTMI_ATTN_H3(128)
    }
#undef FTMI_ATTN_H3
    FTMI_CHECK_LAUNCH();
    return FTMI_OK;
  }
  if (head_dim == 64)
    hipLaunchKernelGGL(attention_kernel<64>, grid, block, 0, s, qkv, row_stride, B, T, H, q_off, k_off,
                       v_off, key_padding_mask, qscale, out, out_stride);
  else
    hipLaunchKernelGGL(attention_kernel<128>, grid, block, 0, s, qkv, row_stride, B, T, H, q_off, k_off,
                       v_off, key_padding_mask, qscale, out, out_stride);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}
