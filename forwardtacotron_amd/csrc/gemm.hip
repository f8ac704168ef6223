// Implicit-GEMM Conv1d / Linear / CBHG-bank / Highway kernels on fp32 MFMA (gfx950).
//
// One kernel template covers every dense contraction of the ForwardTacotron forward pass:
//   BatchNormConv (k = 1..16, pad k//2, ReLU -> BN)   models/common_layers.py:38-52,
//                                                     models/forward_tacotron.py:58-71
//   CBHG bank (K convs in one launch, concatenated)   models/common_layers.py:67-71,92-97
//   CBHG maxpool fused into proj1's operand load      models/common_layers.py:73,100
//   proj2 + residual                                  models/common_layers.py:106-109
//   Linear layers (k = 1)                             pre_highway, lin, post_proj, RNN W_ih
//   Highway layer (W1 | W2 in one GEMM, gating epilogue) models/common_layers.py:22-35
//
// Numerics: exact fp32 (v_mfma_f32_32x32x2_f32 is a k-ordered fmaf chain), no reduced
// precision anywhere.  Tiling: 128x128 block tile, BK = 16, 4 waves each owning a 64x64
// sub-tile = 2x2 MFMA 32x32 tiles; operands staged through LDS (double buffered, one
// barrier per K-step, global loads for step k+1 issued before the MFMAs of step k).
// Inside a BK = 16 chunk lane half h consumes k = 8h + s at MFMA s (s = 0..7) for both
// operands, so every lane reads its fragments with two ds_read_b128 per operand; the
// LDS row stride of 20 floats makes those reads bank-conflict free (5i mod 16 distinct).
//
// Second path, "x6" (mma = 1): the same contraction on the bf16 matrix pipe (16x the fp32
// MFMA rate).  Both fp32 operands are split while staged into LDS, a = a1 + a2 + a3 with
// a1 = bf16(a), a2 = bf16(a - a1), a3 = bf16(a - a1 - a2) (each difference is exact in
// fp32), and every 16x16x32 tile accumulates the six cross products with i + j <= 4
// (a1b1, a1b2, a2b1, a1b3, a2b2, a3b1) in fp32 — the dropped terms are < 2^-24 relative,
// so the result is fp32-accurate (emulated: max err 5-7e-7 vs 2e-6 for a plain fp32 GEMM
// at K = 256..6144) at 16/6 = 2.7x the fp32 MFMA rate.
//
// Third path, "h3" (mma = 2, the default): the same contraction in THREE f16 MFMAs per
// fp32 product (16/3 = 5.3x the fp32 MFMA rate).  Both operands are split into an f16 head
// and a SCALED f16 tail (Ootomo & Yokota, arXiv:2203.03341):
//   a = a_h + 2^-11 a_t,   a_h = f16(a), a_t = f16((a - a_h) * 2^11)
// The weights (pre-split once by ftmi_split_weights_f16, per output column n pre-scaled by
// a power of two s_n so that |w| s_n < 16) are stored as three f16 planes
//   B0 = 2^11 w_h,  B1 = w_t,  B2 = w_h            (w = w_h + 2^-11 w_t after scaling)
// and one fp32 accumulator collects   a_h B0 + a_h B1 + a_t B2 = 2^11 (a w - 2^-22 a_t w_t),
// multiplied back by colscale[n] = 2^-11 / s_n (exact) in the epilogue.  The scaled tails
// keep 11 significant bits down to |a| ~ 2^-24 (no subnormal tail loss); the dropped term is
// < 2^-22 relative.  The only range limit is |a| < 65504 for the activations: an overflow
// makes the accumulator non-finite, which the epilogue reports through *status (bit 0);
// the model layer then recomputes the call on the fp32 path.
#include "common.h"

namespace {

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 16;
constexpr int LDS_STRIDE = 20;  // floats per staged row (16 + 4 pad)
constexpr int MAX_GROUPS = 16;

enum { EPI_CONV = 0, EPI_HIGHWAY = 1 };

struct GemmGroup {
  const float *w;  // [N][Ktot]
  const __bf16 *w3;  // optional pre-split weights [3][N][Kpad], Kpad = roundup(Ktot, 32)
                     // (bf16 pieces for mma = 1, f16 planes B0/B1/B2 for mma = 2)
  const float *colscale;  // mma = 2: per-column 2^-11 / s_n after the f16 planes
  int Kpad;
  const float *bias;
  const float *scale;
  const float *shift;
  int N, k, pad, Ktot;
  int ycol0;   // first output column of this group
  int ntiles;  // number of BN tiles
  int tile0;   // first linear block index of this group
};

struct GemmParams {
  const float *x;
  int64_t x_stride;
  int B, T, Cin, M;
  int To;  // output frames per sequence (rows of y are (b, t < To))
  int relu, ngroups;
  const float *residual;
  int64_t res_stride;
  float *y;
  int64_t y_stride;
  float *yt;
  int yt_channels;
  // highway epilogue
  const float *b1;
  const float *b2;
  // split-K: blocks with blockIdx.y = s accumulate K chunks [s*kc_per, (s+1)*kc_per) and
  // store raw partial sums to part[s][M][N]; splitk_epilogue_kernel finishes the tile
  int split;
  int kc_per;
  int split_req;  // the caller's split_k (the slab kernel re-derives split / kc_per from it)
  int diag;       // slab kernel timing experiments (FTMI_SLAB_DIAG, diagnostic build only)
  int band;       // slab kernels: column-band tile order (FTMI_SLAB_BAND, see slab_tile)
  float *part;
  int ldp;  // skinny kernel: columns of a partial-sum row (all groups, output order)
  int force_part;  // skinny kernel: partial sums even with one split (highway finish)
  unsigned *status;  // mma = 2: bit 0 set when an accumulator became non-finite
  // slab kernel, EPI_CONV: store maxpool(2, 1) of the finished rows (CBHG bank -> its pooled
  // input of proj1, common_layers.py:100): y[t] = max(v[t - 1], v[t]), y[0] = v[0] per
  // sequence.  Tiles then step by SL_BM - 1 rows and carry one halo row.
  int pool_out;
  // slab kernel, f16x3 activation rows ("split rows": per row C f16 heads, then C f16
  // tails, x_stride / y_stride still counted in floats): x_split = the operand x is given
  // split (staged as is, no split while staging; its producer checked the f16 range);
  // y_split_c > 0 = the pool_out epilogue writes y as split rows of y_split_c channels
  int x_split;
  int y_split_c;
  // conv_bank_halves_kernel: per-slice arrival counters (zero between launches)
  unsigned *tile_cnt;
  // conv_bank_halves_kernel (FTMI_BANK_IMAGE): the stream-order weight image — every wave's
  // weight fragments in the order it loads them, 1 KB per wave load (bank_halves_pack_kernel)
  const _Float16 *wimg;
  GemmGroup g[MAX_GROUPS];
};

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// matrix-fragment type and MFMA of the pre-split kernels: bf16 pieces (x6) or f16 (h3)
template <bool H3>
struct Frag {
  typedef bf16x8 T;
};
template <>
struct Frag<true> {
  typedef f16x8 T;
};
__device__ __forceinline__ f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

constexpr float H3_SCALE = 2048.f;  // 2^11: the tail scale of the f16 split

// a = a_h + 2^-11 a_t  (f16 head, scaled f16 tail)
__device__ __forceinline__ void split2h(f32x4 v, f16x4 &h, f16x4 &t) {
  h = __builtin_convertvector(v, f16x4);
  t = __builtin_convertvector((v - __builtin_convertvector(h, f32x4)) * H3_SCALE, f16x4);
}

// highway output g relu(x1) + (1 - g) x with one fixed rounding sequence in every kernel
// (no compiler-chosen contraction: the fused stack is bit-identical to the per-layer path)
__device__ __forceinline__ float highway_mix(float g, float x1, float x) {
#pragma clang fp contract(off)
  return fmaf(g, fmaxf(x1, 0.f), (1.f - g) * x);
}

constexpr int X6_BK = 32;
constexpr int X6_STRIDE = 48;  // bf16 per staged row (32 + 16 pad): 96-B rows make the
                               // ds_read_b128 fragment reads of 16x16x32 conflict free
constexpr int X6_PIECE = BM * X6_STRIDE;  // bf16 per (operand, piece) image

__device__ __forceinline__ f32x4 fmax4(f32x4 a, f32x4 b) {
  f32x4 r;
  r.x = fmaxf(a.x, b.x);
  r.y = fmaxf(a.y, b.y);
  r.z = fmaxf(a.z, b.z);
  r.w = fmaxf(a.w, b.w);
  return r;
}

template <int EPI, bool MAXPOOL>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][BM * LDS_STRIDE];

  // ---- locate (group, m-tile, n-tile); groups are ordered heaviest first -------------
  const int tile = blockIdx.x;
  int gi = 0;
  while (gi + 1 < p.ngroups && tile >= p.g[gi + 1].tile0) ++gi;
  const GemmGroup &G = p.g[gi];
  const int lt = tile - G.tile0;
  const int mt = lt / G.ntiles;
  const int nt = lt - mt * G.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- loader assignment: rows lr and lr+64 of both A and B tiles, float4 #lq ------
  const int lr = tid >> 2, lq = tid & 3;
  int ab[2], at[2];
  bool aok[2], bok[2];
  const float *wrow[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int m = m0 + lr + 64 * q;
    aok[q] = m < p.M;
    const int mm = aok[q] ? m : 0;
    ab[q] = mm / p.To;
    at[q] = mm - ab[q] * p.To;
    const int n = n0 + lr + 64 * q;
    bok[q] = n < G.N;
    wrow[q] = G.w + (int64_t)(bok[q] ? n : 0) * G.Ktot + 4 * lq;
  }

  const int nk = G.Ktot / BK;
  f32x4 ra[2], rb[2];

  auto gload = [&](int kc) {
    const int kk = kc * BK;
    const int j = kk / p.Cin;
    const int c0 = kk - j * p.Cin;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ts = at[q] + j - G.pad;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (aok[q] && ts >= 0 && ts < p.T) {
        const float *src = p.x + ((int64_t)ab[q] * p.T + ts) * p.x_stride + c0 + 4 * lq;
        v = *(const f32x4 *)src;
        if (MAXPOOL && ts > 0) v = fmax4(v, *(const f32x4 *)(src - p.x_stride));
      }
      ra[q] = v;
      f32x4 w = {0.f, 0.f, 0.f, 0.f};
      if (bok[q]) w = *(const f32x4 *)(wrow[q] + kk);
      rb[q] = w;
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *(f32x4 *)&lds[buf][0][(lr + 64 * q) * LDS_STRIDE + 4 * lq] = ra[q];
      *(f32x4 *)&lds[buf][1][(lr + 64 * q) * LDS_STRIDE + 4 * lq] = rb[q];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int fi = lane & 31, fh = lane >> 5;
  auto compute = [&](int buf) {
    const float *As = lds[buf][0];
    const float *Bs = lds[buf][1];
    f32x4 a[2][2], b[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int v = 0; v < 2; ++v)
        a[mi][v] = *(const f32x4 *)&As[(wm * 64 + mi * 32 + fi) * LDS_STRIDE + 8 * fh + 4 * v];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int v = 0; v < 2; ++v)
        b[ni][v] = *(const f32x4 *)&Bs[(wn * 64 + ni * 32 + fi) * LDS_STRIDE + 8 * fh + 4 * v];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi][s >> 2][s & 3],
                                                             b[ni][s >> 2][s & 3],
                                                             acc[mi][ni], 0, 0, 0);
  };

  // ---- main loop: one barrier per K-step ---------------------------------------------
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) gload(kc + 1);
    compute(cur);
    if (kc + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ---------------------------------------------------------------------
  if constexpr (EPI == EPI_CONV) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = n0 + wn * 64 + ni * 32 + fi;
        if (col >= G.N) continue;
        const float bias = G.bias ? G.bias[col] : 0.f;
        const float sc = G.scale ? G.scale[col] : 1.f;
        const float sh = G.scale ? G.shift[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (row >= p.M) continue;
          float v = acc[mi][ni][r];
          if (G.bias) v += bias;
          if (p.relu) v = fmaxf(v, 0.f);
          if (G.scale) v = v * sc + sh;
          if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
          if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
          if (p.yt) {
            const int b = row / p.To, t = row - b * p.To;
            p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
          }
        }
      }
  } else {
    // Highway: packed column block pair (2q, 2q+1) = (W1, W2) rows 32q..32q+31.
    if (n0 + wn * 64 >= G.N) return;
    const int col = (n0 + wn * 64) / 2 + fi;
    const float b1 = p.b1[col], b2 = p.b2[col];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (row >= p.M) continue;
        const float x1 = acc[mi][0][r] + b1;
        const float x2 = acc[mi][1][r] + b2;
        const float g = ftmi_sigmoid(x2);
        const float xin = p.x[(int64_t)row * p.x_stride + col];
        p.y[(int64_t)row * p.y_stride + col] = highway_mix(g, x1, xin);
      }
  }
}


// ---------------------------------------------------------------------------------------
// bf16x6 path.  128x128 block tile, BK = 32, 4 waves (2x2) each owning 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16.  One LDS image [operand 2][piece 3][row 128][48] bf16 = 72 KB,
// two workgroups per CU: while one splits / stages a chunk the other's MFMAs run.  Chunk
// k+1's global loads are issued before chunk k's MFMAs (loads go to registers; their
// split into pieces happens after the MFMAs, then one barrier pair per chunk).
// Global loads are branch-free: out-of-range rows / taps / K read a clamped in-bounds
// address and are zeroed by a select.
__device__ __forceinline__ void split3(f32x4 v, bf16x4 &h1, bf16x4 &h2, bf16x4 &h3) {
  h1 = __builtin_convertvector(v, bf16x4);
  const f32x4 r1 = v - __builtin_convertvector(h1, f32x4);
  h2 = __builtin_convertvector(r1, bf16x4);
  const f32x4 r2 = r1 - __builtin_convertvector(h2, f32x4);
  h3 = __builtin_convertvector(r2, bf16x4);
}

__device__ __forceinline__ f32x4 sel4(bool ok, f32x4 v) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  return ok ? v : z;
}

template <int EPI, bool MAXPOOL>
__global__ __launch_bounds__(256, 2) void conv_gemm_x6_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 3 * X6_PIECE];

  const int tile = blockIdx.x;
  int gi = 0;
  while (gi + 1 < p.ngroups && tile >= p.g[gi + 1].tile0) ++gi;
  const GemmGroup &G = p.g[gi];
  const int lt = tile - G.tile0;
  const int mt = lt / G.ntiles;
  const int nt = lt - mt * G.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // loader: rows lr + 32q (q = 0..3) of both operands, float4 #lc of the 32-wide chunk
  const int lr = tid >> 3, lc = tid & 7;
  const float *arow[4];  // sequence start of the A row (b, t = 0)
  int at[4];
  bool aok[4], bok[4];
  const float *wrow[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + lr + 32 * q;
    aok[q] = m < p.M;
    const int mm = aok[q] ? m : 0;
    const int b = mm / p.To;
    at[q] = mm - b * p.To;
    arow[q] = p.x + (int64_t)b * p.T * p.x_stride;
    const int n = n0 + lr + 32 * q;
    bok[q] = n < G.N;
    wrow[q] = G.w + (int64_t)(bok[q] ? n : 0) * G.Ktot;
  }
  int nk = (G.Ktot + X6_BK - 1) / X6_BK;
  int kc0 = 0;
  if (p.split > 1) {
    kc0 = blockIdx.y * p.kc_per;
    nk = min(nk - kc0, p.kc_per);
  }
  // this thread's K index k = kc*32 + 4*lc  ->  (tap j, channel c), advanced per chunk
  int kk = kc0 * X6_BK + 4 * lc, tj = kk / p.Cin, tc = kk - tj * p.Cin;

  auto gload = [&](f32x4 (&ra)[4], f32x4 (&rb)[4]) {
    const bool kok = kk < G.Ktot;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ts = at[q] + tj - G.pad;
      const bool ok = kok && aok[q] && ts >= 0 && ts < p.T;
      const float *src = arow[q] + (int64_t)(ok ? ts : 0) * p.x_stride + (ok ? tc : 0);
      f32x4 v = *(const f32x4 *)src;
      if (MAXPOOL) {
        const bool okp = ok && ts > 0;
        const f32x4 u = *(const f32x4 *)(src - (okp ? p.x_stride : 0));
        v = fmax4(v, u);
      }
      ra[q] = sel4(ok, v);
      rb[q] = sel4(kok && bok[q], *(const f32x4 *)(wrow[q] + (kok ? kk : 0)));
    }
    kk += X6_BK;
    tc += X6_BK;
    while (tc >= p.Cin) {
      tc -= p.Cin;
      ++tj;
    }
  };
  auto swrite = [&](const f32x4 (&ra)[4], const f32x4 (&rb)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int off = (lr + 32 * q) * X6_STRIDE + 4 * lc;
      bf16x4 h1, h2, h3;
      split3(ra[q], h1, h2, h3);
      *(bf16x4 *)(lds + 0 * X6_PIECE + off) = h1;
      *(bf16x4 *)(lds + 1 * X6_PIECE + off) = h2;
      *(bf16x4 *)(lds + 2 * X6_PIECE + off) = h3;
      split3(rb[q], h1, h2, h3);
      *(bf16x4 *)(lds + 3 * X6_PIECE + off) = h1;
      *(bf16x4 *)(lds + 4 * X6_PIECE + off) = h2;
      *(bf16x4 *)(lds + 5 * X6_PIECE + off) = h3;
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = 8 * (lane >> 4);
  auto compute = [&]() {
    bf16x8 a[4][3], b[4][3];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        a[mi][pc] = *(const bf16x8 *)(lds + pc * X6_PIECE + (wm * 64 + mi * 16 + fr) * X6_STRIDE + fk);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        b[ni][pc] = *(const bf16x8 *)(lds + (3 + pc) * X6_PIECE + (wn * 64 + ni * 16 + fr) * X6_STRIDE + fk);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        f32x4 c = acc[mi][ni];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][2], b[ni][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][1], b[ni][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][0], b[ni][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][1], b[ni][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][0], b[ni][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi][0], b[ni][0], c, 0, 0, 0);
        acc[mi][ni] = c;
      }
  };

  // two register sets: chunk k+2's loads are in flight while chunk k is computed
  f32x4 ra0[4], rb0[4], ra1[4], rb1[4];
  gload(ra0, rb0);
  if (nk > 1) gload(ra1, rb1);
  for (int kc = 0; kc < nk; kc += 2) {
    swrite(ra0, rb0);
    __syncthreads();
    if (kc + 2 < nk) gload(ra0, rb0);
    compute();
    __syncthreads();
    if (kc + 1 >= nk) break;
    swrite(ra1, rb1);
    __syncthreads();
    if (kc + 3 < nk) gload(ra1, rb1);
    compute();
    __syncthreads();
  }

  if (p.split > 1) {  // raw partial sums; the epilogue runs in splitk_epilogue_kernel
    float *part = p.part + (size_t)blockIdx.y * p.M * G.N;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wn * 64 + ni * 16 + (lane & 15);
      if (col >= G.N) continue;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4) + i;
          if (row < p.M) part[(size_t)row * G.N + col] = acc[mi][ni][i];
        }
    }
    return;
  }

  // epilogue: tile (mi, ni) element (row 4*(lane>>4) + i, col lane & 15)
  const int er = 4 * (lane >> 4);
  if constexpr (EPI == EPI_CONV) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wn * 64 + ni * 16 + fr;
      if (col >= G.N) continue;
      const float bias = G.bias ? G.bias[col] : 0.f;
      const float sc = G.scale ? G.scale[col] : 1.f;
      const float sh = G.scale ? G.shift[col] : 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + er + i;
          if (row >= p.M) continue;
          float v = acc[mi][ni][i];
          if (G.bias) v += bias;
          if (p.relu) v = fmaxf(v, 0.f);
          if (G.scale) v = v * sc + sh;
          if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
          if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
          if (p.yt) {
            const int b = row / p.To, t = row - b * p.To;
            p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
          }
        }
    }
  } else {
    // packed column blocks of 32: tiles ni = 0,1 are W1 columns, ni = 2,3 the matching W2
    if (n0 + wn * 64 >= G.N) return;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int col = (n0 + wn * 64) / 2 + ni * 16 + fr;
      const float b1 = p.b1[col], b2 = p.b2[col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + er + i;
          if (row >= p.M) continue;
          const float x1 = acc[mi][ni][i] + b1;
          const float x2 = acc[mi][ni + 2][i] + b2;
          const float g = ftmi_sigmoid(x2);
          const float xin = p.x[(int64_t)row * p.x_stride + col];
          p.y[(int64_t)row * p.y_stride + col] = highway_mix(g, x1, xin);
        }
    }
  }
}

// ---------------------------------------------------------------------------------------
// bf16x6, software-pipelined variant ("x6p"): ONE workgroup per CU (4 waves, one per SIMD),
// LDS double-buffered (2 x 72 KB).  In iteration k each wave reads chunk k's fragments from
// buffer k&1, and between its MFMAs splits chunk k+1 (already in registers) into buffer
// (k+1)&1; chunk k+2's global loads are issued at the top of the iteration into the register
// set chunk k+1 just vacated (two register sets, loop unrolled by two so every index is
// static).  One barrier per chunk.
template <int EPI, bool MAXPOOL>
__global__ __launch_bounds__(256, 1) void conv_gemm_x6p_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 2 * 3 * X6_PIECE];

  const int tile = blockIdx.x;
  int gi = 0;
  while (gi + 1 < p.ngroups && tile >= p.g[gi + 1].tile0) ++gi;
  const GemmGroup &G = p.g[gi];
  const int lt = tile - G.tile0;
  const int mt = lt / G.ntiles;
  const int nt = lt - mt * G.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int lr = tid >> 3, lc = tid & 7;
  const float *arow[4];
  int at[4];
  bool aok[4], bok[4];
  const float *wrow[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + lr + 32 * q;
    aok[q] = m < p.M;
    const int mm = aok[q] ? m : 0;
    const int b = mm / p.To;
    at[q] = mm - b * p.To;
    arow[q] = p.x + (int64_t)b * p.T * p.x_stride;
    const int n = n0 + lr + 32 * q;
    bok[q] = n < G.N;
    wrow[q] = G.w + (int64_t)(bok[q] ? n : 0) * G.Ktot;
  }
  int nk = (G.Ktot + X6_BK - 1) / X6_BK;
  int kc0 = 0;
  if (p.split > 1) {
    kc0 = blockIdx.y * p.kc_per;
    nk = min(nk - kc0, p.kc_per);
  }
  int kk = kc0 * X6_BK + 4 * lc, tj = kk / p.Cin, tc = kk - tj * p.Cin;

  auto gload = [&](f32x4 (&ra)[4], f32x4 (&rb)[4]) {
    const bool kok = kk < G.Ktot;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ts = at[q] + tj - G.pad;
      const bool ok = kok && aok[q] && ts >= 0 && ts < p.T;
      const float *src = arow[q] + (int64_t)(ok ? ts : 0) * p.x_stride + (ok ? tc : 0);
      f32x4 v = *(const f32x4 *)src;
      if (MAXPOOL) {
        const bool okp = ok && ts > 0;
        v = fmax4(v, *(const f32x4 *)(src - (okp ? p.x_stride : 0)));
      }
      ra[q] = sel4(ok, v);
      rb[q] = sel4(kok && bok[q], *(const f32x4 *)(wrow[q] + (kok ? kk : 0)));
    }
    kk += X6_BK;
    tc += X6_BK;
    while (tc >= p.Cin) {
      tc -= p.Cin;
      ++tj;
    }
  };
  auto split_store = [&](__bf16 *base, int q, f32x4 va, f32x4 vb) {
    const int off = (lr + 32 * q) * X6_STRIDE + 4 * lc;
    bf16x4 h1, h2, h3;
    split3(va, h1, h2, h3);
    *(bf16x4 *)(base + 0 * X6_PIECE + off) = h1;
    *(bf16x4 *)(base + 1 * X6_PIECE + off) = h2;
    *(bf16x4 *)(base + 2 * X6_PIECE + off) = h3;
    split3(vb, h1, h2, h3);
    *(bf16x4 *)(base + 3 * X6_PIECE + off) = h1;
    *(bf16x4 *)(base + 4 * X6_PIECE + off) = h2;
    *(bf16x4 *)(base + 5 * X6_PIECE + off) = h3;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = 8 * (lane >> 4);
  // MFMAs on buffer `cur`, interleaved with staging the next chunk into `nxt`
  auto step = [&](const __bf16 *cur, __bf16 *nxt, bool stage, const f32x4 (&ra)[4],
                  const f32x4 (&rb)[4]) {
    bf16x8 b[4][3];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        b[ni][pc] = *(const bf16x8 *)(cur + (3 + pc) * X6_PIECE + (wn * 64 + ni * 16 + fr) * X6_STRIDE + fk);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      bf16x8 a[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        a[pc] = *(const bf16x8 *)(cur + pc * X6_PIECE + (wm * 64 + mi * 16 + fr) * X6_STRIDE + fk);
      if (stage) split_store(nxt, mi, ra[mi], rb[mi]);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        f32x4 c = acc[mi][ni];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[ni][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[ni][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[ni][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[ni][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[ni][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[ni][0], c, 0, 0, 0);
        acc[mi][ni] = c;
      }
    }
  };

  __bf16 *buf0 = lds, *buf1 = lds + 2 * 3 * X6_PIECE;
  f32x4 ra0[4], rb0[4], ra1[4], rb1[4];
  // prologue: chunk 0 -> buf0, chunk 1 -> registers set 1
  gload(ra0, rb0);
#pragma unroll
  for (int q = 0; q < 4; ++q) split_store(buf0, q, ra0[q], rb0[q]);
  if (nk > 1) gload(ra1, rb1);
  __syncthreads();
  int kc = 0;
  for (; kc + 1 < nk; kc += 2) {
    // even iteration: compute buf0 (chunk kc), stage chunk kc+1 (set 1) into buf1
    if (kc + 2 < nk) gload(ra0, rb0);
    step(buf0, buf1, true, ra1, rb1);
    __syncthreads();
    // odd iteration: compute buf1 (chunk kc+1), stage chunk kc+2 (set 0) into buf0
    if (kc + 3 < nk) gload(ra1, rb1);
    step(buf1, buf0, kc + 2 < nk, ra0, rb0);
    __syncthreads();
  }
  if (kc < nk) step(buf0, buf1, false, ra1, rb1);  // odd chunk count: last chunk in buf0

  if (p.split > 1) {  // raw partial sums; the epilogue runs in splitk_epilogue_kernel
    float *part = p.part + (size_t)blockIdx.y * p.M * G.N;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wn * 64 + ni * 16 + (lane & 15);
      if (col >= G.N) continue;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4) + i;
          if (row < p.M) part[(size_t)row * G.N + col] = acc[mi][ni][i];
        }
    }
    return;
  }

  // epilogue: tile (mi, ni) element (row 4*(lane>>4) + i, col lane & 15)
  const int er = 4 * (lane >> 4);
  if constexpr (EPI == EPI_CONV) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wn * 64 + ni * 16 + fr;
      if (col >= G.N) continue;
      const float bias = G.bias ? G.bias[col] : 0.f;
      const float sc = G.scale ? G.scale[col] : 1.f;
      const float sh = G.scale ? G.shift[col] : 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + er + i;
          if (row >= p.M) continue;
          float v = acc[mi][ni][i];
          if (G.bias) v += bias;
          if (p.relu) v = fmaxf(v, 0.f);
          if (G.scale) v = v * sc + sh;
          if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
          if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
          if (p.yt) {
            const int b = row / p.To, t = row - b * p.To;
            p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
          }
        }
    }
  } else {
    // packed column blocks of 32: tiles ni = 0,1 are W1 columns, ni = 2,3 the matching W2
    if (n0 + wn * 64 >= G.N) return;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int col = (n0 + wn * 64) / 2 + ni * 16 + fr;
      const float b1 = p.b1[col], b2 = p.b2[col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + er + i;
          if (row >= p.M) continue;
          const float x1 = acc[mi][ni][i] + b1;
          const float x2 = acc[mi][ni + 2][i] + b2;
          const float g = ftmi_sigmoid(x2);
          const float xin = p.x[(int64_t)row * p.x_stride + col];
          p.y[(int64_t)row * p.y_stride + col] = highway_mix(g, x1, xin);
        }
    }
  }
}


// ---------------------------------------------------------------------------------------
// bf16x6 with PRE-SPLIT weights ("x6b", used when the caller passes w_split).  The 4 waves
// tile the 128x128 block along M (each 32 rows x 128 cols = 2 x 8 tiles of 16x16), so each
// wave loads and splits only ITS OWN activation rows, straight into MFMA A-fragments in
// registers — the activations never go through LDS.  The weights were split into bf16
// pieces once (ftmi_split_weights); each 32-deep chunk of them is staged with 16-B loads
// and ds_write_b128 into a double-buffered LDS image shared by the 4 waves.  Compared with
// the x6 kernel this halves the split VALU work and the LDS write traffic (the binding
// resource there) and needs one barrier per chunk.
// H3 = true is the f16 path (mma = 2): the same staging of three weight planes, the
// activations split into two f16 fragments (head, scaled tail) and three MFMAs per tile.
template <int EPI, bool MAXPOOL, bool H3>
__global__ __launch_bounds__(256, 2) void conv_gemm_x6b_kernel(const GemmParams p) {
  typedef typename Frag<H3>::T frag;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 3 * X6_PIECE];  // [buf][piece][n][48]

  const int tile = blockIdx.x;
  int gi = 0;
  while (gi + 1 < p.ngroups && tile >= p.g[gi + 1].tile0) ++gi;
  const GemmGroup &G = p.g[gi];
  const int lt = tile - G.tile0;
  const int mt = lt / G.ntiles;
  const int nt = lt - mt * G.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;  // fragment row / k-segment (8 k each)

  // ---- A: this lane's rows (per mi) and K position --------------------------------
  const float *arow[2];
  int at[2];
  bool aok[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int m = m0 + wave * 32 + mi * 16 + fr;
    aok[mi] = m < p.M;
    const int mm = aok[mi] ? m : 0;
    const int b = mm / p.To;
    at[mi] = mm - b * p.To;
    arow[mi] = p.x + (int64_t)b * p.T * p.x_stride;
  }
  int nk = (G.Ktot + X6_BK - 1) / X6_BK;
  int kc0 = 0;
  if (p.split > 1) {
    kc0 = blockIdx.y * p.kc_per;
    nk = min(nk - kc0, p.kc_per);
  }
  int kk = kc0 * X6_BK + 8 * fs, tj = kk / p.Cin, tc = kk - tj * p.Cin;
  // Loads go to registers RAW: the zero-padding select and the maxpool max are applied
  // when the chunk is split (two iterations later), so no s_waitcnt is forced at the load.
  // Every load is unconditional (addresses clamped in range): static wait counters.
  struct ARaw {
    f32x4 v[2][2];
    f32x4 u[MAXPOOL ? 2 : 1][2];  // maxpool: the previous frame's row
    unsigned okm;
  };
  auto loadA = [&](ARaw &r) {
    const bool kok = kk < G.Ktot;
    unsigned okm = 0;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int ts = at[mi] + tj - G.pad;
      const bool ok = kok && aok[mi] && ts >= 0 && ts < p.T;
      const float *src = arow[mi] + (int64_t)(ok ? ts : 0) * p.x_stride + (ok ? tc : 0);
      r.v[mi][0] = *(const f32x4 *)src;
      r.v[mi][1] = *(const f32x4 *)(src + 4);
      if constexpr (MAXPOOL) {
        const float *sp = src - ((ok && ts > 0) ? p.x_stride : 0);
        r.u[mi][0] = *(const f32x4 *)sp;
        r.u[mi][1] = *(const f32x4 *)(sp + 4);
      }
      okm |= (unsigned)ok << mi;
    }
    r.okm = okm;
    kk += X6_BK;
    tc += X6_BK;
    // Cin >= 16 (checked on the host): at most two wraps per 32-wide chunk
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const bool wrap = tc >= p.Cin;
      tc -= wrap ? p.Cin : 0;
      tj += wrap;
    }
  };
  float amax = 0.f;  // H3: largest |activation| fed to the f16 split (range guard)
  auto splitA = [&](const ARaw &r, frag (&a)[2][H3 ? 2 : 3]) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      f32x4 v0 = r.v[mi][0], v1 = r.v[mi][1];
      if constexpr (MAXPOOL) {
        v0 = fmax4(v0, r.u[mi][0]);
        v1 = fmax4(v1, r.u[mi][1]);
      }
      const bool ok = (r.okm >> mi) & 1u;
      v0 = sel4(ok, v0);
      v1 = sel4(ok, v1);
      if constexpr (H3) {
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w))));
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w))));
        f16x4 l1, l2, h1, h2;
        split2h(v0, l1, l2);
        split2h(v1, h1, h2);
        a[mi][0] = __builtin_shufflevector(l1, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        a[mi][1] = __builtin_shufflevector(l2, h2, 0, 1, 2, 3, 4, 5, 6, 7);
      } else {
        bf16x4 l1, l2, l3, h1, h2, h3;
        split3(v0, l1, l2, l3);
        split3(v1, h1, h2, h3);
        a[mi][0] = __builtin_shufflevector(l1, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        a[mi][1] = __builtin_shufflevector(l2, h2, 0, 1, 2, 3, 4, 5, 6, 7);
        a[mi][2] = __builtin_shufflevector(l3, h3, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  };

  // ---- B: 6 x 16 B of pre-split pieces per thread per chunk ------------------------
  // Rows n >= N read row N-1 (clamped, no select): they only feed output columns that
  // are never stored.  Chunks past the end re-read the last chunk (clamped).
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const __bf16 *bsrc[6];
  int boff[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int idx = tid + 256 * i;
    const int pc = idx >> 9, rem = idx & 511, nl = rem >> 2, seg = rem & 3;
    const int n = n0 + nl < G.N ? n0 + nl : G.N - 1;
    bsrc[i] = G.w3 + ((int64_t)pc * G.N + n) * G.Kpad + kc0 * X6_BK + seg * 8;
    boff[i] = pc * X6_PIECE + nl * X6_STRIDE + seg * 8;
  }
  const int kb_last = (nk - 1) * X6_BK;
  int kb = 0;  // chunk offset (elements) of the next B load
  auto loadB = [&](u32x4 (&rb)[6]) {
    const int o = kb < kb_last ? kb : kb_last;
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[i] = *(const u32x4 *)(bsrc[i] + o);
    kb += X6_BK;
  };
  auto storeB = [&](const u32x4 (&rb)[6], int buf) {
#pragma unroll
    for (int i = 0; i < 6; ++i) *(u32x4 *)(lds + buf * 3 * X6_PIECE + boff[i]) = rb[i];
  };

  f32x4 acc[2][8];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto mfma_chunk = [&](const frag (&a)[2][H3 ? 2 : 3], int buf) {
    const __bf16 *cur = lds + buf * 3 * X6_PIECE;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      frag b[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        b[pc] = *(const frag *)(cur + pc * X6_PIECE + (ni * 16 + fr) * X6_STRIDE + 8 * fs);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        f32x4 c = acc[mi][ni];
        if constexpr (H3) {  // small terms first: a_t w_h, a_h w_t, then a_h 2^11 w_h
          c = mma16(a[mi][1], b[2], c);
          c = mma16(a[mi][0], b[1], c);
          c = mma16(a[mi][0], b[0], c);
        } else {
          c = mma16(a[mi][2], b[0], c);
          c = mma16(a[mi][1], b[1], c);
          c = mma16(a[mi][0], b[2], c);
          c = mma16(a[mi][1], b[0], c);
          c = mma16(a[mi][0], b[1], c);
          c = mma16(a[mi][0], b[0], c);
        }
        acc[mi][ni] = c;
      }
    }
  };

  // chunk c lives in LDS buffer c & 1 and (H3) A register set c & 1; the B registers hold
  // the next chunk to stage.  Prefetch distance: A two chunks on the f16 path, one on the
  // bf16 path (its three-piece fragments leave no room for a second set), B one.
  constexpr bool DEEP = H3;
  ARaw ra0, ra1;
  u32x4 rb[6];
  loadA(ra0);
  loadB(rb);  // chunk 0
  if constexpr (DEEP) loadA(ra1);
  storeB(rb, 0);
  loadB(rb);  // chunk 1
  __syncthreads();
  // one step: split chunk kc, prefetch the A chunk DEEP ? kc+2 : kc+1 into the freed set,
  // stage B kc+1 into LDS and prefetch B kc+2, MFMAs on chunk kc, barrier
  auto step = [&](int kc, ARaw &ras) {
    frag a[2][H3 ? 2 : 3];
    splitA(ras, a);
    loadA(ras);
    if (kc + 1 < nk) storeB(rb, (kc + 1) & 1);
    loadB(rb);
    mfma_chunk(a, kc & 1);
    __syncthreads();
  };
  for (int kc = 0; kc < nk; kc += 2) {
    step(kc, ra0);
    if (kc + 1 >= nk) break;
    step(kc + 1, DEEP ? ra1 : ra0);
  }

  if constexpr (H3) {  // undo the 2^11 / column pre-scaling; report f16 range overflow
    bool bad = !(amax <= 65504.f);
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int col = n0 + ni * 16 + fr;
      const float cs = G.colscale[col < G.N ? col : G.N - 1];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wave * 32 + mi * 16 + 4 * fs + i;
          bad |= col < G.N && row >= 0 && row < p.M && !__builtin_isfinite(acc[mi][ni][i]);
          acc[mi][ni][i] *= cs;
        }
    }
    if (bad && p.status) atomicOr(p.status, 1u);
  }

  const int er = 4 * fs;
  if (p.split > 1) {  // raw partial sums; the epilogue runs in splitk_epilogue_kernel
    float *part = p.part + (size_t)blockIdx.y * p.M * G.N;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int col = n0 + ni * 16 + fr;
      if (col >= G.N) continue;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wave * 32 + mi * 16 + er + i;
          if (row < p.M) part[(size_t)row * G.N + col] = acc[mi][ni][i];
        }
    }
    return;
  }
  if constexpr (EPI == EPI_CONV) {
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int col = n0 + ni * 16 + fr;
      if (col >= G.N) continue;
      const float bias = G.bias ? G.bias[col] : 0.f;
      const float sc = G.scale ? G.scale[col] : 1.f;
      const float sh = G.scale ? G.shift[col] : 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wave * 32 + mi * 16 + er + i;
          if (row >= p.M) continue;
          float v = acc[mi][ni][i];
          if (G.bias) v += bias;
          if (p.relu) v = fmaxf(v, 0.f);
          if (G.scale) v = v * sc + sh;
          if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
          if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
          if (p.yt) {
            const int b = row / p.To, t = row - b * p.To;
            p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
          }
        }
    }
  } else {
    // packed 32-row blocks [W1 | W2] per 64 columns: tiles ni = 4q + {0,1} are W1,
    // ni = 4q + {2,3} the matching W2 columns (q = 0, 1)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (n0 + q * 64 >= G.N) continue;
        const int ni = 4 * q + h;
        const int col = n0 / 2 + q * 32 + h * 16 + fr;
        const float b1 = p.b1[col], b2 = p.b2[col];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = m0 + wave * 32 + mi * 16 + er + i;
            if (row >= p.M) continue;
            const float x1 = acc[mi][ni][i] + b1;
            const float x2 = acc[mi][ni + 2][i] + b2;
            const float g = ftmi_sigmoid(x2);
            const float xin = p.x[(int64_t)row * p.x_stride + col];
            p.y[(int64_t)row * p.y_stride + col] = highway_mix(g, x1, xin);
          }
      }
  }
}

// ---- slab kernel: k-tap convolutions on the f16x3 path (mma = 2, To == T, one group) ----
// A 256 x 128 output tile per workgroup, 8 waves as 4 (rows) x 2 (columns) of 64 x 64.
// Per 32-channel chunk the input rows [m0 - pad, m0 + 256 + k - 1 - pad) are read ONCE,
// split into f16 head / scaled tail while staged into LDS (the "slab"), and serve all k taps:
// tap j reads slab row r + j for output row r; a row whose frame t + j - pad falls outside
// its sequence takes zero (per-row tap masks).  The x6b kernel re-reads every input row k
// times through L2 with a 128 x 128 tile; here the operand bytes per MFMA drop ~3x for
// k = 3.  B moves two f16 planes per tap (B0 = 2^11 w_h, B1 = w_t); the third, w_h, is B0 *
// 2^-11 in registers (exact: a power-of-two rescale of an f16 value back to itself).
// Steps are (chunk, tap): B double buffered per step, the slab double buffered per chunk.
constexpr int SL_BM = 256;
constexpr int SL_BN = 128;
constexpr int SL_MAXK = 16;
constexpr int SL_SR = SL_BM + SL_MAXK - 1;          // slab rows
constexpr int SL_P = 48;                            // halves per LDS row: 96-B pitch keeps
                                                    // the ds_read_b128 fragments conflict free
constexpr int SL_ZROW = SL_SR;                       // an all-zero row after the slab rows:
                                                    // masked taps read it (no selects)
constexpr int SL_AIMG = (SL_SR + 1) * SL_P;         // halves per (buffer, plane) slab image
constexpr int SL_BIMG = SL_BN * SL_P;               // halves per (buffer, plane) B image
constexpr int SL_TP = SL_BN + 4;                    // floats per row of the epilogue tile

// Tile of slab-kernel block bid (conv_gemm_slab_kernel, conv_gemm_slabp_kernel): blocks b
// and b + 8 run on the same XCD under round-robin dispatch (placement only ever affects
// speed), so XCD x = bid & 7 takes the row tiles mt = 8 lr + x.  band = 0: within an XCD, all
// VT (group, column) tiles of a row tile are consecutive — its slab rows shared through L2.
// band = CB > 0: the XCD walks its row tiles once per band of CB consecutive (group, column)
// tiles, so one band's weight planes stay L2-resident while every row tile of the XCD
// passes (a 1024-column layer's 9.4 MB of planes do not fit a 4 MB L2; two 128-column tiles'
// 2.4 MB do), at the price of re-reading each row tile once per band.
__device__ __forceinline__ void slab_tile(int bid, int MT, int VT, int band, int &mt, int &v8) {
  if (MT < 8) {  // few row tiles: a compact grid, row tile fastest (spread over the XCDs)
    mt = bid % MT;
    v8 = bid / MT;
    return;
  }
  const int x = bid & 7, s8 = bid >> 3;
  if (band <= 0 || band >= VT) {
    const int q8 = s8 / VT;
    mt = q8 * 8 + x;
    v8 = s8 - q8 * VT;
    return;
  }
  const int MTx = (MT + 7) >> 3;           // row tiles per XCD (padded grid)
  const int per = MTx * band, b = s8 / per, rem = s8 - b * per;
  const int cbn = min(band, VT - b * band);  // the last band may be narrower
  const int lr = rem / cbn;
  mt = lr * 8 + x;
  v8 = b * band + (rem - lr * cbn);
  if (lr >= MTx) mt = MT;  // (never: rem < MTx * cbn) — out of range, the block returns
}


// The slab kernels' epilogue: the finished fp32 tile [SL_BM][SL_TP] (colscale applied) in
// LDS -> split-K partials, or bias / ReLU / BN / residual (conv: plain, transposed or pooled
// rows, optionally as f16x3 split rows), or the highway gating.  Every store moves 16 B.
template <int EPI, int NTHR>
__device__ __forceinline__ void slab_epilogue(const GemmParams &p, const GemmGroup &G,
                                              float *tile, int m0, int n0, int tid) {
  const int rows = min(SL_BM, p.M - m0);
  const int ncols = min(SL_BN, G.N - n0);  // a multiple of 4 (slab_ok)

  if (p.split > 1) {  // raw partial sums; splitk_epilogue_kernel finishes
    float *part = p.part + (size_t)blockIdx.y * p.M * G.N;
    for (int idx = tid; idx < SL_BM * (SL_BN / 4); idx += NTHR) {
      const int r = idx >> 5, c = (idx & 31) * 4;
      if (r < rows && c < ncols)
        *(f32x4 *)(part + (size_t)(m0 + r) * G.N + n0 + c) = *(const f32x4 *)(tile + r * SL_TP + c);
    }
    return;
  }
  if constexpr (EPI == EPI_CONV) {
    if (p.pool_out) {  // finish every row in the tile, then store max(row - 1, row)
      for (int idx = tid; idx < SL_BM * (SL_BN / 4); idx += NTHR) {
        const int r = idx >> 5, c = (idx & 31) * 4;
        if (r >= rows || c >= ncols) continue;
        const int col = n0 + c;
        f32x4 v = *(const f32x4 *)(tile + r * SL_TP + c);
        if (G.bias) v += *(const f32x4 *)(G.bias + col);
        if (p.relu) v = fmax4(v, (f32x4){0.f, 0.f, 0.f, 0.f});
        if (G.scale) v = v * *(const f32x4 *)(G.scale + col) + *(const f32x4 *)(G.shift + col);
        *(f32x4 *)(tile + r * SL_TP + c) = v;
      }
      __syncthreads();
      float ymax = 0.f;
      for (int idx = tid; idx < SL_BM * (SL_BN / 4); idx += NTHR) {
        const int r = idx >> 5, c = (idx & 31) * 4;
        if (r == 0 || r >= rows || c >= ncols) continue;
        const int row = m0 + r, col = n0 + c;
        f32x4 v = *(const f32x4 *)(tile + r * SL_TP + c);
        if (row % p.T > 0) v = fmax4(v, *(const f32x4 *)(tile + (r - 1) * SL_TP + c));
        if (p.y_split_c) {  // split rows for the next f16x3 GEMM (proj1), range-checked here
          ymax = fmaxf(ymax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          f16x4 h, t;
          split2h(v, h, t);
          _Float16 *yr = (_Float16 *)(p.y + (int64_t)row * p.y_stride) + G.ycol0 + col;
          *(f16x4 *)yr = h;
          *(f16x4 *)(yr + p.y_split_c) = t;
        } else {
          *(f32x4 *)(p.y + (int64_t)row * p.y_stride + G.ycol0 + col) = v;
        }
      }
      if (!(ymax <= 65504.f) && p.status) atomicOr(p.status, 1u);
      return;
    }
    for (int idx = tid; idx < SL_BM * (SL_BN / 4); idx += NTHR) {
      const int r = idx >> 5, c = (idx & 31) * 4;
      if (r >= rows || c >= ncols) continue;
      const int row = m0 + r, col = n0 + c;
      f32x4 v = *(const f32x4 *)(tile + r * SL_TP + c);
      if (G.bias) v += *(const f32x4 *)(G.bias + col);
      if (p.relu) v = fmax4(v, (f32x4){0.f, 0.f, 0.f, 0.f});
      if (G.scale) v = v * *(const f32x4 *)(G.scale + col) + *(const f32x4 *)(G.shift + col);
      if (p.residual) v += *(const f32x4 *)(p.residual + (int64_t)row * p.res_stride + col);
      if (p.y) *(f32x4 *)(p.y + (int64_t)row * p.y_stride + G.ycol0 + col) = v;
      if (p.yt) *(f32x4 *)(tile + r * SL_TP + c) = v;  // finished values for the yt pass
    }
    if (p.yt) {  // (B, N, To) copy: consecutive lanes take consecutive frames
      __syncthreads();
      for (int idx = tid; idx < SL_BM * SL_BN; idx += NTHR) {
        const int r = idx & (SL_BM - 1), c = idx / SL_BM;
        if (r >= rows || c >= ncols) continue;
        const int row = m0 + r, b = row / p.To, t = row - b * p.To;
        p.yt[((int64_t)b * p.yt_channels + G.ycol0 + n0 + c) * p.To + t] = tile[r * SL_TP + c];
      }
    }
  } else {
    // highway: packed 32-column blocks [W1 | W2] per 64 GEMM columns; GEMM columns
    // q*64 + h (W1) and q*64 + 32 + h (W2) of the tile give output column n0/2 + q*32 + h
    for (int idx = tid; idx < SL_BM * (SL_BN / 8); idx += NTHR) {
      const int r = idx >> 4, o = (idx & 15) * 4, q = o >> 5, h = o & 31;
      if (r >= rows || q * 64 >= ncols) continue;
      const int row = m0 + r, col = n0 / 2 + o;
      const f32x4 x1 = *(const f32x4 *)(tile + r * SL_TP + q * 64 + h) + *(const f32x4 *)(p.b1 + col);
      const f32x4 x2 = *(const f32x4 *)(tile + r * SL_TP + q * 64 + 32 + h) + *(const f32x4 *)(p.b2 + col);
      const f32x4 xin = *(const f32x4 *)(p.x + (int64_t)row * p.x_stride + col);
      f32x4 out;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = ftmi_sigmoid(x2[e]);
        out[e] = highway_mix(g, x1[e], xin[e]);
      }
      *(f32x4 *)(p.y + (int64_t)row * p.y_stride + col) = out;
    }
  }
}

// WS (warp-specialised, 768 threads): waves 0-7 only read fragments and issue MFMAs; waves
// 8-11 do all staging (global loads, the slab's f16 split, LDS stores), so the staging VALU
// and load waits never sit in the MFMA waves' instruction streams.  !WS: all 8 waves do both.
template <int EPI, bool MAXPOOL, bool WS>
__global__ __launch_bounds__(WS ? 768 : 512, 1) void conv_gemm_slab_kernel(const GemmParams p) {
  constexpr int NTHR = WS ? 768 : 512;              // threads per workgroup
  constexpr int NSTG = WS ? 256 : 512;              // staging threads
  constexpr int SL_ASLOTS = (SL_SR * 8 + NSTG - 1) / NSTG;  // float4 slab loads per thread
  constexpr int SL_BSLOTS = 1024 / NSTG;            // 16-B B loads per thread per step
  // slab images [buf][h|t][row][48], then B images [buf][B0|B1][n][48]; the epilogue reuses
  // the whole array as the fp32 output tile
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 2 * SL_AIMG + 2 * 2 * SL_BIMG];
  static_assert(SL_BM * SL_TP * 4 <= sizeof(lds), "epilogue tile");
  _Float16 *const lds_a = lds;
  _Float16 *const lds_b = lds + 2 * 2 * SL_AIMG;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  // XCD-aware order: blocks b and b + 8 run on the same XCD, and the tiles of one row tile
  // (every column tile of every group: a conv bank's groups all read the same input rows)
  // are consecutive in that XCD's order, so its slab rows are shared through L2.  Groups
  // (conv bank: one per kernel size, heaviest first) all have NT column tiles.
  const int TS = p.pool_out ? SL_BM - 1 : SL_BM;  // rows a tile produces
  const int MT = (p.M + TS - 1) / TS, NT = p.g[0].ntiles, VT = p.ngroups * NT;
  // With fewer than 8 row tiles (small batches) that order would put every working block on
  // one XCD: the grid is then compact, row tile fastest, and consecutive blocks spread.
  int mt, v8;
  slab_tile(blockIdx.x, MT, VT, p.band, mt, v8);
  const int gi = v8 / NT, nt = v8 - gi * NT;
  if (mt >= MT) return;  // the grid is padded to whole XCD rounds
  const GemmGroup &G = p.g[gi];
  // pool_out: the tile's row 0 is the halo row m0 = mt * TS - 1 (only feeds the pooling)
  const int m0 = p.pool_out ? mt * TS - 1 : mt * SL_BM, n0 = nt * SL_BN;
  const int k = G.k, pad = G.pad, Cin = p.Cin;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = (wave >> 2) & 1;
  const int fr = lane & 15, fs = lane >> 4;  // fragment row / k-segment (8 k each)
  const bool is_mma = !WS || wave < 8;       // wave-uniform roles
  const bool is_stg = !WS || wave >= 8;
  const int stid = WS ? tid - 512 : tid;     // staging thread index (valid when is_stg)

  // 32-channel chunks; with Cin % 32 != 0 the last chunk is partial: its missing channels
  // are zero in the slab and in the staged B (cbase + chunk offset + lane channel >= Cin)
  int nch = (Cin + 31) / 32, c_begin = 0;
  if (p.split > 1) {  // split over channel chunks: blockIdx.y = s takes [s kc_per, ...)
    c_begin = blockIdx.y * p.kc_per;
    nch = min(nch - c_begin, p.kc_per);
  }
  const int nsteps = nch * k;

  // ---- slab loads: slot i = slab row sr (input row m0 - pad + sr), channels seg*4..+3 ----
  // Every load is unconditional with a clamped address (static wait counters); clamped
  // rows only feed taps that the row masks zero.
  const int SR = SL_BM + k - 1;
  // the 16 lanes of one ds_write_b64 group write slab rows sr and sr + 2 (conflict free);
  // slot i of a staging lane is slab row sr0 + (NSTG / 8) i
  const int sr0 = 4 * (stid >> 5) + ((stid >> 4) & 1) + 2 * ((stid >> 3) & 1);
  const int adst0 = sr0 * SL_P + (stid & 7) * 4;
  unsigned aoff[SL_ASLOTS];
  unsigned prev = 0;  // maxpool: bit i = slot i's frame has a predecessor in its sequence
#pragma unroll
  for (int i = 0; i < SL_ASLOTS; ++i) {
    int mp = m0 - pad + sr0 + (NSTG / 8) * i;
    mp = mp < 0 ? 0 : (mp >= p.M ? p.M - 1 : mp);
    aoff[i] = (unsigned)mp * (unsigned)p.x_stride;  // row start; + channel at the load
    if constexpr (MAXPOOL) prev |= (unsigned)(mp % p.T > 0) << i;
  }
  struct ARaw {
    f32x4 v[SL_ASLOTS];
    f32x4 u[MAXPOOL ? SL_ASLOTS : 1];
    bool ok;  // this lane's 4 channels exist (all slots of a lane share them)
  };
  const unsigned cbase = (unsigned)c_begin * 32u, aseg = (unsigned)(stid & 7) * 4u;
  const unsigned a_last = (unsigned)(nch - 1) * 32u;
  unsigned ach = 0;  // channel offset (within this split) of the next slab load
  auto loadA = [&](ARaw &r) {
    const unsigned ch = cbase + (ach < a_last ? ach : a_last) + aseg;
    r.ok = ch < (unsigned)Cin;
    const unsigned o = r.ok ? ch : 0u;
    if (!MAXPOOL && p.x_split) {  // split rows: 4 heads + the same 4 tails in one register
#pragma unroll
      for (int i = 0; i < SL_ASLOTS; ++i) {
        const _Float16 *xr = (const _Float16 *)(p.x + aoff[i]) + o;
        const u32x2 h = *(const u32x2 *)xr, t = *(const u32x2 *)(xr + Cin);
        r.v[i] = __builtin_bit_cast(f32x4, ((u32x4){h.x, h.y, t.x, t.y}));
      }
      ach += 32;
      return;
    }
#pragma unroll
    for (int i = 0; i < SL_ASLOTS; ++i) {
      r.v[i] = *(const f32x4 *)(p.x + aoff[i] + o);
      // CBHG maxpool(2, 1) fused: max(x[t - 1], x[t]); x[0] at t = 0
      if constexpr (MAXPOOL)
        r.u[i] = *(const f32x4 *)(p.x + aoff[i] - ((prev >> i) & 1u ? (unsigned)p.x_stride : 0u) + o);
    }
    ach += 32;
  };
  float amax = 0.f;  // range guard: largest |activation| fed to the f16 split
  auto storeA = [&](const ARaw &r, int buf) {
    _Float16 *dst = lds_a + buf * 2 * SL_AIMG;
#pragma unroll
    for (int i = 0; i < SL_ASLOTS; ++i) {
      if (sr0 + (NSTG / 8) * i >= SR) continue;
      const int adst = adst0 + (NSTG / 8) * i * SL_P;
      f32x4 v = r.v[i];
      if (!MAXPOOL && p.x_split) {  // already split (and range-checked by the producer)
        u32x4 b = __builtin_bit_cast(u32x4, v);
        if (!r.ok) b = (u32x4){0u, 0u, 0u, 0u};
        *(u32x2 *)(dst + adst) = (u32x2){b.x, b.y};
        *(u32x2 *)(dst + SL_AIMG + adst) = (u32x2){b.z, b.w};
        continue;
      }
      if constexpr (MAXPOOL) v = fmax4(v, r.u[i]);
      v = sel4(r.ok, v);
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      f16x4 h, t;
      split2h(v, h, t);
      *(f16x4 *)(dst + adst) = h;
      *(f16x4 *)(dst + SL_AIMG + adst) = t;
    }
  };

  // ---- B: planes B0 / B1 of tap j, channels of the chunk; 2 x 16 B per thread per step ---
  // Rows n >= N read row N-1 (their output columns are never stored); steps past the end
  // re-read the last step (clamped).
  const _Float16 *w16 = (const _Float16 *)G.w3;
  const _Float16 *bsrc[SL_BSLOTS];
  int bdst[SL_BSLOTS];
#pragma unroll
  for (int i = 0; i < SL_BSLOTS; ++i) {
    // the 8 lanes of one ds_write_b128 group write rows nl and nl + 2 (bank offset 16 of 32:
    // conflict free); rows 4g + {0, 1, 2, 3} come from lane pairs (2g, 2g + 1)
    const int idx = stid + NSTG * i, pl = idx >> 9, rem = idx & 511, seg = rem & 3;
    const int pr = rem >> 3, nl = 4 * (pr >> 1) + (pr & 1) + 2 * ((rem >> 2) & 1);
    const int n = n0 + nl < G.N ? n0 + nl : G.N - 1;
    bsrc[i] = w16 + ((int64_t)pl * G.N + n) * G.Kpad;  // row start; + tap / channel at the load
    bdst[i] = pl * SL_BIMG + nl * SL_P + seg * 8;
  }
  struct BRaw {
    u32x4 v[SL_BSLOTS];
    bool ok;  // this lane's 8 channels exist
  };
  const int bseg = (stid & 3) * 8;
  int bj = 0, bc = 0;  // tap / chunk of the next B load
  auto loadB = [&](BRaw &rb) {
    const bool in = bc < nch;
    const int ch = (int)cbase + (in ? bc : nch - 1) * 32 + bseg;
    rb.ok = ch < Cin;
    const int off = (in ? bj : k - 1) * Cin + (rb.ok ? ch : 0);
#pragma unroll
    for (int i = 0; i < SL_BSLOTS; ++i) rb.v[i] = *(const u32x4 *)(bsrc[i] + off);
    if (++bj == k) {
      bj = 0;
      ++bc;
    }
  };
  auto storeB = [&](const BRaw &rb, int buf) {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL_BSLOTS; ++i)
      *(u32x4 *)(lds_b + buf * 2 * SL_BIMG + bdst[i]) = rb.ok ? rb.v[i] : z;
  };

  // ---- per-row tap masks: bit j set iff frame t + j - pad lies inside the sequence -------
  unsigned vmask[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = m0 + wm * 64 + mi * 16 + fr;
    unsigned msk = 0;
    if (m >= 0 && m < p.M) {
      const int t = m % p.T;
      const int lo = max(pad - t, 0), hi = min(p.T - 1 + pad - t, k - 1);
      if (lo <= hi) msk = (2u << hi) - (1u << lo);
    }
    vmask[mi] = msk;
  }

  auto zero_acc = [](f32x4 (&acc)[4][4]) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };
  // A-fragment addresses without a multiply per fragment: the row (wm 64 + mi 16 + fr + j)
  // is the lane's base + j SL_P (per step) + mi 16 SL_P (the instruction's immediate), and a
  // masked tap's zero row is selected as an offset from that same immediate (the select
  // before a multiply cost a quarter-rate v_mul_lo_u32 per fragment; the same addresses)
  const int a_row0 = (wm * 64 + fr) * SL_P + fs * 8, a_zrow = SL_ZROW * SL_P + fs * 8;
  auto mfma_step = [&](f32x4 (&acc)[4][4], int abuf, int bbuf, int j) {
    const _Float16 *Ab = lds_a + abuf * 2 * SL_AIMG;
    const _Float16 *Bb = lds_b + bbuf * 2 * SL_BIMG;
    f16x8 ah[4], at[4];
    const int a_rowj = a_row0 + j * SL_P;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const bool ok = (vmask[mi] >> j) & 1u;
      const int o = (ok ? a_rowj : a_zrow - mi * 16 * SL_P) + mi * 16 * SL_P;
      ah[mi] = *(const f16x8 *)(Ab + o);
      at[mi] = *(const f16x8 *)(Ab + SL_AIMG + o);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int o = (wn * 64 + ni * 16 + fr) * SL_P + fs * 8;
      const f16x8 b0 = *(const f16x8 *)(Bb + o);
      const f16x8 b1 = *(const f16x8 *)(Bb + SL_BIMG + o);
      const f16x8 bh = b0 * (_Float16)(1.0f / H3_SCALE);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {  // small terms first, as in x6b
        f32x4 c = acc[mi][ni];
        c = mma16(at[mi], bh, c);
        c = mma16(ah[mi], b1, c);
        c = mma16(ah[mi], b0, c);
        acc[mi][ni] = c;
      }
    }
  };
  // undo the 2^11 / column scaling; true when an accumulator of a stored element is not
  // finite (range guard)
  auto finish_acc = [&](f32x4 (&acc)[4][4]) -> bool {
    bool bad = false;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wn * 64 + ni * 16 + fr;
      const float cs = G.colscale[col < G.N ? col : G.N - 1];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wm * 64 + mi * 16 + 4 * fs + i;
          bad |= col < G.N && row < p.M && !__builtin_isfinite(acc[mi][ni][i]);
          acc[mi][ni][i] *= cs;
        }
    }
    return bad;
  };
  // the tile goes through LDS (the pipeline buffers are free by then) so that every store
  // moves whole rows, 16 B per lane: the fragment layout would write 64-B pieces of 4 rows
  float *tile = (float *)lds;  // [SL_BM][SL_TP]
  auto write_tile = [&](const f32x4 (&acc)[4][4]) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          tile[(wm * 64 + mi * 16 + 4 * fs + i) * SL_TP + wn * 64 + ni * 16 + fr] = acc[mi][ni][i];
  };

  // ---- pipeline: step s = (chunk c, tap j) uses slab buffer c & 1 and B buffer s & 1 ------
  // At step s: stage B s+1 (register set (s+1) & 1, loaded two steps ago) and, on a chunk's
  // last tap, slab c+1; reload that B set with step s+3 and the slab registers with chunk
  // c+2; MFMAs; barrier.
  if (tid < 2 * 2 * SL_P / 8) {  // the zero rows of both buffers and planes
    const int img = tid / (SL_P / 8), part = tid % (SL_P / 8);
    *(u32x4 *)(lds_a + img * SL_AIMG + SL_ZROW * SL_P + part * 8) = (u32x4){0u, 0u, 0u, 0u};
  }
  bool bad;
  if constexpr (WS) {
    // Two loops with the same barrier count (1 + nsteps + 1): the staging waves never hold
    // accumulators and the MFMA waves never hold staging registers.
    if (is_stg) {
      ARaw ra;
      BRaw rb0, rb1;
      loadA(ra);
      loadB(rb0);  // step 0
      storeA(ra, 0);
      storeB(rb0, 0);
      loadB(rb1);  // step 1
      loadB(rb0);  // step 2
      if (nch > 1) loadA(ra);  // chunk 1
      __syncthreads();
      int c = 0, j = 0;
      auto sstep = [&](int s, BRaw &rbs) {
        const bool last_tap = j == k - 1 && c + 1 < nch;
        if (s + 1 < nsteps) storeB(rbs, (s + 1) & 1);
        if (last_tap) storeA(ra, (c + 1) & 1);
        loadB(rbs);
        if (last_tap) loadA(ra);
        __syncthreads();
        if (++j == k) {
          j = 0;
          ++c;
        }
      };
      for (int s = 0; s < nsteps; s += 2) {
        sstep(s, rb1);
        if (s + 1 >= nsteps) break;
        sstep(s + 1, rb0);
      }
      bad = !(amax <= 65504.f);
      __syncthreads();  // the MFMA waves write the tile
    } else {
      f32x4 acc[4][4];
      zero_acc(acc);
      __syncthreads();
      int c = 0, j = 0;
      for (int s = 0; s < nsteps; ++s) {
        mfma_step(acc, c & 1, s & 1, j);
        __syncthreads();
        if (++j == k) {
          j = 0;
          ++c;
        }
      }
      bad = finish_acc(acc);
      write_tile(acc);  // every wave is past its last fragment read (the loop's barrier)
      __syncthreads();
    }
  } else {
    f32x4 acc[4][4];
    zero_acc(acc);
    ARaw ra;
    BRaw rb0, rb1;
    loadA(ra);
    loadB(rb0);  // step 0
    storeA(ra, 0);
    storeB(rb0, 0);
    loadB(rb1);  // step 1
    loadB(rb0);  // step 2
    if (nch > 1) loadA(ra);  // chunk 1
    __syncthreads();
    int c = 0, j = 0;
#ifdef FTMI_DIAG
    const int diag = p.diag;  // timing experiments: results invalid when set
#else
    constexpr int diag = 0;
#endif
    auto step = [&](int s, BRaw &rbs) {
      const bool last_tap = j == k - 1 && c + 1 < nch;
      // MFMAs first: the staging below (LDS stores of the next B / slab, the slab's f16
      // split, the next loads) is independent of them and fills the matrix pipe's shadow
      if (!(diag & 2)) mfma_step(acc, c & 1, s & 1, j);
      if (s + 1 < nsteps) storeB(rbs, (s + 1) & 1);
      if (last_tap) storeA(ra, (c + 1) & 1);
      if (!(diag & 4)) {
        loadB(rbs);
        if (last_tap) loadA(ra);
      }
      if (!(diag & 1)) __syncthreads();
      if (++j == k) {
        j = 0;
        ++c;
      }
    };
    for (int s = 0; s < nsteps; s += 2) {
      step(s, rb1);
      if (s + 1 >= nsteps) break;
      step(s + 1, rb0);
    }
    bad = !(amax <= 65504.f);
    bad |= finish_acc(acc);
    __syncthreads();  // every wave is past its last fragment read
    write_tile(acc);
    __syncthreads();
  }
  if (bad && p.status) atomicOr(p.status, 1u);
  slab_epilogue<EPI, NTHR>(p, G, tile, m0, n0, tid);
}

// ---- slab kernel with fragment prefetch (default for single-group k = 1 GEMMs) ----------
// The slab kernel above stalls at the top of every step: the step's B plane is stored just
// before the barrier, so every wave issues its 16 fragment reads after it and waits for them
// (PMC at the c5 k9 FFN conv, warp-specialised form: MFMA busy 59 %, waves parked in waitcnt /
// barrier 41 % of their cycles).  Here the fragments of step s + 1 are read DURING step s,
// into a second register set, while the MFMAs of step s run: the B planes are triple-buffered
// (B(s + 2) is stored in iteration s, so B(s + 1) is visible one barrier earlier) and so is
// the slab (chunk c is stored in iteration c k - 2).  The LDS images drop the 96-B padded
// pitch for unpadded 64-B rows whose 16-B segments are XOR-swizzled by row bit 2
// (segment s of row r at s ^ 2 ((r >> 2) & 1)): conflict-free ds_read_b128 fragment reads for
// 16 consecutive rows from any first row (every tap shift), 3 + 3 buffers in 150 KB.
// 512 threads: every wave multiplies and stages (the register budget of the warp-specialised
// 768-thread form cannot hold two fragment sets).  Bit-identical to conv_gemm_slab_kernel
// (same MFMA order and operands).  Measured (tools/slabp_ab.py, c3 / c5 shapes): k = 1
// GEMMs 6-10 % faster than the 512-thread slab kernel; multi-tap convs and banks 0-6 %
// SLOWER than the warp-specialised one: the staging (slab split, addresses) now sits in
// the MFMA waves' instruction stream, ~200 VALU per 48 MFMAs per step, which the MFMA
// issue shadow cannot absorb — the LDS wait it removes was not the only cost.
constexpr int SP_ROW = 32;                     // halves per LDS row (32 channels, no pad)
constexpr int SP_AIMG = (SL_SR + 1) * SP_ROW;  // halves per (buffer, plane) slab image
constexpr int SP_BIMG = SL_BN * SP_ROW;        // halves per (buffer, plane) B image
constexpr int SP_NBUF = 3;
__device__ __forceinline__ int sp_off(int r, int seg) {  // half offset of (row, 16-B segment)
  return r * SP_ROW + ((seg ^ (((r >> 2) & 1) << 1)) << 3);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void conv_gemm_slabp_kernel(const GemmParams p) {
  constexpr int NTHR = 512;
  constexpr int ASLOTS = (SL_SR * 8 + NTHR - 1) / NTHR;  // 4-channel slab items per thread
  constexpr int BSLOTS = 1024 / NTHR;                    // 16-B B items per thread and step
  __shared__ __attribute__((aligned(16))) _Float16 lds[SP_NBUF * 2 * SP_AIMG + SP_NBUF * 2 * SP_BIMG];
  static_assert(SL_BM * SL_TP * 4 <= sizeof(lds), "epilogue tile");
  _Float16 *const lds_a = lds;
  _Float16 *const lds_b = lds + SP_NBUF * 2 * SP_AIMG;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  // tile order: conv_gemm_slab_kernel's (XCD-aware)
  const int TS = p.pool_out ? SL_BM - 1 : SL_BM;
  const int MT = (p.M + TS - 1) / TS, NT = p.g[0].ntiles, VT = p.ngroups * NT;
  int mt, v8;
  slab_tile(blockIdx.x, MT, VT, p.band, mt, v8);
  const int gi = v8 / NT, nt = v8 - gi * NT;
  if (mt >= MT) return;
  const GemmGroup &G = p.g[gi];
  const int m0 = p.pool_out ? mt * TS - 1 : mt * SL_BM, n0 = nt * SL_BN;
  const int k = G.k, pad = G.pad, Cin = p.Cin;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int fr = lane & 15, fs = lane >> 4;
  int nch = (Cin + 31) / 32, c_begin = 0;
  if (p.split > 1) {
    c_begin = blockIdx.y * p.kc_per;
    nch = min(nch - c_begin, p.kc_per);
  }
  const int nsteps = nch * k;

  // ---- slab staging: item i = (slab row tid / 8 + 64 i, 8-B granule tid & 7 = 4 channels);
  // 32 lanes store 4 whole 64-B rows (all 64 banks once) -----------------------------------
  const int SR = SL_BM + k - 1;
  const int g8 = tid & 7, sr0 = tid >> 3;
  unsigned aoff[ASLOTS];
#pragma unroll
  for (int i = 0; i < ASLOTS; ++i) {
    int mp = m0 - pad + sr0 + 64 * i;
    mp = mp < 0 ? 0 : (mp >= p.M ? p.M - 1 : mp);  // clamped rows only feed masked taps
    aoff[i] = (unsigned)mp * (unsigned)p.x_stride;
  }
  const unsigned cbase = (unsigned)c_begin * 32u, aseg = (unsigned)g8 * 4u;
  const unsigned a_last = (unsigned)(nch - 1) * 32u;
  unsigned ach = 0;
  struct ARaw {
    f32x4 v[ASLOTS];
    bool ok;
  };
  auto loadA = [&](ARaw &r) {
    const unsigned ch = cbase + (ach < a_last ? ach : a_last) + aseg;
    r.ok = ch < (unsigned)Cin;
    const unsigned o = r.ok ? ch : 0u;
    if (p.x_split) {  // split rows: 4 heads + the same 4 tails in one register
#pragma unroll
      for (int i = 0; i < ASLOTS; ++i) {
        const _Float16 *xr = (const _Float16 *)(p.x + aoff[i]) + o;
        const u32x2 h = *(const u32x2 *)xr, t = *(const u32x2 *)(xr + Cin);
        r.v[i] = __builtin_bit_cast(f32x4, ((u32x4){h.x, h.y, t.x, t.y}));
      }
    } else {
#pragma unroll
      for (int i = 0; i < ASLOTS; ++i) r.v[i] = *(const f32x4 *)(p.x + aoff[i] + o);
    }
    ach += 32;
  };
  float amax = 0.f;
  auto storeA = [&](const ARaw &r, int buf) {
    _Float16 *dst = lds_a + buf * 2 * SP_AIMG;
#pragma unroll
    for (int i = 0; i < ASLOTS; ++i) {
      const int sr = sr0 + 64 * i;
      if (sr >= SR) continue;
      const int o = sp_off(sr, g8 >> 1) + (g8 & 1) * 4;
      if (p.x_split) {
        u32x4 b = __builtin_bit_cast(u32x4, r.v[i]);
        if (!r.ok) b = (u32x4){0u, 0u, 0u, 0u};
        *(u32x2 *)(dst + o) = (u32x2){b.x, b.y};
        *(u32x2 *)(dst + SP_AIMG + o) = (u32x2){b.z, b.w};
        continue;
      }
      const f32x4 v = sel4(r.ok, r.v[i]);
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      f16x4 h, t;
      split2h(v, h, t);
      *(f16x4 *)(dst + o) = h;
      *(f16x4 *)(dst + SP_AIMG + o) = t;
    }
  };

  // ---- B: item = (plane, row n, 16-B segment = 8 channels) -------------------------------
  const _Float16 *w16 = (const _Float16 *)G.w3;
  const _Float16 *bsrc[BSLOTS];
  int bdst[BSLOTS];
#pragma unroll
  for (int i = 0; i < BSLOTS; ++i) {
    const int idx = tid + NTHR * i, pl = idx >> 9, rem = idx & 511, nl = rem >> 2, seg = rem & 3;
    const int n = n0 + nl < G.N ? n0 + nl : G.N - 1;
    bsrc[i] = w16 + ((int64_t)pl * G.N + n) * G.Kpad + seg * 8;
    bdst[i] = pl * SP_BIMG + sp_off(nl, seg);
  }
  struct BRaw {
    u32x4 v[BSLOTS];
    bool ok;
  };
  int bj = 0, bc = 0;  // tap / chunk of the next B load
  auto loadB = [&](BRaw &rb) {
    const bool in = bc < nch;
    const int ch = (int)cbase + (in ? bc : nch - 1) * 32 + (tid & 3) * 8;
    rb.ok = ch < Cin;
    const int off = (in ? bj : k - 1) * Cin + (rb.ok ? ch - (tid & 3) * 8 : 0);
#pragma unroll
    for (int i = 0; i < BSLOTS; ++i) rb.v[i] = *(const u32x4 *)(bsrc[i] + off);
    if (++bj == k) {
      bj = 0;
      ++bc;
    }
  };
  auto storeB = [&](const BRaw &rb, int buf) {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < BSLOTS; ++i)
      *(u32x4 *)(lds_b + buf * 2 * SP_BIMG + bdst[i]) = rb.ok ? rb.v[i] : z;
  };

  unsigned vmask[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = m0 + wm * 64 + mi * 16 + fr;
    unsigned msk = 0;
    if (m >= 0 && m < p.M) {
      const int t = m % p.T;
      const int lo = max(pad - t, 0), hi = min(p.T - 1 + pad - t, k - 1);
      if (lo <= hi) msk = (2u << hi) - (1u << lo);
    }
    vmask[mi] = msk;
  }

  struct Frag {
    f16x8 ah[4], at[4], b0[4], b1[4];
  };
  auto read_frags = [&](Frag &f, int c, int j, int bbuf) {
    const _Float16 *Ab = lds_a + (c % SP_NBUF) * 2 * SP_AIMG;
    const _Float16 *Bb = lds_b + bbuf * 2 * SP_BIMG;
    // row wm 64 + mi 16 + fr + j: mi 16 changes neither the swizzle bit (row bit 2) nor
    // anything but the immediate, so one sp_off per step and a select per fragment (the
    // zero row as an offset from the same immediate): the same addresses
    const int o_j = sp_off(wm * 64 + fr + j, fs), o_z = sp_off(SL_ZROW, fs);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const bool ok = (vmask[mi] >> j) & 1u;
      const int o = (ok ? o_j : o_z - mi * 16 * SP_ROW) + mi * 16 * SP_ROW;
      f.ah[mi] = *(const f16x8 *)(Ab + o);
      f.at[mi] = *(const f16x8 *)(Ab + SP_AIMG + o);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int o = sp_off(wn * 64 + ni * 16 + fr, fs);
      f.b0[ni] = *(const f16x8 *)(Bb + o);
      f.b1[ni] = *(const f16x8 *)(Bb + SP_BIMG + o);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto mfma_frags = [&](const Frag &f) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const f16x8 bh = f.b0[ni] * (_Float16)(1.0f / H3_SCALE);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {  // small terms first
        f32x4 c = acc[mi][ni];
        c = mma16(f.at[mi], bh, c);
        c = mma16(f.ah[mi], f.b1[ni], c);
        c = mma16(f.ah[mi], f.b0[ni], c);
        acc[mi][ni] = c;
      }
    }
  };

  // ---- prologue: slab 0 (and 1 when k == 1), B steps 0 and 1; loads of B 2 / 3, slab next --
  if (tid < SP_NBUF * 2 * (SP_ROW / 8)) {  // the zero rows of every slab buffer and plane
    const int img = tid / (SP_ROW / 8), part = tid % (SP_ROW / 8);
    *(u32x4 *)(lds_a + img * SP_AIMG + SL_ZROW * SP_ROW + part * 8) = (u32x4){0u, 0u, 0u, 0u};
  }
  ARaw ra;
  BRaw rb0, rb1;
  loadA(ra);
  loadB(rb0);
  loadB(rb1);
  storeA(ra, 0);
  storeB(rb0, 0);
  storeB(rb1, 1);
  loadB(rb0);  // step 2
  loadB(rb1);  // step 3
  int next_a = 1;  // next chunk whose slab is stored (in iteration next_a * k - 2)
  if (nch > 1) {
    loadA(ra);
    if (k == 1) {
      storeA(ra, 1);
      next_a = 2;
      if (nch > 2) loadA(ra);
    }
  }
  __syncthreads();
  Frag f0, f1;
  read_frags(f0, 0, 0, 0);
  int c1 = k == 1 ? 1 : 0, j1 = k == 1 ? 0 : 1;  // chunk / tap of step s + 1
  auto iter = [&](int s, BRaw &rbs, Frag &cur, Frag &nxt) {
    if (s + 2 < nsteps) {
      storeB(rbs, (s + 2) % SP_NBUF);
      loadB(rbs);  // step s + 4 (clamped)
    }
    if (next_a < nch && s == next_a * k - 2) {
      storeA(ra, next_a % SP_NBUF);
      if (++next_a < nch) loadA(ra);
    }
    // fragments of step s + 1 (clamped at the end: a harmless re-read) under the MFMAs of s
    const bool more = s + 1 < nsteps;
    read_frags(nxt, more ? c1 : nch - 1, more ? j1 : k - 1, (more ? s + 1 : s) % SP_NBUF);
    mfma_frags(cur);
    __syncthreads();
    if (++j1 == k) {
      j1 = 0;
      ++c1;
    }
  };
  for (int s = 0; s < nsteps; s += 2) {
    iter(s, rb0, f0, f1);
    if (s + 1 >= nsteps) break;
    iter(s + 1, rb1, f1, f0);
  }
  bool bad = !(amax <= 65504.f);
  // colscale, range guard, then the tile through LDS (every wave is past its reads)
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col = n0 + wn * 64 + ni * 16 + fr;
    const float cs = G.colscale[col < G.N ? col : G.N - 1];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm * 64 + mi * 16 + 4 * fs + i;
        bad |= col < G.N && row < p.M && !__builtin_isfinite(acc[mi][ni][i]);
        acc[mi][ni][i] *= cs;
      }
  }
  float *tile = (float *)lds;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        tile[(wm * 64 + mi * 16 + 4 * fs + i) * SL_TP + wn * 64 + ni * 16 + fr] = acc[mi][ni][i];
  __syncthreads();
  if (bad && p.status) atomicOr(p.status, 1u);
  slab_epilogue<EPI, NTHR>(p, G, tile, m0, n0, tid);
}

// ---- conv bank walk: the pooled bank of a narrow input (the CBHG postnet: Cin = 80) -------
// The slab kernel gives every (group, column tile) its own block, so the c3 postnet bank ran
// 16 blocks per 255-row tile, each re-staging the same 80-channel slab and paying its own
// prologue and LDS-tile epilogue for 3 k steps of MFMAs (0.64-0.66 ms, 24 % of the f16x3
// ceiling).  Here one block owns a (255-row pooled tile, 128-column tile) and WALKS every group
// over a slab staged once: all 3 chunks of the input rows (f16 head / scaled tail, 101 KB) stay
// in LDS for the whole walk, the B planes of step s + 1 are staged under step s (2 buffers) and
// the group loop holds no epilogue state.  A group's epilogue works on the accumulators in
// registers: the maxpool's previous row is the lane 16 below (ds_bpermute), the block of 16
// rows above, or — for a wave's first row — the last row of the wave above through a 4 KB LDS
// halo; neighbouring column pairs are exchanged by DPP and byte-permuted so each lane stores
// 4 B of two columns.  Same MFMA order and operands as the slab kernel (bit-identical output).
// Measured (tools/bank_walk_ab.py, c3 postnet bank): 0.54 ms against the slab kernel's 0.64-0.65
// = 29 % of the ceiling; with no epilogue 0.43, with neither MFMAs nor epilogue 0.22 (the
// step skeleton: fragment reads, B staging, barrier) — the MFMAs do not overlap the skeleton.
// Not kept: fragment prefetch across steps (10 VGPR spills, 0.60 ms), two B register sets
// (0.59 ms), per-wave B fragments from L2 without LDS staging or per-step barriers (0.82 ms).  Limits: Cin <= 96, K <= 8, T >= 4, N % 128 == 0, groups k = K .. 1 heaviest
// first with pad k / 2.
constexpr int BW_MAXK = 8;
constexpr int BW_MAXCH = 3;                    // 32-channel chunks resident (Cin <= 96)
constexpr int BW_SR = SL_BM + BW_MAXK - 1;     // slab rows
constexpr int BW_ZROW = BW_SR;                 // the all-zero row (masked taps)
constexpr int BW_AIMG = (BW_SR + 1) * SP_ROW;  // halves per (chunk, plane) slab image
constexpr int BW_NBUF = 2;                     // B buffers

__global__ __launch_bounds__(512, 1) void conv_bank_walk_kernel(const GemmParams p) {
  constexpr int NTHR = 512;
  constexpr int BSLOTS = 1024 / NTHR;
  constexpr int NGRAN = BW_MAXCH * 8;                      // 4-channel granules per slab row
  constexpr int ASLOTS = (BW_SR * NGRAN + NTHR - 1) / NTHR;  // slab granules per thread
  __shared__ __attribute__((aligned(16))) _Float16 lds[BW_MAXCH * 2 * BW_AIMG + BW_NBUF * 2 * SP_BIMG];
  __shared__ float halo[2][4][SL_BN];  // [walk parity][wave row][column]: a wave's last row
  _Float16 *const lds_a = lds;
  _Float16 *const lds_b = lds + BW_MAXCH * 2 * BW_AIMG;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  constexpr int TS = SL_BM - 1;  // pooled rows a tile produces (row 0 is the halo row)
  const int MT = (p.M + TS - 1) / TS, NT = p.g[0].ntiles;
  int mt, nt;
  slab_tile(blockIdx.x, MT, NT, 0, mt, nt);  // a row tile's column tiles on one XCD
  if (mt >= MT) return;                      // the grid is padded to whole XCD rounds
  const int m0 = mt * TS - 1, n0 = nt * SL_BN;
  const int Cin = p.Cin, nch = (Cin + 31) / 32, NG = p.ngroups, N = p.g[0].N;
  const int PMAX = NG / 2;  // the heaviest group's halo: slab row 0 = input row m0 - PMAX
#ifdef FTMI_DIAG
  // timing experiments (FTMI_SLAB_DIAG, results invalid): bit 0 = every B load from the first
  // step's (L2-hot) lines, bit 1 = no MFMAs, bit 2 = no epilogue (finish / stores),
  // bit 3 = no epilogue stores (split rows)
  const int diag = p.diag;
#else
  constexpr int diag = 0;
#endif
  // Group g has k = NG - g taps (pad k / 2); its f16x3 block (ftmi_split_weights_f16 layout:
  // 3 planes [N][Kpad], then N column scales, 16-B padded) sits right before group g - 1's, the
  // BN affine at (k - 1) N — all arithmetic, so the walk issues no scalar loads per step (their
  // waits would also drain the LDS reads); bank_walk_ok checks the layout on the host.
  auto kpad = [&](int k) { return (k * Cin + 31) & ~31; };
  auto block_bytes = [&](int k) { return (int64_t)6 * N * kpad(k) + ((4 * N + 15) & ~15); };
  const char *const wblk0 = (const char *)p.g[0].w3;
  const float *const bnsc = p.g[NG - 1].scale, *const bnsh = p.g[NG - 1].shift;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int fr = lane & 15, fs = lane >> 4;

  // ---- the slab, once: item = (slab row, 4-channel granule); channels >= Cin are zero ----
  const int SR = SL_BM + NG - 1;
  float amax = 0.f;
  {
    f32x4 v[ASLOTS];
#pragma unroll
    for (int i = 0; i < ASLOTS; ++i) {
      const int it = tid + NTHR * i, sr = it / NGRAN, q = it - sr * NGRAN;
      int mp = m0 - PMAX + sr;
      mp = mp < 0 ? 0 : (mp >= p.M ? p.M - 1 : mp);  // clamped rows only feed masked taps
      const bool ok = sr < SR && q * 4 < Cin;
      v[i] = ok ? *(const f32x4 *)(p.x + (int64_t)mp * p.x_stride + q * 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < ASLOTS; ++i) {
      const int it = tid + NTHR * i, sr = it / NGRAN, q = it - sr * NGRAN;
      if (sr >= SR) continue;
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
      f16x4 h, t;
      split2h(v[i], h, t);
      _Float16 *dst = lds_a + (q >> 3) * 2 * BW_AIMG + sp_off(sr, (q & 7) >> 1) + (q & 1) * 4;
      *(f16x4 *)dst = h;
      *(f16x4 *)(dst + BW_AIMG) = t;
    }
    if (tid < BW_MAXCH * 2 * (SP_ROW / 8)) {  // the zero row of every chunk and plane
      const int img = tid / (SP_ROW / 8), part = tid % (SP_ROW / 8);
      *(u32x4 *)(lds_a + img * BW_AIMG + BW_ZROW * SP_ROW + part * 8) = (u32x4){0u, 0u, 0u, 0u};
    }
  }

  // ---- B: item = (plane, row n, 16-B segment); the walk's steps are (group, chunk, tap) ----
  int bdst[BSLOTS], brow[BSLOTS];
#pragma unroll
  for (int i = 0; i < BSLOTS; ++i) {
    const int idx = tid + NTHR * i, pl = idx >> 9, rem = idx & 511, nl = rem >> 2, seg = rem & 3;
    const int n = n0 + nl < N ? n0 + nl : N - 1;
    brow[i] = pl * N + n;
    bdst[i] = pl * SP_BIMG + sp_off(nl, seg);
  }
  struct BRaw {
    u32x4 v[BSLOTS];
    bool ok;
  };
  // The walk order k0, k0 - 1, .., 1, NG, .., k0 + 1 with k0 rotating over the blocks of an
  // XCD: blocks that run together reach their epilogues (130 KB of stores each, drained before
  // the next B staging: the loads wait on the same counter) at different times instead of
  // all at once.  Any order gives the same bits (each group owns its accumulators).
  const int k0 = NG - (int)((blockIdx.x >> 3) % NG);
  const char *wk0 = wblk0;
  for (int k = NG - 1; k >= k0; --k) wk0 -= block_bytes(k);
  int bk = k0, bc = 0, bj = 0, bn = 0;  // taps (group) / chunk / tap of the next B load, groups done
  const char *bw = wk0;                  // that group's block
  auto loadB = [&](BRaw &rb) {           // past the last step: a harmless re-read
    rb.ok = bc * 32 + (tid & 3) * 8 < Cin;
    const _Float16 *w16 = (const _Float16 *)((diag & 1) ? wblk0 : bw) +
                          ((diag & 1) ? 0 : bj * Cin + (rb.ok ? bc * 32 : 0)) + (tid & 3) * 8;
    const int kp = kpad(bk);
#pragma unroll
    for (int i = 0; i < BSLOTS; ++i) rb.v[i] = *(const u32x4 *)(w16 + (int64_t)brow[i] * kp);
    if (bn < NG && ++bj == bk) {
      bj = 0;
      if (++bc == nch) {
        bc = 0;
        ++bn;
        if (bk == 1) {
          bk = NG;
          bw = wblk0;
        } else {
          bw -= block_bytes(--bk);
        }
      }
    }
  };
  auto storeB = [&](const BRaw &rb, int buf) {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < BSLOTS; ++i)
      *(u32x4 *)(lds_b + buf * 2 * SP_BIMG + bdst[i]) = rb.ok ? rb.v[i] : z;
  };

  // rows of this lane's A fragments: in range, and their frame within the sequence
  int tfr[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = m0 + wm * 64 + mi * 16 + fr;
    // rows outside [0, M) get a frame no tap offset brings into [0, T): one unsigned compare
    tfr[mi] = m >= 0 && m < p.M ? m % p.T : -(1 << 20);
  }
  struct Frag {
    f16x8 ah[4], at[4], b0[4], b1[4];
  };
  auto read_frags = [&](Frag &f, int k, int c, int j, int bbuf) {
    const int d = j - k / 2;  // the tap's row offset
    const _Float16 *Ab = lds_a + c * 2 * BW_AIMG;
    const _Float16 *Bb = lds_b + bbuf * 2 * SP_BIMG;
    // one sp_off per step, a select per fragment (the slabp kernel's form: same addresses)
    const int o_d = sp_off(wm * 64 + fr + d + PMAX, fs), o_z = sp_off(BW_ZROW, fs);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const bool ok = (unsigned)(tfr[mi] + d) < (unsigned)p.T;
      const int o = (ok ? o_d : o_z - mi * 16 * SP_ROW) + mi * 16 * SP_ROW;
      f.ah[mi] = *(const f16x8 *)(Ab + o);
      f.at[mi] = *(const f16x8 *)(Ab + BW_AIMG + o);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int o = sp_off(wn * 64 + ni * 16 + fr, fs);
      f.b0[ni] = *(const f16x8 *)(Bb + o);
      f.b1[ni] = *(const f16x8 *)(Bb + SP_BIMG + o);
    }
  };
  f32x4 acc[4][4];
  auto zero_acc = [&] {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  auto mfma_frags = [&](const Frag &f) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const f16x8 bh = f.b0[ni] * (_Float16)(1.0f / H3_SCALE);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {  // small terms first (the slab kernel's order)
        f32x4 c = acc[mi][ni];
        c = mma16(f.at[mi], bh, c);
        c = mma16(f.ah[mi], f.b1[ni], c);
        c = mma16(f.ah[mi], f.b0[ni], c);
        acc[mi][ni] = c;
      }
    }
  };

  // ---- a group's epilogue (VALU-lean: a wave64 VALU op costs 4 cycles, the epilogue runs 8
  // times per block; the first form, ~3,100 instructions, cost 7 us per group) ---------------
  // Per lane: frame of its first output row of block mi (row -1, tile 0's halo row, as frame
  // T - 1 so that row 0 is a sequence start), and bit 4 mi + i = row 4 fs + i of block mi is
  // stored (not the halo row, inside [0, M)).  Rows outside [0, M) hold exact zeros and the
  // clamped columns do not exist (N % 128 == 0), so the range guards need no masks.
  int tst[4];
  unsigned vrow = 0;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int R = wm * 64 + mi * 16 + 4 * fs, r = m0 + R;
    tst[mi] = r >= 0 ? r % p.T : p.T - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) vrow |= (unsigned)(R + i > 0 && r + i < p.M) << (4 * mi + i);
  }
  // part 1 (before a barrier): colscale, range guard, ReLU / BN in place, and the wave's last
  // row into the halo
  float nf = 0.f;  // NaN once an accumulator was not finite (x * 0 + nf)
  auto finish = [&](const float (&cs)[4], const float (&sc)[4], const float (&sh)[4], int par) {
    // opaque copies: without them LICM hoists the epilogue's group-invariant row / column
    // terms out of the walk and keeps them live across it (256 VGPRs + spills)
    int ln = lane, wv = wave;
    asm volatile("" : "+v"(ln), "+s"(wv));
    const int efr = ln & 15, efs = ln >> 4, ewm = wv & 3, ewn = wv >> 2;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          nf = fmaf(acc[mi][ni][i], 0.f, nf);
          float v = acc[mi][ni][i] * cs[ni];  // (a bank has no bias: bank_walk_ok)
          if (p.relu) v = fmaxf(v, 0.f);
          if (bnsc) v = v * sc[ni] + sh[ni];
          acc[mi][ni][i] = v;
        }
      if (efs == 3) halo[par][ewm][ewn * 64 + ni * 16 + efr] = acc[3][ni][3];
    }
  };
  // part 2 (after the barrier): y[t] = max(v[t - 1], v[t]) within a sequence, stored
  float ymax = 0.f;
  auto store_pooled = [&](int k, int par) {
    int ln = lane, wv = wave, mb = m0;
    asm volatile("" : "+v"(ln), "+s"(wv), "+s"(mb));
    const int efr = ln & 15, efs = ln >> 4, ewm = wv & 3, ewn = wv >> 2;
    const int ycol0 = (k - 1) * N, cw = n0 + ewn * 64;  // the wave's first column
    const bool ev = (efr & 1) == 0;
    float up[4];  // per ni: row 15 of the block above (lanes fs = 0 take it)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) up[ni] = ewm > 0 ? halo[par][ewm - 1][ewn * 64 + ni * 16 + efr] : 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      // the sequence start among the lane's 4 rows (T >= 4: at most one): position 0..3, or 4
      const int zp = tst[mi] ? p.T - tst[mi] : 0;
      bool st[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) st[i] = zp == i;
      f32x4 o[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float s3 = __shfl(acc[mi][ni][3], (ln - 16) & 63);
        const float prev0 = efs ? s3 : up[ni];
        up[ni] = s3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = acc[mi][ni][i], pv = i ? acc[mi][ni][i - 1] : prev0;
          o[ni][i] = st[i] ? a : fmaxf(a, pv);
          ymax = fmaxf(ymax, fabsf(o[ni][i]));
        }
      }
      const int R0 = ewm * 64 + mi * 16 + 4 * efs;
      if (p.y_split_c) {
        // column pairs (fr even: rows 0 / 1 of columns fr, fr + 1; fr odd: rows 2 / 3 of
        // fr - 1, fr): each lane sends its partner the word the partner stores (DPP lane ^ 1),
        // then two byte permutes build its own rows, the even column's half first
        unsigned hw[2][4], tw[2][4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          f16x4 h, tl;
          split2h(o[ni], h, tl);
          const u32x2 hb = __builtin_bit_cast(u32x2, h), tb = __builtin_bit_cast(u32x2, tl);
          const unsigned hx = __builtin_amdgcn_mov_dpp(ev ? hb.y : hb.x, 0xB1, 0xF, 0xF, false);
          const unsigned tx = __builtin_amdgcn_mov_dpp(ev ? tb.y : tb.x, 0xB1, 0xF, 0xF, false);
          const unsigned ha = ev ? hb.x : hx, hbv = ev ? hx : hb.y;
          const unsigned ta = ev ? tb.x : tx, tbv = ev ? tx : tb.y;
          hw[0][ni] = __builtin_amdgcn_perm(hbv, ha, 0x05040100u);
          hw[1][ni] = __builtin_amdgcn_perm(hbv, ha, 0x07060302u);
          tw[0][ni] = __builtin_amdgcn_perm(tbv, ta, 0x05040100u);
          tw[1][ni] = __builtin_amdgcn_perm(tbv, ta, 0x07060302u);
        }
        const int ra = ev ? 0 : 2;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (!((vrow >> (4 * mi + ra + q)) & 1u)) continue;
          _Float16 *yr = (_Float16 *)(p.y + (int64_t)(mb + R0 + ra + q) * p.y_stride) + ycol0 + cw +
                         (efr & ~1);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            if (diag & 8) continue;
            *(unsigned *)(yr + ni * 16) = hw[q][ni];
            *(unsigned *)(yr + p.y_split_c + ni * 16) = tw[q][ni];
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (!((vrow >> (4 * mi + i)) & 1u)) continue;
          float *yr = p.y + (int64_t)(mb + R0 + i) * p.y_stride + ycol0 + cw + efr;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) yr[ni * 16] = o[ni][i];
        }
      }
    }
  };

  // ---- the walk: groups, each c outer / j inner as the slab kernel -------------------------
  // Step s (global over the walk) reads B buffer s & 1, stored in step s - 1 from registers
  // loaded in step s - 2; its fragments are read at the step's top (the other wave of the SIMD
  // covers that wait with its MFMAs).  The epilogue sits between the groups' step loops, so
  // none of its values is live in them; the group's column scales and BN affine are loaded
  // before its steps.
  const int S = nch * NG * (NG + 1) / 2;
  BRaw rb;
  loadB(rb);
  storeB(rb, 0);
  loadB(rb);  // step 1
  __syncthreads();
  int s = 0, kc = k0;
  const char *ew = wk0;  // the group's block
  for (int gn = 0; gn < NG; ++gn) {
    float cs[4], sc[4], sh[4];
    {
      const float *colscale = (const float *)(ew + (int64_t)6 * N * kpad(kc));
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int cc = n0 + wn * 64 + ni * 16 + fr;
        cs[ni] = colscale[cc];
        sc[ni] = bnsc ? bnsc[(kc - 1) * N + cc] : 1.f;
        sh[ni] = bnsc ? bnsh[(kc - 1) * N + cc] : 0.f;
      }
    }
    const int ng = nch * kc;
    int u = 0, c = 0, j = 0;
    auto step = [&](BRaw &rs) {  // rs holds B(s + 1)
      Frag f;
      read_frags(f, kc, c, j, s & 1);
      if (s + 1 < S) {
        storeB(rs, (s + 1) & 1);
        loadB(rs);  // step s + 2 (clamped)
      }
      if (!(diag & 2)) mfma_frags(f);
      __syncthreads();
      ++s;
      ++u;
      if (++j == kc) {
        j = 0;
        ++c;
      }
    };
    while (u < ng) step(rb);
    if (!(diag & 4)) finish(cs, sc, sh, gn & 1);
    __syncthreads();  // the halo
    if (!(diag & 4)) store_pooled(kc, gn & 1);
    zero_acc();
    if (kc == 1) {
      kc = NG;
      ew = wblk0;
    } else {
      ew -= block_bytes(--kc);
    }
  }
  const bool bad = nf != 0.f || !(amax <= 65504.f) || (p.y_split_c && !(ymax <= 65504.f));
  if (bad && p.status) atomicOr(p.status, 1u);
}

// ---- skinny kernel: few output rows (M <= SK_MMAX, e.g. batch 1), the weight stream binds --
// At B = 1 (BASELINE config c2: T = 120 phonemes) a conv moves its whole weight block for a
// handful of rows: the prenet bank reads 35.65 MB of weight planes for 120 x 4096 outputs, so
// the bound is HBM, not MFMA.  Work unit = (128-row tile, group, 64 output columns, two
// 32-channel chunks): the block stages the rows of its chunks ONCE into an f16 head / scaled
// tail slab (the slab kernel's layout, taps read shifted rows, masked taps a zero row), then
// every wave streams the f16 weight planes of ITS 16 columns straight from HBM into
// registers (no LDS, no barrier after the prologue, 4 steps of prefetch) and multiplies them
// against the slab: 3 f16 MFMAs per fp32 product (f16x3, as the slab kernel).  Channel
// chunks beyond the block's two go to other blocks (blockIdx.y): their raw partial sums land
// in part[s][M][ldp] (output-column order) and skinny_finish_kernel adds them in split order
// (deterministic) and applies the epilogue; with one split the wave finishes its columns.
#ifndef SKINNY_PF
#define SKINNY_PF 4
#endif
constexpr int SK_BM = 128;
constexpr int SK_BN = 64;   // 4 column sets of 16 (x 2 step halves = 8 waves)
constexpr int SK_CPB = 2;   // 32-channel chunks per block
constexpr int SK_SR = SK_BM + SL_MAXK - 1;
constexpr int SK_ZROW = SK_SR;
constexpr int SK_AIMG = (SK_SR + 1) * SL_P;  // halves per (chunk, plane) slab image
constexpr int SK_MMAX = 256;
constexpr int SK_MMAX_NARROW = 1024;
constexpr int SK_PF = SKINNY_PF;  // weight-fragment prefetch depth (steps)

// BANK = the balanced schedule of a CBHG conv bank (groups k = K .. 1 in g[0 .. K-1], equal
// widths, K even): a block takes two 16-column sets of the group pair (k, K + 1 - k) — four
// (group, column set) units — and the 8 waves pair them so that each SIMD runs one unit of
// each group of the pair (waves w and w + 4 share a SIMD): every SIMD, and every block,
// streams (K + 1) / 2 of the average weight bytes, instead of blocks of the k = K group
// moving K times the bytes of the k = 1 group's.  The slab is the heavier group's (its halo
// covers the lighter group's taps, read at a row offset).
#ifdef FTMI_SKINNY_STAMPS
// diagnostic build only: per-block s_memtime at phase boundaries (wave 0 and wave 7)
__device__ unsigned long long ftmi_skinny_stamps[4096 * 8];
#define SKSTAMP(i)                                                                         \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x == 0 || threadIdx.x == 448)) {             \
      __builtin_amdgcn_sched_barrier(0);                                                   \
      ftmi_skinny_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (threadIdx.x ? 4 : 0) + \
                         (i)] = __builtin_amdgcn_s_memtime();                              \
      __builtin_amdgcn_sched_barrier(0);                                                   \
    }                                                                                      \
  } while (0)
#else
#define SKSTAMP(i) \
  do {             \
  } while (0)
#endif

// DIAG (timing experiments only, FTMI_SKINNY_DIAG on the bank schedule; results invalid):
// bit 0 = the A fragments read once before the loop (no LDS reads in it), bit 1 = no MFMAs
// (the loaded weights feed one VALU add), bit 2 = every weight load from one L2-hot line.
// Instantiated only in the diagnostic build (-DFTMI_DIAG, libftmi_stamps.so).
// NM (one sequence in the rows, B = 1: c2): no tap masks — the slab rows outside the sequence
// are staged as zeros (conv_bank_halves_kernel's mask-free form; bit-identical).
template <bool MAXPOOL, bool BANK = false, int DIAG = 0, bool NM = false>
__global__ __launch_bounds__(512, 1) void conv_gemm_skinny_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[SK_CPB * 2 * SK_AIMG];
  SKSTAMP(0);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int MT = (p.M + SK_BM - 1) / SK_BM, NT = p.g[0].ntiles;
  // consecutive blocks: row tiles, then column blocks of the heaviest group first; a
  // compact grid, so consecutive blocks land on different XCDs
  const int bid = blockIdx.x, mt = bid % MT, v = bid / MT;
  int gi, nt;
  if constexpr (BANK) {  // v = (pair, two column sets): pair-units 2v, 2v + 1
    const int NC = p.g[0].N / 16;
    gi = (2 * v) / NC;  // the pair's heavier group (k = K - gi)
    nt = (2 * v) % NC;  // first of the block's two 16-column sets
  } else {
    gi = v / NT;
    nt = v - gi * NT;
  }
  const GemmGroup &G = p.g[gi];
  const int m0 = mt * SK_BM, k = G.k, pad = G.pad, Cin = p.Cin;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;
  const int nch_all = (Cin + 31) / 32;
  const int c_begin = blockIdx.y * p.kc_per;
  const int nch = min(nch_all - c_begin, p.kc_per);  // >= 1 (no empty splits)

  // ---- prologue: the slab of this block's chunks (one float4 of 4 channels per item); every
  // load is issued before the first split / store, so their latencies overlap.  Item = (row
  // chunk r = (tid >> 3) + 64 i = c SK_SR + sr, channel segment tid & 7): the slab always has
  // SK_SR rows (rows past this group's BM + k - 1 are staged and never read), so the indexing
  // divides by constants only, and every load is unconditional (clamped; a load inside a
  // branch makes the compiler wait for it there — conv_bank_halves_kernel's finding).
  // Channels past Cin read a valid clamped address: their weights are zeroed at use. ----
  constexpr int SK_ASLOTS = (SK_CPB * SK_SR + 63) / 64;
  const int seg = tid & 7;
  f32x4 av[SK_ASLOTS], au[MAXPOOL ? SK_ASLOTS : 1];
#pragma unroll
  for (int i = 0; i < SK_ASLOTS; ++i) {
    const int r = min((tid >> 3) + 64 * i, nch * SK_SR - 1), c = r / SK_SR, sr = r - c * SK_SR;
    const int ch0 = (c_begin + c) * 32 + seg * 4, ch = ch0 < Cin ? ch0 : 0;
    int m = m0 - pad + sr;
    const bool inseq = m >= 0 && m < p.M;
    m = m < 0 ? 0 : (m >= p.M ? p.M - 1 : m);  // clamped rows only feed masked taps
    const float *src = p.x + (int64_t)m * p.x_stride + ch;
    av[i] = *(const f32x4 *)src;
    // CBHG maxpool(2, 1) fused: max(x[t - 1], x[t]); x[0] at t = 0
    if constexpr (MAXPOOL) au[i] = *(const f32x4 *)(src - (m % p.T > 0 ? p.x_stride : 0));
    if constexpr (NM) {  // the zero padding itself (the pooled padding is zero too)
      av[i] = inseq ? av[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (MAXPOOL) au[i] = inseq ? au[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < SK_ASLOTS; ++i) {
    const int r = (tid >> 3) + 64 * i, c = r / SK_SR, sr = r - c * SK_SR;
    if (r >= nch * SK_SR) break;
    f32x4 x = av[i];
    if ((c_begin + c) * 32 + seg * 4 >= Cin) x = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (MAXPOOL) x = fmax4(x, au[i]);
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
    f16x4 h, t;
    split2h(x, h, t);
    _Float16 *dst = lds + c * 2 * SK_AIMG + sr * SL_P + seg * 4;
    *(f16x4 *)dst = h;
    *(f16x4 *)(dst + SK_AIMG) = t;
  }
  if (tid < SK_CPB * 2 * (SL_P / 8)) {  // the zero row of every (chunk, plane) image
    const int img = tid / (SL_P / 8), part = tid % (SL_P / 8);
    *(u32x4 *)(lds + img * SK_AIMG + SK_ZROW * SL_P + part * 8) = (u32x4){0u, 0u, 0u, 0u};
  }
  __syncthreads();
  SKSTAMP(1);
  bool bad = !(amax <= 65504.f);

  // 8 waves: wave w multiplies columns col0 + [0, 16) (column set w & 3) over one half of
  // the steps (w >> 2); the two halves meet in LDS after the loop.  BANK: unit slot cw =
  // (group of the pair: w >> 2, column set: (w >> 1) & 1), half w & 1
  int cw, half, gw, col0;
  if constexpr (BANK) {
    cw = ((wave >> 2) << 1) | ((wave >> 1) & 1);
    half = wave & 1;
    gw = (wave >> 2) ? p.ngroups - 1 - gi : gi;
    col0 = (nt + ((wave >> 1) & 1)) * 16;
  } else {
    cw = wave & 3;
    half = wave >> 2;
    gw = gi;
    col0 = nt * SK_BN + cw * 16;  // this wave's 16 columns of group gi
  }
  gw = __builtin_amdgcn_readfirstlane(gw);
  const GemmGroup &GW = p.g[gw];
  const int kw = GW.k, padw = GW.pad, dp = pad - padw;  // slab row offset of this group's taps
  const int nsteps = nch * kw, hs = (nsteps + 1) / 2;
  const int s_begin = half ? hs : 0, s_end = half ? nsteps : hs;
  // the epilogue's per-column parameters, requested now: their latency hides under the
  // weight stream instead of opening the tail
  const int ecol = col0 + fr < GW.N ? col0 + fr : GW.N - 1;
  const bool fin = !half && col0 < GW.N;
  const bool direct = !(p.split > 1 || p.force_part);
  const float e_cs = fin ? GW.colscale[ecol] : 1.f;
  const float e_bias = fin && direct && GW.bias ? GW.bias[ecol] : 0.f;
  const float e_sc = fin && direct && GW.scale ? GW.scale[ecol] : 1.f;
  const float e_sh = fin && direct && GW.scale ? GW.shift[ecol] : 0.f;
  f32x4 acc[8];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) acc[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (col0 < GW.N && s_end > s_begin) {  // wave-uniform; no barrier inside
    // per-row tap masks: bit j set iff frame t + j - pad lies inside the sequence
    unsigned vmask[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = m0 + mi * 16 + fr;
      unsigned msk = 0;
      if (m < p.M) {
        const int t = m % p.T;
        const int lo = max(padw - t, 0), hi = min(p.T - 1 + padw - t, kw - 1);
        if (lo <= hi) msk = (2u << hi) - (1u << lo);
      }
      vmask[mi] = msk;
    }
    // weight planes B0 = 2^11 w_h, B1 = w_t of column n, taps j, channels of step s
    const int n = col0 + fr < GW.N ? col0 + fr : GW.N - 1;
    const _Float16 *w0 = (const _Float16 *)GW.w3 + (int64_t)n * GW.Kpad;
    const int64_t plane = (int64_t)GW.N * GW.Kpad;
    // step s = (tap j = s / nch, chunk c = s % nch): the chunks of one tap are adjacent
    // 64-B pieces of a weight row, so consecutive steps read whole 128-B lines
    // Loads are unconditional (a missing channel segment of a partial chunk reads channel 0
    // and is zeroed at use): a select on a loaded value would force a wait at the load.
    auto loadB = [&](int s, f16x8 &b0, f16x8 &b1) {
      const int j = nch == 2 ? s >> 1 : s, c = s - j * nch;  // nch is 1 or 2 (SK_CPB)
      const int ch = (c_begin + c) * 32 + fs * 8;
      const int off = (DIAG & 4) ? fs * 8 : j * Cin + (ch < Cin ? ch : 0);  // Cin % 16 == 0
      b0 = *(const f16x8 *)(w0 + off);
      b1 = *(const f16x8 *)(w0 + plane + off);
    };
    // Every step issues exactly one (clamped) weight load pair and the loop body has no
    // branch at all; a step's 16 A fragments are read from the slab before its 24 MFMAs.
    // (Measured alternatives, c2 prenet bank / proj1: the loop fully unrolled with exact
    // per-step vmcnt waits 21.7 / 18.5 us, an 8-step ring 23.5 / 20.6, against 21.1 / 15.8
    // for this form: the waves are not bound by the weight-load latency alone.)
    f16x8 rb0[SK_PF], rb1[SK_PF];
    f16x8 dh[(DIAG & 1) ? 8 : 1], dt[(DIAG & 1) ? 8 : 1];
    if constexpr (DIAG & 1) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        dh[mi] = *(const f16x8 *)(lds + (mi * 16 + fr) * SL_P + fs * 8);
        dt[mi] = *(const f16x8 *)(lds + SK_AIMG + (mi * 16 + fr) * SL_P + fs * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < SK_PF; ++u) loadB(min(s_begin + u, s_end - 1), rb0[u], rb1[u]);
    for (int s0 = s_begin; s0 < s_end; s0 += SK_PF) {
#pragma unroll
      for (int u = 0; u < SK_PF; ++u) {
        const int s = s0 + u;
        {  // steps past the end (nsteps rounded up to SK_PF) multiply zeros: no branch
          const int sl = min(s, s_end - 1), j = nch == 2 ? sl >> 1 : sl, c = sl - j * nch;
          const _Float16 *Ab = lds + c * 2 * SK_AIMG;
          f16x8 ah[8], at[8];
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
            if constexpr (DIAG & 1) {
              ah[mi] = dh[mi];
              at[mi] = dt[mi];
            } else {
              // the slab kernel's multiply-free address form (same addresses)
              const bool ok = NM || ((vmask[mi] >> j) & 1u) != 0;
              const int o = (ok ? fr * SL_P + fs * 8 + (j + dp) * SL_P
                                : SK_ZROW * SL_P + fs * 8 - mi * 16 * SL_P) + mi * 16 * SL_P;
              ah[mi] = *(const f16x8 *)(Ab + o);
              at[mi] = *(const f16x8 *)(Ab + SK_AIMG + o);
            }
          }
          const f16x8 z = {};
          const bool bok = s < s_end && (c_begin + c) * 32 + fs * 8 < Cin;
          const f16x8 b0 = bok ? rb0[u] : z, b1 = bok ? rb1[u] : z;
          const f16x8 bh = b0 * (_Float16)(1.0f / H3_SCALE);
          if constexpr (DIAG & 2) {
            acc[0][0] += (float)bh[0] + (float)b1[0] + (float)ah[u & 7][0] + (float)at[u & 7][0];
          } else {
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) acc[mi] = mma16(at[mi], bh, acc[mi]);  // small terms first
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) acc[mi] = mma16(ah[mi], b1, acc[mi]);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) acc[mi] = mma16(ah[mi], b0, acc[mi]);
          }
        }
        // refill the slot in place (a copy of a pending load would wait for it)
        loadB(min(s + SK_PF, s_end - 1), rb0[u], rb1[u]);
      }
    }
  }
  SKSTAMP(2);
  // the second half's sums join the first half's through LDS (the slab is dead by then)
  __syncthreads();
  f32x4 *red = (f32x4 *)lds;  // [column set][mi][lane]
  if (half) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) red[(cw * 8 + mi) * 64 + lane] = acc[mi];
  }
  __syncthreads();
  if (!half && col0 < GW.N) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) acc[mi] += red[(cw * 8 + mi) * 64 + lane];
    // lane (fr, fs) holds rows mi*16 + 4 fs + i of column col0 + fr
    const int col = col0 + fr;
    const bool cok = col < GW.N;
    const float cs = e_cs;
    if (!direct) {
      float *part = p.part + (size_t)blockIdx.y * p.M * p.ldp + GW.ycol0;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + mi * 16 + 4 * fs + i;
          if (cok && row < p.M) {
            bad |= !__builtin_isfinite(acc[mi][i]);
            part[(size_t)row * p.ldp + col] = acc[mi][i] * cs;
          }
        }
    } else {
      const float bias = e_bias, sc = e_sc, sh = e_sh;  // (unused for !cok columns)
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + mi * 16 + 4 * fs + i;
          if (!cok || row >= p.M) continue;
          bad |= !__builtin_isfinite(acc[mi][i]);
          float y = acc[mi][i] * cs + bias;
          if (p.relu) y = fmaxf(y, 0.f);
          if (GW.scale) y = y * sc + sh;
          if (p.residual) y += p.residual[(int64_t)row * p.res_stride + col];
          if (p.y) p.y[(int64_t)row * p.y_stride + GW.ycol0 + col] = y;
          if (p.yt) {
            const int b = row / p.To, t = row - b * p.To;
            p.yt[((int64_t)b * p.yt_channels + GW.ycol0 + col) * p.To + t] = y;
          }
        }
    }
  }
  SKSTAMP(3);
  if (bad && p.status) atomicOr(p.status, 1u);
}

// ---- the c2 conv bank in one launch: channel halves + pairwise last-arriver finish ------
// (FTMI_BANK_HALVES; common_layers.py:67-71,92-97 at B = 1, T = 120, K = 16, Cin = 256)
// What bounds this bank is how fast each CU pulls its share of the 35.65 MB of weight
// planes, and the fixed costs around that stream (tools/probe_stream.hip, warm: the bank's
// access pattern with every load of a wave issued up front 6.3 us per launch, with a 4-step
// ring 10.0 us, an empty launch 3.1 us).  So:
//  * a block = (group pair (k, K + 1 - k), one 16-column set of each group, one HALF of the
//    input channels): 8 x 16 x 2 = 256 blocks, one per CU, each streaming (K + 1) taps x
//    Cin / 2 channels x 16 columns x 2 planes = 139 KB; the two halves of a unit are blocks
//    b and b + 8 (one XCD under round-robin dispatch: placement only ever affects speed);
//  * every wave issues ALL its weight loads at once, right after its slab loads: the whole
//    139 KB of a CU is in flight from the start and the MFMAs consume the steps as they land
//    (in-order vmcnt), instead of a ring refilled one step at a time;
//  * the slab holds only the block's channel half (Cin / 2 x (RM + K - 1) rows, f16 head /
//    scaled tail, the skinny kernel's layout and tap masks);
//  * the 8 waves split the unit's 4 (K + 1) (group, tap, chunk) steps round-robin and meet
//    in LDS in wave order; the two halves meet through memory: both write their sums
//    write-through (16-B sc1 stores, fragment order); each wave waits for its own stores and
//    bumps its slice's counter (agent-scope atomic, 8 per unit); the wave whose add returns
//    1 resets the counter, reads its partner wave's sums (16-B sc1 loads), adds them to its
//    own (a + b == b + a: deterministic whichever half arrives last) and applies colscale,
//    ReLU and the BN affine (MI355X_MICROARCH.md "Valid forms", the first row of the sc1
//    table, at wave granularity).  No split partials for a finish launch, no second launch.
constexpr int BH_MAXCH = 4;  // 32-channel chunks per half: Cin <= 256

#ifdef FTMI_SKINNY_STAMPS
// diagnostic build only: per-block s_memtime at phase boundaries (tid 0 = wave 0, tid 448 =
// wave 7): [0] start, [1] slab staged, [2] wave 0's loop done, [3] wave 7's loop done,
// [4] the waves' sums reduced, [5] published + counted, [6] end (wave 0), [7] end (wave 7)
#define BHSTAMP(i, t)                                                                       \
  do {                                                                                      \
    if (threadIdx.x == (t)) {                                                               \
      __builtin_amdgcn_sched_barrier(0);                                                    \
      ftmi_skinny_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();              \
      __builtin_amdgcn_sched_barrier(0);                                                    \
    }                                                                                       \
  } while (0)
#else
#define BHSTAMP(i, t) \
  do {                \
  } while (0)
#endif

// DIAG (timing experiments only, FTMI_BANK_HALVES_DIAG; results invalid): bit 0 = no MFMAs
// (the loaded weights feed one VALU add), bit 1 = no A-fragment LDS reads (fixed fragments),
// bit 2 = no partner exchange (each block stores its own half's sums as the output), bit 4 =
// no weight loads, bit 3 = the same weight bytes per block read as 1 KB contiguous runs from
// the start of the split-weight buffer (c2 prenet: 256 x 139 KB of its 53 MB; results
// invalid), bit 5 = every weight load before the slab wait, bit 6 = a step's 8 row
// fragments read at once instead of in two blocks of 4, bit 7 = every weight load up front
// behind a workgroup barrier after the slab loads' issue, bits 8 / 9 = the first 2 / 4 steps'
// weight loads before the slab wait instead of 6 (bits 5-9: valid results)
//
// Address arithmetic is compile-time wherever it can be (measured with the phase stamps of a
// first version: the slab staging took ~12 k cycles with NO weight loads at all — ~1,300
// instructions per wave, most of them integer divisions by the runtime slab height and chunk
// count — against ~3 k for the same loads in tools/probe_slab.hip): NCH (32-channel chunks
// per half) is a template parameter, the slab always holds RM + 15 rows (a lighter pair's
// extra rows are staged and never read), a thread's slab items share one channel segment
// (tid & 7), and the tap masks step through the rows without a division per row.
//
// Kernel arguments live in memory the first load of a launch misses in every cache, so a
// chain of DEPENDENT argument loads (N -> the block's group -> that group's pointers) costs
// a round trip each before the first data load can issue: KT (groups) and NCT (16-column sets
// per group) are template parameters for the c2 prenet bank (16, 16), so a block's group
// index comes from blockIdx alone and every argument load issues in the first batch; 0 = read
// them at run time (other banks).  The weight loads of the first NPRE (6) steps go out with the
// slab, the rest right after the barrier: the slab wait no longer queues behind the whole
// 139 KB stream (vector memory returns in issue order), and the loop's first steps overlap
// the stream's remainder.
//
// PK (FTMI_BANK_IMAGE): the weights come from the stream-order image instead of the split
// planes: the 16 B a lane loads for a step sit next to its neighbours', so each wave load
// is one contiguous 1 KB run (from the planes it touches 16 half-used 128-B lines, their
// other halves loaded by the next step).  Measured with the bit-3 timing variant's layout
// (r4c stamps): 17.8 vs 20.4 us per call.
//
// NM (one sequence in the row tile, B = 1: the c2 prenet bank): no tap masks.  The slab rows
// outside the sequence are staged as zeros (the conv's zero padding), so every tap reads its
// row directly: a fragment's LDS address is the lane's base + a per-step scalar + a
// compile-time row-block offset (the instruction's immediate), instead of a mask test, a
// select and a quarter-rate multiply per fragment (measured in the ISA: ~7 VALU per
// fragment, 56 per step and wave on the MFMA loop's issue path).  The products of the masked
// taps were +0 x w either way: bit-identical.
template <int MI, int NCH, int DIAG = 0, int KT = 0, int NCT = 0, bool PK = false, bool NM = false>
__global__ __launch_bounds__(512, 1) void conv_bank_halves_kernel(const GemmParams p) {
  BHSTAMP(0, 0);
  constexpr int RM = MI * 16;
  constexpr int SRM = RM + SL_MAXK - 1;   // staged slab rows (every pair)
  constexpr int AIMG = (SRM + 1) * SL_P;  // halves per (chunk, plane) image; row SRM is zero
  constexpr int SLAB_BYTES = NCH * 2 * AIMG * 2;
  constexpr int NIT = 2 * MI * 64;  // f32x4 items of a block's sums: [group of pair][mi][lane]
  constexpr int RED_BYTES = 8 * NIT * 16;
  constexpr int LDS_BYTES = SLAB_BYTES > RED_BYTES ? SLAB_BYTES : RED_BYTES;
  constexpr int NS = (NCH * (SL_MAXK + 1) + 7) / 8;  // steps per wave (at most)
  static_assert(NIT % 512 == 0, "items per thread");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  _Float16 *const lds = (_Float16 *)smem;
  f32x4 *const red = (f32x4 *)smem;  // aliases the slab after the loop
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int NC = NCT ? NCT : p.g[0].N >> 4, K = KT ? KT : p.ngroups;
  const int b = blockIdx.x, h = (b >> 3) & 1, u = (b & 7) | ((b >> 4) << 3);
  const int gi = __builtin_amdgcn_readfirstlane(u / NC);
  const int cset = u - gi * NC, gl = K - 1 - gi;
  const GemmGroup &GH = p.g[gi];  // the pair's heavy group (k = K - gi): its slab
  const GemmGroup &GL = p.g[gl];
  const int kh = GH.k, padh = GH.pad, kl = GL.k, padl = GL.pad, dpl = padh - padl;
  const int Cin = p.Cin, c_half = h * (NCH * 32);  // channels of this half
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;
  const int col = cset * 16 + fr;  // < N (N % 16 == 0: host check)

  // Every load of the prologue is unconditional: a load inside a branch makes the compiler
  // wait for it — and, in issue order, for every load before it — right there.
  // ---- the slab loads: item (row-chunk r = (tid >> 3) + 64 i, channel segment tid & 7);
  // r = c SRM + sr ----
  constexpr int ASLOTS = (NCH * SRM + 63) / 64;
  const int seg = tid & 7;
  f32x4 av[ASLOTS];
#pragma unroll
  for (int i = 0; i < ASLOTS; ++i) {  // past the slab: a clamped (unused) reload
    const int r = min((tid >> 3) + 64 * i, NCH * SRM - 1), c = r / SRM, sr = r - c * SRM;
    int m = sr - padh;  // one row tile: m0 = 0
    const bool inseq = m >= 0 && m < p.M;
    m = m < 0 ? 0 : (m >= p.M ? p.M - 1 : m);  // clamped rows only feed masked taps
    av[i] = *(const f32x4 *)(p.x + (int64_t)m * p.x_stride + c_half + c * 32 + seg * 4);
    if constexpr (NM)  // the zero padding itself (applied after the load issues: no wait here)
      av[i] = inseq ? av[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // ---- the weight fragments of this wave's CONTIGUOUS step range [q0, q1) of the unit's
  // (group, tap, chunk) list, heavy group first, chunks fastest (consecutive steps of a wave
  // read the two halves of each 128-B weight line back to back); clamped, so a step past the
  // range reloads its last one and is never used.  The first NPRE steps now, the rest after
  // the barrier. ----
  const int QH = NCH * kh, Q = QH + NCH * kl;
  const int q0 = (wave * Q) >> 3, q1 = ((wave + 1) * Q) >> 3;
  const _Float16 *wh = (const _Float16 *)GH.w3 + (int64_t)col * GH.Kpad + c_half + fs * 8;
  const _Float16 *wl = (const _Float16 *)GL.w3 + (int64_t)col * GL.Kpad + c_half + fs * 8;
  const int64_t planeh = (int64_t)GH.N * GH.Kpad, planel = (int64_t)GL.N * GL.Kpad;
  f16x8 rb0[NS], rb1[NS];
  auto wload = [&](int i) {
    const int q = max(min(q0 + i, q1 - 1), 0);  // an empty range (q1 == q0 == 0) stays on step 0
    const bool hv = q < QH;
    const int qq = hv ? q : q - QH, j = qq / NCH, c = qq - j * NCH;
    const _Float16 *src = (hv ? wh : wl) + j * Cin + c * 32;
    if constexpr (DIAG & 16) {  // no weight loads at all
      rb0[i] = rb1[i] = (f16x8){};
    } else if constexpr (DIAG & 8) {  // the same bytes per block as 1 KB contiguous runs
      const _Float16 *cb = (const _Float16 *)p.g[K - 1].w3 + (size_t)b * 69632 +
                           (wave * 2 * NS + 2 * i) * 512 + lane * 8;
      rb0[i] = *(const f16x8 *)cb;
      rb1[i] = *(const f16x8 *)(cb + 512);
    } else if constexpr (PK) {  // slot [block][wave][step][plane][lane]; past the range: its last
      const int ii = max(min(i, q1 - q0 - 1), 0);
      const _Float16 *cb = p.wimg + ((int64_t)(b * 8 + wave) * NS + ii) * 1024 + lane * 8;
      rb0[i] = *(const f16x8 *)cb;
      rb1[i] = *(const f16x8 *)(cb + 512);
    } else {
      rb0[i] = *(const f16x8 *)src;
      rb1[i] = *(const f16x8 *)(src + (hv ? planeh : planel));
    }
  };
  // bit 5: every step up front; bits 8 / 9: the first 2 / 4 steps (timing variants); else
  // 6 (r4g stamps, image kernel: 2 / 4 / 6 steps 18.3 / 17.6 / 17.5 us per call, the
  // longest block 33.7 / 33.3 / 32.6 k cycles; every step up front behind a barrier, bit 7:
  // 18.7, the slab wait then queues behind the whole stream)
  constexpr int NPRE0 = (DIAG & 256) ? 2 : (DIAG & 512) ? 4 : 6;
  constexpr int NPRE = (DIAG & (32 | 128)) ? NS : (NS < NPRE0 ? NS : NPRE0);
  if constexpr (DIAG & 128) {
    // every wave's slab loads are issued before any wave's weight loads (a barrier with no
    // wait: vector memory is served in issue order per CU, so the slab no longer queues
    // behind other waves' weight streams)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < NPRE; ++i) wload(i);
  // keep the issue order: the scheduler would otherwise sink loads below the slab's use
  __builtin_amdgcn_sched_barrier(0);

  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < ASLOTS; ++i) {
    const int r = (tid >> 3) + 64 * i, c = r / SRM, sr = r - c * SRM;
    if (r >= NCH * SRM) break;
    const f32x4 x = av[i];
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
    f16x4 hh, tt;
    split2h(x, hh, tt);
    _Float16 *dst = lds + c * 2 * AIMG + sr * SL_P + seg * 4;
    *(f16x4 *)dst = hh;
    *(f16x4 *)(dst + AIMG) = tt;
  }
  if (tid < NCH * 2 * (SL_P / 8)) {  // the zero row of every (chunk, plane) image
    const int img = tid / (SL_P / 8), part = tid % (SL_P / 8);
    *(u32x4 *)(lds + img * AIMG + SRM * SL_P + part * 8) = (u32x4){0u, 0u, 0u, 0u};
  }
  bool bad = !(amax <= 65504.f);
  // per-row tap masks of both groups (heavy in bits 0-15, light in 16-31): bit j set iff
  // frame t + j - pad lies in the sequence; t = row mod T stepped 16 rows at a time
  unsigned msk[MI];
  {
    int t = fr % p.T;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = mi * 16 + fr;
      unsigned a = 0, c = 0;
      if (m < p.M) {
        int lo = max(padh - t, 0), hi = min(p.T - 1 + padh - t, kh - 1);
        if (lo <= hi) a = (2u << hi) - (1u << lo);
        lo = max(padl - t, 0), hi = min(p.T - 1 + padl - t, kl - 1);
        if (lo <= hi) c = (2u << hi) - (1u << lo);
      }
      msk[mi] = a | (c << 16);
      t += 16;
      while (t >= p.T) t -= p.T;
    }
  }
  // LDS stores done, then the barrier: the weight loads stay in flight across it (no vmcnt
  // wait here — __syncthreads could drain them)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  BHSTAMP(1, 0);
#pragma unroll
  for (int i = NPRE; i < NS; ++i) wload(i);
  // the epilogue's per-column parameters, behind every weight load (vector memory completes
  // in issue order: ahead of the slab they held its wait back by a miss's latency); absent
  // parameters read the column scales and are replaced at use (unconditional loads)
  const float cs_h = GH.colscale[col], cs_l = GL.colscale[col];
  const float sc_h0 = (GH.scale ? GH.scale : GH.colscale)[col];
  const float sh_h0 = (GH.scale ? GH.shift : GH.colscale)[col];
  const float sc_l0 = (GL.scale ? GL.scale : GL.colscale)[col];
  const float sh_l0 = (GL.scale ? GL.shift : GL.colscale)[col];
  const float bi_h0 = (GH.bias ? GH.bias : GH.colscale)[col];
  const float bi_l0 = (GL.bias ? GL.bias : GL.colscale)[col];
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acch[MI], accl[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) acch[mi] = accl[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // a step's row fragments in blocks of 4: each accumulator still adds at . bh, ah . b1,
  // ah . b0 in that order (the skinny kernel's per-accumulator order), with half the A
  // fragments live at once
  constexpr int MB = (DIAG & 64) ? MI : (MI < 4 ? MI : 4);  // bit 6: all row fragments at once
  auto step = [&](f32x4 (&acc)[MI], const _Float16 *Ab, int sh_j, int dr, f16x8 b0, f16x8 b1) {
    const f16x8 bh = b0 * (_Float16)(1.0f / H3_SCALE);
#pragma unroll
    for (int m0 = 0; m0 < MI; m0 += MB) {
      f16x8 ah[MB], at[MB];
#pragma unroll
      for (int mm = 0; mm < MB; ++mm) {
        const int mi = m0 + mm;
        const bool ok = NM || ((msk[mi] >> sh_j) & 1u) != 0;
        // masked form: the zero row selected as an offset from the same immediate (the slab
        // kernel's multiply-free address, the same addresses)
        const int o = NM ? (fr + dr) * SL_P + fs * 8 + mi * 16 * SL_P
                         : (ok ? (fr + dr) * SL_P + fs * 8 : SRM * SL_P + fs * 8 - mi * 16 * SL_P) +
                               mi * 16 * SL_P;
        if constexpr (DIAG & 2) {
          ah[mm] = b1;
          at[mm] = bh;
        } else {
          ah[mm] = *(const f16x8 *)(Ab + o);
          at[mm] = *(const f16x8 *)(Ab + AIMG + o);
        }
      }
      if constexpr (DIAG & 1) {
        acc[m0][0] += (float)bh[0] + (float)b1[0] + (float)ah[0][0] + (float)at[MB - 1][0];
        continue;
      }
#pragma unroll
      for (int mm = 0; mm < MB; ++mm) acc[m0 + mm] = mma16(at[mm], bh, acc[m0 + mm]);  // small terms first
#pragma unroll
      for (int mm = 0; mm < MB; ++mm) acc[m0 + mm] = mma16(ah[mm], b1, acc[m0 + mm]);
#pragma unroll
      for (int mm = 0; mm < MB; ++mm) acc[m0 + mm] = mma16(ah[mm], b0, acc[m0 + mm]);
    }
  };
  // the heavy group's steps, then the light group's: two code regions, each updating its
  // own accumulators in place (one loop choosing the set per step made the compiler copy
  // both sets at every join); the steps' weights were issued in this order
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int q = q0 + i;
    if (q < q1 && q < QH) {  // wave-uniform
      const int j = q / NCH, c = q - j * NCH;
      step(acch, lds + c * 2 * AIMG, j, j, rb0[i], rb1[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int q = q0 + i;
    if (q < q1 && q >= QH) {  // wave-uniform
      const int qq = q - QH, j = qq / NCH, c = qq - j * NCH;
      step(accl, lds + c * 2 * AIMG, j + 16, j + dpl, rb0[i], rb1[i]);
    }
  }
  BHSTAMP(2, 0);
  BHSTAMP(3, 448);

  // ---- the waves' sums meet in LDS, in wave order (the slab is dead after the barrier):
  // only the waves whose range holds steps of a group write and are summed for it ----
  const bool has_h = q0 < QH, has_l = q1 > QH;
  __syncthreads();
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    if (has_h) red[(wave * 2 + 0) * MI * 64 + mi * 64 + lane] = acch[mi];
    if (has_l) red[(wave * 2 + 1) * MI * 64 + mi * 64 + lane] = accl[mi];
  }
  __syncthreads();
  // thread t owns items e = t + 512 r: (group of the pair ug, fragment mi, lane ln); the
  // waves holding heavy steps are 0 .. wlast_h, light ones wfirst_l .. 7
  int wlast_h = 0, wfirst_l = 7;  // exactly the waves whose has_h / has_l held above
#pragma unroll
  for (int w = 7; w >= 0; --w)
    if (((w * Q) >> 3) < QH) {
      wlast_h = w;
      break;
    }
#pragma unroll
  for (int w = 0; w < 8; ++w)
    if ((((w + 1) * Q) >> 3) > QH) {
      wfirst_l = w;
      break;
    }
  constexpr int IPT = NIT / 512;
  f32x4 v[IPT];
  int eo[IPT];
#pragma unroll
  for (int r = 0; r < IPT; ++r) {
    const int e = tid + 512 * r, ug = e / (MI * 64);
    eo[r] = e;
    const int w0 = ug ? wfirst_l : 0, w1 = ug ? 7 : wlast_h;
    // every partial read at once (slots past w1 re-read w1's, never added), then summed in
    // wave order: one LDS round trip instead of one per wave, the same additions
    f32x4 pv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] = red[min(w0 + k, w1) * NIT + e];
    f32x4 s = pv[0];
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (w0 + k <= w1) s += pv[k];  // wave-uniform
    v[r] = s;
  }
  BHSTAMP(4, 0);
  // ---- write-through publish of this half's sums, then an arrival counter PER WAVE: wave w
  // owns row fragment w of both groups (items e = tid + 512 r), publishes them, waits for its
  // own stores and adds to the unit's counter w; the wave whose add returns 1 (its partner
  // wave in the other half has published) finishes that slice.  No block barrier: each
  // slice is finished by whichever half's wave arrives last (MI355X_MICROARCH.md "Valid
  // forms": each storing wave signalling for itself, the last adder told by the value its
  // add returned, loads after that add has returned) ----
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.part, (short)0, 0x7FFFFFF0, 0x00020000);
  const int ubase = (u * 2) * NIT * 16;  // bytes: [unit][half][item]; < 2^31 (host check)
#pragma unroll
  for (int r = 0; r < IPT; ++r)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[r]), rs,
                                           ubase + (h * NIT + eo[r]) * 16, 0, 16 /* sc1 */);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores done
  unsigned old = 0;
  if (lane == 0) {
    unsigned *const cnt = p.tile_cnt + u * 8 + wave;
    old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 1u)  // both halves' waves have added: zero for the next launch
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool last = (DIAG & 4) ? h == 0 : __builtin_amdgcn_readfirstlane(old) == 1u;
  BHSTAMP(5, 0);
  if (last) {
    u32x4 pr[IPT];
#pragma unroll
    for (int r = 0; r < IPT; ++r)
      pr[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, ubase + ((1 - h) * NIT + eo[r]) * 16, 0,
                                                    16 /* sc1 */);
#pragma unroll
    for (int r = 0; r < IPT; ++r) {
      const int e = eo[r], ug = e / (MI * 64), mi = (e >> 6) % MI;
      const f32x4 s = (DIAG & 4) ? v[r] : v[r] + __builtin_bit_cast(f32x4, pr[r]);  // commutative
      const GemmGroup &GW = ug ? GL : GH;
      const float cs = ug ? cs_l : cs_h;
      const float sc = (ug ? GL.scale : GH.scale) ? (ug ? sc_l0 : sc_h0) : 1.f;
      const float sh = (ug ? GL.scale : GH.scale) ? (ug ? sh_l0 : sh_h0) : 0.f;
      const float bi = (ug ? GL.bias : GH.bias) ? (ug ? bi_l0 : bi_h0) : 0.f;
      float *yc = p.y + GW.ycol0 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = mi * 16 + 4 * fs + i;
        if (row >= p.M) continue;
        bad |= !__builtin_isfinite(s[i]);
        float y = s[i] * cs + bi;
        if (p.relu) y = fmaxf(y, 0.f);
        if (GW.scale) y = y * sc + sh;
        yc[(int64_t)row * p.y_stride] = y;
      }
    }
  }
  if (bad && p.status) atomicOr(p.status, 1u);
  BHSTAMP(6, 0);
  BHSTAMP(7, 448);
}

// steps per wave of conv_bank_halves_kernel (its NS) and the halves of its weight image
constexpr int bh_steps(int nch) { return (nch * (SL_MAXK + 1) + 7) / 8; }
static int64_t bank_halves_image_halves(int K, int N, int Cin) {
  return (int64_t)(K / 2) * (N / 16) * 2 * 8 * bh_steps(Cin / 64) * 1024;
}

// The weight image of conv_bank_halves_kernel<..., PK = true>: block b, wave w, step slot i,
// plane pl, lane l hold the 8 halves that lane loads for that step in the plane-reading
// kernel — the same (unit, half, step range, clamp) arithmetic, with the one difference that
// a wave whose range is empty copies step 0 (the kernel loads that slot and never uses it).
// Built once per weights version (ops.bank_halves_image); p.wimg is the output here.
template <int NCH>
__global__ __launch_bounds__(512) void bank_halves_pack_kernel(const GemmParams p) {
  constexpr int NS = bh_steps(NCH);
  const int NC = p.g[0].N >> 4, K = p.ngroups;
  const int b = blockIdx.x, h = (b >> 3) & 1, u = (b & 7) | ((b >> 4) << 3);
  const int gi = u / NC, cset = u - gi * NC, gl = K - 1 - gi;
  const GemmGroup &GH = p.g[gi];
  const GemmGroup &GL = p.g[gl];
  const int Cin = p.Cin, c_half = h * (NCH * 32);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4, col = cset * 16 + fr;
  const int QH = NCH * GH.k, Q = QH + NCH * GL.k;
  const int q0 = (wave * Q) >> 3, q1 = ((wave + 1) * Q) >> 3;
  const _Float16 *wh = (const _Float16 *)GH.w3 + (int64_t)col * GH.Kpad + c_half + fs * 8;
  const _Float16 *wl = (const _Float16 *)GL.w3 + (int64_t)col * GL.Kpad + c_half + fs * 8;
  const int64_t planeh = (int64_t)GH.N * GH.Kpad, planel = (int64_t)GL.N * GL.Kpad;
  _Float16 *dst = (_Float16 *)p.wimg + (int64_t)(b * 8 + wave) * NS * 1024 + lane * 8;
  for (int i = 0; i < NS; ++i) {
    const int q = max(min(q0 + i, q1 - 1), 0);
    const bool hv = q < QH;
    const int qq = hv ? q : q - QH, j = qq / NCH, c = qq - j * NCH;
    const _Float16 *src = (hv ? wh : wl) + j * Cin + c * 32;
    *(f16x8 *)(dst + i * 1024) = *(const f16x8 *)src;
    *(f16x8 *)(dst + i * 1024 + 512) = *(const f16x8 *)(src + (hv ? planeh : planel));
  }
}

// sum of the skinny kernel's split partials + the conv epilogue; blockIdx.y is the group
// (uniform: its parameters stay scalar loads).  L = 4 lanes share an element when there
// are many splits (L = 1 below 8): lane q adds splits q, q + L, ... in order and xor-
// shuffles combine the L sums in a fixed order, so the result is deterministic and the
// dependent load chains are L times shorter.
template <int L>
__global__ __launch_bounds__(256) void skinny_finish_kernel(const GemmParams p) {
  const GemmGroup &G = p.g[blockIdx.y];
  const int N = G.N, q = threadIdx.x & (L - 1);
  const int64_t total = (int64_t)p.M * p.ldp, n_el = (int64_t)p.M * N;
  for (int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L; idx < n_el;
       idx += (int64_t)gridDim.x * (256 / L)) {  // the L lanes of an element iterate together
    const int row = (int)(idx / N), col = (int)(idx - (int64_t)row * N);
    const int64_t pi = (int64_t)row * p.ldp + G.ycol0 + col;
    // eight / four splits' loads issued together, added in split order (the same sums as
    // one by one)
    float v = 0.f;
    int s = q;
    for (; s + 7 * L < p.split; s += 8 * L) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = p.part[(size_t)(s + u * L) * total + pi];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += a[u];
    }
    for (; s + 3 * L < p.split; s += 4 * L) {
      const float a0 = p.part[(size_t)s * total + pi], a1 = p.part[(size_t)(s + L) * total + pi];
      const float a2 = p.part[(size_t)(s + 2 * L) * total + pi];
      const float a3 = p.part[(size_t)(s + 3 * L) * total + pi];
      v += a0;
      v += a1;
      v += a2;
      v += a3;
    }
    for (; s < p.split; s += L) v += p.part[(size_t)s * total + pi];
    if constexpr (L == 4) {
      v += __shfl_xor(v, 1, 4);
      v += __shfl_xor(v, 2, 4);
      if (q) continue;
    }
    if (G.bias) v += G.bias[col];
    if (p.relu) v = fmaxf(v, 0.f);
    if (G.scale) v = v * G.scale[col] + G.shift[col];
    if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
    if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
    if (p.yt) {
      const int b = row / p.To, t = row - b * p.To;
      p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
    }
  }
}

// the skinny kernel's highway finish (common_layers.py:22-35): GEMM columns q*64 + h (W1)
// and q*64 + 32 + h (W2) of output column o = q*32 + h, summed over the splits in order,
// then g = sigmoid(x W2 + b2), y = g * relu(x W1 + b1) + (1 - g) * x
__global__ __launch_bounds__(256) void skinny_highway_finish_kernel(const GemmParams p) {
  const int C = p.g[0].N / 2;
  const int64_t total = (int64_t)p.M * p.ldp, n_el = (int64_t)p.M * C;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < n_el;
       idx += (int64_t)gridDim.x * 256) {
    const int row = (int)(idx / C), o = (int)(idx - (int64_t)row * C);
    const int c1 = (o >> 5) * 64 + (o & 31);
    const int64_t pi = (int64_t)row * p.ldp + c1;
    float v1 = 0.f, v2 = 0.f;
    int s = 0;
    for (; s + 1 < p.split; s += 2) {  // two splits' loads together, added in split order
      const float a0 = p.part[(size_t)s * total + pi], b0 = p.part[(size_t)s * total + pi + 32];
      const float a1 = p.part[(size_t)(s + 1) * total + pi];
      const float b1 = p.part[(size_t)(s + 1) * total + pi + 32];
      v1 += a0;
      v2 += b0;
      v1 += a1;
      v2 += b1;
    }
    for (; s < p.split; ++s) {
      v1 += p.part[(size_t)s * total + pi];
      v2 += p.part[(size_t)s * total + pi + 32];
    }
    const float g = ftmi_sigmoid(v2 + p.b2[o]);
    const float xin = p.x[(int64_t)row * p.x_stride + o];
    p.y[(int64_t)row * p.y_stride + o] = highway_mix(g, v1 + p.b1[o], xin);
  }
}

// w [N][K] fp32 -> [3][N][Kpad] bf16 pieces (w = p0 + p1 + p2 exactly), zero K padding
__global__ void split_weights_kernel(const float *__restrict__ w, int64_t N, int64_t K,
                                     int64_t Kpad, __bf16 *__restrict__ out) {
  const int64_t total = N * Kpad;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / Kpad, k = i - n * Kpad;
    const float v = k < K ? w[n * K + k] : 0.f;
    const __bf16 h1 = (__bf16)v;
    const float r1 = v - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    const __bf16 h3 = (__bf16)(r1 - (float)h2);
    out[i] = h1;
    out[total + i] = h2;
    out[2 * total + i] = h3;
  }
}

// w [N][K] fp32 -> f16 planes [3][N][Kpad] (B0 = 2^11 w_h, B1 = w_t, B2 = w_h of the
// column-scaled row w s_n) followed by colscale[N] = 2^-11 / s_n.  One workgroup per row:
// s_n = 2^-e with the smallest e >= 0 such that max|w[n]| s_n < 16 (so 2^11 w_h stays
// inside the f16 range).
// frag: planes in the fragment-major order [N/16][Kpad/32][64 lanes][8] of the
// v_mfma_f32_16x16x32_f16 B operand (lane = n % 16 + 16 ((k / 8) % 4), element k % 8) —
// the layout of ftmi_highway_stack; else row-major [N][Kpad].
__global__ __launch_bounds__(256) void split_weights_f16_kernel(const float *__restrict__ w,
                                                                int64_t N, int64_t K, int64_t Kpad,
                                                                _Float16 *__restrict__ out,
                                                                float *__restrict__ colscale,
                                                                int frag) {
  __shared__ float red[4];
  const int64_t n = blockIdx.x;
  const float *row = w + n * K;
  float m = 0.f;
  for (int64_t k = threadIdx.x; k < K; k += 256) m = fmaxf(m, fabsf(row[k]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int ex = 0;
  if (__builtin_isfinite(m) && m > 0.f) frexpf(m, &ex);  // m = f * 2^ex, f in [0.5, 1)
  const int e = ex > 4 ? ex - 4 : 0;                     // m * 2^-e < 2^4
  const int64_t plane = N * Kpad;
  for (int64_t k = threadIdx.x; k < Kpad; k += 256) {
    const float v = k < K ? ldexpf(row[k], -e) : 0.f;
    const _Float16 h = (_Float16)v;
    const _Float16 t = (_Float16)((v - (float)h) * H3_SCALE);
    const int64_t o = frag ? ((n >> 4) * (Kpad / 32) + (k >> 5)) * 512 + ((k >> 3) & 3) * 128 +
                                 (n & 15) * 8 + (k & 7)
                           : n * Kpad + k;
    out[o] = (_Float16)((float)h * H3_SCALE);
    out[plane + o] = t;
    out[2 * plane + o] = h;
  }
  if (threadIdx.x == 0) colscale[n] = ldexpf(1.f, e - 11);
}

// Split-K finish: v = sum_s part[s][m][n] (fixed order: deterministic), then the
// EPI_CONV epilogue (bias, ReLU, BN, residual, plain and transposed stores).
// fp32 rows -> f16x3 split rows (include/ftmi.h): 4 channels per thread, range-checked
__global__ __launch_bounds__(256) void split_rows_kernel(const float *__restrict__ x,
                                                         int64_t x_stride, int64_t rows, int C,
                                                         float *__restrict__ y, int64_t y_stride,
                                                         unsigned *status) {
  const int C4 = C >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * C4) return;
  const int64_t r = i / C4;
  const int c = (int)(i - r * C4) * 4;
  const f32x4 v = *(const f32x4 *)(x + r * x_stride + c);
  f16x4 h, t;
  split2h(v, h, t);
  _Float16 *yr = (_Float16 *)(y + r * y_stride) + c;
  *(f16x4 *)yr = h;
  *(f16x4 *)(yr + C) = t;
  const float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  if (!(m <= 65504.f) && status) atomicOr(status, 1u);
}

__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const GemmParams p) {
  const GemmGroup &G = p.g[0];
  const int64_t total = (int64_t)p.M * G.N;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int row = (int)(idx / G.N), col = (int)(idx - (int64_t)row * G.N);
    float v = p.part[idx];
    for (int s = 1; s < p.split; ++s) v += p.part[(size_t)s * total + idx];
    if (G.bias) v += G.bias[col];
    if (p.relu) v = fmaxf(v, 0.f);
    if (G.scale) v = v * G.scale[col] + G.shift[col];
    if (p.residual) v += p.residual[(int64_t)row * p.res_stride + col];
    if (p.y) p.y[(int64_t)row * p.y_stride + G.ycol0 + col] = v;
    if (p.yt) {
      const int b = row / p.To, t = row - b * p.To;
      p.yt[((int64_t)b * p.yt_channels + G.ycol0 + col) * p.To + t] = v;
    }
  }
}

// ---- highway stack: pre_highway -> L highways -> GRU input projection, one launch -------
// models/common_layers.py:110-115 (CBHG: x = pre_highway(x); for h in highways: x = h(x);
// then the bidirectional GRU, whose input projection x W_ih^T + b_ih is the last GEMM here).
// The unfused chain writes and re-reads the (M, 256) activations in HBM between every layer
// and its short-K launches (K = 256: 8 k-steps per 256 x 128 tile) are prologue-bound.  Here
// one workgroup owns 64 rows x all 256 channels for the whole chain: 8 waves, wave w owns h
// columns [32w, 32w + 32).  Each layer's output is split (f16 head / scaled tail, as the
// other f16x3 kernels) into one of two LDS images — the next layer's A operand — while the
// wave keeps its own 64 x 32 block in fp32 registers: exactly the x its next gating needs,
// since the W1 and W2 columns of one h column (packed 32-column blocks) land in the same lane.
// B fragments (the pre-split f16 planes; every workgroup reads the same 1.4 MB, L2-resident)
// are loaded straight into registers three k-steps ahead; each GEMM runs in 16-column
// halves (a highway's W1 tile with its W2 tile) to keep that ring in the register budget.
// (A 128-row variant with 8 waves x 128 x 32 measured 671 vs 694 us at the c3 postnet and
// 209 vs 121 us at the prenet, where 100 tiles leave CUs idle: dropped.)  Per k-step, per product, the MFMA
// order and the epilogue arithmetic are the slab kernel's, so the result is bit-identical to
// the unfused chain.  HBM traffic per row: Cp floats in, n_out floats out (+ C with h).
constexpr int HS_BM = 64;
constexpr int HS_C = 256;
constexpr int HS_P = HS_C + 16;  // halves per LDS row: conflict-free ds_read_b128 fragments
constexpr int HS_IMG = HS_BM * HS_P;
constexpr int HS_MAXL = 8;
constexpr int HS_NPASS = 512;  // output-projection columns per pass (8 waves x 64)

struct HwStackParams {
  const float *x;
  int64_t x_stride;
  int M, Cp, kp_pre;      // rows, input channels, K of the pre_highway planes (roundup 32)
  const _Float16 *w_pre;  // f16 planes [3][C][kp_pre] (B0 = 2^11 w_h, B1 = w_t, B2 = w_h)
  const float *cs_pre;    // its column scales
  int L;
  const _Float16 *w_hw[HS_MAXL];  // [3][2C][C], W1 | W2 packed in 32-row blocks
  const float *cs_hw[HS_MAXL];
  const float *b1[HS_MAXL];
  const float *b2[HS_MAXL];
  const _Float16 *w_out;  // [3][n_out][C] (null: no projection)
  const float *cs_out;
  const float *b_out;
  int n_out;
  float *y;
  int64_t y_stride;
  float *h;  // optional: the last highway's output (fp32)
  int64_t h_stride;
  unsigned *status;
};

// acc[mi][ni] (rows 16 mi + 4 fs + i, GEMM column of bp[ni] + fr) = A x B^T over nks k-steps
// of 32, f16x3 (small terms first, as the slab kernel).  bp[ni]: the lane's B0 row + 8 fs.
template <int NI, int MI = 4>
__device__ __forceinline__ void hs_step(f32x4 (&acc)[MI][NI], const _Float16 *Ah,
                                        const _Float16 *At, const f16x8 (&b0)[NI],
                                        const f16x8 (&b1)[NI], int ks, int fr, int fs) {
  f16x8 bh[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) bh[ni] = b0[ni] * (_Float16)(1.0f / H3_SCALE);
  if constexpr (MI > 4) {  // the A fragments of row block mi + 1 read under the MFMAs of mi,
                           // one block ahead only (register budget: sched barriers)
    f16x8 ah = *(const f16x8 *)(Ah + fr * HS_P + 32 * ks + 8 * fs);
    f16x8 at = *(const f16x8 *)(At + fr * HS_P + 32 * ks + 8 * fs);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      f16x8 nh = ah, nt = at;
      if (mi + 1 < MI) {
        const int o = (16 * (mi + 1) + fr) * HS_P + 32 * ks + 8 * fs;
        nh = *(const f16x8 *)(Ah + o);
        nt = *(const f16x8 *)(At + o);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        f32x4 c = acc[mi][ni];
        c = mma16(at, bh[ni], c);
        c = mma16(ah, b1[ni], c);
        c = mma16(ah, b0[ni], c);
        acc[mi][ni] = c;
      }
      __builtin_amdgcn_sched_barrier(0);
      ah = nh;
      at = nt;
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {  // A fragments one row block at a time (register budget)
    const int o = (16 * mi + fr) * HS_P + 32 * ks + 8 * fs;
    const f16x8 ah = *(const f16x8 *)(Ah + o);
    const f16x8 at = *(const f16x8 *)(At + o);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      f32x4 c = acc[mi][ni];
      c = mma16(at, bh[ni], c);
      c = mma16(ah, b1[ni], c);
      c = mma16(ah, b0[ni], c);
      acc[mi][ni] = c;
    }
  }
}

// acc[mi][ni] (rows 16 mi + 4 fs + i, GEMM column of bp[ni] + fr) = A x B^T over nks k-steps
// of 32, f16x3 (small terms first, as the slab kernel).  bp[ni]: the lane's B0 row + 8 fs.
// B fragments rotate through three register sets, loaded three k-steps ahead (the loop is
// kept rolled and the steps fenced by sched barriers: otherwise the compiler hoists further
// loads and LDS reads across steps and spills).
template <int NI, int MI = 4>
__device__ __forceinline__ void hs_gemm_acc(f32x4 (&acc)[MI][NI], const _Float16 *Ah,
                                            const _Float16 *At, const _Float16 *const (&bp)[NI],
                                            int64_t plane, int nks, int fr, int fs) {
  // three register sets in a ring: the loads of k-step ks + 3 are issued right after step
  // ks consumed its set (one step of look-ahead left the L2 latency exposed: the MFMAs of a
  // step are ~800 cycles per wave, a loaded L2 round trip is more)
  f16x8 x0[NI], x1[NI], y0[NI], y1[NI], z0[NI], z1[NI];
  auto load = [&](f16x8 (&r0)[NI], f16x8 (&r1)[NI], int ks) {
    const int k = ks < nks ? ks : nks - 1;  // past the end: a clamped (unused) re-read
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      r0[ni] = *(const f16x8 *)(bp[ni] + 512 * k);
      r1[ni] = *(const f16x8 *)(bp[ni] + plane + 512 * k);
    }
  };
  load(x0, x1, 0);
  load(y0, y1, 1);
  load(z0, z1, 2);
#pragma unroll 1
  for (int ks = 0; ks < nks; ks += 3) {
    hs_step<NI, MI>(acc, Ah, At, x0, x1, ks, fr, fs);
    load(x0, x1, ks + 3);
    __builtin_amdgcn_sched_barrier(0);  // no hoisting across steps (register budget)
    if (ks + 1 >= nks) break;
    hs_step<NI, MI>(acc, Ah, At, y0, y1, ks + 1, fr, fs);
    load(y0, y1, ks + 4);
    __builtin_amdgcn_sched_barrier(0);
    if (ks + 2 >= nks) break;
    hs_step<NI, MI>(acc, Ah, At, z0, z1, ks + 2, fr, fs);
    load(z0, z1, ks + 5);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NI, int MI = 4>
__device__ __forceinline__ void hs_gemm(f32x4 (&acc)[MI][NI], const _Float16 *Ah,
                                        const _Float16 *At, const _Float16 *const (&bp)[NI],
                                        int64_t plane, int nks, int fr, int fs) {
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};
  hs_gemm_acc<NI, MI>(acc, Ah, At, bp, plane, nks, fr, fs);
}

// BM = 64: two LDS images, ping-pong (each layer reads one, writes the other); BM = 96: one
// image of 96 rows, overwritten in place behind a barrier (104 KB) — each weight fragment a
// wave fetches then feeds 6 row blocks instead of 4, cutting the per-CU L2 fetch per flop,
// which is what bounds this kernel, by a third.
template <int BM>
__global__ __launch_bounds__(512, 1) void highway_stack_kernel(const HwStackParams p) {
  constexpr int MI = BM / 16, NIMG = BM == 64 ? 2 : 1, IMG = BM * HS_P;
  static_assert(BM == 64 || BM == 96, "rows per workgroup");
  __shared__ __attribute__((aligned(16))) _Float16 lds[NIMG * 2 * IMG];  // [image][head|tail]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;
  // column block of this wave, rotated per workgroup so that the CUs of one XCD (blocks
  // b, b + 8, ...) stream different weight rows at any moment instead of all hitting the
  // same L2 lines (channel hot spots); the arithmetic per column is unchanged
  const int cb = (wave + (blockIdx.x >> 3)) & 7;
  // the lane's B0 fragment of columns [n0, n0 + 16), k-step 0, in the fragment-major planes
  // [N/16][Kpad/32][64 lanes][8] (ftmi_split_weights_f16_frag): every wave load is one
  // contiguous 1-KB run (8 whole cache lines; row-major planes cost 16 half lines, measured
  // 1.48x slower at c3: the per-CU fetch rate, not MFMA, bounds this kernel)
  auto bptr = [&](const _Float16 *base, int n0, int Kpad) -> const _Float16 * {
    return base + (int64_t)(n0 >> 4) * (Kpad / 32) * 512 + lane * 8;
  };
  const int m0 = blockIdx.x * BM;
  float amax = 0.f;  // range guard: largest |activation| fed to the f16 split

  // ---- the input rows (Cp channels, zero-padded to kp_pre; rows past M zero) -> image 0
  const int q4 = p.kp_pre / 4;
  for (int e = tid; e < BM * q4; e += 512) {
    const int r = e / q4, c = (e - r * q4) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m0 + r < p.M && c < p.Cp) v = *(const f32x4 *)(p.x + (int64_t)(m0 + r) * p.x_stride + c);
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    f16x4 hh, tt;
    split2h(v, hh, tt);
    *(f16x4 *)(lds + r * HS_P + c) = hh;
    *(f16x4 *)(lds + IMG + r * HS_P + c) = tt;
  }
  __syncthreads();

  f32x4 xs[MI][2];  // this wave's BM x 32 block of the current activations, fp32
  auto put = [&](int img) {  // xs -> LDS image img (split)
    _Float16 *Hd = lds + img * 2 * IMG, *Tl = Hd + IMG;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = xs[mi][nj][i];
          amax = fmaxf(amax, fabsf(v));
          const _Float16 hh = (_Float16)v;
          const int o = (16 * mi + 4 * fs + i) * HS_P + 32 * cb + 16 * nj + fr;
          Hd[o] = hh;
          Tl[o] = (_Float16)((v - (float)hh) * H3_SCALE);
        }
  };

  // ---- pre_highway (Linear, no bias): x W_pre^T, K = kp_pre
  {
    f32x4 acc[MI][2];
    const _Float16 *bp[2];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      bp[ni] = bptr(p.w_pre, 32 * cb + 16 * ni, p.kp_pre);
    hs_gemm<2, MI>(acc, lds, lds + IMG, bp, (int64_t)HS_C * p.kp_pre, p.kp_pre / 32, fr, fs);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const float cs = p.cs_pre[32 * cb + 16 * ni + fr];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) xs[mi][ni] = acc[mi][ni] * cs;
    }
  }
  int cur = NIMG - 1;
  if (NIMG == 1) __syncthreads();  // every wave is done reading the input image
  put(cur);
  __syncthreads();

  // ---- highways: g = sigmoid(x W2^T + b2), x <- g relu(x W1^T + b1) + (1 - g) x
  for (int l = 0; l < p.L; ++l) {
    const _Float16 *A = lds + cur * 2 * IMG;
    // two halves: W1 tile nj with its W2 tile (GEMM columns 64 cb + 16 nj, + 32), so one
    // half's accumulators and B ring stay small
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) {
      f32x4 acc[MI][2];
      const _Float16 *bp[2] = {bptr(p.w_hw[l], 64 * cb + 16 * nj, HS_C),
                               bptr(p.w_hw[l], 64 * cb + 32 + 16 * nj, HS_C)};
      hs_gemm<2, MI>(acc, A, A + IMG, bp, (int64_t)2 * HS_C * HS_C, HS_C / 32, fr, fs);
      const int col = 32 * cb + 16 * nj + fr;
      const float c1 = p.cs_hw[l][64 * cb + 16 * nj + fr];
      const float c2 = p.cs_hw[l][64 * cb + 32 + 16 * nj + fr];
      const float bb1 = p.b1[l][col], bb2 = p.b2[l][col];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float x1, x2;
          {
#pragma clang fp contract(off)
            // rounded like the slab kernel: the column scale, then the bias
            x1 = acc[mi][0][i] * c1 + bb1;
            x2 = acc[mi][1][i] * c2 + bb2;
          }
          const float g = ftmi_sigmoid(x2);
          xs[mi][nj][i] = highway_mix(g, x1, xs[mi][nj][i]);
        }
    }
    if (NIMG == 2) {
      cur ^= 1;  // the image read two layers ago: every wave passed the barrier since
    } else {
      __syncthreads();  // every wave is done reading the image it overwrites
    }
    put(cur);
    __syncthreads();
  }
  if (p.h) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * mi + 4 * fs + i;
        if (row >= p.M) continue;
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
          p.h[(int64_t)row * p.h_stride + 32 * cb + 16 * nj + fr] = xs[mi][nj][i];
      }
  }

  // ---- output projection (the GRU's x W_ih^T + b_ih), HS_NPASS columns per pass
  if (p.w_out) {
    const _Float16 *A = lds + cur * 2 * IMG;
    for (int q = 0; q < 2 * p.n_out / HS_NPASS; ++q) {  // 256 columns (32 per wave) a pass
      f32x4 acc[MI][2];
      const int n0 = (HS_NPASS / 2) * q + 32 * cb;
      const _Float16 *bp[2] = {bptr(p.w_out, n0, HS_C), bptr(p.w_out, n0 + 16, HS_C)};
      hs_gemm<2, MI>(acc, A, A + IMG, bp, (int64_t)p.n_out * HS_C, HS_C / 32, fr, fs);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = n0 + 16 * ni + fr;
        const float cs = p.cs_out[col], b = p.b_out ? p.b_out[col] : 0.f;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
#pragma clang fp contract(off)
            const int row = m0 + 16 * mi + 4 * fs + i;
            float v = acc[mi][ni][i] * cs;
            if (p.b_out) v += b;
            if (row < p.M) p.y[(int64_t)row * p.y_stride + col] = v;
          }
      }
    }
  }
  if (!(amax <= 65504.f) && p.status) atomicOr(p.status, 1u);
}

// ---- the CBHG tail for few rows, spread over the chip (c2: 120 / 816 rows) -------------
// highway_stack_kernel gives one workgroup 64 rows x ALL 256 channels, so at batch 1 (120
// prenet rows: 2 workgroups; 816 postnet rows: 13) a few CUs stream the whole 3-4 MB of
// weight planes each (~100 us).  Here a row block is spread over HSS_P = 16 workgroups, each
// owning 16 output channels of every layer (and n_out / 16 columns of the output
// projection): it streams 1/16 of the weights, and the layers' activations are exchanged
// between the 16 workgroups of a row block through memory after each layer.  Exchange
// (MI355X_MICROARCH.md "Valid forms", first row of the sc1 table): a workgroup writes its
// 64 x 16 slice of the layer's output, split into the f16 head / scaled-tail image layout,
// with 16-B sc1 stores; every storing wave waits for its stores (vmcnt(0)); a barrier; one
// lane adds to the row block's counter (agent scope) and polls it (sc1 loads, bounded) until
// all 16 have added for this layer; a barrier; then every wave loads the full 64 x 256 image
// with sc1 loads into LDS.  The image buffers alternate by layer parity: a workgroup writes
// layer l + 2's slice only after all 16 have published layer l + 1, which each did after
// reading layer l's image.  Per accumulator the k-step, product and epilogue order of
// highway_stack_kernel (hs_gemm over the same fragment-major planes, one 16-row block per
// wave): the results are bit-identical to it.  Every workgroup must be resident at once
// (RB x 16 <= the CU count: the host checks); a spin past the bound sets the status word's
// timeout bit (FTMI_STATUS_RNN_TIMEOUT) instead of hanging.
constexpr int HSS_P = 16;       // workgroups (channel slices) per row block
constexpr int HSS_MAXRB = 16;   // row blocks: M <= 1024
constexpr int HSS_CNT = 32;     // words between row-block counters (one 128-B line each)

struct HsSpread {
  unsigned *cnt;    // [RB][HSS_CNT] arrival counters, zeroed before the launch
  _Float16 *xb;     // [2][RB][2 planes][HS_BM][HS_P] exchange images
  unsigned spin;    // poll bound
};

template <int NO>
__global__ __launch_bounds__(512, 1) void highway_spread_kernel(const HwStackParams p,
                                                               const HsSpread q) {
  constexpr int IMG = HS_IMG;
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * IMG];           // head | tail
  __shared__ __attribute__((aligned(16))) _Float16 pub[2 * HS_BM * 16];   // the slice, split
  __shared__ int s_abort;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;
  const int s = blockIdx.x % HSS_P, rb = blockIdx.x / HSS_P;
  const int m0 = rb * HS_BM, mi = wave & 3;
  const int RB = (p.M + HS_BM - 1) / HS_BM;
  auto bptr = [&](const _Float16 *base, int n0, int Kpad) -> const _Float16 * {
    return base + (int64_t)(n0 >> 4) * (Kpad / 32) * 512 + lane * 8;
  };
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(q.xb, (short)0, 0x7FFFFFF0, 0x00020000);
  const int img_halves = 2 * HS_BM * HS_P;  // one (parity, row block) image
  float amax = 0.f;
  if (tid == 0) s_abort = 0;

  // ---- the input rows -> the LDS image (as highway_stack_kernel)
  const int q4 = p.kp_pre / 4;
  for (int e = tid; e < HS_BM * q4; e += 512) {
    const int r = e / q4, c = (e - r * q4) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m0 + r < p.M && c < p.Cp) v = *(const f32x4 *)(p.x + (int64_t)(m0 + r) * p.x_stride + c);
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    f16x4 hh, tt;
    split2h(v, hh, tt);
    *(f16x4 *)(lds + r * HS_P + c) = hh;
    *(f16x4 *)(lds + IMG + r * HS_P + c) = tt;
  }
  __syncthreads();
  const _Float16 *Ah = lds + 16 * mi * HS_P, *At = lds + IMG + 16 * mi * HS_P;

  // waves 0-3: rows 16 mi + 4 fs + i, channel 16 s + fr of the current activations (fp32)
  f32x4 xs = {0.f, 0.f, 0.f, 0.f};
  if (wave < 4) {  // pre_highway (no bias)
    f32x4 acc[1][1];
    const _Float16 *bp[1] = {bptr(p.w_pre, 16 * s, p.kp_pre)};
    hs_gemm<1, 1>(acc, Ah, At, bp, (int64_t)HS_C * p.kp_pre, p.kp_pre / 32, fr, fs);
    xs = acc[0][0] * p.cs_pre[16 * s + fr];
  }

  // publish xs as layer l's slice, wait for the row block's 16 slices, load the image
  auto exchange = [&](int l) -> bool {
    if (wave < 4) {  // the slice, split, into pub [plane][row][16]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = xs[i];
        amax = fmaxf(amax, fabsf(v));
        const _Float16 hh = (_Float16)v;
        const int o = (16 * mi + 4 * fs + i) * 16 + fr;
        pub[o] = hh;
        pub[HS_BM * 16 + o] = (_Float16)((v - (float)hh) * H3_SCALE);
      }
    }
    __syncthreads();
    const int par = l & 1;
    const int base = (par * RB + rb) * img_halves;  // halves
    if (tid < 256) {  // 16-B chunk (plane, row, half of the 16 channels), write-through
      const int pl = tid >> 7, row = (tid >> 1) & 63, c8 = tid & 1;
      const u32x4 v = *(const u32x4 *)(pub + (pl * HS_BM + row) * 16 + 8 * c8);
      const int off = (base + (pl * HS_BM + row) * HS_P + 16 * s + 8 * c8) * 2;
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's stores done
    __syncthreads();
    if (tid == 0) {
      unsigned *c = q.cnt + rb * HSS_CNT;
      __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = (unsigned)HSS_P * (l + 1);
      unsigned spins = 0;
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > q.spin) {
          s_abort = 1;
          if (p.status) atomicOr(p.status, FTMI_STATUS_RNN_TIMEOUT);
          break;
        }
      }
    }
    __syncthreads();
    if (s_abort) return false;
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // chunk e = (plane, row, 16-B piece of the 256 channels)
      const int e = tid + 512 * j, pl = e >> 11, row = (e >> 5) & 63, c = e & 31;
      v[j] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, (base + (pl * HS_BM + row) * HS_P + 8 * c) * 2, 0, 16 /* sc1 */);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = tid + 512 * j, pl = e >> 11, row = (e >> 5) & 63, c = e & 31;
      *(u32x4 *)(lds + pl * IMG + row * HS_P + 8 * c) = v[j];
    }
    __syncthreads();
    return true;
  };

  // ---- highways: g = sigmoid(x W2^T + b2), x <- g relu(x W1^T + b1) + (1 - g) x
  for (int l = 0; l < p.L; ++l) {
    if (!exchange(l)) return;
    if (wave < 4) {
      const int cb = s >> 1, nj = s & 1;  // the stack kernel's (column block, half)
      f32x4 acc[1][2];
      const _Float16 *bp[2] = {bptr(p.w_hw[l], 64 * cb + 16 * nj, HS_C),
                               bptr(p.w_hw[l], 64 * cb + 32 + 16 * nj, HS_C)};
      hs_gemm<2, 1>(acc, Ah, At, bp, (int64_t)2 * HS_C * HS_C, HS_C / 32, fr, fs);
      const int col = 16 * s + fr;
      const float c1 = p.cs_hw[l][64 * cb + 16 * nj + fr];
      const float c2 = p.cs_hw[l][64 * cb + 32 + 16 * nj + fr];
      const float bb1 = p.b1[l][col], bb2 = p.b2[l][col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x1, x2;
        {
#pragma clang fp contract(off)
          x1 = acc[0][0][i] * c1 + bb1;
          x2 = acc[0][1][i] * c2 + bb2;
        }
        const float g = ftmi_sigmoid(x2);
        xs[i] = highway_mix(g, x1, xs[i]);
      }
    }
  }
  if (p.h && wave < 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + 16 * mi + 4 * fs + i;
      if (row < p.M) p.h[(int64_t)row * p.h_stride + 16 * s + fr] = xs[i];
    }
  }

  // ---- output projection: columns [n_out / 16 s, + n_out / 16), two halves of NO tiles
  if (p.w_out) {
    if (!exchange(p.L)) return;
    const int n0 = (p.n_out / HSS_P) * s + (wave >> 2) * 16 * NO;
    f32x4 acc[1][NO];
    const _Float16 *bp[NO];
#pragma unroll
    for (int ni = 0; ni < NO; ++ni) bp[ni] = bptr(p.w_out, n0 + 16 * ni, HS_C);
    hs_gemm<NO, 1>(acc, Ah, At, bp, (int64_t)p.n_out * HS_C, HS_C / 32, fr, fs);
#pragma unroll
    for (int ni = 0; ni < NO; ++ni) {
      const int col = n0 + 16 * ni + fr;
      const float cs = p.cs_out[col], b = p.b_out ? p.b_out[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma clang fp contract(off)
        const int row = m0 + 16 * mi + 4 * fs + i;
        float v = acc[0][ni][i] * cs;
        if (p.b_out) v += b;
        if (row < p.M) p.y[(int64_t)row * p.y_stride + col] = v;
      }
    }
  }
  if (!(amax <= 65504.f) && p.status) atomicOr(p.status, 1u);
}

// ---- row-panel projection: y = [LayerNorm](x W^T + b [+ residual]) --------------------
// The k = 1 contractions of a FastPitch FFT block (models/fast_pitch.py:56-91, the
// reference's FFTBlock): self_attn.in_proj (K = d, N = 3d), out_proj + residual -> norm1
// (K = N = d) and conv2 (k = 1) + residual -> norm2 (K = d_fft, N = d).  At d = 256 these are
// short-K or narrow-N GEMMs: the 256 x 128 slab tiles run them at 90-170 TF/s, prologue and
// epilogue bound, and each LayerNorm is one more read + write of the rows.  Here a workgroup
// owns 64 rows: their channels are staged once per 256-channel chunk into an f16 head /
// scaled tail LDS image (the highway stack's layout and k-step code, hs_gemm_acc), the 8
// waves sweep 256-column panels (wave = 32 columns, B fragments from the L2-resident
// fragment-major planes), and the epilogue applies colscale and bias into an LDS row tile,
// then adds the residual and — for a 256-column output — runs the LayerNorm one wave per
// row with layernorm_kernel<4>'s arithmetic, writing each row once with coalesced stores.
// Per k-step, product and epilogue rounding the slab kernel's order: the projection
// values are bit-identical to conv1d's.  HBM per row: K floats in, N out (+ N residual).
constexpr int PP_BM = 64;
constexpr int PP_KC = HS_C;    // channels per staged chunk
constexpr int PP_TP = HS_C + 4;  // floats per LDS tile row (conflict-free fragment stores)

struct PanelParams {
  const float *x;
  int64_t x_stride;
  int M, K, kpad, N;
  const _Float16 *w;  // split_weights_f16_frag planes [3][N/16][kpad/32][64][8]
  const float *cs;    // their column scales
  const float *bias;
  const float *res;
  int64_t res_stride;
  const float *ln_g, *ln_b;  // LayerNorm over the N = 256 columns (null: none)
  float eps;
  float *y;
  int64_t y_stride;
  unsigned *status;
  // ftmi_panel_proj_qkv: panels 1 and 2 (K, V of the in_proj output) go to the attention
  // workspace as f16 head / scaled tail planes instead of y (ftmi_attention's layout: K
  // [B*H][Tp][hd], V transposed [B*H][hd][Tp]); rows are (b, key) = (row / T, row % T)
  _Float16 *kv;
  int T, H, hd, Tp;
};

// Persistent over row tiles (grid = min(tiles, CUs)): the next job's channels (the next
// chunk, or the next tile's first) are loaded into registers right after the current chunk
// is staged, so their HBM latency hides behind this chunk's MFMAs (the residual rows of a
// panel are issued at once ahead of its tile writes); one workgroup per CU (136 KB LDS).
__global__ __launch_bounds__(512) void panel_proj_kernel(const PanelParams p) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * HS_IMG];   // head | tail
  __shared__ __attribute__((aligned(16))) float tile[PP_BM * PP_TP];  // finished panel rows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fs = lane >> 4;
  // column block of this wave, rotated per workgroup (highway_stack_kernel: spreads the
  // concurrent B reads of one XCD over different weight lines)
  const int cb = (wave + (blockIdx.x >> 3)) & 7;
  const int ntiles = (p.M + PP_BM - 1) / PP_BM;
  const int nch = (p.kpad + PP_KC - 1) / PP_KC, nq = p.N / HS_C;
  const bool ln = p.ln_g != nullptr;
  float amax = 0.f;
  f32x4 ra[8];  // one job's channels: rows wave + 8 u, channels c0 + 4 lane .. + 3
  auto load_job = [&](int t, int c) {
    const int c0 = c * PP_KC, kc = min(PP_KC, p.kpad - c0);
    const float *xb = p.x + (int64_t)(t * PP_BM + wave) * p.x_stride + c0 + 4 * lane;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ra[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (4 * lane < kc && t * PP_BM + wave + 8 * u < p.M && c0 + 4 * lane < p.K)
        ra[u] = *(const f32x4 *)(xb + (int64_t)8 * u * p.x_stride);
    }
  };
  auto store_job = [&](int c) {  // ra -> the LDS image (f16 head / scaled tail)
    if (4 * lane >= min(PP_KC, p.kpad - c * PP_KC)) return;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x4 v = ra[u];
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      f16x4 hh, tt;
      split2h(v, hh, tt);
      const int o = (wave + 8 * u) * HS_P + 4 * lane;
      *(f16x4 *)(lds + o) = hh;
      *(f16x4 *)(lds + HS_IMG + o) = tt;
    }
  };
  // the residual of panel q, in the row pass's layout: LN — wave w rows 8w + u, columns
  // lane + 64 j (rv[u][j]); plain — rows w + 8u, columns 4 lane .. + 3 (rv[u] as a float4)
  float rv[8][4];
  auto load_res = [&](int t, int q) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = t * PP_BM + (ln ? 8 * wave + u : wave + 8 * u);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (p.res && row < p.M) {
        const float *rr = p.res + (int64_t)row * p.res_stride + HS_C * q;
        if (ln) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = rr[lane + 64 * j];
        } else {
          v = *(const f32x4 *)(rr + 4 * lane);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) rv[u][j] = v[j];
    }
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  load_job(t, 0);
#pragma unroll 1
  for (;; ) {
#pragma unroll 1
    for (int q = 0; q < nq; ++q) {
      f32x4 acc[4][2];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int c = 0; c < nch; ++c) {
        if (nch > 1 || q == 0) {  // one chunk: staged once for every panel
          __syncthreads();        // every wave is past its reads of the image
          store_job(c);
          __syncthreads();
          // the next job's channels, in flight during this chunk's MFMAs
          if (c + 1 < nch)
            load_job(t, c + 1);
          else if (nch > 1 && q + 1 < nq)
            load_job(t, 0);
          else if (t + (int)gridDim.x < ntiles)
            load_job(t + gridDim.x, 0);
        }
        const _Float16 *bp[2];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          bp[ni] = p.w + (int64_t)((HS_C * q + 32 * cb + 16 * ni) >> 4) * (p.kpad / 32) * 512 +
                   lane * 8 + 512 * (PP_KC / 32) * c;
        hs_gemm_acc<2>(acc, lds, lds + HS_IMG, bp, (int64_t)p.N * p.kpad,
                       min(PP_KC, p.kpad - c * PP_KC) / 32, fr, fs);
      }
      // ---- epilogue, the slab kernel's rounding order: t = acc colscale (+ bias) into the
      // LDS row tile, then row passes: (+ residual), [LayerNorm], coalesced stores
      load_res(t, q);  // in flight during the tile writes and the barrier
      if (q > 0) __syncthreads();  // the previous panel's row pass is done with the tile
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = HS_C * q + 32 * cb + 16 * ni + fr;
        const float cs = p.cs[col], b = p.bias ? p.bias[col] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
#pragma clang fp contract(off)
            float v = acc[mi][ni][i] * cs;
            if (p.bias) v += b;
            tile[(16 * mi + 4 * fs + i) * PP_TP + 32 * cb + 16 * ni + fr] = v;
          }
      }
      __syncthreads();
      const int m0 = t * PP_BM;
      if (p.kv && q >= 1) {  // K / V panel -> split planes (the attention split pass's values)
        const int64_t plane = (int64_t)(p.M / p.T) * p.H * p.Tp * p.hd;
        float amax = 0.f;
        if (q == 1) {  // K rows: lane = 4 consecutive columns of one head
          const int c = 4 * lane, hh = c / p.hd, d = c - hh * p.hd;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int r = wave + 8 * u, row = m0 + r;
            if (row >= p.M) continue;
            const int b = row / p.T, key = row - b * p.T;
            const f32x4 v = *(const f32x4 *)(tile + r * PP_TP + c);
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            f16x4 h4, t4;
            split2h(v, h4, t4);
            const int64_t o = ((int64_t)(b * p.H + hh) * p.Tp + key) * p.hd + d;
            *(f16x4 *)(p.kv + o) = h4;
            *(f16x4 *)(p.kv + plane + o) = t4;
          }
        } else {  // V^T: a thread takes 4 consecutive keys (rows) of one column, 8 B per plane
          // where they are 4 aligned keys of one sequence; a wave-instruction covers 16
          // columns x 4 row quads (conflict-free LDS reads at the 260-float pitch)
          for (int e = tid; e < HS_C * (PP_BM / 4); e += 512) {
            const int l = e & 63, wv = e >> 6;
            const int c = (wv & 15) * 16 + (l & 15), r0 = ((wv >> 4) * 4 + (l >> 4)) * 4;
            const int hh = c / p.hd, d = c - hh * p.hd;
            const int row0 = m0 + r0, b0 = row0 / p.T, key0 = row0 - b0 * p.T;
            f32x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = tile[(r0 + i) * PP_TP + c];
            if (row0 + 3 < p.M && key0 + 3 < p.T && (key0 & 3) == 0) {
              amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
              f16x4 h4, t4;
              split2h(v, h4, t4);
              const int64_t o = 2 * plane + ((int64_t)(b0 * p.H + hh) * p.hd + d) * p.Tp + key0;
              *(f16x4 *)(p.kv + o) = h4;
              *(f16x4 *)(p.kv + o + plane) = t4;
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int row = row0 + i;
                if (row >= p.M) break;
                const int b = row / p.T, key = row - b * p.T;
                amax = fmaxf(amax, fabsf(v[i]));
                const _Float16 h1 = (_Float16)v[i];
                const int64_t o = 2 * plane + ((int64_t)(b * p.H + hh) * p.hd + d) * p.Tp + key;
                p.kv[o] = h1;
                p.kv[o + plane] = (_Float16)((v[i] - (float)h1) * H3_SCALE);
              }
            }
          }
        }
        if (!(amax <= 65504.f) && p.status) atomicOr(p.status, 1u);
      } else if (!ln) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = wave + 8 * u, row = m0 + r;
          if (row >= p.M) continue;
          f32x4 v = *(const f32x4 *)(tile + r * PP_TP + 4 * lane);
          if (p.res) v += (f32x4){rv[u][0], rv[u][1], rv[u][2], rv[u][3]};
          *(f32x4 *)(p.y + (int64_t)row * p.y_stride + HS_C * q + 4 * lane) = v;
        }
      } else {  // one wave per row: layernorm_kernel<4>'s arithmetic (fp64 sums, same order)
        float gm[4], bt[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          gm[j] = p.ln_g[lane + 64 * j];
          bt[j] = p.ln_b[lane + 64 * j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = 8 * wave + u, row = m0 + r;
          if (row >= p.M) break;
          float v[4];
          double sm = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = tile[r * PP_TP + lane + 64 * j];
            if (p.res) v[j] += rv[u][j];
            sm += v[j];
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o);
          const double mean = sm / HS_C;
          double sq = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double d = (double)v[j] - mean;
            sq += d * d;
          }
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
          const float rstd = (float)(1.0 / sqrt(sq / HS_C + (double)p.eps));
          const float meanf = (float)mean;
          const float nb = -(rstd * meanf);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#pragma clang fp contract(off)
            p.y[(int64_t)row * p.y_stride + lane + 64 * j] = (v[j] * rstd + nb) * gm[j] + bt[j];
          }
        }
      }
    }
    t += gridDim.x;
    if (t >= ntiles) break;
  }
  if (!(amax <= 65504.f) && p.status) atomicOr(p.status, 1u);
}

static int x6_variant() {
  static const int v = [] {
    const char *e = getenv("FTMI_GEMM_X6");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// FTMI_GEMM_SLAB=0 routes the slab-eligible convolutions to the x6b kernel (A/B timing)
static bool slab_enabled() {
  static const bool v = [] {
    const char *e = getenv("FTMI_GEMM_SLAB");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// slab kernel eligibility: same-length output, Cin % 16 == 0, k taps within the slab halo,
// groups of equal width (conv bank), 32-bit activation offsets; a k = 1 GEMM only from one
// whole column tile (N >= 128: the FastPitch predictors' N = 128 projections 23.3 -> 17.2
// us at 12,800 rows; narrower Linear layers, N = 80, run faster on the 128 x 128 x6b tiles).
// FTMI_GEMM_SLAB_MIN (MACs, read per call; default 0) keeps smaller contractions on the
// x6b kernel: tests use it to cover both kernels, A/B runs to size the choice (taking
// the slab for every eligible shape measured fastest on c3: 10.01 vs 10.19 ms/step with
// an 8 GMAC bar)
constexpr int64_t SL_MIN_MACS = 0;
static int64_t slab_min_macs() {
  const char *e = getenv("FTMI_GEMM_SLAB_MIN");
  return e ? atoll(e) : SL_MIN_MACS;
}
static bool al16(const void *q) { return ((uintptr_t)q & 15u) == 0; }
static bool slab_ok(const GemmParams &p, int epi) {
  const GemmGroup &g = p.g[0];
  int64_t macs = 0;
  for (int i = 0; i < p.ngroups; ++i) macs += (int64_t)p.M * p.g[i].N * p.g[i].Ktot;
  static const int nmin = [] {  // FTMI_SLAB_K1_NMIN: narrowest k = 1 GEMM on the slab kernels
    const char *e = getenv("FTMI_SLAB_K1_NMIN");
    return e ? atoi(e) : SL_BN;
  }();
  if (!(slab_enabled() && p.To == p.T && p.Cin % 16 == 0 && (g.k > 1 || g.N >= nmin) &&
        macs >= slab_min_macs() && (int64_t)p.M * p.x_stride < ((int64_t)1 << 31)))
    return false;
  if (p.ngroups > 1 && p.split_req > 1) return false;  // the split-K finish is single-group
  for (int i = 0; i < p.ngroups; ++i) {
    const GemmGroup &gi = p.g[i];
    if (gi.k > SL_MAXK || gi.ntiles != g.ntiles || gi.N % 4) return false;
    // the epilogue moves float4s: 16-B aligned rows and per-column vectors
    if (p.y && (!al16(p.y + gi.ycol0) || p.y_stride % 4)) return false;
    if (!al16(gi.bias) || !al16(gi.scale) || !al16(gi.shift)) return false;
  }
  if (p.residual && (!al16(p.residual) || p.res_stride % 4)) return false;
  if (epi == EPI_HIGHWAY && (p.split_req > 1 || !al16(p.b1) || !al16(p.b2))) return false;
  return true;
}

// The warp-specialised slab kernel (768 threads) for multi-tap convolutions and banks,
// where the slab split is most of the staging work (measured 7-14 % faster at c3 shapes);
// the 512-thread form for k = 1 (equal or faster there).  FTMI_GEMM_SLAB_WS=0/1 forces one.
static bool slab_ws(const GemmParams &p) {
  static const int v = [] {
    const char *e = getenv("FTMI_GEMM_SLAB_WS");
    return e ? atoi(e) : -1;
  }();
  return v < 0 ? (p.g[0].k > 1 || p.ngroups > 1) : v != 0;
}

// The fragment-prefetch slab kernel for single-group k = 1 GEMMs (LSTM / GRU input
// projections: 6-10 % faster than the 512-thread slab kernel); multi-tap convolutions and
// banks keep the warp-specialised kernel (the prefetch kernel stages in its MFMA waves,
// ~200 VALU per 48 MFMAs, and measured 4-6 % slower there: DESIGN.md section 4).
// FTMI_SLAB_PF (read per call): 0 = never, 1 = every slab launch without input pooling.
static bool slab_pf_enabled(const GemmParams &p) {
  const char *e = getenv("FTMI_SLAB_PF");
  if (e) return atoi(e) != 0;
  return p.ngroups == 1 && p.g[0].k == 1;
}

static int launch_slab(const GemmParams &p, int epi, bool maxpool, hipStream_t s) {
  GemmParams q = p;
  const int nch = (q.Cin + 31) / 32;
  q.split = 1;
#ifdef FTMI_DIAG
  static const int diag = [] {
    const char *e = getenv("FTMI_SLAB_DIAG");
    return e ? atoi(e) : 0;
  }();
  q.diag = diag;
#endif
  // column bands of 2 (slab_tile): tools/gemm_one.py under rocprofv3, band 0 -> 2: c5 FFN conv
  // 1179 -> 1147 us (L2->fabric reads 913 -> 662 MB per launch), c3 prenet bank 803 -> 713,
  // postnet bank 710 -> 683, LSTM input projection 305 -> 297; proj1 (2 column tiles)
  // unchanged.  FTMI_SLAB_BAND (read per call) overrides, 0 = the row-tile order.
  const char *be = getenv("FTMI_SLAB_BAND");
  q.band = be ? atoi(be) : 2;
  q.kc_per = nch;
  if (p.split_req > 1 && p.part) {  // split over channel chunks, no empty splits
    q.kc_per = (nch + p.split_req - 1) / p.split_req;
    q.split = (nch + q.kc_per - 1) / q.kc_per;
  }
  const int TS = q.pool_out ? SL_BM - 1 : SL_BM;
  const int MT = (q.M + TS - 1) / TS;
  const int nblk = (MT < 8 ? MT : (MT + 7) / 8 * 8) * q.ngroups * q.g[0].ntiles;  // whole XCD rounds
  dim3 grid(nblk, q.split), block(512);
  if (!maxpool && slab_pf_enabled(q)) {
    if (epi == EPI_HIGHWAY)
      hipLaunchKernelGGL(conv_gemm_slabp_kernel<EPI_HIGHWAY>, grid, block, 0, s, q);
    else
      hipLaunchKernelGGL(conv_gemm_slabp_kernel<EPI_CONV>, grid, block, 0, s, q);
  } else if (slab_ws(q)) {
    block = dim3(768);
    if (epi == EPI_HIGHWAY)
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_HIGHWAY, false, true>), grid, block, 0, s, q);
    else if (maxpool)
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_CONV, true, true>), grid, block, 0, s, q);
    else
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_CONV, false, true>), grid, block, 0, s, q);
  } else {
    if (epi == EPI_HIGHWAY)
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_HIGHWAY, false, false>), grid, block, 0, s, q);
    else if (maxpool)
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_CONV, true, false>), grid, block, 0, s, q);
    else
      hipLaunchKernelGGL((conv_gemm_slab_kernel<EPI_CONV, false, false>), grid, block, 0, s, q);
  }
  FTMI_CHECK_LAUNCH();
  if (q.split > 1) {
    const int64_t total = (int64_t)q.M * q.g[0].N;
    const int eb = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(eb), dim3(256), 0, s, q);
    FTMI_CHECK_LAUNCH();
  }
  return FTMI_OK;
}

// skinny kernel eligibility (FTMI_GEMM_SKINNY=0, read per call, turns it off): few rows,
// same-length output, conv epilogue, groups of equal width, and at most SK_CPB chunks per
// block for the caller's split (partials in p.part when it splits)
static bool skinny_ok(const GemmParams &p, int epi) {
  const char *e = getenv("FTMI_GEMM_SKINNY");
  if (e && atoi(e) == 0) return false;
  // narrow single-group linears (lin / post_proj at batch 1: N = 80) up to SK_MMAX_NARROW
  // rows: the 128 x 128 tiles would give them a handful of workgroups
  // highway layers up to SK_MMAX_NARROW rows too, always through partial sums (the gating
  // pairs columns 32 apart, which the highway finish reads)
  const bool hw = epi == EPI_HIGHWAY;
  const bool narrow = p.ngroups == 1 && (p.g[0].N <= SK_BN * 2 || hw) && p.M <= SK_MMAX_NARROW;
  if ((epi != EPI_CONV && !hw) || p.To != p.T || p.Cin % 16 || p.M <= 0) return false;
  if (hw && (!p.part || p.ngroups != 1)) return false;
  if (p.M > SK_MMAX && !narrow) return false;
  for (int i = 0; i < p.ngroups; ++i)
    if (p.g[i].k > SL_MAXK || p.g[i].N != p.g[0].N || !p.g[i].w3 || !p.g[i].colscale) return false;
  const int nch = (p.Cin + 31) / 32, S = p.split_req > 1 ? p.split_req : 1;
  const int kc_per = (nch + S - 1) / S;
  if (kc_per > SK_CPB) return false;
  return (nch + kc_per - 1) / kc_per == 1 || p.part != nullptr;
}

// FTMI_BANK_BALANCED=0 (read per call) keeps a conv bank on the one-group-per-block schedule
static bool bank_balanced_enabled() {
  const char *e = getenv("FTMI_BANK_BALANCED");
  return !(e && atoi(e) == 0);
}

static int launch_skinny(const GemmParams &p, int epi, bool maxpool, hipStream_t s) {
  GemmParams q = p;
  q.force_part = epi == EPI_HIGHWAY;
  const int nch = (q.Cin + 31) / 32, S = q.split_req > 1 ? q.split_req : 1;
  q.kc_per = (nch + S - 1) / S;
  q.split = (nch + q.kc_per - 1) / q.kc_per;  // no empty splits
  const int NT = (q.g[0].N + SK_BN - 1) / SK_BN, MT = (q.M + SK_BM - 1) / SK_BM;
  q.ldp = 0;
  for (int i = 0; i < q.ngroups; ++i) {
    q.g[i].ntiles = NT;
    q.ldp = max(q.ldp, q.g[i].ycol0 + q.g[i].N);
  }
  // a CBHG bank (groups k = K .. 1, even K, 16-column multiples): the balanced schedule
  bool bank = q.ngroups >= 2 && q.ngroups % 2 == 0 && !maxpool && epi == EPI_CONV &&
              q.g[0].N % 32 == 0 && bank_balanced_enabled();
  for (int i = 0; bank && i < q.ngroups; ++i) bank = q.g[i].k == q.ngroups - i;
  if (bank) {
    dim3 grid(MT * (q.ngroups / 2) * (q.g[0].N / 32), q.split), block(512);
#ifdef FTMI_DIAG
    const char *dg = getenv("FTMI_SKINNY_DIAG");  // timing experiments (results invalid)
    switch (dg ? atoi(dg) : 0) {
#define FTMI_SK_DIAG(D_)                                                                   \
  case D_:                                                                                 \
    hipLaunchKernelGGL((conv_gemm_skinny_kernel<false, true, D_>), grid, block, 0, s, q); \
    break;
      FTMI_SK_DIAG(1) FTMI_SK_DIAG(2) FTMI_SK_DIAG(3) FTMI_SK_DIAG(4) FTMI_SK_DIAG(7)
#undef FTMI_SK_DIAG
      default:
        hipLaunchKernelGGL((conv_gemm_skinny_kernel<false, true>), grid, block, 0, s, q);
    }
#else
    if (q.T == q.M)  // one sequence: the mask-free form
      hipLaunchKernelGGL((conv_gemm_skinny_kernel<false, true, 0, true>), grid, block, 0, s, q);
    else
      hipLaunchKernelGGL((conv_gemm_skinny_kernel<false, true>), grid, block, 0, s, q);
#endif
  } else {
    dim3 grid(MT * q.ngroups * NT, q.split), block(512);
    const bool nm = q.T == q.M;  // one sequence: the mask-free form
    if (maxpool && nm)
      hipLaunchKernelGGL((conv_gemm_skinny_kernel<true, false, 0, true>), grid, block, 0, s, q);
    else if (maxpool)
      hipLaunchKernelGGL(conv_gemm_skinny_kernel<true>, grid, block, 0, s, q);
    else if (nm)
      hipLaunchKernelGGL((conv_gemm_skinny_kernel<false, false, 0, true>), grid, block, 0, s, q);
    else
      hipLaunchKernelGGL(conv_gemm_skinny_kernel<false>, grid, block, 0, s, q);
  }
  FTMI_CHECK_LAUNCH();
  if (q.force_part) {
    const int64_t n_el = (int64_t)q.M * (q.g[0].N / 2);
    const int eb = (int)((n_el + 255) / 256 < 2048 ? (n_el + 255) / 256 : 2048);
    hipLaunchKernelGGL(skinny_highway_finish_kernel, dim3(eb), dim3(256), 0, s, q);
    FTMI_CHECK_LAUNCH();
  } else if (q.split > 1) {
    const int64_t n_el = (int64_t)q.M * q.g[0].N;
    if (q.split >= 8) {  // 64 elements per 256-thread block
      const int eb = (int)((n_el + 63) / 64 < 2048 ? (n_el + 63) / 64 : 2048);
      hipLaunchKernelGGL(skinny_finish_kernel<4>, dim3(eb, q.ngroups), dim3(256), 0, s, q);
    } else {
      const int eb = (int)((n_el + 255) / 256 < 1024 ? (n_el + 255) / 256 : 1024);
      hipLaunchKernelGGL(skinny_finish_kernel<1>, dim3(eb, q.ngroups), dim3(256), 0, s, q);
    }
    FTMI_CHECK_LAUNCH();
  }
  return FTMI_OK;
}

// conv_bank_halves_kernel (FTMI_BANK_HALVES): one row tile (M <= 128), groups k = K .. 1 of
// equal 16-column-multiple widths, Cin a multiple of 64 up to 256, plain conv epilogue into
// y, the counters + sums workspace; units a multiple of 8 (the block -> (unit, half) map)
static bool bank_halves_ok(const GemmParams &p) {
  if (p.M <= 0 || p.M > 128 || p.ngroups < 2 || p.ngroups % 2 || p.To != p.T) return false;
  if (p.Cin % 64 || p.Cin > 2 * BH_MAXCH * 32) return false;
  if (!p.y || p.yt || p.residual || p.x_split || p.pool_out || p.y_split_c) return false;
  if (!p.tile_cnt || !p.part || p.g[0].N % 16) return false;
  const int units = (p.ngroups / 2) * (p.g[0].N / 16);
  if (units % 8 || units * 8 > FTMI_BANK_COUNTERS) return false;  // 8 counters per unit
  for (int i = 0; i < p.ngroups; ++i)
    if (p.g[i].k != p.ngroups - i || p.g[i].N != p.g[0].N || !p.g[i].w3 || !p.g[i].colscale)
      return false;
  return true;
}

// floats of the FTMI_BANK_HALVES workspace after the counters: [unit][half][2 MI 64 lanes][4]
static int64_t bank_halves_floats(int M, int K, int N) {
  const int MI = M <= 64 ? 4 : 8;
  return (int64_t)(K / 2) * (N / 16) * 2 * (2 * MI * 64) * 4;
}

static int launch_bank_halves(const GemmParams &p, hipStream_t s) {
  const int units = (p.ngroups / 2) * (p.g[0].N / 16);
  const dim3 grid(2 * units), block(512);
  const int nch = p.Cin / 64;
  const bool prenet = p.ngroups == 16 && p.g[0].N == 256 && nch == 4;  // c2: (KT, NCT) = (16, 16)
#ifdef FTMI_DIAG
  // timing variants of the c2 prenet bank (results invalid for some bits): diagnostic build only
  const char *dg = getenv("FTMI_BANK_HALVES_DIAG");
  const int diag = dg && prenet && p.M > 64 ? atoi(dg) : 0;  // any other value: the masked form
  if (diag && p.wimg) {
    switch (diag) {
#define FTMI_BH_DIAG(D_)                                                                          \
  case D_:                                                                                        \
    hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, D_, 16, 16, true>), grid, block, 0, s, p);    \
    break;
      FTMI_BH_DIAG(1) FTMI_BH_DIAG(2) FTMI_BH_DIAG(3) FTMI_BH_DIAG(4) FTMI_BH_DIAG(16)
      FTMI_BH_DIAG(18) FTMI_BH_DIAG(32) FTMI_BH_DIAG(128) FTMI_BH_DIAG(256) FTMI_BH_DIAG(512)
#undef FTMI_BH_DIAG
      default:
        hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, 0, 16, 16, true>), grid, block, 0, s, p);
    }
    FTMI_CHECK_LAUNCH();
    return FTMI_OK;
  }
#endif
#define FTMI_BH_NCH(MI_, PK_)                                                                            \
  switch (nch) {                                                                                         \
    case 1: hipLaunchKernelGGL((conv_bank_halves_kernel<MI_, 1, 0, 0, 0, PK_>), grid, block, 0, s, p); break; \
    case 2: hipLaunchKernelGGL((conv_bank_halves_kernel<MI_, 2, 0, 0, 0, PK_>), grid, block, 0, s, p); break; \
    case 3: hipLaunchKernelGGL((conv_bank_halves_kernel<MI_, 3, 0, 0, 0, PK_>), grid, block, 0, s, p); break; \
    default: hipLaunchKernelGGL((conv_bank_halves_kernel<MI_, 4, 0, 0, 0, PK_>), grid, block, 0, s, p);       \
  }
  if (p.wimg) {  // the stream-order weight image
    if (p.M <= 64) {
      FTMI_BH_NCH(4, true)
    } else if (prenet && p.T == p.M) {  // one sequence: the mask-free form
      hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, 0, 16, 16, true, true>), grid, block, 0, s, p);
    } else if (prenet) {
      hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, 0, 16, 16, true>), grid, block, 0, s, p);
    } else {
      FTMI_BH_NCH(8, true)
    }
  } else if (p.M <= 64) {
    FTMI_BH_NCH(4, false)
  } else if (prenet && p.T == p.M) {
    hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, 0, 16, 16, false, true>), grid, block, 0, s, p);
  } else if (prenet) {
    hipLaunchKernelGGL((conv_bank_halves_kernel<8, 4, 0, 16, 16>), grid, block, 0, s, p);
  } else {
    FTMI_BH_NCH(8, false)
  }
#undef FTMI_BH_NCH
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

// conv_bank_walk_kernel: a pooled f16x3 bank on fp32 input rows of at most 96 channels, groups
// k = K .. 1 (K <= 8, pad k / 2) of equal widths (16-column multiples), no split.
// By default only with at least BW_MIN_BLOCKS blocks (two per CU of the 256: the walk has
// one block per row and column tile, the slab kernel 16 per row tile, so a few-tile bank —
// c2's postnet, 4 row tiles — would leave the chip idle); FTMI_BANK_WALK (read per call) = 0
// never, 1 at any size.
constexpr int BW_MIN_BLOCKS = 512;
int64_t split_block_bytes(int64_t N, int64_t K, int mma);
static bool bank_walk_ok(const GemmParams &p) {
  const char *e = getenv("FTMI_BANK_WALK");
  if (e && atoi(e) == 0) return false;
  const int64_t blocks = (p.M + SL_BM - 2) / (SL_BM - 1) * ((p.g[0].N + SL_BN - 1) / SL_BN);
  if (!e && blocks < BW_MIN_BLOCKS) return false;
  if (!p.pool_out || p.x_split || p.residual || p.yt || !p.y || p.split_req > 1) return false;
  if (p.Cin <= 0 || p.Cin > BW_MAXCH * 32 || p.Cin % 16 || p.To != p.T || p.M <= 0) return false;
  if (p.T < 4 || p.ngroups < 2 || p.ngroups > BW_MAXK || p.g[0].N % SL_BN) return false;
  // the layout the kernel derives from group 0 (set_bank_groups, ftmi_split_weights_f16)
  const int NG = p.ngroups, N = p.g[0].N;
  const GemmGroup &g1 = p.g[NG - 1];  // k = 1: BN affine of column block 0
  const char *blk = (const char *)p.g[0].w3;
  for (int i = 0; i < NG; ++i) {
    const GemmGroup &g = p.g[i];
    const int k = NG - i, kp = (k * p.Cin + 31) / 32 * 32;
    if (i > 0) blk -= split_block_bytes(N, (int64_t)k * p.Cin, 2);
    if (g.k != k || g.pad != k / 2 || g.N != N || g.Kpad != kp || g.ycol0 != (k - 1) * N)
      return false;
    if ((const char *)g.w3 != blk || (const char *)g.colscale != blk + (int64_t)6 * N * kp)
      return false;
    if (g.bias || (g.scale != (g1.scale ? g1.scale + (int64_t)(k - 1) * N : nullptr)) ||
        (g.shift != (g1.scale ? g1.shift + (int64_t)(k - 1) * N : nullptr)) || !g.shift != !g.scale)
      return false;
  }
  return true;
}

static int launch_bank_walk(const GemmParams &p, hipStream_t s) {
  GemmParams q = p;
  q.g[0].ntiles = (q.g[0].N + SL_BN - 1) / SL_BN;
#ifdef FTMI_DIAG
  const char *de = getenv("FTMI_SLAB_DIAG");
  q.diag = de ? atoi(de) : 0;
#endif
  const int MT = (q.M + SL_BM - 2) / (SL_BM - 1);
  const int nblk = (MT < 8 ? MT : (MT + 7) / 8 * 8) * q.g[0].ntiles;  // whole XCD rounds
  hipLaunchKernelGGL(conv_bank_walk_kernel, dim3(nblk), dim3(512), 0, s, q);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

int launch(const GemmParams &p, int epi, bool maxpool, int nblocks, int mma, hipStream_t s) {
  if (nblocks <= 0) return FTMI_OK;
  dim3 grid(nblocks), block(256);
  bool presplit = (mma == 1 && x6_variant() != 3) || mma == 2;
  for (int i = 0; i < p.ngroups; ++i) presplit &= p.g[i].w3 != nullptr;
  if (mma == 2 && !presplit) return FTMI_E_ARG;  // the f16 path needs the split planes
  if (p.pool_out) {  // only the slab kernel pools its output
    GemmParams q = p;
    q.split_req = 0;
    q.part = nullptr;
    if (!(mma == 2 && presplit && epi == EPI_CONV && !maxpool && !p.residual && !p.yt &&
          p.y && slab_ok(q, epi)))
      return FTMI_E_UNSUPPORTED;
    if (bank_walk_ok(q)) return launch_bank_walk(q, s);
    return launch_slab(q, epi, false, s);
  }
  if (p.y_split_c) return FTMI_E_UNSUPPORTED;  // split output rows: pool_out only
  if (p.x_split) {  // split operand rows: only the slab kernel stages them
    if (!(mma == 2 && presplit && !maxpool && slab_ok(p, epi))) return FTMI_E_UNSUPPORTED;
    return launch_slab(p, epi, false, s);
  }
  if (mma == 2 && presplit && skinny_ok(p, epi)) return launch_skinny(p, epi, maxpool, s);
  if (p.ngroups > 1 && p.split_req > 1) {  // a bank split only serves the skinny kernel
    GemmParams q = p;
    q.split_req = 0;
    q.part = nullptr;
    return launch(q, epi, maxpool, nblocks, mma, s);
  }
  if (mma == 2 && slab_ok(p, epi)) return launch_slab(p, epi, maxpool, s);
  if (presplit) {
    dim3 g2(nblocks, p.split > 1 ? p.split : 1);
    if (mma == 2) {
      if (epi == EPI_HIGHWAY)
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_HIGHWAY, false, true>), g2, block, 0, s, p);
      else if (maxpool)
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_CONV, true, true>), g2, block, 0, s, p);
      else
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_CONV, false, true>), g2, block, 0, s, p);
    } else {
      if (epi == EPI_HIGHWAY)
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_HIGHWAY, false, false>), g2, block, 0, s, p);
      else if (maxpool)
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_CONV, true, false>), g2, block, 0, s, p);
      else
        hipLaunchKernelGGL((conv_gemm_x6b_kernel<EPI_CONV, false, false>), g2, block, 0, s, p);
    }
    FTMI_CHECK_LAUNCH();
    if (p.split > 1) {
      const int64_t total = (int64_t)p.M * p.g[0].N;
      const int eb = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
      hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(eb), block, 0, s, p);
      FTMI_CHECK_LAUNCH();
    }
    return FTMI_OK;
  }
  if (mma == 1 && x6_variant() == 2) {  // software-pipelined variant
    dim3 g2(nblocks, p.split > 1 ? p.split : 1);
    if (epi == EPI_HIGHWAY)
      hipLaunchKernelGGL((conv_gemm_x6p_kernel<EPI_HIGHWAY, false>), g2, block, 0, s, p);
    else if (maxpool)
      hipLaunchKernelGGL((conv_gemm_x6p_kernel<EPI_CONV, true>), g2, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_gemm_x6p_kernel<EPI_CONV, false>), g2, block, 0, s, p);
    FTMI_CHECK_LAUNCH();
    if (p.split > 1) {
      const int64_t total = (int64_t)p.M * p.g[0].N;
      const int eb = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
      hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(eb), block, 0, s, p);
      FTMI_CHECK_LAUNCH();
    }
    return FTMI_OK;
  }
  if (mma == 1 && p.split > 1) {
    dim3 g2(nblocks, p.split);
    if (maxpool)
      hipLaunchKernelGGL((conv_gemm_x6_kernel<EPI_CONV, true>), g2, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_gemm_x6_kernel<EPI_CONV, false>), g2, block, 0, s, p);
    FTMI_CHECK_LAUNCH();
    const int64_t total = (int64_t)p.M * p.g[0].N;
    const int eb = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(eb), block, 0, s, p);
    FTMI_CHECK_LAUNCH();
    return FTMI_OK;
  }
  if (mma == 1) {
    if (epi == EPI_HIGHWAY)
      hipLaunchKernelGGL((conv_gemm_x6_kernel<EPI_HIGHWAY, false>), grid, block, 0, s, p);
    else if (maxpool)
      hipLaunchKernelGGL((conv_gemm_x6_kernel<EPI_CONV, true>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_gemm_x6_kernel<EPI_CONV, false>), grid, block, 0, s, p);
    FTMI_CHECK_LAUNCH();
    return FTMI_OK;
  }
  if (epi == EPI_HIGHWAY)
    hipLaunchKernelGGL((conv_gemm_kernel<EPI_HIGHWAY, false>), grid, block, 0, s, p);
  else if (maxpool)
    hipLaunchKernelGGL((conv_gemm_kernel<EPI_CONV, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<EPI_CONV, false>), grid, block, 0, s, p);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

// bytes of one weight's pre-split block: bf16 pieces (mma = 1) or f16 planes + colscale
int64_t split_block_bytes(int64_t N, int64_t K, int mma) {
  const int64_t planes = 3 * N * ((K + X6_BK - 1) / X6_BK * X6_BK) * 2;
  return mma == 2 ? planes + (4 * N + 15) / 16 * 16 : planes;
}

void set_split(GemmGroup &g, const void *block, int mma) {
  g.w3 = (const __bf16 *)block;
  g.colscale = (block && mma == 2) ? (const float *)((const char *)block + 3LL * g.N * g.Kpad * 2)
                                   : nullptr;
}

}  // namespace

extern "C" int ftmi_conv1d(const ftmi_conv_args *a, ftmi_stream_t stream) {
  if (!a || !a->x || !a->w || (!a->y && !a->yt)) return FTMI_E_ARG;
  if (a->B <= 0 || a->T <= 0 || a->Cin <= 0 || a->N <= 0 || a->k <= 0) return FTMI_E_ARG;
  if (a->Cin % 16 != 0) return FTMI_E_SHAPE;
  if (a->mma < 0 || a->mma > 2) return FTMI_E_ARG;
  if (a->mma == 2 && !a->w_split) return FTMI_E_ARG;
  if (a->pad < 0 || a->pad >= a->k + a->T) return FTMI_E_SHAPE;
  if ((a->bn_scale == nullptr) != (a->bn_shift == nullptr)) return FTMI_E_ARG;
  if (!ftmi_aligned16(a->x) || !ftmi_aligned16(a->w) || (a->x_stride & 3)) return FTMI_E_ALIGN;
  if (a->w_split && !ftmi_aligned16(a->w_split)) return FTMI_E_ALIGN;
  const int To = a->T_out > 0 ? a->T_out : a->T;
  if ((int64_t)a->B * To > INT32_MAX) return FTMI_E_SHAPE;
  GemmParams p = {};
  p.x = a->x;
  p.x_stride = a->x_stride;
  p.B = a->B;
  p.T = a->T;
  p.To = To;
  p.Cin = a->Cin;
  p.M = a->B * To;
  p.relu = a->relu;
  p.ngroups = 1;
  p.residual = a->residual;
  p.res_stride = a->res_stride;
  p.y = a->y;
  p.y_stride = a->y_stride;
  p.yt = a->yt;
  p.yt_channels = a->N;
  p.status = a->status;
  p.x_split = a->x_split != 0;
  if (p.x_split && (a->mma != 2 || a->maxpool || a->x_stride < a->Cin))
    return FTMI_E_UNSUPPORTED;
  GemmGroup &g = p.g[0];
  g.w = a->w;
  g.Kpad = (a->k * a->Cin + X6_BK - 1) / X6_BK * X6_BK;
  g.bias = a->bias;
  g.scale = a->bn_scale;
  g.shift = a->bn_shift;
  g.N = a->N;
  g.k = a->k;
  g.pad = a->pad;
  g.Ktot = a->k * a->Cin;
  g.ycol0 = 0;
  g.ntiles = (a->N + BN - 1) / BN;
  g.tile0 = 0;
  set_split(g, a->w_split, a->mma);
  const int mtiles = (p.M + BM - 1) / BM;
  p.split = 1;
  if (a->split_k > 1) {
    if (a->mma == 0 || !a->split_ws) return FTMI_E_ARG;
    const int nkc = (g.Ktot + X6_BK - 1) / X6_BK;
    const int kc_per = (nkc + a->split_k - 1) / a->split_k;
    p.split = (nkc + kc_per - 1) / kc_per;  // no empty splits
    p.kc_per = kc_per;
    p.split_req = a->split_k;
    p.part = a->split_ws;
  }
  return launch(p, EPI_CONV, a->maxpool != 0, mtiles * g.ntiles, a->mma, ftmi_hs(stream));
}

namespace {
// the bank's groups, heaviest first (group gi has k = K - gi taps, pad k / 2, output columns
// (k - 1) Cout ..): weights, split blocks (w_split: ftmi_split_weights[_f16] blocks of
// k = 1 .. K back to back), BN affine; returns the tile count of the generic kernels
int set_bank_groups(GemmParams &p, const float *w, const void *w_split, int K, int Cout, int mma,
                    const float *bn_scale, const float *bn_shift) {
  const int Cin = p.Cin;
  const int mtiles = (p.M + BM - 1) / BM;
  const int ntiles = (Cout + BN - 1) / BN;
  int tile0 = 0;
  for (int gi = 0; gi < K; ++gi) {
    const int ks = K - gi;  // heaviest group first
    const int gidx = ks - 1;
    GemmGroup &g = p.g[gi];
    g.w = w ? w + (int64_t)Cout * Cin * gidx * (gidx + 1) / 2 : nullptr;
    g.Kpad = (ks * Cin + X6_BK - 1) / X6_BK * X6_BK;
    g.N = Cout;
    const void *blk = nullptr;
    if (w_split) {  // per-group split blocks back to back (ftmi_split_weights[_f16] layout)
      int64_t off = 0;
      for (int j = 0; j < gidx; ++j) off += split_block_bytes(Cout, (int64_t)(j + 1) * Cin, mma);
      blk = (const char *)w_split + off;
    }
    set_split(g, blk, mma);
    g.bias = nullptr;
    g.scale = bn_scale ? bn_scale + (int64_t)gidx * Cout : nullptr;
    g.shift = bn_shift ? bn_shift + (int64_t)gidx * Cout : nullptr;
    g.k = ks;
    g.pad = ks / 2;
    g.Ktot = ks * Cin;
    g.ycol0 = gidx * Cout;
    g.ntiles = ntiles;
    g.tile0 = tile0;
    tile0 += mtiles * ntiles;
  }
  return tile0;
}

// the shapes FTMI_BANK_HALVES accepts, independent of the row count
bool bank_halves_shape(int Cin, int K, int Cout) {
  return Cin > 0 && Cin % 64 == 0 && Cin <= 2 * BH_MAXCH * 32 && K >= 2 && K % 2 == 0 &&
         K <= MAX_GROUPS && Cout > 0 && Cout % 16 == 0 && ((K / 2) * (Cout / 16)) % 8 == 0 &&
         (K / 2) * (Cout / 16) * 8 <= FTMI_BANK_COUNTERS;
}
}  // namespace

extern "C" int64_t ftmi_conv_bank_halves_image_bytes(int32_t Cin, int32_t K, int32_t Cout) {
  if (!bank_halves_shape(Cin, K, Cout)) return 0;
  return bank_halves_image_halves(K, Cout, Cin) * 2 + (int64_t)K * Cout * 4;
}

extern "C" int ftmi_conv_bank_halves_image(const void *w_split, int32_t Cin, int32_t K,
                                           int32_t Cout, void *image, ftmi_stream_t stream) {
  if (!w_split || !image) return FTMI_E_ARG;
  if (!bank_halves_shape(Cin, K, Cout)) return FTMI_E_UNSUPPORTED;
  if (!ftmi_aligned16(w_split) || !ftmi_aligned16(image)) return FTMI_E_ALIGN;
  GemmParams p = {};
  p.Cin = Cin;
  p.M = 1;
  p.ngroups = K;
  set_bank_groups(p, nullptr, w_split, K, Cout, 2, nullptr, nullptr);
  p.wimg = (const _Float16 *)image;
  const hipStream_t s = ftmi_hs(stream);
  const dim3 grid(2 * (K / 2) * (Cout / 16)), block(512);
  switch (Cin / 64) {
    case 1: hipLaunchKernelGGL(bank_halves_pack_kernel<1>, grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL(bank_halves_pack_kernel<2>, grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL(bank_halves_pack_kernel<3>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(bank_halves_pack_kernel<4>, grid, block, 0, s, p);
  }
  FTMI_CHECK_LAUNCH();
  // the column scales of the groups k = 1 .. K after the weights
  char *cs = (char *)image + bank_halves_image_halves(K, Cout, Cin) * 2;
  for (int gi = 0; gi < K; ++gi) {
    const int gidx = K - 1 - gi;
    const hipError_t e = hipMemcpyAsync(cs + (int64_t)gidx * Cout * 4, p.g[gi].colscale,
                                        (size_t)Cout * 4, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return (int)e;
  }
  return FTMI_OK;
}

extern "C" int64_t ftmi_conv_bank_halves_ws_floats(int32_t B, int32_t T, int32_t K, int32_t Cout) {
  if (B <= 0 || T <= 0 || K <= 0 || Cout <= 0 || (int64_t)B * T > 128) return 0;
  return FTMI_BANK_COUNTERS + bank_halves_floats(B * T, K, Cout);
}

extern "C" int ftmi_conv_bank(const float *x, int64_t x_stride, int32_t B, int32_t T,
                              int32_t Cin, const float *w, const void *w_split, int32_t K,
                              int32_t Cout, const float *bn_scale, const float *bn_shift,
                              float *y, int64_t y_stride, int32_t mma, uint32_t *status,
                              ftmi_stream_t stream) {
  return ftmi_conv_bank_split(x, x_stride, B, T, Cin, w, w_split, K, Cout, bn_scale, bn_shift,
                              y, y_stride, mma, status, 0, nullptr, 0, stream);
}

#ifdef FTMI_SKINNY_STAMPS
extern "C" int ftmi_debug_skinny_stamps(unsigned long long *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ftmi_skinny_stamps),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" int ftmi_conv_bank_split(const float *x, int64_t x_stride, int32_t B, int32_t T,
                                    int32_t Cin, const float *w, const void *w_split, int32_t K,
                                    int32_t Cout, const float *bn_scale, const float *bn_shift,
                                    float *y, int64_t y_stride, int32_t mma, uint32_t *status,
                                    int32_t split_k, float *split_ws, int32_t pool_out,
                                    ftmi_stream_t stream) {
  if (split_k > 1 && !split_ws && !(pool_out & FTMI_BANK_POOL)) return FTMI_E_ARG;
  if (!x || !w || !bn_scale || !bn_shift || !y) return FTMI_E_ARG;
  if (B <= 0 || T <= 0 || Cin <= 0 || Cout <= 0 || K <= 0) return FTMI_E_ARG;
  if (mma < 0 || mma > 2 || (mma == 2 && !w_split)) return FTMI_E_ARG;
  if (K > MAX_GROUPS) return FTMI_E_UNSUPPORTED;
  if (Cin % 16 != 0) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || !ftmi_aligned16(w) || (x_stride & 3)) return FTMI_E_ALIGN;
  if (w_split && !ftmi_aligned16(w_split)) return FTMI_E_ALIGN;
  if ((int64_t)B * T > INT32_MAX) return FTMI_E_SHAPE;
  GemmParams p = {};
  p.x = x;
  p.x_stride = x_stride;
  p.B = B;
  p.T = T;
  p.To = T;
  p.Cin = Cin;
  p.M = B * T;
  p.relu = 1;
  p.ngroups = K;
  p.y = y;
  p.y_stride = y_stride;
  p.status = status;
  if (pool_out & ~(FTMI_BANK_POOL | FTMI_BANK_Y_SPLIT | FTMI_BANK_X_SPLIT | FTMI_BANK_HALVES |
                   FTMI_BANK_IMAGE))
    return FTMI_E_ARG;
  const bool halves = (pool_out & FTMI_BANK_HALVES) != 0;
  const bool image = (pool_out & FTMI_BANK_IMAGE) != 0;
  if (image && !halves) return FTMI_E_ARG;
  if (halves && (!split_ws || mma != 2 || (pool_out & ~(FTMI_BANK_HALVES | FTMI_BANK_IMAGE))))
    return FTMI_E_ARG;
  p.pool_out = pool_out & FTMI_BANK_POOL;
  if (pool_out & FTMI_BANK_Y_SPLIT) {  // split output rows need the pooled epilogue
    if (!p.pool_out) return FTMI_E_UNSUPPORTED;
    p.y_split_c = K * Cout;
    if (y_stride < (int64_t)K * Cout) return FTMI_E_SHAPE;
  }
  p.x_split = (pool_out & FTMI_BANK_X_SPLIT) != 0;
  if (p.x_split && mma != 2) return FTMI_E_UNSUPPORTED;
  const int tile0 = set_bank_groups(p, w, image ? nullptr : w_split, K, Cout, mma, bn_scale,
                                    bn_shift);
  if (halves) {  // one launch: channel halves, the unit's last half finishes it
    p.tile_cnt = (unsigned *)split_ws;
    p.part = split_ws + FTMI_BANK_COUNTERS;
    if (image) {  // the stream-order image: weights, then the groups' column scales
      if (!ftmi_aligned16(w_split)) return FTMI_E_ALIGN;
      p.wimg = (const _Float16 *)w_split;
      const float *cs =
          (const float *)(p.wimg + bank_halves_image_halves(K, Cout, Cin));
      for (int gi = 0; gi < K; ++gi) {
        p.g[gi].w3 = (const __bf16 *)w_split;  // (not read by the image kernel)
        p.g[gi].colscale = cs + (int64_t)(K - 1 - gi) * Cout;
      }
    }
    if (!bank_halves_ok(p)) return FTMI_E_UNSUPPORTED;
    return launch_bank_halves(p, ftmi_hs(stream));
  }
  if (split_k > 1) {
    p.split_req = split_k;
    p.part = split_ws;
  }
  return launch(p, EPI_CONV, false, tile0, mma, ftmi_hs(stream));
}

extern "C" int ftmi_highway(const float *x, int64_t x_stride, int64_t M, int32_t C,
                            const float *w12, const void *w12_split, const float *b1,
                            const float *b2, float *y, int64_t y_stride, int32_t mma,
                            uint32_t *status, ftmi_stream_t stream) {
  return ftmi_highway_split(x, x_stride, M, C, w12, w12_split, b1, b2, y, y_stride, mma,
                            status, 0, nullptr, stream);
}

extern "C" int ftmi_highway_split(const float *x, int64_t x_stride, int64_t M, int32_t C,
                                  const float *w12, const void *w12_split, const float *b1,
                                  const float *b2, float *y, int64_t y_stride, int32_t mma,
                                  uint32_t *status, int32_t split_k, float *split_ws,
                                  ftmi_stream_t stream) {
  if (!x || !w12 || !b1 || !b2 || !y) return FTMI_E_ARG;
  if (split_k >= 1 && !split_ws) return FTMI_E_ARG;
  if (M <= 0 || C <= 0) return FTMI_E_ARG;
  if (mma < 0 || mma > 2 || (mma == 2 && !w12_split)) return FTMI_E_ARG;
  if (C % 32 != 0 || C % 16 != 0) return FTMI_E_SHAPE;
  if (M > INT32_MAX) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || !ftmi_aligned16(w12) || (x_stride & 3)) return FTMI_E_ALIGN;
  if (w12_split && !ftmi_aligned16(w12_split)) return FTMI_E_ALIGN;
  if (x == y) return FTMI_E_ARG;
  GemmParams p = {};
  p.x = x;
  p.x_stride = x_stride;
  p.B = 1;
  p.T = (int)M;
  p.To = (int)M;
  p.Cin = C;
  p.M = (int)M;
  p.ngroups = 1;
  p.y = y;
  p.y_stride = y_stride;
  p.b1 = b1;
  p.b2 = b2;
  p.status = status;
  GemmGroup &g = p.g[0];
  g.w = w12;
  g.Kpad = (C + X6_BK - 1) / X6_BK * X6_BK;
  g.N = 2 * C;
  g.k = 1;
  g.pad = 0;
  g.Ktot = C;
  g.ntiles = (2 * C + BN - 1) / BN;
  g.tile0 = 0;
  set_split(g, w12_split, mma);
  const int mtiles = (p.M + BM - 1) / BM;
  if (split_k >= 1 && mma == 2 && w12_split) {  // skinny kernel: partial sums + highway finish
    GemmParams q = p;
    q.split_req = split_k;
    q.part = split_ws;
    if (skinny_ok(q, EPI_HIGHWAY)) return launch_skinny(q, EPI_HIGHWAY, false, ftmi_hs(stream));
  }
  return launch(p, EPI_HIGHWAY, false, mtiles * g.ntiles, mma, ftmi_hs(stream));
}

// f16 planes + column scales of a split_weights_f16 block [3][N][Kpad] + colscale[N]
static const float *f16_colscale(const void *w3, int64_t N, int64_t K) {
  const int64_t Kpad = (K + X6_BK - 1) / X6_BK * X6_BK;
  return (const float *)((const char *)w3 + 3 * N * Kpad * 2);
}

// the parameters of ftmi_highway_stack[_spread] (FTMI_OK or the argument error)
static int hs_params(HwStackParams &p, const float *x, int64_t x_stride, int64_t M, int32_t Cp,
                     int32_t C, const void *w_pre_split, int32_t L,
                     const void *const *w_hw_split, const float *const *b1,
                     const float *const *b2, const void *w_out_split, const float *b_out,
                     int32_t n_out, float *y, int64_t y_stride, float *h, int64_t h_stride,
                     uint32_t *status) {
  if (!x || !w_pre_split || M <= 0 || Cp <= 0 || L < 0) return FTMI_E_ARG;
  if (L > 0 && (!w_hw_split || !b1 || !b2)) return FTMI_E_ARG;
  if (w_out_split ? (!y || n_out <= 0) : (n_out != 0 || y != nullptr)) return FTMI_E_ARG;
  if (!y && !h) return FTMI_E_ARG;
  if (C != HS_C || Cp > HS_C || Cp % 4 != 0 || L > HS_MAXL) return FTMI_E_SHAPE;
  if (n_out % HS_NPASS != 0 || M > INT32_MAX) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || (x_stride & 3) || !ftmi_aligned16(w_pre_split)) return FTMI_E_ALIGN;
  if (w_out_split && !ftmi_aligned16(w_out_split)) return FTMI_E_ALIGN;
  if ((const float *)x == y || (const float *)x == h) return FTMI_E_ARG;
  p = HwStackParams{};
  p.x = x;
  p.x_stride = x_stride;
  p.M = (int)M;
  p.Cp = Cp;
  p.kp_pre = (Cp + X6_BK - 1) / X6_BK * X6_BK;
  p.w_pre = (const _Float16 *)w_pre_split;
  p.cs_pre = f16_colscale(w_pre_split, C, Cp);
  p.L = L;
  for (int l = 0; l < L; ++l) {
    if (!w_hw_split[l] || !b1[l] || !b2[l] || !ftmi_aligned16(w_hw_split[l])) return FTMI_E_ARG;
    p.w_hw[l] = (const _Float16 *)w_hw_split[l];
    p.cs_hw[l] = f16_colscale(w_hw_split[l], 2 * C, C);
    p.b1[l] = b1[l];
    p.b2[l] = b2[l];
  }
  if (w_out_split) {
    p.w_out = (const _Float16 *)w_out_split;
    p.cs_out = f16_colscale(w_out_split, n_out, C);
    p.b_out = b_out;
    p.n_out = n_out;
    p.y = y;
    p.y_stride = y_stride;
  }
  p.h = h;
  p.h_stride = h_stride;
  p.status = status;
  return FTMI_OK;
}

extern "C" int ftmi_highway_stack(const float *x, int64_t x_stride, int64_t M, int32_t Cp,
                                  int32_t C, const void *w_pre_split, int32_t L,
                                  const void *const *w_hw_split, const float *const *b1,
                                  const float *const *b2, const void *w_out_split,
                                  const float *b_out, int32_t n_out, float *y, int64_t y_stride,
                                  float *h, int64_t h_stride, uint32_t *status,
                                  ftmi_stream_t stream) {
  HwStackParams p;
  const int rc = hs_params(p, x, x_stride, M, Cp, C, w_pre_split, L, w_hw_split, b1, b2,
                           w_out_split, b_out, n_out, y, y_stride, h, h_stride, status);
  if (rc != FTMI_OK) return rc;
  // 96 rows per workgroup once the grid still fills the chip (FTMI_HS_BM = 64 / 96, read per
  // call, forces one; 128 rows would need ~290 VGPRs and spills)
  const char *e = getenv("FTMI_HS_BM");
  const int bm = e ? atoi(e) : (M >= 96 * 256 ? 96 : 64);
  if (bm == 96) {
    const unsigned blocks = (unsigned)((M + 95) / 96);
    hipLaunchKernelGGL(highway_stack_kernel<96>, dim3(blocks), dim3(512), 0, ftmi_hs(stream), p);
  } else {
    const unsigned blocks = (unsigned)((M + HS_BM - 1) / HS_BM);
    hipLaunchKernelGGL(highway_stack_kernel<64>, dim3(blocks), dim3(512), 0, ftmi_hs(stream), p);
  }
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int64_t ftmi_highway_stack_spread_ws_bytes(int64_t M) {
  if (M <= 0 || M > (int64_t)HSS_MAXRB * HS_BM) return 0;
  const int64_t RB = (M + HS_BM - 1) / HS_BM;
  return RB * HSS_CNT * 4 + 2 * RB * 2 * HS_BM * HS_P * 2;
}

extern "C" int32_t ftmi_highway_stack_spread_blocks(int64_t M) {
  if (M <= 0 || M > (int64_t)HSS_MAXRB * HS_BM) return 0;
  return (int32_t)((M + HS_BM - 1) / HS_BM * HSS_P);
}

extern "C" int ftmi_highway_stack_spread(const float *x, int64_t x_stride, int64_t M, int32_t Cp,
                                         int32_t C, const void *w_pre_split, int32_t L,
                                         const void *const *w_hw_split, const float *const *b1,
                                         const float *const *b2, const void *w_out_split,
                                         const float *b_out, int32_t n_out, float *y,
                                         int64_t y_stride, float *h, int64_t h_stride,
                                         uint32_t *status, void *ws, ftmi_stream_t stream) {
  HwStackParams p;
  const int rc = hs_params(p, x, x_stride, M, Cp, C, w_pre_split, L, w_hw_split, b1, b2,
                           w_out_split, b_out, n_out, y, y_stride, h, h_stride, status);
  if (rc != FTMI_OK) return rc;
  if (!ws) return FTMI_E_ARG;
  if (!ftmi_aligned16(ws)) return FTMI_E_ALIGN;
  const int blocks = ftmi_highway_stack_spread_blocks(M);
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  // every workgroup resident at once (they wait on each other); n_out split in two halves
  // of n_out / 512 16-column tiles per slice
  if (blocks <= 0 || blocks > cus || (w_out_split && n_out > 3 * HS_NPASS)) return FTMI_E_UNSUPPORTED;
  {
    const int nk = w_out_split ? n_out / HS_NPASS : 1;
    const void *k = nk == 1 ? (const void *)highway_spread_kernel<1>
                  : nk == 2 ? (const void *)highway_spread_kernel<2>
                            : (const void *)highway_spread_kernel<3>;
    if (int rc2 = ftmi_resident_ok(k, blocks, 512, 0)) return rc2;
  }
  const int RB = blocks / HSS_P;
  HsSpread q;
  q.cnt = (unsigned *)ws;
  q.xb = (_Float16 *)((char *)ws + (int64_t)RB * HSS_CNT * 4);
  q.spin = 1u << 22;
  hipStream_t s = ftmi_hs(stream);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)RB * HSS_CNT * 4, s);
  if (e != hipSuccess) return (int)e;
  switch (w_out_split ? n_out / HS_NPASS : 1) {
    case 1: hipLaunchKernelGGL(highway_spread_kernel<1>, dim3(blocks), dim3(512), 0, s, p, q); break;
    case 2: hipLaunchKernelGGL(highway_spread_kernel<2>, dim3(blocks), dim3(512), 0, s, p, q); break;
    default: hipLaunchKernelGGL(highway_spread_kernel<3>, dim3(blocks), dim3(512), 0, s, p, q);
  }
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

static int panel_launch(PanelParams &p, int64_t M, hipStream_t stream) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const int64_t tiles = (M + PP_BM - 1) / PP_BM;
  const unsigned blocks = (unsigned)(tiles < cus ? tiles : cus);
  hipLaunchKernelGGL(panel_proj_kernel, dim3(blocks), dim3(512), 0, stream, p);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_panel_proj_qkv(const float *x, int64_t x_stride, int32_t B, int32_t T,
                                   int32_t K, const void *w_split_frag, int32_t d,
                                   const float *bias, int32_t heads, float *q_out,
                                   int64_t q_stride, void *kv_workspace, int64_t workspace_bytes,
                                   uint32_t *status, ftmi_stream_t stream) {
  if (!x || !w_split_frag || !q_out || !kv_workspace || B <= 0 || T <= 0 || K <= 0) return FTMI_E_ARG;
  if (d != HS_C || heads <= 0 || d % heads) return FTMI_E_SHAPE;
  const int hd = d / heads;
  if (hd != 64 && hd != 128) return FTMI_E_UNSUPPORTED;
  const int64_t M = (int64_t)B * T;
  if (K % 4 || M > INT32_MAX || x_stride < K || q_stride < d) return FTMI_E_SHAPE;
  if (workspace_bytes < ftmi_attention_workspace_bytes(B, T, heads, hd)) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || (x_stride & 3) || !ftmi_aligned16(w_split_frag) ||
      !ftmi_aligned16(q_out) || (q_stride & 3) || !ftmi_aligned16(kv_workspace))
    return FTMI_E_ALIGN;
  if ((const float *)x == q_out) return FTMI_E_ARG;
  PanelParams p = {};
  p.x = x;
  p.x_stride = x_stride;
  p.M = (int)M;
  p.K = K;
  p.kpad = (K + X6_BK - 1) / X6_BK * X6_BK;
  p.N = 3 * d;
  p.w = (const _Float16 *)w_split_frag;
  p.cs = f16_colscale(w_split_frag, 3 * d, K);
  p.bias = bias;
  p.y = q_out;
  p.y_stride = q_stride;
  p.status = status;
  p.kv = (_Float16 *)kv_workspace;
  p.T = T;
  p.H = heads;
  p.hd = hd;
  p.Tp = (T + 63) / 64 * 64;
  return panel_launch(p, M, ftmi_hs(stream));
}

extern "C" int ftmi_panel_proj(const float *x, int64_t x_stride, int64_t M, int32_t K,
                               const void *w_split_frag, int32_t N, const float *bias,
                               const float *residual, int64_t res_stride, const float *ln_gamma,
                               const float *ln_beta, float eps, float *y, int64_t y_stride,
                               uint32_t *status, ftmi_stream_t stream) {
  if (!x || !w_split_frag || !y || M < 0 || K <= 0 || N <= 0) return FTMI_E_ARG;
  if (!ln_gamma != !ln_beta) return FTMI_E_ARG;
  if (K % 4 || N % HS_C || (ln_gamma && N != HS_C) || M > INT32_MAX) return FTMI_E_SHAPE;
  if (x_stride < K || y_stride < N || (residual && res_stride < N)) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || (x_stride & 3) || !ftmi_aligned16(w_split_frag)) return FTMI_E_ALIGN;
  // the rows of x are re-read after other workgroups' rows of y are written (chunks,
  // panels): no aliasing; y may alias the residual (each element read before its write)
  if ((const float *)x == y) return FTMI_E_ARG;
  if (M == 0) return FTMI_OK;
  PanelParams p = {};
  p.x = x;
  p.x_stride = x_stride;
  p.M = (int)M;
  p.K = K;
  p.kpad = (K + X6_BK - 1) / X6_BK * X6_BK;
  p.N = N;
  p.w = (const _Float16 *)w_split_frag;
  p.cs = f16_colscale(w_split_frag, N, K);
  p.bias = bias;
  p.res = residual;
  p.res_stride = res_stride;
  p.ln_g = ln_gamma;
  p.ln_b = ln_beta;
  p.eps = eps;
  p.y = y;
  p.y_stride = y_stride;
  p.status = status;
  return panel_launch(p, M, ftmi_hs(stream));
}

extern "C" int64_t ftmi_split_weights_f16_bytes(int64_t N, int64_t K) {
  return split_block_bytes(N, K, 2);
}

static int split_f16(const float *w, int64_t N, int64_t K, void *out, int frag,
                     ftmi_stream_t stream) {
  if (!w || !out || N <= 0 || K <= 0) return FTMI_E_ARG;
  if (N > INT32_MAX || (frag && N % 16 != 0)) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(out)) return FTMI_E_ALIGN;
  const int64_t Kpad = (K + X6_BK - 1) / X6_BK * X6_BK;
  hipLaunchKernelGGL(split_weights_f16_kernel, dim3((unsigned)N), dim3(256), 0, ftmi_hs(stream), w,
                     N, K, Kpad, (_Float16 *)out,
                     (float *)((char *)out + 3 * N * Kpad * 2), frag);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_split_weights_f16(const float *w, int64_t N, int64_t K, void *out,
                                      ftmi_stream_t stream) {
  return split_f16(w, N, K, out, 0, stream);
}

extern "C" int ftmi_split_weights_f16_frag(const float *w, int64_t N, int64_t K, void *out,
                                           ftmi_stream_t stream) {
  return split_f16(w, N, K, out, 1, stream);
}

extern "C" int ftmi_split_rows(const float *x, int64_t x_stride, int64_t rows, int32_t C,
                               float *y, int64_t y_stride, uint32_t *status,
                               ftmi_stream_t stream) {
  if (!x || !y || rows < 0 || C <= 0) return FTMI_E_ARG;
  if (C % 4 || x_stride < C || y_stride < C) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(x) || (x_stride & 3) || !ftmi_aligned16(y) || (y_stride & 3))
    return FTMI_E_ALIGN;
  if ((void *)x == (void *)y) return FTMI_E_ARG;  // rows are rewritten in another layout
  const int64_t n = rows * (C / 4);
  if (n == 0) return FTMI_OK;
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     ftmi_hs(stream), x, x_stride, rows, C, y, y_stride, status);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_split_weights(const float *w, int64_t N, int64_t K, void *out,
                                  ftmi_stream_t stream) {
  if (!w || !out || N <= 0 || K <= 0) return FTMI_E_ARG;
  if (!ftmi_aligned16(out)) return FTMI_E_ALIGN;
  const int64_t Kpad = (K + X6_BK - 1) / X6_BK * X6_BK;
  const int64_t total = N * Kpad;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(split_weights_kernel, dim3(blocks), dim3(256), 0, ftmi_hs(stream), w, N, K,
                     Kpad, (__bf16 *)out);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int64_t ftmi_split_weights_bytes(int64_t N, int64_t K) {
  return 3 * N * ((K + X6_BK - 1) / X6_BK * X6_BK) * 2;
}
