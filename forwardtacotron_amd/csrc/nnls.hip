// The reference's mel pseudo-inverse, reproduced on gfx950: librosa 0.7.2 util.nnls
// (feature.inverse.mel_to_stft, called by utils/dsp.py:91-102) minimises 0.5||A X - M||^2,
// X >= 0, per block of 127 frames with scipy.optimize.fmin_l_bfgs_b (L-BFGS-B 3.0, history
// m = n_bins, pgtol 1e-5, factr 1e7, 20 line-search steps), started from the float32
// least-squares solution clipped at 0.  This file runs that algorithm — not another solver
// with the same objective: the minimiser is not unique (80 equations, 513 unknowns per
// frame), so only the same iterates give the reference's magnitudes.
//
// Every routine below restates one of L-BFGS-B 3.0's (lbfgsb.f / scipy's __lbfgsb.c, lower
// bound 0 on every variable, nbd = 1): projgr, cauchy (generalized Cauchy point with the
// breakpoints taken in increasing order), freev, formk (the incremental WN1 update and the
// two Cholesky factors), cmprlb, subsm (with the 3.0 projection / backtrack), lnsrlb +
// dcsrch / dcstep (More'-Thuente), matupd, formt, bmv.  Arithmetic is float64 throughout, in
// the reference's expression order (fp contract off); the inner products are sums in a
// different order than BLAS's, so the iterates agree to rounding, not bit for bit.
//
// Execution (one "block" = one 127-frame L-BFGS-B problem, n = 513 x frames variables):
// a per-block state machine advanced by seven phase kernels that the host issues in a cycle
// (ftmi_nnls_lbfgsb_cycles) — EVAL (f, g at a line-search trial), CAUCHY (the update of the
// previous iteration + the Cauchy sweep), WALK (breakpoints in order until the GCP), FREEV
// (free set, WN1's new row, cmprlb's r, subsm's W'Zr), FORMK (entering / leaving terms, the
// factorisation of the middle matrix), SUBSM (the subspace step, projection, line-search set-up)
// and BACKTRACK.  A kernel only acts on the blocks whose state names its phase.  The sweeps
// run over G workgroups per block (each a contiguous range of frames); their partial sums go
// to per-workgroup slots and the LAST workgroup to arrive (agent-scope counter) reduces them
// in workgroup order (deterministic) and runs the phase's scalar part.  Vectors live in a
// caller workspace (HBM); the history S / Y as [m][n] rows.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr double EPSMCH = 2.220446049250313e-16;
constexpr double PGTOL = 1e-5;
constexpr double FTOL_FACTR = 1e7 * EPSMCH;  // factr * epsmch
constexpr int MAXLS = 20;
constexpr int NT = 256;         // threads per workgroup, every phase kernel
constexpr int NW = NT / 64;
constexpr int CAP = 1024;       // breakpoints sorted per walk chunk
constexpr int KCHUNK = 256;     // target chunk size
constexpr int MC = 32;          // history columns whose small matrices the scalar parts stage in LDS
constexpr int MMAX = 513;       // history columns at most (the reference's m = n_bins for n_fft 1024)

enum Phase { PH_DONE = 0, PH_EVAL = 1, PH_CAUCHY = 2, PH_WALK = 3, PH_FREEV = 4, PH_FORMK = 5,
             PH_SUBSM = 6, PH_BACKTRACK = 7 };
// status bits (NnlsState::status)
enum { ST_CONV = 1, ST_ABNORMAL = 2, ST_MEMCAP = 4, ST_TIES = 8, ST_MAXITER = 16 };

struct NnlsState {
  double f, fold, sbgnrm, theta, f1, f2, f2_org, dtm, tsum, tj, stp, dtd, dnorm, stpmx;
  double gd, gdold, rr, dr, alpha;
  // dcsrch
  double ls_finit, ls_ginit, ls_gtest, ls_width, ls_width1, ls_stx, ls_fx, ls_gx, ls_sty,
      ls_fy, ls_gy, ls_stmin, ls_stmax, ls_stpmax;
  int phase, it, col, iupdat, updatd, pending, nbreak, nfree_c, bnded, kpassed, nfree, nenter,
      nleave, iword, ibd, ifun, ls_brackt, ls_stage, cur, status, nfev, nskip, nseg,
      walk_done, bk_count, backtrack;
  unsigned arrive;
};

struct Args {
  const float *mel;   // (B, n_mels, F) (log mel if denorm)
  int B, F, n_mels, nb, denorm;
  const int32_t *blocks;  // [n_blocks][4]: item, first frame, frames, 0
  int n_blocks, groups, m, mref, ncmax, maxiter, dbg_stop;
  const float *rowvals;
  const int32_t *rowptr, *rowlo, *bin_rows;
  const float *bin_w;
  const double *pinv;  // [nb][n_mels] float64
  unsigned char *ws;
  int64_t blk_bytes;   // workspace bytes per block
  int64_t n_pad;
  float *S;            // (B, F, nb)
  int *active;         // device: number of blocks not done
};

// ---- per-block workspace views ----------------------------------------------------------
struct Blk {
  NnlsState *st;
  double *X[2], *G[2], *Z, *DD, *R, *WS, *WY;
  unsigned long long *BKEY;
  int32_t *BIDX, *CHG;
  int8_t *IW, *PF;
  double *SY, *SS, *WT, *WN1, *WN, *P, *C, *WA, *WV, *V, *WBP, *NEWROW, *PART, *DELTA;
  int item, f0, nc, n;
};

__host__ __device__ inline int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }
// partial-sum slots per workgroup: 6 per history column in blocks of 8, plus 16 scalars
__host__ __device__ inline int nslots(int m) { return 6 * ((m + 7) / 8 * 8) + 16; }

// one block's workspace, carved in a fixed order (the same walk sizes it on the host:
// base = nullptr, v = nullptr)
__host__ __device__ inline int64_t carve(unsigned char *base, int64_t n_pad, int m, int groups,
                                         Blk *v) {
  int64_t o = 0;
  const int64_t m2 = 2 * m;
  auto take = [&](int64_t sz) {
    unsigned char *r = base + o;
    o += align256(sz);
    return r;
  };
  Blk t;
  t.st = (NnlsState *)take(sizeof(NnlsState));
  t.X[0] = (double *)take(8 * n_pad);
  t.X[1] = (double *)take(8 * n_pad);
  t.G[0] = (double *)take(8 * n_pad);
  t.G[1] = (double *)take(8 * n_pad);
  t.Z = (double *)take(8 * n_pad);
  t.DD = (double *)take(8 * n_pad);
  t.R = (double *)take(8 * n_pad);
  t.WS = (double *)take(8 * n_pad * m);
  t.WY = (double *)take(8 * n_pad * m);
  t.BKEY = (unsigned long long *)take(8 * n_pad);
  t.BIDX = (int32_t *)take(4 * n_pad);
  t.CHG = (int32_t *)take(4 * n_pad);
  t.IW = (int8_t *)take(n_pad);
  t.PF = (int8_t *)take(n_pad);
  t.SY = (double *)take(8LL * m * m);
  t.SS = (double *)take(8LL * m * m);
  t.WT = (double *)take(8LL * m * m);
  t.WN1 = (double *)take(8 * m2 * m2);
  t.WN = (double *)take(8 * m2 * m2);
  t.P = (double *)take(8 * m2);
  t.C = (double *)take(8 * m2);
  t.WA = (double *)take(8 * m2);
  t.WV = (double *)take(8 * m2);
  t.V = (double *)take(8 * m2);
  t.WBP = (double *)take(8 * m2);
  t.NEWROW = (double *)take(8LL * 4 * m);
  t.PART = (double *)take(8LL * groups * nslots(m));
  t.DELTA = (double *)take(8LL * 6 * m * m);
  if (v) *v = t;
  return o;
}

__device__ inline double *xbuf(const Blk &b, int i) { return i ? b.X[1] : b.X[0]; }
__device__ inline double *gbuf(const Blk &b, int i) { return i ? b.G[1] : b.G[0]; }

__device__ inline Blk blk_view(const Args &a, int blk) {
  Blk v;
  carve(a.ws + (int64_t)blk * a.blk_bytes, a.n_pad, a.m, a.groups, &v);
  const int32_t *bt = a.blocks + 4 * blk;
  v.item = bt[0];
  v.f0 = bt[1];
  v.nc = bt[2];
  v.n = v.nc * a.nb;
  return v;
}

// ---- reductions ----------------------------------------------------------------------------
__device__ inline double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
// (value, index) minimum, ties to the smaller index
__device__ inline void wave_argmin(double &v, int &i) {
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o);
    const int oi = __shfl_xor(i, o);
    if (ov < v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}

// workgroup sums of `cnt` per-thread values acc[0..cnt) into out[0..cnt) (out in global
// memory, written by thread 0..cnt-1 after the barrier); red: LDS of NW * cnt doubles
template <int CNT>
__device__ inline void wg_sums(const double (&acc)[CNT], int cnt, double *red, double *out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    if (j < cnt) {
      const double s = wave_sum(acc[j]);
      if (lane == 0) red[j * NW + w] = s;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < cnt; j += NT) {
    double s = 0.0;
    for (int q = 0; q < NW; ++q) s += red[j * NW + q];
    out[j] = s;
  }
  __syncthreads();
}

// the calling workgroup's element range [e0, e1) of the block, whole frames
__device__ inline void wg_range(const Blk &b, int nb, int groups, int g, int &fl0, int &fl1) {
  fl0 = (int)((int64_t)b.nc * g / groups);
  fl1 = (int)((int64_t)b.nc * (g + 1) / groups);
}

// last workgroup of the block to finish this phase? (all partials visible to it)
__device__ inline bool arrive_last(NnlsState *st, int groups) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == (unsigned)groups - 1);
    if (last) {
      __hip_atomic_store(&st->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
    }
  }
  __syncthreads();
  return last;
}

// ---- L-BFGS-B small-matrix routines (single thread; matrices row-major [i][j] = A(i, j)) --
// bmv: product of the 2col x 2col middle matrix M with v (lbfgsb.f bmv); wt holds the
// upper Cholesky factor J' of T = theta S'S + L D^-1 L'.  Returns false on a zero pivot.
__device__ bool bmv(int m, int col, const double *sy, const double *wt, const double *v,
                    double *p) {
  if (col == 0) return true;
  p[col] = v[col];
  for (int i = 1; i < col; ++i) {
    double sum = 0.0;
    for (int k = 0; k < i; ++k) sum = sum + sy[i * m + k] * v[k] / sy[k * m + k];
    p[col + i] = v[col + i] + sum;
  }
  // solve J' ^T x = p2 (dtrsl job 11: trans(wt) x = b, wt upper)
  for (int i = 0; i < col; ++i) {
    double s = p[col + i];
    for (int k = 0; k < i; ++k) s = s - wt[k * m + i] * p[col + k];
    if (wt[i * m + i] == 0.0) return false;
    p[col + i] = s / wt[i * m + i];
  }
  for (int i = 0; i < col; ++i) p[i] = v[i] / sqrt(sy[i * m + i]);
  // solve J' x = p2 (job 01)
  for (int i = col - 1; i >= 0; --i) {
    double s = p[col + i];
    for (int k = i + 1; k < col; ++k) s = s - wt[i * m + k] * p[col + k];
    p[col + i] = s / wt[i * m + i];
  }
  for (int i = 0; i < col; ++i) p[i] = -p[i] / sqrt(sy[i * m + i]);
  for (int i = 0; i < col; ++i) {
    double sum = 0.0;
    for (int k = i + 1; k < col; ++k) sum = sum + sy[k * m + i] * p[col + k] / sy[i * m + i];
    p[i] = p[i] + sum;
  }
  return true;
}

// dpofa: upper Cholesky factor of the leading n x n of a (leading dimension ld) in place;
// false if not positive definite
__device__ bool dpofa(double *a, int ld, int n) {
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int k = 0; k < j; ++k) {
      double t = a[k * ld + j];
      for (int i = 0; i < k; ++i) t = t - a[i * ld + k] * a[i * ld + j];
      t = t / a[k * ld + k];
      a[k * ld + j] = t;
      s = s + t * t;
    }
    s = a[j * ld + j] - s;
    if (s <= 0.0) return false;
    a[j * ld + j] = sqrt(s);
  }
  return true;
}

// dtrsl on an upper triangular a (ld): job 11 solves trans(a) x = b, job 01 solves a x = b
__device__ bool trsl_t(const double *a, int ld, int n, double *b) {
  for (int j = 0; j < n; ++j) {
    double s = b[j];
    for (int k = 0; k < j; ++k) s = s - a[k * ld + j] * b[k];
    if (a[j * ld + j] == 0.0) return false;
    b[j] = s / a[j * ld + j];
  }
  return true;
}
__device__ bool trsl_n(const double *a, int ld, int n, double *b) {
  for (int j = n - 1; j >= 0; --j) {
    double s = b[j];
    for (int k = j + 1; k < n; ++k) s = s - a[j * ld + k] * b[k];
    if (a[j * ld + j] == 0.0) return false;
    b[j] = s / a[j * ld + j];
  }
  return true;
}

// the leading col x col of a (leading dimension lda) into a compact LDS copy (all threads)
__device__ inline void stage_in(double *dst, const double *src, int lda, int col) {
  for (int i = threadIdx.x; i < col * col; i += NT) {
    const int r = i / col, c = i - r * col;
    dst[i] = src[r * lda + c];
  }
}
__device__ inline void stage_out(double *dst, int lda, const double *src, int col) {
  for (int i = threadIdx.x; i < col * col; i += NT) {
    const int r = i / col, c = i - r * col;
    dst[r * lda + c] = src[i];
  }
}

// formt: T = theta S'S + L D^-1 L' (upper) and its Cholesky factor into wt
__device__ bool formt(int m, int col, const double *sy, const double *ss, double theta,
                      double *wt) {
  for (int j = 0; j < col; ++j) wt[j] = theta * ss[j];
  for (int i = 1; i < col; ++i)
    for (int j = i; j < col; ++j) {
      const int k1 = (i < j ? i : j);
      double ddum = 0.0;
      for (int k = 0; k < k1; ++k) ddum = ddum + sy[i * m + k] * sy[j * m + k] / sy[k * m + k];
      wt[i * m + j] = ddum + theta * ss[i * m + j];
    }
  return dpofa(wt, m, col);
}


// ---- wave- / workgroup-parallel forms of the small-matrix routines (long histories: the
// serial forms above are O(col^2) / O(col^3) chains of dependent loads).  Same operations in
// the same order per element (column-oriented substitution subtracts in the reference's k
// order); the right-looking Cholesky reduces each entry in the same j order as dpofa's ddot.
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// element j of a lane-strided register vector (element k lives in lane k % 64, slot k / 64)
template <int NPL>
__device__ inline double wget(const double (&r)[NPL], int j) {
  const int u = j >> 6;
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (q == u) v = r[q];
  return __shfl(v, j & 63);
}

// trans(U) x = b, U upper (dtrsl job 11), x lane-strided in registers; false on a zero pivot
template <int NPL>
__device__ bool wtrsl_t(const double *U, int ld, int n, double (&x)[NPL]) {
  const int lane = threadIdx.x & 63;
  for (int j = 0; j < n; ++j) {
    const double d = U[j * ld + j];
    if (d == 0.0) return false;
    const double xj = wget<NPL>(x, j) / d;
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      const int k = lane + 64 * q;
      if (k == j) x[q] = xj;
      else if (k > j && k < n) x[q] = x[q] - U[j * ld + k] * xj;
    }
  }
  return true;
}

// U x = b, U upper (dtrsl job 01)
template <int NPL>
__device__ bool wtrsl_n(const double *U, int ld, int n, double (&x)[NPL]) {
  const int lane = threadIdx.x & 63;
  for (int j = n - 1; j >= 0; --j) {
    const double d = U[j * ld + j];
    if (d == 0.0) return false;
    const double xj = wget<NPL>(x, j) / d;
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      const int k = lane + 64 * q;
      if (k == j) x[q] = xj;
      else if (k < j) x[q] = x[q] - U[k * ld + j] * xj;
    }
  }
  return true;
}

// bmv by one wave: p = M v (all 64 lanes call it; v and p in memory, 2 col entries)
template <int NPL>
__device__ bool wbmv_t(int ld, int col, const double *sy, const double *wt, const double *v,
                       double *p) {
  const int lane = threadIdx.x & 63;
  double a[NPL], bq[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int i = lane + 64 * q;
    a[q] = bq[q] = 0.0;
    if (i < col) {
      double sum = 0.0;
      for (int k = 0; k < i; ++k) sum = sum + sy[i * ld + k] * v[k] / sy[k * ld + k];
      a[q] = (i == 0) ? v[col] : v[col + i] + sum;
      bq[q] = v[i] / sqrt(sy[i * ld + i]);
    }
  }
  if (!wtrsl_t<NPL>(wt, ld, col, a)) return false;
  if (!wtrsl_n<NPL>(wt, ld, col, a)) return false;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int i = lane + 64 * q;
    if (i < col) bq[q] = -bq[q] / sqrt(sy[i * ld + i]);
  }
  // p1_i += sum_{k > i} sy(k, i) p2_k / sy(i, i), k ascending
  double sums[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) sums[q] = 0.0;
  for (int k = 1; k < col; ++k) {
    const double p2k = wget<NPL>(a, k);
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      const int i = lane + 64 * q;
      if (i < k) sums[q] = sums[q] + sy[k * ld + i] * p2k / sy[i * ld + i];
    }
  }
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int i = lane + 64 * q;
    if (i < col) {
      p[i] = bq[q] + sums[q];
      p[col + i] = a[q];
    }
  }
  wave_sync();
  return true;
}

__device__ bool wbmv(int ld, int col, const double *sy, const double *wt, const double *v, double *p) {
  if (col == 0) return true;
  if (col <= 64) return wbmv_t<1>(ld, col, sy, wt, v, p);
  if (col <= 128) return wbmv_t<2>(ld, col, sy, wt, v, p);
  if (col <= 256) return wbmv_t<4>(ld, col, sy, wt, v, p);
  return wbmv_t<9>(ld, col, sy, wt, v, p);
}

// trans(U) x = b then U y = x' with the first `neg` entries of x negated in between (subsm's
// K^-1: dtrsl 11, negate, dtrsl 01), x in memory (2 col entries), one wave
template <int NPL>
__device__ bool wsolve_k_t(const double *U, int ld, int n, int neg, double *x) {
  const int lane = threadIdx.x & 63;
  double r[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int k = lane + 64 * q;
    r[q] = k < n ? x[k] : 0.0;
  }
  if (!wtrsl_t<NPL>(U, ld, n, r)) return false;
#pragma unroll
  for (int q = 0; q < NPL; ++q)
    if (lane + 64 * q < neg) r[q] = -r[q];
  if (!wtrsl_n<NPL>(U, ld, n, r)) return false;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int k = lane + 64 * q;
    if (k < n) x[k] = r[q];
  }
  wave_sync();
  return true;
}
__device__ bool wsolve_k(const double *U, int ld, int n, int neg, double *x) {
  if (n <= 64) return wsolve_k_t<1>(U, ld, n, neg, x);
  if (n <= 128) return wsolve_k_t<2>(U, ld, n, neg, x);
  if (n <= 256) return wsolve_k_t<4>(U, ld, n, neg, x);
  if (n <= 512) return wsolve_k_t<8>(U, ld, n, neg, x);
  return wsolve_k_t<17>(U, ld, n, neg, x);
}

// dpofa by the whole workgroup (right-looking); every thread gets the same result
__device__ bool wg_dpofa(double *a, int ld, int n) {
  __shared__ int fail;
  for (int j = 0; j < n; ++j) {
    if (threadIdx.x == 0) {
      const double d = a[j * ld + j];
      fail = !(d > 0.0);
      if (!fail) a[j * ld + j] = sqrt(d);
    }
    __syncthreads();
    if (fail) return false;
    const double piv = a[j * ld + j];
    for (int k = j + 1 + threadIdx.x; k < n; k += NT) a[j * ld + k] = a[j * ld + k] / piv;
    __syncthreads();
    const int mm = n - j - 1;
    for (int idx = threadIdx.x; idx < mm * mm; idx += NT) {
      const int i = j + 1 + idx / mm, k = j + 1 + idx % mm;
      if (k >= i) a[i * ld + k] = a[i * ld + k] - a[j * ld + i] * a[j * ld + k];
    }
    __syncthreads();
  }
  return true;
}

// formt by the whole workgroup: T into wt, then its Cholesky factor
__device__ bool wg_formt(int ld, int col, const double *sy, const double *ss, double theta,
                         double *wt) {
  for (int idx = threadIdx.x; idx < col * col; idx += NT) {
    const int i = idx / col, j = idx - i * col;
    if (j < i) continue;
    double ddum = 0.0;
    for (int k = 0; k < i; ++k) ddum = ddum + sy[i * ld + k] * sy[j * ld + k] / sy[k * ld + k];
    wt[i * ld + j] = (i == 0) ? theta * ss[j] : ddum + theta * ss[i * ld + j];
  }
  __syncthreads();
  return wg_dpofa(wt, ld, col);
}

// ---- dcsrch / dcstep (MINPACK-2, as called by lnsrlb: ftol 1e-3, gtol 0.9, xtol 0.1) ----
__device__ void dcstep(double &stx, double &fx, double &dx, double &sty, double &fy, double &dy,
                       double &stp, double fp, double dp, int &brackt, double stpmin,
                       double stpmax) {
  const double sgnd = dp * (dx / fabs(dx));
  double stpf, stpc, stpq, theta, s, gamma, p, q, r;
  if (fp > fx) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp < stx) gamma = -gamma;
    p = (gamma - dx) + theta;
    q = ((gamma - dx) + gamma) + dp;
    r = p / q;
    stpc = stx + r * (stp - stx);
    stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    if (fabs(stpc - stx) < fabs(stpq - stx)) stpf = stpc;
    else stpf = stpc + (stpq - stpc) / 2.0;
    brackt = 1;
  } else if (sgnd < 0.0) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp > stx) gamma = -gamma;
    p = (gamma - dp) + theta;
    q = ((gamma - dp) + gamma) + dx;
    r = p / q;
    stpc = stp + r * (stx - stp);
    stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (fabs(stpc - stp) > fabs(stpq - stp)) stpf = stpc;
    else stpf = stpq;
    brackt = 1;
  } else if (fabs(dp) < fabs(dx)) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt(fmax(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    p = (gamma - dp) + theta;
    q = (gamma + (dx - dp)) + gamma;
    r = p / q;
    if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
    else if (stp > stx) stpc = stpmax;
    else stpc = stpmin;
    stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (brackt) {
      if (fabs(stpc - stp) < fabs(stpq - stp)) stpf = stpc;
      else stpf = stpq;
      if (stp > stx) stpf = fmin(stp + 0.66 * (sty - stp), stpf);
      else stpf = fmax(stp + 0.66 * (sty - stp), stpf);
    } else {
      if (fabs(stpc - stp) > fabs(stpq - stp)) stpf = stpc;
      else stpf = stpq;
      stpf = fmin(stpmax, stpf);
      stpf = fmax(stpmin, stpf);
    }
  } else {
    if (brackt) {
      theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      s = fmax(fmax(fabs(theta), fabs(dy)), fabs(dp));
      gamma = s * sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      p = (gamma - dp) + theta;
      q = ((gamma - dp) + gamma) + dy;
      r = p / q;
      stpc = stp + r * (sty - stp);
      stpf = stpc;
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  if (fp > fx) {
    sty = stp;
    fy = fp;
    dy = dp;
  } else {
    if (sgnd < 0.0) {
      sty = stx;
      fy = fx;
      dy = dx;
    }
    stx = stp;
    fx = fp;
    dx = dp;
  }
  stp = stpf;
}

// dcsrch 'START' (stpmin = 0); returns false on an input error (lnsrlb then fails)
__device__ bool dcsrch_start(NnlsState &s, double f, double g, double stp, double stpmax) {
  if (stp < 0.0 || stp > stpmax || g >= 0.0) return false;
  s.ls_brackt = 0;
  s.ls_stage = 1;
  s.ls_finit = f;
  s.ls_ginit = g;
  s.ls_gtest = 1e-3 * g;
  s.ls_width = stpmax - 0.0;
  s.ls_width1 = s.ls_width / 0.5;
  s.ls_stx = 0.0;
  s.ls_fx = f;
  s.ls_gx = g;
  s.ls_sty = 0.0;
  s.ls_fy = f;
  s.ls_gy = g;
  s.ls_stmin = 0.0;
  s.ls_stmax = stp + 4.0 * stp;
  s.ls_stpmax = stpmax;
  return true;
}

// one dcsrch call after an evaluation: returns 0 = FG (stp updated), 1 = CONV / WARN
__device__ int dcsrch_step(NnlsState &s, double f, double g, double &stp) {
  const double stpmin = 0.0, stpmax = s.ls_stpmax, xtol = 0.1;
  const double ftest = s.ls_finit + stp * s.ls_gtest;
  if (s.ls_stage == 1 && f <= ftest && g >= 0.0) s.ls_stage = 2;
  bool stop = false;
  if (s.ls_brackt && (stp <= s.ls_stmin || stp >= s.ls_stmax)) stop = true;
  if (s.ls_brackt && s.ls_stmax - s.ls_stmin <= xtol * s.ls_stmax) stop = true;
  if (stp == stpmax && f <= ftest && g <= s.ls_gtest) stop = true;
  if (stp == stpmin && (f > ftest || g >= s.ls_gtest)) stop = true;
  if (f <= ftest && fabs(g) <= 0.9 * (-s.ls_ginit)) stop = true;
  if (stop) return 1;
  const double gt = s.ls_gtest;
  if (s.ls_stage == 1 && f <= s.ls_fx && f > ftest) {
    const double fm = f - stp * gt;
    double fxm = s.ls_fx - s.ls_stx * gt;
    double fym = s.ls_fy - s.ls_sty * gt;
    const double gm = g - gt;
    double gxm = s.ls_gx - gt;
    double gym = s.ls_gy - gt;
    dcstep(s.ls_stx, fxm, gxm, s.ls_sty, fym, gym, stp, fm, gm, s.ls_brackt, s.ls_stmin,
           s.ls_stmax);
    s.ls_fx = fxm + s.ls_stx * gt;
    s.ls_fy = fym + s.ls_sty * gt;
    s.ls_gx = gxm + gt;
    s.ls_gy = gym + gt;
  } else {
    dcstep(s.ls_stx, s.ls_fx, s.ls_gx, s.ls_sty, s.ls_fy, s.ls_gy, stp, f, g, s.ls_brackt,
           s.ls_stmin, s.ls_stmax);
  }
  if (s.ls_brackt) {
    if (fabs(s.ls_sty - s.ls_stx) >= 0.66 * s.ls_width1) stp = s.ls_stx + 0.5 * (s.ls_sty - s.ls_stx);
    s.ls_width1 = s.ls_width;
    s.ls_width = fabs(s.ls_sty - s.ls_stx);
  }
  if (s.ls_brackt) {
    s.ls_stmin = fmin(s.ls_stx, s.ls_sty);
    s.ls_stmax = fmax(s.ls_stx, s.ls_sty);
  } else {
    s.ls_stmin = stp + 1.1 * (stp - s.ls_stx);
    s.ls_stmax = stp + 4.0 * (stp - s.ls_stx);
  }
  stp = fmax(stp, stpmin);
  stp = fmin(stp, stpmax);
  if ((s.ls_brackt && (stp <= s.ls_stmin || stp >= s.ls_stmax)) ||
      (s.ls_brackt && s.ls_stmax - s.ls_stmin <= xtol * s.ls_stmax))
    stp = s.ls_stx;
  return 0;
}

__device__ void finish_block(NnlsState &s, int *active, int status) {
  s.status |= status;
  s.phase = PH_DONE;
  atomicSub(active, 1);
}

// memory refresh (lbfgsb.f: info != 0 -> col = 0, head = 1, theta = 1, iupdat = 0)
__device__ void refresh(NnlsState &s) {
  s.col = 0;
  s.theta = 1.0;
  s.iupdat = 0;
  s.updatd = 0;
  s.pending = 0;
  s.phase = PH_CAUCHY;
}

// line-search failure (lnsrlb info != 0 or iback >= 20): restore the previous iterate, then
// refresh the memory, or stop (ABNORMAL_TERMINATION_IN_LNSRCH) when it is already empty
__device__ void ls_failed(NnlsState &s, int *active) {
  s.f = s.fold;  // x, g: the cur buffers were never overwritten
  if (s.col == 0) {
    finish_block(s, active, ST_ABNORMAL);
  } else {
    refresh(s);
  }
}

// lnsrlb entry: set up the line search from z (d = z - x, its dot products reduced by the
// sweep) and request the first trial
__device__ void ls_begin(NnlsState &s, int *active, double dtd, double gd, double stpmx_min,
                         int stpmx_zero) {
  s.dtd = dtd;
  s.dnorm = sqrt(dtd);
  double stpmx = 1e10;
  if (s.it == 0) {
    stpmx = 1.0;
  } else {
    if (stpmx_zero) stpmx = 0.0;
    else if (stpmx_min < stpmx) stpmx = stpmx_min;
  }
  s.stpmx = stpmx;
  s.stp = (s.it == 0) ? fmin(1.0 / s.dnorm, stpmx) : 1.0;
  s.fold = s.f;
  s.ifun = 0;
  s.gd = gd;
  s.gdold = gd;
  if (gd >= 0.0 || !dcsrch_start(s, s.f, gd, s.stp, stpmx)) {
    ls_failed(s, active);
    return;
  }
  s.ifun = 1;  // the first trial is requested (iback = ifun - 1 = 0)
  s.phase = PH_EVAL;
}

// the GCP is known: cmprlb's wa = M c (bmv), then FREEV.  Wave-collective (64 lanes);
// lane 0 writes the state.
__device__ void gcp_done(NnlsState &s, const Blk &b, int ld, const double *sy, const double *wt,
                         const double *cvec) {
  const int col = s.col;
  const bool ok = col == 0 || wbmv(ld, col, sy, wt, cvec, b.WA);
  if ((threadIdx.x & 63) == 0) {
    if (!ok) {
      refresh(s);
      s.bk_count = 0;
    } else {
      s.phase = PH_FREEV;
    }
  }
}

// debug stop (ftmi_nnls_lbfgsb_args.dbg_stop = 16 * iteration + phase): the block ends
// right before that phase of that iteration, its workspace holding the state it had there
__device__ inline bool dbg_hit(const Args &a, NnlsState &s, int g) {
  if (a.dbg_stop == 0 || a.dbg_stop != 16 * s.it + s.phase) return false;
  __syncthreads();
  if (g == 0 && threadIdx.x == 0) finish_block(s, a.active, 0);
  return true;
}

// ---- phase kernels ---------------------------------------------------------------------------

// x0 = clip(float32(pinv M), 0) per frame (the reference's float32 lstsq start; pinv in
// float64, the result rounded to float32 like LAPACK sgelsd's), state reset, phase EVAL
__global__ __launch_bounds__(NT) void nnls_start_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  __shared__ double m_s[512];
  for (int fl = fl0; fl < fl1; ++fl) {
    const int f = b.f0 + fl;
    __syncthreads();
    for (int i = threadIdx.x; i < a.n_mels; i += NT) {
      const float v = a.mel[((int64_t)b.item * a.n_mels + i) * a.F + f];
      m_s[i] = a.denorm ? (double)(float)exp((double)v) : (double)v;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.nb; k += NT) {
      double acc = 0.0;
      const double *pr = a.pinv + (int64_t)k * a.n_mels;
      for (int i = 0; i < a.n_mels; ++i) acc = acc + pr[i] * m_s[i];
      float x0 = (float)acc;
      x0 = x0 > 0.f ? x0 : 0.f;  // np.clip(x, 0, None)
      const int e = fl * a.nb + k;
      b.X[0][e] = (double)x0;
      b.PF[e] = 1;
      b.IW[e] = 0;
    }
  }
  if (g == 0) {
    const int m2 = 2 * a.m;
    for (int i = threadIdx.x; i < m2 * m2; i += NT) b.WN1[i] = 0.0;
  }
  if (g == 0 && threadIdx.x == 0) {
    NnlsState &s = *b.st;
    s = NnlsState{};
    s.theta = 1.0;
    s.cur = 0;
    s.phase = PH_EVAL;
  }
}

// EVAL: f and g at x (the start point, or a line-search trial x = z | stp d + t), with
// gd = g.d and the projected-gradient norm; dcsrch decides
__global__ __launch_bounds__(NT) void nnls_eval_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != PH_EVAL) return;
  if (dbg_hit(a, s, g)) return;
  const bool first = (s.nfev == 0);
  const int cur = s.cur, nxt = first ? cur : cur ^ 1;
  const double stp = s.stp;
  double *xo = xbuf(b, nxt), *go = gbuf(b, nxt);
  const double *t = xbuf(b, cur);
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  __shared__ double xs[2112];
  __shared__ double diff[512];
  __shared__ double red[NW * 4];
  double f_acc = 0.0, gd_acc = 0.0, sbg = 0.0;
  for (int fl = fl0; fl < fl1; ++fl) {
    const int f = b.f0 + fl;
    const int e0 = fl * a.nb;
    __syncthreads();
    for (int k = threadIdx.x; k < a.nb; k += NT) {
      const int e = e0 + k;
      double x;
      if (first) {
        x = xo[e];
      } else {
        const double d = b.Z[e] - t[e];
        x = (stp == 1.0) ? b.Z[e] : stp * d + t[e];
        xo[e] = x;
      }
      xs[k] = x;
    }
    for (int i = threadIdx.x; i < a.n_mels; i += NT) {
      const float v = a.mel[((int64_t)b.item * a.n_mels + i) * a.F + f];
      diff[i] = a.denorm ? (double)(float)exp((double)v) : (double)v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.n_mels; i += NT) {
      const int lo = a.rowlo[i], p0 = a.rowptr[i], cnt = a.rowptr[i + 1] - p0;
      double acc = 0.0;
      for (int q = 0; q < cnt; ++q) acc = acc + (double)a.rowvals[p0 + q] * xs[lo + q];
      const double dv = acc - diff[i];
      diff[i] = dv;
      f_acc = f_acc + dv * dv;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.nb; k += NT) {
      const int e = e0 + k;
      const int r0 = a.bin_rows[2 * k], r1 = a.bin_rows[2 * k + 1];
      double gv = 0.0;
      if (r0 >= 0) gv = gv + (double)a.bin_w[2 * k] * diff[r0];
      if (r1 >= 0) gv = gv + (double)a.bin_w[2 * k + 1] * diff[r1];
      go[e] = gv;
      if (!first) gd_acc = gd_acc + gv * (b.Z[e] - t[e]);
      const double x = xs[k];
      const double gi = gv < 0.0 ? gv : fmin(x, gv);  // projgr, l = 0
      sbg = fmax(sbg, fabs(gi));
    }
  }
  // partials: f, gd, sbgnrm (max)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f_acc = wave_sum(f_acc);
  gd_acc = wave_sum(gd_acc);
  sbg = wave_max(sbg);
  if (lane == 0) {
    red[w] = f_acc;
    red[NW + w] = gd_acc;
    red[2 * NW + w] = sbg;
  }
  __syncthreads();
  const int ns = nslots(a.m);
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int q = 0; q < NW; ++q) {
      s0 += red[q];
      s1 += red[NW + q];
      s2 = fmax(s2, red[2 * NW + q]);
    }
    b.PART[g * ns + 0] = s0;
    b.PART[g * ns + 1] = s1;
    b.PART[g * ns + 2] = s2;
  }
  if (!arrive_last(b.st, a.groups)) return;
  if (threadIdx.x != 0) return;
  double fs = 0.0, gds = 0.0, sb = 0.0;
  for (int q = 0; q < a.groups; ++q) {
    fs += b.PART[q * ns + 0];
    gds += b.PART[q * ns + 1];
    sb = fmax(sb, b.PART[q * ns + 2]);
  }
  const double fval = 0.5 * fs;
  s.nfev += 1;
  if (first) {
    s.f = fval;
    s.sbgnrm = sb;
    if (sb <= PGTOL) {
      finish_block(s, a.active, ST_CONV);
      return;
    }
    s.pending = 0;
    s.phase = PH_CAUCHY;
    return;
  }
  // a line-search trial: dcsrch on (f, g.d)
  double stpn = s.stp;
  const int conv = dcsrch_step(s, fval, gds, stpn);
  if (!conv) {
    // another trial; lnsrlb: ifun += 1, iback = ifun - 1 >= maxls -> restore + refresh
    s.ifun += 1;
    if (s.ifun - 1 >= MAXLS) {
      ls_failed(s, a.active);
      return;
    }
    s.stp = stpn;
    return;  // phase stays EVAL (x, g of this trial are discarded)
  }
  // NEW_X: accept the trial
  s.cur = nxt;
  s.f = fval;
  s.gd = gds;
  s.sbgnrm = sb;
  s.it += 1;
  if (sb <= PGTOL) {
    finish_block(s, a.active, ST_CONV);
    return;
  }
  if (s.it >= a.maxiter) {
    finish_block(s, a.active, ST_MAXITER);
    return;
  }
  const double ddum = fmax(fmax(fabs(s.fold), fabs(s.f)), 1.0);
  if ((s.fold - s.f) <= FTOL_FACTR * ddum) {
    finish_block(s, a.active, ST_CONV);
    return;
  }
  double dr, dd;
  if (s.stp == 1.0) {
    dr = s.gd - s.gdold;
    dd = -s.gdold;
  } else {
    dr = (s.gd - s.gdold) * s.stp;
    dd = -s.gdold * s.stp;
  }
  if (dr <= EPSMCH * dd) {
    s.nskip += 1;
    s.updatd = 0;
    s.pending = 0;
  } else {
    if (s.iupdat + 1 > a.mref || s.iupdat + 1 > a.m) {
      // the reference's history wraps at m = n_bins updates (not restated); a workspace
      // with fewer columns than needed: the caller reruns with a larger one
      finish_block(s, a.active, s.iupdat + 1 > a.m ? ST_MEMCAP : ST_ABNORMAL);
      return;
    }
    s.dr = dr;
    s.pending = 1;
  }
  s.phase = PH_CAUCHY;
}

// CAUCHY: (pending update) s = stp (z - t), y = g - g_old into the history, S'y / S's
// entries and y'y; then the Cauchy sweep: iwhere, d = -g on moving variables, f1, p = W'd,
// the breakpoint list
__global__ __launch_bounds__(NT) void nnls_cauchy_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != PH_CAUCHY) return;
  if (dbg_hit(a, s, g)) return;
  const int m = a.m, ns = nslots(m);
  const int cur = s.cur;
  const double *x = xbuf(b, cur), *gv = gbuf(b, cur), *xprev = xbuf(b, cur ^ 1), *gprev = gbuf(b, cur ^ 1);
  const int pend = s.pending;
  const int col0 = s.col;                       // columns before the update
  const int coln = pend ? col0 + 1 : col0;      // columns of this Cauchy step
  const double stp = s.stp;
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  const int e0 = fl0 * a.nb, e1 = fl1 * a.nb;
  __shared__ double red[NW * 48];
  double *part = b.PART + g * ns;
  // (1) scalars + the new history column
  {
    double f1 = 0.0, rr = 0.0;
    int nfc = 0, unb = 0;
    double *wsn = b.WS + (int64_t)col0 * a.n_pad, *wyn = b.WY + (int64_t)col0 * a.n_pad;
    for (int e = e0 + threadIdx.x; e < e1; e += NT) {
      if (pend) {
        const double d = b.Z[e] - xprev[e];
        const double sv = (stp == 1.0) ? d : stp * d;
        const double yv = gv[e] - gprev[e];
        wsn[e] = sv;
        wyn[e] = yv;
        rr = rr + yv * yv;
      }
      const double neggi = -gv[e];
      const bool xlower = x[e] <= 0.0;
      int iw = 0;
      if (xlower) {
        if (neggi <= 0.0) iw = 1;
      } else if (fabs(neggi) <= 0.0) {
        iw = -3;
      }
      b.IW[e] = (int8_t)iw;
      if (iw == 0) {
        f1 = f1 - neggi * neggi;
        if (neggi < 0.0) {
          const double tb = x[e] / (-neggi);  // tl / (-neggi), tl = x - l
          const int slot = atomicAdd(&s.bk_count, 1);
          b.BKEY[slot] = (unsigned long long)__double_as_longlong(tb);
          b.BIDX[slot] = e;
        } else {
          nfc += 1;
          if (fabs(neggi) > 0.0) unb = 1;
        }
      }
    }
    double acc[4] = {f1, rr, (double)nfc, (double)unb};
    // unb is an OR: summed, tested > 0
    wg_sums<4>(acc, 4, red, part);
  }
  // (2) p = W'd over the columns (incl. the new one) and the new S'y / S's entries
  // (sy(col, j) = s.y_j, ss(j, col) = s_j.s for j < col0), JB columns per sweep
  constexpr int JB = 8;
  for (int j0 = 0; j0 < coln; j0 += JB) {
    double acc[4 * JB];
#pragma unroll
    for (int q = 0; q < 4 * JB; ++q) acc[q] = 0.0;
    for (int e = e0 + threadIdx.x; e < e1; e += NT) {
      const int iw = b.IW[e];
      const double dc = (iw == 0) ? -gv[e] : 0.0;
      double sv = 0.0;
      if (pend) sv = b.WS[(int64_t)col0 * a.n_pad + e];
#pragma unroll
      for (int q = 0; q < JB; ++q) {
        const int j = j0 + q;
        if (j < coln) {
          const double wy = b.WY[(int64_t)j * a.n_pad + e], ws = b.WS[(int64_t)j * a.n_pad + e];
          acc[q] = acc[q] + wy * dc;
          acc[JB + q] = acc[JB + q] + ws * dc;
          if (pend && j < col0) {
            acc[2 * JB + q] = acc[2 * JB + q] + sv * wy;
            acc[3 * JB + q] = acc[3 * JB + q] + ws * sv;
          }
        }
      }
    }
    wg_sums<4 * JB>(acc, 4 * JB, red, part + 4 + 4 * j0);
  }
  if (!arrive_last(b.st, a.groups)) return;
  // ---- scalar part: the small matrices staged in LDS when col <= MC; formt by the whole
  // workgroup, bmv by wave 0, the state by thread 0 ----
  __shared__ double msy[MC * MC], mss[MC * MC], mwt[MC * MC];
  if (threadIdx.x == 0) {
    double f1 = 0.0, rr = 0.0, nfc = 0.0, unb = 0.0;
    for (int q = 0; q < a.groups; ++q) {
      const double *pq = b.PART + q * ns;
      f1 += pq[0];
      rr += pq[1];
      nfc += pq[2];
      unb += pq[3];
    }
    s.f1 = f1;
    s.rr = rr;
    s.nfree_c = (int)nfc;
    s.bnded = unb > 0.0 ? 0 : 1;
    s.nbreak = s.bk_count;
    if (pend) {
      // matupd (lbfgsb.f): the new column's S'Y row and S'S column
      const int c = col0;  // 0-based index of the new column
      for (int j = 0; j < c; ++j) {
        double syv = 0.0, ssv = 0.0;
        for (int q = 0; q < a.groups; ++q) {
          const double *pq = b.PART + q * ns + 4;
          const int jb = (j / JB) * JB, jj = j - jb;
          syv += pq[4 * jb + 2 * JB + jj];
          ssv += pq[4 * jb + 3 * JB + jj];
        }
        b.SY[c * m + j] = syv;
        b.SS[j * m + c] = ssv;
      }
      b.SS[c * m + c] = (stp == 1.0) ? s.dtd : stp * stp * s.dtd;
      b.SY[c * m + c] = s.dr;
      s.col = coln;
      s.iupdat += 1;
      s.updatd = 1;
      s.theta = rr / s.dr;
      s.pending = 0;
    }
  }
  __syncthreads();
  const int col = coln;
  const bool sm = col <= MC;
  const int ld = sm ? col : m;
  double *SYp = sm ? msy : b.SY, *SSp = sm ? mss : b.SS, *WTp = sm ? mwt : b.WT;
  if (sm) {
    stage_in(msy, b.SY, m, col);
    stage_in(mss, b.SS, m, col);
    if (!pend) stage_in(mwt, b.WT, m, col);
  }
  __syncthreads();
  const double theta = s.theta;
  bool ok = true;
  if (pend) ok = wg_formt(ld, col, SYp, SSp, theta, WTp);
  if (pend && ok && sm) stage_out(b.WT, m, mwt, col);
  // p, c, M p in LDS (the lanes exchange them), copied out at the end
  __shared__ double vP[2 * MMAX], vC[2 * MMAX], vV[2 * MMAX];
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  if (!ok) {
    if (lane == 0) {
      refresh(s);  // redo the Cauchy step with an empty memory
      s.bk_count = 0;
    }
    return;
  }
  for (int j = lane; j < col; j += 64) {
    double py = 0.0, ps = 0.0;
    for (int q = 0; q < a.groups; ++q) {
      const double *pq = b.PART + q * ns + 4;
      const int jb = (j / JB) * JB, jj = j - jb;
      py += pq[4 * jb + jj];
      ps += pq[4 * jb + JB + jj];
    }
    vP[j] = py;
    vP[col + j] = ps * theta;  // dscal(col, theta, p(col+1))
    vC[j] = 0.0;
    vC[col + j] = 0.0;
  }
  wave_sync();
  auto flush = [&]() {
    wave_sync();
    for (int j = lane; j < 2 * col; j += 64) {
      b.P[j] = vP[j];
      b.C[j] = vC[j];
    }
  };
  const int nbreak = s.nbreak;
  const double f1 = s.f1;
  if (lane == 0) {
    s.kpassed = 0;
    s.nseg = 0;
    s.tsum = 0.0;
    s.tj = 0.0;
    s.walk_done = 0;
    s.nenter = s.nleave = 0;
  }
  if (nbreak == 0 && s.nfree_c == 0) {
    // d = 0: xcp = x (lbfgsb.f cauchy returns before the loop); c = 0
    if (lane == 0) s.dtm = 0.0;
    flush();
    gcp_done(s, b, ld, SYp, WTp, vC);
    return;
  }
  double vp = 0.0;
  if (col > 0) {
    if (!wbmv(ld, col, SYp, WTp, vP, vV)) {
      if (lane == 0) {
        refresh(s);
        s.bk_count = 0;
      }
      return;
    }
    // v'p in the reference's order (every lane the same sum)
    for (int j = 0; j < 2 * col; ++j) vp = vp + vV[j] * vP[j];
  }
  const double f2o = -theta * f1;
  const double f2 = f2o - vp;
  const double dtm0 = -f1 / f2;
  if (lane == 0) {
    s.f2_org = f2o;
    s.f2 = f2;
    s.dtm = dtm0;
    s.nseg = 1;
  }
  if (nbreak == 0) {
    // goto 888
    const double dtm = fmax(dtm0, 0.0);
    for (int j = lane; j < 2 * col; j += 64) vC[j] = vC[j] + dtm * vP[j];
    if (lane == 0) {
      s.dtm = dtm;
      s.tsum = dtm;
    }
    flush();
    gcp_done(s, b, ld, SYp, WTp, vC);
    return;
  }
  flush();
  if (lane == 0) s.phase = PH_WALK;
}

// WALK (one workgroup per block): the breakpoints in increasing order — chunks of the
// smallest remaining ones found by a radix select on the float64 bit patterns, sorted in
// LDS — and the Cauchy loop over them (lbfgsb.f cauchy, labels 777 / 888 / 999)
__global__ __launch_bounds__(NT) void nnls_walk_kernel(const Args a) {
  const int blk = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != PH_WALK) return;
  if (dbg_hit(a, s, 0)) return;
  const int m = a.m;
  __shared__ unsigned hist[2048];
  __shared__ unsigned long long skey[CAP];
  __shared__ int sidx[CAP];
  __shared__ unsigned long long bound_sh;
  __shared__ int cnt_sh, stop_sh;
  const int nbreak = s.nbreak;
  const double *x = xbuf(b, s.cur), *gv = gbuf(b, s.cur);
  // the small matrices and vectors of the serial loop in LDS (col <= MC): the loop's loads
  // form a dependent chain
  // the vectors of the serial loop always in LDS (lanes exchange them), the matrices too when
  // col <= MC (read-only here; L2-resident otherwise)
  __shared__ double msy[MC * MC], mwt[MC * MC], mp[2 * MMAX], mc[2 * MMAX], mwbp[2 * MMAX],
      mv[2 * MMAX];
  const int colw = s.col;
  const bool sm = colw <= MC;
  const int ld = sm ? colw : m;
  const double *SYp = sm ? msy : b.SY, *WTp = sm ? mwt : b.WT;
  double *Pp = mp, *Cp = mc, *WBPp = mwbp, *Vp = mv;
  if (sm) {
    stage_in(msy, b.SY, m, colw);
    stage_in(mwt, b.WT, m, colw);
  }
  for (int j = threadIdx.x; j < 2 * colw; j += NT) {
    mp[j] = b.P[j];
    mc[j] = b.C[j];
  }
  __syncthreads();
  // the Cauchy loop's scalars, held in wave 0's registers across the chunks
  const double theta = s.theta;
  const int bnded = s.bnded;
  const double w_f2org = s.f2_org;
  double w_tj = s.tj, w_tsum = s.tsum, w_f1 = s.f1, w_f2 = s.f2, w_dtm = s.dtm;
  int w_kpassed = s.kpassed, w_nseg = s.nseg, w_done = 0;
  unsigned long long last = 0ull;
  bool have_last = false;
  while (true) {
    // ---- select: the smallest boundary B with count(last < key <= B) >= KCHUNK (or all),
    // digit by digit from the top, keeping the count within CAP
    unsigned long long prefix = 0;
    int plen = 0;
    unsigned below = 0;  // candidates with key < prefix block
    unsigned long long bound = ~0ull;
    while (true) {
      const int dl = (64 - plen) >= 11 ? 11 : (64 - plen);
      const int shift = 64 - plen - dl;
      for (int i = threadIdx.x; i < 2048; i += NT) hist[i] = 0;
      __syncthreads();
      for (int i = threadIdx.x; i < nbreak; i += NT) {
        const unsigned long long k = b.BKEY[i];
        if (have_last && k <= last) continue;
        if (plen > 0 && (k >> (64 - plen)) != (prefix >> (64 - plen))) continue;
        atomicAdd(&hist[(unsigned)((k >> shift) & ((1ull << dl) - 1))], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned cum = below, dsel = (1u << dl) - 1;
        unsigned before = below;
        int done = 0;
        for (unsigned d = 0; d < (1u << dl); ++d) {
          before = cum;
          cum += hist[d];
          if (cum >= KCHUNK) {
            dsel = d;
            break;
          }
          if (d == (1u << dl) - 1) dsel = d;  // every candidate fits below KCHUNK
        }
        unsigned long long pfx = prefix | ((unsigned long long)dsel << shift);
        if (cum <= CAP || plen + dl >= 64) {
          // all candidates with key < (pfx + 1) << shift
          bound = (shift > 0) ? (pfx | ((1ull << shift) - 1)) : pfx;
          done = 1;
          if (cum > CAP) s.status |= ST_TIES;
        } else {
          below = before;
          prefix = pfx;
        }
        bound_sh = bound;
        cnt_sh = done ? 1 : 0;
        // publish the refined prefix through LDS too
        hist[0] = (unsigned)(prefix >> 32);
        hist[1] = (unsigned)prefix;
        hist[2] = below;
      }
      __syncthreads();
      const int done = cnt_sh;
      if (!done) {
        prefix = ((unsigned long long)hist[0] << 32) | hist[1];
        below = hist[2];
        plen += dl;
        __syncthreads();
        continue;
      }
      bound = bound_sh;
      __syncthreads();
      break;
    }
    // ---- gather + sort the chunk
    if (threadIdx.x == 0) cnt_sh = 0;
    for (int i = threadIdx.x; i < CAP; i += NT) {
      skey[i] = ~0ull;
      sidx[i] = 0x7fffffff;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbreak; i += NT) {
      const unsigned long long k = b.BKEY[i];
      if (have_last && k <= last) continue;
      if (k > bound) continue;
      const int slot = atomicAdd(&cnt_sh, 1);
      if (slot < CAP) {
        skey[slot] = k;
        sidx[slot] = b.BIDX[i];
      }
    }
    __syncthreads();
    const int cnt = cnt_sh < CAP ? cnt_sh : CAP;
    // bitonic sort by (key, index)
    for (int kk = 2; kk <= CAP; kk <<= 1) {
      for (int jj = kk >> 1; jj > 0; jj >>= 1) {
        for (int i = threadIdx.x; i < CAP; i += NT) {
          const int ixj = i ^ jj;
          if (ixj > i) {
            const bool up = (i & kk) == 0;
            const unsigned long long ka = skey[i], kb = skey[ixj];
            const int ia = sidx[i], ib = sidx[ixj];
            const bool gt = (ka > kb) || (ka == kb && ia > ib);
            if (gt == up) {
              skey[i] = kb;
              skey[ixj] = ka;
              sidx[i] = ib;
              sidx[ixj] = ia;
            }
          }
        }
        __syncthreads();
      }
    }
    // ---- the Cauchy loop over this chunk (wave 0; the scalars uniform in its lanes)
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      int stop = 0;
      for (int q = 0; q < cnt; ++q) {
        const double tj0 = w_tj;
        const int ibp = sidx[q];
        const double tj = __longlong_as_double((long long)skey[q]);
        const double dt = tj - tj0;
        if (w_dtm < dt) {  // the minimiser is within this interval
          stop = 1;
          break;
        }
        w_tj = tj;
        w_tsum = w_tsum + dt;
        w_kpassed += 1;
        const int nleft = nbreak - w_kpassed;
        const double dibp = -gv[ibp];
        if (lane == 0) b.IW[ibp] = 1;  // fixed at the lower bound: xcp = 0, d = 0
        const double zibp = 0.0 - x[ibp];
        if (nleft == 0 && nbreak == b.n) {
          w_dtm = dt;
          for (int j = lane; j < 2 * colw; j += 64) Cp[j] = Cp[j] + w_dtm * Pp[j];
          w_done = 2;  // label 999: xcp needs no daxpy
          stop = 2;
          break;
        }
        w_nseg += 1;
        const double dibp2 = dibp * dibp;
        double f1 = w_f1 + dt * w_f2 + dibp2 - theta * dibp * zibp;
        double f2 = w_f2 - theta * dibp2;
        if (colw > 0) {
          for (int j = lane; j < colw; j += 64) {
            Cp[j] = Cp[j] + dt * Pp[j];
            Cp[colw + j] = Cp[colw + j] + dt * Pp[colw + j];
            WBPp[j] = b.WY[(int64_t)j * a.n_pad + ibp];
            WBPp[colw + j] = theta * b.WS[(int64_t)j * a.n_pad + ibp];
          }
          wave_sync();
          if (!wbmv(ld, colw, SYp, WTp, WBPp, Vp)) {
            w_done = 3;  // info != 0: refresh
            stop = 3;
            break;
          }
          double wmc = 0.0, wmp = 0.0, wmw = 0.0;
          for (int j = lane; j < 2 * colw; j += 64) {
            wmc = wmc + Cp[j] * Vp[j];
            wmp = wmp + Pp[j] * Vp[j];
            wmw = wmw + WBPp[j] * Vp[j];
          }
          wmc = wave_sum(wmc);
          wmp = wave_sum(wmp);
          wmw = wave_sum(wmw);
          for (int j = lane; j < 2 * colw; j += 64) Pp[j] = Pp[j] + (-dibp) * WBPp[j];
          wave_sync();
          f1 = f1 + dibp * wmc;
          f2 = f2 + 2.0 * dibp * wmp - dibp2 * wmw;
        }
        f2 = fmax(EPSMCH * w_f2org, f2);
        w_f1 = f1;
        w_f2 = f2;
        if (nleft > 0) {
          w_dtm = -f1 / f2;
        } else if (bnded) {
          w_f1 = 0.0;
          w_f2 = 0.0;
          w_dtm = 0.0;
        } else {
          w_dtm = -f1 / f2;
        }
      }
      if (!stop && w_kpassed >= nbreak) stop = 1;  // every breakpoint passed: label 888
      if (!stop && cnt == 0) {  // cannot happen unless > CAP equal keys were cut (ST_TIES)
        if (lane == 0) s.status |= ST_TIES;
        stop = 1;
      }
      if (lane == 0) stop_sh = stop;
    }
    __syncthreads();
    const int stop = stop_sh;
    if (stop) break;
    last = bound;
    have_last = true;
    __syncthreads();
  }
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (w_done == 3) {
      if (lane == 0) {
        refresh(s);
        s.bk_count = 0;
      }
    } else {
      if (w_done != 2) {
        // label 888
        if (w_dtm <= 0.0) w_dtm = 0.0;
        w_tsum = w_tsum + w_dtm;
        for (int j = lane; j < 2 * colw; j += 64) Cp[j] = Cp[j] + w_dtm * Pp[j];
      }
      if (lane == 0) {
        s.tj = w_tj;
        s.tsum = w_tsum;
        s.f1 = w_f1;
        s.f2 = w_f2;
        s.dtm = w_dtm;
        s.kpassed = w_kpassed;
        s.nseg = w_nseg;
        s.walk_done = w_done;
      }
      wave_sync();
      gcp_done(s, b, ld, SYp, WTp, Cp);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * colw; j += NT) {
    b.P[j] = mp[j];
    b.C[j] = mc[j];
  }
}

// xcp of element e after the walk (lbfgsb.f cauchy: xcp = x + tsum d with d = -g on the
// variables still moving, 0 on those fixed at a breakpoint, x elsewhere)
__device__ inline double xcp_of(int iw, double x, double g, double tsum, bool done999) {
  if (iw == 1) return 0.0;
  if (iw == 0 && !done999) return x + tsum * (-g);
  return x;
}

// FREEV: free set at the GCP, entering / leaving lists; formk's new WN1 row (if updatd);
// cmprlb's r = -theta (xcp - x) - g + W M c on the free variables; subsm's W'Zr
__global__ __launch_bounds__(NT) void nnls_freev_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != PH_FREEV) return;
  if (dbg_hit(a, s, g)) return;
  const int m = a.m, ns = nslots(m);
  const int cur = s.cur, col = s.col;
  const double *x = xbuf(b, cur), *gv = gbuf(b, cur);
  const double theta = s.theta, tsum = s.tsum;
  const bool done999 = s.walk_done == 2;
  const bool count_chg = s.it > 0;
  const bool subspace_possible = col > 0;
  const bool newrow = s.updatd && col > 0;
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  const int e0 = fl0 * a.nb, e1 = fl1 * a.nb;
  __shared__ double red[NW * 48];
  double *part = b.PART + g * ns;
  {
    // entering / leaving variables, listed per workgroup in element order (a workgroup-wide
    // rank per round, so the list — and formk's sums over it — are deterministic): entering
    // from e0 up, leaving from e1 - 1 down
    __shared__ int wc[2 * NW];
    double nf = 0.0;
    int ne = 0, nl = 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int base = e0; base < e1; base += NT) {
      const int e = base + threadIdx.x;
      bool enter = false, leave = false;
      if (e < e1) {
        const bool fr = b.IW[e] <= 0;
        nf += fr ? 1.0 : 0.0;
        if (count_chg) {
          const bool pf = b.PF[e] != 0;
          enter = fr && !pf;
          leave = !fr && pf;
        }
        b.PF[e] = fr ? 1 : 0;
        // r on free variables (cmprlb), before the W M c terms
        if (subspace_possible) {
          const double xc = xcp_of(b.IW[e], x[e], gv[e], tsum, done999);
          b.R[e] = fr ? (-theta * (xc - x[e]) - gv[e]) : 0.0;
        }
      }
      if (count_chg) {
        const unsigned long long me = __ballot(enter), ml = __ballot(leave);
        const unsigned long long lt = (1ull << lane) - 1;
        if (lane == 0) {
          wc[w] = __popcll(me);
          wc[NW + w] = __popcll(ml);
        }
        __syncthreads();
        int be = ne, bl = nl;
        for (int q = 0; q < NW; ++q) {
          if (q < w) {
            be += wc[q];
            bl += wc[NW + q];
          }
          ne += wc[q];
          nl += wc[NW + q];
        }
        __syncthreads();
        if (enter) b.CHG[e0 + be + __popcll(me & lt)] = e;
        if (leave) b.CHG[e1 - 1 - (bl + __popcll(ml & lt))] = e;
      }
    }
    double acc[3] = {nf, (double)ne, (double)nl};
    wg_sums<3>(acc, 3, red, part);
    if (threadIdx.x == 0) {
      part[1] = (double)ne;  // exact counts (every thread holds the workgroup totals)
      part[2] = (double)nl;
    }
  }
  if (subspace_possible) {
    // r += W M c (wa = M c made by the walk's scalar part), columns in order, and formk's
    // new row (c = col - 1): Y'ZZ'Y(c, j), S'AA'S(c, j), S'AA'Y(c, j) [L_a], S'ZZ'Y(j, c) [R_z]
    const int c = col - 1;
    constexpr int JB = 8;
    // (a) r: every column, sequentially per element (the reference's order)
    for (int e = e0 + threadIdx.x; e < e1; e += NT) {
      if (b.IW[e] > 0) continue;
      double r = b.R[e];
      for (int j = 0; j < col; ++j) {
        const double a1 = b.WA[j], a2 = theta * b.WA[col + j];
        r = r + b.WY[(int64_t)j * a.n_pad + e] * a1 + b.WS[(int64_t)j * a.n_pad + e] * a2;
      }
      b.R[e] = r;
    }
    // (b) new row sums + W'Zr
    for (int j0 = 0; j0 < col; j0 += JB) {
      double acc[6 * JB];
#pragma unroll
      for (int q = 0; q < 6 * JB; ++q) acc[q] = 0.0;
      for (int e = e0 + threadIdx.x; e < e1; e += NT) {
        const bool fr = b.IW[e] <= 0;
        const double r = fr ? b.R[e] : 0.0;
        const double yc = newrow ? b.WY[(int64_t)c * a.n_pad + e] : 0.0;
        const double sc = newrow ? b.WS[(int64_t)c * a.n_pad + e] : 0.0;
#pragma unroll
        for (int q = 0; q < JB; ++q) {
          const int j = j0 + q;
          if (j < col) {
            const double wy = b.WY[(int64_t)j * a.n_pad + e], ws = b.WS[(int64_t)j * a.n_pad + e];
            if (fr) {
              acc[q] = acc[q] + wy * r;
              acc[JB + q] = acc[JB + q] + ws * r;
              if (newrow) {
                acc[2 * JB + q] = acc[2 * JB + q] + yc * wy;   // Y'ZZ'Y(c, j)
                acc[5 * JB + q] = acc[5 * JB + q] + ws * yc;   // R_z(j, c) = s_j'ZZ'y_c
              }
            } else if (newrow) {
              acc[3 * JB + q] = acc[3 * JB + q] + sc * ws;     // S'AA'S(c, j)
              acc[4 * JB + q] = acc[4 * JB + q] + sc * wy;     // L_a(c, j) = s_c'AA'y_j
            }
          }
        }
      }
      wg_sums<6 * JB>(acc, 6 * JB, red, part + 4 + 6 * j0);
    }
  }
  if (!arrive_last(b.st, a.groups)) return;
  if (threadIdx.x != 0) return;
  double nf = 0.0;
  int ne = 0, nl = 0;
  for (int q = 0; q < a.groups; ++q) {
    nf += b.PART[q * ns];
    ne += (int)b.PART[q * ns + 1];
    nl += (int)b.PART[q * ns + 2];
  }
  s.nfree = (int)nf;
  s.nenter = ne;
  s.nleave = nl;
  s.bk_count = 0;
  constexpr int JB = 8;
  auto gsum = [&](int j, int slot) {
    double v = 0.0;
    const int jb = (j / JB) * JB, jj = j - jb;
    for (int q = 0; q < a.groups; ++q) v += b.PART[q * ns + 4 + 6 * jb + slot * JB + jj];
    return v;
  };
  if (s.nfree == 0 || col == 0) {
    s.backtrack = 0;
    s.phase = PH_SUBSM;  // z = xcp (label 555)
    return;
  }
  for (int j = 0; j < col; ++j) {
    b.WV[j] = gsum(j, 0);
    b.WV[col + j] = theta * gsum(j, 1);
    if (newrow) {
      b.NEWROW[j] = gsum(j, 2);
      b.NEWROW[m + j] = gsum(j, 3);
      b.NEWROW[2 * m + j] = gsum(j, 4);
      b.NEWROW[3 * m + j] = gsum(j, 5);
    }
  }
  s.phase = PH_FORMK;
}

// FORMK (one workgroup per block): WN1's new row / column (updatd), the entering / leaving
// variables' terms on the old part, WN, its two Cholesky factors (lbfgsb.f formk); then
// subsm's K^-1 W'Zr
__global__ __launch_bounds__(NT) void nnls_formk_kernel(const Args a) {
  const int blk = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != PH_FORMK) return;
  if (dbg_hit(a, s, 0)) return;
  const int m = a.m, m2 = 2 * m, col = s.col, ns = nslots(m);
  const bool updatd = s.updatd;
  const bool wrk = (s.nenter > 0) || (s.nleave > 0) || updatd;
  // WN and its factorisation in LDS when 2 col <= 64
  __shared__ double mwn[64 * 64];
  __shared__ int fok;
  const int col2 = 2 * col;
  const bool sm = col2 <= 64;
  const int ldw = sm ? col2 : m2;
  double *wn = sm ? mwn : b.WN;
  double *wn1 = b.WN1;  // [2m][2m], rows/cols: Y block 0..m-1, S block m..2m-1
  if (wrk) {
    const int upcl = updatd ? col - 1 : col;
    // entering / leaving sums for the old part: DELTA[0]: Y'Y enter, [1]: Y'Y leave,
    // [2]: S'S enter, [3]: S'S leave, [4]: S'Y enter (is, jy), [5]: S'Y leave
    const int npair = upcl * upcl;
    for (int pq = threadIdx.x; pq < npair; pq += NT) {
      const int i = pq / upcl, j = pq - i * upcl;
      const double *yi = b.WY + (int64_t)i * a.n_pad, *yj = b.WY + (int64_t)j * a.n_pad;
      const double *si = b.WS + (int64_t)i * a.n_pad, *sj = b.WS + (int64_t)j * a.n_pad;
      double t[6] = {0, 0, 0, 0, 0, 0};
      for (int gq = 0; gq < a.groups; ++gq) {
        int fl0, fl1;
        wg_range(b, a.nb, a.groups, gq, fl0, fl1);
        const int ge0 = fl0 * a.nb, ge1 = fl1 * a.nb;
        const int neg = (int)b.PART[gq * ns + 1], nlg = (int)b.PART[gq * ns + 2];
        for (int q = 0; q < neg; ++q) {
          const int k = b.CHG[ge0 + q];
          if (j <= i) {
            t[0] = t[0] + yi[k] * yj[k];
            t[2] = t[2] + si[k] * sj[k];
          }
          t[4] = t[4] + si[k] * yj[k];
        }
        for (int q = 0; q < nlg; ++q) {
          const int k = b.CHG[ge1 - 1 - q];
          if (j <= i) {
            t[1] = t[1] + yi[k] * yj[k];
            t[3] = t[3] + si[k] * sj[k];
          }
          t[5] = t[5] + si[k] * yj[k];
        }
      }
      // the old part of WN1 (lbfgsb.f formk): each entry owned by this thread
      if (j <= i) {
        wn1[i * m2 + j] = wn1[i * m2 + j] + t[0] - t[1];
        wn1[(m + i) * m2 + (m + j)] = wn1[(m + i) * m2 + (m + j)] - t[2] + t[3];
      }
      if (i <= j) wn1[(m + i) * m2 + j] = wn1[(m + i) * m2 + j] + t[4] - t[5];
      else wn1[(m + i) * m2 + j] = wn1[(m + i) * m2 + j] - t[4] + t[5];
    }
    if (updatd) {
      // the new row / column (c = col - 1), summed by FREEV
      const int c = col - 1;
      for (int j = threadIdx.x; j <= c; j += NT) {
        wn1[c * m2 + j] = b.NEWROW[j];                   // Y'ZZ'Y(c, j)
        wn1[(m + c) * m2 + (m + j)] = b.NEWROW[m + j];   // S'AA'S(c, j)
        wn1[(m + c) * m2 + j] = (j == c) ? b.NEWROW[3 * m + c] : b.NEWROW[2 * m + j];  // L_a(c, j) | R_z(c, c)
        if (j < c) wn1[(m + j) * m2 + c] = b.NEWROW[3 * m + j];  // R_z(j, c)
      }
    }
    __syncthreads();
    // WN (upper triangle, 2col x 2col)
    const double th = s.theta;
    for (int idx = threadIdx.x; idx < col * col; idx += NT) {
      const int iy = idx / col, jy = idx - iy * col;
      const int is = col + iy, is1 = m + iy;
      if (jy <= iy) {
        const int js = col + jy, js1 = m + jy;
        double v = wn1[iy * m2 + jy] / th;
        if (jy == iy) v = v + b.SY[iy * m + iy];
        wn[jy * ldw + iy] = v;
        wn[js * ldw + is] = wn1[is1 * m2 + js1] * th;
      }
      wn[jy * ldw + is] = (jy < iy) ? -wn1[is1 * m2 + jy] : wn1[is1 * m2 + jy];
    }
    __syncthreads();
    bool ok = wg_dpofa(wn, ldw, col);
    if (ok) {
      // dtrsl(wn, col, wn(1, js), 11) per column js of the (1,2) block: independent columns
      for (int js = col + threadIdx.x; js < col2; js += NT) {
        for (int j = 0; j < col; ++j) {
          double sum = wn[j * ldw + js];
          for (int k = 0; k < j; ++k) sum = sum - wn[k * ldw + j] * wn[k * ldw + js];
          wn[j * ldw + js] = sum / wn[j * ldw + j];
        }
      }
      __syncthreads();
      for (int idx = threadIdx.x; idx < col * col; idx += NT) {
        const int is = col + idx / col, js = col + idx % col;
        if (js < is) continue;
        double d = 0.0;
        for (int k = 0; k < col; ++k) d = d + wn[k * ldw + is] * wn[k * ldw + js];
        wn[is * ldw + js] = wn[is * ldw + js] + d;
      }
      __syncthreads();
      ok = wg_dpofa(wn + col * ldw + col, ldw, col);
    }
    if (threadIdx.x == 0) fok = ok;
    __syncthreads();
    if (ok && sm) stage_out(b.WN, m2, mwn, col2);
  } else {
    if (sm) stage_in(mwn, b.WN, m2, col2);
    if (threadIdx.x == 0) fok = 1;
    __syncthreads();
  }
  if (threadIdx.x >= 64) return;
  // subsm: wv = K^-1 wv (dtrsl job 11, negate the first col, dtrsl job 01) by wave 0
  const bool ok = fok && wsolve_k(wn, ldw, col2, col, b.WV);
  if (threadIdx.x == 0) {
    if (!ok) {
      refresh(s);
    } else {
      s.backtrack = 0;
      s.phase = PH_SUBSM;
    }
  }
}

// SUBSM: d = (1/theta) r + (1/theta^2) Z'W wv on the free variables, z = max(0, xcp + d)
// (3.0's projection), and lnsrlb's set-up over d = z - x: d'd, g'd, the step bound; the
// backtrack ratio if the projected step is not a descent direction.  BACKTRACK: z = xcp +
// alpha d with the blocking variable at its bound, then the same set-up.
template <bool BACK>
__global__ __launch_bounds__(NT) void nnls_subsm_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  NnlsState &s = *b.st;
  if (s.phase != (BACK ? PH_BACKTRACK : PH_SUBSM)) return;
  if (dbg_hit(a, s, g)) return;
  const int m = a.m, ns = nslots(m);
  const int cur = s.cur, col = s.col;
  const double *x = xbuf(b, cur), *gv = gbuf(b, cur);
  const double theta = s.theta, tsum = s.tsum;
  const bool done999 = s.walk_done == 2;
  const bool sub = !BACK && col > 0 && s.nfree > 0;
  const double alpha = s.alpha;
  const int ibd = s.ibd;
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  const int e0 = fl0 * a.nb, e1 = fl1 * a.nb;
  __shared__ double red[NW * 8];
  __shared__ int redi[NW * 2];
  double dtd = 0.0, gd = 0.0, stpmin = 1e10, amin = 1.0;
  int stpzero = 0, iword = 0, aidx = 0x7fffffff;
  const double ith = 1.0 / theta;
  for (int e = e0 + threadIdx.x; e < e1; e += NT) {
    const int iw = b.IW[e];
    const double xe = x[e], ge = gv[e];
    const double xc = xcp_of(iw, xe, ge, tsum, done999);
    double z = xc;
    if (iw <= 0 && (sub || BACK)) {
      double dd;
      if (BACK) {
        dd = b.DD[e];
        if (alpha < 1.0 && e == ibd) {
          dd = 0.0;
          z = 0.0;
        }
        z = z + alpha * dd;
      } else {
        dd = b.R[e];
        for (int j = 0; j < col; ++j)
          dd = dd + b.WY[(int64_t)j * a.n_pad + e] * b.WV[j] / theta +
               b.WS[(int64_t)j * a.n_pad + e] * b.WV[col + j];
        dd = dd * ith;
        b.DD[e] = dd;
        z = fmax(0.0, xc + dd);
        if (z == 0.0) iword = 1;
        // backtrack ratio (subsm, alpha loop over the free variables in order)
        if (dd < 0.0) {
          const double temp2 = 0.0 - xc;
          // reference index order: bin-major (k * nc + frame)
          const int fl = e / a.nb, k = e - fl * a.nb;
          const int eref = k * b.nc + fl;
          double cand = 2.0;
          if (temp2 >= 0.0) cand = 0.0;
          else if (dd * 1.0 < temp2) cand = temp2 / dd;
          if (cand < 1.0 && (cand < amin || (cand == amin && eref < aidx))) {
            amin = cand;
            aidx = eref;
          }
        }
      }
    }
    b.Z[e] = z;
    const double d = z - xe;
    dtd = dtd + d * d;
    gd = gd + ge * d;
    if (d < 0.0) {
      const double a2 = 0.0 - xe;
      if (a2 >= 0.0) stpzero = 1;
      else if (a2 / d < stpmin) stpmin = a2 / d;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  dtd = wave_sum(dtd);
  gd = wave_sum(gd);
  double smin = stpmin;
  for (int o = 32; o > 0; o >>= 1) smin = fmin(smin, __shfl_xor(smin, o));
  wave_argmin(amin, aidx);
  int flags = (stpzero ? 1 : 0) | (iword ? 2 : 0);
  for (int o = 32; o > 0; o >>= 1) flags |= __shfl_xor(flags, o);
  if (lane == 0) {
    red[w] = dtd;
    red[NW + w] = gd;
    red[2 * NW + w] = smin;
    red[3 * NW + w] = amin;
    redi[w] = aidx;
    redi[NW + w] = flags;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s0 = 0, s1 = 0, s2 = 1e10, s3 = 1.0;
    int i3 = 0x7fffffff, fl = 0;
    for (int q = 0; q < NW; ++q) {
      s0 += red[q];
      s1 += red[NW + q];
      s2 = fmin(s2, red[2 * NW + q]);
      if (red[3 * NW + q] < s3 || (red[3 * NW + q] == s3 && redi[q] < i3)) {
        s3 = red[3 * NW + q];
        i3 = redi[q];
      }
      fl |= redi[NW + q];
    }
    double *pq = b.PART + g * ns;
    pq[0] = s0;
    pq[1] = s1;
    pq[2] = s2;
    pq[3] = s3;
    pq[4] = (double)i3;
    pq[5] = (double)fl;
  }
  if (!arrive_last(b.st, a.groups)) return;
  if (threadIdx.x != 0) return;
  double dtds = 0, gds = 0, smn = 1e10, am = 1.0;
  int ai = 0x7fffffff, fl = 0;
  for (int q = 0; q < a.groups; ++q) {
    const double *pq = b.PART + q * ns;
    dtds += pq[0];
    gds += pq[1];
    smn = fmin(smn, pq[2]);
    const int iq = (int)pq[4];
    if (pq[3] < am || (pq[3] == am && iq < ai)) {
      am = pq[3];
      ai = iq;
    }
    fl |= (int)pq[5];
  }
  if (!BACK && sub && (fl & 2) && gds > 0.0) {
    // positive directional derivative in the projection: backtrack along d from xcp
    s.alpha = am;
    if (am < 1.0) {
      // the blocking variable, back to the workspace index
      const int k = ai / b.nc, fr = ai - k * b.nc;
      s.ibd = fr * a.nb + k;
    } else {
      s.ibd = -1;
    }
    s.phase = PH_BACKTRACK;
    return;
  }
  ls_begin(s, a.active, dtds, gds, smn, fl & 1);
}

__global__ __launch_bounds__(NT) void nnls_finish_kernel(const Args a) {
  const int blk = blockIdx.y, g = blockIdx.x;
  Blk b = blk_view(a, blk);
  int fl0, fl1;
  wg_range(b, a.nb, a.groups, g, fl0, fl1);
  const double *x = xbuf(b, b.st->cur);
  for (int fl = fl0; fl < fl1; ++fl) {
    float *o = a.S + ((int64_t)b.item * a.F + b.f0 + fl) * a.nb;
    for (int k = threadIdx.x; k < a.nb; k += NT) o[k] = (float)x[fl * a.nb + k];
  }
}

// frames past an item's length: zero magnitudes (the batched layout's padding)
__global__ void nnls_zero_tail_kernel(float *S, int B, int F, int nb, const int32_t *frames) {
  const int b = blockIdx.y;
  const int Fb = frames ? min(frames[b], F) : F;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + (int64_t)Fb * nb;
       i < (int64_t)F * nb; i += (int64_t)gridDim.x * blockDim.x)
    S[(int64_t)b * F * nb + i] = 0.f;
}

__global__ void nnls_status_kernel(const Args a, int *status_out, double *info) {
  for (int blk = blockIdx.x * blockDim.x + threadIdx.x; blk < a.n_blocks; blk += gridDim.x * blockDim.x) {
    Blk b = blk_view(a, blk);
    const int st = b.st->status;
    if (st & ~(ST_CONV | ST_MAXITER)) atomicOr(status_out, st & ~(ST_CONV | ST_MAXITER));
    atomicMax(status_out + 1, b.st->it);
    if (info) {
      info[4 * blk + 0] = b.st->it;
      info[4 * blk + 1] = b.st->nfev;
      info[4 * blk + 2] = b.st->f;
      info[4 * blk + 3] = b.st->sbgnrm;
    }
  }
}

bool check_args(const ftmi_nnls_lbfgsb_args *p) {
  return p && p->mel && p->blocks && p->rowvals && p->rowptr && p->rowlo && p->bin_rows &&
         p->bin_w && p->pinv && p->workspace && p->S && p->active && p->B > 0 && p->F > 0 &&
         p->n_mels > 0 && p->n_mels <= 512 && p->n_bins > 0 && p->n_bins <= 2112 &&
         p->n_blocks > 0 && p->groups > 0 && p->groups <= 64 && p->m > 0 && p->max_frames > 0;
}

Args make_args(const ftmi_nnls_lbfgsb_args *p) {
  Args a;
  a.mel = p->mel;
  a.B = p->B;
  a.F = p->F;
  a.n_mels = p->n_mels;
  a.nb = p->n_bins;
  a.denorm = p->denorm;
  a.blocks = p->blocks;
  a.n_blocks = p->n_blocks;
  a.groups = p->groups;
  a.m = p->m;
  a.mref = p->n_bins;  // librosa: fmin_l_bfgs_b(..., m=A.shape[1])
  a.ncmax = p->max_frames;
  a.maxiter = p->maxiter > 0 ? p->maxiter : 15000;
  a.dbg_stop = p->dbg_stop;
  a.rowvals = p->rowvals;
  a.rowptr = p->rowptr;
  a.rowlo = p->rowlo;
  a.bin_rows = p->bin_rows;
  a.bin_w = p->bin_w;
  a.pinv = p->pinv;
  a.ws = (unsigned char *)p->workspace;
  a.n_pad = ((int64_t)p->n_bins * p->max_frames + 255) & ~(int64_t)255;
  a.blk_bytes = carve(nullptr, a.n_pad, a.m, a.groups, nullptr);
  a.S = p->S;
  a.active = p->active;
  return a;
}

}  // namespace

extern "C" int64_t ftmi_nnls_lbfgsb_workspace_bytes(int32_t n_blocks, int32_t n_bins,
                                                    int32_t max_frames, int32_t m, int32_t groups) {
  if (n_blocks <= 0 || n_bins <= 0 || max_frames <= 0 || m <= 0 || groups <= 0) return 0;
  const int64_t n_pad = ((int64_t)n_bins * max_frames + 255) & ~(int64_t)255;
  return (int64_t)n_blocks * carve(nullptr, n_pad, m, groups, nullptr);
}

extern "C" int ftmi_nnls_lbfgsb_start(const ftmi_nnls_lbfgsb_args *p, ftmi_stream_t stream) {
  if (!check_args(p)) return FTMI_E_ARG;
  const Args a = make_args(p);
  const hipStream_t s = ftmi_hs(stream);
  hipLaunchKernelGGL(nnls_start_kernel, dim3(a.groups, a.n_blocks), dim3(NT), 0, s, a);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_nnls_lbfgsb_cycles(const ftmi_nnls_lbfgsb_args *p, int32_t cycles,
                                       ftmi_stream_t stream) {
  if (!check_args(p) || cycles < 0) return FTMI_E_ARG;
  const Args a = make_args(p);
  const hipStream_t s = ftmi_hs(stream);
  const dim3 sweep(a.groups, a.n_blocks), single(a.n_blocks);
  for (int c = 0; c < cycles; ++c) {
    hipLaunchKernelGGL(nnls_eval_kernel, sweep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_cauchy_kernel, sweep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_walk_kernel, single, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_freev_kernel, sweep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_formk_kernel, single, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_subsm_kernel<false>, sweep, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(nnls_subsm_kernel<true>, sweep, dim3(NT), 0, s, a);
    FTMI_CHECK_LAUNCH();
  }
  return FTMI_OK;
}

extern "C" int ftmi_nnls_lbfgsb_finish(const ftmi_nnls_lbfgsb_args *p, const int32_t *frames,
                                       int32_t *status, double *info, ftmi_stream_t stream) {
  if (!check_args(p) || !status) return FTMI_E_ARG;
  const Args a = make_args(p);
  const hipStream_t s = ftmi_hs(stream);
  hipLaunchKernelGGL(nnls_finish_kernel, dim3(a.groups, a.n_blocks), dim3(NT), 0, s, a);
  hipLaunchKernelGGL(nnls_zero_tail_kernel, dim3(64, a.B), dim3(256), 0, s, a.S, a.B, a.F, a.nb,
                     frames);
  hipLaunchKernelGGL(nnls_status_kernel, dim3(1), dim3(256), 0, s, a, (int *)status, info);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}
