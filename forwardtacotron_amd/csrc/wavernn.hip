// WaveRNN vocoder (reference: models/fatchord_version.py, the `gen_forward.py wavernn`
// option) on gfx950.
//
//   wr_stretch_conv_kernel   Stretch2d(s, 1) + Conv2d(1, 1, (1, 2s+1), pad (0, s)), one
//                            UpsampleNetwork.up_layers pair (:74-81, :88), on time-major rows
//   wavernn_kernel           the sample loop of WaveRNN.generate (:203-241) — or, teacher-
//                            forced, WaveRNN.forward (:145-169) — as ONE persistent launch
//   wr_unfold_kernel         generate's tail (:246-261): mu-law decode, xfade_and_unfold
//                            (:343-406), crop, 20-hop fade-out; float64 like the reference
//
// The sample loop.  Per step t and fold b the reference computes
//   x = I([s_{t-1}, m_t, a1_t]);  h1 = GRU1(x, h1);  x += h1;  h2 = GRU2([x, a2_t], h2);
//   x += h2;  y1 = relu(fc1([x, a3_t]));  y2 = relu(fc2([y1, a4_t]));  l = fc3(y2);
//   s_t ~ Categorical(softmax(l))  (RAW)  |  discretized mix-of-logistics draw (MOL)
// Everything that does not depend on the sample chain is moved off it (host packing,
// float64, once per weights version):
//   W_ih1 x + b_ih1  = G1(m_t, a1_t) + u1 s_{t-1},  u1 = W_ih1 w0  (w0 = I.weight[:, 0])
//   W_ih2 [x, a2] + b = Q(m_t, a1_t, a2_t) + u2 s_{t-1} + W_ih2a h1
//   fc1([x, a3])     = R(m_t, a1_t, a3_t) + v1 s_{t-1} + W_fc1a (h1 + h2)
//   fc2([y1, a4])    = S(a4_t) + W_fc2a y1
// G1, Q, R, S split into a per-FRAME part (the aux features are constant over a hop: one
// small GEMM on the caller side, `cond` rows) and a per-SAMPLE part from the 80 upsampled
// mel features (`wm`, computed here in the idle phase of each step).  What stays on the
// chain per step: W_hh1 h1 / W_hh2 h2 (both from the previous step: off the chain too),
// W_ih2a h1_t, W_fc1a (h1 + h2), W_fc2a y1, W_fc3 y2 and the draw — five all-to-all edges.
//
// Decomposition: 256 workgroups (one per CU, co-residency checked by an arrival barrier
// with a bounded spin).  With two or more folds they form TWO INSTANCES of 128 workgroups,
// each the whole pipeline for half of the folds: the per-step cost is the hand-off latency
// of the five edges, which does not shrink with fewer folds, so two half-size pipelines
// side by side run twice the folds per unit of time.  Per instance (NI instances,
// 512 threads per workgroup at NI = 2), two roles:
//   GRU workgroups: UG = 4 NI units of both GRUs (3 UG gate rows of W_hh1, W_hh2, W_ih2a
//     in VGPRs), the cell updates, h1 / h2 publication.
//   FC workgroups: FR = 4 NI rows of fc1 and fc2, NCR rows of fc3, the Gumbel draw of
//     those rows, publication of y1, y2 and the rows' best (value, index).
// Matrix-vector products are exact fp32 FMAs on the VALU: a 16-wide MFMA tile would carry
// B <= 32 live columns at most and the chain is bound by the hand-offs, not the flops.
// Thread layout of a product: slot s = tid / 8 owns (row, k-part), its 8 lanes hold
// interleaved 4-float chunks of that row's k-part, placed so that the slots of one wave
// read one contiguous run of the vector per instruction (conflict-free; slots of other
// rows read the same addresses: broadcast); the 8 lanes meet by DPP adds, the k-parts in
// a fixed order through LDS.
//
// Hand-off: the data is the flag (rnn.hip): every exchanged value carries the step tag in
// its mantissa LSB (the tagged value is the one used everywhere), two parity halves,
// write-through (`sc1`) 4-byte stores, `sc1` 16-byte polls until every word carries the tag
// (MI355X_MICROARCH.md, data-tagged granules).  The draw's partials are 8-byte {value,
// index|tag} granules written by one store.  Parity double buffering is race-free: a
// producer of step t has acquired s_{t-1}, which every workgroup published only after
// consuming step t-2's data.  Every spin is bounded: a timeout sets the error word and
// FTMI_STATUS_RNN_TIMEOUT in *status, never a silent result.
//
// Randomness: Philox4x32-10 (Salmon et al., Random123), key = seed, counter (t, b, k/4, 0)
// for class k of RAW (the Gumbel form argmax_k l_k - log(-log u_k) of torch.multinomial's
// single draw argmax p_k / E_k, E_k ~ Exp(1)); MOL: counters (t, b, k/4, 1) for the
// mixture choice and (t, b, 0, 2) for the logistic draw, mapped to uniform_(1e-5, 1-1e-5)
// like utils/distribution.py:113,122.  oracle/wr_torch_cpu.py restates the same stream.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int WR_R = 512;    // rnn_dims
constexpr int WR_F = 512;    // fc_dims
constexpr int WR_NM = 80;    // mel features (feat_dims)
constexpr int WR_NA = 32;    // aux_dims = res_out_dims / 4
constexpr int WR_NT = 256;   // threads per workgroup of a single-instance launch
constexpr int WR_NF = 128;   // FC workgroups of a single-instance launch (draw-slot stride)
constexpr int WR_GRID = 256; // workgroups per launch
constexpr int WR_NBMAX = 32;         // folds per launch
constexpr int WR_COND = 6 * WR_R + 2 * WR_F;  // cond row: [G1 3R | Q 3R | R F | S F]
// exchange slots: h1, h2, y1, y2 ([2][NBV][512] floats each), then the draw partials
// ([2][NBV][128] 8-byte granules)
constexpr int XS_VEC = 2 * WR_NBMAX * 512;   // floats per vector slot
constexpr int XS_Z = 2 * WR_NBMAX * WR_NF * 2;  // words of the draw slot
constexpr int WS_CTRL = 128;                 // control words (error, arrival, diag stamps)
constexpr int WS_STAMPS = 64;                // 2 x 16 u64 phase sums (FTMI_WR_STAMPS=1)
constexpr unsigned SPIN_DEFAULT = 1u << 22;
constexpr unsigned STATUS_TIMEOUT = 4u;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned step_tag(int t) { return (((unsigned)t >> 1) & 1u) ^ 1u; }
__device__ __forceinline__ float tagged(float v, int t) {
  return __uint_as_float((__float_as_uint(v) & ~1u) | step_tag(t));
}
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Philox4x32-10 (Random123): 10 rounds of two 32x32->64 multiplies
__device__ __forceinline__ u32x4 philox(u32x4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    c = (u32x4){hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ float u01(unsigned x) {  // (0, 1), exact in fp32
  return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-08f;
}
__device__ __forceinline__ unsigned pword(const u32x4 &v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// lane exchanges inside groups of 8 lanes by DPP (no LDS round trip like ds_bpermute):
// quad_perm [1,0,3,2] (xor 1), quad_perm [2,3,0,1] (xor 2), row_half_mirror (i <-> 7 - i)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// sum over the 8 lanes of a group (every lane gets it)
__device__ __forceinline__ float sum8(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  return v;
}

struct WrParams {
  const float *w_hh1, *w_hh2, *w_ih2a;  // [3R][R]
  const float *w_fc1a, *w_fc2a;         // [F][R], [F][F]
  const float *w_fc3, *b_fc3;           // [NC][F], [NC]
  const float *b_hh1, *b_hh2;           // [3R]
  const float *u1, *u2, *v1;            // [3R], [3R], [F]
  const float *wm;                      // [6R + F][80]: mel columns of G1 | Q | R
  const float *cond;                    // (n_frames + 1) rows of WR_COND floats
  const float *mel;                     // (items * item_rows) rows of 80 floats
  int bias_row;                         // cond row of a padded position (biases only)
  int item_rows, frames_per_item, hop, fold_stride, batched;
  int fold0;                            // first fold of this launch (batched: its offset)
  const float *xin;                     // teacher-forced input samples (B_total, L) or NULL
  float *samples;                       // generate: (B_total, L) output samples
  float *logits;                        // teacher-forced: (B_total, L, NC) or NULL
  float *xch;                           // exchange slots
  unsigned *ws;                         // control words
  unsigned *status;
  int B, L, NC, mol;
  int stamps;                           // diag: per-phase s_memtime sums of WG 0 / WG 128
  unsigned k0, k1;                      // Philox key
  unsigned spin_limit;
};

__device__ __forceinline__ void report_timeout(const WrParams &p) {
  __hip_atomic_store(p.ws, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (p.status) atomicOr(p.status, STATUS_TIMEOUT);
}

// position of fold b (launch-local), step t in the conditioning rows
struct Pos {
  int mel_row;    // -1: padded (zero) position
  int cond_row;
};
__device__ __forceinline__ Pos position(const WrParams &p, int b, int t) {
  const int fb = p.fold0 + b;
  const int g = p.batched ? fb * p.fold_stride + t : t;
  const int item = p.batched ? 0 : fb;
  Pos r;
  if (t < p.L && g < p.item_rows) {
    r.mel_row = item * p.item_rows + g;
    r.cond_row = item * p.frames_per_item + g / p.hop;
  } else {
    r.mel_row = -1;
    r.cond_row = p.bias_row;
  }
  return r;
}

// Geometry of one instance (a replica of the weight-distributed pipeline over its own
// share of the folds): NI instances x (NG GRU + NF FC workgroups) = 256 workgroups of
// NT = 256 NI threads; a GRU workgroup owns UG = 4 NI units, an FC workgroup FR = 4 NI rows.
template <int NI>
struct Geo {
  static constexpr int NT = WR_NT * NI;
  static constexpr int W = WR_GRID / NI;  // workgroups per instance
  static constexpr int NG = W / 2, NF = W / 2;
  static constexpr int UG = WR_R / NG, FR = WR_F / NF;
  static constexpr int SLOTS = NT / 8;
};

// Two instances (NI = 2): a GRU workgroup's idle-phase weights (W_hh1, W_hh2: 48 active
// slots x 8 lanes x 32 floats each) live in LDS, [matrix][j][lane][4] so a wave's 16-B reads
// are consecutive; only W_ih2a (on the sample chain) stays in VGPRs: 512 threads leave half
// the registers of a one-instance workgroup.
template <int NI>
struct WlDims {
  static constexpr int LANES = NI == 2 ? 6 * (WR_R / (WR_GRID / NI / 2)) * 8 : 0;  // 6 UG slots x 8
  static constexpr int FLOATS = NI == 2 ? 2 * 8 * LANES * 4 : 1;
};

template <int NBV, int NI>
struct WrShared {
  // every member read with 16-B LDS accesses is 16-B aligned (a misaligned vec made the
  // one-instance products 4x slower: wl is a single float there)
  __attribute__((aligned(16))) float wl[WlDims<NI>::FLOATS];  // NI = 2: W_hh1 / W_hh2
  __attribute__((aligned(16))) float vec[NBV * 512];  // the acquired vector (h1 / h2 / y1 / y2)
  float part[3][Geo<NI>::SLOTS][NBV];  // per-slot partial sums of the products
  float partm[Geo<NI>::SLOTS][NBV];    // per-slot partial sums of the mel conditioning
  __attribute__((aligned(16))) float melv[NBV * WR_NM];  // this step's mel rows
  float sval[NBV];               // s_{t-1}
  unsigned long long stamp[12];  // diag phase sums (thread 0)
  int abort_flag;
};

// acquire the tagged vector of exchange slot `slot`, step t, into LDS (add: accumulate).
// Every chunk of the thread is requested at once, then only the stale ones are polled
// again (a serial poll per chunk would pay the hand-off latency once per chunk).  On a
// timeout the workgroup's abort flag is set; the caller barriers and checks it.
template <int NBV, int NI>
__device__ __forceinline__ void acquire_vec(const WrParams &p, WrShared<NBV, NI> &sh, int slot, int t,
                                            bool add) {
  constexpr int NT = Geo<NI>::NT;
  constexpr int PER = NBV * 128 / NT;  // 16-B chunks per thread
  const int tid = threadIdx.x;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.xch, (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned want = step_tag(t);
  const int soff = (slot * XS_VEC + (t & 1) * WR_NBMAX * 512) * 4;
  u32x4 r[PER];
  unsigned stale = 0;  // bit i: chunk i still to be (re)loaded
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    r[i] = (u32x4){0u, 0u, 0u, 0u};
    if (((tid + i * NT) >> 7) < p.B) stale |= 1u << i;
  }
  for (unsigned spins = 0; stale; ++spins) {
    // compiler memory barrier: the poll stores nothing, so LICM could hoist the loads out
    // and spin on stale values (as rnn.hip's polls once did)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (stale & (1u << i))
        r[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (unsigned)((tid + i * NT) * 16), soff, 16);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (stale & (1u << i)) {
        const u32x4 v = r[i];
        const bool fresh = want ? ((v.x & v.y & v.z & v.w) & 1u) != 0u
                                : ((v.x | v.y | v.z | v.w) & 1u) == 0u;
        if (fresh) stale &= ~(1u << i);
      }
    if (stale && spins > p.spin_limit) {
      sh.abort_flag = 1;
      report_timeout(p);
      break;
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const f32x4 v = __builtin_bit_cast(f32x4, r[i]);
    f32x4 *dst = (f32x4 *)&sh.vec[(tid + i * NT) * 4];
    if (add) *dst = *dst + v;
    else *dst = v;
  }
}

__device__ __forceinline__ void publish(const WrParams &p, int slot, int t, int b, int col, float v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.xch, (short)0, 0x7FFFFFF0, 0x00020000);
  const int soff = (slot * XS_VEC + (t & 1) * WR_NBMAX * 512) * 4;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (unsigned)((b * 512 + col) * 4),
                                        soff, 16);
}

// draw slot granule (t, b, producer f): {value (tagged LSB), index | tag << 16}
__device__ __forceinline__ void publish_z(const WrParams &p, int t, int b, int f, float v, int idx) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.xch, (short)0, 0x7FFFFFF0, 0x00020000);
  const int soff = (4 * XS_VEC + (t & 1) * WR_NBMAX * WR_NF * 2) * 4;
  const u32x2 g = {__float_as_uint(tagged(v, t)), (unsigned)idx | (step_tag(t) << 16)};
  __builtin_amdgcn_raw_buffer_store_b64(g, rsrc, (unsigned)(((b * WR_NF) + f) * 8), soff, 16);
}

// s_t (the sample drawn from step t's logits) of every fold into sh.sval; with `store`
// also to p.samples.  Producers of the draw slot: RAW the 128 FC workgroups (their rows'
// best Gumbel score and its class), MOL the NC logits.  8 threads per fold, each with its
// (up to 8) 16-byte granule pairs requested at once.  On a timeout the abort flag is set
// (visible after the internal barrier).
template <int NBV, int NI>
__device__ __forceinline__ void acquire_sample(const WrParams &p, WrShared<NBV, NI> &sh, int t, bool store) {
  const int tid = threadIdx.x;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.xch, (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned want = step_tag(t);
  const int soff = (4 * XS_VEC + (t & 1) * WR_NBMAX * WR_NF * 2) * 4;
  const int np = p.mol ? p.NC : Geo<NI>::NF / 2;  // RAW: the fc3 half of the FC workgroups
  const int b = tid >> 3, part = tid & 7;
  constexpr int PER = Geo<NI>::NF / 16;
  u32x4 r[PER];
  unsigned stale = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    r[i] = (u32x4){0u, 0u, 0u, 0u};
    if (b < p.B && part * 2 + 16 * i < np) stale |= 1u << i;
  }
  for (unsigned spins = 0; stale; ++spins) {
    asm volatile("" ::: "memory");  // keep the poll's loads in the loop (see above)
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (stale & (1u << i))
        r[i] = __builtin_amdgcn_raw_buffer_load_b128(
            rsrc, (unsigned)((b * WR_NF + part * 2 + 16 * i) * 8), soff, 16);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (stale & (1u << i)) {
        const u32x4 v = r[i];
        const bool two = part * 2 + 16 * i + 1 < np;
        const bool f0 = (v.x & 1u) == want && ((v.y >> 16) & 1u) == want;
        const bool f1 = !two || ((v.z & 1u) == want && ((v.w >> 16) & 1u) == want);
        if (f0 && f1) stale &= ~(1u << i);
      }
    if (stale && spins > p.spin_limit) {
      sh.abort_flag = 1;
      report_timeout(p);
      break;
    }
  }
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  if (b < p.B) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = part * 2 + 16 * i;
      if (q >= np) continue;
      const u32x4 v = r[i];
      const float v0 = __uint_as_float(v.x), v1 = __uint_as_float(v.z);
      const int i0 = (int)(v.y & 0xFFFFu), i1 = (int)(v.w & 0xFFFFu);
      if (p.mol) {
        sh.vec[b * 512 + q] = v0;
        if (q + 1 < np) sh.vec[b * 512 + q + 1] = v1;
      } else {
        if (v0 > best || (v0 == best && i0 < bidx)) best = v0, bidx = i0;
        if (q + 1 < np && (v1 > best || (v1 == best && i1 < bidx))) best = v1, bidx = i1;
      }
    }
  }
  if (!p.mol) {
    {  // (max, first index) over the fold's 8 lanes
      float ob = dppf<0xB1>(best);
      int oi = dppi<0xB1>(bidx);
      if (ob > best || (ob == best && oi < bidx)) best = ob, bidx = oi;
      ob = dppf<0x4E>(best);
      oi = dppi<0x4E>(bidx);
      if (ob > best || (ob == best && oi < bidx)) best = ob, bidx = oi;
      ob = dppf<0x141>(best);
      oi = dppi<0x141>(bidx);
      if (ob > best || (ob == best && oi < bidx)) best = ob, bidx = oi;
    }
    if (part == 0 && b < NBV) {
      // reference :237: 2 * idx.float() / (n_classes - 1.) - 1. in fp32
      const float v = (2.0f * (float)bidx) / (float)(p.NC - 1) - 1.0f;
      sh.sval[b] = b < p.B ? v : 0.f;
    }
  }
  __syncthreads();
  if (p.mol) {
    if (tid < p.B) {
      // utils/distribution.py:105-127 for one step, fp32, each op rounded like torch's
      const int nr = p.NC / 3;
      const float *l = &sh.vec[tid * 512];
      int am = 0;
      float bt = -INFINITY;
      for (int k = 0; k < nr; ++k) {
        const u32x4 w = philox((u32x4){(unsigned)t, (unsigned)(p.fold0 + tid), (unsigned)(k >> 2), 1u},
                               p.k0, p.k1);
        const float u = 1e-5f + u01(pword(w, k & 3)) * (1.0f - 2e-5f);
        const float tv = l[k] - logf(-logf(u));
        if (tv > bt) bt = tv, am = k;
      }
      const u32x4 w2 = philox((u32x4){(unsigned)t, (unsigned)(p.fold0 + tid), 0u, 2u}, p.k0, p.k1);
      const float u = 1e-5f + u01(w2.x) * (1.0f - 2e-5f);
      const float mean = l[nr + am];
      const float ls = fmaxf(l[2 * nr + am], -32.23619130191664f);  // log(1e-14), fp32
      const float d = logf(u) - logf(1.0f - u);
      float x = mean + expf(ls) * d;
      x = fminf(fmaxf(x, -1.0f), 1.0f);
      sh.sval[tid] = x;
    }
    __syncthreads();
  }
  if (store && tid < p.B && p.samples) p.samples[(size_t)(p.fold0 + tid) * p.L + t] = sh.sval[tid];
}

// this step's mel rows, fetched one step ahead into registers (the global-load latency
// hides behind a whole step) and stored to LDS at the top of the step
template <int NBV, int NI>
struct MelPrefetch {
  static constexpr int NT = Geo<NI>::NT;
  static constexpr int N = (NBV * (WR_NM / 4) + NT - 1) / NT;
  f32x4 r[N];
  __device__ __forceinline__ void fetch(const WrParams &p, int t) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int f = threadIdx.x + i * NT;
      const int b = f / (WR_NM / 4), c = (f % (WR_NM / 4)) * 4;
      r[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (f < NBV * (WR_NM / 4) && b < p.B) {
        const Pos ps = position(p, b, t);
        if (ps.mel_row >= 0) r[i] = *(const f32x4 *)&p.mel[(size_t)ps.mel_row * WR_NM + c];
      }
    }
  }
  __device__ __forceinline__ void store(WrShared<NBV, NI> &sh) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int f = threadIdx.x + i * NT;
      if (f < NBV * (WR_NM / 4)) *(f32x4 *)&sh.melv[f * 4] = r[i];
    }
  }
};

// (k = kbase + j JS + 4 kl + e: the lanes of a wave read contiguous runs, conflict-free).
// Four folds per pass with independent accumulators: one wave per SIMD cannot hide the
// LDS and FMA latencies of a single fold's chain.  Folds past B read the zeroed rows of
// the vector (B is rounded up to 4 <= NBV); their partials are never read.
template <int NJ, int JS>
__device__ __forceinline__ void matvec(const float (&w)[NJ * 4], const float *vec, int kbase,
                                       int kl, float *out, bool active, int B) {
  for (int b = 0; b < B; b += 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NJ; j += 2) {
      // two k-chunks of four folds in flight (8 loads); the barrier keeps the compiler from
      // hoisting every chunk's loads (a register per loaded float) while letting the
      // arithmetic of this pair sink below the next pair's loads
      f32x4 h[2][4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          h[jj][q] = *(const f32x4 *)&vec[(b + q) * 512 + kbase + (j + jj) * JS + kl * 4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q] = fmaf(w[4 * (j + jj)], h[jj][q].x, acc[q]);
          acc[q] = fmaf(w[4 * (j + jj) + 1], h[jj][q].y, acc[q]);
          acc[q] = fmaf(w[4 * (j + jj) + 2], h[jj][q].z, acc[q]);
          acc[q] = fmaf(w[4 * (j + jj) + 3], h[jj][q].w, acc[q]);
        }
      __builtin_amdgcn_sched_barrier(0x0006);  // only VALU / SALU may cross
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = sum8(acc[q]);
    if (active && kl == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) out[b + q] = acc[q];
    }
  }
}

// the same product with the lane's weights read from LDS (wl: [j][lanes][4], this lane's
// column), once per four-fold block
template <int NJ, int JS, int LANES>
__device__ __forceinline__ void matvec_lds(const float *wl, const float *vec, int kbase, int kl,
                                           float *out, bool active, int B) {
  const int lane = threadIdx.x < LANES ? threadIdx.x : 0;
  for (int b = 0; b < B; b += 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NJ; j += 2) {
      f32x4 h[2][4], w[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        w[jj] = *(const f32x4 *)&wl[((j + jj) * LANES + lane) * 4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          h[jj][q] = *(const f32x4 *)&vec[(b + q) * 512 + kbase + (j + jj) * JS + kl * 4];
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q] = fmaf(w[jj].x, h[jj][q].x, acc[q]);
          acc[q] = fmaf(w[jj].y, h[jj][q].y, acc[q]);
          acc[q] = fmaf(w[jj].z, h[jj][q].z, acc[q]);
          acc[q] = fmaf(w[jj].w, h[jj][q].w, acc[q]);
        }
      __builtin_amdgcn_sched_barrier(0x0006);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = sum8(acc[q]);
    if (active && kl == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) out[b + q] = acc[q];
    }
  }
}

// mel conditioning: 80 = 8 lanes x 10, lane kl takes k = kl + 8 j; four folds per pass
__device__ __forceinline__ void matvec_mel(const float (&w)[10], const float *melv, int kl, float *out,
                                           bool active, int B) {
  for (int b = 0; b < B; b += 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 10; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = fmaf(w[j], melv[(b + q) * WR_NM + kl + 8 * j], acc[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = sum8(acc[q]);
    if (active && kl == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) out[b + q] = acc[q];
    }
  }
}

template <int NBV, int NI>
__global__ __launch_bounds__(Geo<NI>::NT, 1) void wavernn_kernel(const WrParams p0) {
  using G = Geo<NI>;
  constexpr int NT = G::NT, UG = G::UG, FR = G::FR, NG = G::NG;
  __shared__ WrShared<NBV, NI> sh;
  const int tid = threadIdx.x;
  const int s = tid >> 3, kl = tid & 7;
  // this workgroup's instance: its folds and exchange buffers
  const int inst = blockIdx.x / G::W, local = blockIdx.x % G::W;
  WrParams p = p0;
  {
    const int bi = (p0.B + NI - 1) / NI;
    p.fold0 = p0.fold0 + inst * bi;
    p.B = p0.B - inst * bi < bi ? p0.B - inst * bi : bi;
    p.xch = p0.xch + (size_t)inst * (4 * XS_VEC + XS_Z);
  }
  // diag (FTMI_WR_STAMPS=1): thread 0 of instance 0's first GRU and first FC workgroup sum
  // s_memtime deltas per phase into the workspace (timing only; outputs unchanged)
  const bool stamping = p.stamps && tid == 0 && (blockIdx.x == 0 || blockIdx.x == NG);
  if (tid < 12) sh.stamp[tid] = 0;
  if (tid == 0) sh.stamp[11] = __builtin_amdgcn_s_memtime();  // slot 11: last stamp
#define WR_STAMP(i)                                              \
  do {                                                           \
    if (stamping) {                                              \
      const unsigned long long now__ = __builtin_amdgcn_s_memtime(); \
      sh.stamp[i] += now__ - sh.stamp[11];                       \
      sh.stamp[11] = now__;                                      \
    }                                                            \
  } while (0)

  // ---- arrival barrier: all WR_GRID workgroups must be resident (bounded) -----------
  if (tid == 0) {
    sh.abort_flag = 0;
    __hip_atomic_fetch_add(p.ws + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(p.ws + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)WR_GRID) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > p.spin_limit) {
        sh.abort_flag = 1;
        report_timeout(p);
        break;
      }
    }
  }
  for (int i = tid; i < NBV * 512; i += NT) sh.vec[i] = 0.f;
  for (int i = tid; i < NBV; i += NT) sh.sval[i] = 0.f;
  __syncthreads();
  if (sh.abort_flag || p.B <= 0) return;

  const bool gru = local < NG;
  if (gru) {
    // ================================ GRU workgroup =====================================
    const int u0 = local * UG;
    const bool act = s < 6 * UG;  // 3 UG gate rows x 2 k-parts
    const int r = s >> 1, kp = s & 1;
    // inactive slots (s >= 6 UG) hold a valid row's weights: their sums are never stored
    const int rc = act ? r : 0;
    const int mrow = (rc / UG) * WR_R + u0 + rc % UG;
    constexpr bool WL = NI == 2;
    constexpr int LANES = WlDims<NI>::LANES;
    float w1[WL ? 1 : 32], w2[WL ? 1 : 32], w3[32], wmr[10];
    {
      // one base address per matrix, 16-B loads at immediate offsets (k = 64 j + 32 kp + 4 kl + e)
      const size_t off = (size_t)mrow * WR_R + kp * 32 + kl * 4;
      const float *a1 = p.w_hh1 + off, *a2 = p.w_hh2 + off, *a3 = p.w_ih2a + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 x1 = *(const f32x4 *)(a1 + j * 64), x2 = *(const f32x4 *)(a2 + j * 64),
                    x3 = *(const f32x4 *)(a3 + j * 64);
#pragma unroll
        for (int e = 0; e < 4; ++e) w3[4 * j + e] = x3[e];
        if constexpr (WL) {
          if (tid < LANES) {
            *(f32x4 *)&sh.wl[(j * LANES + tid) * 4] = x1;
            *(f32x4 *)&sh.wl[((8 + j) * LANES + tid) * 4] = x2;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) w1[4 * j + e] = x1[e], w2[4 * j + e] = x2[e];
        }
      }
    }
    __syncthreads();
    {  // mel rows: slot s < 6 UG = (block s / 3 UG: G1 | Q, gate row s % 3 UG)
      const int sc = act ? s : 0;
      const int rr = sc % (3 * UG);
      const int row = (sc / (3 * UG)) * 3 * WR_R + (rr / UG) * WR_R + u0 + rr % UG;
      const float *am = p.wm + (size_t)row * WR_NM + kl;
#pragma unroll
      for (int j = 0; j < 10; ++j) wmr[j] = am[8 * j];
    }
    // cell thread (unit cu, fold cb)
    const bool cell = tid < UG * p.B;
    const int cu = tid % UG, cb = tid / UG;
    const int unit = u0 + cu;
    float bh1[3], bh2[3], uu1[3], uu2[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      bh1[q] = p.b_hh1[q * WR_R + unit];
      bh2[q] = p.b_hh2[q * WR_R + unit];
      uu1[q] = p.u1[q * WR_R + unit];
      uu2[q] = p.u2[q * WR_R + unit];
    }
    float h1 = 0.f, h2 = 0.f;
    // conditioning of the cell's unit (frame terms) and the mel rows, one step ahead
    float gn[3] = {0.f, 0.f, 0.f}, qn[3] = {0.f, 0.f, 0.f};
    auto fetch_cond = [&](int t) {
      if (cell) {
        const Pos ps = position(p, cb, t);
        const float *crow = p.cond + (size_t)ps.cond_row * WR_COND;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          gn[q] = crow[q * WR_R + unit];
          qn[q] = crow[3 * WR_R + q * WR_R + unit];
        }
      }
    };
    MelPrefetch<NBV, NI> mp;
    mp.fetch(p, 0);
    fetch_cond(0);

    for (int t = 0; t < p.L; ++t) {
      // ---- idle phase: everything not on the sample chain --------------------------
      float gc[3], qc[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) gc[q] = gn[q], qc[q] = qn[q];
      mp.store(sh);
      if (t + 1 < p.L) {
        mp.fetch(p, t + 1);
        fetch_cond(t + 1);
      }
      if constexpr (WL)  // W_hh1 h1_{t-1}
        matvec_lds<8, 64, LANES>(sh.wl, sh.vec, kp * 32, kl, sh.part[0][s], act, p.B);
      else
        matvec<8, 64>(w1, sh.vec, kp * 32, kl, sh.part[0][s], act, p.B);
      __syncthreads();
      WR_STAMP(0);
      if (t > 0) acquire_vec(p, sh, 1, t - 1, false);  // h2_{t-1}
      __syncthreads();
      WR_STAMP(1);
      if (sh.abort_flag) return;
      if constexpr (WL)  // W_hh2 h2_{t-1}
        matvec_lds<8, 64, LANES>(sh.wl + 8 * LANES * 4, sh.vec, kp * 32, kl, sh.part[1][s], act, p.B);
      else
        matvec<8, 64>(w2, sh.vec, kp * 32, kl, sh.part[1][s], act, p.B);
      matvec_mel(wmr, sh.melv, kl, sh.partm[s], act, p.B);
      // ---- the chain: s_{t-1} -------------------------------------------------------
      __syncthreads();
      WR_STAMP(2);
      if (t > 0) acquire_sample(p, sh, t - 1, !p.xin && local == 0);  // teacher-forced: pace only
      if (p.xin && tid < p.B) sh.sval[tid] = p.xin[(size_t)(p.fold0 + tid) * p.L + t];
      __syncthreads();
      WR_STAMP(3);
      if (sh.abort_flag) return;
      float sv = 0.f;
      if (cell) {
        sv = sh.sval[cb];
        float gi[3], gh[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int rw = q * UG + cu;
          gh[q] = sh.part[0][2 * rw][cb] + sh.part[0][2 * rw + 1][cb];
          gi[q] = (gc[q] + sh.partm[rw][cb]) + uu1[q] * sv;
        }
        const float rg = sigm(gi[0] + (gh[0] + bh1[0]));
        const float zg = sigm(gi[1] + (gh[1] + bh1[1]));
        const float ng = tanhf(gi[2] + rg * (gh[2] + bh1[2]));
        h1 = tagged(ng + zg * (h1 - ng), t);
        publish(p, 0, t, cb, unit, h1);
      }
      acquire_vec(p, sh, 0, t, false);  // h1_t
      __syncthreads();
      WR_STAMP(4);
      if (sh.abort_flag) return;
      matvec<8, 64>(w3, sh.vec, kp * 32, kl, sh.part[2][s], act, p.B);  // W_ih2a h1_t
      __syncthreads();
      WR_STAMP(5);
      if (cell) {
        float gi[3], gh[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int rw = q * UG + cu;
          gh[q] = sh.part[1][2 * rw][cb] + sh.part[1][2 * rw + 1][cb];
          const float gx = sh.part[2][2 * rw][cb] + sh.part[2][2 * rw + 1][cb];
          gi[q] = ((qc[q] + sh.partm[3 * UG + rw][cb]) + uu2[q] * sv) + gx;
        }
        const float rg = sigm(gi[0] + (gh[0] + bh2[0]));
        const float zg = sigm(gi[1] + (gh[1] + bh2[1]));
        const float ng = tanhf(gi[2] + rg * (gh[2] + bh2[2]));
        h2 = tagged(ng + zg * (h2 - ng), t);
        publish(p, 1, t, cb, unit, h2);
      }
      WR_STAMP(6);
      // sh.vec keeps h1_t: the next step's W_hh1 product reads it
    }
    if (!p.xin && local == 0) {  // the last sample
      __syncthreads();
      acquire_sample(p, sh, p.L - 1, true);
    }
  } else {
    // ================================= FC workgroup =====================================
    // fc1: every FC workgroup, FR rows.  fc2 / fc3 on disjoint halves of the FC workgroups
    // (2 FR rows each): an edge's price grows with its consumers, so y1 is read by half
    // of them (the fc2 half) and y2 by the other half (fc3), not by all.
    constexpr int HF = G::NF / 2, FR2 = 2 * FR;
    const int f = local - NG;
    const bool fc2role = f < HF;
    const int r0 = f * FR;
    const int r = s >> 3, kp = s & 7;      // fc1: FR rows x 8 k-parts (2 chunks per lane)
    const int r2 = s >> 2, kp2 = s & 3;    // fc2 / fc3: FR2 rows x 4 k-parts (4 chunks)
    const int q0 = (fc2role ? f : f - HF) * FR2;  // first fc2 (fc3) row of this workgroup
    float wf1[8], wf23[16], wmr[10];
    const bool act23 = fc2role || q0 + r2 < p.NC;
    {
      const float *a1 = p.w_fc1a + (size_t)(r0 + r) * WR_R + kp * 32 + kl * 4;  // k = 256 j + ..
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 x1 = *(const f32x4 *)(a1 + j * 256);
#pragma unroll
        for (int e = 0; e < 4; ++e) wf1[4 * j + e] = x1[e];
      }
      const float *a2 = fc2role ? p.w_fc2a + (size_t)(q0 + r2) * WR_F
                                : p.w_fc3 + (size_t)(act23 ? q0 + r2 : 0) * WR_F;
      a2 += kp2 * 32 + kl * 4;  // k = 128 j + 32 kp2 + 4 kl + e
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 x2 = *(const f32x4 *)(a2 + j * 128);
#pragma unroll
        for (int e = 0; e < 4; ++e) wf23[4 * j + e] = x2[e];
      }
    }
    const bool actm = s < FR;
    {
      const float *am = p.wm + (size_t)(6 * WR_R + r0 + (actm ? s : 0)) * WR_NM + kl;
#pragma unroll
      for (int j = 0; j < 10; ++j) wmr[j] = am[8 * j];
    }
    // cell threads: fc1 (row cr, fold cb); fc2 (row cr2, fold cb2)
    const bool cell = tid < FR * p.B;
    const int cr = tid % FR, cb = tid / FR;
    const bool cell2 = fc2role && tid < FR2 * p.B;
    const int cr2 = tid % FR2, cb2 = tid / FR2;
    const float vv1 = p.v1[r0 + cr];
    float rn = 0.f, sn = 0.f;
    auto fetch_cond = [&](int t) {
      if (cell) {
        const Pos ps = position(p, cb, t);
        rn = p.cond[(size_t)ps.cond_row * WR_COND + 6 * WR_R + r0 + cr];
      }
      if (cell2) {
        const Pos ps = position(p, cb2, t);
        sn = p.cond[(size_t)ps.cond_row * WR_COND + 6 * WR_R + WR_F + q0 + cr2];
      }
    };
    MelPrefetch<NBV, NI> mp;
    mp.fetch(p, 0);
    fetch_cond(0);

    for (int t = 0; t < p.L; ++t) {
      const float rc = rn, sc = sn;
      mp.store(sh);
      if (t + 1 < p.L) {
        mp.fetch(p, t + 1);
        fetch_cond(t + 1);
      }
      __syncthreads();
      matvec_mel(wmr, sh.melv, kl, sh.partm[s], actm, p.B);
      WR_STAMP(0);
      // ---- s_{t-1} -------------------------------------------------------------------
      if (t > 0) acquire_sample(p, sh, t - 1, false);
      WR_STAMP(1);
      if (p.xin && tid < p.B) sh.sval[tid] = p.xin[(size_t)(p.fold0 + tid) * p.L + t];
      // ---- h1_t + h2_t ----------------------------------------------------------------
      acquire_vec(p, sh, 0, t, false);
      __syncthreads();
      if (sh.abort_flag) return;
      WR_STAMP(2);
      acquire_vec(p, sh, 1, t, true);
      __syncthreads();
      if (sh.abort_flag) return;
      WR_STAMP(3);
      matvec<2, 256>(wf1, sh.vec, kp * 32, kl, sh.part[0][s], true, p.B);
      __syncthreads();
      WR_STAMP(4);
      if (cell) {
        float acc = sh.part[0][cr * 8][cb];
#pragma unroll
        for (int i = 1; i < 8; ++i) acc += sh.part[0][cr * 8 + i][cb];
        const float pre = ((rc + sh.partm[cr][cb]) + vv1 * sh.sval[cb]) + acc;
        publish(p, 2, t, cb, r0 + cr, tagged(fmaxf(pre, 0.f), t));
      }
      if (fc2role) {
        acquire_vec(p, sh, 2, t, false);  // y1
        __syncthreads();
        if (sh.abort_flag) return;
        WR_STAMP(5);
        matvec<4, 128>(wf23, sh.vec, kp2 * 32, kl, sh.part[1][s], true, p.B);
        __syncthreads();
        WR_STAMP(6);
        if (cell2) {
          float acc = sh.part[1][cr2 * 4][cb2];
#pragma unroll
          for (int i = 1; i < 4; ++i) acc += sh.part[1][cr2 * 4 + i][cb2];
          publish(p, 3, t, cb2, q0 + cr2, tagged(fmaxf(sc + acc, 0.f), t));
        }
      } else {
        acquire_vec(p, sh, 3, t, false);  // y2
        __syncthreads();
        if (sh.abort_flag) return;
        WR_STAMP(7);
        matvec<4, 128>(wf23, sh.vec, kp2 * 32, kl, sh.part[2][s], act23, p.B);
        __syncthreads();
        WR_STAMP(8);
        // ---- fc3 rows of this workgroup: logits and Gumbel scores (one thread per
        // (row, fold): the Philox rounds and logs in parallel), then the draw's partial(s)
        if (tid < FR2 * p.B) {
          const int rr = tid % FR2, b = tid / FR2, k = q0 + rr;
          float z = -INFINITY;
          if (k < p.NC) {
            float l = sh.part[2][rr * 4][b];
#pragma unroll
            for (int i = 1; i < 4; ++i) l += sh.part[2][rr * 4 + i][b];
            l = l + p.b_fc3[k];
            if (p.logits) p.logits[((size_t)(p.fold0 + b) * p.L + t) * p.NC + k] = l;
            if (p.mol) {
              publish_z(p, t, b, k, l, k);  // MOL: every logit is a granule of its own
            } else {
              const u32x4 w = philox((u32x4){(unsigned)t, (unsigned)(p.fold0 + b), (unsigned)(k >> 2), 0u},
                                     p.k0, p.k1);
              z = l - logf(-logf(u01(pword(w, k & 3))));
            }
          }
          sh.partm[rr][b] = z;  // the mel partials of this step are consumed
        }
        __syncthreads();
        if (!p.mol && tid < p.B) {  // RAW: the best (score, class) of these rows
          float best = sh.partm[0][tid];
          int bidx = q0;
#pragma unroll
          for (int rr = 1; rr < FR2; ++rr)
            if (sh.partm[rr][tid] > best) best = sh.partm[rr][tid], bidx = q0 + rr;
          publish_z(p, t, tid, f - HF, best, bidx);
        }
        WR_STAMP(9);
      }
    }
  }
  if (stamping) {
    unsigned long long *dst = (unsigned long long *)(p.ws + WS_STAMPS) + (blockIdx.x == 0 ? 0 : 16);
    for (int i = 0; i < 11; ++i) dst[i] = sh.stamp[i];
  }
#undef WR_STAMP
}

__global__ void wr_stretch_conv_kernel(const float *x, int64_t xs_b, int W, int C, int s,
                                       const float *w, float *y, int64_t ys_b, int Wout, int crop0,
                                       int B) {
  const int64_t n = (int64_t)B * Wout * C;
  const int taps = 2 * s + 1;
  const int64_t Ws = (int64_t)W * s;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int64_t jb = i / C;
    const int j = (int)(jb % Wout), b = (int)(jb / Wout);
    const float *xb = x + b * xs_b;
    float acc = 0.f;
    for (int k = 0; k < taps; ++k) {
      const int64_t q = (int64_t)j + crop0 + k - s;
      const float v = (q >= 0 && q < Ws) ? xb[(q / s) * C + c] : 0.f;
      acc = fmaf(w[k], v, acc);
    }
    y[b * ys_b + (int64_t)j * C + c] = acc;
  }
}

// numpy.linspace(start, stop, num)[i] (float64: i * step + start, last = stop)
__device__ __forceinline__ double np_linspace(double start, double stop, int num, int i) {
  if (num > 1 && i == num - 1) return stop;
  if (num <= 1) return start;
  const double step = (stop - start) / (double)(num - 1);
  return (double)i * step + start;
}

__device__ __forceinline__ double mu_decode(double y, int mu_law, int n_classes) {
  if (!mu_law) return y;
  // DSP.decode_mu_law(y, n_classes, from_labels=False): sign(y)/mu * ((1+mu)^|y| - 1),
  // mu = n_classes - 1; (1+mu) = 2^bits: (1+mu)^|y| = 2^(bits |y|), bits |y| exact
  const double mu = (double)(n_classes - 1);
  const double sg = y > 0.0 ? 1.0 : (y < 0.0 ? -1.0 : 0.0);
  const double bits = log2((double)n_classes);
  return sg / mu * (exp2(bits * fabs(y)) - 1.0);
}

__global__ void wr_unfold_kernel(const float *smp, int B, int L, int target, int overlap,
                                 int batched, int mu_law, int n_classes, int wave_len, int nf,
                                 double *out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= wave_len) return;
  double v;
  if (batched) {
    const int stride = target + overlap;
    const int silence = overlap / 2, fade_len = overlap - silence;
    auto term = [&](int i) -> double {
      const int pos = j - i * stride;
      double y = mu_decode((double)smp[(size_t)i * L + pos], mu_law, n_classes);
      if (pos < overlap) {  // fade_in = [zeros(silence), sqrt(0.5 (1 + t))]
        const double g = pos < silence ? 0.0
                                       : sqrt(0.5 * (1.0 + np_linspace(-1.0, 1.0, fade_len, pos - silence)));
        y = y * g;
      }
      if (pos >= L - overlap) {  // fade_out = [ones(silence), sqrt(0.5 (1 - t))]
        const int q = pos - (L - overlap);
        const double g = q < silence ? 1.0 : sqrt(0.5 * (1.0 - np_linspace(-1.0, 1.0, fade_len, q - silence)));
        y = y * g;
      }
      return y;
    };
    const int ihi = j / stride;
    v = 0.0;
    if (ihi >= 1 && ihi - 1 < B && j - (ihi - 1) * stride < L) v = v + term(ihi - 1);
    if (ihi < B) v = v + term(ihi);
  } else {
    v = mu_decode((double)smp[j], mu_law, n_classes);
  }
  if (nf > 0 && j >= wave_len - nf) v = v * np_linspace(1.0, 0.0, nf, j - (wave_len - nf));
  out[j] = v;
}

unsigned g_wr_spin = SPIN_DEFAULT;

int cu_count() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return cus;
}

}  // namespace

constexpr int WR_NI_MAX = 2;  // instances per launch

extern "C" int64_t ftmi_wavernn_workspace_bytes(void) {
  return (int64_t)(WS_CTRL + WR_NI_MAX * (4 * XS_VEC + XS_Z)) * 4;
}

extern "C" uint32_t ftmi_set_wavernn_spin_limit(uint32_t limit) {
  const uint32_t old = g_wr_spin;
  g_wr_spin = limit ? limit : SPIN_DEFAULT;
  return old;
}

extern "C" int ftmi_wavernn(const ftmi_wavernn_args *a, ftmi_stream_t stream) {
  if (!a) return FTMI_E_ARG;
  if (!a->w_hh1 || !a->w_hh2 || !a->w_ih2a || !a->w_fc1a || !a->w_fc2a || !a->w_fc3 ||
      !a->b_fc3 || !a->b_hh1 || !a->b_hh2 || !a->u1 || !a->u2 || !a->v1 || !a->wm || !a->cond ||
      !a->mel || !a->workspace)
    return FTMI_E_ARG;
  if (a->B <= 0 || a->L <= 0 || a->hop <= 0 || a->item_rows <= 0 || a->frames_per_item <= 0)
    return FTMI_E_ARG;
  if (a->rnn_dims != WR_R || a->fc_dims != WR_F || a->feat_dims != WR_NM || a->aux_dims != WR_NA)
    return FTMI_E_UNSUPPORTED;
  // RAW: 2^bits <= 512 classes (the fc3 rows of the FC workgroups' fc3 half)
  if (a->mol ? a->n_classes != 30
             : (a->n_classes < 2 || a->n_classes > WR_F || (a->n_classes & (a->n_classes - 1)) != 0))
    return FTMI_E_UNSUPPORTED;
  if (a->xin ? !a->logits : !a->samples) return FTMI_E_ARG;
  if (a->batched && a->fold_stride <= 0) return FTMI_E_ARG;
  if (!ftmi_aligned16(a->mel) || !ftmi_aligned16(a->workspace)) return FTMI_E_ALIGN;
  if (cu_count() < WR_GRID) return FTMI_E_UNSUPPORTED;
  hipStream_t s = ftmi_hs(stream);
  WrParams p{};
  p.w_hh1 = a->w_hh1, p.w_hh2 = a->w_hh2, p.w_ih2a = a->w_ih2a;
  p.w_fc1a = a->w_fc1a, p.w_fc2a = a->w_fc2a, p.w_fc3 = a->w_fc3, p.b_fc3 = a->b_fc3;
  p.b_hh1 = a->b_hh1, p.b_hh2 = a->b_hh2, p.u1 = a->u1, p.u2 = a->u2, p.v1 = a->v1;
  p.wm = a->wm, p.cond = a->cond, p.mel = a->mel;
  p.bias_row = a->bias_row, p.item_rows = a->item_rows, p.frames_per_item = a->frames_per_item;
  p.hop = a->hop, p.fold_stride = a->fold_stride, p.batched = a->batched;
  p.xin = a->xin, p.samples = a->samples, p.logits = a->logits;
  unsigned *ws = (unsigned *)a->workspace;
  p.ws = ws;
  p.xch = (float *)(ws + WS_CTRL);
  p.status = a->status;
  p.L = a->L, p.NC = a->n_classes, p.mol = a->mol;
  p.k0 = (unsigned)(a->seed & 0xFFFFFFFFull), p.k1 = (unsigned)(a->seed >> 32);
  p.spin_limit = g_wr_spin;
  static const int stamps_env = [] {
    const char *v = getenv("FTMI_WR_STAMPS");
    return v ? atoi(v) : 0;
  }();
  p.stamps = stamps_env;
  // two instances (each the whole pipeline on 128 workgroups, half the folds) whenever
  // there are two folds to share: the per-step hand-off latency is paid once for both
  const int per_launch = WR_NBMAX;  // NI = 2: 2 x 16 (the LDS holds the GRU weights)
  for (int f0 = 0; f0 < a->B; f0 += p.B) {
    p.fold0 = f0;
    p.B = a->B - f0 < per_launch ? a->B - f0 : per_launch;
    // two instances from two folds on (c2-size mel, 19 folds: 23.95 against 31.8 us/step
    // with one); FTMI_WR_NI=1 forces one instance (A/B runs)
    static const int ni_env = [] {
      const char *v = getenv("FTMI_WR_NI");
      return v ? atoi(v) : 2;
    }();
    const int ni = (p.B >= 2 && ni_env != 1) ? 2 : 1;
    const int bi = (p.B + ni - 1) / ni;
    hipError_t e = hipMemsetAsync(a->workspace, 0, (size_t)ftmi_wavernn_workspace_bytes(), s);
    if (e != hipSuccess) return (int)e;
#define FTMI_WR_LAUNCH(NBV_, NI_)                                                            \
  do {                                                                                       \
    if (int rc = ftmi_resident_ok((const void *)wavernn_kernel<NBV_, NI_>, WR_GRID, WR_NT * NI_, 0)) \
      return rc;                                                                             \
    hipLaunchKernelGGL((wavernn_kernel<NBV_, NI_>), dim3(WR_GRID), dim3(WR_NT * NI_), 0, s, p); \
  } while (0)
    if (ni == 1) {
      p.B = p.B < WR_NBMAX ? p.B : WR_NBMAX;  // one instance: <= 32 folds per launch
      if (p.B <= 8) FTMI_WR_LAUNCH(8, 1);
      else if (p.B <= 16) FTMI_WR_LAUNCH(16, 1);
      else FTMI_WR_LAUNCH(32, 1);
    } else {
      if (bi <= 8) FTMI_WR_LAUNCH(8, 2);
      else FTMI_WR_LAUNCH(16, 2);
    }
#undef FTMI_WR_LAUNCH
    FTMI_CHECK_LAUNCH();
  }
  return FTMI_OK;
}

extern "C" int ftmi_wr_stretch_conv(const float *x, int64_t x_batch_stride, int32_t B, int32_t W,
                                    int32_t C, int32_t scale, const float *w, float *y,
                                    int64_t y_batch_stride, int32_t W_out, int32_t crop0,
                                    ftmi_stream_t stream) {
  if (!x || !w || !y) return FTMI_E_ARG;
  if (B <= 0 || W <= 0 || C <= 0 || scale <= 0 || W_out <= 0 || crop0 < 0) return FTMI_E_ARG;
  if ((int64_t)crop0 + W_out > (int64_t)W * scale) return FTMI_E_SHAPE;
  const int64_t n = (int64_t)B * W_out * C;
  const int blocks = (int)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(wr_stretch_conv_kernel, dim3(blocks), dim3(256), 0, ftmi_hs(stream), x,
                     x_batch_stride, W, C, scale, w, y, y_batch_stride, W_out, crop0, B);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

extern "C" int ftmi_wr_unfold(const float *samples, int32_t B, int32_t L, int32_t target,
                              int32_t overlap, int32_t batched, int32_t mu_law, int32_t n_classes,
                              int32_t wave_len, int32_t fade_len, double *out,
                              ftmi_stream_t stream) {
  if (!samples || !out) return FTMI_E_ARG;
  if (B <= 0 || L <= 0 || wave_len <= 0 || fade_len < 0 || n_classes < 2) return FTMI_E_ARG;
  if (mu_law && (n_classes & (n_classes - 1)) != 0) return FTMI_E_UNSUPPORTED;
  if (batched && (target < 0 || overlap < 0 || L != target + 2 * overlap)) return FTMI_E_SHAPE;
  if (wave_len < fade_len) return FTMI_E_SHAPE;  // the reference's fade-out needs 20 hops
  if (batched ? (int64_t)wave_len > (int64_t)B * (target + overlap) + overlap : wave_len > L)
    return FTMI_E_SHAPE;
  hipLaunchKernelGGL(wr_unfold_kernel, dim3((wave_len + 255) / 256), dim3(256), 0, ftmi_hs(stream),
                     samples, B, L, target, overlap, batched, mu_law, n_classes, wave_len, fade_len, out);
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}
