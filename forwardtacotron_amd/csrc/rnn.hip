// Persistent bidirectional GRU / LSTM recurrence (gfx950).
//
// Reference semantics: PyTorch nn.GRU / nn.LSTM, one layer, bidirectional, batch_first,
// h0 = c0 = 0, both directions over the full padded length (no packing) — used by
//   CBHG.rnn                 models/common_layers.py:84,118   (GRU, H = 256)
//   SeriesPredictor.rnn      models/forward_tacotron.py:39,53 (GRU, H = 64 / 128)
//   ForwardTacotron.lstm     models/forward_tacotron.py:165-168,321 (LSTM, H = 512)
// The input projections x W_ih^T + b are computed beforehand by the GEMM kernel; this
// kernel only runs the sequential part  gates_t = xp_t + W_hh h_{t-1}  + cell update.
//
// Decomposition.  The batch is cut into chunks of NB = 16 sequences; a GROUP is one
// (direction, chunk) pair and owns an independent recurrence.  A group is spread over
// BPG = H / U workgroups, each owning U hidden units (all G gates: R = G*U rows of W_hh)
// whose W_hh slice stays in VGPRs for the whole sequence.  The 4 waves of a workgroup are
// WK (K-split) x WR (row-split); per step each wave computes its rows' partial gate sums over
// its K range with MFMA, the WK partials are summed through LDS, and 256 threads apply the
// cell update to the U x 16 (unit, sequence) cells they own (c / h state in registers).
//
// Matrix path (MODE):
//   2 (FTMI_MMA_F16X3, default): W = W_h + 2^-11 W_t (f16 head + scaled f16 tail, kept in
//     VGPRs: 4 B per weight) and h = h_h + 2^-11 h_t; three v_mfma_f32_16x16x32_f16 per
//     tile accumulate  W_t h_h + W_h h_t + W_h (2^11 h_h) = 2^11 W h  (dropped term
//     < 2^-22 relative), scaled back by 2^-11 (exact) before the K-split reduction.  h is a
//     tanh / sigmoid*tanh output, |h| < 1, so 2^11 h_h never leaves the f16 range; a W_hh
//     entry beyond the f16 range sets bit 1 of *status (the caller then reruns on mode 1).
//   1 (FTMI_MMA_BF16X6): W and h split into three bf16 pieces each, the six cross products
//     with i + j <= 4 on v_mfma_f32_16x16x32_bf16 — fp32-accurate (see gemm.hip).
//   0 (FTMI_MMA_F32): v_mfma_f32_16x16x4_f32.
//
// h hand-off between the BPG workgroups of a group: the data is the flag.  Each exchanged
// h value carries a step tag in its mantissa LSB (h_tag: a <= 1 ulp change; the tagged value
// is used everywhere: state, exchange and layer output).  A fifth "comm" wave per workgroup
// writes the workgroup's new h slice (one 16-B store per lane) into an exchange buffer
// hx[t & 1][group][16*H] kept in MFMA-fragment order; consumer waves sc1-load their K range
// of it (1 KB of consecutive bytes per wave-instruction) and re-load until every value
// carries the tag of the step they need.  4-byte accesses are single-copy atomic, so torn
// 16-byte stores only delay a read; no flag, counter, drain or barrier is on the path
// (MI355X_MICROARCH.md "Valid forms", R2).  Parity double buffering is race-free because a
// workgroup can only produce h_{t+1} after it read every workgroup's h_t.  The compute waves
// never store to global memory, so their loads (input-projection prefetch, h) are never held
// behind a store in the in-order vmcnt.  Two store modes, chosen per launch:
//   XCD-local: a start-of-launch census reads each workgroup's XCC_ID (s_getreg) and, when
//     every XCD received exactly the workgroups of whole groups, forms the groups from
//     co-located workgroups; h is then stored with PLAIN stores (kept in that XCD's L2) and
//     read by sc1 loads served from the same L2.  Correct by construction because group
//     membership comes from the measured XCD, never from an assumed dispatch order.
//   global (fallback when the census is unbalanced, or disabled): sc1 write-through
//     stores, groups by blockIdx.
// BPG == 1 groups never leave the workgroup: h goes through LDS.  Every spin is bounded;
// on timeout the call's error word is set and the workgroup leaves the time loop.
//
// Packed sequences (forward(), models/forward_tacotron.py:224-230): with lengths != NULL
// frames t >= lengths[b] output pad_value, and the reverse direction keeps h = c = 0
// until t = lengths[b]-1, exactly like pack_padded_sequence + pad_packed_sequence.
#include "common.h"

// ---- diagnostic build only (-DFTMI_RNN_STAMPS): per-phase s_memtime sums per workgroup
#ifdef FTMI_RNN_STAMPS
__device__ unsigned long long ftmi_rnn_stamps[2048 * 8];
#define STAMP(i)                                                                      \
  do {                                                                                \
    if (threadIdx.x == 0) {                                                           \
      __builtin_amdgcn_sched_barrier(0);                                              \
      unsigned long long now__;                                                       \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" \
                   : "=s"(now__)::"memory");                                         \
      __builtin_amdgcn_sched_barrier(0);                                              \
      st_acc[i] += now__ - st_last;                                                   \
      st_last = now__;                                                                \
    }                                                                                 \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif
// timing experiments (FTMI_RNN_DIAG, results invalid when set): diagnostic build only
#ifdef FTMI_DIAG
#define RNN_DIAG(p) ((p).diag)
#else
#define RNN_DIAG(p) ((void)(p), 0u)
#endif

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr float H3_SCALE = 2048.f;      // 2^11: tail scale of the f16 split
constexpr float H3_UNSCALE = 1.f / 2048.f;

constexpr int NB = 16;              // sequences per group (MFMA 16x16 columns)
constexpr int RED_STRIDE = NB + 1;  // LDS partial-sum row stride (floats)
// Default bound of every spin (census barrier, h hand-off); ftmi_set_rnn_spin_limit changes
// it (tests force the timeout path with a tiny limit).
constexpr unsigned SPIN_LIMIT_DEFAULT = 1u << 22;
unsigned g_spin_limit = SPIN_LIMIT_DEFAULT;
// status-word bit set when a workgroup gave up waiting (include/ftmi.h FTMI_STATUS_RNN_TIMEOUT)
constexpr unsigned STATUS_TIMEOUT = 4u;
constexpr int CNT_PAD = 32;  // one 128-B line per counter
// workspace word offsets (in 32-bit words) of the control block
constexpr int WS_ERR = 0;
constexpr int WS_CENSUS = 1 * CNT_PAD;   // 8 per-XCD slot counters, one line each
constexpr int WS_ARRIVE = 9 * CNT_PAD;   // census barrier
constexpr int WS_FLAGS = 10 * CNT_PAD;   // XCD-local mode: 64 flag words per group
constexpr int FLAGS_PER_GROUP = 64;
constexpr int WS_GROUPS_OF(int ngroups) { return WS_FLAGS + ngroups * FLAGS_PER_GROUP; }

struct RnnParams {
  const float *xp;
  int64_t xp_stride;
  int T_src;
  const int32_t *index;
  const float *xp_zero;
  const float *w_hh;
  const float *b_hh;
  float *y;
  int64_t y_stride;
  const int32_t *lengths;
  float pad_value;
  float *hx;  // [2][ngroups_total][16*H]
  int B, T;
  int ngroups_total;
  int chunk0;     // first batch chunk of this launch
  int ngroups;    // groups in this launch
  int xcd_local;  // 1: try the census-based XCD-local mode
  unsigned *ws;   // control words (see WS_*)
  unsigned *status;  // optional: bit 1 = a W_hh entry overflowed f16 (mode 2)
  unsigned spin_limit;  // bound of every spin (g_spin_limit at launch)
  int psleep;  // s_sleep(1) count before a step's first h poll (FTMI_RNN_PSLEEP; valid results)
  int diag;  // timing experiments only (FTMI_RNN_DIAG, diagnostic build only; 32 = one MFMA
             // per product, 64 = a quarter of the h loads, 128 = cell without
             // transcendentals — rnn_bidir_kernel f16x3): bit 0 =
             // input projections from one L2-hot row, bit 1 = no hand-off waits,
             // bit 2 = no drain
};

// workspace: [control: err, census, flags, counters][hx: 2 * 2*nchunks * 16*H floats], sized
// for chunks of 8 sequences: the most groups any kernel form runs (a spread GRU on
// rnn_bidir_kernel: 8 live sequences per group in the same 16-column slab format)
constexpr int WS_CHUNK = 8;
static int64_t ws_chunks(int64_t B) { return (B + WS_CHUNK - 1) / WS_CHUNK; }
static int64_t ctl_bytes(int64_t nchunks) {
  return (WS_GROUPS_OF((int)(2 * nchunks)) + 2 * nchunks * CNT_PAD) * (int64_t)sizeof(unsigned);
}

// host-side guard before a launch: the exchange words a kernel form indexes (2 parities x
// ngroups_total slabs of slab_words) fit the exchange region of the workspace for (B, H)
static bool hx_fits(const RnnParams &p, int H, int64_t slab_words) {
  return 2 * (int64_t)p.ngroups_total * slab_words <= 2 * (2 * ws_chunks(p.B)) * NB * (int64_t)H;
}

__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float fast_tanh(float x) { return 2.0f * fast_sigmoid(2.0f * x) - 1.0f; }

__device__ __forceinline__ void split3x8(const float (&v)[8], bf16x8 &h1, bf16x8 &h2, bf16x8 &h3) {
  typedef float f32x8 __attribute__((ext_vector_type(8)));
  f32x8 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = v[i];
  h1 = __builtin_convertvector(x, bf16x8);
  const f32x8 r1 = x - __builtin_convertvector(h1, f32x8);
  h2 = __builtin_convertvector(r1, bf16x8);
  const f32x8 r2 = r1 - __builtin_convertvector(h2, f32x8);
  h3 = __builtin_convertvector(r2, bf16x8);
}

// x = h + 2^-11 t (f16 head, scaled f16 tail); s = 2^11 h (exact for |x| < 32)
__device__ __forceinline__ void split2h8(const float (&v)[8], f16x8 &h, f16x8 &t) {
  typedef float f32x8 __attribute__((ext_vector_type(8)));
  f32x8 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = v[i];
  h = __builtin_convertvector(x, f16x8);
  t = __builtin_convertvector((x - __builtin_convertvector(h, f32x8)) * H3_SCALE, f16x8);
}

// Step tag carried in the mantissa LSB of every exchanged h value.  Buffer half t & 1 holds
// h_t over h_{t-2} (or the zeroed workspace before step 2): the tags of t and t - 2 differ,
// and step 0/1's tag (1) differs from the zero fill.
__device__ __forceinline__ unsigned h_tag(int t) { return (((unsigned)t >> 1) & 1u) ^ 1u; }

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

// bounded relaxed poll (one lane): returns false on timeout
__device__ __forceinline__ bool poll_ge(unsigned *w, unsigned target, unsigned limit) {
  unsigned spins = 0;
  while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > limit) return false;
  }
  return true;
}

// a workgroup gave up waiting: the call's output is invalid.  Recorded in the workspace
// error word and in the caller's status word (bit 2), which the model entry points read
// (ops.run_checked raises RnnTimeout) — never a silently wrong result.
__device__ __forceinline__ void report_timeout(const RnnParams &p) {
  __hip_atomic_store(p.ws + WS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (p.status) atomicOr(p.status, STATUS_TIMEOUT);
}

// NBL: live sequences per group (16, or 8 to spread a recurrence over twice the groups: every
// workgroup then acquires and stores half the h bytes per step; the MFMA columns past NBL are
// dead)
// U = 8 (the spread postnet GRU, H = 256, f16x3, CST): a group of 16 live sequences spreads
// over 32 workgroups of 8 units (24 W_hh rows in 2 row blocks, 8 dead): the same 256
// workgroups at B = 64 as 16 units with 8 live sequences (legacy_nbl), with two thirds of
// the MFMAs per wave and 128 cells per workgroup (waves 0-1 own them).  Measured at B = 64,
// T = 1368: 1.11-1.12 against 1.39 us/step (tools/rnn_diag.py, profiles/r5_rnn_diag.txt).
template <int CELL, int H, int U, int WK, int MODE, bool CST = false, int NBL = NB>
__global__ __launch_bounds__(H / U == 1 ? 256 : 320, 1) void rnn_bidir_kernel(
    const RnnParams p) {
  constexpr bool X6 = MODE != 0;  // 16x16x32 fragment layout (bf16x6 and f16x3)
  constexpr bool H3 = MODE == 2;
  constexpr int G = CELL ? 4 : 3;
  constexpr int R = G * U;
  constexpr int RB = (R + 15) / 16;  // the GRU at U = 8: 24 rows in 2 row blocks, 8 dead
  constexpr int WR = 4 / WK;
  constexpr int RBW = RB / WR;  // row blocks per wave
  constexpr int KW = H / WK;    // K range per wave
  constexpr int NL = KW / 16;   // float4s of h operand per lane
  constexpr int KS = KW / 32;   // bf16 k-steps per wave (X6)
  constexpr int KB = KW / 4;    // f32 k-blocks per wave (!X6)
  constexpr int BPG = H / U;
  constexpr bool LOCAL = BPG == 1;
  constexpr int CELLS = U * NB;
  constexpr bool HALFCELL = CELLS < 256;  // U = 8: threads 0..127 own the cells
  constexpr int CPT = HALFCELL ? 1 : CELLS / 256;
  static_assert((R % 16 == 0 || U == 8) && (U % 16 == 0 || U == 8) && H % U == 0 &&
                    RB % WR == 0 && (CELLS % 256 == 0 || CELLS == 128), "shape");
  static_assert(X6 ? (KW % 32 == 0) : (KB % 4 == 0), "K split");
  // CST: the compute waves store their own tagged h chunks right after the cell update (each
  // wave's 16 chunks are its own cells: CPT == 1), the comm wave only the y rows — barrier C
  // and the comm wave's stage read leave the h hand-off's critical path
  static_assert(!CST || (H3 && !LOCAL && CPT == 1 && (U == 16 || U == 8)), "compute-wave h stores");
  static_assert(U != 8 || (CST && CELL == 0 && NBL == NB), "U = 8: the spread GRU's CST form");
  static_assert(NBL == NB || (NBL == 8 && !LOCAL), "live sequences per group");
  constexpr int RR = RB * 16;                     // reduction rows (dead ones included)
  constexpr float GSC = H3 ? H3_UNSCALE : 1.f;     // scale of the reduced W_hh h sums

  __shared__ __attribute__((aligned(16))) float red[WK * RR * RED_STRIDE];
  __shared__ __attribute__((aligned(16))) float hloc[LOCAL ? 2 * 16 * H : 4];
  // multi-workgroup groups: the new h slice and y values of this workgroup, handed from the
  // compute waves to the comm wave (cell c = seq * U + unit; float4 f = 4 units)
  __shared__ __attribute__((aligned(16))) float hstage[LOCAL ? 4 : CELLS];
  __shared__ __attribute__((aligned(16))) float ystage[LOCAL ? 4 : CELLS];
  __shared__ int s_abort, s_group, s_bi, s_mode;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave % WK, wr = wave / WK;
  const int ls = lane >> 4, lc = lane & 15;

  // ---- group assignment (census for the XCD-local mode) ----------------------------
  if (tid == 0) {
    int mode = 0, group = blockIdx.x % p.ngroups, bi = blockIdx.x / p.ngroups, abort = 0;
    if (!LOCAL && p.xcd_local) {
      const unsigned x = xcc_id();
      const unsigned slot = __hip_atomic_fetch_add(p.ws + WS_CENSUS + x * CNT_PAD, 1u,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(p.ws + WS_ARRIVE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!poll_ge(p.ws + WS_ARRIVE, gridDim.x, p.spin_limit)) {
        abort = 1;
        report_timeout(p);
      } else if (p.ngroups % 8 == 0 || (int)gridDim.x == 8 * BPG) {
        // ngroups a multiple of 8: ngroups / 8 groups per XCD.  Fewer groups (small
        // batches): the grid is padded to one group's worth of workgroups per XCD, XCD x
        // hosts group x and the XCDs past the last group retire their workgroups.
        const int gpx = p.ngroups % 8 == 0 ? p.ngroups / 8 : 1;
        const unsigned per = (unsigned)gpx * BPG;
        bool balanced = true;
        for (int i = 0; i < 8; ++i)
          balanced &= __hip_atomic_load(p.ws + WS_CENSUS + i * CNT_PAD, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) == per;
        if (balanced) {
          mode = 1;
          group = (int)(x * gpx + slot / BPG);
          bi = (int)(slot % BPG);
        }
      }
    }
    s_mode = mode;
    s_group = group;
    s_bi = bi;
    s_abort = abort;
  }
  __syncthreads();
  if (s_abort) return;
  // padded grid: the surplus workgroups (census: XCDs past the last group; fallback order:
  // bi >= BPG) leave after the census barrier
  if (s_group >= p.ngroups || s_bi >= BPG) return;
  const int group = s_group, bi = s_bi;
  const bool xcd_mode = s_mode == 1;
  const int dir = group & 1;
  const int chunk = p.chunk0 + (group >> 1);
  const int gglob = p.chunk0 * 2 + group;
  const int u0 = bi * U;
  unsigned *cnt = p.ws + WS_GROUPS_OF(p.ngroups_total) + gglob * CNT_PAD;
  unsigned *flags = p.ws + WS_FLAGS + gglob * FLAGS_PER_GROUP;
  static_assert(BPG <= FLAGS_PER_GROUP, "flags");

  // ---- comm wave (wave 4, multi-workgroup groups only) ---------------------------------
  // Owns every global store of the step, so the compute waves issue only loads (vmcnt
  // counts loads and stores together, in issue order: a store would hold back the loads
  // issued after it).  Per step: (compute: h acquire, MFMA) barrier B -> (compute: cells ->
  // LDS stage) barrier C -> store this workgroup's tagged h slice (one float4 per lane per
  // 256 cells) and the y rows.  No flag, counter or drain: readiness travels IN the data
  // (MI355X_MICROARCH.md "Valid forms", R2: the data is the flag).
  if constexpr (!LOCAL) {
    if (wave == 4) {
      constexpr int F4 = CELLS / 4;  // float4s of the slice
      constexpr int FPL = F4 < 64 ? 1 : F4 / 64;   // per lane (U = 8: lanes 0..31)
      static_assert(F4 % 64 == 0 || F4 == 32, "comm wave tiling");
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.hx, (short)0, 0x7FFFFFF0, 0x00020000);
      const int hxp = p.ngroups_total * 16 * H * 4;  // bytes between the parity halves
      unsigned hofs[FPL];
      int yb[FPL], k0s[FPL];
      bool ok[FPL];
#pragma unroll
      for (int i = 0; i < FPL; ++i) {
        const int f = lane + 64 * i;
        {  // y: float4 f = 4 units of one sequence
          const int bl = f / (U / 4);
          yb[i] = chunk * NBL + bl;
          k0s[i] = u0 + (f % (U / 4)) * 4;
          ok[i] = f < F4 && bl < NBL && yb[i] < p.B;
        }
        if constexpr (H3) {  // h: 16-B chunk f = (seq, 8 units, plane) of f16 halves
          const int bl = f / (U / 4), rem = f % (U / 4), plane = rem & 1;
          const int k0 = u0 + (rem >> 1) * 8;
          const int kwv = k0 / KW, r = k0 % KW, q = r % 32;
          const int ln = (q >> 3) * 16 + bl;
          hofs[i] = (unsigned)((gglob * 16 * H * 2 +
                                ((kwv * NL + (r / 32) * 2 + plane) * 64 + ln) * 8) * 2);
        } else {  // h: float4 f = 4 units of one sequence, fp32
          const int bl = f / (U / 4);
          const int k0 = u0 + (f % (U / 4)) * 4;
          const int kwv = k0 / KW, r = k0 % KW;
          int ln, idx4;
          if constexpr (X6) {
            const int q = r % 32;
            ln = (q >> 3) * 16 + bl;
            idx4 = (r / 32) * 2 + ((q & 7) >> 2);
          } else {
            ln = (r / KB) * 16 + bl;
            idx4 = (r % KB) >> 2;
          }
          hofs[i] = (unsigned)((gglob * 16 * H + ((kwv * NL + idx4) * 64 + ln) * 4) * 4);
        }
      }
      __syncthreads();  // the compute waves' set-up barrier
      for (int t = 0; t < p.T; ++t) {
        const int tt = dir ? (p.T - 1 - t) : t;
        __syncthreads();  // B
        if (s_abort) break;
        __syncthreads();  // C: the stage holds the tagged h_t and y_t
        const int soff = (t & 1) * hxp;
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int i = 0; i < (CST ? 0 : FPL); ++i) {
          // every sequence slot of the chunk, the batch tail's too: consumers check the tags
          // of all 16 columns of their fragments
          const u32x4 v = *(const u32x4 *)&hstage[(lane + 64 * i) * 4];
          if (NBL != NB && (lane + 64 * i) / (U / 4) >= NBL) continue;  // dead sequence
          if (xcd_mode)  // stays in this XCD's L2, read back by same-XCD sc1 loads
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, hofs[i], soff, 0);
          else  // write-through (sc1)
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, hofs[i], soff, 16);
        }
#pragma unroll
        for (int i = 0; i < FPL; ++i) {
          const f32x4 v = *(const f32x4 *)&ystage[((lane + 64 * i) % F4) * 4];
          if (ok[i]) *(f32x4 *)(p.y + ((size_t)yb[i] * p.T + tt) * p.y_stride + dir * H + k0s[i]) = v;
        }
      }
      return;
    }
  }

  // ---- W_hh slice -> VGPR A-fragments (loaded once) ---------------------------------
  // row block rb = wr*RBW + i, lane row lc; X6: k = wk*KW + ks*32 + 8*ls + j (j < 8)
  //                                        f32: k = wk*KW + ls*KB + kb
  const float *wdir = p.w_hh + (size_t)dir * (G * H) * H;
  bf16x8 wa[(X6 && !H3) ? RBW : 1][(X6 && !H3) ? KS : 1][3];
  f16x8 wh[H3 ? RBW : 1][H3 ? KS : 1][2];  // [head, scaled tail]
  float wf[X6 ? 1 : RBW][X6 ? 1 : KB];
  bool wbad = false;
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    const int lrow0 = (wr * RBW + i) * 16 + lc;
    const bool rlive = lrow0 < R;  // a dead row (R % 16 != 0) multiplies zeros
    const int lrow = rlive ? lrow0 : 0;
    const int grow = (lrow / U) * H + u0 + (lrow % U);
    const float *src = wdir + (size_t)grow * H + wk * KW;
    if constexpr (X6) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float v[8];
        const f32x4 a = *(const f32x4 *)(src + ks * 32 + 8 * ls);
        const f32x4 b = *(const f32x4 *)(src + ks * 32 + 8 * ls + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        if (!rlive)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 0.f;
        if constexpr (H3) {
          split2h8(v, wh[i][ks][0], wh[i][ks][1]);
#pragma unroll
          for (int e = 0; e < 8; ++e) wbad |= !(__builtin_fabsf(v[e]) <= 65504.f);
        } else {
          split3x8(v, wa[i][ks][0], wa[i][ks][1], wa[i][ks][2]);
        }
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; kb += 4) {
        const f32x4 v = *(const f32x4 *)(src + ls * KB + kb);
        wf[i][kb] = v.x;
        wf[i][kb + 1] = v.y;
        wf[i][kb + 2] = v.z;
        wf[i][kb + 3] = v.w;
      }
    }
  }

  if (wbad && p.status) atomicOr(p.status, 2u);

  // ---- per-thread cells: cell c = tid + 256*j -> (unit u = c % U, seq b = c / U) ------
  int cu[CPT], cb[CPT], cbl[CPT], len[CPT], hxo[CPT];
  bool cvalid[CPT];
  float hstate[CPT], cstate[CPT], bhh[CPT][G];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = tid + 256 * j;
    cu[j] = c % U;
    const int bl = c / U;
    cbl[j] = bl;
    cb[j] = chunk * NBL + bl;
    cvalid[j] = bl < NBL && cb[j] < p.B;
    hstate[j] = 0.f;
    cstate[j] = 0.f;
    len[j] = (p.lengths && cvalid[j]) ? p.lengths[cb[j]] : p.T;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      bhh[j][g] = (CELL == 0) ? p.b_hh[dir * G * H + g * H + u0 + cu[j]] : 0.f;
    }
    // fragment-order position of (seq bl, unit k) in the group's 16*H slab
    const int k = u0 + cu[j];
    const int kwv = k / KW, r = k % KW;
    int ln, idx4, e;
    if constexpr (X6) {
      const int q = r % 32;
      ln = (q >> 3) * 16 + bl;
      idx4 = (r / 32) * 2 + ((q & 7) >> 2);
      e = q & 3;
    } else {
      ln = (r / KB) * 16 + bl;
      idx4 = (r % KB) >> 2;
      e = r & 3;
    }
    hxo[j] = ((kwv * NL + idx4) * 64 + ln) * 4 + e;
  }

  // ---- h operand source ----------------------------------------------------------------
  const int slab = 16 * H;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.hx, (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned hoff = (unsigned)((gglob * slab + wk * NL * 256 + lane * 4) * 4);
  const int hx_par = p.ngroups_total * slab * 4;  // bytes between the two parity halves
  unsigned cst_off = 0;  // CST: the exchange offset of stage chunk 16 wave + lane
  if constexpr (CST) {
    const int f = 16 * wave + (lane & 15);
    const int bl = f / (U / 4), rem = f % (U / 4), plane = rem & 1;
    const int k0 = u0 + (rem >> 1) * 8;
    const int kwv = k0 / KW, r = k0 % KW, q = r % 32;
    const int ln = (q >> 3) * 16 + bl;
    cst_off = (unsigned)((gglob * 16 * H * 2 + ((kwv * NL + (r / 32) * 2 + plane) * 64 + ln) * 8) * 2);
  }

  // input projections (independent of h), fetched two steps ahead through register rings
  // of three sets; with the LengthRegulator map the frame's source row index is fetched a
  // step before its projection row.  Every load is unconditional (clamped, valid address)
  // so no value is ever selected or copied before its use: the compiler's vmcnt waits stay
  // counted instead of draining (vector memory completes in issue order).
  const int32_t *iptr[CPT];
  size_t brow[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int b = cvalid[j] ? cb[j] : 0;
    iptr[j] = p.index ? p.index + (size_t)b * p.T : (const int32_t *)p.ws;
    brow[j] = (size_t)b * p.T_src;
  }
  const float *xcol = p.xp + dir * G * H + u0;   // + src row * stride + gate * H + unit
  const float *zcol = (p.index ? p.xp_zero : p.xp) + dir * G * H + u0;
  auto frame = [&](int t) { return dir ? (p.T - 1 - t) : t; };
  auto load_idx = [&](int t, int (&ir)[CPT]) {
    const int tt = frame(t < p.T ? t : p.T - 1);
#pragma unroll
    for (int j = 0; j < CPT; ++j) ir[j] = iptr[j][p.index ? tt : 0];
  };
  auto load_gx = [&](int t, const int (&ir)[CPT], float (&g)[CPT][G]) {
    const int tt = frame(t < p.T ? t : p.T - 1);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int src = p.index ? ir[j] : tt;
      const float *row = src >= 0 ? xcol + (brow[j] + src) * p.xp_stride : zcol;
      if (RNN_DIAG(p) & 1) row = zcol;  // timing experiment: L2-hot rows
#pragma unroll
      for (int gi = 0; gi < G; ++gi) g[j][gi] = row[gi * H + cu[j]];
    }
  };
  float g0[CPT][G], g1[CPT][G], g2[CPT][G];
  int i0[CPT], i1[CPT], i2[CPT];
  load_idx(0, i0);
  load_idx(1, i1);
  load_gx(0, i0, g0);
  load_gx(1, i1, g1);
  load_idx(2, i2);
  if (LOCAL)
    for (int i = tid; i < 16 * H; i += 256) hloc[i] = 0.f;
  __syncthreads();

#ifdef FTMI_RNN_STAMPS
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = 0;
  if (tid == 0) st_last = __builtin_amdgcn_s_memtime();
#endif

  // one time step; returns false when the launch must stop (hand-off timeout)
  auto step = [&](int t, const float (&gx)[CPT][G], float (&gnext)[CPT][G],
                  const int (&inext)[CPT], int (&iload)[CPT]) -> bool {
    const int tt = frame(t);
    STAMP(0);
    // h_{t-1} operand: NL float4 per lane (fragment order), zero at t = 0.  f16x3 groups of
    // several workgroups exchange h pre-split: hr[2 ks] = 8 heads, hr[2 ks + 1] = 8 scaled
    // tails (f16), used as MFMA operands directly.
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    constexpr bool HSPLIT = H3 && !LOCAL;
    float hv[HSPLIT ? 1 : NL * 4];
    u32x4 hr[NL];
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < (HSPLIT ? 1 : NL * 4); ++i) hv[i] = 0.f;
#pragma unroll
      for (int i = 0; i < NL; ++i) hr[i] = (u32x4){0u, 0u, 0u, 0u};
    } else if constexpr (LOCAL) {
      const float *hb = hloc + ((t - 1) & 1) * slab + wk * NL * 256 + lane * 4;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const f32x4 v = *(const f32x4 *)(hb + i * 256);
        hv[4 * i] = v.x;
        hv[4 * i + 1] = v.y;
        hv[4 * i + 2] = v.z;
        hv[4 * i + 3] = v.w;
      }
    } else {
      if constexpr (NBL != NB) {  // dead columns multiply zeros
#pragma unroll
        for (int i = 0; i < NL; ++i) hr[i] = (u32x4){0u, 0u, 0u, 0u};
      }
      // Tagged acquire: every exchanged h value carries h_tag(step) in its mantissa LSB;
      // re-load until this wave's whole K range carries the tag of h_{t-1}.  4-byte
      // accesses are single-copy atomic, so a torn 16-byte store only delays the read;
      // every load of the exchange buffer is sc1 (L2-served).
      const int soff = ((t - 1) & 1) * hx_par;
      for (int i = 0; i < p.psleep; ++i) __builtin_amdgcn_s_sleep(1);
      // fp32 words carry the tag in bit 0; f16 pairs in bits 0 and 16 (both halves)
      const unsigned tmask = HSPLIT ? 0x00010001u : 1u;
      const bool want1 = h_tag(t - 1) != 0u;  // uniform
      const bool hlive = (lane & 15) < NBL;  // this lane's h column is a live sequence
      for (unsigned spins = 0;; ++spins) {
        // a compiler memory barrier: the loop stores nothing, so without it LICM hoists the
        // loads out and the loop spins on the first values (it did once the timing switches
        // left the product build)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < NL; ++i)
          if ((NBL == NB || hlive) && !((RNN_DIAG(p) & 64) && i >= NL / 4))  // 64: a quarter
            hr[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, hoff + i * 1024, soff, 16);
        // every tag equals want iff (want 1) the AND of all words has the tag bits set,
        // (want 0) their OR has none: a 3-input reduction instead of a test per word
        bool fresh;
        if (want1) {
          u32x4 a = hr[0];
#pragma unroll
          for (int i = 1; i < NL; ++i) a &= hr[i];
          fresh = ((a.x & a.y & a.z & a.w) & tmask) == tmask;
        } else {
          u32x4 o = hr[0];
#pragma unroll
          for (int i = 1; i < NL; ++i) o |= hr[i];
          fresh = ((o.x | o.y | o.z | o.w) & tmask) == 0u;
        }
        if (__all(fresh || !hlive) || (RNN_DIAG(p) & 2) != 0) break;
        if (spins > p.spin_limit) {
          if (lane == 0) {
            s_abort = 1;
            report_timeout(p);
          }
          break;
        }
        // no back-off: a poll is an L2 round trip already, and an s_sleep between polls
        // measured +9 % per step on the postnet GRU (FTMI_RNN_DIAG bit 16 restores it)
        if (RNN_DIAG(p) & 16) __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int i = 0; i < (HSPLIT ? 0 : NL); ++i) {
        // NB: bit_cast the whole vector; extracting u32 lanes one by one and bit-casting
        // each is miscompiled by ROCm 7.2 (every lane reads element 0).
        const f32x4 v = __builtin_bit_cast(f32x4, hr[i]);
        hv[4 * i] = v.x;
        hv[4 * i + 1] = v.y;
        hv[4 * i + 2] = v.z;
        hv[4 * i + 3] = v.w;
      }
    }
    STAMP(1);
    load_gx(t + 2, inext, gnext);
    load_idx(t + 3, iload);
    STAMP(2);

    // partial gates over this wave's K range
    f32x4 acc[RBW];
#pragma unroll
    for (int i = 0; i < RBW; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (H3) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = HSPLIT ? 0.f : hv[HSPLIT ? 0 : ks * 8 + e];
        f16x8 hh, ht;
        if constexpr (HSPLIT) {  // pre-split by the producer
          hh = __builtin_bit_cast(f16x8, hr[2 * ks]);
          ht = __builtin_bit_cast(f16x8, hr[2 * ks + 1]);
        } else {
          split2h8(v, hh, ht);
        }
        const f16x8 hs = hh * (_Float16)H3_SCALE;  // 2^11 h_h: exact, |h| < 1
#pragma unroll
        for (int i = 0; i < RBW; ++i) {
          f32x4 c = acc[i];
          if (!(RNN_DIAG(p) & 32)) {  // 32: the big term only (timing)
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i][ks][1], hh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i][ks][0], ht, c, 0, 0, 0);
          }
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i][ks][0], hs, c, 0, 0, 0);
          acc[i] = c;
        }
      }
      // the 2^11 scale of the products stays in the partial sums: the cell applies 2^-11
      // in its first FMA (exact: a power of two), off the MFMA -> LDS critical path
    } else if constexpr (X6) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = hv[ks * 8 + e];
        bf16x8 h1, h2, h3;
        split3x8(v, h1, h2, h3);
#pragma unroll
        for (int i = 0; i < RBW; ++i) {
          f32x4 c = acc[i];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][2], h1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][1], h2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][0], h3, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][1], h1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][0], h2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks][0], h1, c, 0, 0, 0);
          acc[i] = c;
        }
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < RBW; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[i][kb], hv[kb], acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RBW; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        red[(wk * RR + (wr * RBW + i) * 16 + ls * 4 + e) * RED_STRIDE + lc] = acc[i][e];
    __syncthreads();
    if (!LOCAL && s_abort) return false;  // a wave timed out acquiring h_{t-1}
    STAMP(3);

    // cell update
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      if (HALFCELL && tid >= CELLS) continue;  // U = 8: waves 2-3 own no cells
      const int bl = cbl[j];
      float gs[G], gi[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int row = g * U + cu[j];
        float sum = red[row * RED_STRIDE + bl];
#pragma unroll
        for (int w = 1; w < WK; ++w) sum += red[(w * RR + row) * RED_STRIDE + bl];
        gs[g] = sum;  // H3: 2^11 (W_hh h)
        gi[g] = gx[j][g];
      }
      float hn;
      if (RNN_DIAG(p) & 128) {  // 128: no transcendentals (timing)
        hn = 0.25f * (fmaf(gs[0], GSC, gi[0]) + fmaf(gs[1], GSC, gi[1]) +
                      fmaf(gs[2], GSC, gi[2]) + (CELL ? fmaf(gs[G - 1], GSC, gi[G - 1]) : 0.f));
        hn = fminf(fmaxf(hn, -0.9f), 0.9f);
      } else if (CELL == 0) {
        // ATen GRU cell: r, z, n ; h' = n + z * (h - n)
        const float r = fast_sigmoid(gi[0] + fmaf(gs[0], GSC, bhh[j][0]));
        const float z = fast_sigmoid(gi[1] + fmaf(gs[1], GSC, bhh[j][1]));
        const float n = fast_tanh(gi[2] + r * fmaf(gs[2], GSC, bhh[j][2]));
        hn = n + z * (hstate[j] - n);
      } else {
        // LSTM cell: i, f, g, o
        const float ig = fast_sigmoid(fmaf(gs[0], GSC, gi[0]));
        const float fg = fast_sigmoid(fmaf(gs[1], GSC, gi[1]));
        const float gg = fast_tanh(fmaf(gs[2], GSC, gi[2]));
        const float og = fast_sigmoid(fmaf(gs[3], GSC, gi[3]));
        cstate[j] = fg * cstate[j] + ig * gg;
        hn = og * fast_tanh(cstate[j]);
      }
      if (tt >= len[j]) {  // packed-sequence padding: reverse direction restarts from zero
        hn = 0.f;
        cstate[j] = 0.f;
      }
      if constexpr (HSPLIT) {
        // exchanged pre-split: head h_h = f16(h) and scaled tail f16((h - h_h) 2^11), each
        // carrying the step tag in its mantissa LSB; the tail is taken AFTER the head's tag
        // bit is set, so the pair still represents h to ~2^-21 (the head's tag error is
        // absorbed by the tail).  The state and the output stay exact fp32.
        const unsigned short tg = (unsigned short)h_tag(t);
        const _Float16 h16 = __builtin_bit_cast(
            _Float16, (unsigned short)((__builtin_bit_cast(unsigned short, (_Float16)hn) & 0xFFFEu) | tg));
        const _Float16 t16 = __builtin_bit_cast(
            _Float16, (unsigned short)((__builtin_bit_cast(unsigned short,
                                                           (_Float16)((hn - (float)h16) * H3_SCALE)) &
                                        0xFFFEu) | tg));
        // chunk (seq, 8 units, plane) of halves: the comm wave's 16-B order
        _Float16 *hs16 = (_Float16 *)hstage;
        const int base = ((bl * (U / 8) + cu[j] / 8) * 2) * 8 + (cu[j] % 8);
        hs16[base] = h16;
        hs16[base + 8] = t16;
      } else if constexpr (!LOCAL) {
        // multi-workgroup groups: h_t carries the step tag in its mantissa LSB (a <= 1 ulp
        // change); the same tagged value is the state, the exchange and the layer output
        hn = __uint_as_float((__float_as_uint(hn) & ~1u) | h_tag(t));
      }
      const float yout = tt >= len[j] ? p.pad_value : hn;
      hstate[j] = hn;
      if constexpr (LOCAL) {
        if (cvalid[j]) {
          hloc[(t & 1) * slab + hxo[j]] = hn;
          p.y[((size_t)cb[j] * p.T + tt) * p.y_stride + dir * H + u0 + cu[j]] = yout;
        }
      } else {  // to the comm wave: cell c = bl * U + unit is also its float4 order
        const int c = bl * U + cu[j];
        if constexpr (!HSPLIT) hstage[c] = hn;
        ystage[c] = yout;
      }
    }
    if constexpr (CST) {
      // this wave's cells (sequences 4 wave .. 4 wave + 3, all 16 units) are the stage's
      // chunks 16 wave .. 16 wave + 15: read back (same wave, LDS in order) and store
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < 16 && (16 * wave + lane) / (U / 4) < NBL) {  // live sequences only
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = *(const u32x4 *)&hstage[(16 * wave + lane) * 4];
        if (xcd_mode)
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, cst_off, (t & 1) * hx_par, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, cst_off, (t & 1) * hx_par, 16);
      }
    }
    STAMP(4);
    __syncthreads();  // LOCAL: h_t visible in LDS; else: staged for the comm wave
    STAMP(5);
    return true;
  };

  for (int t = 0; t < p.T; t += 3) {
    if (!step(t, g0, g2, i2, i0)) break;
    if (t + 1 >= p.T || !step(t + 1, g1, g0, i0, i1)) break;
    if (t + 2 >= p.T || !step(t + 2, g2, g1, i1, i2)) break;
  }
#ifdef FTMI_RNN_STAMPS
  if (tid == 0)
    for (int i = 0; i < 6; ++i) ftmi_rnn_stamps[blockIdx.x * 8 + i] = st_acc[i];
#endif
}

// ---- small batches (B <= 4, e.g. batch-1 generation, config c2): exact fp32 GEMV -----
// At B = 1 the MFMA kernel above multiplies 16-column tiles with one live column and runs
// three f16 products per fp32 product on the per-step critical chain.  Here a group is one
// DIRECTION (all B <= NBV sequences), spread over BPG = H / U workgroups that each own U
// hidden units (R = G*U rows of W_hh, fp32, in VGPRs).  Thread (row pair rg, k-segment ks)
// holds 2 rows x SEG = H / 8 weights; per step it multiplies them by its segment of h_{t-1}
// (LDS, broadcast to the 8 row pairs of a wave), the 8 segments of a row are summed with
// xor shuffles, and U*B threads apply the cell update to the (unit, sequence) cells they
// own.  Exact fp32 FMAs, no split: the recurrence is fp32 like the reference's.  The h
// hand-off is the MFMA kernel's: step-tagged values (mantissa LSB), two parity halves,
// polled with sc1 loads, the census placing a direction's workgroups on one XCD (plain
// stores, L2-local) with the global write-through fallback.  Layout of a group's slab in
// the exchange buffer: [sequence][H] floats.
constexpr int GV_KSEG = 8;  // k-segments per row (lanes summed by shuffles)
constexpr int GV_RPT = 2;   // rows per thread

// KSEG: k-segments per row (GV_KSEG, or 16 — the default for H = 512 / 256: twice the
// threads, half the FMA chain per thread, one more shuffle stage)
template <int CELL, int H, int U, int NBV, int KSEG = GV_KSEG>
__global__ __launch_bounds__((CELL ? 4 : 3) * U / GV_RPT * KSEG) void rnn_gemv_kernel(
    const RnnParams p) {
  constexpr int G = CELL ? 4 : 3;
  constexpr int R = G * U;
  constexpr int NT = R / GV_RPT * KSEG;  // threads
  constexpr int SEG = H / KSEG;
  constexpr int SEGP = SEG + 4;             // LDS pitch of a segment: conflict-free b128 reads
  constexpr int BPG = H / U;
  constexpr int HF4 = H / 4;                // float4 of one sequence's h
  static_assert(R % GV_RPT == 0 && SEG % 4 == 0 && U * NBV <= NT && NT % 64 == 0, "shape");
  static_assert(BPG <= FLAGS_PER_GROUP, "group size");
  __shared__ __attribute__((aligned(16))) float hl[2][NBV * KSEG * SEGP];
  __shared__ float red[R][NBV];
  __shared__ int s_abort, s_group, s_bi, s_mode;

  const int tid = threadIdx.x, lane = tid & 63;
  const int ks = tid % KSEG, rg = tid / KSEG;

  // ---- group (= direction) assignment: the census of the MFMA kernel ----------------
  if (tid == 0) {
    int mode = 0, group = blockIdx.x % p.ngroups, bi = blockIdx.x / p.ngroups, abort = 0;
    if (p.xcd_local) {
      const unsigned x = xcc_id();
      const unsigned slot = __hip_atomic_fetch_add(p.ws + WS_CENSUS + x * CNT_PAD, 1u,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(p.ws + WS_ARRIVE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!poll_ge(p.ws + WS_ARRIVE, gridDim.x, p.spin_limit)) {
        abort = 1;
        report_timeout(p);
      } else if ((int)gridDim.x == 8 * BPG) {  // XCD x hosts group x (x < 2)
        bool balanced = true;
        for (int i = 0; i < 8; ++i)
          balanced &= __hip_atomic_load(p.ws + WS_CENSUS + i * CNT_PAD, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) == (unsigned)BPG;
        if (balanced) {
          mode = 1;
          group = (int)x;
          bi = (int)slot;
        }
      }
    }
    s_mode = mode;
    s_group = group;
    s_bi = bi;
    s_abort = abort;
  }
  __syncthreads();
  if (s_abort) return;
  if (s_group >= p.ngroups || s_bi >= BPG) return;  // surplus workgroups of the padded grid
  const int dir = s_group, u0 = s_bi * U;
  const bool xcd_mode = s_mode == 1;

  // ---- W_hh rows (gate g, unit u0 + u) of this thread's pair, its k-segment, fp32 ------
  const float *wdir = p.w_hh + (size_t)dir * (G * H) * H;
  float w[GV_RPT][SEG];
#pragma unroll
  for (int i = 0; i < GV_RPT; ++i) {
    const int r = rg * GV_RPT + i;
    const float *src = wdir + (size_t)((r / U) * H + u0 + r % U) * H + ks * SEG;
#pragma unroll
    for (int j = 0; j < SEG; j += 4) {
      const f32x4 v = *(const f32x4 *)(src + j);
      w[i][j] = v.x;
      w[i][j + 1] = v.y;
      w[i][j + 2] = v.z;
      w[i][j + 3] = v.w;
    }
  }

  // ---- the cell of this thread (threads < U * B): unit cu, sequence cb -----------------
  const bool is_cell = tid < U * p.B;
  const int cu = tid % U, cb = is_cell ? tid / U : 0;
  float hstate = 0.f, cstate = 0.f, bhh[G];
#pragma unroll
  for (int g = 0; g < G; ++g) bhh[g] = (CELL == 0) ? p.b_hh[dir * G * H + g * H + u0 + cu] : 0.f;
  const int len = (p.lengths && is_cell) ? p.lengths[cb] : p.T;
  const int32_t *iptr = p.index ? p.index + (size_t)cb * p.T : (const int32_t *)p.ws;
  const float *xcol = p.xp + dir * G * H + u0 + cu;
  const float *zcol = (p.index ? p.xp_zero : p.xp) + dir * G * H + u0 + cu;
  auto frame = [&](int t) { return dir ? (p.T - 1 - t) : t; };
  auto load_idx = [&](int t) -> int { return iptr[p.index ? frame(t < p.T ? t : p.T - 1) : 0]; };
  auto load_gx = [&](int t, int ir, float (&g)[G]) {
    const int tt = frame(t < p.T ? t : p.T - 1);
    const int src = p.index ? ir : tt;
    const float *row = src >= 0 ? xcol + ((size_t)cb * p.T_src + src) * p.xp_stride : zcol;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) g[gi] = row[gi * H];
  };
  float g0[G], g1[G], g2[G];
  int i0 = load_idx(0), i1 = load_idx(1);
  load_gx(0, i0, g0);
  load_gx(1, i1, g1);
  int i2 = load_idx(2);

  // ---- exchange: parity halves [2][2 dirs][NBV][H] --------------------------------------
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.hx, (short)0, 0x7FFFFFF0, 0x00020000);
  const int par_bytes = 2 * NBV * H * 4;
  const int nf4 = p.B * HF4;  // float4 of h a workgroup acquires per step
  const unsigned hx_off = (unsigned)(((dir * NBV + cb) * H + u0 + cu) * 4);  // this cell's h

  auto step = [&](int t, const float (&gx)[G], float (&gnext)[G], int inext, int &iload) -> bool {
    const int tt = frame(t);
    float *hb = hl[t & 1];
    // ---- acquire h_{t-1} (zero at t = 0) into LDS, segment-padded ------------------------
    const unsigned want = h_tag(t - 1);
    for (int f = tid; f < nf4; f += NT) {
      const int b = f / HF4, k = (f - b * HF4) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (t > 0) {
        const unsigned off = (unsigned)(((dir * NBV + b) * H + k) * 4);
        const int soff = ((t - 1) & 1) * par_bytes;
        for (unsigned spins = 0;; ++spins) {
          asm volatile("" ::: "memory");  // keep the load in the loop (see rnn_bidir_kernel)
          typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, soff, 16);
          const bool fresh = want ? ((r.x & r.y & r.z & r.w) & 1u) != 0u
                                  : ((r.x | r.y | r.z | r.w) & 1u) == 0u;
          if (fresh || (RNN_DIAG(p) & 2)) {
            v = __builtin_bit_cast(f32x4, r);
            break;
          }
          if (spins > p.spin_limit) {
            s_abort = 1;
            report_timeout(p);
            break;
          }
        }
      }
      *(f32x4 *)&hb[b * KSEG * SEGP + (k / SEG) * SEGP + k % SEG] = v;
    }
    // sequences past B (NBV > B): zero segments
    for (int f = nf4 + tid; f < NBV * HF4; f += NT) {
      const int b = f / HF4, k = (f - b * HF4) * 4;
      *(f32x4 *)&hb[b * KSEG * SEGP + (k / SEG) * SEGP + k % SEG] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if (s_abort) return false;
    if (is_cell) {  // the projections two steps ahead (independent of h)
      load_gx(t + 2, inext, gnext);
      iload = load_idx(t + 3);
    }
    // ---- partial gate sums over this thread's segment, then over the 8 segments ---------
    float acc[GV_RPT][NBV];
#pragma unroll
    for (int i = 0; i < GV_RPT; ++i)
#pragma unroll
      for (int b = 0; b < NBV; ++b) acc[i][b] = 0.f;
#pragma unroll
    for (int b = 0; b < NBV; ++b) {
      const float *hs = hb + b * KSEG * SEGP + ks * SEGP;
#pragma unroll
      for (int j = 0; j < SEG; j += 4) {
        const f32x4 hv = *(const f32x4 *)(hs + j);
#pragma unroll
        for (int i = 0; i < GV_RPT; ++i) {
          acc[i][b] = fmaf(w[i][j], hv.x, acc[i][b]);
          acc[i][b] = fmaf(w[i][j + 1], hv.y, acc[i][b]);
          acc[i][b] = fmaf(w[i][j + 2], hv.z, acc[i][b]);
          acc[i][b] = fmaf(w[i][j + 3], hv.w, acc[i][b]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GV_RPT; ++i)
#pragma unroll
      for (int b = 0; b < NBV; ++b) {
        float v = acc[i][b];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        if constexpr (KSEG == 16) v += __shfl_xor(v, 8);
        acc[i][b] = v;
      }
    if (ks < GV_RPT)
#pragma unroll
      for (int b = 0; b < NBV; ++b)
        red[rg * GV_RPT + ks][b] = ks == 0 ? acc[0][b] : acc[GV_RPT - 1][b];
    __syncthreads();
    // ---- cell update (the MFMA kernel's formulas) -----------------------------------------
    if (is_cell) {
      float gs[G];
#pragma unroll
      for (int g = 0; g < G; ++g) gs[g] = red[g * U + cu][cb];
      float hn;
      if (CELL == 0) {
        const float r = fast_sigmoid(gx[0] + (gs[0] + bhh[0]));
        const float z = fast_sigmoid(gx[1] + (gs[1] + bhh[1]));
        const float n = fast_tanh(gx[2] + r * (gs[2] + bhh[2]));
        hn = n + z * (hstate - n);
      } else {
        const float ig = fast_sigmoid(gx[0] + gs[0]);
        const float fg = fast_sigmoid(gx[1] + gs[1]);
        const float gg = fast_tanh(gx[2] + gs[2]);
        const float og = fast_sigmoid(gx[3] + gs[3]);
        cstate = fg * cstate + ig * gg;
        hn = og * fast_tanh(cstate);
      }
      if (tt >= len) {
        hn = 0.f;
        cstate = 0.f;
      }
      hn = __uint_as_float((__float_as_uint(hn) & ~1u) | h_tag(t));
      hstate = hn;
      const float yout = tt >= len ? p.pad_value : hn;
      const int soff = (t & 1) * par_bytes;
      if (xcd_mode)  // stays in this XCD's L2, read back by same-XCD sc1 loads
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), rsrc, hx_off, soff, 0);
      else  // write-through (sc1)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hn), rsrc, hx_off, soff, 16);
      p.y[((size_t)cb * p.T + tt) * p.y_stride + dir * H + u0 + cu] = yout;
    }
    return true;
  };

  for (int t = 0; t < p.T; t += 3) {
    if (!step(t, g0, g2, i2, i0)) break;
    if (t + 1 >= p.T || !step(t + 1, g1, g0, i0, i1)) break;
    if (t + 2 >= p.T || !step(t + 2, g2, g1, i1, i2)) break;
  }
}

template <int CELL, int H, int U, int KSEG = GV_KSEG>
int launch_gemv(RnnParams p, int max_blocks, hipStream_t s) {
  constexpr int BPG = H / U;
  constexpr int NT = (CELL ? 4 : 3) * U / GV_RPT * KSEG;
  if (8 * BPG > max_blocks) return FTMI_E_UNSUPPORTED;
  p.chunk0 = 0;
  p.ngroups = 2;
  // one direction's BPG workgroups per XCD (the census seats direction x on XCD x; the
  // other XCDs' workgroups retire after the census barrier)
  const int nblk = p.xcd_local ? 8 * BPG : 2 * BPG;
#define FTMI_GEMV_LAUNCH(NBV_)                                                             \
  if (int rc = ftmi_resident_ok((const void *)rnn_gemv_kernel<CELL, H, U, NBV_, KSEG>, nblk, NT, 0)) \
    return rc;                                                                               \
  hipLaunchKernelGGL((rnn_gemv_kernel<CELL, H, U, NBV_, KSEG>), dim3(nblk), dim3(NT), 0, s, p); \
  break;
  switch (p.B) {
    case 1: FTMI_GEMV_LAUNCH(1)
    case 2: FTMI_GEMV_LAUNCH(2)
    default: FTMI_GEMV_LAUNCH(4)
  }
#undef FTMI_GEMV_LAUNCH
  FTMI_CHECK_LAUNCH();
  return FTMI_OK;
}

template <int CELL, int H, int U, int WK, int MODE, bool CST = false, int NBL = NB>
int launch_rnn(RnnParams p, int nchunks, int max_blocks, hipStream_t s) {
  if (NBL != NB) {  // chunks of NBL sequences (the caller counted chunks of NB)
    nchunks = (p.B + NBL - 1) / NBL;
    p.ngroups_total = 2 * nchunks;
  }
  if (!hx_fits(p, H, (int64_t)NB * H)) return FTMI_E_SHAPE;  // never index past the workspace
  constexpr int BPG = H / U;
  int max_groups = (max_blocks / BPG) & ~1;
  if (max_groups < 2) return FTMI_E_UNSUPPORTED;
  for (int c0 = 0; c0 < nchunks; c0 += max_groups / 2) {
    const int nc = (nchunks - c0) < max_groups / 2 ? (nchunks - c0) : max_groups / 2;
    p.chunk0 = c0;
    p.ngroups = 2 * nc;
    if (c0 > 0) {  // the census words are per launch
      hipError_t e = hipMemsetAsync(p.ws + WS_CENSUS, 0, (WS_FLAGS - WS_CENSUS) * 4, s);
      if (e != hipSuccess) return (int)e;
    }
    // fewer than 8 groups (small batches): pad the grid to BPG workgroups per XCD so that
    // each group can run inside one XCD (the census picks the layout); FTMI_RNN_PAD=0 off
    static const int pad_env = [] {
      const char *v = getenv("FTMI_RNN_PAD");
      return v ? atoi(v) : 1;
    }();
    int nblk = p.ngroups * BPG;
    if (BPG > 1 && pad_env && p.xcd_local && p.ngroups < 8 && 8 * BPG <= max_blocks)
      nblk = 8 * BPG;
    if (int rc = ftmi_resident_ok((const void *)rnn_bidir_kernel<CELL, H, U, WK, MODE, CST, NBL>,
                                  nblk, BPG == 1 ? 256 : 320, 0))
      return rc;
    hipLaunchKernelGGL((rnn_bidir_kernel<CELL, H, U, WK, MODE, CST, NBL>), dim3(nblk),
                       dim3(BPG == 1 ? 256 : 320), 0, s, p);
    FTMI_CHECK_LAUNCH();
  }
  return FTMI_OK;
}

int device_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

}  // namespace

// B <= GV_MAXB: the exact-fp32 GEMV recurrence (rnn_gemv_kernel), 16 units per workgroup;
// FTMI_RNN_GEMV=0 keeps the MFMA kernel
constexpr int GV_MAXB = 4;
static bool gemv_path(int cell, int B, int H) {
  const char *v = getenv("FTMI_RNN_GEMV");  // read per call: tests switch it
  const int env = v ? atoi(v) : 1;
  return env && B <= GV_MAXB && ((cell == 1 && H == 512) || (cell == 0 && (H == 64 || H == 128 || H == 256)));
}
static int xcd_local_env() {
  static const int v = [] {
    const char *e = getenv("FTMI_RNN_XCD_LOCAL");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// hidden units per workgroup of the instance ftmi_rnn_bidir dispatches (see there)
static int rnn_units(int cell, int H, int mma) {
  if (cell == 0 && H == 64) {
    static const int u64 = [] {
      const char *v = getenv("FTMI_RNN_U64");
      return v ? atoi(v) : 32;
    }();
    return (mma == 2 && u64 == 32) ? 32 : 64;
  }
  return 16;
}

// FTMI_RNN_CSTORE=0 (read per call) keeps the comm wave's h stores: measured at c3, the
// compute waves' own stores take the postnet GRU 1.315 -> 1.116 us/step, the LSTM 1.55 ->
// 1.535 (barrier C and the stage read leave the hand-off's critical path)
static bool cst_enabled() {
  const char *v = getenv("FTMI_RNN_CSTORE");
  return !(v && atoi(v) == 0);
}
// live sequences per group of a spread f16x3 GRU on rnn_bidir_kernel: 8 when twice the groups
// still fit the device at once (the c3 postnet GRU: 256 instead of 128 workgroups, half the h
// bytes per workgroup and step); FTMI_RNN_NB=16 keeps 16 (read per call)
static int legacy_nbl(int cell, int B, int H, int mma, bool spread, int maxb) {
  const char *v = getenv("FTMI_RNN_NB");
  if (!spread || mma != 2 || cell != 0 || H != 256 || !cst_enabled() ||
      (v && atoi(v) == 16))
    return NB;
  return 2 * ((B + 7) / 8) * (H / 16) <= maxb ? 8 : NB;
}

// The spread postnet GRU (H 256, f16x3, CST) on workgroups of 8 units (rnn_bidir_kernel
// U = 8) while every group's workgroups fit one per CU (B <= 64 on 256 CUs: 8 groups x 32);
// FTMI_RNN_U8=0 (read per call: tests switch it) keeps 16 units.  Rejected this round and
// removed: U = 8 for the LSTM (64 workgroups per group, two per CU — both of the same group
// under the census layout, so no MFMA time is saved, and five-wave workgroups at 150 VGPRs
// were not reliably co-resident two per CU: the census timed out), the GRU at U = 8 with 8
// live sequences (1.48 against 1.39 us/step) and one barrier per step (parity-buffered
// partials: LSTM 1.59 against 1.53, GRU at U = 8 1.18 against 1.11).
static bool u8_path(int cell, int B, int H, int mma, bool spread, int maxb) {
  if (!spread || mma != 2 || !cst_enabled() || cell != 0 || H != 256) return false;
  const char *v = getenv("FTMI_RNN_U8");
  if (v && atoi(v) == 0) return false;
  const int ngroups = 2 * ((B + NB - 1) / NB);
  return (ngroups < 8 ? 8 : ngroups) * (H / 8) <= maxb;
}

extern "C" int32_t ftmi_rnn_blocks(int32_t cell, int32_t B, int32_t H, int32_t mma) {
  if (B <= 0 || H <= 0 || H % 16 != 0) return 0;
  const bool spread = (mma & FTMI_RNN_SPREAD) != 0;
  mma &= 0xFF;
  if (gemv_path(cell, B, H)) return (xcd_local_env() ? 8 : 2) * (H / 16);  // launch_gemv
  if (u8_path(cell, B, H, mma, spread, device_cu_count())) {  // launch_rnn U = 8: one group
    const int ngroups = 2 * ((B + NB - 1) / NB);                // pass, padded to 8 groups
    return (ngroups < 8 && xcd_local_env() ? 8 : ngroups) * (H / 8);
  }
  const int bpg = H / rnn_units(cell, H, mma);
  const int maxb = device_cu_count();
  const int max_groups = (maxb / bpg) & ~1;
  if (max_groups < 2) return 0;
  const int nbl = legacy_nbl(cell, B, H, mma, spread, maxb);
  const int nchunks = (B + nbl - 1) / nbl;
  const int ngroups = 2 * (nchunks < max_groups / 2 ? nchunks : max_groups / 2);
  int nblk = ngroups * bpg;
  if (bpg > 1 && ngroups < 8 && 8 * bpg <= maxb) nblk = 8 * bpg;  // launch_rnn's padding
  return nblk;
}

extern "C" int64_t ftmi_rnn_workspace_bytes(int32_t B, int32_t H, int32_t cell) {
  (void)cell;
  if (B <= 0 || H <= 0) return 0;
  const int64_t nchunks = ws_chunks(B);
  return ctl_bytes(nchunks) + 2 * (2 * nchunks) * NB * (int64_t)H * (int64_t)sizeof(float);
}


extern "C" uint32_t ftmi_set_rnn_spin_limit(uint32_t limit) {
  const unsigned prev = g_spin_limit;
  g_spin_limit = limit ? limit : SPIN_LIMIT_DEFAULT;
  return prev;
}

extern "C" int64_t ftmi_rnn_error_offset(int32_t B) {
  (void)B;
  return WS_ERR * (int64_t)sizeof(unsigned);
}

// the launch set-up of ftmi_rnn_bidir: clears the workspace (control words and the exchange buffer) and fills the common parameters
static int rnn_setup(RnnParams &p, int B, int T, int H, int cell, const float *w_hh,
                     const float *b_hh, const int32_t *lengths, float pad_value, float *y,
                     int64_t y_stride, uint32_t *status, void *sync, hipStream_t s,
                     int &nchunks) {
  nchunks = (B + NB - 1) / NB;
  const int64_t ctl = ctl_bytes(ws_chunks(B));
  const int64_t wsb = ftmi_rnn_workspace_bytes(B, H, cell);
  hipError_t e = hipMemsetAsync(sync, 0, (size_t)wsb, s);
  if (e != hipSuccess) return (int)e;
  p.w_hh = w_hh;
  p.b_hh = b_hh;
  p.y = y;
  p.y_stride = y_stride;
  p.lengths = lengths;
  p.pad_value = pad_value;
  p.B = B;
  p.T = T;
  p.ngroups_total = 2 * nchunks;
  p.xcd_local = xcd_local_env();
  p.ws = (unsigned *)sync;
  p.hx = (float *)((char *)sync + ctl);
  p.status = status;
  p.spin_limit = g_spin_limit;
#ifdef FTMI_DIAG
  static const int diag_env = [] {
    const char *v = getenv("FTMI_RNN_DIAG");
    return v ? atoi(v) : 0;
  }();
  p.diag = diag_env;
#endif
  // s_sleep(1) count before a step's first h poll (rnn_bidir_kernel): the first poll then
  // lands after the producers' stores instead of a round trip before them.  Interleaved A/B
  // at c3 (tools/rnn_env_ab.py, two boxes): 3 -> LSTM 1.55 -> 1.52-1.54, postnet GRU 1.32 ->
  // 1.27 us/step; 6 made the LSTM slower again (1.58-1.61)
  // (-1 = unset: 3, and 6 for the spread postnet GRU on 8-unit workgroups — its producers
  // store later in the step: 1.12-1.13 -> 1.08 us/step at c3, round 5, profiles/r5_rnn_diag.txt)
  static const int psleep_env = [] {
    const char *v = getenv("FTMI_RNN_PSLEEP");
    return v ? atoi(v) : -1;
  }();
  p.psleep = psleep_env < 0 ? 3 : psleep_env;
  return FTMI_OK;
}

// first-poll delay of the U = 8 spread GRU (see rnn_setup)
static int u8_psleep() {
  const char *v = getenv("FTMI_RNN_PSLEEP");
  return v ? atoi(v) : 6;
}

extern "C" int ftmi_rnn_bidir(int32_t cell, int32_t B, int32_t T, int32_t H, const float *xp,
                              int64_t xp_stride, int32_t T_src, const int32_t *index,
                              const float *xp_zero, const float *w_hh, const float *b_hh,
                              const int32_t *lengths, float pad_value, float *y,
                              int64_t y_stride, int32_t mma, uint32_t *status, void *sync,
                              ftmi_stream_t stream) {
  if (!xp || !w_hh || !y || !sync) return FTMI_E_ARG;
  if (B <= 0 || T <= 0 || H <= 0 || T_src <= 0) return FTMI_E_ARG;
  const bool spread = (mma & FTMI_RNN_SPREAD) != 0;
  mma &= ~FTMI_RNN_SPREAD;
  if (mma < 0 || mma > 2) return FTMI_E_ARG;
  if (cell == 0 && !b_hh) return FTMI_E_ARG;
  if (index && !xp_zero) return FTMI_E_ARG;
  if (!index && T_src != T) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(w_hh) || !ftmi_aligned16(sync)) return FTMI_E_ALIGN;
  if (!ftmi_aligned16(y) || (y_stride & 3)) return FTMI_E_ALIGN;  // float4 row stores
  // the kernel forms below: GRU H 64 / 128 / 256, LSTM H 512 — refused before any HIP call
  // (the workspace memset), so an unsupported shape leaves no HIP error behind
  if (cell == 1 ? H != 512 : (cell != 0 || (H != 64 && H != 128 && H != 256)))
    return FTMI_E_UNSUPPORTED;
  hipStream_t s = ftmi_hs(stream);
  RnnParams p = {};
  int nchunks = 0;
  const int rc = rnn_setup(p, B, T, H, cell, w_hh, b_hh, lengths, pad_value, y, y_stride,
                           status, sync, s, nchunks);
  if (rc != FTMI_OK) return rc;
  p.xp = xp;
  p.xp_stride = xp_stride;
  p.T_src = T_src;
  p.index = index;
  p.xp_zero = xp_zero;
  const int maxb = device_cu_count();
  // small batches: exact fp32 GEMV recurrence (any mma: it is exact)
  if (gemv_path(cell, B, H)) {
    // H = 512 / 256: 16 k-segments per row (512 / 384 threads, half the FMA chain per thread):
    // c2 LSTM 1.26 -> 1.17-1.18, postnet GRU 1.01 -> 0.96-0.97 us/step (tools/rnn_diag.py,
    // two interleaved rounds; 32 segments: 1.32-1.34 / 1.07-1.08).  FTMI_RNN_GEMV_KSEG=8 (read
    // per call) keeps 8.
    const char *kv = getenv("FTMI_RNN_GEMV_KSEG");
    const bool k8 = kv && atoi(kv) == 8;
    if (cell == 1) return k8 ? launch_gemv<1, 512, 16>(p, maxb, s) : launch_gemv<1, 512, 16, 16>(p, maxb, s);
    if (H == 256) return k8 ? launch_gemv<0, 256, 16>(p, maxb, s) : launch_gemv<0, 256, 16, 16>(p, maxb, s);
    if (H == 128) return launch_gemv<0, 128, 16>(p, maxb, s);
    return launch_gemv<0, 64, 16>(p, maxb, s);
  }
#define FTMI_RNN_MODES(CELL_, H_, U_, WKX_, WKF_)                                   \
  switch (mma) {                                                                    \
    case 2: return launch_rnn<CELL_, H_, U_, WKX_, 2>(p, nchunks, maxb, s);          \
    case 1: return launch_rnn<CELL_, H_, U_, WKX_, 1>(p, nchunks, maxb, s);          \
    default: return launch_rnn<CELL_, H_, U_, WKF_, 0>(p, nchunks, maxb, s);         \
  }
  // H = 64 on the f16x3 path: 32 units per workgroup (2 per group, h exchanged through L2)
  // 1.19 us/step against 1.45 for one workgroup per group (h in LDS) at B = 64;
  // FTMI_RNN_U64=64 selects the single-workgroup form
  if (cell == 0 && H == 64) {
    if (rnn_units(cell, H, mma) == 32) return launch_rnn<0, 64, 32, 2, 2>(p, nchunks, maxb, s);
    FTMI_RNN_MODES(0, 64, 64, 2, 4)
  }
  // H = 128: 16 units per workgroup (8 workgroups per group): 1.04 us/step against 2.33 with
  // 64 units (2 workgroups) at B = 64 — the per-step cell and MFMA work of a workgroup
  // shrinks 4x for one more hop in the exchange
  if (cell == 0 && H == 128) FTMI_RNN_MODES(0, 128, 16, 4, 4)
  // H = 256 / 512: 16 units per workgroup (32 units measured 1.84 against 1.19 us/step for
  // the H = 256 GRU; the LSTM's W_hh slice does not fit the VGPRs at 32 units)
  // f16x3, 16 units per workgroup: the compute waves store their own h (CST) and a spread
  // GRU runs 8 live sequences per group (legacy_nbl).  H = 128 keeps the form above (it
  // returned before this block since round 3; legacy_nbl agrees, so ftmi_rnn_blocks reports
  // the launch's real workgroup count)
  if (mma == 2 && cst_enabled() && ((cell == 1 && H == 512) || (cell == 0 && H == 256))) {
    const bool nb8 = legacy_nbl(cell, B, H, mma, spread, maxb) == 8;
    if (u8_path(cell, B, H, mma, spread, maxb)) {
      p.psleep = u8_psleep();
      return launch_rnn<0, 256, 8, 4, 2, true>(p, nchunks, maxb, s);
    }
    if (cell == 1) return launch_rnn<1, 512, 16, 4, 2, true>(p, nchunks, maxb, s);
    return nb8 ? launch_rnn<0, 256, 16, 4, 2, true, 8>(p, nchunks, maxb, s)
               : launch_rnn<0, 256, 16, 4, 2, true>(p, nchunks, maxb, s);
  }
  if (cell == 0 && H == 256) FTMI_RNN_MODES(0, 256, 16, 4, 4)
  if (cell == 1 && H == 512) FTMI_RNN_MODES(1, 512, 16, 4, 4)
#undef FTMI_RNN_MODES
  return FTMI_E_UNSUPPORTED;
}

#ifdef FTMI_RNN_STAMPS
extern "C" int ftmi_debug_rnn_stamps(unsigned long long *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ftmi_rnn_stamps),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif
