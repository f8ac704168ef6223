// Persistent bidirectional GRU / LSTM recurrence (gfx950, fp32 MFMA 16x16x4).
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
// BPG = H / U workgroups, each owning U hidden units (all G gates of them, R = G*U rows
// of W_hh).  The workgroup keeps its W_hh slice in VGPRs for the whole sequence, laid out
// as MFMA A-fragments: wave w covers k in [w*H/4, (w+1)*H/4) and lane slot s = lane>>4
// takes k = w*KW + s*KB + kb at MFMA kb, so every lane's fragments (and its h operand) are
// KB consecutive floats.  Per step each wave produces R x 16 partial gate sums over its
// quarter of K, the four partials are summed through LDS, and 256 threads apply the cell
// update to the U x 16 (unit, sequence) cells they own (c / h state lives in registers).
//
// Hand-off between the BPG workgroups of a group (MI355X_MICROARCH.md "Valid forms",
// row 1): new h values go to a small exchange buffer hx[t & 1][group][16*H] in the call's
// workspace, stored in MFMA-FRAGMENT ORDER ([wave][kb/4][lane][4]) so that every consumer
// wave-instruction reads 1 KB of consecutive bytes (sc1 loads bypass L1: a row-major image
// made each instruction touch 64 lines and fetch every line 8 times) (parity double buffering is race-free because a workgroup can only start
// step t+1 after every workgroup of its group finished step t) with write-through (sc1)
// stores; every storing wave drains
// vmcnt(0); after a workgroup barrier ONE lane adds 1 to the group's arrival counter
// (agent-scope atomic).  Before step t, ONE lane polls that counter with relaxed sc1
// loads until it reaches t*BPG, the workgroup barrier releases the other waves, and all
// loads of the handed-off h are sc1 buffer loads.  The layer output y is written with
// plain stores (nothing in the launch reads it back), so it may hold padding values.
//
// Packed sequences (forward(), models/forward_tacotron.py:224-230): with lengths != NULL
// frames t >= lengths[b] output pad_value, and the reverse direction keeps h = c = 0
// until t = lengths[b]-1, exactly like pack_padded_sequence + pad_packed_sequence.
// Every spin is bounded; on timeout the call's error word is set and the workgroup leaves
// the time loop.
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

namespace {

constexpr int NB = 16;              // sequences per group (MFMA 16x16 columns)
constexpr int RED_STRIDE = NB + 1;  // LDS partial-sum row stride (floats)
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int CNT_PAD = 32;  // one 128-B line per group counter

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
  float *hx;  // [2][nchunks*NB][2H]
  int B, T;
  int nrows_hx;  // rows per parity half of hx (= nchunks * NB)
  int chunk0;   // first batch chunk of this launch
  int ngroups;  // groups in this launch
  unsigned *cnt;
  unsigned *err;
};

template <int CELL, int H, int U>
__global__ __launch_bounds__(256, 1) void rnn_bidir_kernel(const RnnParams p) {
  constexpr int G = CELL ? 4 : 3;
  constexpr int R = G * U;
  constexpr int RB = R / 16;
  constexpr int KW = H / 4;
  constexpr int KB = KW / 4;
  constexpr int BPG = H / U;
  constexpr int CELLS = U * NB;
  constexpr int CPT = CELLS / 256;
  static_assert(U % 16 == 0 && H % U == 0 && KB % 4 == 0 && CELLS % 256 == 0, "shape");

  __shared__ __attribute__((aligned(16))) float red[4 * R * RED_STRIDE];
  __shared__ int s_abort;

  const int group = blockIdx.x % p.ngroups;
  const int bi = blockIdx.x / p.ngroups;
  const int dir = group & 1;
  const int chunk = p.chunk0 + (group >> 1);
  const int u0 = bi * U;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ls = lane >> 4, lc = lane & 15;
  unsigned *cnt = p.cnt + (size_t)(p.chunk0 * 2 + group) * CNT_PAD;

  // ---- W_hh slice -> VGPR A-fragments (loaded once) ---------------------------------
  float wf[RB][KB];
  {
    const float *wdir = p.w_hh + (size_t)dir * (G * H) * H;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int lrow = rb * 16 + lc;
      const int grow = (lrow / U) * H + u0 + (lrow % U);
      const float *src = wdir + (size_t)grow * H + wave * KW + ls * KB;
#pragma unroll
      for (int kb = 0; kb < KB; kb += 4) {
        const f32x4 v = *(const f32x4 *)(src + kb);
        wf[rb][kb] = v.x;
        wf[rb][kb + 1] = v.y;
        wf[rb][kb + 2] = v.z;
        wf[rb][kb + 3] = v.w;
      }
    }
  }

  // ---- per-thread cells: cell c = tid + 256*j -> (unit u = c % U, seq b = c / U) ------
  int cu[CPT], cb[CPT];
  bool cvalid[CPT];
  float hstate[CPT], cstate[CPT], bhh[CPT][G];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = tid + 256 * j;
    cu[j] = c % U;
    cb[j] = chunk * NB + c / U;
    cvalid[j] = cb[j] < p.B;
    hstate[j] = 0.f;
    cstate[j] = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g)
      bhh[j][g] = (CELL == 0) ? p.b_hh[dir * G * H + g * H + u0 + cu[j]] : 0.f;
  }

  // ---- h operand source: this group's fragment-ordered slab of the exchange buffer ---
  // slab (16*H floats) = [wave 4][kbq KB/4][lane 64][4]; (seq bl, unit k) lives at
  //   (((k / KW) * (KB/4) + (k % KB) / 4) * 64 + ((k % KW) / KB) * 16 + bl) * 4 + (k % 4)
  const int gglob = 2 * chunk + dir;
  const int slab = 16 * H;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.hx, (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned hoff = (unsigned)(((gglob * slab) + wave * (KB / 4) * 256 + lane * 4) * 4);
  const int hx_par = p.nrows_hx * 2 * H * 4;  // bytes between the two parity halves
  int hxo[CPT];  // this thread's cells in the slab
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int k = u0 + cu[j], bl = cb[j] - chunk * NB;
    hxo[j] = gglob * slab + (((k / KW) * (KB / 4) + (k % KB) / 4) * 64 + ((k % KW) / KB) * 16 + bl) * 4 + (k % 4);
  }
  int len[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) len[j] = (p.lengths && cvalid[j]) ? p.lengths[cb[j]] : p.T;

  if (tid == 0) s_abort = 0;
  __syncthreads();
#ifdef FTMI_RNN_STAMPS
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = 0;
  if (tid == 0) st_last = __builtin_amdgcn_s_memtime();
#endif

  // input projections (independent of h): step t+1's rows are fetched during step t
  auto load_gx = [&](int t, float (&g)[CPT][G]) {
    const int tt = dir ? (p.T - 1 - t) : t;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int b = cvalid[j] ? cb[j] : 0;
      int src = tt;
      if (p.index) src = p.index[(size_t)b * p.T + tt];
      const float *row = src >= 0 ? p.xp + ((size_t)b * p.T_src + src) * p.xp_stride : p.xp_zero;
#pragma unroll
      for (int gi = 0; gi < G; ++gi) g[j][gi] = row[dir * G * H + gi * H + u0 + cu[j]];
    }
  };
  float gx[CPT][G], gxn[CPT][G];
  load_gx(0, gx);

  for (int t = 0; t < p.T; ++t) {
    const int tt = dir ? (p.T - 1 - t) : t;

    STAMP(0);  // xp gather issued (and landed, in the stamp build)
    // wait until every workgroup of the group has published h_{t-1}
    if (BPG > 1 && t > 0) {
      if (tid == 0) {
        const unsigned target = (unsigned)t * BPG;
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_LIMIT) {
            s_abort = 1;
            __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
      if (s_abort) break;
    }

    STAMP(1);  // group arrival observed
    // h_{t-1} operand (sc1 loads), zero at t = 0
    float hf[KB];
    if (t == 0) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) hf[kb] = 0.f;
    } else {
      const int soff = ((t - 1) & 1) * hx_par;
#pragma unroll
      for (int kb = 0; kb < KB; kb += 4) {
        // NB: bit_cast the whole vector; extracting u32 lanes one by one and bit-casting
        // each is miscompiled by ROCm 7.2 (every lane reads element 0).
        const f32x4 v = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, hoff + kb * 256, soff, 16));
        hf[kb] = v.x;
        hf[kb + 1] = v.y;
        hf[kb + 2] = v.z;
        hf[kb + 3] = v.w;
      }
    }

    if (t + 1 < p.T) load_gx(t + 1, gxn);
    STAMP(2);  // h operand landed
    // partial gates over this wave's quarter of K
    f32x4 acc[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[rb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[rb][kb], hf[kb], acc[rb], 0, 0, 0);

#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[(wave * R + rb * 16 + ls * 4 + i) * RED_STRIDE + lc] = acc[rb][i];
    __syncthreads();
    STAMP(3);  // MFMAs + partial sums in LDS

    // cell update
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int bl = cb[j] - chunk * NB;
      float gs[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int row = g * U + cu[j];
        gs[g] = red[(0 * R + row) * RED_STRIDE + bl] + red[(1 * R + row) * RED_STRIDE + bl] +
                red[(2 * R + row) * RED_STRIDE + bl] + red[(3 * R + row) * RED_STRIDE + bl];
      }
      float hn;
      if (CELL == 0) {
        // ATen GRU cell: r, z, n ; h' = n + z * (h - n)
        const float r = ftmi_sigmoid(gx[j][0] + (gs[0] + bhh[j][0]));
        const float z = ftmi_sigmoid(gx[j][1] + (gs[1] + bhh[j][1]));
        const float n = tanhf(gx[j][2] + r * (gs[2] + bhh[j][2]));
        hn = n + z * (hstate[j] - n);
      } else {
        // LSTM cell: i, f, g, o
        const float ig = ftmi_sigmoid(gx[j][0] + gs[0]);
        const float fg = ftmi_sigmoid(gx[j][1] + gs[1]);
        const float gg = tanhf(gx[j][2] + gs[2]);
        const float og = ftmi_sigmoid(gx[j][3] + gs[3]);
        cstate[j] = fg * cstate[j] + ig * gg;
        hn = og * tanhf(cstate[j]);
      }
      float yout = hn;
      if (tt >= len[j]) {  // packed-sequence padding: reverse direction restarts from zero
        hn = 0.f;
        cstate[j] = 0.f;
        yout = p.pad_value;
      }
      hstate[j] = hn;
      if (cvalid[j]) {
        __hip_atomic_store(p.hx + (size_t)(t & 1) * p.nrows_hx * 2 * H + hxo[j], hn,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p.y[((size_t)cb[j] * p.T + tt) * p.y_stride + dir * H + u0 + cu[j]] = yout;
      }
    }

#pragma unroll
    for (int j = 0; j < CPT; ++j)
#pragma unroll
      for (int gi = 0; gi < G; ++gi) gx[j][gi] = gxn[j][gi];
    STAMP(4);  // cell update + stores issued
    // publish: every storing wave drains, barrier, one lane arrives
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (BPG > 1 && tid == 0)
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    STAMP(5);  // drained + arrived
  }
#ifdef FTMI_RNN_STAMPS
  if (tid == 0)
    for (int i = 0; i < 6; ++i) ftmi_rnn_stamps[blockIdx.x * 8 + i] = st_acc[i];
#endif
}

template <int CELL, int H, int U>
int launch_rnn(RnnParams p, int nchunks, int max_blocks, hipStream_t s) {
  constexpr int BPG = H / U;
  int max_groups = (max_blocks / BPG) & ~1;
  if (max_groups < 2) return FTMI_E_UNSUPPORTED;
  for (int c0 = 0; c0 < nchunks; c0 += max_groups / 2) {
    const int nc = (nchunks - c0) < max_groups / 2 ? (nchunks - c0) : max_groups / 2;
    p.chunk0 = c0;
    p.ngroups = 2 * nc;
    hipLaunchKernelGGL((rnn_bidir_kernel<CELL, H, U>), dim3(p.ngroups * BPG), dim3(256), 0, s, p);
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

// workspace: [counters: 2*nchunks lines][err: 1 line][hx: 2 * nchunks*NB * 2H floats]
extern "C" int64_t ftmi_rnn_workspace_bytes(int32_t B, int32_t H, int32_t cell) {
  (void)cell;
  if (B <= 0 || H <= 0) return 0;
  const int64_t nchunks = (B + NB - 1) / NB;
  return (2 * nchunks * CNT_PAD + CNT_PAD) * (int64_t)sizeof(unsigned) +
         2 * nchunks * NB * 2 * (int64_t)H * (int64_t)sizeof(float);
}

extern "C" int ftmi_rnn_bidir(int32_t cell, int32_t B, int32_t T, int32_t H, const float *xp,
                              int64_t xp_stride, int32_t T_src, const int32_t *index,
                              const float *xp_zero, const float *w_hh, const float *b_hh,
                              const int32_t *lengths, float pad_value, float *y,
                              int64_t y_stride, void *sync, ftmi_stream_t stream) {
  if (!xp || !w_hh || !y || !sync) return FTMI_E_ARG;
  if (B <= 0 || T <= 0 || H <= 0 || T_src <= 0) return FTMI_E_ARG;
  if (cell == 0 && !b_hh) return FTMI_E_ARG;
  if (index && !xp_zero) return FTMI_E_ARG;
  if (!index && T_src != T) return FTMI_E_SHAPE;
  if (!ftmi_aligned16(w_hh) || !ftmi_aligned16(sync)) return FTMI_E_ALIGN;
  hipStream_t s = ftmi_hs(stream);
  const int nchunks = (B + NB - 1) / NB;
  const int64_t wsb = ftmi_rnn_workspace_bytes(B, H, cell);
  hipError_t e = hipMemsetAsync(sync, 0, (size_t)wsb, s);
  if (e != hipSuccess) return (int)e;
  RnnParams p = {};
  p.xp = xp;
  p.xp_stride = xp_stride;
  p.T_src = T_src;
  p.index = index;
  p.xp_zero = xp_zero;
  p.w_hh = w_hh;
  p.b_hh = b_hh;
  p.y = y;
  p.y_stride = y_stride;
  p.lengths = lengths;
  p.pad_value = pad_value;
  p.B = B;
  p.T = T;
  p.nrows_hx = nchunks * NB;
  p.cnt = (unsigned *)sync;
  p.err = (unsigned *)sync + 2 * nchunks * CNT_PAD;
  p.hx = (float *)((unsigned *)sync + (2 * nchunks + 1) * CNT_PAD);
  const int maxb = device_cu_count();
  if (cell == 0 && H == 64) return launch_rnn<0, 64, 64>(p, nchunks, maxb, s);
  if (cell == 0 && H == 128) return launch_rnn<0, 128, 128>(p, nchunks, maxb, s);
  if (cell == 0 && H == 256) return launch_rnn<0, 256, 16>(p, nchunks, maxb, s);
  if (cell == 1 && H == 512) return launch_rnn<1, 512, 16>(p, nchunks, maxb, s);
  return FTMI_E_UNSUPPORTED;
}

extern "C" int64_t ftmi_rnn_error_offset(int32_t B) {
  const int64_t nchunks = (B + NB - 1) / NB;
  return 2 * nchunks * CNT_PAD * (int64_t)sizeof(unsigned);
}

#ifdef FTMI_RNN_STAMPS
extern "C" int ftmi_debug_rnn_stamps(unsigned long long *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ftmi_rnn_stamps),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif
