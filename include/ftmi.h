/*
 * ftmi.h — C ABI of libftmi.so, the MI355X (gfx950) hot path of ForwardTacotron
 * inference (reference: tarepan/ForwardTacotron, models/forward_tacotron.py).
 *
 * Every entry point:
 *   - works on CALLER-OWNED device buffers (plain pointers + sizes, fp32 unless stated);
 *   - enqueues on the given HIP stream (ftmi_stream_t = hipStream_t, NULL = null stream)
 *     and never synchronises, allocates or frees;
 *   - returns 0 on success, an FTMI_E_* code (>= 1000) for argument / shape errors
 *     detected on the host, or a hipError_t (< 1000) if a launch failed.
 *
 * Layout convention: sequences are CHANNELS-LAST, (B, T, C) rows of C floats with a
 * row stride given in floats. The reference's (B, C, T) tensors are produced only at
 * the API edge (mel / mel_post outputs) through the transposed-store option.
 *
 * Each function names the reference code it replaces (file:line in the reference).
 */
#ifndef FTMI_H
#define FTMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *ftmi_stream_t; /* hipStream_t */

enum {
  FTMI_OK = 0,
  FTMI_E_ARG = 1001,         /* null pointer / non-positive size */
  FTMI_E_SHAPE = 1002,       /* shape constraint violated (e.g. Cin % 16 != 0) */
  FTMI_E_UNSUPPORTED = 1003, /* configuration without a compiled kernel */
  FTMI_E_ALIGN = 1004        /* pointer / stride not 16-byte aligned */
};

/* Matrix-core path of the dense contractions (conv1d / conv_bank / highway):
 *   FTMI_MMA_F32     v_mfma_f32_32x32x2_f32: exact fp32 products, 157 TFLOP/s peak.
 *   FTMI_MMA_BF16X6  each fp32 operand split into three bf16 pieces (a = a1+a2+a3, exact),
 *                    the six cross products with i+j <= 4 on v_mfma_f32_16x16x32_bf16 with
 *                    fp32 accumulation: fp32-accurate (dropped terms < 2^-24 relative) at
 *                    16/6 of the fp32 MFMA rate.
 *   FTMI_MMA_F16X3   (default) each operand split into an f16 head and a 2^11-scaled f16
 *                    tail; weights pre-split by ftmi_split_weights_f16 (three f16 planes
 *                    + a power-of-two column scale); three v_mfma_f32_16x16x32_f16 per
 *                    product, fp32 accumulation: fp32-level accuracy (dropped terms
 *                    < 2^-22 relative) at 16/3 of the fp32 MFMA rate.  Activations must
 *                    stay below 65504 in magnitude: otherwise the output is invalid and
 *                    bit 0 of *status (optional) is set — recompute on FTMI_MMA_F32. */
enum { FTMI_MMA_F32 = 0, FTMI_MMA_BF16X6 = 1, FTMI_MMA_F16X3 = 2 };

/* Bits of the optional device status word (uint32_t *status) the kernels OR into; the
 * caller zeroes it, runs, and reads it once after the stream completed:
 *   FTMI_STATUS_F16_RANGE    an f16x3 GEMM saw an activation beyond the f16 range (its
 *                            output is invalid: recompute on FTMI_MMA_F32)
 *   FTMI_STATUS_WHH_RANGE    a recurrence's W_hh entry is beyond the f16 range (idem)
 *   FTMI_STATUS_RNN_TIMEOUT  a recurrence workgroup gave up waiting for its group (not all
 *                            workgroups co-resident): the output is invalid — an error,
 *                            not a precision event */
enum { FTMI_STATUS_F16_RANGE = 1, FTMI_STATUS_WHH_RANGE = 2, FTMI_STATUS_RNN_TIMEOUT = 4 };

/* ftmi_conv_bank_split pool_out flags (ABI 10; 0 / 1 keep their ABI 9 meaning) */
enum { FTMI_BANK_POOL = 1,    /* y = CBHG maxpool(2, 1) of the bank output */
       FTMI_BANK_Y_SPLIT = 2, /* with FTMI_BANK_POOL: y as f16x3 split rows of K*Cout */
       FTMI_BANK_X_SPLIT = 4, /* x given as f16x3 split rows of Cin (FTMI_MMA_F16X3) */
       FTMI_BANK_HALVES = 16, /* ABI 15 (alone, FTMI_MMA_F16X3): the few-row bank in ONE
                                 launch — a block per (group pair, 16-column set, half of the
                                 input channels), each wave's weight stream issued at once, the
                                 unit's two halves combined in-kernel by the last to arrive
                                 (deterministic).  B*T <= 128, Cin % 64 == 0, Cin <= 256, K even,
                                 (K / 2)(Cout / 16) % 8 == 0 and <= 512; else FTMI_E_UNSUPPORTED.  split_ws:
                                 ftmi_conv_bank_halves_ws_floats(B, T, K, Cout) floats, the first
                                 FTMI_BANK_COUNTERS zeroed once by the caller (every launch leaves
                                 them zero); split_k is ignored.  One workspace per stream. */
       FTMI_BANK_IMAGE = 32   /* ABI 16, with FTMI_BANK_HALVES: w_split is the bank's
                                 stream-order weight image (ftmi_conv_bank_halves_image), which
                                 the kernel reads as one contiguous 1 KB run per wave load;
                                 same results bit for bit. */ };
enum { FTMI_BANK_COUNTERS = 4096 };

/* ABI version; bumped on any signature change (14: ftmi_panel_proj_qkv, ftmi_attention_kv;
 * 15: FTMI_BANK_HALVES, ftmi_conv_bank_halves_ws_floats; 16: FTMI_BANK_IMAGE,
 * ftmi_conv_bank_halves_image[_bytes]; 17: FTMI_BANK_PAIR, ftmi_conv_args.x_plane / x_fin;
 * 18: rejected variants removed — FTMI_BANK_LAST, FTMI_BANK_PAIR, ftmi_conv_args.x_plane /
 * x_fin, ftmi_gru_bidir_fused; ftmi_highway_stack_spread[_ws_bytes|_blocks] added;
 * 19: ftmi_nnls_lbfgsb_*, ftmi_set_resident_cu_limit, the persistent-launch guard,
 * ftmi_griffinlim_iter, ftmi_istft_fused). */
int ftmi_abi_version(void);
/* sha256 (hex) of the sources this library was built from (the .hip and .h files of
 * forwardtacotron_amd/csrc and include/ftmi.h): the Python binding refuses a library whose
 * id differs from the sources next to it (a stale prebuilt binary). */
const char *ftmi_build_id(void);
/* Static string for an error code (FTMI_E_* or hipError_t). */
const char *ftmi_strerror(int code);
/* Persistent kernels (ftmi_rnn_bidir, ftmi_highway_stack_spread, ftmi_wavernn) hold every
 * workgroup of their grid resident while they wait on each other: each checks, before it
 * launches anything, that the kernel's occupancy times the CU count covers its grid, and
 * returns FTMI_E_UNSUPPORTED otherwise (ABI 19).  This sets the CU count the check assumes
 * (0 = the device's; a test hook for the refusal path); returns the previous setting. */
int32_t ftmi_set_resident_cu_limit(int32_t cus);

/* ------------------------------------------------------------------------------------
 * Embedding gather.  out[n, :] = table[ids[n], :]
 * Replaces nn.Embedding forward: models/forward_tacotron.py:125,304 and the predictor
 * embeddings :31,47.  Ids outside [0, num_rows) produce a zero row and set *err = 1
 * (the reference raises IndexError); err may be NULL.
 * ---------------------------------------------------------------------------------- */
int ftmi_embedding(const int64_t *ids, int64_t n, const float *table, int64_t num_rows,
                   int64_t dim, float *out, int32_t *err, ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Fused Conv1d (implicit GEMM on fp32 MFMA) over channels-last sequences.
 *   acc[b,t,n] = sum_{j<k} sum_c w[n, j*Cin + c] * xin[b, t + j - pad, c]   (zero outside [0,T))
 *   for t in [0, T_out)
 *   v = acc (+ bias[n]) ; relu? max(v,0) ; bn? v*bn_scale[n] + bn_shift[n] ; (+ residual)
 *   xin[b,t,:] = x[b,t,:]                              if maxpool == 0
 *              = max(x[b,t-1,:], x[b,t,:]) (t>0), x[b,0,:] (t==0)   if maxpool == 1
 * Replaces BatchNormConv (models/forward_tacotron.py:58-71, models/common_layers.py:38-52),
 * the CBHG maxpool+projections+residual (common_layers.py:100-109), nn.Linear layers
 * (k = 1: pre_highway :113, lin / post_proj forward_tacotron.py:322,326, RNN input
 * projections).  w is packed [N][k*Cin] (tap-major K).  Requires Cin % 16 == 0 and
 * 16-byte aligned x / w / y with strides % 4 == 0.  yt (optional) receives the same
 * values transposed to (B, N, T) — the reference's mel layout.
 * ---------------------------------------------------------------------------------- */
typedef struct ftmi_conv_args {
  const float *x;
  int64_t x_stride; /* floats between consecutive (b,t) rows of x */
  int32_t B, T, Cin;
  const float *w; /* [N][k*Cin] */
  int32_t N, k, pad;
  const float *bias;     /* [N] or NULL */
  int32_t relu;          /* 0 / 1 */
  const float *bn_scale; /* [N] or NULL (BN eval folded: gamma / sqrt(var + eps)) */
  const float *bn_shift; /* [N] (beta - mean * scale) */
  int32_t maxpool;       /* 0 / 1 */
  const float *residual; /* (B,T,N) rows with res_stride, or NULL */
  int64_t res_stride;
  float *y; /* (B,T,N) rows with y_stride, or NULL if only yt is wanted */
  int64_t y_stride;
  float *yt; /* (B,N,T_out) or NULL */
  int32_t T_out; /* output frames per sequence, 0 = T (even k in PyTorch gives T+1) */
  int32_t mma;   /* matrix path: FTMI_MMA_F32, FTMI_MMA_BF16X6 or FTMI_MMA_F16X3 */
  int32_t split_k;  /* > 1: split K over that many workgroups (FTMI_MMA_BF16X6 / F16X3);
                       partial sums go to split_ws and a second launch sums them in fixed
                       order (deterministic) and applies the epilogue */
  float *split_ws;  /* split_k * B*T_out * N floats of caller-owned workspace, or NULL */
  const void *w_split; /* FTMI_MMA_BF16X6: optional ftmi_split_weights pieces (skips the
                          per-call weight split); FTMI_MMA_F16X3: REQUIRED
                          ftmi_split_weights_f16 planes */
  uint32_t *status;    /* optional device word: bit 0 set on f16 range overflow (F16X3) */
  int32_t x_split;     /* ABI 10: x holds f16x3 SPLIT ROWS (below) instead of floats; only
                          FTMI_MMA_F16X3 without maxpool on the slab kernel (B*T_out > 256
                          rows), else FTMI_E_UNSUPPORTED.  x_stride (floats) >= Cin. */
} ftmi_conv_args;

/* f16x3 split rows (ABI 10): the activation layout one f16x3 GEMM hands the next.  Row r
 * of a (rows, C) operand with row stride S floats holds, as halves, C heads h = f16(v) then
 * C scaled tails t = f16((v - h) * 2^11) (v = h + 2^-11 t to ~2^-22 relative): the same 4
 * bytes per element as fp32, the split done once by the producer instead of by every
 * column tile of every consumer, which also checks the f16 range (status bit 0). */

/* Split fp32 weights [N][K] once into three bf16 pieces (w = p0 + p1 + p2 exactly), laid
 * out [3][N][Kpad], Kpad = roundup(K, 32), zero padded; out must hold
 * ftmi_split_weights_bytes(N, K) bytes (16-byte aligned). */
int64_t ftmi_split_weights_bytes(int64_t N, int64_t K);
int ftmi_split_weights(const float *w, int64_t N, int64_t K, void *out, ftmi_stream_t stream);

/* Split fp32 weights [N][K] once for FTMI_MMA_F16X3: per row n a power-of-two scale
 * s_n = 2^-e (smallest e >= 0 with max|w[n]| s_n < 16), h = f16(w s_n),
 * t = f16((w s_n - h) * 2^11); layout: f16 planes [3][N][Kpad] = (2^11 h, t, h), Kpad =
 * roundup(K, 32), zero padded, then float colscale[N] = 2^-11 / s_n.  out must hold
 * ftmi_split_weights_f16_bytes(N, K) bytes (16-byte aligned).  The conv bank's w_split
 * is each group's block back to back. */
int64_t ftmi_split_weights_f16_bytes(int64_t N, int64_t K);
int ftmi_split_weights_f16(const float *w, int64_t N, int64_t K, void *out,
                           ftmi_stream_t stream);

int ftmi_conv1d(const ftmi_conv_args *args, ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * CBHG convolution bank: K BatchNormConvs with kernel sizes 1..K (pad k//2, ReLU then
 * BN, output sliced to T), concatenated on channels (common_layers.py:67-71,92-97).
 *   y[b,t, g*Cout + n] = BN_g(relu(sum_{j<=g} sum_c w_g[n, j*Cin+c] * x[b, t+j-(g+1)/2, c]))
 * w: the K packed weights back to back, group g is [Cout][(g+1)*Cin] starting at float
 * offset Cout*Cin*g*(g+1)/2.  bn_scale / bn_shift: [K*Cout].  y: (B,T,K*Cout) rows.
 * w_split: each group's ftmi_split_weights (BF16X6, optional) or ftmi_split_weights_f16
 * (F16X3, required) block back to back.  status: as in ftmi_conv_args.
 * ---------------------------------------------------------------------------------- */
int ftmi_conv_bank(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t Cin,
                   const float *w, const void *w_split, int32_t K, int32_t Cout,
                   const float *bn_scale,
                   const float *bn_shift, float *y, int64_t y_stride, int32_t mma,
                   uint32_t *status, ftmi_stream_t stream);

/* ftmi_conv_bank with a channel split (ABI 6): when B*T <= 256 and mma == FTMI_MMA_F16X3
 * the bank runs on the weight-streaming "skinny" kernel (B = 1 generation, BASELINE config
 * c2), whose blocks take ceil(ceil(Cin/32) / split_k) <= 2 channel chunks each and leave
 * raw partial sums in split_ws (split_k * B*T * K*Cout floats, caller-owned), summed in split
 * order by a finishing launch (deterministic).  split_k <= 1 / split_ws NULL: as
 * ftmi_conv_bank.  Other shapes ignore the split.  ftmi_conv1d takes the same kernel for
 * B*T_out <= 256 (its split_k / split_ws as documented there).
 * pool_out (ABI 9, flags since ABI 10): FTMI_BANK_POOL — y receives the CBHG maxpool(2, 1)
 * of the bank output (common_layers.py:73,100: y[t] = max(bank[t - 1], bank[t]) within each
 * sequence, y[0] = bank[0]) — the input proj1 then reads with ftmi_conv_args.maxpool = 0;
 * only on the f16x3 slab kernel (mma = FTMI_MMA_F16X3, B*T > 256 rows, no split), elsewhere
 * FTMI_E_UNSUPPORTED.  | FTMI_BANK_Y_SPLIT: y as split rows (proj1 then reads them with
 * ftmi_conv_args.x_split = 1).  FTMI_BANK_X_SPLIT: x is given as split rows. */
/* Floats of the FTMI_BANK_HALVES workspace (counters included) for a bank of B*T <= 128
 * rows, K groups of Cout columns; 0 for other sizes. */
int64_t ftmi_conv_bank_halves_ws_floats(int32_t B, int32_t T, int32_t K, int32_t Cout);
/* Bytes of the FTMI_BANK_IMAGE weight image of a bank (Cin input channels, K groups of Cout
 * columns; any B*T); 0 for shapes FTMI_BANK_HALVES refuses. */
int64_t ftmi_conv_bank_halves_image_bytes(int32_t Cin, int32_t K, int32_t Cout);
/* Builds that image (16-B aligned, ftmi_conv_bank_halves_image_bytes bytes) from the bank's
 * f16x3 split blocks (the FTMI_MMA_F16X3 w_split of ftmi_conv_bank_split); stream-ordered.
 * Once per weights version: it replaces `w_split` (a prepared layout like the split blocks
 * themselves, models/common_layers.py:68-71's bank weights reordered, not recomputed). */
int ftmi_conv_bank_halves_image(const void *w_split, int32_t Cin, int32_t K, int32_t Cout,
                                void *image, ftmi_stream_t stream);
int ftmi_conv_bank_split(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t Cin,
                         const float *w, const void *w_split, int32_t K, int32_t Cout,
                         const float *bn_scale, const float *bn_shift, float *y,
                         int64_t y_stride, int32_t mma, uint32_t *status, int32_t split_k,
                         float *split_ws, int32_t pool_out, ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * One highway layer (common_layers.py:22-35):
 *   g = sigmoid(x W2^T + b2);  y = g * relu(x W1^T + b1) + (1 - g) * x
 * w12: [2C][C] with rows interleaved in blocks of 32: rows 64q..64q+31 = W1 rows
 * 32q..32q+31, rows 64q+32..64q+63 = W2 rows 32q..32q+31.  Requires C % 32 == 0.
 * w12_split: ftmi_split_weights (BF16X6, optional) / ftmi_split_weights_f16 (F16X3,
 * required) of w12.  status: as in ftmi_conv_args.  y must not alias x.
 * ---------------------------------------------------------------------------------- */
int ftmi_highway(const float *x, int64_t x_stride, int64_t M, int32_t C, const float *w12,
                 const void *w12_split, const float *b1, const float *b2, float *y,
                 int64_t y_stride, int32_t mma, uint32_t *status, ftmi_stream_t stream);

/* ftmi_highway with a channel split (ABI 6): split_k >= 1 with M <= 1024 rows and
 * mma == FTMI_MMA_F16X3 runs the weight-streaming skinny kernel, whose blocks leave raw
 * partial sums of x [W1|W2]^T in split_ws (split_k * M * 2C floats, caller-owned) and a
 * finishing launch sums them in split order and applies the gating (deterministic).
 * split_k = 0 / other shapes: as ftmi_highway. */
int ftmi_highway_split(const float *x, int64_t x_stride, int64_t M, int32_t C,
                       const float *w12, const void *w12_split, const float *b1,
                       const float *b2, float *y, int64_t y_stride, int32_t mma,
                       uint32_t *status, int32_t split_k, float *split_ws,
                       ftmi_stream_t stream);

/* CBHG highway stack in one launch (ABI 9; common_layers.py:110-115 + the GRU's input
 * projection): h = x W_pre^T (pre_highway, no bias), then L highway layers as ftmi_highway,
 * then y = h W_out^T + b_out.  Activations stay on chip between layers; the result is
 * bit-identical to the unfused ftmi_conv1d / ftmi_highway chain on FTMI_MMA_F16X3.
 *   x: M rows of Cp floats (Cp % 4 == 0, Cp <= C), C == 256 (the CBHG channels)
 * Every weight operand is an ftmi_split_weights_f16_FRAG block (fragment-major planes):
 *   w_pre_split: of W_pre [C][Cp]
 *   w_hw_split[l], b1[l], b2[l]: host arrays of L (<= 8) device pointers — the block of
 *     each highway's packed w12 [2C][C] and its biases
 *   w_out_split: of W_out [n_out][C] (n_out % 512 == 0) and b_out
 *     (nullable) -> y (M x n_out, row stride y_stride); NULL with n_out = 0, y = NULL: none
 *   h: optional (nullable) copy of the last highway's output (M x C, row stride h_stride)
 * status: bit 0 when an activation is beyond the f16 range (rerun on the unfused exact path).
 * ---------------------------------------------------------------------------------- */
/* ftmi_split_weights_f16 with the planes in the fragment-major order of the 16x16x32 f16
 * MFMA B operand, [N/16][Kpad/32][64][8] (lane = n % 16 + 16 ((k / 8) % 4), element k % 8;
 * ABI 9): same byte size (ftmi_split_weights_f16_bytes), N % 16 == 0. */
int ftmi_split_weights_f16_frag(const float *w, int64_t N, int64_t K, void *out,
                                ftmi_stream_t stream);

/* fp32 rows (rows, C) -> f16x3 split rows (ABI 10; the operand of ftmi_conv_args.x_split /
 * FTMI_BANK_X_SPLIT) for an activation that is also needed in fp32 (a CBHG input is its
 * residual too).  Sets status bit 0 (optional word) if |x| > 65504.  C % 4 == 0, strides in
 * floats >= C, 16-B aligned, y must not alias x. */
int ftmi_split_rows(const float *x, int64_t x_stride, int64_t rows, int32_t C, float *y,
                    int64_t y_stride, uint32_t *status, ftmi_stream_t stream);

int ftmi_highway_stack(const float *x, int64_t x_stride, int64_t M, int32_t Cp, int32_t C,
                       const void *w_pre_split, int32_t L, const void *const *w_hw_split,
                       const float *const *b1, const float *const *b2,
                       const void *w_out_split, const float *b_out, int32_t n_out, float *y,
                       int64_t y_stride, float *h, int64_t h_stride, uint32_t *status,
                       ftmi_stream_t stream);

/* The same CBHG tail for few rows (ABI 18; batch-1 generation, BASELINE config c2: the
 * prenet's 120 and the postnet's 816 rows), spread over the chip: each 64-row block over 16
 * workgroups that own 16 channels of every layer (and n_out / 16 output columns) and exchange
 * the layers' activations through `ws` — bit-identical to ftmi_highway_stack.  M <= 1024,
 * n_out <= 1536, and the ftmi_highway_stack_spread_blocks(M) workgroups must all be resident
 * at once (<= the CU count; they wait on each other: run it where no other persistent kernel
 * holds the CUs it needs), else FTMI_E_UNSUPPORTED.  ws: 16-B aligned device workspace of
 * ftmi_highway_stack_spread_ws_bytes(M) bytes, one per stream (its counters are zeroed by
 * the call).  A workgroup that waits past its spin bound sets FTMI_STATUS_RNN_TIMEOUT.
 * Replaces common_layers.py:110-118 (pre_highway, highways, the GRU's input GEMM). */
int64_t ftmi_highway_stack_spread_ws_bytes(int64_t M);
int32_t ftmi_highway_stack_spread_blocks(int64_t M);
int ftmi_highway_stack_spread(const float *x, int64_t x_stride, int64_t M, int32_t Cp,
                              int32_t C, const void *w_pre_split, int32_t L,
                              const void *const *w_hw_split, const float *const *b1,
                              const float *const *b2, const void *w_out_split,
                              const float *b_out, int32_t n_out, float *y, int64_t y_stride,
                              float *h, int64_t h_stride, uint32_t *status, void *ws,
                              ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Bidirectional single-layer GRU / LSTM recurrence, PyTorch semantics, h0 = c0 = 0,
 * both directions over the full padded length (no packing), output [fwd | bwd].
 *   GRU  (cell = 0, gates r,z,n): common_layers.py:84,118 and forward_tacotron.py:39,53
 *   LSTM (cell = 1, gates i,f,g,o): forward_tacotron.py:165-168,321
 * xp: precomputed input projections, rows of 2*G*H floats ([dir][gate][unit]), already
 *     including b_ih (GRU) or b_ih + b_hh (LSTM); row for (b, t) is
 *       xp + (b*T_src + src)*xp_stride,  src = t if index == NULL else index[b*T + t];
 *     src < 0 selects xp_zero (the projection of a zero input row: the biases), 2*G*H.
 *     (index = LengthRegulator map: the LSTM reads phoneme-rate projections directly.)
 * w_hh: [2][G*H][H] (PyTorch weight_hh_l0 then weight_hh_l0_reverse).
 * b_hh: [2][G*H] for GRU (added inside the recurrence), ignored (may be NULL) for LSTM.
 * lengths: int32 [B] or NULL.  Packed-sequence semantics (pack_padded_sequence +
 *     pad_packed_sequence, forward_tacotron.py:224-230): frames t >= lengths[b] output
 *     pad_value and the reverse direction starts from h = c = 0 at t = lengths[b]-1.
 * y:    (B, T, 2H) rows with y_stride.
 * mma:  matrix path of W_hh h: FTMI_MMA_F16X3 (default; W_hh split in-kernel, bit 1 of
 *     *status set if an entry exceeds the f16 range — rerun with FTMI_MMA_BF16X6),
 *     FTMI_MMA_BF16X6 or FTMI_MMA_F32.  status: optional device word.  ABI 12: OR
 *     FTMI_RNN_SPREAD into mma to let the call spread a small-H recurrence over the whole
 *     device (fewer sequences per workgroup group: lower step latency, more workgroups —
 *     for a recurrence that runs alone; ftmi_rnn_blocks takes the same flag).
 * sync: 16-byte aligned device workspace of ftmi_rnn_workspace_bytes() bytes (zeroed by
 *     the call; holds the arrival counters and the h exchange buffer).  After the stream
 *     has completed, the 32-bit word at byte offset ftmi_rnn_error_offset() is non-zero if
 *     a workgroup timed out waiting for its group (not all workgroups resident); the same
 *     event sets FTMI_STATUS_RNN_TIMEOUT in *status.
 * Supported H: GRU 64, 128, 256; LSTM 512 (the ForwardTacotron config).
 * ---------------------------------------------------------------------------------- */
enum { FTMI_RNN_SPREAD = 0x100 };
int64_t ftmi_rnn_workspace_bytes(int32_t B, int32_t H, int32_t cell);
int64_t ftmi_rnn_error_offset(int32_t B);
/* Workgroups the (first) launch of ftmi_rnn_bidir(cell, B, H, mma) occupies: each is
 * persistent (one per CU) and waits on the others, so recurrences issued concurrently on
 * several streams must not exceed the CU count together (the host serialises them
 * otherwise).  0 for an unsupported shape. */
int32_t ftmi_rnn_blocks(int32_t cell, int32_t B, int32_t H, int32_t mma);
/* Test / diagnostic hook: bound of every recurrence spin (polls per wait) for launches
 * issued after the call; 0 restores the default (2^22).  Returns the previous bound. */
uint32_t ftmi_set_rnn_spin_limit(uint32_t limit);
int ftmi_rnn_bidir(int32_t cell, int32_t B, int32_t T, int32_t H, const float *xp,
                   int64_t xp_stride, int32_t T_src, const int32_t *index,
                   const float *xp_zero, const float *w_hh, const float *b_hh,
                   const int32_t *lengths, float pad_value, float *y, int64_t y_stride,
                   int32_t mma, uint32_t *status, void *sync, ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Duration post-processing of ForwardTacotron.generate + LengthRegulator counts:
 *   if sum_{b,t} trunc_int64(dur) <= 0: dur[:] = fill_value   (forward_tacotron.py:254-255,
 *                                                               only when apply_fill != 0)
 *   dur[dur < 0] = 0                    (in place, common_layers.py:13)
 *   count = int64(trunc(fp32(dur + 0.5)))  (common_layers.py:16)
 *   offsets[b, 0..T] = exclusive prefix sum of counts; totals[b] = offsets[b, T]
 * Single launch, bit-exact. offsets: int32 [B][T+1]; totals: int32 [B];
 * fill_flag (optional int32[1]) receives 1 if the fill rule fired.
 * ---------------------------------------------------------------------------------- */
int ftmi_duration_counts(float *dur, int32_t B, int32_t T, int32_t apply_fill,
                         float fill_value, int32_t *offsets, int32_t *totals,
                         int32_t *fill_flag, ftmi_stream_t stream);

/* Batch-sharded form of the fill-2 rule: the reference decides on the sum
 * over the WHOLE batch, so each shard computes its partial sum (ftmi_duration_trunc_sum:
 * out[0] = sum_{b,t} trunc_int64(dur)), the host all-reduces it (RCCL SUM, device int64),
 * and ftmi_duration_counts_global applies the rule with that global sum, then clips /
 * counts / scans exactly like ftmi_duration_counts. */
int ftmi_duration_trunc_sum(const float *dur, int32_t B, int32_t T, int64_t *out,
                            ftmi_stream_t stream);
int ftmi_duration_counts_global(float *dur, int32_t B, int32_t T, const int64_t *global_sum,
                                float fill_value, int32_t *offsets, int32_t *totals,
                                int32_t *fill_flag, ftmi_stream_t stream);

/* Frame -> phoneme index map of the LengthRegulator: index[b, f] = t such that
 * offsets[b,t] <= f < offsets[b,t+1], or -1 for f >= totals[b] (zero padding,
 * pad_sequence in common_layers.py:18).  index: int32 [B][T_mel]. */
int ftmi_lr_index(const int32_t *offsets, int32_t B, int32_t T, int32_t T_mel,
                  int32_t *index, ftmi_stream_t stream);

/* LengthRegulator expansion (common_layers.py:12-19): y[b,f,:] = x[b,index[b,f],:] or 0. */
int ftmi_length_regulate(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t C,
                         const int32_t *index, int32_t T_mel, float *y, int64_t y_stride,
                         ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Pitch / energy conditioning (forward_tacotron.py:308-314):
 *   x[b,t,c] = (x[b,t,c] + P[b,t,c] * pitch_strength) + E[b,t,c] * energy_strength
 *   P = Conv1d(1 -> C, k=3, pad=1, bias)(pitch[b,:]) at t (same for E with energy).
 * pitch / energy: (B, T) contiguous. wp / we: [C][3]; bp / be: [C].
 * ---------------------------------------------------------------------------------- */
int ftmi_series_proj_add(float *x, int64_t x_stride, int32_t B, int32_t T, int32_t C,
                         const float *pitch, const float *wp, const float *bp,
                         float pitch_strength, const float *energy, const float *we,
                         const float *be, float energy_strength, ftmi_stream_t stream);

/* ------------------------------------------------------------------------------------
 * SeriesPredictor head (forward_tacotron.py:41,54-55): out[m] = (x[m,:] . w + bias[0]) / alpha
 * x: M rows of C floats (row stride x_stride); bias: device float[1] or NULL; out: M floats.
 * ---------------------------------------------------------------------------------- */
int ftmi_rowdot(const float *x, int64_t x_stride, int64_t M, int32_t C, const float *w,
                const float *bias, float alpha, float *out, ftmi_stream_t stream);

/* ====================================================================================
 * Audio path: utils/dsp.py (DSP.wav_to_mel :71-87, griffinlim :89-103), whose arithmetic
 * is librosa 0.7.2 (requirements.txt:2): core.stft / core.istft / filters.mel /
 * util.nnls / core.griffinlim.  Plans (host-built once per DSP config, device buffers):
 *   window  double[n_fft]     periodic Hann of win_length, zero-padded to n_fft (centred)
 *   win_sq  double[n_fft]     window**2 (window_sumsquare's envelope)
 *   twiddle double[n_fft][2]  exp(-2 pi i k / n_fft), k < n_fft / 2
 * n_fft: power of two in [16, 4096].  center=True, pad_mode='reflect' throughout.
 * Spectra are FRAME-major complex64 (B, F, n_fft/2+1) (interleaved re, im floats); mel
 * is (B, n_mels, F).  `lengths` (samples) / `frames` (frames) are optional device int32
 * per-item limits (NULL: L / F for every item); frames past an item's count are skipped.
 * ==================================================================================== */

/* complex STFT (librosa core.stft: rfft(window * frame) in fp64, stored complex64) of
 * audio rows y (B, L) with row stride y_stride; F = 1 + L // hop frames. */
int ftmi_stft(const float *y, int64_t y_stride, int32_t B, int64_t L, const int32_t *lengths,
              int32_t n_fft, int32_t hop, const double *window, const void *twiddle, int32_t F,
              const int32_t *frames, void *X, ftmi_stream_t stream);

/* DSP.wav_to_mel (utils/dsp.py:71-87): mel[b,i,f] = sum_k basis[i,k] |STFT|[b,f,k]
 * (fp64 accumulation over the row support [mel_lo[i], mel_hi[i]) of basis [n_mels][nb]),
 * then log(max(., 1e-5)) when log_norm (DSP.normalize :105-107). */
int ftmi_mel_spectrogram(const float *y, int64_t y_stride, int32_t B, int64_t L,
                         const int32_t *lengths, int32_t n_fft, int32_t hop, const double *window,
                         const void *twiddle, int32_t F, const int32_t *frames, const float *basis,
                         const int32_t *mel_lo, const int32_t *mel_hi, int32_t n_mels,
                         int32_t log_norm, float *mel, ftmi_stream_t stream);

/* One fast Griffin-Lim analysis step (librosa core.griffinlim loop body): rebuilt =
 * STFT(y); angles = rebuilt - c * tprev (first: rebuilt); angles /= |angles| + 1e-16;
 * X = S * angles (next synthesis input); tprev = rebuilt.  S: (B, F, nb) float32;
 * tprev, X: (B, F, nb) complex64.  c = momentum / (1 + momentum). */
int ftmi_griffinlim_stft(const float *y, int64_t y_stride, int32_t B, int64_t L,
                         const int32_t *lengths, int32_t n_fft, int32_t hop, const double *window,
                         const void *twiddle, int32_t F, const int32_t *frames, const float *S,
                         void *tprev, float c, int32_t first, void *X, ftmi_stream_t stream);

/* X = S * angles elementwise (complex64 = float32 * complex64, numpy rounding): the
 * Griffin-Lim synthesis input for the initial phases.  n = number of bins in total. */
int ftmi_spec_mul(const float *S, const void *angles, int64_t n, void *X, ftmi_stream_t stream);

/* Griffin-Lim's random initial phases (librosa 0.7.2 core.griffinlim:
 * np.exp(2j * np.pi * np.random.rand(n_bins, T))) from the host's uniform draws u (B, n_bins,
 * T) float64, bin-major as numpy draws them: angles (B, T, n_bins) complex64, frame-major
 * (float64 cos / sin, rounded to complex64).  ABI 11. */
int ftmi_unit_phases(const double *u, int32_t B, int32_t n_bins, int32_t T, void *angles,
                     ftmi_stream_t stream);

/* librosa core.istft (center=True): per-frame fp64 irfft * window, overlap-added in frame
 * order with float32 rounding, divided by the window sum-square where > FLT_MIN, cropped
 * by n_fft/2.  Item b yields hop * (frames_b - 1) samples into y[b, :], zero-filled up to
 * y_len.  work: ftmi_istft_workspace_bytes(B, F, n_fft) bytes. */
int64_t ftmi_istft_workspace_bytes(int32_t B, int32_t F, int32_t n_fft);
int ftmi_istft(const void *X, int32_t B, int32_t F, const int32_t *frames, int32_t n_fft,
               int32_t hop, const double *window, const double *win_sq, const void *twiddle,
               void *work, float *y, int64_t y_stride, int64_t y_len, ftmi_stream_t stream);

/* One fast Griffin-Lim iteration in ONE launch (ABI 19; librosa 0.7.2 core.griffinlim loop
 * body, utils/dsp.py:91-102): rebuilt = stft(istft(Xin)); angles = rebuilt - c * tprev
 * (first: rebuilt); angles /= |angles| + 1e-16; Xout = S * angles; tprev = rebuilt — the
 * ISTFT (fp64 irfft, float32 overlap-add in frame order, window sum-square division,
 * center crop) and the STFT (reflect padding) of ftmi_istft / ftmi_griffinlim_stft, fused
 * per tile of 16 frames with the audio kept on chip.  Xin != Xout (neighbouring tiles read
 * Xin's halo frames); spectra (B, F, n_fft/2+1) complex64 frame-major, item b's first
 * frames[b] frames (NULL: F).  n_fft = 1024, hop = 256 only (else FTMI_E_UNSUPPORTED).
 * window / win_sq: [n_fft] float64, twiddle: [n_fft/2] complex128 (the ftmi_stft plan). */
int ftmi_griffinlim_iter(const void *Xin, void *Xout, const float *S, void *tprev, int32_t B,
                         int32_t F, const int32_t *frames, int32_t n_fft, int32_t hop,
                         const double *window, const double *win_sq, const void *twiddle,
                         float c, int32_t first, ftmi_stream_t stream);
/* ftmi_istft in one launch, no workspace (ABI 19; same sizes as ftmi_griffinlim_iter). */
int ftmi_istft_fused(const void *X, int32_t B, int32_t F, const int32_t *frames, int32_t n_fft,
                     int32_t hop, const double *window, const double *win_sq, const void *twiddle,
                     float *y, int64_t y_stride, int64_t y_len, ftmi_stream_t stream);

/* mel -> linear magnitude (librosa feature.inverse.mel_to_stft, power=1, via util.nnls):
 * per frame min ||A x - m||^2, x >= 0, m = exp(mel) when denorm (DSP.denormalize
 * :109-110).  Solved by FISTA (`iters` steps of 1/L = inv_L) from the clipped
 * minimum-norm solution pinv(A) m.  A is given sparse: row i holds nonzeros
 * rowvals[rowptr[i] .. rowptr[i+1]) for bins rowlo[i] ...; bin k feeds mel rows
 * bin_rows[2k], bin_rows[2k+1] (-1: none) with weights bin_w[2k], bin_w[2k+1]; pinv is
 * [n_bins][n_mels].  nnz = rowptr[n_mels].  S: (B, F, n_bins) float32. */
int ftmi_mel_nnls(const float *mel, int32_t B, int32_t F, const int32_t *frames, int32_t n_mels,
                  int32_t n_bins, int32_t denorm, int32_t nnz, const float *rowvals,
                  const int32_t *rowptr, const int32_t *rowlo, const int32_t *bin_rows,
                  const float *bin_w, const float *pinv, float inv_L, int32_t iters, float *S,
                  ftmi_stream_t stream);

/* The reference's NNLS itself (ABI 19): librosa 0.7.2 util.nnls — scipy fmin_l_bfgs_b
 * (L-BFGS-B 3.0, m = n_bins, pgtol 1e-5, factr 1e7, maxls 20) on blocks of up to
 * `max_frames` frames (127 for n_fft 1024: MAX_MEM_BLOCK // (n_bins * 4)), started from the
 * float32 least-squares solution clipped at 0 — so S is the reference's to rounding, not
 * just another minimiser (librosa/util/utils.py nnls, _nnls_lbfgs_block).
 * blocks: device [n_blocks][4] int32 (item, first frame, frames, 0); groups: workgroups per
 * block for the sweeps (1..64); m: history columns the workspace holds (the reference keeps
 * n_bins; a block that needs more stops with bit 4 in status[0]: rerun with a larger m);
 * pinv: [n_bins][n_mels] float64; active: device int32 the caller sets to n_blocks before
 * ftmi_nnls_lbfgsb_start — each block decrements it when done.  Drive it like scipy's
 * driver loop: start, then ftmi_nnls_lbfgsb_cycles (one cycle advances every block by one
 * L-BFGS-B iteration or one extra line-search evaluation) until *active reads 0, then
 * ftmi_nnls_lbfgsb_finish (writes S (B, F, n_bins), zero past frames[b]; status: device
 * int32[2] the caller zeroes: [0] |= failure bits of any block (2 abnormal line search,
 * 4 history full, 8 > 1024 equal breakpoints), [1] = max iterations; info: NULL or device
 * double[n_blocks][4] = per block (iterations, f evaluations, f, projected-gradient norm)). */
typedef struct {
  const float *mel; /* (B, n_mels, F) */
  int32_t B, F, n_mels, n_bins, denorm;
  const int32_t *blocks;
  int32_t n_blocks, groups, m, max_frames;
  int32_t maxiter;   /* scipy's maxiter (0: its default 15000) */
  int32_t dbg_stop;  /* 0; else stop each block before phase (dbg_stop & 15) of iteration dbg_stop >> 4 */
  const float *rowvals;
  const int32_t *rowptr, *rowlo, *bin_rows;
  const float *bin_w;
  const double *pinv;
  void *workspace; /* ftmi_nnls_lbfgsb_workspace_bytes(n_blocks, n_bins, max_frames, m, groups) */
  float *S;
  int32_t *active;
} ftmi_nnls_lbfgsb_args;
int64_t ftmi_nnls_lbfgsb_workspace_bytes(int32_t n_blocks, int32_t n_bins, int32_t max_frames,
                                         int32_t m, int32_t groups);
int ftmi_nnls_lbfgsb_start(const ftmi_nnls_lbfgsb_args *args, ftmi_stream_t stream);
int ftmi_nnls_lbfgsb_cycles(const ftmi_nnls_lbfgsb_args *args, int32_t cycles,
                            ftmi_stream_t stream);
int ftmi_nnls_lbfgsb_finish(const ftmi_nnls_lbfgsb_args *args, const int32_t *frames,
                            int32_t *status, double *info, ftmi_stream_t stream);

/* ====================================================================================
 * FastPitch transformer (models/fast_pitch.py).  Activations channels-last (B, T, C).
 * ==================================================================================== */

/* nn.Embedding + PositionalEncoding (fast_pitch.py:16-33, eval: dropout is identity):
 * out[b,t,:] = table[ids[b,t],:] + scale[0] * pe[t,:] (float32 multiply, then add).
 * pe: [T_max][dim] rows (the reference buffer (max_len, 1, dim)); scale: device float[1]. */
int ftmi_embedding_posenc(const int64_t *ids, int32_t B, int32_t T, const float *table,
                          int64_t rows, int32_t dim, const float *pe, const float *scale,
                          float *out, int32_t *err, ftmi_stream_t stream);

/* LengthRegulator (common_layers.py:12-19) fused with the postnet's PositionalEncoding:
 * y[b,t,:] = (index[b,t] >= 0 ? x[b,index[b,t],:] : 0) + scale[0] * pe[t,:].
 * x: (B, T, C) rows; index: (B, T_mel) from ftmi_lr_index; y: (B, T_mel, C) rows. */
int ftmi_lr_posenc(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t C,
                   const int32_t *index, int32_t T_mel, const float *pe, const float *scale,
                   float *y, int64_t y_stride, ftmi_stream_t stream);

/* nn.LayerNorm(C) over rows (FFTBlock.norm1/norm2 :64-65, ForwardTransformer.norm :112):
 * biased variance, y = (x*rstd - rstd*mean)*gamma + beta.  C <= 1024; y may alias x. */
int ftmi_layernorm(const float *x, int64_t x_stride, int64_t M, int32_t C, const float *gamma,
                   const float *beta, float eps, float *y, int64_t y_stride, ftmi_stream_t stream);

/* Row-panel projection (ABI 13) — the k = 1 contractions of a FastPitch FFT block
 * (models/fast_pitch.py:56-91: self_attn in_proj, out_proj + residual -> norm1, conv2 with
 * kernel 1 + residual -> norm2) with their epilogue in one launch:
 *   v = x W^T + bias (+ residual);   y = ln_gamma ? LayerNorm(v) : v
 * (nn.LayerNorm over the N columns: biased variance, eps, y = (v*rstd - rstd*mean)*gamma +
 * beta as ftmi_layernorm).  x: M rows of K floats (K % 4 == 0, 16-B aligned, x_stride % 4
 * == 0); w_split_frag: ftmi_split_weights_f16_frag of W [N][K]; N % 256 == 0, N == 256 with
 * LayerNorm; bias, residual (M x N, res_stride), ln_gamma / ln_beta (both or neither):
 * nullable.  y (M x N, y_stride) must not alias x; it may alias residual.  f16x3 arithmetic:
 * the projection values are bit-identical to ftmi_conv1d's on FTMI_MMA_F16X3 with the same
 * planes in row-major order; status bit 0 (optional word) when |x| > 65504 (rerun
 * unfused on FTMI_MMA_F32). */
int ftmi_panel_proj(const float *x, int64_t x_stride, int64_t M, int32_t K,
                    const void *w_split_frag, int32_t N, const float *bias,
                    const float *residual, int64_t res_stride, const float *ln_gamma,
                    const float *ln_beta, float eps, float *y, int64_t y_stride,
                    uint32_t *status, ftmi_stream_t stream);

/* nn.MultiheadAttention self-attention core (FFTBlock.forward :76-79; torch
 * multi_head_attention_forward math path): per batch b and head h,
 *   O = softmax((Q * qscale) K^T + mask) V,  Q/K/V = qkv[b, :, off + h*head_dim ...]
 * from the packed in_proj output rows (row stride row_stride floats; q/k/v column
 * offsets q_off/k_off/v_off).  key_padding_mask: (B, T) bytes, nonzero = padded key
 * (-inf), or NULL.  qscale = float32(sqrt(1/head_dim)).  out: (B, T, H*head_dim) rows of
 * stride out_stride.  head_dim in {64, 128}.  mma (ABI 8): FTMI_MMA_F16X3 (default: both
 * contractions on the f16x3 split, softmax fp32; an operand beyond the f16 range sets
 * FTMI_STATUS_F16_RANGE in *status, optional) or FTMI_MMA_F32 (fp32 MFMA).  workspace
 * (ABI 9, nullable): with >= ftmi_attention_workspace_bytes caller-owned bytes the f16x3
 * path splits K and V once per call into f16 planes there (instead of once per query tile
 * inside the attention kernel); results are identical. */
int64_t ftmi_attention_workspace_bytes(int32_t B, int32_t T, int32_t H, int32_t head_dim);
int ftmi_attention(const float *qkv, int64_t row_stride, int32_t B, int32_t T, int32_t H,
                   int32_t head_dim, int32_t q_off, int32_t k_off, int32_t v_off,
                   const uint8_t *key_padding_mask, float qscale, float *out,
                   int64_t out_stride, int32_t mma, uint32_t *status, void *workspace,
                   int64_t workspace_bytes, ftmi_stream_t stream);

/* ABI 14: the attention split pass folded into the in_proj projection.
 * ftmi_panel_proj_qkv = ftmi_panel_proj of self_attn.in_proj (models/fast_pitch.py:76; W
 * [3d][K], d = 256, no residual / LayerNorm) on B*T rows that writes only the Q third as fp32
 * rows (q_out, q_stride >= d) and K / V into kv_workspace (>= ftmi_attention_workspace_bytes
 * (B, T, heads, d / heads) bytes) as the f16 head / scaled-tail planes ftmi_attention's split
 * pass would write for the same values (K [B*heads][Tp][hd], V [B*heads][hd][Tp], Tp = T
 * rounded up to 64; keys T..Tp-1 are never written: the attention kernels zero them while
 * staging the last key tile, so the workspace may hold anything there — including the
 * non-finite values an earlier, overflowing call stored).
 * ftmi_attention_kv = ftmi_attention (f16x3) with Q rows q (row_stride) and K / V taken from
 * such a workspace: no split pass.  The pair computes exactly what ftmi_panel_proj +
 * ftmi_attention with a workspace compute (bit-identical); |value| > 65504 sets status bit 0. */
int ftmi_panel_proj_qkv(const float *x, int64_t x_stride, int32_t B, int32_t T, int32_t K,
                        const void *w_split_frag, int32_t d, const float *bias, int32_t heads,
                        float *q_out, int64_t q_stride, void *kv_workspace,
                        int64_t workspace_bytes, uint32_t *status, ftmi_stream_t stream);
int ftmi_attention_kv(const float *q, int64_t row_stride, int32_t B, int32_t T, int32_t H,
                      int32_t head_dim, const uint8_t *key_padding_mask, float qscale,
                      float *out, int64_t out_stride, uint32_t *status,
                      const void *kv_workspace, int64_t workspace_bytes,
                      ftmi_stream_t stream);


/* ---- WaveRNN vocoder (models/fatchord_version.py; gen_forward.py `wavernn`) -------------
 * Fixed architecture of the reference config (config.yaml:189-198): rnn_dims = fc_dims = 512,
 * feat_dims = 80, aux_dims = res_out_dims / 4 = 32; RAW with n_classes = 2^bits <= 512, or
 * MOL (n_classes = 30).  Anything else returns FTMI_E_UNSUPPORTED. */

/* One UpsampleNetwork.up_layers pair (:74-81, :88): Stretch2d(scale, 1) then
 * Conv2d(1, 1, (1, 2 scale + 1), padding (0, scale), no bias) along time, on time-major rows:
 *   y[b, j, c] = sum_i w[i] xs[j + crop0 + i - scale, c],  xs[q] = x[b, q / scale, c]
 * (zero outside [0, W scale)).  x (B, W, C) rows, y (B, W_out, C); crop0 + W_out <= W scale
 * (the final layer writes only the [indent, -indent) crop of :89). */
int ftmi_wr_stretch_conv(const float *x, int64_t x_batch_stride, int32_t B, int32_t W, int32_t C,
                         int32_t scale, const float *w, float *y, int64_t y_batch_stride,
                         int32_t W_out, int32_t crop0, ftmi_stream_t stream);

/* Arguments of ftmi_wavernn.  Weights are fp32, packed once per weights version (float64
 * products, forwardtacotron_amd/wavernn.py `_pack`):
 *   w_hh1, w_hh2 [3R][R]          rnn1/rnn2.weight_hh_l0 (gate rows r, z, n)
 *   w_ih2a [3R][R]                rnn2.weight_ih_l0[:, :R] (the x + h1 part)
 *   w_fc1a [F][R], w_fc2a [F][F]  fc1.weight[:, :R], fc2.weight[:, :F]
 *   w_fc3 [NC][F], b_fc3 [NC]     fc3
 *   b_hh1, b_hh2 [3R]             rnn1/rnn2.bias_hh_l0
 *   u1 = W_ih1 w0, u2 = W_ih2a w0 [3R], v1 = W_fc1a w0 [F]   (w0 = I.weight[:, 0]: the
 *                                 sample's column, carried through the linear layers)
 *   wm [3R + 3R + F][80]          mel columns of G1 = W_ih1 I, Q = W_ih2a I, R = W_fc1a I
 *   cond (bias_row + 1) rows of [3R | 3R | F | F] floats: per mel FRAME the aux terms of
 *                                 G1, Q (+ W_ih2b a2), R (+ W_fc1b a3), S = W_fc2b a4, with
 *                                 every bias folded in; row bias_row = biases only (padding)
 *   mel (items * item_rows, 80)   upsampled mel rows (UpsampleNetwork output)
 * Position of fold b, step t: batched: sample g = b fold_stride + t of item 0 (fold_stride
 * = target + overlap, fold_with_overlap :294-341); else g = t of item b.  g >= item_rows
 * is the fold padding (zero conditioning).  cond row = item frames_per_item + g / hop.
 * Mode: xin == NULL: generate — samples (B, L) receives each fold's drawn samples (:237 /
 * distribution.py:127 values); xin (B, L): teacher-forced forward — logits (B, L, NC).
 * seed: Philox4x32-10 key of the draws (oracle/wr_torch_cpu.py PhiloxSampler).
 * workspace: >= ftmi_wavernn_workspace_bytes() bytes, 16-B aligned (zeroed by the call). */
typedef struct {
  const float *w_hh1, *w_hh2, *w_ih2a, *w_fc1a, *w_fc2a, *w_fc3, *b_fc3, *b_hh1, *b_hh2;
  const float *u1, *u2, *v1, *wm, *cond, *mel;
  const float *xin;
  float *samples, *logits;
  void *workspace;
  uint32_t *status;
  uint64_t seed;
  int32_t bias_row, item_rows, frames_per_item, hop, fold_stride, batched;
  int32_t B, L, n_classes, mol;
  int32_t rnn_dims, fc_dims, feat_dims, aux_dims;
} ftmi_wavernn_args;

/* The sample loop of WaveRNN.generate (:203-241) — teacher-forced: WaveRNN.forward
 * (:145-169) — for B folds as persistent launches of 256 workgroups (one per CU; fewer CUs:
 * FTMI_E_UNSUPPORTED), <= 32 folds per launch.  A workgroup that cannot meet the others
 * (not co-resident) sets FTMI_STATUS_RNN_TIMEOUT in *status: the output is then invalid. */
int64_t ftmi_wavernn_workspace_bytes(void);
int ftmi_wavernn(const ftmi_wavernn_args *args, ftmi_stream_t stream);
uint32_t ftmi_set_wavernn_spin_limit(uint32_t limit);

/* generate's tail (:246-261) in float64: samples (B, L) -> mu-law decode
 * (DSP.decode_mu_law(y, n_classes, False), utils/dsp.py:156-161; n_classes a power of two)
 * -> batched: xfade_and_unfold (:343-406), else fold 0 -> [:wave_len] -> the last fade_len
 * samples times linspace(1, 0, fade_len) (generate: fade_len = 20 hop; 0: none).
 * wave_len >= fade_len (the reference raises otherwise). */
int ftmi_wr_unfold(const float *samples, int32_t B, int32_t L, int32_t target, int32_t overlap,
                   int32_t batched, int32_t mu_law, int32_t n_classes, int32_t wave_len,
                   int32_t fade_len, double *out, ftmi_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FTMI_H */
