"""Tensor-level wrappers over libftmi.so.

Every function takes HIP device tensors (fp32 unless stated), allocates the outputs with
torch's caching allocator (plumbing only), and enqueues ONE ftmi_* entry point on
torch's current stream.  Nothing here computes on the host or falls back to torch ops:
a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import ConvArgs
from .probe import launch

_f32 = torch.float32

# Matrix path of the dense contractions (include/ftmi.h FTMI_MMA_*): 2 = f16x3 split
# (default; fp32-level accuracy at 5.3x the fp32 MFMA rate, activations < 65504),
# 1 = bf16x6 split (fp32-accurate, 2.7x), 0 = plain fp32 MFMA.  FTMI_MMA overrides.
MMA = int(os.environ.get('FTMI_MMA', '2'))
# the recurrences' W_hh h path (same codes; FTMI_RNN_MMA overrides)
RNN_MMA = int(os.environ.get('FTMI_RNN_MMA', '2'))

# Status word (include/ftmi.h FTMI_STATUS_*).  Every GEMM / recurrence launch ORs into a
# per-device word: bit 0 = an f16x3 accumulator became non-finite (an activation beyond the
# f16 range), bit 1 = a W_hh entry beyond the f16 range, bit 2 = a recurrence workgroup
# timed out waiting for its group (its output is invalid).  The model entry points zero it,
# run, read it once at the end: bit 2 raises RnnTimeout; bits 0-1 run the call again under
# `exact_paths()` (fp32 MFMA everywhere), which has no range limit.
STATUS_F16_RANGE, STATUS_WHH_RANGE, STATUS_RNN_TIMEOUT = 1, 2, 4
_STATUS = {}
_FORCED = []  # stack of (gemm mma, rnn mma) overrides


def status_word(device) -> torch.Tensor:
    t = _STATUS.get(device)  # fast path: an indexed torch.device seen before
    if t is not None:
        return t
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    t = _STATUS.get(dev)
    if t is None:
        t = _STATUS[dev] = torch.zeros(1, device=dev, dtype=torch.int32)
    return t


def forced_exact() -> bool:
    """True inside exact_paths() (the range guard's rerun): nothing captured may replay."""
    return bool(_FORCED)


@contextlib.contextmanager
def exact_paths():
    """Run the enclosed calls on the range-unlimited fp32 MFMA paths (GEMMs and
    recurrences)."""
    _FORCED.append((0, 0))
    try:
        yield
    finally:
        _FORCED.pop()


def _gemm_mma(mma: Optional[int], w_split):
    """(matrix path, w_split pointer) of one GEMM launch.  f16x3 needs the f16 planes
    (uint8 block of split_weights_f16); without them the launch uses bf16x6, which takes
    its bf16 pieces (split_weights) or splits the weights in-kernel."""
    m = _FORCED[-1][0] if _FORCED else (MMA if mma is None else mma)
    has16 = w_split is not None and w_split.dtype == torch.uint8
    hasbf = w_split is not None and w_split.dtype == torch.bfloat16
    if m == 2 and not has16:
        m = 1
    ptr = w_split.data_ptr() if (m == 2 and has16) or (m == 1 and hasbf) else None
    return m, ptr


def _rnn_mma() -> int:
    return _FORCED[-1][1] if _FORCED else RNN_MMA


class RnnTimeout(RuntimeError):
    """A persistent recurrence could not run all its workgroups at once (another stream's
    persistent kernels held CUs): its output is invalid, so the call fails."""


def run_checked(fn, device, reduce=None):
    """fn() with the status-word checks: zero the word, run, read it (one host sync).
    A recurrence timeout reruns fn() once with the recurrences compact
    (compact_recurrences()); a second one raises RnnTimeout.  A range bit (f16x3 overflow) runs fn() again
    under exact_paths() — which calls the model's pitch / energy callbacks a second time
    (the first pass's callback outputs derive from the out-of-range predictions and are not
    reused).  reduce(word) -> word combines the status over ranks (sharded generation)
    before the decision."""
    st = status_word(device)

    def attempt():
        st.zero_()
        res = fn()
        s = st if reduce is None else reduce(st)
        w = int(s.item())
        if w & STATUS_RNN_TIMEOUT:
            raise RnnTimeout('a recurrence workgroup timed out waiting for its group (not all '
                             'workgroups co-resident): the result is invalid')
        return res, w

    try:
        out, w = attempt()
    except RnnTimeout:
        # a persistent recurrence could not seat every workgroup at once: another kernel
        # (an RCCL collective, a copy, another process) held CUs past the spin limit.  The
        # launch is rerun once in the compact form (a spread recurrence otherwise takes all
        # 256 CUs); a second timeout raises.
        with compact_recurrences():
            out, w = attempt()
    if w and not _FORCED:
        # the rerun is checked like the first pass (a timeout there raises too; its range
        # bits cannot recur on the range-unlimited paths); afterwards the word shows the
        # bits that caused it, as the call's record
        with exact_paths():
            out, _ = attempt()
        st.fill_(w)
    return out


_COMPACT = []  # non-empty: recurrences ignore `spread` (run_checked's timeout rerun)


@contextlib.contextmanager
def compact_recurrences():
    """Run the enclosed recurrences in their compact form (`spread` ignored: 16 live sequences
    per group, fewer workgroups than CUs where the shape allows)."""
    _COMPACT.append(True)
    try:
        yield
    finally:
        _COMPACT.pop()


def _num_cus() -> int:
    n = getattr(_num_cus, 'v', None)
    if n is None:
        n = _num_cus.v = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return n


SLAB = os.environ.get('FTMI_GEMM_SLAB', '1') != '0'


SLAB_K1_NMIN = int(os.environ.get('FTMI_SLAB_K1_NMIN', 128))  # gemm.hip slab_ok


def _slab(mma: int, T: int, To: int, Cin: int, k: int, N: int, M: int) -> bool:
    """Whether ftmi_conv1d takes the slab kernel (gemm.hip slab_ok)."""
    return (SLAB and mma == 2 and To == T and Cin % 16 == 0 and k <= 16 and (k > 1 or N >= SLAB_K1_NMIN)
            and M * N * k * Cin >= int(os.environ.get('FTMI_GEMM_SLAB_MIN', 0)))


SKINNY_MMAX = 256          # gemm.hip SK_MMAX
SKINNY_MMAX_NARROW = 1024  # gemm.hip SK_MMAX_NARROW (single group, N <= 128)


def _skinny(mma: int, T: int, To: int, Cin: int, k: int, M: int, N: Optional[int] = None) -> bool:
    """Whether a conv takes the weight-streaming skinny kernel (gemm.hip skinny_ok): few
    rows (B = 1 generation) — or a narrow single-group linear (N <= 128) with up to 1024
    rows — f16x3, same-length output.  N = None: a multi-group call (conv bank)."""
    rows_ok = 0 < M <= SKINNY_MMAX or (N is not None and N <= 128 and 0 < M <= SKINNY_MMAX_NARROW)
    return (os.environ.get('FTMI_GEMM_SKINNY', '1') != '0' and mma == 2 and To == T
            and Cin % 16 == 0 and k <= 16 and rows_ok)


def _skinny_split(Cin: int) -> int:
    """Channel split of the skinny kernel: two 32-channel chunks per block."""
    nch = -(-Cin // 32)
    per = int(os.environ.get('FTMI_SKINNY_CPB', 2))  # chunks per block (1 or 2; A/B runs)
    return -(-nch // per)


def _split_k(M: int, N: int, K: int, mma: int, slab: bool = False, Cin: int = 0) -> int:
    """Split K when the tile grid cannot fill the chip (x6 / h3 kernels: 2 workgroups per
    CU; slab kernel: 256 x 128 tiles, 1 per CU, split over 32-channel chunks) and K is long
    enough for the partial-sum round trip to pay."""
    if slab:
        # one workgroup per CU: model the time as (rounds of workgroups) x (steps per
        # workgroup, ~1.8 us each) + the partial-sum round trip of a split (sp x M x N fp32
        # written and read back, priced at 1 TB/s, plus 20 us for the finishing launch —
        # calibrated below)
        tiles = -(-M // 256) * -(-N // 128)
        cus = _num_cus()
        nch = -(-Cin // 32)
        k = K // Cin if Cin else 1

        # the round trip as measured in the model's phoneme phase (round 5, r5_timeline_c3:
        # 24-39 us for 2 splits of 12,800 x 256 beside the other streams — the old 5 TB/s +
        # 5 us model priced it at 15 us and split proj2 / the predictor convs where the
        # finish costs more than it saves): 1 TB/s + 20 us.  Interleaved A/B (5 / 3 rounds,
        # profiles/r5_ab_splitk*.jsonl): c3 8.12-8.20 -> 8.01-8.15, c5 11.33-11.40 ->
        # 11.19-11.26 ms/step, c2 unchanged (2.59-2.65 / 2.60-2.68)
        def t_us(sp):
            run = -(-tiles * sp // cus) * -(-nch // sp) * k * 1.8
            return run + (sp * M * N * 8 / 1e6 + 20.0 if sp > 1 else 0.0)
        return int(min(range(1, min(8, nch) + 1), key=t_us))
    if mma == 0 or K < 2048:
        return 1
    tiles = -(-M // 128) * -(-N // 128)
    slots = 2 * _num_cus()
    if tiles >= slots:
        return 1
    return int(min(8, -(-slots // tiles), K // 1024))


if hasattr(torch._C, '_cuda_getCurrentRawStream'):
    def _stream() -> int:
        """hipStream_t of torch's current stream (the raw-handle query skips the Stream
        object torch.cuda.current_stream() builds: host time on every launch)."""
        return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
else:  # pragma: no cover
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('forwardtacotron_amd ops run on a HIP device only (got a CPU '
                               'tensor); there is no CPU fallback')


def _rows(x: torch.Tensor) -> Tuple[int, int, int, int]:
    """(B, T, C, row_stride) of a channels-last (B, T, C) view with uniformly strided rows."""
    if x.dim() != 3 or x.stride(2) != 1 or x.stride(0) != x.size(1) * x.stride(1):
        raise ValueError(f'expected a (B, T, C) channels-last view with uniform row stride, got '
                         f'shape {tuple(x.shape)} strides {x.stride()}')
    if x.dtype != _f32:
        raise TypeError('fp32 expected')
    return x.size(0), x.size(1), x.size(2), x.stride(1)


def embedding(ids: torch.Tensor, table: torch.Tensor, err: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn.Embedding forward: (B, T) int64 -> (B, T, dim)."""
    _dev(ids, table)
    ids = ids.contiguous()
    if ids.dtype != torch.int64:
        ids = ids.long()
    table = table.contiguous()
    out = torch.empty(*ids.shape, table.size(1), device=table.device, dtype=_f32)
    n, d = ids.numel(), table.size(1)
    launch('ftmi_embedding', f'embedding[n={n},d={d}]', 0, n * 8 + 2 * n * d * 4,
           ids.data_ptr(), n, table.data_ptr(), table.size(0), d, out.data_ptr(), _ptr(err),
           _stream())
    return out


def split_weights(w: torch.Tensor) -> torch.Tensor:
    """fp32 [N][K] -> bf16 [3][N][roundup(K, 32)] pieces (w = p0 + p1 + p2 exactly), the
    pre-split operand of the bf16x6 GEMM path (`ftmi_split_weights`)."""
    _dev(w)
    if w.dim() != 2 or w.dtype != _f32 or not w.is_contiguous():
        raise ValueError('split_weights: contiguous fp32 [N][K] expected')
    N, K = w.shape
    Kp = (K + 31) // 32 * 32
    out = torch.empty(3, N, Kp, device=w.device, dtype=torch.bfloat16)
    launch('ftmi_split_weights', f'split_weights[N={N},K={K}]', 0, 4.0 * N * K + 6.0 * N * Kp,
           w.data_ptr(), N, K, out.data_ptr(), _stream())
    return out


def split_weights_f16(w: torch.Tensor, frag: bool = False) -> torch.Tensor:
    """fp32 [N][K] -> the f16x3 operand of `ftmi_split_weights_f16` (uint8 bytes: f16 planes
    [3][N][roundup(K, 32)] = (2^11 h, t, h) of the power-of-two column-scaled rows, then
    float colscale[N]).  frag: the planes in the fragment-major order of
    `ftmi_split_weights_f16_frag` (the operand of `highway_stack`)."""
    _dev(w)
    if w.dim() != 2 or w.dtype != _f32 or not w.is_contiguous():
        raise ValueError('split_weights_f16: contiguous fp32 [N][K] expected')
    N, K = w.shape
    nbytes = int(_lib.load().ftmi_split_weights_f16_bytes(N, K))
    out = torch.empty(nbytes, device=w.device, dtype=torch.uint8)
    name = 'ftmi_split_weights_f16_frag' if frag else 'ftmi_split_weights_f16'
    launch(name, f'split_weights_f16[N={N},K={K}{",frag" if frag else ""}]', 0,
           4.0 * N * K + nbytes, w.data_ptr(), N, K, out.data_ptr(), _stream())
    return out


def presplit_for(w: torch.Tensor, mma: Optional[int] = None) -> Optional[torch.Tensor]:
    """The pre-split operand of a packed weight for the matrix path `mma` (default MMA):
    f16 planes (2), bf16 pieces (1), None (0)."""
    m = MMA if mma is None else mma
    if m == 2:
        return split_weights_f16(w)
    return split_weights(w) if m == 1 else None


def split_bank_weights(w: torch.Tensor, K: int, Cin: int, Cout: int,
                       mma: Optional[int] = None) -> Optional[torch.Tensor]:
    """Pre-split blocks of a packed conv bank: group g's `presplit_for` block of the
    [Cout][(g+1) Cin] weight, back to back (the `w_split` layout of `ftmi_conv_bank`)."""
    parts, off = [], 0
    for g in range(K):
        n = Cout * Cin * (g + 1)
        blk = presplit_for(w[off:off + n].view(Cout, (g + 1) * Cin), mma)
        if blk is None:
            return None
        parts.append(blk.reshape(-1).view(torch.uint8))
        off += n
    return torch.cat(parts)


def conv1d(x: torch.Tensor, w: torch.Tensor, k: int, pad: int, *, bias=None, relu=False,
           bn=None, maxpool=False, residual=None, out=None, out_t=None, want_y=True,
           T_out: int = 0, mma: Optional[int] = None, w_split: Optional[torch.Tensor] = None,
           x_split: bool = False):
    """Fused Conv1d (+bias, ReLU, BN, residual) on a channels-last (B, T, Cin) view.

    w: packed [N][k*Cin].  Returns (y, yt) where y is (B, T_out, N) (or `out`) and yt is
    the optional (B, N, T_out) transposed copy (`out_t`).  w_split: optional
    `split_weights(w)` (bf16x6 path without the per-call weight split).  x_split: x holds
    f16x3 split rows (include/ftmi.h, e.g. conv_bank(split_out=True)); f16x3 slab kernel
    only (the C side refuses other shapes with FTMI_E_UNSUPPORTED).
    """
    _dev(x, w, bias, residual, out, out_t, w_split)
    B, T, Cin, xs = _rows(x)
    N = w.size(0)
    To = T_out or T
    if w.size(1) != k * Cin:
        raise ValueError(f'packed weight {tuple(w.shape)} does not match k={k}, Cin={Cin}')
    y = None
    if want_y:
        y = out if out is not None else torch.empty(B, To, N, device=x.device, dtype=_f32)
        _rows(y)
    if residual is not None:
        _rows(residual)
    a = ConvArgs()
    a.x, a.x_stride, a.B, a.T, a.Cin = x.data_ptr(), xs, B, T, Cin
    a.w, a.N, a.k, a.pad = w.data_ptr(), N, k, pad
    a.bias = _ptr(bias)
    a.relu = int(relu)
    if bn is not None:
        a.bn_scale, a.bn_shift = bn[0].data_ptr(), bn[1].data_ptr()
    a.maxpool = int(maxpool)
    if residual is not None:
        a.residual, a.res_stride = residual.data_ptr(), residual.stride(1)
    if y is not None:
        a.y, a.y_stride = y.data_ptr(), y.stride(1)
    a.yt = _ptr(out_t)
    a.T_out = To
    a.mma, a.w_split = _gemm_mma(mma, w_split)
    a.status = status_word(x.device).data_ptr()
    a.x_split = int(x_split)
    M = B * To
    if _skinny(a.mma, T, To, Cin, k, M, N):
        sk = _skinny_split(Cin)
    else:
        sk = _split_k(M, N, k * Cin, a.mma, _slab(a.mma, T, To, Cin, k, N, M), Cin)
    if sk > 1:
        part = torch.empty(sk * M * N, device=x.device, dtype=_f32)
        a.split_k, a.split_ws = sk, part.data_ptr()
    label = (f'conv1d[M={M},N={N},K={k * Cin}{",maxpool" if maxpool else ""}'
             f'{",xsplit" if x_split else ""},mma={a.mma}]')
    launch('ftmi_conv1d', label, 2.0 * M * N * k * Cin,
           4.0 * (B * T * Cin + N * k * Cin + M * N * (1 + (residual is not None))),
           ctypes.byref(a), _stream())
    return y, out_t


POOL_BANK = os.environ.get('FTMI_POOL_BANK', '1') != '0'
# the pooled bank hands proj1 its operand as f16x3 split rows (split once, not per column
# tile of proj1: c3 proj1 -2..3 %; a round-3 shell A/B loop, since replaced by tools/ab_bench.py); FTMI_SPLIT_ROWS=0: fp32 rows
SPLIT_ROWS = os.environ.get('FTMI_SPLIT_ROWS', '1') != '0'
# FTMI_SPLIT_BANK_IN=1: the bank also takes its own input split once (split_rows) instead of
# per group / column tile — measured neutral at c3 (the bank kernel saved what the extra
# split launch cost; a round-3 shell A/B loop, since replaced by tools/ab_bench.py), so off by default
SPLIT_BANK_IN = os.environ.get('FTMI_SPLIT_BANK_IN', '0') == '1'


def bank_pools(x: torch.Tensor, K: int, Cout: int, mma: Optional[int] = None, w_split=None) -> bool:
    """Whether conv_bank(pool=True) applies (gemm.hip launch: the f16x3 slab kernel, not the
    few-row skinny kernel): then the bank stores the CBHG maxpool of its output itself."""
    m, wsp = _gemm_mma(mma, w_split)
    B, T, Cin = x.size(0), x.size(1), x.size(2)
    return (POOL_BANK and m == 2 and wsp is not None and not _skinny(m, T, T, Cin, K, B * T)
            and _slab(m, T, T, Cin, K, Cout, B * T))


def bank_halves_image(w_split: Optional[torch.Tensor], K: int, Cin: int,
                      Cout: int) -> Optional[torch.Tensor]:
    """The stream-order weight image of the one-launch few-row bank
    (`ftmi_conv_bank_halves_image`: every wave's weight fragments in its load order, one
    contiguous 1 KB run per wave load), built once per weights version from the f16x3 split
    blocks `split_bank_weights` made; None when those are not f16 planes or the shape has no
    halves kernel.  FTMI_BANK_IMAGE=0 (read when the weights are packed) keeps the planes."""
    if (w_split is None or w_split.dtype != torch.uint8 or not w_split.is_cuda
            or os.environ.get('FTMI_BANK_IMAGE', '1') == '0'):
        return None
    lib = _lib.load()
    n = int(lib.ftmi_conv_bank_halves_image_bytes(Cin, K, Cout))
    if n <= 0:
        return None
    img = torch.empty(n, device=w_split.device, dtype=torch.uint8)
    launch('ftmi_conv_bank_halves_image', f'bank_halves_image[K={K},Cin={Cin},Cout={Cout}]', 0,
           2.0 * n, w_split.data_ptr(), Cin, K, Cout, img.data_ptr(), _stream())
    return img


def conv_bank(x: torch.Tensor, w: torch.Tensor, K: int, Cout: int, scale: torch.Tensor,
              shift: torch.Tensor, mma: Optional[int] = None,
              w_split: Optional[torch.Tensor] = None, pool: bool = False,
              split_out: bool = False, x_split: bool = False,
              w_image: Optional[torch.Tensor] = None) -> torch.Tensor:
    """CBHG conv bank, (B, T, Cin) -> (B, T, K*Cout); pool: the maxpool(2, 1) of it
    (common_layers.py:73,100), stored by the bank kernel (see bank_pools); split_out (with
    pool): stored as f16x3 split rows for proj1 (conv1d(x_split=True)); x_split: x holds
    split rows (split_rows); w_image: `bank_halves_image(w_split, ...)`, read instead of
    w_split where the one-launch few-row kernel runs (same results bit for bit)."""
    if split_out and not pool:
        raise ValueError('split_out needs pool')
    _dev(x, w, scale, shift, w_split)
    B, T, Cin, xs = _rows(x)
    y = torch.empty(B, T, K * Cout, device=x.device, dtype=_f32)
    M = B * T
    flops = 2.0 * M * Cout * Cin * K * (K + 1) / 2
    mma, wsp = _gemm_mma(mma, w_split)
    sk, part, last = 0, None, 0
    if not pool and not x_split and _bank_halves(mma, B, T, Cin, K, Cout):
        # the few-row bank in one launch (gemm.hip conv_bank_halves_kernel)
        n = int(_lib.load().ftmi_conv_bank_halves_ws_floats(B, T, K, Cout)) - BANK_COUNTERS
        sk, part, last = 2, _bank_workspace(n, x.device), BANK_HALVES
        if w_image is not None:
            _dev(w_image)
            wsp, last = w_image.data_ptr(), BANK_HALVES | BANK_IMAGE
    elif not pool and _skinny(mma, T, T, Cin, K, M) and _skinny_split(Cin) > 1:
        sk = _skinny_split(Cin)  # weight-streaming kernel: partial sums, finished in order
        part = torch.empty(sk * M * K * Cout, device=x.device, dtype=_f32)
    launch('ftmi_conv_bank_split', f'conv_bank[M={M},K={K},Cin={Cin},mma={mma}'
           f'{",pool" if pool else ""}{",split" if split_out else ""}{",xsplit" if x_split else ""}'
           ']',
           flops, 4.0 * (M * Cin + Cout * Cin * K * (K + 1) / 2 + M * K * Cout),
           x.data_ptr(), xs, B, T, Cin, w.data_ptr(), wsp, K, Cout,
           scale.data_ptr(), shift.data_ptr(), y.data_ptr(), y.stride(-2), mma,
           status_word(x.device).data_ptr(), sk, _ptr(part),
           int(pool) | (2 * int(split_out)) | (4 * int(x_split)) | last, _stream())
    return y


BANK_COUNTERS = 4096  # include/ftmi.h FTMI_BANK_COUNTERS
BANK_HALVES, BANK_IMAGE = 16, 32  # include/ftmi.h FTMI_BANK_HALVES / _IMAGE


def _bank_halves(mma: int, B: int, T: int, Cin: int, K: int, Cout: int) -> bool:
    """Whether conv_bank takes the one-launch channel-halves kernel (gemm.hip
    bank_halves_ok): f16x3, one row tile of at most 128 rows (batch-1 generation, BASELINE
    config c2), Cin a multiple of 64 up to 256, even K, (K / 2)(Cout / 16) a multiple of 8 up
    to 512 (8 arrival counters per unit).
    FTMI_BANK_HALVES=0 (read per call) keeps the channel-split kernel + finish."""
    return (os.environ.get('FTMI_BANK_HALVES', '1') != '0' and mma == 2 and 0 < B * T <= 128
            and Cin % 64 == 0 and Cin <= 256 and K % 2 == 0 and Cout % 16 == 0
            and (K // 2) * (Cout // 16) % 8 == 0 and (K // 2) * (Cout // 16) <= 512 and K <= 16)
_BANK_WS = {}


def _bank_workspace(n_part: int, device) -> torch.Tensor:
    """The FTMI_BANK_HALVES workspace of the current stream: BANK_COUNTERS counters (zero
    once; every launch leaves them zero) followed by n_part floats of partial sums.  One per
    (device, stream) — launches on one stream are ordered, so they may share it — kept alive
    for graph replays that captured its address; grown (a new zeroed buffer) when too small."""
    stream = torch.cuda.current_stream(device)
    key = (torch.device(device), stream.cuda_stream)
    t = _BANK_WS.get(key)
    if t is None or t.numel() < BANK_COUNTERS + n_part:
        if t is not None:  # the old buffer may still be in use by queued work
            _BANK_OLD.append(t)
        t = _BANK_WS[key] = torch.zeros(BANK_COUNTERS + n_part, device=device, dtype=_f32)
    return t


_BANK_OLD = []  # superseded workspaces (kept: a captured graph may still replay them)


def split_rows(x: torch.Tensor) -> torch.Tensor:
    """(B, T, C) fp32 rows -> the same-size buffer holding them as f16x3 split rows (per row C
    f16 heads then C scaled tails, include/ftmi.h), range-checked into the status word."""
    _dev(x)
    B, T, C, xs = _rows(x)
    y = torch.empty(B, T, C, device=x.device, dtype=_f32)
    launch('ftmi_split_rows', f'split_rows[M={B * T},C={C}]', 0.0, 8.0 * B * T * C,
           x.data_ptr(), xs, B * T, C, y.data_ptr(), y.stride(1),
           status_word(x.device).data_ptr(), _stream())
    return y


def highway(x: torch.Tensor, w12: torch.Tensor, b1: torch.Tensor, b2: torch.Tensor,
            out: Optional[torch.Tensor] = None, mma: Optional[int] = None,
            w_split: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(x, w12, b1, b2, out, w_split)
    B, T, C, xs = _rows(x)
    y = out if out is not None else torch.empty(B, T, C, device=x.device, dtype=_f32)
    M = B * T
    mma, wsp = _gemm_mma(mma, w_split)
    sk, part = 0, None
    if (mma == 2 and wsp is not None and os.environ.get('FTMI_GEMM_SKINNY', '1') != '0'
            and C % 16 == 0 and 0 < M <= SKINNY_MMAX_NARROW):
        sk = _skinny_split(C)  # weight-streaming kernel: partials + the highway finish
        part = torch.empty(sk * M * 2 * C, device=x.device, dtype=_f32)
    launch('ftmi_highway_split', f'highway[M={M},C={C},mma={mma}]', 2.0 * M * 2 * C * C,
           4.0 * (2 * M * C + 2 * C * C),
           x.data_ptr(), xs, M, C, w12.data_ptr(), wsp, b1.data_ptr(),
           b2.data_ptr(), y.data_ptr(), y.stride(1), mma, status_word(x.device).data_ptr(),
           sk, _ptr(part), _stream())
    return y


HS_C, HS_NPASS, HS_MAXL = 256, 512, 8  # gemm.hip highway_stack_kernel shape limits
# The fused stack below FTMI_HS_MIN rows falls back to the per-layer launches.  Round 4
# moved the default 256 -> 64: at c2 (the prenet's 120 rows) the one launch replaces four
# skinny GEMMs + four finish launches, c2 2.81 / 2.96 / 2.83 -> 2.80 / 2.81 / 2.80 ms per
# step (tools/ab_bench.py, 3 interleaved rounds, profiles/r4_ab_c2_env.jsonl)
HS_MIN_ROWS = int(os.environ.get('FTMI_HS_MIN', 64))


def highway_stack_ok(M: int, Cp: int, C: int, L: int, n_out: int, splits) -> bool:
    """Whether `highway_stack` applies: the f16x3 path is the one in force (not inside
    exact_paths()), every weight has its f16 planes, and the shapes fit the kernel."""
    if os.environ.get('FTMI_HS', '1') == '0' or (_FORCED and _FORCED[-1][0] != 2):
        return False
    if not _FORCED and MMA != 2:
        return False
    return (C == HS_C and 0 < Cp <= C and Cp % 4 == 0 and L <= HS_MAXL
            and n_out % HS_NPASS == 0 and M >= max(HS_MIN_ROWS, 1)
            and all(w is not None and w.dtype == torch.uint8 for w in splits))


def highway_stack(x: torch.Tensor, pre_split: torch.Tensor, C: int, hw_splits, b1s, b2s,
                  out_split: Optional[torch.Tensor], b_out: Optional[torch.Tensor], n_out: int,
                  want_h: bool = False, spread: bool = True):
    """CBHG pre_highway -> highways -> GRU input projection in one launch
    (`ftmi_highway_stack`; models/common_layers.py:110-115).  x: (B, T, Cp) channels-last;
    every weight block is `split_weights_f16(w, frag=True)`.  spread=False keeps the
    one-workgroup-per-64-rows kernel where the spread one would apply (its workgroups must
    be co-resident: the caller decides).  Returns (y (B, T, n_out) or None, h (B, T, C) or
    None)."""
    _dev(x, pre_split, out_split, b_out, *hw_splits, *b1s, *b2s)
    B, T, Cp, xs = _rows(x)
    M = B * T
    L = len(hw_splits)
    y = torch.empty(B, T, n_out, device=x.device, dtype=_f32) if out_split is not None else None
    h = torch.empty(B, T, C, device=x.device, dtype=_f32) if want_h else None
    arr = ctypes.c_void_p * max(L, 1)
    w_arr = arr(*[w.data_ptr() for w in hw_splits])
    b1_arr = arr(*[b.data_ptr() for b in b1s])
    b2_arr = arr(*[b.data_ptr() for b in b2s])
    flops = 2.0 * M * C * (Cp + L * 2 * C + n_out)
    nbytes = 4.0 * M * (Cp + n_out + (C if want_h else 0))
    args = (x.data_ptr(), xs, M, Cp, C, pre_split.data_ptr(), L, ctypes.addressof(w_arr),
            ctypes.addressof(b1_arr), ctypes.addressof(b2_arr), _ptr(out_split), _ptr(b_out),
            n_out if out_split is not None else 0, _ptr(y), y.stride(1) if y is not None else 0,
            _ptr(h), h.stride(1) if h is not None else 0, status_word(x.device).data_ptr())
    if spread and hs_spread_blocks(M, n_out if out_split is not None else 0) > 0:
        ws = _spread_workspace(int(_lib.load().ftmi_highway_stack_spread_ws_bytes(M)), x.device)
        launch('ftmi_highway_stack_spread', f'highway_stack_spread[M={M},Cp={Cp},L={L},N={n_out}]',
               flops, nbytes, *args, ws.data_ptr(), _stream())
    else:
        launch('ftmi_highway_stack', f'highway_stack[M={M},Cp={Cp},L={L},N={n_out}]', flops,
               nbytes, *args, _stream())
    return y, h


def hs_spread_blocks(M: int, n_out: int = 0) -> int:
    """Workgroups of the spread CBHG tail (`ftmi_highway_stack_spread`) for M rows, or 0 when
    `highway_stack` runs the one-workgroup-per-64-rows kernel: M <= 1024 rows, n_out <= 1536,
    all of them resident at once.  FTMI_HS_SPREAD=0 (read per call) keeps that kernel."""
    if os.environ.get('FTMI_HS_SPREAD', '1') == '0' or n_out > 1536:
        return 0
    n = int(_lib.load().ftmi_highway_stack_spread_blocks(M))
    return n if 0 < n <= _num_cus() else 0


_SPREAD_WS = {}


def _spread_workspace(nbytes: int, device) -> torch.Tensor:
    """The spread tail's exchange workspace of the current stream (one per (device, stream):
    launches on one stream are ordered), kept alive for graph replays that captured its
    address; grown when too small."""
    stream = torch.cuda.current_stream(device)
    key = (torch.device(device), stream.cuda_stream)
    t = _SPREAD_WS.get(key)
    if t is None or t.numel() < nbytes:
        if t is not None:
            _BANK_OLD.append(t)  # a captured graph may still replay the old buffer
        t = _SPREAD_WS[key] = torch.zeros(max(nbytes, 16), device=device, dtype=torch.uint8)
    return t


PANEL_N = 256  # gemm.hip panel_proj_kernel: output columns per panel (LayerNorm width)


def panel_ok(K: int, N: int, ln: bool, split) -> bool:
    """Whether `panel_proj` applies: the f16x3 path is in force (not inside exact_paths()),
    the weight has its fragment-major f16 planes, and the shape fits the kernel
    (FTMI_PANEL=0 keeps the slab GEMM + LayerNorm launches)."""
    if os.environ.get('FTMI_PANEL', '1') == '0' or (_FORCED and _FORCED[-1][0] != 2):
        return False
    if not _FORCED and MMA != 2:
        return False
    return (split is not None and split.dtype == torch.uint8 and K % 4 == 0
            and N % PANEL_N == 0 and (N == PANEL_N or not ln))


def panel_proj(x: torch.Tensor, w_frag: torch.Tensor, N: int, bias: Optional[torch.Tensor] = None,
               residual: Optional[torch.Tensor] = None, ln=None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = [LayerNorm](x W^T + bias [+ residual]) in one launch (`ftmi_panel_proj`): the k = 1
    projections of a FastPitch FFT block (models/fast_pitch.py:56-91) with their residual
    add and norm.  x: (B, T, K) channels-last; w_frag: split_weights_f16(W, frag=True);
    ln: (gamma, beta, eps) or None.  out may be the residual (in place), never x."""
    _dev(x, w_frag, bias, residual)
    B, T, K, xs = _rows(x)
    M = B * T
    y = out if out is not None else torch.empty(B, T, N, device=x.device, dtype=_f32)
    rs = 0
    if residual is not None:
        if tuple(residual.shape) != (B, T, N):
            raise ValueError(f'residual shape {tuple(residual.shape)} != {(B, T, N)}')
        rs = _rows(residual)[3]
    if tuple(y.shape) != (B, T, N):
        raise ValueError(f'out shape {tuple(y.shape)} != {(B, T, N)}')
    _rows(y)
    g, b, eps = ln if ln is not None else (None, None, 0.0)
    launch('ftmi_panel_proj', f'panel_proj[M={M},K={K},N={N}{",ln" if ln is not None else ""}]',
           2.0 * M * N * K, 4.0 * M * (K + N * (2 if residual is not None else 1)),
           x.data_ptr(), xs, M, K, w_frag.data_ptr(), N, _ptr(bias), _ptr(residual), rs,
           _ptr(g), _ptr(b), float(eps), y.data_ptr(), y.stride(1),
           status_word(x.device).data_ptr(), _stream())
    return y


_KV_WS = {}


def _kv_workspace(nbytes: int, device) -> torch.Tensor:
    """The attention K / V plane workspace of the current stream (ftmi_panel_proj_qkv /
    ftmi_attention_kv), reused by every call on the stream (stream order separates the
    layers' uses); grown when too small.  The planes' pad keys T..Tp-1 are never written;
    the attention kernels zero them while staging (a stale value there, even an inf left by
    an overflowing call that reran on the exact path, never reaches the output)."""
    stream = torch.cuda.current_stream(device)
    key = (torch.device(device), stream.cuda_stream)
    t = _KV_WS.get(key)
    if t is None or t.numel() < nbytes:
        if t is not None:
            _KV_OLD.append(t)  # may still be read by queued work
        t = _KV_WS[key] = torch.zeros(nbytes, device=device, dtype=torch.uint8)
    return t


_KV_OLD = []


def kv_fused_ok(T: int, d: int, heads: int, w_frag) -> bool:
    """Whether FastPitch's in_proj + attention take ftmi_panel_proj_qkv + ftmi_attention_kv
    (the split pass folded into the projection): f16x3 in force, the attention would
    presplit (T > 256), d = 256, head_dim 64 / 128.  FTMI_KV_FUSED=0 turns it off."""
    return (os.environ.get('FTMI_KV_FUSED', '1') != '0' and panel_ok(d, 3 * d, False, w_frag)
            and ATTN_PRESPLIT and T > 256 and d == PANEL_N and d % heads == 0
            and d // heads in (64, 128))


def panel_proj_qkv(x: torch.Tensor, w_frag: torch.Tensor, d: int, heads: int,
                   bias: Optional[torch.Tensor] = None):
    """in_proj with the attention's K / V split folded in (`ftmi_panel_proj_qkv`): returns
    (q rows (B, T, d), the K / V plane workspace) for attention_kv."""
    _dev(x, w_frag, bias)
    B, T, K, xs = _rows(x)
    q = torch.empty(B, T, d, device=x.device, dtype=_f32)
    nws = int(_lib.load().ftmi_attention_workspace_bytes(B, T, heads, d // heads))
    ws = _kv_workspace(nws, x.device)
    launch('ftmi_panel_proj_qkv', f'panel_proj[M={B * T},K={K},N={3 * d},qkv]',
           2.0 * B * T * 3 * d * K, 4.0 * B * T * (K + d) + 2.0 * nws / 4 * 2,
           x.data_ptr(), xs, B, T, K, w_frag.data_ptr(), d, _ptr(bias), heads, q.data_ptr(),
           q.stride(1), ws.data_ptr(), nws, status_word(x.device).data_ptr(), _stream())
    return q, ws


def attention_kv(q: torch.Tensor, ws: torch.Tensor, heads: int,
                 key_padding_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """attention on Q rows with K / V from panel_proj_qkv's workspace (`ftmi_attention_kv`)."""
    _dev(q, ws, key_padding_mask)
    B, T, d, rs = _rows(q)
    hd = d // heads
    out = torch.empty(B, T, d, device=q.device, dtype=_f32)
    kpm = None
    if key_padding_mask is not None:
        kpm = key_padding_mask.to(torch.uint8).contiguous()
    launch('ftmi_attention_kv', f'attention[B={B},T={T},H={heads},hd={hd},mma=2,kv]',
           4.0 * B * heads * T * T * hd, 4.0 * (B * T * d * 2),
           q.data_ptr(), rs, B, T, heads, hd, _ptr(kpm), float(np.float32(np.sqrt(1.0 / hd))),
           out.data_ptr(), out.stride(1), status_word(q.device).data_ptr(), ws.data_ptr(),
           ws.numel(), _stream())
    return out


RNN_SPREAD = 0x100  # include/ftmi.h FTMI_RNN_SPREAD


def rnn_blocks(cell: int, B: int, H: int, mma: Optional[int] = None) -> int:
    """Persistent workgroups one ftmi_rnn_bidir launch occupies (ftmi_rnn_blocks)."""
    m = _rnn_mma() if mma is None else mma
    return int(_lib.load().ftmi_rnn_blocks(cell, B, H, m))


def rnn_bidir(cell: int, xp: torch.Tensor, H: int, w_hh: torch.Tensor, b_hh: Optional[torch.Tensor],
              T: Optional[int] = None, index: Optional[torch.Tensor] = None,
              xp_zero: Optional[torch.Tensor] = None, lengths: Optional[torch.Tensor] = None,
              pad_value: float = 0.0, check: bool = False,
              ws: Optional[torch.Tensor] = None, mma: Optional[int] = None,
              spread: bool = False) -> torch.Tensor:
    """Bidirectional GRU (cell=0) / LSTM (cell=1) recurrence -> (B, T, 2H).

    xp: (B, T_src, 2*G*H) input projections; index: (B, T) int32 frame -> row map.
    check=True synchronises and raises RnnTimeout if a workgroup gave up waiting.
    mma: matrix path of W_hh h (default RNN_MMA; exact_paths() forces fp32).
    spread: FTMI_RNN_SPREAD — the recurrence may occupy every CU (fewer sequences per
    workgroup group, lower step latency); only for a recurrence that runs alone (the
    decoder LSTM, the postnet GRU), never beside other persistent recurrences.
    """
    mma = (_rnn_mma() if mma is None or _FORCED else mma)
    if lengths is not None:  # host-side lengths (as pack_padded_sequence takes) are fine
        lengths = lengths.to(device=xp.device, dtype=torch.int32).contiguous()
    _dev(xp, w_hh, b_hh, index, xp_zero, lengths)
    B, T_src, _, xs = _rows(xp)
    T = T if T is not None else T_src
    y = torch.empty(B, T, 2 * H, device=xp.device, dtype=_f32)
    lib = _lib.load()
    need = int(lib.ftmi_rnn_workspace_bytes(B, H, cell)) // 4 + 4
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, device=xp.device, dtype=torch.int32)
    if index is not None:
        assert index.dtype == torch.int32 and index.is_contiguous() and index.shape == (B, T)
    G = 4 if cell else 3
    label = f'rnn_bidir[{"lstm" if cell else "gru"},B={B},T={T},H={H},mma={mma}]'
    # recurrent contraction W_hh h per step and direction; bytes: xp rows read per frame,
    # W_hh once, y written once
    launch('ftmi_rnn_bidir', label, 2.0 * B * T * 2 * G * H * H,
           4.0 * (B * T * 2 * G * H + 2 * G * H * H + B * T * 2 * H),
           cell, B, T, H, xp.data_ptr(), xs, T_src, _ptr(index), _ptr(xp_zero),
           w_hh.data_ptr(), _ptr(b_hh), _ptr(lengths), float(pad_value), y.data_ptr(), y.stride(1),
           int(mma) | (RNN_SPREAD if spread and not _COMPACT else 0), status_word(xp.device).data_ptr(),
           ws.data_ptr(), _stream())
    if check:
        torch.cuda.current_stream().synchronize()
        off = int(lib.ftmi_rnn_error_offset(B)) // 4
        if int(ws[off].item()) != 0:
            raise RnnTimeout('ftmi_rnn_bidir: a workgroup timed out waiting for its group')
    return y


def duration_counts(dur: torch.Tensor, apply_fill: bool, fill_value: float = 2.0):
    """In place: fill-2 rule (optional) + clip; returns (offsets (B,T+1), totals (B,), fill_flag)."""
    _dev(dur)
    if dur.dtype != _f32 or not dur.is_contiguous() or dur.dim() != 2:
        raise ValueError('dur must be a contiguous (B, T) fp32 tensor')
    B, T = dur.shape
    offsets = torch.empty(B, T + 1, device=dur.device, dtype=torch.int32)
    totals = torch.empty(B, device=dur.device, dtype=torch.int32)
    flag = torch.empty(1, device=dur.device, dtype=torch.int32)
    launch('ftmi_duration_counts', f'duration_counts[B={B},T={T}]', 0, B * T * 12,
           dur.data_ptr(), B, T, int(apply_fill), float(fill_value),
           offsets.data_ptr(), totals.data_ptr(), flag.data_ptr(), _stream())
    return offsets, totals, flag


def duration_trunc_sum(dur: torch.Tensor) -> torch.Tensor:
    """sum_{b,t} int64(trunc(dur)) as a device int64[1] (the fill-2 rule's statistic)."""
    _dev(dur)
    B, T = dur.shape
    out = torch.empty(1, device=dur.device, dtype=torch.int64)
    launch('ftmi_duration_trunc_sum', f'duration_trunc_sum[B={B},T={T}]', 0, 4.0 * B * T,
           dur.data_ptr(), B, T, out.data_ptr(), _stream())
    return out


def duration_counts_global(dur: torch.Tensor, global_sum: torch.Tensor, fill_value: float = 2.0):
    """duration_counts with the fill-2 decision taken on a batch-global sum (device int64[1])."""
    _dev(dur, global_sum)
    if dur.dtype != _f32 or not dur.is_contiguous() or dur.dim() != 2:
        raise ValueError('dur must be a contiguous (B, T) fp32 tensor')
    B, T = dur.shape
    offsets = torch.empty(B, T + 1, device=dur.device, dtype=torch.int32)
    totals = torch.empty(B, device=dur.device, dtype=torch.int32)
    flag = torch.empty(1, device=dur.device, dtype=torch.int32)
    launch('ftmi_duration_counts_global', f'duration_counts[B={B},T={T}]', 0, B * T * 12,
           dur.data_ptr(), B, T, global_sum.data_ptr(), float(fill_value), offsets.data_ptr(),
           totals.data_ptr(), flag.data_ptr(), _stream())
    return offsets, totals, flag


def lr_index(offsets: torch.Tensor, T_mel: int) -> torch.Tensor:
    _dev(offsets)
    B, T1 = offsets.shape
    index = torch.empty(B, T_mel, device=offsets.device, dtype=torch.int32)
    launch('ftmi_lr_index', f'lr_index[B={B},T_mel={T_mel}]', 0, 4.0 * B * (T1 + T_mel),
           offsets.data_ptr(), B, T1 - 1, T_mel, index.data_ptr(), _stream())
    return index


def length_regulate(x: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    _dev(x, index)
    B, T, C, xs = _rows(x)
    T_mel = index.size(1)
    y = torch.empty(B, T_mel, C, device=x.device, dtype=_f32)
    launch('ftmi_length_regulate', f'length_regulate[B={B},T={T},T_mel={T_mel},C={C}]', 0,
           4.0 * (B * T * C + B * T_mel * (C + 1)),
           x.data_ptr(), xs, B, T, C, index.data_ptr(), T_mel, y.data_ptr(), y.stride(1), _stream())
    return y


def series_proj_add(x: torch.Tensor, pitch: torch.Tensor, wp, bp, ps: float, energy: torch.Tensor,
                    we, be, es: float) -> torch.Tensor:
    """In place on x (B, T, C): x += proj(pitch)*ps ; x += proj(energy)*es."""
    _dev(x, pitch, energy, wp, bp, we, be)
    B, T, C, xs = _rows(x)
    pitch = pitch.reshape(B, T).to(_f32).contiguous()
    energy = energy.reshape(B, T).to(_f32).contiguous()
    launch('ftmi_series_proj_add', f'series_proj_add[B={B},T={T},C={C}]', 14.0 * B * T * C,
           4.0 * (2 * B * T * C + 2 * B * T + 8 * C),
           x.data_ptr(), xs, B, T, C, pitch.data_ptr(), wp.data_ptr(),
           bp.data_ptr(), float(ps), energy.data_ptr(), we.data_ptr(), be.data_ptr(), float(es),
           _stream())
    return x


def rowdot(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], alpha: float) -> torch.Tensor:
    """(x . w + bias) / alpha over the last dim: (B, T, C) -> (B, T)."""
    _dev(x, w, bias)
    B, T, C, xs = _rows(x)
    out = torch.empty(B, T, device=x.device, dtype=_f32)
    launch('ftmi_rowdot', f'rowdot[M={B * T},C={C}]', 2.0 * B * T * C, 4.0 * (B * T * (C + 1) + C),
           x.data_ptr(), xs, B * T, C, w.data_ptr(), _ptr(bias), float(alpha),
           out.data_ptr(), _stream())
    return out


# --------------------------------------------------------------------------------------
# FastPitch transformer (csrc/transformer.hip)

def embedding_posenc(ids: torch.Tensor, table: torch.Tensor, pe: torch.Tensor,
                     scale: torch.Tensor) -> torch.Tensor:
    """(B, T) ids -> table[ids] + scale * pe[:T]  (B, T, dim)."""
    _dev(ids, table, pe, scale)
    B, T = ids.shape
    dim = table.size(1)
    ids = ids.contiguous().to(torch.int64)
    out = torch.empty(B, T, dim, device=ids.device, dtype=_f32)
    launch('ftmi_embedding_posenc', f'embedding_posenc[n={B * T},d={dim}]', B * T * dim * 2.0,
           8.0 * B * T + 12.0 * B * T * dim,
           ids.data_ptr(), B, T, table.data_ptr(), table.size(0), dim, pe.data_ptr(),
           scale.data_ptr(), out.data_ptr(), None, _stream())
    return out


def lr_posenc(x: torch.Tensor, index: torch.Tensor, pe: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """LengthRegulator expansion (index map) + scale * pe[:T_mel]: (B, T_mel, C)."""
    _dev(x, index, pe, scale)
    B, T, C, xs = _rows(x)
    T_mel = index.size(1)
    y = torch.empty(B, T_mel, C, device=x.device, dtype=_f32)
    launch('ftmi_lr_posenc', f'lr_posenc[B={B},T_mel={T_mel},C={C}]', 2.0 * B * T_mel * C,
           4.0 * (B * T * C + B * T_mel * (2 * C + 1)),
           x.data_ptr(), xs, B, T, C, index.data_ptr(), T_mel, pe.data_ptr(), scale.data_ptr(),
           y.data_ptr(), y.stride(1), _stream())
    return y


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(x, gamma, beta, out)
    B, T, C, xs = _rows(x)
    y = out if out is not None else torch.empty(B, T, C, device=x.device, dtype=_f32)
    launch('ftmi_layernorm', f'layernorm[M={B * T},C={C}]', 8.0 * B * T * C, 8.0 * B * T * C,
           x.data_ptr(), xs, B * T, C, gamma.data_ptr(), beta.data_ptr(), float(eps),
           y.data_ptr(), y.stride(1), _stream())
    return y


ATTN_PRESPLIT = os.environ.get('FTMI_ATTN_PRESPLIT', '1') != '0'


def attention(qkv: torch.Tensor, heads: int, key_padding_mask: Optional[torch.Tensor] = None,
              mma: Optional[int] = None, presplit: Optional[bool] = None) -> torch.Tensor:
    """Self-attention core of nn.MultiheadAttention on packed in_proj rows (B, T, 3d).
    mma: 2 = f16x3 contractions (default, MMA), 0 = fp32 MFMA (exact_paths(), MMA 0/1).
    presplit (f16x3; default: ATTN_PRESPLIT and T > 512): K and V split once into f16
    planes in a workspace instead of per query tile (identical results; measured at c5's
    postnet T = 1400: 825 -> 618 us incl. the split pass, slower at T = 200)."""
    _dev(qkv, key_padding_mask)
    m = _FORCED[-1][0] if _FORCED else (MMA if mma is None else mma)
    m = 2 if m == 2 else 0
    B, T, C3, rs = _rows(qkv)
    d = C3 // 3
    hd = d // heads
    out = torch.empty(B, T, d, device=qkv.device, dtype=_f32)
    kpm = None
    if key_padding_mask is not None:
        kpm = key_padding_mask.to(torch.uint8).contiguous()
    qscale = float(np.float32(np.sqrt(1.0 / hd)))
    ws, nws = None, 0
    if presplit is None:  # the transposed kernel with the split pass against its in-kernel
        # split (tools/attn_short_ab.py, B = 64, masked): T 300-400 0.91-0.95x, T 600 1.01x,
        # T 1000 1.01-1.06x, T 1400 1.02-1.08x
        presplit = ATTN_PRESPLIT and T > 512
    if m == 2 and presplit:
        nws = int(_lib.load().ftmi_attention_workspace_bytes(B, T, heads, hd))
        ws = torch.empty(nws, device=qkv.device, dtype=torch.uint8)
    launch('ftmi_attention', f'attention[B={B},T={T},H={heads},hd={hd},mma={m}]',
           4.0 * B * heads * T * T * hd, 4.0 * (B * T * C3 + B * T * d),
           qkv.data_ptr(), rs, B, T, heads, hd, 0, d, 2 * d, _ptr(kpm), qscale,
           out.data_ptr(), out.stride(1), m, status_word(qkv.device).data_ptr(), _ptr(ws), nws,
           _stream())
    return out


# ---- WaveRNN vocoder (csrc/wavernn.hip) --------------------------------------------------

def wr_stretch_conv(x: torch.Tensor, scale: int, w: torch.Tensor, W_out: Optional[int] = None,
                    crop0: int = 0) -> torch.Tensor:
    """Stretch2d(scale, 1) + Conv2d(1, 1, (1, 2 scale + 1), pad (0, scale)) along time on
    (B, W, C) rows -> (B, W_out, C) (default W * scale; crop0 = first output sample)."""
    _dev(x, w)
    x = x.contiguous()
    w = w.reshape(-1).float().contiguous()
    B, W, C = x.shape
    if w.numel() != 2 * scale + 1:
        raise ValueError(f'smoothing kernel of {w.numel()} taps for scale {scale}')
    W_out = W * scale if W_out is None else W_out
    y = torch.empty(B, W_out, C, device=x.device, dtype=_f32)
    launch('ftmi_wr_stretch_conv', f'wr_stretch_conv[B={B},W={W},C={C},s={scale}]',
           2.0 * B * W_out * C * (2 * scale + 1), 4.0 * (B * W * C + B * W_out * C),
           x.data_ptr(), W * C, B, W, C, scale, w.data_ptr(), y.data_ptr(), W_out * C, W_out, crop0,
           _stream())
    return y


def wavernn(args, B: int, L: int, flops: float, device) -> None:
    """Enqueue ftmi_wavernn (args: a filled _lib.WaveRNNArgs; the caller keeps every buffer
    alive).  The status word pointer is set here."""
    args.status = status_word(device).data_ptr()
    mode = 'forward' if args.xin else 'generate'
    launch('ftmi_wavernn', f'wavernn[{mode},B={B},L={L},NC={args.n_classes}]', flops,
           4.0 * B * L * (1 + (args.n_classes if args.logits else 0)), ctypes.byref(args), _stream())


def wavernn_workspace(device) -> torch.Tensor:
    n = int(_lib.load().ftmi_wavernn_workspace_bytes())
    return torch.empty(n // 4, device=device, dtype=torch.int32)


def wr_unfold(samples: torch.Tensor, target: int, overlap: int, batched: bool, mu_law: bool,
              n_classes: int, wave_len: int, fade_len: int) -> torch.Tensor:
    """generate's tail in float64 on the device: (B, L) samples -> (wave_len,) wave
    (fade_len: the final linear fade-out, 20 hop in generate, 0 for none)."""
    _dev(samples)
    samples = samples.contiguous()
    B, L = samples.shape
    out = torch.empty(wave_len, device=samples.device, dtype=torch.float64)
    launch('ftmi_wr_unfold', f'wr_unfold[B={B},L={L}]', 0, 4.0 * B * L + 8.0 * wave_len,
           samples.data_ptr(), B, L, target, overlap, int(batched), int(mu_law), n_classes,
           wave_len, fade_len, out.data_ptr(), _stream())
    return out
