"""`utils/dsp.py` (reference) on libftmi.so: the DSP class with the same constructor,
``from_config``, ``wav_to_mel``, ``griffinlim``, ``normalize`` / ``denormalize``,
``save_wav`` and the mu-law / label helpers.

The reference delegates the arithmetic to librosa 0.7.2 (``requirements.txt:2``); here the
STFT / log-mel, ISTFT, Griffin-Lim and the mel pseudo-inverse run as HIP kernels
(``csrc/dsp.hip``, entry points in ``include/ftmi.h``).  The host side only builds the
per-config plan once (window, fp64 twiddles, the Slaney mel filterbank, its sparse form
and pseudo-inverse) and moves arrays between numpy and the device, so
``wav_to_mel(np.ndarray) -> np.ndarray`` and ``griffinlim(np.ndarray) -> np.ndarray``
keep the reference's signatures.  The batched device entry points
(``mel_spectrogram`` / ``griffinlim_batch``) take and return HIP tensors.

Not carried over (outside the hot path, need absent libraries): ``load_wav`` resampling
(librosa), ``trim_silence`` (librosa.effects), ``trim_long_silences`` (webrtcvad).
"""
from __future__ import annotations

import ctypes
import os
import wave
from pathlib import Path
from typing import Any, Dict, Optional, Tuple, Union

import numpy as np
import scipy.signal
import torch

from . import _lib
from .probe import launch


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# --- plan (host-built constants; librosa 0.7.2 definitions) ----------------------------------

def _hz_to_mel(f: np.ndarray) -> np.ndarray:
    """Slaney mel scale (librosa core.hz_to_mel, htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    m = f / f_sp
    if m.ndim:
        hi = f >= min_log_hz
        m[hi] = min_log_mel + np.log(f[hi] / min_log_hz) / logstep
    elif f >= min_log_hz:
        m = min_log_mel + np.log(f / min_log_hz) / logstep
    return m


def _mel_to_hz(m: np.ndarray) -> np.ndarray:
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    f = f_sp * m
    hi = m >= min_log_mel
    f[hi] = min_log_hz * np.exp(logstep * (m[hi] - min_log_mel))
    return f


def mel_basis(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: Optional[float]) -> np.ndarray:
    """librosa filters.mel(sr, n_fft, n_mels, fmin, fmax) (htk=False, norm=1, float32):
    triangles in float64 stored to float32, then scaled in place by 2/(f[i+2]-f[i])."""
    fmax = float(sr) / 2 if fmax is None else fmax
    nb = 1 + n_fft // 2
    w = np.zeros((n_mels, nb), dtype=np.float32)
    fftf = np.linspace(0, float(sr) / 2, nb, endpoint=True)
    melf = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fd = np.diff(melf)
    ramps = np.subtract.outer(melf, fftf)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fd[i], ramps[i + 2] / fd[i + 1]))
    w *= (2.0 / (melf[2:n_mels + 2] - melf[:n_mels]))[:, None]
    return w


class DspPlan:
    """Device constants of one DSP configuration (built once per device)."""

    def __init__(self, sr: int, n_fft: int, hop: int, win_length: int, n_mels: int,
                 fmin: float, fmax: float, device) -> None:
        if n_fft & (n_fft - 1) or not 16 <= n_fft <= 4096:
            raise ValueError('n_fft must be a power of two in [16, 4096]')
        self.n_fft, self.hop, self.n_mels, self.nb = n_fft, hop, n_mels, n_fft // 2 + 1
        dev = torch.device(device)
        win = scipy.signal.get_window('hann', win_length, fftbins=True)
        lp = (n_fft - win_length) // 2
        win = np.pad(win, (lp, n_fft - win_length - lp))
        tw = np.exp(-2j * np.pi * np.arange(n_fft // 2) / n_fft)
        A = mel_basis(sr, n_fft, n_mels, fmin, fmax)
        nz = A > 0
        lo = np.array([np.argmax(r) if r.any() else 0 for r in nz], dtype=np.int32)
        hi = np.array([len(r) - np.argmax(r[::-1]) if r.any() else 0 for r in nz], dtype=np.int32)
        rowptr = np.zeros(n_mels + 1, dtype=np.int32)
        rowptr[1:] = np.cumsum(hi - lo)
        vals = np.concatenate([A[i, lo[i]:hi[i]] for i in range(n_mels)]).astype(np.float32)
        bin_rows = np.full((self.nb, 2), -1, dtype=np.int32)
        bin_w = np.zeros((self.nb, 2), dtype=np.float32)
        for k in range(self.nb):
            rows = [i for i in range(n_mels) if lo[i] <= k < hi[i]]
            if len(rows) > 2:
                raise ValueError('mel filterbank with more than two filters per bin')
            for j, i in enumerate(rows):
                bin_rows[k, j], bin_w[k, j] = i, A[i, k]
        A64 = A.astype(np.float64)
        self.inv_L = float(1.0 / np.linalg.norm(A64, 2) ** 2)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.window = t(win.astype(np.float64))
        self.win_sq = t((win ** 2).astype(np.float64))
        self.twiddle = t(np.stack([tw.real, tw.imag], -1).astype(np.float64))
        self.basis_np = A
        self.basis = t(A)
        self.mel_lo, self.mel_hi = t(lo), t(hi)
        self.nnz = int(rowptr[-1])
        self.rowvals, self.rowptr, self.rowlo = t(vals), t(rowptr), t(lo)
        self.bin_rows, self.bin_w = t(bin_rows), t(bin_w)
        pinv64 = np.linalg.pinv(A64)
        self.pinv = t(pinv64.astype(np.float32))
        self.pinv64 = t(pinv64)
        # librosa util.nnls block width: MAX_MEM_BLOCK // (n_bins * itemsize of float32)
        self.nnls_cols = max(1, (2 ** 8 * 2 ** 10) // (self.nb * 4))

    def frames(self, n_samples: int) -> int:
        return 1 + n_samples // self.hop


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('forwardtacotron_amd.dsp runs on a HIP device only (got a CPU '
                               'tensor); there is no CPU fallback')


# --- device entry points ---------------------------------------------------------------------

def stft(plan: DspPlan, y: torch.Tensor, lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Complex STFT of audio rows y (B, L): (B, F, n_fft/2+1) complex64, frame-major."""
    _need_cuda(y, lengths)
    B, L = y.shape
    F = plan.frames(L)
    X = torch.empty(B, F, plan.nb, dtype=torch.complex64, device=y.device)
    launch('ftmi_stft', f'stft[B={B},F={F},n={plan.n_fft}]', 0, 4.0 * B * L + 8.0 * B * F * plan.nb,
           y.data_ptr(), y.stride(0), B, L, _p(lengths), plan.n_fft, plan.hop,
           plan.window.data_ptr(), plan.twiddle.data_ptr(), F, None, X.data_ptr(), _stream())
    return X


def mel_spectrogram(plan: DspPlan, y: torch.Tensor, lengths: Optional[torch.Tensor] = None,
                    log_norm: bool = True) -> torch.Tensor:
    """Batched DSP.wav_to_mel: audio rows (B, L) float32 -> (B, n_mels, 1 + L // hop)."""
    _need_cuda(y, lengths)
    if y.dtype != torch.float32 or y.dim() != 2 or y.stride(1) != 1:
        raise ValueError('audio rows (B, L) float32 with unit stride expected')
    B, L = y.shape
    F = plan.frames(L)
    mel = torch.empty(B, plan.n_mels, F, device=y.device)
    launch('ftmi_mel_spectrogram', f'mel_spectrogram[B={B},F={F},n={plan.n_fft}]', 0,
           4.0 * B * L + 4.0 * B * F * plan.n_mels,
           y.data_ptr(), y.stride(0), B, L, _p(lengths), plan.n_fft, plan.hop,
           plan.window.data_ptr(), plan.twiddle.data_ptr(), F, None, plan.basis.data_ptr(),
           plan.mel_lo.data_ptr(), plan.mel_hi.data_ptr(), plan.n_mels, int(log_norm),
           mel.data_ptr(), _stream())
    return mel


def istft(plan: DspPlan, X: torch.Tensor, frames: Optional[torch.Tensor] = None,
          y_len: Optional[int] = None, work: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, F, nb) complex64 frame-major -> audio rows (B, hop*(F-1)) (item b valid for
    hop*(frames[b]-1) samples, zero after)."""
    _need_cuda(X, frames)
    B, F, nb = X.shape
    if nb != plan.nb or X.dtype != torch.complex64 or not X.is_contiguous():
        raise ValueError('contiguous (B, F, n_fft/2+1) complex64 expected')
    y_len = plan.hop * (F - 1) if y_len is None else y_len
    y = torch.empty(B, max(y_len, 1), device=X.device)
    if work is None:
        work = torch.empty(_lib.load().ftmi_istft_workspace_bytes(B, F, plan.n_fft),
                           dtype=torch.uint8, device=X.device)
    launch('ftmi_istft', f'istft[B={B},F={F},n={plan.n_fft}]', 0,
           8.0 * B * F * nb + 16.0 * B * F * plan.n_fft + 4.0 * B * y_len,
           X.data_ptr(), B, F, _p(frames), plan.n_fft, plan.hop, plan.window.data_ptr(),
           plan.win_sq.data_ptr(), plan.twiddle.data_ptr(), work.data_ptr(), y.data_ptr(),
           y.stride(0), y_len, _stream())
    return y[:, :y_len]


NNLS_METHODS = ('lbfgsb', 'fista')
NNLS_GROUPS = 32  # workgroups per L-BFGS-B block (fixed: the sums, hence S, do not depend on
                  # how many blocks share a launch)
NNLS_WS_CAP = 4 << 30  # workspace bytes per launch chunk


def mel_to_stft(plan: DspPlan, mel: torch.Tensor, frames: Optional[torch.Tensor] = None,
                denorm: bool = True, iters: int = 32, method: str = 'lbfgsb') -> torch.Tensor:
    """librosa feature.inverse.mel_to_stft(power=1) of (B, n_mels, F) (log-)mels:
    (B, F, nb) float32 non-negative magnitudes, frame-major.

    method 'lbfgsb' (default) runs the reference's own NNLS on the device — util.nnls'
    L-BFGS-B over 127-frame blocks, same iterates to rounding (ftmi_nnls_lbfgsb_*) — so S is
    the reference's S.  'fista' is the fast per-frame solver (`iters` FISTA steps, default
    32): a
    minimiser of the same objective, but the minimiser is not unique, so its S (and the
    Griffin-Lim wav built on it) is NOT the reference's (tests/test_gpu_dsp.py states by how
    much)."""
    _need_cuda(mel, frames)
    if mel.dtype != torch.float32 or not mel.is_contiguous() or mel.size(1) != plan.n_mels:
        raise ValueError('contiguous (B, n_mels, F) float32 expected')
    if method not in NNLS_METHODS:
        raise ValueError(f'method must be one of {NNLS_METHODS}')
    B, _, F = mel.shape
    if method == 'lbfgsb':
        return _nnls_lbfgsb(plan, mel, frames, denorm)
    S = torch.empty(B, F, plan.nb, device=mel.device)
    launch('ftmi_mel_nnls', f'mel_nnls[B={B},F={F},iters={iters}]', 0,
           4.0 * B * F * (plan.n_mels + plan.nb),
           mel.data_ptr(), B, F, _p(frames), plan.n_mels, plan.nb, int(denorm), plan.nnz,
           plan.rowvals.data_ptr(), plan.rowptr.data_ptr(), plan.rowlo.data_ptr(),
           plan.bin_rows.data_ptr(), plan.bin_w.data_ptr(), plan.pinv.data_ptr(),
           ctypes.c_float(plan.inv_L), iters, S.data_ptr(), _stream())
    return S


def _nnls_lbfgsb(plan: DspPlan, mel: torch.Tensor, frames: Optional[torch.Tensor],
                 denorm: bool, maxiter: int = 0, info: Optional[list] = None,
                 debug: Optional[dict] = None) -> torch.Tensor:
    """The host loop around ftmi_nnls_lbfgsb_* — what scipy's fmin_l_bfgs_b driver is around
    setulb: start, then cycles (every block advances one L-BFGS-B iteration or one extra
    line-search evaluation per cycle) until the device's count of running blocks reads 0.
    Blocks as librosa 0.7.2 util.nnls cuts them (127 frames of each item's mel).  maxiter:
    scipy's (0: 15000); info: a list that receives per block (iterations, f evaluations, f,
    projected-gradient norm); debug (tools/nnls_diag.py): {'stop': 16 * iteration + phase}
    ends the blocks there and receives the workspace and its geometry."""
    lib = _lib.load()
    B, _, F = mel.shape
    dev = mel.device
    fr = [F] * B if frames is None else [min(int(v), F) for v in frames.cpu().tolist()]
    nc = plan.nnls_cols
    blocks = [(b, s0, min(nc, fb - s0), 0) for b, fb in enumerate(fr) for s0 in range(0, fb, nc)]
    S = torch.empty(B, F, plan.nb, device=dev)
    fr_dev = None if frames is None else frames.to(device=dev, dtype=torch.int32)
    if not blocks:
        S.zero_()
        return S
    stream = _stream()
    m = 32
    i = 0
    while i < len(blocks):
        per = lib.ftmi_nnls_lbfgsb_workspace_bytes(1, plan.nb, nc, m, NNLS_GROUPS)
        nblk = max(1, min(len(blocks) - i, NNLS_WS_CAP // per))
        chunk = blocks[i:i + nblk]
        ws = torch.empty(per * nblk, dtype=torch.uint8, device=dev)
        bt = torch.tensor(chunk, dtype=torch.int32, device=dev)
        active = torch.full((1,), nblk, dtype=torch.int32, device=dev)
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        a = _lib.NnlsArgs(mel.data_ptr(), B, F, plan.n_mels, plan.nb, int(denorm), bt.data_ptr(),
                          nblk, NNLS_GROUPS, m, nc, maxiter, (debug or {}).get('stop', 0),
                          plan.rowvals.data_ptr(), plan.rowptr.data_ptr(),
                          plan.rowlo.data_ptr(), plan.bin_rows.data_ptr(), plan.bin_w.data_ptr(),
                          plan.pinv64.data_ptr(), ws.data_ptr(), S.data_ptr(), active.data_ptr())
        ap = ctypes.byref(a)
        launch('ftmi_nnls_lbfgsb_start', f'nnls_lbfgsb_start[blocks={nblk}]', 0, 0, ap, stream)
        cycles, step = 0, 4
        while True:
            launch('ftmi_nnls_lbfgsb_cycles', f'nnls_lbfgsb_cycles[blocks={nblk}]', 0, 0, ap, step,
                   stream)
            cycles += step
            if int(active.item()) == 0:
                break
            if cycles > 20 * 15000:
                raise RuntimeError('L-BFGS-B NNLS did not finish')
            step = min(2 * step, 64)
        inf = torch.zeros(nblk, 4, dtype=torch.float64, device=dev)
        launch('ftmi_nnls_lbfgsb_finish', f'nnls_lbfgsb_finish[blocks={nblk}]', 0, 0, ap,
               _p(fr_dev), status.data_ptr(), inf.data_ptr(), stream)
        st = status.cpu().tolist()
        if st[0] & 4 and m < plan.nb:
            # history full (more than 32 updates: the synthetic-weights mels of the tests take
            # ~150): rerun the chunk with the reference's whole history, m = n_bins
            m = plan.nb
            continue
        if st[0] and debug is None:
            raise RuntimeError(f'L-BFGS-B NNLS failed (status {st[0]}: 2 abnormal line search, '
                               '4 history wrap, 8 equal breakpoints, 16 maxiter)')
        if info is not None:
            info.extend(inf.cpu().tolist())
        if debug is not None:
            debug.update(ws=ws, m=m, groups=NNLS_GROUPS, per=per, n_pad=(plan.nb * nc + 255) // 256 * 256)
        i += nblk
    return S


def griffinlim_from_stft(plan: DspPlan, S: torch.Tensor, angles: torch.Tensor, n_iter: int = 32,
                         frames: Optional[torch.Tensor] = None, momentum: float = 0.99) -> torch.Tensor:
    """librosa core.griffinlim (0.7.2 fast GL) of magnitudes S (B, F, nb) from initial unit
    phases `angles` (B, F, nb) complex64 -> audio rows (B, hop*(F-1)).  (A HIP-graph replay of
    this loop measured no faster at batch 1 — 5.98 vs 5.65 ms per gen_forward sentence step:
    the kernels, not the launches, set the pace — so it stays eager.)"""
    _need_cuda(S, angles, frames)
    return _gl_loop(plan, S, angles, n_iter, frames, momentum)


def _gl_fused(plan: DspPlan) -> bool:
    """The one-launch-per-iteration kernels (ftmi_griffinlim_iter / ftmi_istft_fused) cover the
    reference configuration n_fft = 1024, hop = 256, at every batch size, so an item's audio
    does not depend on the batch it is in.  (At batch 1 the three-kernel path is ~10 % faster:
    c2's 102 eight-frame tiles leave most CUs idle, 1.01 vs 0.92 ms per 32 iterations,
    tools/gl_bench.py.)  FTMI_GL_FUSED=0 keeps the three-kernel path (A/B runs, tests)."""
    return plan.n_fft == 1024 and plan.hop == 256 and os.environ.get('FTMI_GL_FUSED', '1') != '0'


def _gl_loop(plan: DspPlan, S: torch.Tensor, angles: torch.Tensor, n_iter: int,
             frames: Optional[torch.Tensor], momentum: float) -> torch.Tensor:
    B, F, nb = S.shape
    dev = S.device
    X = torch.empty(B, F, nb, dtype=torch.complex64, device=dev)
    launch('ftmi_spec_mul', f'spec_mul[n={S.numel()}]', 0, 20.0 * S.numel(),
           S.data_ptr(), angles.data_ptr(), S.numel(), X.data_ptr(), _stream())
    tprev = torch.empty_like(X)
    L = plan.hop * (F - 1)
    c = float(np.float32(momentum / (1 + momentum)))
    if _gl_fused(plan):
        # algorithmic bytes per iteration: X read, S read, tprev read + written, X written
        # (36 B per bin; the halo frames' re-reads of X are not counted)
        X2 = torch.empty_like(X)
        for it in range(n_iter):
            launch('ftmi_griffinlim_iter', f'gl_iter[B={B},F={F}]', 0, 36.0 * S.numel(),
                   X.data_ptr(), X2.data_ptr(), S.data_ptr(), tprev.data_ptr(), B, F, _p(frames),
                   plan.n_fft, plan.hop, plan.window.data_ptr(), plan.win_sq.data_ptr(),
                   plan.twiddle.data_ptr(), ctypes.c_float(c), int(it == 0), _stream())
            X, X2 = X2, X
        y = torch.empty(B, max(L, 1), device=dev)
        launch('ftmi_istft_fused', f'istft_fused[B={B},F={F}]', 0, 8.0 * S.numel() + 4.0 * B * L,
               X.data_ptr(), B, F, _p(frames), plan.n_fft, plan.hop, plan.window.data_ptr(),
               plan.win_sq.data_ptr(), plan.twiddle.data_ptr(), y.data_ptr(), y.stride(0), L,
               _stream())
        return y[:, :L]
    work = torch.empty(_lib.load().ftmi_istft_workspace_bytes(B, F, plan.n_fft), dtype=torch.uint8,
                       device=dev)
    lengths = None if frames is None else (plan.hop * (frames - 1)).to(torch.int32)
    for it in range(n_iter):
        y = istft(plan, X, frames, L, work)
        launch('ftmi_griffinlim_stft', f'gl_stft[B={B},F={F}]', 0, 4.0 * B * L + 28.0 * S.numel(),
               y.data_ptr(), y.stride(0), B, max(L, 1), _p(lengths), plan.n_fft, plan.hop,
               plan.window.data_ptr(), plan.twiddle.data_ptr(), F, _p(frames), S.data_ptr(),
               tprev.data_ptr(), ctypes.c_float(c), int(it == 0), X.data_ptr(), _stream())
    return istft(plan, X, frames, L, work)


# --- the reference class ---------------------------------------------------------------------

class DSP:
    """`utils/dsp.py:12-57`: same constructor arguments and attributes."""

    def __init__(self, num_mels: int, sample_rate: int, hop_length: int, win_length: int,
                 n_fft: int, fmin: float, fmax: float, peak_norm: bool,
                 trim_start_end_silence: bool, trim_silence_top_db: int, pitch_max_freq: int,
                 trim_long_silences: bool, vad_sample_rate: int, vad_window_length: float,
                 vad_moving_average_width: float, vad_max_silence_length: int, bits: int,
                 mu_law: bool, voc_mode: str) -> None:
        self.n_mels = num_mels
        self.sample_rate = sample_rate
        self.hop_length = hop_length
        self.win_length = win_length
        self.n_fft = n_fft
        self.fmin = fmin
        self.fmax = fmax
        self.should_peak_norm = peak_norm
        self.should_trim_start_end_silence = trim_start_end_silence
        self.should_trim_long_silences = trim_long_silences
        self.trim_silence_top_db = trim_silence_top_db
        self.pitch_max_freq = pitch_max_freq
        self.vad_sample_rate = vad_sample_rate
        self.vad_window_length = vad_window_length
        self.vad_moving_average_width = vad_moving_average_width
        self.vad_max_silence_length = vad_max_silence_length
        self.bits = bits
        self.mu_law = mu_law
        self.voc_mode = voc_mode
        self._plans: Dict[Any, DspPlan] = {}
        # FISTA steps of the fast solver: 32 fit the mel 100x closer than the reference's own
        # L-BFGS-B stops (relative residual ~3e-7 against ~4e-5 on speech; 200 steps: 1e-14)
        self.nnls_iters = 32
        # 'lbfgsb': the reference's NNLS (librosa util.nnls), reproduced; 'fista': the fast
        # per-frame solver (another minimiser of the same objective, not the reference's S)
        self.nnls = 'lbfgsb'

    @classmethod
    def from_config(cls, config: Dict[str, Any]) -> 'DSP':
        return DSP(**config['dsp'])

    def plan(self, device=None) -> DspPlan:
        dev = torch.device(device if device is not None else 'cuda')
        if dev.type != 'cuda':
            raise RuntimeError('forwardtacotron_amd.dsp runs on a HIP device only')
        if dev.index is None:
            dev = torch.device('cuda', torch.cuda.current_device())
        if dev not in self._plans:
            self._plans[dev] = DspPlan(self.sample_rate, self.n_fft, self.hop_length,
                                       self.win_length, self.n_mels, self.fmin, self.fmax, dev)
        return self._plans[dev]

    # -- I/O (utils/dsp.py:62-69) --
    def load_wav(self, path: Union[str, Path]) -> np.ndarray:
        """16-bit / float WAV at `sample_rate` (the reference resamples with librosa,
        which is absent: other rates raise)."""
        import scipy.io.wavfile
        sr, wav = scipy.io.wavfile.read(str(path))
        if sr != self.sample_rate:
            raise ValueError(f'{path}: sample rate {sr} != {self.sample_rate} (no resampler)')
        if wav.dtype == np.int16:
            wav = wav.astype(np.float32) / 32768.0
        elif wav.dtype == np.int32:
            wav = wav.astype(np.float32) / 2147483648.0
        wav = wav.astype(np.float32)
        return wav.mean(axis=1) if wav.ndim == 2 else wav

    def save_wav(self, wav: np.ndarray, path: Union[str, Path]) -> None:
        """16-bit PCM WAV (soundfile's default subtype for .wav)."""
        wav = np.asarray(wav, dtype=np.float32)
        pcm = np.clip(np.round(wav * 32767.0), -32768, 32767).astype('<i2')
        with wave.open(str(path), 'wb') as f:
            f.setnchannels(1)
            f.setsampwidth(2)
            f.setframerate(self.sample_rate)
            f.writeframes(pcm.tobytes())

    # -- analysis / synthesis (utils/dsp.py:71-103) --
    def wav_to_mel(self, y, normalize: bool = True):
        """|STFT| -> mel -> log(clip 1e-5).  numpy (L,) -> numpy (n_mels, 1 + L // hop) like
        the reference; a HIP tensor (L,) or (B, L) returns a tensor."""
        if isinstance(y, torch.Tensor):
            _need_cuda(y)
            yy = y.float().reshape(-1, y.shape[-1]).contiguous()
            mel = mel_spectrogram(self.plan(y.device), yy, log_norm=normalize)
            return mel[0] if y.dim() == 1 else mel
        y = np.asarray(y)
        if not np.issubdtype(y.dtype, np.floating) or y.ndim != 1:
            raise ValueError('mono floating-point audio expected')
        t = torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).cuda()[None]
        return mel_spectrogram(self.plan(t.device), t, log_norm=normalize)[0].cpu().numpy()

    def draw_uniforms(self, T: int, random_state=None) -> np.ndarray:
        """The U[0, 1) draw behind griffinlim's initial phases for a T-frame mel, taken from
        the reference's stream (librosa: np.random.rand(n_bins, T), or RandomState
        (random_state)).  Drawn ahead by a caller that has other work to overlap, and passed
        as griffinlim(..., uniforms=u), it is the same draw in the same stream order.
        (gen_forward does not: generate() returns after its end-of-call status read, so no
        device work is left to hide the draw behind; griffinlim queues the NNLS first and
        draws while it runs.)"""
        rng = np.random if random_state is None else np.random.RandomState(random_state)
        return rng.rand(self.n_fft // 2 + 1, T)

    def griffinlim(self, mel, n_iter: int = 32, angles=None, random_state=None, uniforms=None,
                   nnls: Optional[str] = None):
        """exp -> mel_to_stft (NNLS) -> fast Griffin-Lim (32 iterations, momentum 0.99).
        numpy (n_mels, T) -> numpy wav of hop * (T - 1) samples.  The initial phases are
        exp(2 pi i U[0,1)) drawn like librosa (np.random, or RandomState(random_state)),
        shape (n_bins, T); pass `uniforms` (draw_uniforms) to use a draw made ahead, or
        `angles` to fix the phases.  nnls: 'lbfgsb' (the reference's magnitudes; default
        self.nnls) or 'fista' (fast, another minimiser)."""
        is_t = isinstance(mel, torch.Tensor)
        if is_t:
            m, denorm = mel, True  # exp on the device
        else:
            # numpy in, as the reference: its own denormalize (np.exp, float32) on the host, so
            # the NNLS sees the reference's M bit for bit (80 x T exps: microseconds)
            m = torch.from_numpy(np.exp(np.ascontiguousarray(mel, dtype=np.float32))).cuda()
            denorm = False
        _need_cuda(m)
        plan = self.plan(m.device)
        T = m.shape[-1]
        # the NNLS magnitudes first: queued on the device, they run while the host draws the
        # initial phases below (the draw does not depend on them)
        S = mel_to_stft(plan, m.float().reshape(1, plan.n_mels, T).contiguous(), denorm=denorm,
                        iters=self.nnls_iters, method=nnls or self.nnls)
        if angles is None:
            # the reference's draw (librosa: np.random.rand(n_bins, T)); exp(2 pi i u) and the
            # frame-major layout on the device (ftmi_unit_phases: the host exp of 420 k
            # complex values took longer than the whole Griffin-Lim on the GPU)
            if uniforms is None:
                uniforms = self.draw_uniforms(T, random_state)
            if tuple(np.shape(uniforms)) != (plan.nb, T):
                raise ValueError(f'uniforms of shape {np.shape(uniforms)}, expected {(plan.nb, T)}')
            u = torch.from_numpy(np.ascontiguousarray(uniforms, dtype=np.float64)).to(m.device)
            a = torch.empty(1, T, plan.nb, dtype=torch.complex64, device=m.device)
            launch('ftmi_unit_phases', f'unit_phases[T={T}]', 0, 16.0 * plan.nb * T,
                   u.data_ptr(), 1, plan.nb, T, a.data_ptr(), _stream())
        else:
            a = angles if isinstance(angles, torch.Tensor) else torch.from_numpy(
                np.ascontiguousarray(np.asarray(angles, dtype=np.complex64).T))
            a = a.to(m.device).reshape(1, T, plan.nb).contiguous()
        wav = griffinlim_from_stft(plan, S, a, n_iter)[0]
        return wav if is_t else wav.cpu().numpy()

    def griffinlim_batch(self, mel: torch.Tensor, frames: Optional[torch.Tensor] = None,
                         n_iter: int = 32, generator: Optional[torch.Generator] = None,
                         nnls: Optional[str] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Batched Griffin-Lim of (B, n_mels, F) device mels (item b uses its first
        frames[b] frames): returns (wav (B, hop*(F-1)), samples per item).  Initial phases
        from torch's generator on the device."""
        _need_cuda(mel, frames)
        plan = self.plan(mel.device)
        B, _, F = mel.shape
        fr = None if frames is None else frames.to(device=mel.device, dtype=torch.int32)
        u = torch.rand(B, plan.nb, F, dtype=torch.float64, device=mel.device, generator=generator)
        angles = torch.empty(B, F, plan.nb, dtype=torch.complex64, device=mel.device)
        launch('ftmi_unit_phases', f'unit_phases[B={B},T={F}]', 0, 16.0 * B * plan.nb * F,
               u.data_ptr(), B, plan.nb, F, angles.data_ptr(), _stream())
        S = mel_to_stft(plan, mel.float().contiguous(), fr, iters=self.nnls_iters, method=nnls or self.nnls)
        wav = griffinlim_from_stft(plan, S, angles, n_iter, fr)
        n = plan.hop * ((fr if fr is not None else torch.full((B,), F, device=mel.device)) - 1)
        return wav, n

    # -- utils/dsp.py:105-110 --
    def normalize(self, mel):
        if isinstance(mel, torch.Tensor):
            return torch.log(torch.clamp(mel, min=1e-5))
        return np.log(np.clip(mel, a_min=1.e-5, a_max=None))

    def denormalize(self, mel):
        return torch.exp(mel) if isinstance(mel, torch.Tensor) else np.exp(mel)

    def trim_silence(self, wav: np.ndarray) -> np.ndarray:
        raise NotImplementedError('trim_silence needs librosa.effects (absent); preprocessing '
                                  'is outside the inference path')

    def trim_long_silences(self, wav: np.ndarray) -> np.ndarray:
        raise NotImplementedError('trim_long_silences needs webrtcvad (absent); preprocessing '
                                  'is outside the inference path')

    # -- utils/dsp.py:143-165 (vocoder label helpers) --
    @staticmethod
    def label_2_float(x: np.ndarray, bits: float) -> np.ndarray:
        return 2 * x / (2 ** bits - 1.) - 1.

    @staticmethod
    def float_2_label(x: np.ndarray, bits: float) -> np.ndarray:
        assert abs(x).max() <= 1.0
        x = (x + 1.) * (2 ** bits - 1) / 2
        return x.clip(0, 2 ** bits - 1)

    @staticmethod
    def encode_mu_law(x: np.ndarray, mu: float) -> np.ndarray:
        mu = mu - 1
        fx = np.sign(x) * np.log(1 + mu * np.abs(x)) / np.log(1 + mu)
        return np.floor((fx + 1) / 2 * mu + 0.5)

    @staticmethod
    def decode_mu_law(y: np.ndarray, mu: float, from_labels: bool = True) -> np.ndarray:
        if from_labels:
            y = DSP.label_2_float(y, np.log2(mu))
        mu = mu - 1
        return np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)
