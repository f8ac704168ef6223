"""ORACLE — test infrastructure only, never shipped or measured as the product.

A numpy/scipy restatement of the reference's audio path, `utils/dsp.py` (DSP.wav_to_mel
:71-87, normalize :105-107, griffinlim :89-103, denormalize :109-110).  The arithmetic
lives in the third-party dependency **librosa==0.7.2** (pinned at the reference's
`requirements.txt:2`), which is absent from this image; its published algorithms are
restated here function by function (names follow librosa's):

    scipy.signal.get_window / librosa.util.pad_center / util.frame / core.stft /
    core.istft / filters.window_sumsquare / filters.mel (+ mel_frequencies, hz_to_mel,
    mel_to_hz, fft_frequencies) / feature.melspectrogram(S=...) / util.nnls (L-BFGS-B
    blocks of MAX_MEM_BLOCK bytes) / feature.inverse.mel_to_stft / core.griffinlim.

librosa 0.7.2 runs on numpy 1.x, whose numpy.fft computes in float64 whatever the input
precision, and stores into the caller's dtype (complex64 spectra, float32 audio).  numpy
2.x keeps complex64 in single precision, so every FFT here casts to float64 first.

Pinning (tests/test_oracle_dsp.py): the reference's own fixture
`tests/resources/test_mel.npy` (80 x 40, float32) pins the frame count (center=True:
40 = 1 + 10000 // 256) and the log-clip floor (min = log 1e-5).  Its input,
`librosa.util.example_audio_file()`, is not in the image, so the STFT / mel values are
**partially pinned**; Griffin-Lim has no reference test and an unseeded random init
upstream — **parity unpinned** beyond its deterministic restatement (explicit init phases).
"""
from __future__ import annotations

import numpy as np
import scipy.optimize
import scipy.signal

MAX_MEM_BLOCK = 2 ** 8 * 2 ** 10  # librosa.util.MAX_MEM_BLOCK (bytes)


# --- windows / framing --------------------------------------------------------------------

def get_window(win_length: int) -> np.ndarray:
    """scipy.signal.get_window('hann', N, fftbins=True): periodic Hann, float64."""
    return scipy.signal.get_window('hann', win_length, fftbins=True)


def pad_center(w: np.ndarray, size: int) -> np.ndarray:
    """librosa.util.pad_center: zero-pad symmetrically to `size`."""
    lpad = (size - w.shape[-1]) // 2
    return np.pad(w, (lpad, size - w.shape[-1] - lpad))


def frame(y: np.ndarray, frame_length: int, hop_length: int) -> np.ndarray:
    """librosa.util.frame: (frame_length, n_frames) strided view."""
    n_frames = 1 + (len(y) - frame_length) // hop_length
    return np.lib.stride_tricks.as_strided(
        y, shape=(frame_length, n_frames), strides=(y.itemsize, hop_length * y.itemsize))


# --- STFT / ISTFT ----------------------------------------------------------------------------

def stft(y: np.ndarray, n_fft: int = 1024, hop_length: int = 256, win_length: int = 1024,
         center: bool = True) -> np.ndarray:
    """librosa.core.stft (0.7.2), window 'hann', pad_mode 'reflect', dtype complex64:
    rfft(window(f64) * frame) computed in float64 and stored as complex64."""
    w = pad_center(get_window(win_length), n_fft).reshape(-1, 1)
    if center:
        y = np.pad(y, n_fft // 2, mode='reflect')
    fr = frame(np.ascontiguousarray(y), n_fft, hop_length)
    out = np.empty((1 + n_fft // 2, fr.shape[1]), dtype=np.complex64, order='F')
    n_columns = int(MAX_MEM_BLOCK / (out.shape[0] * out.itemsize))
    for s in range(0, out.shape[1], n_columns):
        t = min(s + n_columns, out.shape[1])
        out[:, s:t] = np.fft.rfft(w * fr[:, s:t].astype(np.float64), axis=0)
    return out


def window_sumsquare(n_frames: int, hop_length: int, win_length: int, n_fft: int,
                     dtype=np.float32) -> np.ndarray:
    """librosa.filters.window_sumsquare (norm=None): float32 envelope, frames added in order."""
    n = n_fft + hop_length * (n_frames - 1)
    x = np.zeros(n, dtype=dtype)
    win_sq = pad_center(get_window(win_length) ** 2, n_fft)
    for i in range(n_frames):
        s = i * hop_length
        x[s:min(n, s + n_fft)] += win_sq[:max(0, min(n_fft, n - s))]
    return x


def istft(X: np.ndarray, hop_length: int = 256, win_length: int = 1024,
          center: bool = True, dtype=np.float32) -> np.ndarray:
    """librosa.core.istft (0.7.2): per-frame irfft (float64) * window, overlap-added into a
    float32 signal in frame order, divided by the window sum-square where > tiny, cropped
    by n_fft // 2 on both sides when centered."""
    n_fft = 2 * (X.shape[0] - 1)
    w = pad_center(get_window(win_length), n_fft)
    n_frames = X.shape[1]
    y = np.zeros(n_fft + hop_length * (n_frames - 1), dtype=dtype)
    for i in range(n_frames):
        s = i * hop_length
        ytmp = w * np.fft.irfft(X[:, i].astype(np.complex128), n=n_fft)
        y[s:s + n_fft] = y[s:s + n_fft] + ytmp
    wss = window_sumsquare(n_frames, hop_length, win_length, n_fft, dtype=dtype)
    nz = wss > np.finfo(wss.dtype).tiny
    y[nz] /= wss[nz]
    if center:
        y = y[n_fft // 2:-(n_fft // 2)]
    return y


# --- mel filterbank ------------------------------------------------------------------------

def hz_to_mel(f):
    """librosa.core.hz_to_mel, Slaney (htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        t = f >= min_log_hz
        mels[t] = min_log_mel + np.log(f[t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(m):
    """librosa.core.mel_to_hz, Slaney (htk=False)."""
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        t = m >= min_log_mel
        freqs[t] = min_log_hz * np.exp(logstep * (m[t] - min_log_mel))
    elif m >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel_frequencies(n_mels: int, fmin: float, fmax: float) -> np.ndarray:
    return mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels))


def mel_filters(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float,
                dtype=np.float32) -> np.ndarray:
    """librosa.filters.mel (htk=False, norm=1 Slaney area normalisation): triangles built in
    float64, stored into `dtype`, then scaled in place by 2 / (f[i+2] - f[i])."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=dtype)
    fftfreqs = np.linspace(0, float(sr) / 2, 1 + n_fft // 2, endpoint=True)
    mel_f = mel_frequencies(n_mels + 2, fmin, fmax)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


# --- DSP (utils/dsp.py) -----------------------------------------------------------------------

def wav_to_mel(y: np.ndarray, sr=22050, n_fft=1024, hop_length=256, win_length=1024,
               n_mels=80, fmin=0, fmax=8000, normalize=True) -> np.ndarray:
    """utils/dsp.py:71-87: |stft| (magnitude, complex64 abs) -> mel_basis @ S (float32 dot;
    `S=` is passed, so no power) -> log(clip(., 1e-5)) (`normalize` :105-107)."""
    spec = np.abs(stft(y, n_fft, hop_length, win_length))
    mel = np.dot(mel_filters(sr, n_fft, n_mels, fmin, fmax), spec)
    if normalize:
        mel = np.log(np.clip(mel, 1e-5, None))
    return mel


def _nnls_obj(x, shape, A, B):
    x = x.reshape(shape)
    diff = np.dot(A, x) - B
    return 0.5 * np.sum(diff ** 2), np.dot(A.T, diff).flatten()


def _nnls_lbfgs_block(A, B, x_init=None):
    if x_init is None:
        x_init = np.linalg.lstsq(A, B, rcond=None)[0]
        np.clip(x_init, 0, None, out=x_init)
    shape = x_init.shape
    x, _, _ = scipy.optimize.fmin_l_bfgs_b(_nnls_obj, x_init, args=(shape, A, B),
                                           bounds=[(0, None)] * x_init.size, m=A.shape[1])
    return x.reshape(shape)


def nnls(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """librosa.util.nnls (0.7.2): min ||A x - B||, x >= 0, by L-BFGS-B (history m = A's
    columns) over blocks of MAX_MEM_BLOCK // (513 * 4) = 127 frames, started from the
    clipped least-squares solution."""
    n_columns = int(MAX_MEM_BLOCK // (A.shape[-1] * A.itemsize))
    if B.shape[-1] <= n_columns:
        return _nnls_lbfgs_block(A, B).astype(A.dtype)
    x = np.linalg.lstsq(A, B, rcond=None)[0].astype(A.dtype)
    np.clip(x, 0, None, out=x)
    x_init = x
    for s in range(0, x.shape[-1], n_columns):
        t = min(s + n_columns, B.shape[-1])
        x[:, s:t] = _nnls_lbfgs_block(A, B[:, s:t], x_init=x_init[:, s:t])
    return x


def mel_to_stft(M: np.ndarray, sr=22050, n_fft=1024, fmin=0, fmax=8000) -> np.ndarray:
    """librosa.feature.inverse.mel_to_stft(power=1): nnls(mel_basis(dtype=M.dtype), M)."""
    A = mel_filters(sr, n_fft, M.shape[0], fmin, fmax, dtype=M.dtype)
    return nnls(A, M)


def griffinlim_from_stft(S: np.ndarray, angles0: np.ndarray, n_iter=32, hop_length=256,
                         win_length=1024, momentum=0.99) -> np.ndarray:
    """librosa.core.griffinlim (0.7.2, fast GL): `angles0` (complex64, |.| = 1) replaces
    the upstream unseeded np.random init exp(2 pi i U[0,1))."""
    n_fft = 2 * (S.shape[0] - 1)
    angles = angles0.astype(np.complex64).copy()
    c = np.float32(momentum / (1 + momentum))
    rebuilt = None
    for _ in range(n_iter):
        tprev = rebuilt
        inverse = istft(S * angles, hop_length, win_length)
        rebuilt = stft(inverse, n_fft, hop_length, win_length)
        angles[:] = rebuilt if tprev is None else rebuilt - c * tprev
        angles[:] /= np.abs(angles) + np.float32(1e-16)
    return istft(S * angles, hop_length, win_length)


def random_angles(shape, seed: int) -> np.ndarray:
    """exp(2 pi i U[0,1)) as upstream, from a seeded generator."""
    rng = np.random.RandomState(seed)
    return np.exp(2j * np.pi * rng.rand(*shape)).astype(np.complex64)


def griffinlim(mel: np.ndarray, angles0: np.ndarray, n_iter=32, sr=22050, n_fft=1024,
               hop_length=256, win_length=1024, fmin=0, fmax=8000) -> np.ndarray:
    """utils/dsp.py:89-103: exp (denormalize :109-110) -> mel_to_stft -> griffinlim."""
    S = mel_to_stft(np.exp(mel), sr, n_fft, fmin, fmax)
    return griffinlim_from_stft(S, angles0, n_iter, hop_length, win_length)
