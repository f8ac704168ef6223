"""The audio oracle (oracle/dsp_oracle.py, librosa 0.7.2 restated) against the reference's
own fixture and against the definitions it restates.  CPU only.

Pinning available for utils/dsp.py: `tests/resources/test_mel.npy` of the reference
(copied as tests/golden/ref_test_mel.npy, with the test config's dsp section as
dsp_config.json).  Its input audio (librosa's example file) is absent, so values are not
reproducible: the fixture pins the frame count (center=True) and the log-clip floor —
the STFT / mel path is PARTIALLY pinned; Griffin-Lim is parity-unpinned upstream (no
test, unseeded init) and is checked here through its deterministic restatement."""
import json

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import dsp_oracle as D

CFG = json.loads((GOLDEN / 'dsp_config.json').read_text())['dsp']
REF_MEL = np.load(GOLDEN / 'ref_test_mel.npy', allow_pickle=False)


def test_reference_fixture_pins_framing_and_floor():
    """test_dsp.py:18-23: 10000 samples -> (80, 40) = (n_mels, 1 + 10000 // hop) frames
    (center=True); min == log(1e-5) in float32 (normalize's clip)."""
    assert REF_MEL.shape == (CFG['num_mels'], 1 + 10000 // CFG['hop_length'])
    assert REF_MEL.dtype == np.float32
    assert REF_MEL.min() == np.log(np.float32(1e-5))
    y = np.random.RandomState(0).uniform(-0.5, 0.5, 10000).astype(np.float32)
    y[3000:6000] = 0.0  # digital silence reaches the clip floor like the fixture does
    mel = D.wav_to_mel(y, CFG['sample_rate'], CFG['n_fft'], CFG['hop_length'], CFG['win_length'],
                       CFG['num_mels'], CFG['fmin'], CFG['fmax'])
    assert mel.shape == REF_MEL.shape and mel.dtype == np.float32
    assert mel.min() == REF_MEL.min()


def test_stft_is_windowed_rfft_of_reflect_padded_frames():
    y = np.random.RandomState(1).randn(5000).astype(np.float32)
    X = D.stft(y)
    assert X.shape == (513, 1 + 5000 // 256) and X.dtype == np.complex64
    yp = np.pad(y, 512, mode='reflect').astype(np.float64)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(1024) / 1024)
    for f in (0, 7, X.shape[1] - 1):
        ref = np.fft.rfft(yp[f * 256:f * 256 + 1024] * w)
        np.testing.assert_allclose(X[:, f], ref, rtol=1e-6, atol=1e-5)


def test_istft_inverts_stft():
    """hann(1024) at hop 256 satisfies the window-sum-square normalisation: exact
    reconstruction of the analysed signal up to float32 rounding."""
    y = np.random.RandomState(2).randn(6000).astype(np.float32)
    X = D.stft(y)
    yi = D.istft(X)
    assert yi.shape == (256 * (X.shape[1] - 1),) and yi.dtype == np.float32
    np.testing.assert_allclose(yi, y[:len(yi)], atol=2e-6)


def test_window_sumsquare_interior_constant():
    wss = D.window_sumsquare(20, 256, 1024, 1024)
    np.testing.assert_allclose(wss[1024:-1024], 1.5, rtol=1e-6)


def test_mel_filterbank_shape_and_sparsity():
    A = D.mel_filters(CFG['sample_rate'], CFG['n_fft'], CFG['num_mels'], CFG['fmin'], CFG['fmax'])
    assert A.shape == (80, 513) and A.dtype == np.float32
    assert (A >= 0).all()
    assert ((A > 0).sum(0) <= 2).all()  # each bin feeds at most two triangles
    assert (A > 0).any(1).all()         # no empty channel
    # Slaney area normalisation: each triangle integrates to ~1 over Hz (2/width * width/2)
    fft_hz = np.linspace(0, CFG['sample_rate'] / 2, 513)
    area = (A * (fft_hz[1] - fft_hz[0])).sum(1)
    assert np.all(np.abs(area[10:] - 1) < 0.1) and np.all(np.abs(area[60:] - 1) < 0.01)


def test_product_mel_basis_equals_oracle():
    """The device plan's filterbank (host-built constants) is the restatement, bit for bit."""
    from forwardtacotron_amd.dsp import mel_basis
    for sr, n_fft, n_mels, fmin, fmax in [(22050, 1024, 80, 0, 8000), (16000, 512, 40, 50, None)]:
        a = mel_basis(sr, n_fft, n_mels, fmin, fmax)
        b = D.mel_filters(sr, n_fft, n_mels, fmin, fmax)
        np.testing.assert_array_equal(a, b)


def test_nnls_fits_reference_mel():
    M = np.exp(REF_MEL)
    S = D.mel_to_stft(M)
    A = D.mel_filters(22050, 1024, 80, 0, 8000)
    assert S.shape == (513, 40) and S.dtype == np.float32 and (S >= 0).all()
    resid = np.linalg.norm(A.astype(np.float64) @ S - M) / np.linalg.norm(M)
    assert resid < 1e-3


def test_griffinlim_round_trip_on_reference_mel():
    """GL from the reference fixture: wav of hop * (T - 1) samples whose re-analysed log-mel
    is close to the input (measured mean |d log-mel| 0.11 at seed 0)."""
    ang = D.random_angles((513, 40), 0)
    w = D.griffinlim(REF_MEL, ang)
    assert w.shape == (256 * 39,) and w.dtype == np.float32
    m2 = D.wav_to_mel(w)
    assert np.abs(m2 - REF_MEL).mean() < 0.2
    w2 = D.griffinlim(REF_MEL, ang)
    np.testing.assert_array_equal(w, w2)  # deterministic given the init phases
