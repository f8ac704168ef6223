"""ORACLE — test infrastructure only, never shipped or measured as the product.

A numpy restatement of the reference ForwardTacotron inference path
(tarepan/ForwardTacotron, models/forward_tacotron.py + models/common_layers.py), written
from the reference's semantics, one function per reference function (file:line cited).
It is the checker for the HIP path: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it.

Pinning: tests/test_oracle.py checks this module against the golden vectors produced by
the reference itself (tests/golden/make_goldens.py, generate / generate_jit / forward /
LengthRegulator) — parity PINNED for the model path.

Weights are a {state_dict key: np.ndarray} mapping (reference key names).  Activations
follow the reference layouts ((B, C, T) into convs, (B, T, C) into RNNs / linears).
Arithmetic is fp32 by default (dtype=np.float64 gives a higher-precision oracle).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import numpy as np

Params = Dict[str, np.ndarray]


def _p(sd: Params, key: str, dt) -> np.ndarray:
    return np.asarray(sd[key], dtype=dt)


def sigmoid(x):
    with np.errstate(over='ignore'):  # exp(-x) -> inf gives the correct limit 0
        return 1.0 / (1.0 + np.exp(-x))


# --- layers -------------------------------------------------------------------------------

def embedding(ids: np.ndarray, w: np.ndarray) -> np.ndarray:
    """nn.Embedding (forward_tacotron.py:125,304; :31,47)."""
    return w[ids]


def conv1d(x: np.ndarray, w: np.ndarray, pad: int, bias: Optional[np.ndarray] = None) -> np.ndarray:
    """nn.Conv1d stride 1, zero padding `pad` both sides: (B, C, T) -> (B, O, T + 2pad - k + 1)."""
    B, C, T = x.shape
    O, _, k = w.shape
    xp = np.zeros((B, C, T + 2 * pad), dtype=x.dtype)
    xp[:, :, pad:pad + T] = x
    To = T + 2 * pad - k + 1
    out = np.zeros((B, O, To), dtype=x.dtype)
    for j in range(k):
        out += np.matmul(w[:, :, j], xp[:, :, j:j + To])
    if bias is not None:
        out += bias[None, :, None]
    return out


def batchnorm_eval(x, w, b, rm, rv, eps=1e-5):
    """nn.BatchNorm1d in eval mode, channel axis 1."""
    inv = (1.0 / np.sqrt(rv + eps)).astype(x.dtype)
    alpha = inv * w
    beta = b - rm * alpha
    shp = (1, -1) + (1,) * (x.ndim - 2)
    return x * alpha.reshape(shp) + beta.reshape(shp)


def batch_norm_conv(sd: Params, pre: str, x: np.ndarray, relu: bool, dt) -> np.ndarray:
    """BatchNormConv: Conv1d(pad k//2, no bias) -> ReLU? -> BN (common_layers.py:38-52,
    forward_tacotron.py:58-71)."""
    w = _p(sd, pre + '.conv.weight', dt)
    y = conv1d(x, w, w.shape[2] // 2)
    if relu:
        y = np.maximum(y, 0)
    return batchnorm_eval(y, _p(sd, pre + '.bnorm.weight', dt), _p(sd, pre + '.bnorm.bias', dt),
                          _p(sd, pre + '.bnorm.running_mean', dt),
                          _p(sd, pre + '.bnorm.running_var', dt))


def linear(x, w, b=None):
    y = np.matmul(x, w.T)
    return y + b if b is not None else y


def highway(sd: Params, pre: str, x: np.ndarray, dt) -> np.ndarray:
    """HighwayNetwork (common_layers.py:22-35)."""
    x1 = linear(x, _p(sd, pre + '.W1.weight', dt), _p(sd, pre + '.W1.bias', dt))
    x2 = linear(x, _p(sd, pre + '.W2.weight', dt), _p(sd, pre + '.W2.bias', dt))
    g = sigmoid(x2)
    return g * np.maximum(x1, 0) + (1.0 - g) * x


def _rnn_weights(sd, pre, sfx, dt):
    return (_p(sd, f'{pre}.weight_ih_l0{sfx}', dt), _p(sd, f'{pre}.weight_hh_l0{sfx}', dt),
            _p(sd, f'{pre}.bias_ih_l0{sfx}', dt), _p(sd, f'{pre}.bias_hh_l0{sfx}', dt))


def gru_bidir(sd: Params, pre: str, x: np.ndarray, dt) -> np.ndarray:
    """nn.GRU(batch_first, bidirectional), h0 = 0, gates [r; z; n]:
    r = s(Wir x + bir + Whr h + bhr), z likewise, n = tanh(Win x + bin + r*(Whn h + bhn)),
    h' = (1 - z) n + z h  (common_layers.py:84,118; forward_tacotron.py:39,53)."""
    B, T, _ = x.shape
    outs = []
    for sfx, order in (('', range(T)), ('_reverse', range(T - 1, -1, -1))):
        w_ih, w_hh, b_ih, b_hh = _rnn_weights(sd, pre, sfx, dt)
        H = w_hh.shape[1]
        gi = linear(x, w_ih, b_ih)
        h = np.zeros((B, H), dt)
        y = np.zeros((B, T, H), dt)
        for t in order:
            gh = linear(h, w_hh, b_hh)
            r = sigmoid(gi[:, t, :H] + gh[:, :H])
            z = sigmoid(gi[:, t, H:2 * H] + gh[:, H:2 * H])
            n = np.tanh(gi[:, t, 2 * H:] + r * gh[:, 2 * H:])
            h = n + z * (h - n)
            y[:, t] = h
        outs.append(y)
    return np.concatenate(outs, axis=2)


def lstm_bidir(sd: Params, pre: str, x: np.ndarray, dt, lengths: Optional[np.ndarray] = None,
               pad_value: float = 0.0) -> np.ndarray:
    """nn.LSTM(batch_first, bidirectional), h0 = c0 = 0, gates [i; f; g; o]
    (forward_tacotron.py:165-168,321).  With `lengths`: pack_padded_sequence /
    pad_packed_sequence(padding_value) semantics of forward() (:224-230)."""
    B, T, _ = x.shape
    L = np.full(B, T) if lengths is None else np.asarray(lengths)
    outs = []
    for sfx, order in (('', range(T)), ('_reverse', range(T - 1, -1, -1))):
        w_ih, w_hh, b_ih, b_hh = _rnn_weights(sd, pre, sfx, dt)
        H = w_hh.shape[1]
        gi = linear(x, w_ih, b_ih)
        h = np.zeros((B, H), dt)
        c = np.zeros((B, H), dt)
        y = np.zeros((B, T, H), dt)
        for t in order:
            g = gi[:, t] + linear(h, w_hh, b_hh)
            i_, f_ = sigmoid(g[:, :H]), sigmoid(g[:, H:2 * H])
            g_, o_ = np.tanh(g[:, 2 * H:3 * H]), sigmoid(g[:, 3 * H:])
            c = f_ * c + i_ * g_
            h = o_ * np.tanh(c)
            live = (t < L)[:, None]
            h = np.where(live, h, 0).astype(dt)
            c = np.where(live, c, 0).astype(dt)
            y[:, t] = np.where(live, h, pad_value)
        outs.append(y)
    return np.concatenate(outs, axis=2)


def maxpool_k2_s1_p1(x: np.ndarray) -> np.ndarray:
    """nn.MaxPool1d(2, 1, padding=1)(x)[..., :T]  (common_layers.py:73,100)."""
    y = x.copy()
    y[..., 1:] = np.maximum(x[..., 1:], x[..., :-1])
    return y


def cbhg(sd: Params, pre: str, x: np.ndarray, K: int, dt) -> np.ndarray:
    """CBHG.forward (common_layers.py:86-119): (B, Cin, T) -> (B, T, 2C)."""
    residual = x
    T = x.shape[-1]
    bank = [batch_norm_conv(sd, f'{pre}.conv1d_bank.{i}', x, True, dt)[:, :, :T] for i in range(K)]
    y = maxpool_k2_s1_p1(np.concatenate(bank, axis=1))
    y = batch_norm_conv(sd, f'{pre}.conv_project1', y, True, dt)
    y = batch_norm_conv(sd, f'{pre}.conv_project2', y, False, dt)
    y = (y + residual).transpose(0, 2, 1)
    y = linear(y, _p(sd, f'{pre}.pre_highway.weight', dt))
    i = 0
    while f'{pre}.highways.{i}.W1.weight' in sd:
        y = highway(sd, f'{pre}.highways.{i}', y, dt)
        i += 1
    return gru_bidir(sd, f'{pre}.rnn', y, dt)


def series_predictor(sd: Params, pre: str, ids: np.ndarray, dt, alpha: float = 1.0) -> np.ndarray:
    """SeriesPredictor.forward (forward_tacotron.py:44-55): (B, T) -> (B, T, 1)."""
    x = embedding(ids, _p(sd, f'{pre}.embedding.weight', dt)).transpose(0, 2, 1)
    for i in range(3):
        x = batch_norm_conv(sd, f'{pre}.convs.{i}', x, True, dt)
    x = gru_bidir(sd, f'{pre}.rnn', x.transpose(0, 2, 1), dt)
    x = linear(x, _p(sd, f'{pre}.lin.weight', dt), _p(sd, f'{pre}.lin.bias', dt))
    return (x / np.asarray(alpha, dtype=dt)).astype(dt)


def duration_counts(dur: np.ndarray) -> np.ndarray:
    """int64(fp32(dur + 0.5)) after the in-place clip (common_layers.py:13,16): note this is
    NOT round(): fp32 0.49999997 + 0.5 rounds to 1.0 and counts 1."""
    d = np.where(dur < 0, np.float32(0), dur).astype(np.float32)
    return (d + np.float32(0.5)).astype(np.int64)


def length_regulator(x: np.ndarray, dur: np.ndarray):
    """LengthRegulator.forward (common_layers.py:12-19): returns (expanded, clipped dur).
    x (B, T, C), dur (B, T) fp32."""
    dur = np.where(dur < 0, np.float32(0), dur).astype(np.float32)
    counts = duration_counts(dur)
    rows = [np.repeat(x[b], counts[b], axis=0) for b in range(x.shape[0])]
    T_mel = max(r.shape[0] for r in rows)
    out = np.zeros((x.shape[0], T_mel, x.shape[2]), dtype=x.dtype)
    for b, r in enumerate(rows):
        out[b, :r.shape[0]] = r
    return out, dur


def fill_rule(dur: np.ndarray) -> np.ndarray:
    """generate(): if sum(int64(dur)) <= 0: fill with 2.0 (forward_tacotron.py:254-255)."""
    if np.sum(dur.astype(np.int64)) <= 0:
        return np.full_like(dur, 2.0)
    return dur


# --- model --------------------------------------------------------------------------------

def _encode(sd, ids, pitch, energy, dt, ps=1.0, es=1.0):
    """embedding -> prenet CBHG -> + pitch / energy proj (forward_tacotron.py:304-314)."""
    x = embedding(ids, _p(sd, 'embedding.weight', dt)).transpose(0, 2, 1)
    K = sum(1 for k in sd if k.startswith('prenet.conv1d_bank.') and k.endswith('.conv.weight'))
    x = cbhg(sd, 'prenet', x, K, dt)
    pp = conv1d(pitch.astype(dt), _p(sd, 'pitch_proj.weight', dt), 1, _p(sd, 'pitch_proj.bias', dt))
    x = x + pp.transpose(0, 2, 1) * dt(ps)
    ep = conv1d(energy.astype(dt), _p(sd, 'energy_proj.weight', dt), 1, _p(sd, 'energy_proj.bias', dt))
    x = x + ep.transpose(0, 2, 1) * dt(es)
    return x


def _decode(sd, x, dt, lengths=None, pad_value=-11.5129):
    """LSTM -> lin -> postnet CBHG -> post_proj (forward_tacotron.py:321-327)."""
    x = lstm_bidir(sd, 'lstm', x, dt, lengths=lengths, pad_value=pad_value)
    x = linear(x, _p(sd, 'lin.weight', dt), _p(sd, 'lin.bias', dt)).transpose(0, 2, 1)
    K = sum(1 for k in sd if k.startswith('postnet.conv1d_bank.') and k.endswith('.conv.weight'))
    xp = cbhg(sd, 'postnet', x, K, dt)
    xp = linear(xp, _p(sd, 'post_proj.weight', dt)).transpose(0, 2, 1)
    return x, xp


def generate_mel(sd, ids, dur, pitch, energy, dt=np.float32, ps=1.0, es=1.0):
    """_generate_mel (forward_tacotron.py:289-330)."""
    x = _encode(sd, ids, pitch, energy, dt, ps, es)
    x, dur = length_regulator(x, dur)
    mel, mel_post = _decode(sd, x, dt)
    return {'mel': mel, 'mel_post': mel_post, 'dur': dur, 'pitch': pitch, 'energy': energy}


def generate(sd: Params, ids: np.ndarray, alpha: float = 1.0,
             pitch_function: Callable = lambda x: x, energy_function: Callable = lambda x: x,
             dt=np.float32, ps=1.0, es=1.0):
    """ForwardTacotron.generate (forward_tacotron.py:244-268)."""
    dur = series_predictor(sd, 'dur_pred', ids, dt, alpha)[..., 0]
    dur = fill_rule(dur)
    pitch = pitch_function(series_predictor(sd, 'pitch_pred', ids, dt).transpose(0, 2, 1))
    energy = energy_function(series_predictor(sd, 'energy_pred', ids, dt).transpose(0, 2, 1))
    return generate_mel(sd, ids, dur, pitch, energy, dt, ps, es)


def generate_jit(sd: Params, ids, alpha: float = 1.0, beta: float = 1.0, dt=np.float32):
    """ForwardTacotron.generate_jit (forward_tacotron.py:270-284)."""
    dur = fill_rule(series_predictor(sd, 'dur_pred', ids, dt, alpha)[..., 0])
    pitch = series_predictor(sd, 'pitch_pred', ids, dt).transpose(0, 2, 1) * dt(beta)
    energy = series_predictor(sd, 'energy_pred', ids, dt).transpose(0, 2, 1)
    return generate_mel(sd, ids, dur, pitch, energy, dt)


def forward(sd: Params, batch: Dict[str, np.ndarray], dt=np.float32, padding_value=-11.5129):
    """ForwardTacotron.forward (forward_tacotron.py:184-242), eval mode."""
    ids = batch['x']
    dur_hat = series_predictor(sd, 'dur_pred', ids, dt)[..., 0]
    pitch_hat = series_predictor(sd, 'pitch_pred', ids, dt).transpose(0, 2, 1)
    energy_hat = series_predictor(sd, 'energy_pred', ids, dt).transpose(0, 2, 1)
    x = _encode(sd, ids, batch['pitch'][:, None, :], batch['energy'][:, None, :], dt)
    x, _ = length_regulator(x, batch['dur'].astype(np.float32))
    lens = np.asarray(batch['mel_len'])
    x = x[:, :int(lens.max())]
    mel, mel_post = _decode(sd, x, dt, lengths=lens, pad_value=padding_value)
    T = batch['mel'].shape[2]

    def pad(a):
        a = a[:, :, :T]
        if a.shape[2] < T:
            a = np.concatenate([a, np.full(a.shape[:2] + (T - a.shape[2],), padding_value, a.dtype)], 2)
        return a
    return {'mel': pad(mel), 'mel_post': pad(mel_post), 'dur': dur_hat, 'pitch': pitch_hat,
            'energy': energy_hat}
