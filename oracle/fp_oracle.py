"""ORACLE — test infrastructure only, never shipped or measured as the product.

numpy restatement of the reference FastPitch inference path (models/fast_pitch.py), one
function per reference function (file:line cited).  Only tests/ (and smoke / bench's
cpu_baseline leg) may import it.  Pinned by tests/test_oracle_fastpitch.py against the
golden vectors the reference itself produced (tests/golden/make_goldens_fastpitch.py).

Weights: {state_dict key: np.ndarray}.  Activations (B, T, C).  fp32 by default.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .ft_oracle import conv1d, duration_counts, embedding, fill_rule, length_regulator

Params = Dict[str, np.ndarray]


def _p(sd, k, dt):
    return np.asarray(sd[k], dtype=dt)


def layer_norm(x, w, b, eps=1e-5):
    """nn.LayerNorm over the last dim (biased variance)."""
    xd = x.astype(np.float64)
    mean = xd.mean(-1, keepdims=True)
    var = ((xd - mean) ** 2).mean(-1, keepdims=True)
    return (((xd - mean) / np.sqrt(var + eps)) * w + b).astype(x.dtype)


def softmax(s):
    m = s.max(-1, keepdims=True)
    with np.errstate(invalid='ignore'):
        e = np.exp(s - m)
        return e / e.sum(-1, keepdims=True)


def mha(sd, pre, x, heads, kpm, dt):
    """nn.MultiheadAttention(x, x, x, key_padding_mask) math path
    (torch.nn.functional.multi_head_attention_forward): packed in_proj, q * sqrt(1/E),
    -inf on padded keys, softmax, @ v, out_proj.  x (B, T, d)."""
    B, T, d = x.shape
    hd = d // heads
    qkv = x @ _p(sd, pre + 'in_proj_weight', dt).T + _p(sd, pre + 'in_proj_bias', dt)
    q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    split = lambda t: t.reshape(B, T, heads, hd).transpose(0, 2, 1, 3)
    q, k, v = split(q), split(k), split(v)
    q = q * dt(np.sqrt(1.0 / hd))
    s = q @ k.transpose(0, 1, 3, 2)
    if kpm is not None:
        s = np.where(kpm[:, None, None, :], -np.inf, s).astype(dt)
    o = softmax(s) @ v
    o = o.transpose(0, 2, 1, 3).reshape(B, T, d)
    return o @ _p(sd, pre + 'out_proj.weight', dt).T + _p(sd, pre + 'out_proj.bias', dt)


def fft_block(sd, pre, x, heads, k1, k2, kpm, dt):
    """FFTBlock.forward (fast_pitch.py:70-91), eval (dropout = identity)."""
    x = layer_norm(x + mha(sd, pre + 'self_attn.', x, heads, kpm, dt),
                   _p(sd, pre + 'norm1.weight', dt), _p(sd, pre + 'norm1.bias', dt))
    h = conv1d(x.transpose(0, 2, 1), _p(sd, pre + 'conv1.weight', dt), k1 // 2,
               _p(sd, pre + 'conv1.bias', dt))
    h = np.maximum(h, 0)
    h = conv1d(h, _p(sd, pre + 'conv2.weight', dt), k2 // 2, _p(sd, pre + 'conv2.bias', dt))
    x = x + h.transpose(0, 2, 1)
    return layer_norm(x, _p(sd, pre + 'norm2.weight', dt), _p(sd, pre + 'norm2.bias', dt))


def forward_transformer(sd, pre, x, heads, layers, k1=9, k2=1, kpm=None, dt=np.float32):
    """ForwardTransformer.forward (fast_pitch.py:115-127) + PositionalEncoding (:30-33)."""
    T = x.shape[1]
    pe = _p(sd, pre + 'pos_encoder.pe', dt)[:T, 0, :]
    x = x + _p(sd, pre + 'pos_encoder.scale', dt) * pe
    for i in range(layers):
        x = fft_block(sd, f'{pre}layers.{i}.', x, heads, k1, k2, kpm, dt)
    return layer_norm(x, _p(sd, pre + 'norm.weight', dt), _p(sd, pre + 'norm.bias', dt))


def series_predictor(sd, pre, ids, heads, layers, kpm=None, alpha=1.0, dt=np.float32):
    """SeriesPredictor.forward (fast_pitch.py:152-161): (B, T) -> (B, T) (before the
    trailing unit dim)."""
    h = embedding(ids, _p(sd, pre + 'embedding.weight', dt))
    h = forward_transformer(sd, pre + 'transformer.', h, heads, layers, kpm=kpm, dt=dt)
    y = h @ _p(sd, pre + 'lin.weight', dt).T + _p(sd, pre + 'lin.bias', dt)
    return (y / dt(alpha))[..., 0]


def series_proj(sd, key, s, dt):
    """pitch_proj / energy_proj Conv1d(1 -> d, k3, pad 1) on (B, 1, T) -> (B, T, d)."""
    return conv1d(s, _p(sd, key + '.weight', dt), 1, _p(sd, key + '.bias', dt)).transpose(0, 2, 1)


def _encode(sd, ids, pitch, energy, heads, layers, dt, ps=1.0, es=1.0):
    kpm = ids == 0
    h = embedding(ids, _p(sd, 'embedding.weight', dt))
    h = forward_transformer(sd, 'prenet.', h, heads, layers, kpm=kpm, dt=dt)
    h = h + series_proj(sd, 'pitch_proj', pitch, dt) * dt(ps)
    h = h + series_proj(sd, 'energy_proj', energy, dt) * dt(es)
    return h


def generate_mel(sd, ids, dur, pitch, energy, heads=2, layers=4, dt=np.float32, ps=1.0, es=1.0):
    """_generate_mel (fast_pitch.py:315-340): mel_post is mel."""
    h = _encode(sd, ids, pitch, energy, heads, layers, dt, ps, es)
    h, dur = length_regulator(h, dur)
    h = forward_transformer(sd, 'postnet.', h, heads, layers, dt=dt)
    mel = (h @ _p(sd, 'lin.weight', dt).T + _p(sd, 'lin.bias', dt)).transpose(0, 2, 1)
    return {'mel': mel, 'mel_post': mel, 'dur': dur, 'postnet': h}


def generate(sd, ids, alpha=1.0, pitch_function=lambda p: p, energy_function=lambda e: e,
             pred_heads=2, pred_layers=4, heads=2, layers=4, dt=np.float32):
    """FastPitch.generate (fast_pitch.py:286-303): predictors WITHOUT masks."""
    dur = series_predictor(sd, 'dur_pred.', ids, pred_heads, pred_layers, alpha=alpha, dt=dt)
    dur = fill_rule(dur)
    pitch = pitch_function(series_predictor(sd, 'pitch_pred.', ids, pred_heads, pred_layers,
                                            dt=dt)[:, None, :])
    energy = energy_function(series_predictor(sd, 'energy_pred.', ids, pred_heads, pred_layers,
                                              dt=dt)[:, None, :])
    out = generate_mel(sd, ids, dur, pitch, energy, heads, layers, dt)
    out.update(pitch=pitch, energy=energy)
    return out


def forward(sd, batch, pred_heads=2, pred_layers=4, heads=2, layers=4, dt=np.float32,
            padding_value=-11.5129):
    """FastPitch.forward (fast_pitch.py:233-283): teacher forcing; predictors and prenet
    with the token mask, postnet with the mel-length mask; pad to mel.size(2)."""
    x = batch['x']
    kpm = x == 0
    dur_hat = series_predictor(sd, 'dur_pred.', x, pred_heads, pred_layers, kpm=kpm, dt=dt)
    pitch_hat = series_predictor(sd, 'pitch_pred.', x, pred_heads, pred_layers, kpm=kpm, dt=dt)[:, None]
    energy_hat = series_predictor(sd, 'energy_pred.', x, pred_heads, pred_layers, kpm=kpm, dt=dt)[:, None]
    h = _encode(sd, x, batch['pitch'][:, None, :], batch['energy'][:, None, :], heads, layers, dt)
    h, _ = length_regulator(h, batch['dur'])
    T_mel = h.shape[1]
    mkpm = np.arange(T_mel)[None, :] >= np.asarray(batch['mel_len'])[:, None]
    h = forward_transformer(sd, 'postnet.', h, heads, layers, kpm=mkpm, dt=dt)
    mel = (h @ _p(sd, 'lin.weight', dt).T + _p(sd, 'lin.bias', dt)).transpose(0, 2, 1)
    L = batch['mel'].shape[2]
    mel = mel[:, :, :L]
    if mel.shape[2] < L:
        mel = np.concatenate([mel, np.full(mel.shape[:2] + (L - mel.shape[2],), padding_value,
                                           dtype=mel.dtype)], 2)
    return {'mel': mel, 'mel_post': mel, 'dur': dur_hat, 'pitch': pitch_hat, 'energy': energy_hat}
