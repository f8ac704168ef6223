"""ORACLE (CPU baseline + full-size checker) — test infrastructure only.

A functional torch-CPU restatement of the reference inference path
(models/forward_tacotron.py:244-330, models/common_layers.py:7-119): the SAME ATen CPU
kernels the reference calls (conv1d, batch_norm, the GRU / LSTM ops behind nn.GRU /
nn.LSTM, repeat_interleave), but no nn.Module and no import of the reference.  Because it
runs the reference's kernels it is the honest CPU-speed baseline for bench.py
(cpu_baseline.kind = "port") and the checker for full-size (B = 64) parity on the GPU
box, where the numpy oracle would be slow.  Pinned against the reference goldens by
tests/test_oracle.py.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
from __future__ import annotations

from typing import Callable, Dict

import torch
import torch.nn.functional as F


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(v)


def to_torch(sd, dtype=None) -> Dict[str, torch.Tensor]:
    """{key: CPU tensor}; dtype (e.g. torch.float64: the higher-precision truth of the
    accuracy tests) converts the floating-point entries."""
    out = {k: _t(sd, k).cpu() for k in sd}
    if dtype is not None:
        out = {k: v.to(dtype) if v.is_floating_point() else v for k, v in out.items()}
    return out


def batch_norm_conv(sd, pre, x, relu):
    """BatchNormConv (common_layers.py:38-52 / forward_tacotron.py:58-71)."""
    w = sd[pre + '.conv.weight']
    y = F.conv1d(x, w, padding=w.shape[2] // 2)
    if relu:
        y = F.relu(y)
    return F.batch_norm(y, sd[pre + '.bnorm.running_mean'], sd[pre + '.bnorm.running_var'],
                        sd[pre + '.bnorm.weight'], sd[pre + '.bnorm.bias'], False, 0.1, 1e-5)


def _rnn_params(sd, pre):
    return [sd[f'{pre}.{n}{s}'] for s in ('', '_reverse')
            for n in ('weight_ih_l0', 'weight_hh_l0', 'bias_ih_l0', 'bias_hh_l0')]


def gru(sd, pre, x):
    """nn.GRU(batch_first, bidirectional) forward == torch.gru (common_layers.py:84)."""
    H = sd[pre + '.weight_hh_l0'].shape[1]
    h0 = torch.zeros(2, x.shape[0], H, dtype=x.dtype)
    return torch.gru(x, h0, _rnn_params(sd, pre), True, 1, 0.0, False, True, True)[0]


def lstm(sd, pre, x):
    """nn.LSTM(batch_first, bidirectional) forward == torch.lstm (forward_tacotron.py:165)."""
    H = sd[pre + '.weight_hh_l0'].shape[1]
    z = torch.zeros(2, x.shape[0], H, dtype=x.dtype)
    return torch.lstm(x, (z, z), _rnn_params(sd, pre), True, 1, 0.0, False, True, True)[0]


def cbhg(sd, pre, x, K):
    """CBHG.forward (common_layers.py:86-119)."""
    residual = x
    T = x.size(-1)
    bank = torch.cat([batch_norm_conv(sd, f'{pre}.conv1d_bank.{i}', x, True)[:, :, :T]
                      for i in range(K)], dim=1)
    x = F.max_pool1d(bank, 2, 1, 1)[:, :, :T]
    x = batch_norm_conv(sd, f'{pre}.conv_project1', x, True)
    x = batch_norm_conv(sd, f'{pre}.conv_project2', x, False)
    x = (x + residual).transpose(1, 2)
    x = F.linear(x, sd[f'{pre}.pre_highway.weight'])
    i = 0
    while f'{pre}.highways.{i}.W1.weight' in sd:
        x1 = F.linear(x, sd[f'{pre}.highways.{i}.W1.weight'], sd[f'{pre}.highways.{i}.W1.bias'])
        x2 = F.linear(x, sd[f'{pre}.highways.{i}.W2.weight'], sd[f'{pre}.highways.{i}.W2.bias'])
        g = torch.sigmoid(x2)
        x = g * F.relu(x1) + (1. - g) * x
        i += 1
    return gru(sd, f'{pre}.rnn', x)


def series_predictor(sd, pre, ids, alpha=1.0):
    """SeriesPredictor.forward (forward_tacotron.py:44-55)."""
    x = F.embedding(ids, sd[f'{pre}.embedding.weight']).transpose(1, 2)
    for i in range(3):
        x = batch_norm_conv(sd, f'{pre}.convs.{i}', x, True)
    x = gru(sd, f'{pre}.rnn', x.transpose(1, 2))
    return F.linear(x, sd[f'{pre}.lin.weight'], sd[f'{pre}.lin.bias']) / alpha


def length_regulator(x, dur):
    """LengthRegulator.forward (common_layers.py:12-19), dur clipped in place."""
    dur[dur < 0] = 0.
    rows = [torch.repeat_interleave(x[i], (dur[i] + 0.5).long(), dim=0) for i in range(x.size(0))]
    return torch.nn.utils.rnn.pad_sequence(rows, padding_value=0., batch_first=True)


def _k(sd, pre):
    return sum(1 for k in sd if k.startswith(pre + '.conv1d_bank.') and k.endswith('.conv.weight'))


def generate(sd, ids: torch.Tensor, alpha: float = 1.0,
             pitch_function: Callable = lambda x: x, energy_function: Callable = lambda x: x,
             pitch_strength: float = 1.0, energy_strength: float = 1.0, lr_dur=None):
    """ForwardTacotron.generate (forward_tacotron.py:244-330).  lr_dur (accuracy tests
    only): durations for the LengthRegulator in place of the computed ones, so a float64
    run follows the fp32 reference's frame counts."""
    with torch.no_grad():
        dur = series_predictor(sd, 'dur_pred', ids, alpha).squeeze(2)
        if torch.sum(dur.long()) <= 0:
            torch.fill_(dur, value=2.)
        pitch = pitch_function(series_predictor(sd, 'pitch_pred', ids).transpose(1, 2))
        energy = energy_function(series_predictor(sd, 'energy_pred', ids).transpose(1, 2))
        x = F.embedding(ids, sd['embedding.weight']).transpose(1, 2)
        x = cbhg(sd, 'prenet', x, _k(sd, 'prenet'))
        x = x + F.conv1d(pitch, sd['pitch_proj.weight'], sd['pitch_proj.bias'], padding=1).transpose(1, 2) * pitch_strength
        x = x + F.conv1d(energy, sd['energy_proj.weight'], sd['energy_proj.bias'], padding=1).transpose(1, 2) * energy_strength
        x = length_regulator(x, dur if lr_dur is None else lr_dur.clone().to(dur.dtype))
        x = lstm(sd, 'lstm', x)
        x = F.linear(x, sd['lin.weight'], sd['lin.bias']).transpose(1, 2)
        x_post = cbhg(sd, 'postnet', x, _k(sd, 'postnet'))
        x_post = F.linear(x_post, sd['post_proj.weight']).transpose(1, 2)
    return {'mel': x, 'mel_post': x_post, 'dur': dur, 'pitch': pitch, 'energy': energy}
