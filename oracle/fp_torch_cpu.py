"""ORACLE (CPU baseline + full-size checker) — test infrastructure only.

Functional torch-CPU restatement of the reference FastPitch inference path
(models/fast_pitch.py:16-130, :286-340): the same ATen CPU kernels the reference's modules
call (F.multi_head_attention_forward — the function nn.MultiheadAttention.forward runs with
batch_first=False —, layer_norm, conv1d, linear, repeat_interleave), without nn.Module or
an import of the reference.  bench.py --model fast_pitch times it as the cpu_baseline
("port").  Pinned against the reference goldens in tests/test_oracle_fastpitch.py.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .ft_torch_cpu import to_torch  # noqa: F401  (re-export)


def fft_block(sd, pre, x, heads, kpm):
    """FFTBlock.forward (fast_pitch.py:70-91), x (T, B, d)."""
    d = x.shape[-1]
    a = F.multi_head_attention_forward(
        x, x, x, d, heads, sd[pre + 'self_attn.in_proj_weight'], sd[pre + 'self_attn.in_proj_bias'],
        None, None, False, 0.0, sd[pre + 'self_attn.out_proj.weight'],
        sd[pre + 'self_attn.out_proj.bias'], training=False, key_padding_mask=kpm,
        need_weights=True, attn_mask=None)[0]
    x = F.layer_norm(x + a, (d,), sd[pre + 'norm1.weight'], sd[pre + 'norm1.bias'])
    h = x.permute(1, 2, 0)
    w1, w2 = sd[pre + 'conv1.weight'], sd[pre + 'conv2.weight']
    y = F.conv1d(F.relu(F.conv1d(h, w1, sd[pre + 'conv1.bias'], padding=w1.shape[2] // 2)),
                 w2, sd[pre + 'conv2.bias'], padding=w2.shape[2] // 2)
    x = (h + y).permute(2, 0, 1)
    return F.layer_norm(x, (d,), sd[pre + 'norm2.weight'], sd[pre + 'norm2.bias'])


def forward_transformer(sd, pre, x, heads, layers, kpm=None):
    """ForwardTransformer.forward (fast_pitch.py:115-127), x (B, T, d)."""
    x = x.transpose(0, 1)
    x = x + sd[pre + 'pos_encoder.scale'] * sd[pre + 'pos_encoder.pe'][:x.size(0), :]
    for i in range(layers):
        x = fft_block(sd, f'{pre}layers.{i}.', x, heads, kpm)
    d = x.shape[-1]
    return F.layer_norm(x, (d,), sd[pre + 'norm.weight'], sd[pre + 'norm.bias']).transpose(0, 1)


def series_predictor(sd, pre, x, heads=2, layers=4, kpm=None, alpha=1.0):
    h = F.embedding(x, sd[pre + 'embedding.weight'])
    h = forward_transformer(sd, pre + 'transformer.', h, heads, layers, kpm)
    return F.linear(h, sd[pre + 'lin.weight'], sd[pre + 'lin.bias']) / alpha


def length_regulator(x, dur):
    dur = dur.clone()
    dur[dur < 0] = 0.
    out = [torch.repeat_interleave(x[b], (dur[b] + 0.5).long(), dim=0) for b in range(x.shape[0])]
    return torch.nn.utils.rnn.pad_sequence(out, batch_first=True), dur


@torch.no_grad()
def generate(sd: Dict[str, torch.Tensor], x: torch.Tensor, alpha: float = 1.0,
             heads: int = 2, layers: int = 4) -> Dict[str, torch.Tensor]:
    """FastPitch.generate + _generate_mel (fast_pitch.py:286-340)."""
    dur = series_predictor(sd, 'dur_pred.', x, alpha=alpha).squeeze(2)
    if torch.sum(dur.long()) <= 0:
        dur.fill_(2.)
    pitch = series_predictor(sd, 'pitch_pred.', x).transpose(1, 2)
    energy = series_predictor(sd, 'energy_pred.', x).transpose(1, 2)
    h = F.embedding(x, sd['embedding.weight'])
    h = forward_transformer(sd, 'prenet.', h, heads, layers, kpm=x == 0)
    h = h + F.conv1d(pitch, sd['pitch_proj.weight'], sd['pitch_proj.bias'], padding=1).transpose(1, 2)
    h = h + F.conv1d(energy, sd['energy_proj.weight'], sd['energy_proj.bias'], padding=1).transpose(1, 2)
    h, dur = length_regulator(h, dur)
    h = forward_transformer(sd, 'postnet.', h, heads, layers)
    mel = F.linear(h, sd['lin.weight'], sd['lin.bias']).transpose(1, 2)
    return {'mel': mel, 'mel_post': mel, 'dur': dur, 'pitch': pitch, 'energy': energy}
