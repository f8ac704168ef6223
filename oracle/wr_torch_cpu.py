"""ORACLE (CPU baseline + checker) for the WaveRNN vocoder — test infrastructure only.

A functional torch-CPU restatement of the reference vocoder, models/fatchord_version.py
(ResBlock :14-29, MelResNet :32-49, Stretch2d :52-62, UpsampleNetwork :65-90,
WaveRNN.forward :132-169, generate :171-265, pad_tensor :282-292, fold_with_overlap
:294-341, xfade_and_unfold :343-406) and of the sampling it calls
(utils/distribution.py:93-127 sample_from_discretized_mix_logistic, torch's Categorical for
RAW) plus DSP.decode_mu_law (utils/dsp.py:139-161).  It calls the SAME ATen CPU kernels as
the reference (conv1d, batch_norm, conv2d, gru_cell, linear, softmax, Categorical) but
imports nothing from the reference; pinned against goldens produced by the reference
classes themselves (tests/golden/make_goldens_wavernn.py, tests/test_oracle_wavernn.py).

Samplers (the only source of randomness in generate):
  'reference'      the reference's own draws: torch.distributions.Categorical (RAW) /
                   uniform_ pairs (MOL) from torch's CPU generator — seeded by the caller
                   with torch.manual_seed, this reproduces the reference bit for bit.
  PhiloxSampler    the GPU kernel's counter-based stream (Philox4x32-10, restated in
                   numpy below): same distribution, reproducible on any device; with it the
                   oracle checks the HIP path's sample sequence.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

LOG_SCALE_MIN = float(np.log(1e-14))  # utils/distribution.py:103-104


def _t(sd, k):
    v = sd[k]
    return (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))).cpu()


def to_torch(sd) -> Dict[str, torch.Tensor]:
    return {k: _t(sd, k) for k in sd}


# ------------------------------------------------------------------------------------------
# upsampling network (fatchord_version.py:14-90)

def _bn(sd, pre, x):
    return F.batch_norm(x, sd[pre + '.running_mean'], sd[pre + '.running_var'],
                        sd[pre + '.weight'], sd[pre + '.bias'], False, 0.0, 1e-5)


def mel_resnet(sd, m, res_blocks):
    """MelResNet.forward :43-49 on (B, feat, T) -> (B, res_out, T - 2 pad)."""
    p = 'upsample.resnet.'
    x = F.conv1d(m, sd[p + 'conv_in.weight'])
    x = F.relu(_bn(sd, p + 'batch_norm', x))
    for i in range(res_blocks):  # ResBlock.forward :22-29
        q = f'{p}layers.{i}.'
        r = x
        x = F.relu(_bn(sd, q + 'batch_norm1', F.conv1d(x, sd[q + 'conv1.weight'])))
        x = _bn(sd, q + 'batch_norm2', F.conv1d(x, sd[q + 'conv2.weight'])) + r
    return F.conv1d(x, sd[p + 'conv_out.weight'], sd[p + 'conv_out.bias'])


def stretch2d(x, x_scale, y_scale):
    """Stretch2d.forward :58-62."""
    b, c, h, w = x.size()
    x = x.unsqueeze(-1).unsqueeze(3).repeat(1, 1, 1, y_scale, 1, x_scale)
    return x.view(b, c, h * y_scale, w * x_scale)


def upsample(sd, m, cfg):
    """UpsampleNetwork.forward :83-90: (B, feat, T) -> (mels (B, L, feat), aux (B, L, res_out)),
    L = (T - 2 pad) * prod(upsample_factors)."""
    scales = cfg['upsample_factors']
    total = int(np.prod(scales))
    indent = cfg['pad'] * total
    aux = stretch2d(mel_resnet(sd, m, cfg['res_blocks']).unsqueeze(1), total, 1).squeeze(1)
    x = m.unsqueeze(1)
    for i, s in enumerate(scales):
        x = stretch2d(x, s, 1)
        x = F.conv2d(x, sd[f'upsample.up_layers.{2 * i + 1}.weight'], padding=(0, s))
    x = x.squeeze(1)[:, :, indent:-indent]
    return x.transpose(1, 2), aux.transpose(1, 2)


# ------------------------------------------------------------------------------------------
# folding (fatchord_version.py:282-406)

def pad_tensor(x, pad, side='both'):
    b, t, c = x.size()
    total = t + 2 * pad if side == 'both' else t + pad
    padded = torch.zeros(b, total, c, dtype=x.dtype)
    if side in ('before', 'both'):
        padded[:, pad:pad + t, :] = x
    elif side == 'after':
        padded[:, :t, :] = x
    return padded


def fold_with_overlap(x, target, overlap):
    _, total_len, features = x.size()
    num_folds = (total_len - overlap) // (target + overlap)
    extended_len = num_folds * (overlap + target) + overlap
    remaining = total_len - extended_len
    if remaining != 0:
        num_folds += 1
        x = pad_tensor(x, target + 2 * overlap - remaining, side='after')
    folded = torch.zeros(num_folds, target + 2 * overlap, features, dtype=x.dtype)
    for i in range(num_folds):
        start = i * (target + overlap)
        folded[i] = x[:, start:start + target + 2 * overlap, :]
    return folded


def xfade_and_unfold(y, target, overlap):
    """float64 numpy (num_folds, target + 2 overlap) -> (total_len,), equal-power fades."""
    y = np.array(y, dtype=np.float64)
    num_folds, length = y.shape
    target = length - 2 * overlap
    total_len = num_folds * (target + overlap) + overlap
    silence_len = overlap // 2
    fade_len = overlap - silence_len
    t = np.linspace(-1, 1, fade_len, dtype=np.float64)
    fade_in = np.concatenate([np.zeros(silence_len), np.sqrt(0.5 * (1 + t))])
    fade_out = np.concatenate([np.ones(silence_len), np.sqrt(0.5 * (1 - t))])
    y[:, :overlap] *= fade_in
    y[:, -overlap:] *= fade_out
    unfolded = np.zeros(total_len, dtype=np.float64)
    for i in range(num_folds):
        start = i * (target + overlap)
        unfolded[start:start + length] += y[i]
    return unfolded


def decode_mu_law(y, mu, from_labels=True):
    """DSP.decode_mu_law, utils/dsp.py:156-161 (numpy float64)."""
    if from_labels:
        y = 2 * y / (2 ** math.log2(mu) - 1.) - 1.
    mu = mu - 1
    return np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)


# ------------------------------------------------------------------------------------------
# Philox4x32-10 (the HIP kernel's counter-based generator, csrc/wavernn.hip philox())

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_LO = np.uint64(0xFFFFFFFF)


def philox4x32(ctr: np.ndarray, seed: int) -> np.ndarray:
    """ctr (..., 4) uint32 -> (..., 4) uint32 words; key = (seed & 0xffffffff, seed >> 32)."""
    c = [np.asarray(ctr[..., i], dtype=np.uint32).copy() for i in range(4)]
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over='ignore'):
        for r in range(10):
            p0 = _M0 * c[0].astype(np.uint64)
            p1 = _M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _LO).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _LO).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return np.stack(c, axis=-1)


def uniform01(words: np.ndarray) -> np.ndarray:
    """uint32 -> float32 in (0, 1): (x >> 8 + 0.5) 2^-24 (exact in fp32)."""
    return ((words >> np.uint32(8)).astype(np.float32) + np.float32(0.5)) * np.float32(2.0 ** -24)


class PhiloxSampler:
    """The HIP kernel's draws.  RAW: class k of sequence b at step t takes word k % 4 of
    Philox((t, b, k // 4, 0)); the sample is argmax_k (logit_k - log(-log u_k)) — the Gumbel
    form of torch.multinomial's single draw argmax(p_k / E_k), E_k = -log u_k ~ Exp(1).
    MOL: mixture k's uniform is word k % 4 of Philox((t, b, k // 4, 1)), the logistic
    draw word 0 of Philox((t, b, 0, 2)); both mapped to uniform_(1e-5, 1 - 1e-5) like
    utils/distribution.py:113,122."""

    def __init__(self, seed: int):
        self.seed = int(seed)

    def words(self, t: int, B: int, n: int, kind: int) -> np.ndarray:
        j = np.arange((n + 3) // 4, dtype=np.uint32)
        ctr = np.zeros((B, j.size, 4), dtype=np.uint32)
        ctr[..., 0] = t
        ctr[..., 1] = np.arange(B, dtype=np.uint32)[:, None]
        ctr[..., 2] = j[None, :]
        ctr[..., 3] = kind
        return philox4x32(ctr, self.seed).reshape(B, -1)[:, :n]

    def gumbel_scores(self, logits: torch.Tensor, t: int) -> np.ndarray:
        """float64 z_k = logit_k - log(-log u_k) (the quantity the kernel maximises)."""
        B, n = logits.shape
        u = uniform01(self.words(t, B, n, 0)).astype(np.float64)
        return logits.double().numpy() - np.log(-np.log(u))

    def raw(self, logits: torch.Tensor, t: int) -> torch.Tensor:
        return torch.from_numpy(np.argmax(self.gumbel_scores(logits, t), axis=1))

    def mol_uniforms(self, t: int, B: int, nr_mix: int):
        lo, span = np.float32(1e-5), np.float32(1.0 - 2e-5)
        temp = lo + uniform01(self.words(t, B, nr_mix, 1)) * span
        u = lo + uniform01(self.words(t, B, 1, 2))[:, 0] * span
        return torch.from_numpy(temp), torch.from_numpy(u)


def sample_mol(logits: torch.Tensor, temp_u: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """sample_from_discretized_mix_logistic (utils/distribution.py:93-127) for one step,
    logits (B, 3 nr_mix), with the two uniform draws given (temp_u (B, nr_mix), u (B,))."""
    nr_mix = logits.size(1) // 3
    logit_probs = logits[:, :nr_mix]
    temp = logit_probs - torch.log(-torch.log(temp_u))
    _, argmax = temp.max(dim=-1)
    one_hot = F.one_hot(argmax, nr_mix).float()
    means = torch.sum(logits[:, nr_mix:2 * nr_mix] * one_hot, dim=-1)
    log_scales = torch.clamp(torch.sum(logits[:, 2 * nr_mix:3 * nr_mix] * one_hot, dim=-1),
                             min=LOG_SCALE_MIN)
    x = means + torch.exp(log_scales) * (torch.log(u) - torch.log(1. - u))
    return torch.clamp(torch.clamp(x, min=-1.), max=1.)


def _ref_mol(logits: torch.Tensor) -> torch.Tensor:
    """The reference's own MOL draw order: temp = uniform_ (1, B, nr_mix), u = uniform_ (1, B)."""
    nr_mix = logits.size(1) // 3
    temp_u = torch.empty(1, logits.size(0), nr_mix).uniform_(1e-5, 1.0 - 1e-5)[0]
    u = torch.empty(1, logits.size(0)).uniform_(1e-5, 1.0 - 1e-5)[0]
    return sample_mol(logits, temp_u, u)


# ------------------------------------------------------------------------------------------
# the vocoder

def _dims(sd):
    rnn = sd['rnn1.weight_hh_l0'].shape[1]
    aux = (sd['rnn2.weight_ih_l0'].shape[1] - rnn)
    return rnn, aux


def forward(sd, cfg, x, mels):
    """WaveRNN.forward :132-169 (teacher-forced): x (B, L) samples, mels (B, feat, T) ->
    logits (B, L, n_classes), L = (T - 2 pad) * hop."""
    R, d = _dims(sd)
    B = x.size(0)
    m, aux = upsample(sd, mels, cfg)
    a1, a2, a3, a4 = (aux[:, :, d * i:d * (i + 1)] for i in range(4))
    h = torch.cat([x.unsqueeze(-1), m, a1], dim=2)
    h = F.linear(h, sd['I.weight'], sd['I.bias'])
    res = h
    h1 = _gru_seq(sd, 'rnn1', h, torch.zeros(B, R))
    h = h1 + res
    res = h
    h2 = _gru_seq(sd, 'rnn2', torch.cat([h, a2], dim=2), torch.zeros(B, R))
    h = h2 + res
    h = F.relu(F.linear(torch.cat([h, a3], dim=2), sd['fc1.weight'], sd['fc1.bias']))
    h = F.relu(F.linear(torch.cat([h, a4], dim=2), sd['fc2.weight'], sd['fc2.bias']))
    return F.linear(h, sd['fc3.weight'], sd['fc3.bias'])


def _gru_seq(sd, pre, x, h0):
    out, _ = torch._VF.gru(x, h0.unsqueeze(0), [sd[pre + '.weight_ih_l0'], sd[pre + '.weight_hh_l0'],
                                               sd[pre + '.bias_ih_l0'], sd[pre + '.bias_hh_l0']],
                           True, 1, 0.0, False, False, True)
    return out


def _cell(sd, pre, x, h):
    return torch.gru_cell(x, h, sd[pre + '.weight_ih_l0'], sd[pre + '.weight_hh_l0'],
                          sd[pre + '.bias_ih_l0'], sd[pre + '.bias_hh_l0'])


def conditioning(sd, cfg, mels, batched, target, overlap):
    """generate :185-192: (mels (B', L, feat), aux (B', L, res_out), wave_len)."""
    hop = int(np.prod(cfg['upsample_factors']))
    mels = torch.as_tensor(mels)
    wave_len = (mels.size(-1) - 1) * hop
    mels = pad_tensor(mels.transpose(1, 2), pad=cfg['pad'], side='both')
    m, aux = upsample(sd, mels.transpose(1, 2), cfg)
    if batched:
        m = fold_with_overlap(m, target, overlap)
        aux = fold_with_overlap(aux, target, overlap)
    return m, aux, wave_len


def generate(sd, cfg, mels, batched=True, target=11000, overlap=550, mu_law=True,
             sampler='reference', steps: Optional[int] = None, forced=None, trace=None):
    """WaveRNN.generate :171-265 -> float64 numpy wave.  sampler: 'reference' (torch's RNG,
    the reference's draws) or a PhiloxSampler.  steps: stop after this many samples per
    fold (a bounded CPU baseline; returns the raw (B, steps) sample matrix).  forced:
    (B, L) sample values to feed back instead of drawing (teacher-forced check of a GPU
    sample sequence); trace: list receiving each step's logits."""
    mode = cfg.get('mode', 'RAW')
    n_classes = sd['fc3.weight'].shape[0]
    mu_law = mu_law if mode == 'RAW' else False
    R, d = _dims(sd)
    hop = int(np.prod(cfg['upsample_factors']))
    if sampler == 'reference':
        # generate :180-181 builds two nn.GRUCell modules (get_gru_cell :274-280) whose
        # constructors draw a random init from torch's generator before the weights are
        # replaced: consume the same draws so the sampling sees the reference's stream
        torch.nn.GRUCell(R, R)
        torch.nn.GRUCell(R + d, R)
    with torch.no_grad():
        m, aux, wave_len = conditioning(sd, cfg, mels, batched, target, overlap)
        b_size, seq_len, _ = m.size()
        if steps is not None:
            seq_len = min(seq_len, steps)
        h1 = torch.zeros(b_size, R)
        h2 = torch.zeros(b_size, R)
        x = torch.zeros(b_size, 1)
        aux_split = [aux[:, :, d * i:d * (i + 1)] for i in range(4)]
        output = []
        for i in range(seq_len):
            m_t = m[:, i, :]
            a1_t, a2_t, a3_t, a4_t = (a[:, i, :] for a in aux_split)
            x = torch.cat([x, m_t, a1_t], dim=1)
            x = F.linear(x, sd['I.weight'], sd['I.bias'])
            h1 = _cell(sd, 'rnn1', x, h1)
            x = x + h1
            h2 = _cell(sd, 'rnn2', torch.cat([x, a2_t], dim=1), h2)
            x = x + h2
            x = F.relu(F.linear(torch.cat([x, a3_t], dim=1), sd['fc1.weight'], sd['fc1.bias']))
            x = F.relu(F.linear(torch.cat([x, a4_t], dim=1), sd['fc2.weight'], sd['fc2.bias']))
            logits = F.linear(x, sd['fc3.weight'], sd['fc3.bias'])
            if trace is not None:
                trace.append(logits.clone())
            if forced is not None:
                sample = torch.as_tensor(forced[:, i], dtype=torch.float32)
            elif mode == 'MOL':
                if sampler == 'reference':
                    sample = _ref_mol(logits)
                else:
                    sample = sample_mol(logits, *sampler.mol_uniforms(i, b_size, n_classes // 3))
            else:
                if sampler == 'reference':
                    posterior = F.softmax(logits, dim=1)
                    idx = torch.distributions.Categorical(posterior).sample()
                else:
                    idx = sampler.raw(logits, i)
                sample = 2 * idx.float() / (n_classes - 1.) - 1.
            output.append(sample.view(-1))
            x = sample.view(-1, 1)
    output = torch.stack(output).transpose(0, 1).numpy().astype(np.float64)
    if steps is not None:
        return output
    return finish(output, batched, target, overlap, mu_law, n_classes, wave_len, hop)


def finish(output, batched, target, overlap, mu_law, n_classes, wave_len, hop):
    """generate :246-263 on the (B, L) float64 sample matrix."""
    output = np.array(output, dtype=np.float64)
    if mu_law:
        output = decode_mu_law(output, n_classes, False)
    output = xfade_and_unfold(output, target, overlap) if batched else output[0]
    fade_out = np.linspace(1, 0, 20 * hop)
    output = output[:wave_len]
    output[-20 * hop:] *= fade_out
    return output
