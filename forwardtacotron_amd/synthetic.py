"""Synthetic, LJSpeech-shaped weights and inputs (there is no network for checkpoints or data).

The recipe is deterministic and portable: every state_dict entry is drawn
from its own numpy PCG64 stream seeded by (seed, crc32(key)), so the same 98 MB model is
regenerated bit-identically on any machine from the key names alone — the goldens under
tests/golden/ only store inputs / outputs, never the weights.

  conv / linear / RNN weights  N(0, 1/sqrt(fan_in))
  biases                       N(0, 0.1)
  BatchNorm                    gamma, running_var ~ U(0.75, 1.25); beta, running_mean ~ N(0, 0.1)
  embeddings                   N(0, 1)
  dur_pred.lin                 weight x DUR_GAIN, bias = DUR_BIAS  (~7 frames / phoneme, like
                               LJSpeech; random init would give dur ~0.2 and the fill-2 rule)
  lin / post_proj              weight x MEL_GAIN / POST_GAIN  (mean |mel|, |mel_post| ~ 5,
                               log-mel magnitudes, so the 1e-4 parity bound is meaningful)

FastPitch (model='fast_pitch'): LayerNorm gamma ~ U(0.75, 1.25), beta ~ N(0, 0.1);
pos_encoder.scale ~ U(0.9, 1.1); pos_encoder.pe is the model's own sinusoid buffer (not
drawn); dur_pred.lin weight x FP_DUR_GAIN, bias = FP_DUR_BIAS (~6.5 frames / phoneme);
lin.weight x FP_MEL_GAIN (the transformer output is LayerNorm-ed, O(1) per channel).

WaveRNN vocoder (model='wavernn', models/fatchord_version.py): BatchNorm as above; the
upsampling smoothers `upsample.up_layers.{1,3,5}.weight` keep the reference's own init
(fill 1/k, :78-79); fc3.weight x WR_FC3_GAIN (peaked class posteriors, so the sampled
sequence depends on the logits and not only on the noise).
"""
from __future__ import annotations

import copy
import zlib
from typing import Dict, Iterable, Optional

import numpy as np

DUR_BIAS = 9.0
DUR_GAIN = 5.0
MEL_GAIN = 30.0
POST_GAIN = 6.0
FP_DUR_BIAS = 6.0
FP_DUR_GAIN = 1.5
FP_MEL_GAIN = 4.0
WR_FC3_GAIN = 0.25

# forward_tacotron.model and dsp sections of the reference config.yaml (:9-34, :76-106)
DEFAULT_CONFIG = {
    'tts_model': 'forward_tacotron',
    'dsp': {
        'sample_rate': 22050, 'n_fft': 1024, 'num_mels': 80, 'hop_length': 256,
        'win_length': 1024, 'fmin': 0, 'fmax': 8000, 'peak_norm': False,
        'trim_start_end_silence': True, 'trim_silence_top_db': 60, 'pitch_max_freq': 600,
        'trim_long_silences': False, 'vad_window_length': 30, 'vad_moving_average_width': 8,
        'vad_max_silence_length': 12, 'vad_sample_rate': 16000, 'voc_mode': 'RAW', 'bits': 9,
        'mu_law': True,
    },
    'forward_tacotron': {'model': {
        'embed_dims': 256, 'series_embed_dims': 64,
        'durpred_conv_dims': 256, 'durpred_rnn_dims': 64, 'durpred_dropout': 0.5,
        'pitch_conv_dims': 256, 'pitch_rnn_dims': 128, 'pitch_dropout': 0.5, 'pitch_strength': 1.,
        'energy_conv_dims': 256, 'energy_rnn_dims': 64, 'energy_dropout': 0.5,
        'energy_strength': 1.,
        'prenet_dims': 256, 'prenet_k': 16, 'prenet_dropout': 0.5, 'prenet_num_highways': 4,
        'rnn_dims': 512,
        'postnet_dims': 256, 'postnet_k': 8, 'postnet_num_highways': 4, 'postnet_dropout': 0.,
    }},
}


# fast_pitch.model section of the reference config.yaml (:128-163)
DEFAULT_CONFIG['fast_pitch'] = {'model': {
    'durpred_d_model': 128, 'durpred_n_heads': 2, 'durpred_layers': 4, 'durpred_d_fft': 128,
    'durpred_dropout': 0.5,
    'pitch_d_model': 128, 'pitch_n_heads': 2, 'pitch_layers': 4, 'pitch_d_fft': 128,
    'pitch_dropout': 0.5, 'pitch_strength': 1.0,
    'energy_d_model': 128, 'energy_n_heads': 2, 'energy_layers': 4, 'energy_d_fft': 128,
    'energy_dropout': 0.5, 'energy_strength': 1.0,
    'd_model': 256, 'conv1_kernel': 9, 'conv2_kernel': 1,
    'prenet_layers': 4, 'prenet_heads': 2, 'prenet_fft': 1024, 'prenet_dropout': 0.1,
    'postnet_layers': 4, 'postnet_heads': 2, 'postnet_fft': 1024, 'postnet_dropout': 0.1,
}}


# vocoder.model section of the reference config.yaml (:187-198), and its generation
# defaults (:213-215, gen_forward.py:55-56)
DEFAULT_CONFIG['vocoder'] = {'model': {
    'mode': 'RAW', 'upsample_factors': [4, 8, 8], 'rnn_dims': 512, 'fc_dims': 512,
    'compute_dims': 128, 'res_out_dims': 128, 'res_blocks': 10, 'pad': 2,
}, 'generate': {'gen_batched': True, 'target': 11000, 'overlap': 550}}


def default_config() -> dict:
    return copy.deepcopy(DEFAULT_CONFIG)


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def synthetic_array(key: str, shape, dtype: str, seed: int = 0,
                    model: str = 'forward_tacotron') -> np.ndarray:
    """The value of one state_dict entry under the recipe above."""
    rng = _rng(seed, key)
    leaf = key.rsplit('.', 1)[-1]
    shape = tuple(shape)
    if dtype.startswith('int'):
        return np.zeros(shape, dtype=np.int64)
    if model == 'wavernn':
        if '.up_layers.' in key:
            return np.full(shape, 1.0 / shape[-1], dtype=np.float32)
        if '.batch_norm' in key:
            a = rng.uniform(0.75, 1.25, shape) if leaf in ('weight', 'running_var') else rng.normal(0.0, 0.1, shape)
            return a.astype(np.float32)
        a = _generic(rng, key, leaf, shape)
        if key == 'fc3.weight':
            a = a * WR_FC3_GAIN
        return a.astype(np.float32)
    if model == 'fast_pitch':
        parent = key.rsplit('.', 2)[-2] if key.count('.') >= 1 else ''
        if parent.startswith('norm'):
            a = rng.uniform(0.75, 1.25, shape) if leaf == 'weight' else rng.normal(0.0, 0.1, shape)
            return a.astype(np.float32)
        if leaf == 'scale':
            return rng.uniform(0.9, 1.1, shape).astype(np.float32)
        if key == 'dur_pred.lin.bias':
            return np.full(shape, FP_DUR_BIAS, dtype=np.float32)
        a = _generic(rng, key, leaf, shape)
        if key == 'dur_pred.lin.weight':
            a = a * FP_DUR_GAIN
        elif key == 'lin.weight':
            a = a * FP_MEL_GAIN
        return a.astype(np.float32)
    if '.bnorm.' in key:
        if leaf in ('weight', 'running_var'):
            a = rng.uniform(0.75, 1.25, shape)
        else:
            a = rng.normal(0.0, 0.1, shape)
    else:
        a = _generic(rng, key, leaf, shape)
    if key == 'dur_pred.lin.weight':
        a = a * DUR_GAIN
    elif key == 'dur_pred.lin.bias':
        a = np.full(shape, DUR_BIAS)
    elif key == 'lin.weight':
        a = a * MEL_GAIN
    elif key == 'post_proj.weight':
        a = a * POST_GAIN
    return a.astype(np.float32)


def _generic(rng, key, leaf, shape):
    if 'embedding' in key:
        return rng.normal(0.0, 1.0, shape)
    if leaf.startswith('bias') or leaf.endswith('_bias'):
        return rng.normal(0.0, 0.1, shape)
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    return rng.normal(0.0, 1.0 / np.sqrt(fan_in), shape)


def synthetic_state_dict(template, seed: int = 0, model: str = 'forward_tacotron') -> Dict[str, np.ndarray]:
    """template: a model (anything with state_dict()) or {key: tensor/array}.  Buffers that
    are deterministic functions of the architecture (FastPitch's `pe`) are kept."""
    sd = template.state_dict() if hasattr(template, 'state_dict') else template
    out = {}
    for k, v in sd.items():
        if k.endswith('pos_encoder.pe'):
            out[k] = np.asarray(v.detach().cpu().numpy() if hasattr(v, 'detach') else v)
            continue
        dt = str(v.dtype).replace('torch.', '')
        out[k] = synthetic_array(k, tuple(v.shape), dt, seed, model)
    return out


def load_synthetic(model, seed: int = 0, kind: str = 'forward_tacotron'):
    """Fill a (reference-compatible) model with the synthetic recipe in place; returns it."""
    import torch
    sd = synthetic_state_dict(model, seed, kind)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return model


def synthetic_tokens(B: int, T_max: int, seed: int = 0, min_len: Optional[int] = None,
                     lengths: Optional[Iterable[int]] = None, num_chars: int = 135) -> np.ndarray:
    """(B, T) int64 phoneme ids: lengths U{min_len..T_max} (or given), ids U{1..num_chars-1},
    pad id 0 to the longest; the longest row has length T_max."""
    rng = np.random.Generator(np.random.PCG64([seed, 7919]))
    if lengths is None:
        lo = min_len if min_len is not None else T_max
        lens = rng.integers(lo, T_max + 1, size=B)
        lens[0] = T_max
    else:
        lens = np.asarray(list(lengths))
    T = int(lens.max())
    x = np.zeros((B, T), dtype=np.int64)
    for b, L in enumerate(lens):
        x[b, :L] = rng.integers(1, num_chars, size=int(L))
    return x
