"""FastPitch on MI355X — drop-in for `models/fast_pitch.py`.

Same constructor keywords (:168-199), state_dict keys / shapes / order, ``generate`` /
``forward`` / ``pad`` / ``get_step`` / ``from_config`` / ``from_checkpoint`` surface.
All math runs in libftmi.so; torch allocates buffers and runs the user's callbacks.

Per FFTBlock (:56-91), channels-last (B, T, d), eval numerics (dropout = identity):
  in_proj GEMM (+bias) -> fused flash self-attention (fp32 MFMA, key_padding_mask)
  -> out_proj GEMM (+bias, +residual) -> LayerNorm -> conv1 k9 GEMM (+bias, ReLU)
  -> conv2 k1 GEMM (+bias, +residual) -> LayerNorm
ForwardTransformer (:94-130): token embedding + positional encoding in one kernel (or,
for the postnet, the LengthRegulator expansion + positional encoding in one kernel),
layers, final LayerNorm.
"""
from __future__ import annotations

import math
import os
from pathlib import Path
from typing import Any, Callable, Dict, Optional, Union

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .common_layers import Conv1dParams, LengthRegulator, LinearParams, Packed, pack_conv, presplit
from .forward_tacotron import Embedding, _graphable, _identity

# generate() replays the phoneme phase (three predictors, the prenet, the duration counts:
# ~160 launches over four streams) as a HIP graph, captured on the second sighting of a
# (device, x shape, alpha, callbacks) key; callbacks that are not the identity or graph_safe
# (forward_tacotron.graph_safe) run eagerly between the replay and the launch that reads their
# outputs (a split graph keyed without them).  FTMI_FP_GRAPH=0 keeps it eager.
FP_GRAPH = os.environ.get('FTMI_FP_GRAPH', '1') != '0'
FP_GRAPH_CACHE = 8
from .text.symbols import phonemes


class PositionalEncoding(nn.Module):
    """`fast_pitch.py:16-33`: learnable `scale` (ones) and the sinusoid buffer `pe`
    (max_len, 1, d), computed with the reference's torch ops so the buffer is identical."""

    def __init__(self, d_model: int, dropout: float = 0.1, max_len: int = 5000) -> None:
        super().__init__()
        self.dropout = dropout
        self.scale = nn.Parameter(torch.ones(1))
        pe = torch.zeros(max_len, d_model)
        position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        pe[:, 0::2] = torch.sin(position * div_term)
        pe[:, 1::2] = torch.cos(position * div_term)
        self.register_buffer('pe', pe.unsqueeze(0).transpose(0, 1))

    def rows(self) -> torch.Tensor:
        """pe as contiguous (max_len, d) rows."""
        return self.pe.reshape(self.pe.size(0), -1)


class LayerNormParams(nn.Module):
    """Parameters of nn.LayerNorm(d) (eps 1e-5)."""

    def __init__(self, d: int, eps: float = 1e-5) -> None:
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))

    def forward_cl(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return ops.layernorm(x, self.weight.detach(), self.bias.detach(), self.eps, out=out)


class MultiheadAttentionParams(nn.Module):
    """Parameters of nn.MultiheadAttention(d, heads) (packed in_proj, out_proj Linear)."""

    def __init__(self, d: int, heads: int, dropout: float = 0.0) -> None:
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout = d, heads, dropout
        self.head_dim = d // heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = LinearParams(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)


class FFTBlock(Packed):
    """`fast_pitch.py:56-91`."""

    def __init__(self, d_model: int, nhead: int, conv1_kernel: int, conv2_kernel: int,
                 d_fft: int, dropout: float = 0.1) -> None:
        super().__init__()
        if conv1_kernel % 2 == 0 or conv2_kernel % 2 == 0:
            raise ValueError('even conv kernels change the sequence length (the reference '
                             'residual add fails for them too)')
        self.self_attn = MultiheadAttentionParams(d_model, nhead, dropout)
        self.conv1 = Conv1dParams(d_model, d_fft, conv1_kernel, bias=True)
        self.conv2 = Conv1dParams(d_fft, d_model, conv2_kernel, bias=True)
        self.norm1 = LayerNormParams(d_model)
        self.norm2 = LayerNormParams(d_model)
        self.k1, self.k2, self.heads = conv1_kernel, conv2_kernel, nhead

    def _pack(self):
        a = self.self_attn
        w_in = a.in_proj_weight.detach().contiguous()
        w_out = a.out_proj.weight.detach().contiguous()
        w1, w2 = pack_conv(self.conv1.weight), pack_conv(self.conv2.weight)
        return ((w_in, a.in_proj_bias.detach().contiguous(), presplit(w_in)),
                (w_out, a.out_proj.bias.detach().contiguous(), presplit(w_out)),
                (w1, self.conv1.bias.detach().contiguous(), presplit(w1)),
                (w2, self.conv2.bias.detach().contiguous(), presplit(w2)))

    def _panel_pack(self):
        """Fragment-major f16x3 planes of in_proj, out_proj and (kernel 1) conv2 — the
        operands of ops.panel_proj — cached like every pack (rebuilt with the params)."""
        key = self._pack_key()
        cache = self.__dict__.get('_ftmi_panel')
        if cache is None or cache[0] != key:
            with torch.no_grad():
                (wi, _, _), (wo, _, _), _, (w2, _, _) = self.packed_weights()
                f16 = ops.split_weights_f16
                cache = (key, (f16(wi, frag=True), f16(wo, frag=True),
                               f16(w2, frag=True) if self.k2 == 1 else None))
            self.__dict__['_ftmi_panel'] = cache
        return cache[1]

    def forward_cl(self, x: torch.Tensor, kpm: Optional[torch.Tensor] = None) -> torch.Tensor:
        (wi, bi, si), (wo, bo, so), (w1, b1, s1), (w2, b2, s2) = self.packed_weights()
        d = x.size(2)
        ln1 = (self.norm1.weight.detach(), self.norm1.bias.detach(), self.norm1.eps)
        ln2 = (self.norm2.weight.detach(), self.norm2.bias.detach(), self.norm2.eps)
        # the k = 1 projections with their residual add + LayerNorm as row-panel launches
        # (ops.panel_proj) where the f16x3 path is in force and d fits its 256-column panels;
        # the slab GEMM + layernorm launches otherwise (same projection values)
        panel = ops.panel_ok(d, d, True, si)
        fi, fo, f2 = self._panel_pack() if panel else (None, None, None)
        if panel and ops.kv_fused_ok(x.size(1), d, self.heads, si):
            # the attention's K / V split folded into in_proj (no split pass)
            q, kv = ops.panel_proj_qkv(x, fi, d, self.heads, bias=bi)
            a = ops.attention_kv(q, kv, self.heads, kpm)
            del q
        else:
            if panel:
                qkv = ops.panel_proj(x, fi, 3 * d, bias=bi)
            else:
                qkv, _ = ops.conv1d(x, wi, 1, 0, bias=bi, w_split=si)
            a = ops.attention(qkv, self.heads, kpm)
            del qkv
        if panel:
            h = ops.panel_proj(a, fo, d, bias=bo, residual=x, ln=ln1)
        else:
            h, _ = ops.conv1d(a, wo, 1, 0, bias=bo, residual=x, w_split=so)
            h = self.norm1.forward_cl(h, out=h)
        del a
        f, _ = ops.conv1d(h, w1, self.k1, self.k1 // 2, bias=b1, relu=True, w_split=s1)
        if panel and f2 is not None and ops.panel_ok(f.size(2), d, True, s2):
            return ops.panel_proj(f, f2, d, bias=b2, residual=h, ln=ln2, out=h)
        y, _ = ops.conv1d(f, w2, self.k2, self.k2 // 2, bias=b2, residual=h, w_split=s2)
        del f
        return self.norm2.forward_cl(y, out=y)


class ForwardTransformer(nn.Module):
    """`fast_pitch.py:94-130`."""

    def __init__(self, d_model: int, d_fft: int, layers: int, heads: int, conv1_kernel: int,
                 conv2_kernel: int, dropout: float = 0.1) -> None:
        super().__init__()
        self.d_model = d_model
        self.pos_encoder = PositionalEncoding(d_model, dropout)
        self.layers = nn.ModuleList([FFTBlock(d_model, heads, conv1_kernel, conv2_kernel, d_fft,
                                              dropout) for _ in range(layers)])
        self.norm = LayerNormParams(d_model)

    def _check_len(self, T: int) -> None:
        if T > self.pos_encoder.pe.size(0):
            raise ValueError(f'sequence length {T} exceeds the positional encoding max_len '
                             f'{self.pos_encoder.pe.size(0)}')

    def embed(self, ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
        """Embedding(ids) + positional encoding, fused."""
        self._check_len(ids.size(1))
        return ops.embedding_posenc(ids, table, self.pos_encoder.rows(), self.pos_encoder.scale.detach())

    def expand(self, x: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
        """LengthRegulator(x) + positional encoding, fused (the postnet's input)."""
        self._check_len(index.size(1))
        return ops.lr_posenc(x, index, self.pos_encoder.rows(), self.pos_encoder.scale.detach())

    def layers_cl(self, x: torch.Tensor, kpm: Optional[torch.Tensor] = None) -> torch.Tensor:
        for layer in self.layers:
            x = layer.forward_cl(x, kpm)
        return self.norm.forward_cl(x, out=x)

    def forward(self, x: torch.Tensor, src_pad_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(B, T, d) -> (B, T, d), like the reference (positional encoding added here)."""
        B, T, d = x.shape
        self._check_len(T)
        flat = x.reshape(B * T, d).contiguous()
        ids = torch.arange(B * T, device=x.device, dtype=torch.int64).reshape(B, T)
        h = ops.embedding_posenc(ids, flat, self.pos_encoder.rows(), self.pos_encoder.scale.detach())
        return self.layers_cl(h, src_pad_mask)


class SeriesPredictor(nn.Module):
    """`fast_pitch.py:133-161`: embed -> ForwardTransformer -> Linear(d -> 1) -> / alpha."""

    def __init__(self, num_chars: int, d_model: int, n_heads: int, d_fft: int, layers: int,
                 conv1_kernel: int, conv2_kernel: int, dropout=0.1) -> None:
        super().__init__()
        self.embedding = Embedding(num_chars, d_model)
        self.transformer = ForwardTransformer(heads=n_heads, dropout=dropout, d_model=d_model,
                                              d_fft=d_fft, conv1_kernel=conv1_kernel,
                                              conv2_kernel=conv2_kernel, layers=layers)
        self.lin = LinearParams(d_model, 1)

    def forward_bt(self, x: torch.Tensor, src_pad_mask=None, alpha: float = 1.0) -> torch.Tensor:
        h = self.transformer.embed(x, self.embedding.weight.detach())
        h = self.transformer.layers_cl(h, src_pad_mask)
        return ops.rowdot(h, self.lin.weight.detach().reshape(-1).contiguous(),
                          self.lin.bias.detach(), alpha)

    def forward(self, x: torch.Tensor, src_pad_mask=None, alpha: float = 1.0) -> torch.Tensor:
        return self.forward_bt(x, src_pad_mask, alpha).unsqueeze(-1)


class FastPitch(nn.Module):
    """`models/fast_pitch.py:164-350`."""

    def __init__(self, num_chars: int, durpred_dropout: float, durpred_d_model: int,
                 durpred_n_heads: int, durpred_layers: int, durpred_d_fft: int,
                 pitch_dropout: float, pitch_d_model: int, pitch_n_heads: int, pitch_layers: int,
                 pitch_d_fft: int, energy_dropout: float, energy_d_model: int,
                 energy_n_heads: int, energy_layers: int, energy_d_fft: int,
                 pitch_strength: float, energy_strength: float, d_model: int, conv1_kernel: int,
                 conv2_kernel: int, prenet_layers: int, prenet_heads: int, prenet_fft: int,
                 prenet_dropout: float, postnet_layers: int, postnet_heads: int,
                 postnet_fft: int, postnet_dropout: float, n_mels: int,
                 padding_value=-11.5129) -> None:
        super().__init__()
        self.padding_value = padding_value
        self.lr = LengthRegulator()
        self.dur_pred = SeriesPredictor(num_chars, durpred_d_model, durpred_n_heads, durpred_d_fft,
                                        durpred_layers, conv1_kernel, conv2_kernel, durpred_dropout)
        self.pitch_pred = SeriesPredictor(num_chars, pitch_d_model, pitch_n_heads, pitch_d_fft,
                                          pitch_layers, conv1_kernel, conv2_kernel, pitch_dropout)
        self.energy_pred = SeriesPredictor(num_chars, energy_d_model, energy_n_heads, energy_d_fft,
                                           energy_layers, conv1_kernel, conv2_kernel, energy_dropout)
        self.embedding = Embedding(num_chars, d_model)
        self.prenet = ForwardTransformer(heads=prenet_heads, dropout=prenet_dropout,
                                         conv1_kernel=conv1_kernel, conv2_kernel=conv2_kernel,
                                         d_model=d_model, d_fft=prenet_fft, layers=prenet_layers)
        self.postnet = ForwardTransformer(heads=postnet_heads, dropout=postnet_dropout,
                                          conv1_kernel=conv1_kernel, conv2_kernel=conv2_kernel,
                                          d_model=d_model, d_fft=postnet_fft, layers=postnet_layers)
        self.lin = LinearParams(d_model, n_mels)
        self.register_buffer('step', torch.zeros(1, dtype=torch.long))
        self.pitch_strength = pitch_strength
        self.energy_strength = energy_strength
        self.pitch_proj = Conv1dParams(1, d_model, 3, bias=True)
        self.energy_proj = Conv1dParams(1, d_model, 3, bias=True)
        self.n_mels = n_mels

    def __repr__(self):
        num_params = sum([np.prod(p.size()) for p in self.parameters()])
        return f'FastPitch, num params: {num_params}'

    # ---------------------------------------------------------------------------------
    def _check_device(self, x: torch.Tensor) -> None:
        if not self.embedding.weight.is_cuda:
            raise RuntimeError('forwardtacotron_amd.FastPitch runs on a HIP device only: call '
                               'model.to("cuda") first (there is no CPU path)')
        if x.device != self.embedding.weight.device:
            raise RuntimeError(f'input on {x.device}, model on {self.embedding.weight.device}')

    def _series_proj_weights(self):
        return (self.pitch_proj.weight.detach().reshape(-1, 3).contiguous(),
                self.pitch_proj.bias.detach().contiguous(),
                self.energy_proj.weight.detach().reshape(-1, 3).contiguous(),
                self.energy_proj.bias.detach().contiguous())

    def _encode(self, x, pitch, energy, len_mask):
        """embedding + prenet (key_padding_mask = x == 0) + pitch / energy projections."""
        h = self.prenet.embed(x, self.embedding.weight.detach())
        h = self.prenet.layers_cl(h, len_mask)
        wp, bp, we, be = self._series_proj_weights()
        ops.series_proj_add(h, pitch, wp, bp, self.pitch_strength, energy, we, be,
                            self.energy_strength)
        return h

    def _decode(self, enc, index, kpm=None):
        """LR + posenc (fused) -> postnet layers -> lin -> (B, n_mels, T_mel)."""
        h = self.postnet.expand(enc, index)
        h = self.postnet.layers_cl(h, kpm)
        B, T_mel = index.shape
        mel = torch.empty(B, self.n_mels, T_mel, device=enc.device)
        w, b, w3 = self.lin.packed_weights()
        ops.conv1d(h, w, 1, 0, bias=b, out_t=mel, want_y=False, w_split=w3)
        return mel

    def _side_streams(self, device):
        cache = self.__dict__.setdefault('_ftmi_streams', {})
        if device not in cache:
            cache[device] = [torch.cuda.Stream(device=device) for _ in range(3)]
        return cache[device]


    def __prepare_scriptable__(self):
        """`torch.jit.script(model)` (README.md:149-161 exports the reference this way) is not
        possible here: the compute runs in libftmi.so through ctypes, which TorchScript
        cannot call.  Fail with the reason instead of a TorchScript frontend error; the
        scripted entry point's behaviour is available eagerly (`generate_jit`)."""
        raise RuntimeError(f'{type(self).__name__} runs on libftmi.so (HIP kernels called through '
                           'ctypes) and cannot be compiled by torch.jit.script; call generate_jit / '
                           'generate eagerly')
    def generate(self,
                 x: torch.Tensor,
                 alpha=1.0,
                 pitch_function: Callable[[torch.Tensor], torch.Tensor] = _identity,
                 energy_function: Callable[[torch.Tensor], torch.Tensor] = _identity,
                 batch=None) -> Dict[str, torch.Tensor]:
        """`models/fast_pitch.py:286-303`: predictors without masks; the prenet on side
        streams overlaps the duration path and its one host sync (T_mel).  `batch`: a
        sharded.GlobalBatch when x is one rank's shard of a larger batch.  Runs under the
        f16x3 range guard (ops.run_checked)."""
        if self.training:  # the module-tree walk of eval() is host time on every call
            self.eval()
        self._check_device(x)
        return ops.run_checked(
            lambda: self._generate(x, alpha, pitch_function, energy_function, batch), x.device,
            reduce=None if batch is None else batch.status)

    def _phase(self, x, alpha, pitch_function, energy_function, batch=None, capture=False):
        """The phoneme phase: the prenet on a side stream beside the pitch / energy
        predictors, the duration predictor and counts on the caller's stream, then the
        pitch / energy projections added to the prenet output.  Returns (dur_hat, pitch_hat,
        energy_hat, h, offsets, T_mel); capture=True (graph capture): no host sync, the T_mel
        slot holds max(totals) on the device.  pitch_function = energy_function = None
        (capture only): the predictors' raw outputs, h without their projections (the split
        graph of _phase_graph)."""
        main = torch.cuda.current_stream(x.device)
        s_pitch, s_energy, s_prenet = self._side_streams(x.device)
        for s in (s_pitch, s_energy, s_prenet):
            s.wait_stream(main)
        len_mask = x == 0
        with torch.cuda.stream(s_prenet):
            h = self.prenet.embed(x, self.embedding.weight.detach())
            h = self.prenet.layers_cl(h, len_mask)
        with torch.cuda.stream(s_pitch):
            pitch_hat = self.pitch_pred.forward_bt(x).unsqueeze(1)
            if pitch_function is not None:
                pitch_hat = pitch_function(pitch_hat)
        with torch.cuda.stream(s_energy):
            energy_hat = self.energy_pred.forward_bt(x).unsqueeze(1)
            if energy_function is not None:
                energy_hat = energy_function(energy_hat)
        dur_hat = self.dur_pred.forward_bt(x, alpha=alpha)
        if batch is None:
            offsets, totals, _ = ops.duration_counts(dur_hat, apply_fill=True)
            T_mel = totals.max() if capture else int(totals.max().item())
        else:
            offsets, totals = batch.duration_counts(dur_hat)
            T_mel = batch.t_mel(totals)
        for s, t in ((s_pitch, pitch_hat), (s_energy, energy_hat), (s_prenet, h),
                     (s_prenet, len_mask)):
            main.wait_stream(s)
            if not capture:
                t.record_stream(main)
        if pitch_function is not None and energy_function is not None:
            wp, bp, we, be = self._series_proj_weights()
            ops.series_proj_add(h, pitch_hat, wp, bp, self.pitch_strength, energy_hat, we, be,
                                self.energy_strength)
        return dur_hat, pitch_hat, energy_hat, h, offsets, T_mel

    def _weights_key(self):
        """(data_ptr, _version) of every parameter and buffer (ForwardTacotron._weights_key)."""
        return tuple((t.data_ptr(), t._version) for m in self.modules()
                     for d in (m._parameters, m._buffers) for t in d.values() if t is not None)

    def _phase_graph(self, x, alpha, pitch_fn, energy_fn):
        """The phoneme phase as a HIP graph (ForwardTacotron._phoneme_graph's protocol): a
        key is captured the second time it is seen; x is copied into the static input; dur /
        pitch / energy are cloned out; h and the offsets are consumed by this call's decoder
        (the next replay waits for the decoder's completion event); a weights change drops
        the captured phases.  Returns ((dur, pitch, energy, h, offsets, T_mel), entry) or
        None (run the eager phase)."""
        cache = self.__dict__.setdefault('_ftmi_graphs', {})
        seen = self.__dict__.setdefault('_ftmi_graph_seen', {})
        # callbacks not marked graph_safe run eagerly between the replay and the one launch
        # that reads their outputs (ForwardTacotron._phoneme_graph's split graph)
        split = not (_graphable(pitch_fn) and _graphable(energy_fn))
        key = ((x.device, tuple(x.shape), float(alpha), 'split', ops.MMA) if split else
               (x.device, tuple(x.shape), float(alpha), pitch_fn, energy_fn, ops.MMA))
        cap_p, cap_e = (None, None) if split else (pitch_fn, energy_fn)
        ent = cache.pop(key, None)
        fresh = False
        if ent is None:
            n = seen.get(key, 0)
            if n < 0:
                return None
            if len(seen) >= 64 * FP_GRAPH_CACHE:
                seen.clear()
            seen[key] = n + 1
            if n == 0:
                return None
            wkey = self._weights_key()
            sx = x.clone()
            try:
                self._phase(sx, alpha, cap_p, cap_e, capture=True)  # warm-up
                torch.cuda.synchronize(x.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    outs = self._phase(sx, alpha, cap_p, cap_e, capture=True)
            except Exception:  # pylint: disable=broad-except
                torch.cuda.synchronize(x.device)
                seen[key] = -1
                return None
            ent = {'g': g, 'sx': sx, 'outs': outs, 'wkey': wkey, 'done': torch.cuda.Event()}
            ent['done'].record(torch.cuda.current_stream(x.device))
            fresh = True
            while len(cache) >= FP_GRAPH_CACHE:
                cache.pop(next(iter(cache)))
        cache[key] = ent
        main = torch.cuda.current_stream(x.device)
        main.wait_event(ent['done'])
        ent['sx'].copy_(x)
        ent['g'].replay()
        if not fresh and self._weights_key() != ent['wkey']:
            main.synchronize()
            cache.clear()
            return None
        dur_hat, pitch_hat, energy_hat, h, offsets, tmax = ent['outs']
        t_host = torch.empty((), dtype=tmax.dtype, pin_memory=True)
        t_host.copy_(tmax, non_blocking=True)
        t_ready = torch.cuda.Event()
        t_ready.record(main)
        dur_hat, pitch_hat, energy_hat = dur_hat.clone(), pitch_hat.clone(), energy_hat.clone()
        if split:  # the callbacks on the predictors' outputs, then their projections
            pitch_hat, energy_hat = pitch_fn(pitch_hat), energy_fn(energy_hat)
            wp, bp, we, be = self._series_proj_weights()
            ops.series_proj_add(h, pitch_hat, wp, bp, self.pitch_strength, energy_hat, we, be,
                                self.energy_strength)
        t_ready.synchronize()
        return (dur_hat, pitch_hat, energy_hat, h, offsets, int(t_host)), ent

    def _generate(self, x, alpha, pitch_function, energy_function, batch):
        with torch.no_grad():
            phase = ent = None
            if FP_GRAPH and batch is None and not ops.forced_exact():
                r = self._phase_graph(x, alpha, pitch_function, energy_function)
                if r is not None:
                    phase, ent = r
            if phase is None:
                phase = self._phase(x, alpha, pitch_function, energy_function, batch)
            dur_hat, pitch_hat, energy_hat, h, offsets, T_mel = phase
            index = ops.lr_index(offsets, T_mel)
            mel = self._decode(h, index)
            if ent is not None:  # the decoder has consumed the graph's static buffers
                ent['done'].record(torch.cuda.current_stream(x.device))
            return {'mel': mel, 'mel_post': mel, 'dur': dur_hat,
                    'pitch': pitch_hat, 'energy': energy_hat}

    def _generate_mel(self, x, dur_hat, pitch_hat, energy_hat):
        """`models/fast_pitch.py:315-340`."""
        with torch.no_grad():
            h = self._encode(x, pitch_hat, energy_hat, x == 0)
            offsets, totals, _ = ops.duration_counts(dur_hat, apply_fill=False)
            T_mel = int(totals.max().item())
            mel = self._decode(h, ops.lr_index(offsets, T_mel))
        return {'mel': mel, 'mel_post': mel, 'dur': dur_hat, 'pitch': pitch_hat,
                'energy': energy_hat}

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Teacher-forced pass (`models/fast_pitch.py:233-283`), inference numerics."""
        x = batch['x']
        self._check_device(x)
        if self.training:
            self.step += 1
        return ops.run_checked(lambda: self._forward(batch), x.device)

    def _forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        x = batch['x']
        mel = batch['mel']
        dur = batch['dur']
        mel_lens = batch['mel_len']
        pitch = batch['pitch'].unsqueeze(1)
        energy = batch['energy'].unsqueeze(1)
        with torch.no_grad():
            len_mask = x == 0
            dur_hat = self.dur_pred.forward_bt(x, len_mask)
            pitch_hat = self.pitch_pred.forward_bt(x, len_mask).unsqueeze(1)
            energy_hat = self.energy_pred.forward_bt(x, len_mask).unsqueeze(1)
            h = self._encode(x, pitch, energy, len_mask)
            dur_c = dur.float().contiguous()
            offsets, totals, _ = ops.duration_counts(dur_c, apply_fill=False)
            if dur_c.data_ptr() != dur.data_ptr():
                dur.copy_(dur_c)  # the reference's LR clips batch['dur'] in place
            T_mel = int(totals.max().item())
            index = ops.lr_index(offsets, T_mel)
            lens = mel_lens.to(device=x.device, dtype=torch.int64)
            kpm = torch.arange(T_mel, device=x.device)[None, :] >= lens[:, None]
            out = self._decode(h, index, kpm)
            x_post = self.pad(out, mel.size(2))
            x_mel = self.pad(out, mel.size(2))
        return {'mel': x_mel, 'mel_post': x_post,
                'dur': dur_hat, 'pitch': pitch_hat, 'energy': energy_hat}

    def pad(self, x: torch.Tensor, max_len: int) -> torch.Tensor:
        """`models/fast_pitch.py:305-308`."""
        x = x[:, :, :max_len]
        if x.size(2) < max_len:
            pad = torch.full((x.size(0), x.size(1), max_len - x.size(2)), self.padding_value,
                             device=x.device, dtype=x.dtype)
            x = torch.cat([x, pad], 2)
        return x

    def get_step(self) -> int:
        return self.step.data.item()

    @classmethod
    def from_config(cls, config: Dict[str, Any]) -> 'FastPitch':
        model_config = dict(config['fast_pitch']['model'])
        model_config['num_chars'] = len(phonemes)
        model_config['n_mels'] = config['dsp']['num_mels']
        return FastPitch(**model_config)

    @classmethod
    def from_checkpoint(cls, path: Union[Path, str]) -> 'FastPitch':
        checkpoint = torch.load(path, map_location=torch.device('cpu'), weights_only=True)
        model = FastPitch.from_config(checkpoint['config'])
        model.load_state_dict(checkpoint['model'])
        return model
