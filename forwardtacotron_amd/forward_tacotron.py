"""ForwardTacotron (V2: pitch + energy) on MI355X — drop-in for `models/forward_tacotron.py`.

Same constructor keywords (:93-118), same state_dict keys and shapes (checkpoints from the
reference load unchanged), same ``generate`` / ``generate_jit`` / ``forward`` /
``from_config`` / ``from_checkpoint`` / ``get_step`` surface and return dictionaries.
All math runs in libftmi.so (HIP, gfx950, fp32); torch only allocates device buffers,
moves tokens / results and runs the user's pitch / energy callbacks.

Pipeline of ``generate`` (channels-last activations, one HIP stream):
  predictors  embed -> 3x conv k5 (ReLU, BN) -> GRU in-proj GEMM -> GRU recurrence -> head
  durations   fill-2 rule + clip + counts + scan in one kernel (bit-exact), one host sync
              for T_mel (the reference syncs at the same point, :254 and common_layers.py:16)
  encoder     embed -> CBHG(K=16) -> + pitch/energy conv projections
  decoder     LSTM input projection at PHONEME rate (x W_ih^T + b), the recurrence reads
              it through the LengthRegulator index map: LR(x) W_ih^T == LR(x W_ih^T), so the
              expanded (B, T_mel, 512) tensor and 7x of the projection FLOPs are never needed;
              lin (-> mel, written both channels-last and as (B, 80, T_mel))
  postnet     CBHG(K=8) on the channels-last mel -> post_proj (-> mel_post (B, 80, T_mel))
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Callable, Dict, Union

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .common_layers import (CBHG, BatchNormConv, BiRNN, Conv1dParams, LengthRegulator,
                            LinearParams, Packed, pack_conv)
from .text.symbols import phonemes


def _identity(t: torch.Tensor) -> torch.Tensor:
    """The default pitch / energy callback (the reference's `lambda x: x`)."""
    return t


def graph_safe(fn: Callable[[torch.Tensor], torch.Tensor]) -> Callable[[torch.Tensor], torch.Tensor]:
    """Mark a pitch / energy callback as safe to capture in the phoneme-phase HIP graph: a
    pure function of its tensor argument made of device-side torch ops, whose behaviour
    does not change between calls (no Python-side state it reads changes: closure
    variables, attributes, scalars).  gen_forward.py's `lambda x: x * amp` is, for the run's
    fixed `amp`.  An unmarked callback runs eagerly on every call, as the reference calls
    it (`models/forward_tacotron.py:258-261`); returns fn."""
    fn._ftmi_graph_safe = True
    return fn


def _graphable(fn) -> bool:
    return fn is _identity or getattr(fn, '_ftmi_graph_safe', False) is True


# generate() replays the phoneme phase as a HIP graph (captured per (device, x shape, alpha,
# callbacks), see _phoneme_graph) when the phase is launch-bound: B*T <= GRAPH_MAX_TOKENS.
# Measured: c2 (B = 1, T = 120) 4.18 -> 3.57 ms/step; c3 (B = 64, T = 200) 9.20 -> 9.58, the
# replay loses the prenet stream's priority and the kernels are long enough to hide the host
# issue anyway.  FTMI_GRAPH=0, or GRAPH = False, keeps it eager.
GRAPH = os.environ.get('FTMI_GRAPH', '1') != '0'
GRAPH_MAX_TOKENS = int(os.environ.get('FTMI_GRAPH_MAX_TOKENS', 2048))
GRAPH_CACHE = 8  # captured phases kept per model (least recently used dropped)


class Embedding(nn.Module):
    """Parameters of nn.Embedding(num, dim)."""

    def __init__(self, num: int, dim: int) -> None:
        super().__init__()
        self.num_embeddings, self.embedding_dim = num, dim
        self.weight = nn.Parameter(torch.randn(num, dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.embedding(x, self.weight.detach())


class SeriesPredictor(Packed):
    """`models/forward_tacotron.py:14-55`: embed -> [Conv1d k5 -> ReLU -> BN]x3 -> biGRU ->
    Linear(2h -> 1) -> / alpha."""

    def __init__(self, num_chars, emb_dim=64, conv_dims=256, rnn_dims=64, dropout=0.5):
        super().__init__()
        self.embedding = Embedding(num_chars, emb_dim)
        self.convs = nn.ModuleList([
            BatchNormConv(emb_dim, conv_dims, 5, relu=True),
            BatchNormConv(conv_dims, conv_dims, 5, relu=True),
            BatchNormConv(conv_dims, conv_dims, 5, relu=True),
        ])
        self.rnn = BiRNN(conv_dims, rnn_dims, 'gru')
        self.lin = LinearParams(2 * rnn_dims, 1)
        self.dropout = dropout

    def _pack(self):
        return self.lin.weight.detach().reshape(-1).contiguous(), self.lin.bias.detach().contiguous()

    def forward_bt(self, x: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
        """(B, T) ids -> (B, T) series (before the reference's trailing unsqueeze)."""
        h = ops.embedding(x, self.embedding.weight.detach())
        for conv in self.convs:
            h = conv.forward_cl(h)
        h = self.rnn.forward_cl(h)
        w, b = self.packed_weights()
        return ops.rowdot(h, w, b, alpha)

    def forward(self, x: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
        """(B, T) -> (B, T, 1), like the reference."""
        return self.forward_bt(x, alpha).unsqueeze(-1)


class ForwardTacotron(nn.Module):
    """ForwardTacotron V2; see module docstring.  Reference: models/forward_tacotron.py:74-350."""

    def __init__(self,
                 embed_dims: int,
                 series_embed_dims: int,
                 num_chars: int,
                 durpred_conv_dims: int,
                 durpred_rnn_dims: int,
                 durpred_dropout: float,
                 pitch_conv_dims: int,
                 pitch_rnn_dims: int,
                 pitch_dropout: float,
                 pitch_strength: float,
                 energy_conv_dims: int,
                 energy_rnn_dims: int,
                 energy_dropout: float,
                 energy_strength: float,
                 rnn_dims: int,
                 prenet_dims: int,
                 prenet_k: int,
                 postnet_num_highways: int,
                 prenet_dropout: float,
                 postnet_dims: int,
                 postnet_k: int,
                 prenet_num_highways: int,
                 postnet_dropout: float,
                 n_mels: int,
                 padding_value=-11.5129):
        # the constructor keywords, for the TorchScript archive (jit.model_config)
        ctor = {k: v for k, v in locals().items() if k not in ('self', '__class__')}
        super().__init__()
        self._ctor_kwargs = ctor
        self.rnn_dims = rnn_dims
        self.padding_value = padding_value
        self.register_buffer('step', torch.zeros(1, dtype=torch.long))
        # registration order follows the reference so state_dict() iterates identically
        self.embedding = Embedding(num_chars, embed_dims)
        self.prenet = CBHG(K=prenet_k, in_channels=embed_dims, channels=prenet_dims,
                           proj_channels=[prenet_dims, embed_dims],
                           num_highways=prenet_num_highways, dropout=prenet_dropout)
        self.pitch_pred = SeriesPredictor(num_chars, series_embed_dims, pitch_conv_dims,
                                          pitch_rnn_dims, pitch_dropout)
        self.energy_pred = SeriesPredictor(num_chars, series_embed_dims, energy_conv_dims,
                                           energy_rnn_dims, energy_dropout)
        self.pitch_proj = Conv1dParams(1, 2 * prenet_dims, 3, bias=True)
        self.energy_proj = Conv1dParams(1, 2 * prenet_dims, 3, bias=True)
        self.pitch_strength = pitch_strength
        self.energy_strength = energy_strength
        self.lr = LengthRegulator()
        self.dur_pred = SeriesPredictor(num_chars, series_embed_dims, durpred_conv_dims,
                                        durpred_rnn_dims, durpred_dropout)
        self.lstm = BiRNN(2 * prenet_dims, rnn_dims, 'lstm')
        self.lin = LinearParams(2 * rnn_dims, n_mels)
        self.postnet = CBHG(K=postnet_k, in_channels=n_mels, channels=postnet_dims,
                            proj_channels=[postnet_dims, n_mels],
                            num_highways=postnet_num_highways, dropout=postnet_dropout)
        self.post_proj = LinearParams(2 * postnet_dims, n_mels, bias=False)
        self.n_mels = n_mels
        # the decoder-side recurrences run alone on the device: they may spread over every
        # CU (the phoneme phase's four GRUs share it and keep the compact form)
        self.lstm.spread = self.postnet.rnn.spread = True

    def __repr__(self):
        num_params = sum([np.prod(p.size()) for p in self.parameters()])
        return f'ForwardTacotron, num params: {num_params}'

    # ---------------------------------------------------------------------------------
    def _check_device(self, x: torch.Tensor) -> None:
        if not self.embedding.weight.is_cuda:
            raise RuntimeError('forwardtacotron_amd.ForwardTacotron runs on a HIP device only: '
                               'call model.to("cuda") first (there is no CPU path)')
        if x.device != self.embedding.weight.device:
            raise RuntimeError(f'input on {x.device}, model on {self.embedding.weight.device}')

    def _series_proj_weights(self):
        return (self.pitch_proj.weight.detach().reshape(-1, 3).contiguous(),
                self.pitch_proj.bias.detach().contiguous(),
                self.energy_proj.weight.detach().reshape(-1, 3).contiguous(),
                self.energy_proj.bias.detach().contiguous())

    def _folded_series_weights(self):
        """The pitch / energy projections carried through the LSTM's input projection:
        W_ih (enc + ps proj_p(pitch) + es proj_e(energy)) + b
          = (W_ih enc + b) + ps (W_ih W_p * pitch + W_ih b_p) + es (W_ih W_e * energy + W_ih b_e),
        so the projection of enc can start as soon as the prenet ends and the predictors'
        outputs are added to its (B, T, 4H) rows afterwards (the same series_proj_add kernel
        with 4H-wide weights).  Made once per weights version, in float64."""
        key = (self.lstm._pack_key(), self.pitch_proj.weight._version, self.pitch_proj.bias._version,
               self.energy_proj.weight._version, self.energy_proj.bias._version,
               self.pitch_proj.weight.data_ptr(), self.energy_proj.weight.data_ptr())
        cache = self.__dict__.get('_ftmi_fold')
        if cache is None or cache[0] != key:
            with torch.no_grad():
                w_ih = self.lstm.packed_weights()[0].double()  # [2*4H][In], both directions
                out = []
                for w, b in (self.pitch_proj.weight, self.pitch_proj.bias), \
                            (self.energy_proj.weight, self.energy_proj.bias):
                    out.append((w_ih @ w.detach().double().reshape(-1, 3)).float().contiguous())
                    out.append((w_ih @ b.detach().double()).float().contiguous())
            cache = (key, tuple(out))
            self.__dict__['_ftmi_fold'] = cache
        return cache[1]

    def _encode(self, x: torch.Tensor, pitch: torch.Tensor, energy: torch.Tensor) -> torch.Tensor:
        """embedding -> prenet CBHG -> + pitch / energy projections: (B, T, 2*prenet_dims)."""
        h = ops.embedding(x, self.embedding.weight.detach())
        h = self.prenet.forward_cl(h)
        wp, bp, we, be = self._series_proj_weights()
        ops.series_proj_add(h, pitch, wp, bp, self.pitch_strength, energy, we, be,
                            self.energy_strength)
        return h

    def _decode(self, enc: torch.Tensor, index: torch.Tensor, lengths=None, T_out=None, xp=None):
        """LSTM over LR(enc) (through the index map) -> lin -> postnet -> post_proj.
        xp: the LSTM input projection of enc if already queued (self.lstm.project)."""
        B = enc.size(0)
        T_mel = index.size(1)
        if xp is None:
            xp = self.lstm.project(enc)
        lstm_out = self.lstm.recur(xp, T=T_mel, index=index, lengths=lengths,
                                   pad_value=self.padding_value)
        del xp
        mel_cl = torch.empty(B, T_mel, self.n_mels, device=enc.device)
        mel = torch.empty(B, self.n_mels, T_mel, device=enc.device)
        w, b, w3 = self.lin.packed_weights()
        ops.conv1d(lstm_out, w, 1, 0, bias=b, out=mel_cl, out_t=mel, w_split=w3)
        del lstm_out
        post = self.postnet.forward_cl(mel_cl)
        mel_post = torch.empty(B, self.n_mels, T_mel, device=enc.device)
        w, _, w3 = self.post_proj.packed_weights()
        ops.conv1d(post, w, 1, 0, out_t=mel_post, want_y=False, w_split=w3)
        return mel, mel_post

    # ---------------------------------------------------------------------------------
    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Teacher-forced pass (`models/forward_tacotron.py:184-242`), inference numerics."""
        x = batch['x']
        self._check_device(x)
        if self.training:
            self.step += 1
        return ops.run_checked(lambda: self._forward(batch), x.device)

    def _forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        x = batch['x']
        mel = batch['mel']
        mel_lens = batch['mel_len']
        dur = batch['dur']
        pitch = batch['pitch'].unsqueeze(1)
        energy = batch['energy'].unsqueeze(1)
        with torch.no_grad():
            dur_hat = self.dur_pred.forward_bt(x)
            pitch_hat = self.pitch_pred.forward_bt(x).unsqueeze(1)
            energy_hat = self.energy_pred.forward_bt(x).unsqueeze(1)
            enc = self._encode(x, pitch, energy)
            dur_c = dur.float().contiguous()
            offsets, totals, _ = ops.duration_counts(dur_c, apply_fill=False)
            if dur_c.data_ptr() != dur.data_ptr():
                dur.copy_(dur_c)  # the reference's LR clips batch['dur'] in place
            lens = mel_lens.to(torch.int64)
            T_pack = int(lens.max().item())
            if T_pack > int(totals.max().item()):
                raise RuntimeError('mel_len exceeds the length-regulated sequence length')
            index = ops.lr_index(offsets, T_pack)
            x_mel, x_post = self._decode(enc, index, lengths=lens.to(x.device))
            x_post = self._pad(x_post, mel.size(2))
            x_mel = self._pad(x_mel, mel.size(2))
        return {'mel': x_mel, 'mel_post': x_post,
                'dur': dur_hat, 'pitch': pitch_hat, 'energy': energy_hat}

    def _side_streams(self, device, B: int, T: int = 0):
        """(pitch, energy, prenet) streams.  The prenet CBHG -> LSTM input projection is the
        phoneme phase's critical chain: its stream gets the higher priority
        (FTMI_PRENET_PRIORITY, default -1 = high; 0 = same as the others), so the
        predictors fill the CUs it leaves idle instead of delaying it.
        The four recurrences of the phase (three predictor GRUs, the prenet GRU) are
        persistent kernels whose workgroups wait on each other: run concurrently they must
        fit the CUs together.  The prenet stream's two persistent kernels — the spread CBHG
        tail at few rows (ops.hs_spread_blocks: its workgroups wait on each other too), then
        the prenet GRU — run one after the other, so the larger of them counts beside the
        predictors' three.  When they do not fit (large batches), every stream is the
        caller's (the phase runs serialised) — never a co-residency timeout."""
        cache = self.__dict__.setdefault('_ftmi_streams', {})
        if device not in cache:
            prio = int(os.environ.get('FTMI_PRENET_PRIORITY', '-1'))
            cache[device] = [torch.cuda.Stream(device=device), torch.cuda.Stream(device=device),
                             torch.cuda.Stream(device=device, priority=prio)]
        fits = self.__dict__.setdefault('_ftmi_concurrent', {})
        key = (device, B, T, ops.RNN_MMA, bool(ops._FORCED), os.environ.get('FTMI_HS_SPREAD', '1'))
        if key not in fits:
            preds = (self.dur_pred.rnn, self.pitch_pred.rnn, self.energy_pred.rnn)
            need = sum(ops.rnn_blocks(r.cell, B, r.hidden) for r in preds)
            # the prenet stream's persistent kernels (the spread CBHG tail, then the prenet
            # GRU) run one after the other on it: the larger of the two beside the predictors.
            # The spread tail counts only where it would run (the fused stack applies and
            # spreads at this row count); where predictors + spread tail would not fit, the
            # tail takes the one-workgroup-per-64-rows stack kernel (nothing to co-schedule)
            # and the phase stays concurrent (~900 prenet rows)
            pre = ops.rnn_blocks(self.prenet.rnn.cell, B, self.prenet.rnn.hidden)
            spread = self.prenet.spread_blocks(B * T)
            cus = ops._num_cus()
            use_spread = spread > 0 and need + max(pre, spread) <= cus
            fits[key] = (0 < need + pre <= cus and pre > 0, use_spread)
        concurrent, use_spread = fits[key]
        self.prenet.allow_spread = use_spread
        if not concurrent:
            main = torch.cuda.current_stream(device)
            return [main, main, main]
        return cache[device]

    def _weights_key(self):
        """(data_ptr, _version) of every parameter and buffer: changes on load_state_dict,
        .to(), in-place updates and replaced tensors (the list of tensors is cached and
        rebuilt when an owner no longer holds the same object, like Packed._pack_key)."""
        refs = self.__dict__.get('_ftmi_wrefs')
        if refs is None or any(d.get(n) is not t for d, n, t in refs):
            refs = [(d, n, t) for m in self.modules() for d in (m._parameters, m._buffers)
                    for n, t in d.items() if t is not None]
            self.__dict__['_ftmi_wrefs'] = refs
        return tuple((t.data_ptr(), t._version) for _, _, t in refs)

    def _phoneme_graph(self, x, alpha, pitch_fn, energy_fn):
        """The phoneme phase (unsharded) as a HIP graph: ~40 launches from Python over four
        streams become one replay, which matters where the kernels are short (batch 1: the
        host issue rate, not the device, set the phase's length).
        Keyed on (device, x shape, alpha, the callbacks' identity, matrix paths); a key is
        captured the SECOND time it is seen (a one-off shape — gen_forward.py's sentences
        of different lengths — stays eager: capture costs ~3 eager phases).  The default
        identity and callbacks marked `graph_safe` (pure device-side torch ops whose effect
        does not change between calls) are captured with the phase.  Any other callback —
        gen_forward.py's plain `lambda x: x * amp` — splits it: the graph holds everything
        but the callbacks and the one launch that reads their outputs (the pitch / energy
        projections added to the LSTM input projection, series_proj_add); after each replay
        the callbacks run eagerly on the predictors' outputs (fresh tensors, on the caller's
        stream), as the reference calls them, and that launch follows.  The split graph is
        keyed without the callbacks' identity (they are not in it).  FTMI_GRAPH=0 (or
        forward_tacotron.GRAPH = False) turns capture
        off.  A capture that fails (a callback that syncs or leaves the device) marks the
        key eager for good.
        Static buffers: x is copied in, dur / pitch / energy are cloned out (they go back to
        the caller); enc, the offsets and the LSTM input projection are consumed by this
        call's decoder — the next replay waits for the decoder's completion event
        (generate() records it), so calls on different streams never overwrite buffers a
        decoder still reads.  The entry keeps every module's weight pack alive and the
        model-wide weights key of its capture: after each replay (while it runs) the key is
        compared with the model's, and on a change (load_state_dict, .to(), in-place
        updates) every captured phase is dropped and the call falls back to the eager phase
        (the stale replay read the old, still-allocated packs; its outputs are discarded).
        Returns (phase outputs, entry) or None (run the eager phase)."""
        cache = self.__dict__.setdefault('_ftmi_graphs', {})
        seen = self.__dict__.setdefault('_ftmi_graph_seen', {})
        # split: a callback that is not graph_safe runs eagerly between the captured
        # predictors and the one launch that consumes its output (series_proj_add)
        split = not (_graphable(pitch_fn) and _graphable(energy_fn))
        key = ((x.device, tuple(x.shape), float(alpha), 'split', ops.MMA, ops.RNN_MMA) if split else
               (x.device, tuple(x.shape), float(alpha), pitch_fn, energy_fn, ops.MMA, ops.RNN_MMA))
        cap_p, cap_e = (None, None) if split else (pitch_fn, energy_fn)
        ent = cache.pop(key, None)
        fresh = False
        if ent is None:
            n = seen.get(key, 0)
            if n < 0:
                return None  # capture failed before: eager for good
            if len(seen) >= 64 * GRAPH_CACHE:  # e.g. a new lambda per call: forget sightings
                seen.clear()
            seen[key] = n + 1
            if n == 0:
                return None  # first sighting: eager
            wkey = self._weights_key()
            sx = x.clone()
            try:
                self._phoneme_phase(sx, alpha, cap_p, cap_e, capture=True)  # warm-up
                torch.cuda.synchronize(x.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    outs = self._phoneme_phase(sx, alpha, cap_p, cap_e, capture=True)
            except Exception:  # pylint: disable=broad-except
                torch.cuda.synchronize(x.device)
                seen[key] = -1
                return None
            packs = [m.__dict__.get('_ftmi_pack') for m in self.modules()]
            ent = {'g': g, 'sx': sx, 'outs': outs, 'wkey': wkey, 'packs': packs,
                   'done': torch.cuda.Event()}
            ent['done'].record(torch.cuda.current_stream(x.device))
            fresh = True
            while len(cache) >= GRAPH_CACHE:
                cache.pop(next(iter(cache)))
        cache[key] = ent  # most recently used last
        main = torch.cuda.current_stream(x.device)
        main.wait_event(ent['done'])  # the previous decoder is done with the static buffers
        ent['sx'].copy_(x)
        ent['g'].replay()
        if not fresh and self._weights_key() != ent['wkey']:
            main.synchronize()  # the stale replay must finish before its graph is freed
            cache.clear()
            return None
        dur_hat, pitch_hat, energy_hat, enc, offsets, tmax, xp = ent['outs']
        t_host = torch.empty((), dtype=tmax.dtype, pin_memory=True)
        t_host.copy_(tmax, non_blocking=True)
        t_ready = torch.cuda.Event()
        t_ready.record(main)
        dur_hat, pitch_hat, energy_hat = dur_hat.clone(), pitch_hat.clone(), energy_hat.clone()
        if split:  # the callbacks on the predictors' outputs, then their projections
            pitch_hat, energy_hat = pitch_fn(pitch_hat), energy_fn(energy_hat)
            wp, bp, we, be = self._folded_series_weights()
            ops.series_proj_add(xp, pitch_hat, wp, bp, self.pitch_strength, energy_hat, we,
                                be, self.energy_strength)
        t_ready.synchronize()
        return (dur_hat, pitch_hat, energy_hat, enc, offsets, int(t_host), xp), ent

    def _phoneme_phase(self, x, alpha, pitch_fn, energy_fn, batch=None, capture=False):
        """Duration / pitch / energy predictors and the prenet CBHG are independent: pitch,
        energy and the prenet run on three side streams while the caller's stream runs the
        duration predictor and the LengthRegulator bookkeeping (fill-2 rule, counts, T_mel).
        The prenet stream (high priority: its chain is the phase's critical path) continues
        with the LSTM input projection of the prenet output (independent of the predictors)
        and then, after the pitch / energy streams, adds their projections through W_ih:
        none of it depends on T_mel, so it runs while the duration path finishes and the
        host waits for T_mel (the one host sync, a pinned copy queued right after the
        duration kernel).  Issue order = priority order: prenet, durations, pitch,
        energy.  Returns (dur_hat, pitch_hat, energy_hat, enc, (offsets, index), T_mel, xp)
        with every tensor ready on the caller's stream (xp: the LSTM input projection of enc
        plus the pitch / energy projections, folded through W_ih; enc itself does not carry
        them; index: the LR index map, queued on the caller's stream before it joins the side
        streams).  capture=True (graph capture, see _phoneme_graph): no host sync, the T_mel
        slot holds max(totals) on the device and the offsets slot plain offsets.
        pitch_fn = energy_fn = None (capture only): the predictors' raw outputs are returned
        and xp does not carry their projections yet (the split graph of _phoneme_graph)."""
        main = torch.cuda.current_stream(x.device)
        s_pitch, s_energy, s_prenet = self._side_streams(x.device, x.size(0), x.size(1))
        for s in (s_pitch, s_energy, s_prenet):
            s.wait_stream(main)
        with torch.cuda.stream(s_prenet):
            enc = self.prenet.forward_cl(ops.embedding(x, self.embedding.weight.detach()))
            # the LSTM input projection right after the prenet; the pitch / energy terms are
            # added to its rows once the predictors are done (_folded_series_weights)
            xp = self.lstm.project(enc)
        dur_hat = self.dur_pred.forward_bt(x, alpha=alpha)
        t_host = t_ready = None
        tmax = None
        if batch is None and capture:
            offsets, totals, _ = ops.duration_counts(dur_hat, apply_fill=True)
            tmax = totals.max()
        elif batch is None:
            offsets, totals, _ = ops.duration_counts(dur_hat, apply_fill=True)
            # the one host sync (output size is data dependent): max(totals) goes to pinned
            # host memory now and is read after the T_mel-independent work is queued
            t_host = torch.empty((), dtype=totals.dtype, pin_memory=True)
            t_host.copy_(totals.max(), non_blocking=True)
            t_ready = torch.cuda.Event()
            t_ready.record(main)
        with torch.cuda.stream(s_pitch):
            pitch_hat = self.pitch_pred.forward_bt(x).unsqueeze(1)
            if pitch_fn is not None:
                pitch_hat = pitch_fn(pitch_hat)
        with torch.cuda.stream(s_energy):
            energy_hat = self.energy_pred.forward_bt(x).unsqueeze(1)
            if energy_fn is not None:
                energy_hat = energy_fn(energy_hat)
        if pitch_fn is not None and energy_fn is not None:
            with torch.cuda.stream(s_prenet):
                for s, t in ((s_pitch, pitch_hat), (s_energy, energy_hat)):
                    s_prenet.wait_stream(s)
                    if not capture:
                        t.record_stream(s_prenet)
                wp, bp, we, be = self._folded_series_weights()
                ops.series_proj_add(xp, pitch_hat, wp, bp, self.pitch_strength, energy_hat, we,
                                    be, self.energy_strength)
        if batch is not None:  # a shard of a larger batch (sharded.GlobalBatch): batch-global
            offsets, totals = batch.duration_counts(dur_hat)  # fill rule / T_mel
            T_mel = batch.t_mel(totals)
        index = None
        if not capture:
            if t_ready is not None:
                t_ready.synchronize()
                T_mel = int(t_host)
            # the LR index map only needs the durations: queued before the caller's stream
            # joins the side streams, so it is not held behind the prenet chain's tail
            index = ops.lr_index(offsets, T_mel)
        for s, ts in ((s_pitch, (pitch_hat,)), (s_energy, (energy_hat,)),
                      (s_prenet, (enc, xp))):
            main.wait_stream(s)
            if not capture:
                for t in ts:
                    t.record_stream(main)
        if capture:
            return dur_hat, pitch_hat, energy_hat, enc, offsets, tmax, xp
        return dur_hat, pitch_hat, energy_hat, enc, (offsets, index), T_mel, xp

    def generate(self,
                 x: torch.Tensor,
                 alpha=1.0,
                 pitch_function: Callable[[torch.Tensor], torch.Tensor] = _identity,
                 energy_function: Callable[[torch.Tensor], torch.Tensor] = _identity,
                 batch=None) -> Dict[str, torch.Tensor]:
        """`models/forward_tacotron.py:244-268`.  The callbacks run on the stream of their
        predictor (torch ops issued inside them are ordered after the prediction).
        `batch`: a sharded.GlobalBatch when x is one rank's shard of a larger batch.
        Runs under the f16x3 range guard (ops.run_checked): one status read at the end."""
        if self.training:  # the module-tree walk of eval() is host time on every call
            self.eval()
        self._check_device(x)

        # only callbacks known to be pure are captured (graph_safe): a replay would freeze any
        # Python-side state an arbitrary callback reads; any other callback runs eagerly
        # between the captured predictors and the launch that consumes its output
        graph = GRAPH and batch is None and x.numel() <= GRAPH_MAX_TOKENS

        def run():
            with torch.no_grad():
                phase = ent = None
                if graph and not ops.forced_exact():
                    r = self._phoneme_graph(x, alpha, pitch_function, energy_function)
                    if r is not None:
                        phase, ent = r
                if phase is None:
                    phase = self._phoneme_phase(x, alpha, pitch_function, energy_function, batch)
                dur_hat, pitch_hat, energy_hat, enc, offsets, T_mel, xp = phase
                out = self._generate_mel(x, dur_hat, pitch_hat, energy_hat, enc=enc,
                                         lr=(offsets, T_mel), xp=xp)
                if ent is not None:  # the decoder has consumed the graph's static buffers
                    ent['done'].record(torch.cuda.current_stream(x.device))
                return out
        return ops.run_checked(run, x.device, reduce=None if batch is None else batch.status)

    def __prepare_scriptable__(self):
        """`torch.jit.script(model)` (the reference's export, README.md:149-161): the compute
        runs in libftmi.so through ctypes, which TorchScript cannot compile, so what gets
        scripted is `jit.ScriptedForwardTacotron` — the reference's scriptable surface
        (`forward(batch)`, `generate_jit(x, alpha, beta)`) over dispatcher operators
        (`torch.ops.ftmi.*`) that run this model's HIP path.  The scripted module carries the
        constructor keywords and the weights, so a torch.jit.save'd archive loads and runs
        in any process that has imported forwardtacotron_amd."""
        from .jit import ScriptedForwardTacotron
        return ScriptedForwardTacotron(self)

    def generate_jit(self, x: torch.Tensor, alpha: float = 1.0, beta: float = 1.0) -> Dict[str, torch.Tensor]:
        """`models/forward_tacotron.py:270-284` (pitch scaled by beta, no callbacks)."""
        self._check_device(x)

        def run():
            with torch.no_grad():
                dur_hat, pitch_hat, energy_hat, enc, offsets, T_mel, xp = self._phoneme_phase(
                    x, alpha, lambda p: p * beta, lambda e: e)
                return self._generate_mel(x, dur_hat, pitch_hat, energy_hat, enc=enc,
                                          lr=(offsets, T_mel), xp=xp)
        return ops.run_checked(run, x.device)

    def get_step(self) -> int:
        return self.step.data.item()

    def _generate_mel(self, x, dur_hat, pitch_hat, energy_hat, enc=None, lr=None, xp=None):
        """`models/forward_tacotron.py:289-330`.  enc: the prenet output if already computed;
        lr: (offsets, T_mel) if the LengthRegulator counts were already computed (then
        dur_hat has already been clipped / filled in place); xp: the LSTM input projection
        with the pitch / energy terms if already queued (then enc is not read)."""
        if enc is None:
            enc = self.prenet.forward_cl(ops.embedding(x, self.embedding.weight.detach()))
        if xp is None:
            wp, bp, we, be = self._series_proj_weights()
            ops.series_proj_add(enc, pitch_hat, wp, bp, self.pitch_strength, energy_hat, we, be,
                                self.energy_strength)
        index = None
        if lr is None:
            offsets, totals, _ = ops.duration_counts(dur_hat, apply_fill=False)
            T_mel = int(totals.max().item())  # the one host sync: output size is data dependent
        else:
            offsets, T_mel = lr
            if isinstance(offsets, tuple):  # (offsets, index map already queued)
                offsets, index = offsets
        if index is None:
            index = ops.lr_index(offsets, T_mel)
        mel, mel_post = self._decode(enc, index, xp=xp)
        return {'mel': mel, 'mel_post': mel_post, 'dur': dur_hat,
                'pitch': pitch_hat, 'energy': energy_hat}

    def _pad(self, x: torch.Tensor, max_len: int) -> torch.Tensor:
        """`models/forward_tacotron.py:332-335` (crop / pad the time axis with padding_value)."""
        x = x[:, :, :max_len]
        if x.size(2) < max_len:
            pad = torch.full((x.size(0), x.size(1), max_len - x.size(2)), self.padding_value,
                             device=x.device, dtype=x.dtype)
            x = torch.cat([x, pad], 2)
        return x

    @classmethod
    def from_config(cls, config: Dict[str, Any]) -> 'ForwardTacotron':
        model_config = config['forward_tacotron']['model']
        model_config['num_chars'] = len(phonemes)
        model_config['n_mels'] = config['dsp']['num_mels']
        return ForwardTacotron(**model_config)

    @classmethod
    def from_checkpoint(cls, path: Union[Path, str]) -> 'ForwardTacotron':
        checkpoint = torch.load(path, map_location=torch.device('cpu'), weights_only=True)
        model = ForwardTacotron.from_config(checkpoint['config'])
        model.load_state_dict(checkpoint['model'])
        return model
