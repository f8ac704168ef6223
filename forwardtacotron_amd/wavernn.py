"""WaveRNN vocoder of the reference (`models/fatchord_version.py`, the `gen_forward.py
wavernn` option) on libftmi.so.

Same constructor keywords, parameter / buffer names and shapes (`state_dict` keys equal the
reference's: tests/golden/wavernn_state_dict_keys.json), `from_config`, `from_checkpoint`,
`generate(mels, batched, target, overlap, mu_law, silent)` returning the float64 numpy wave,
teacher-forced `forward(x, mels)`, `fold_with_overlap`, `xfade_and_unfold`, `pad_tensor`,
`get_step`, `num_params`.  No torch compute layers: the upsampling network runs on the
GEMM kernels (BatchNorm folded into the 1x1 / k5 convolutions) and `ftmi_wr_stretch_conv`,
the sample loop on ONE persistent launch (`ftmi_wavernn`, csrc/wavernn.hip), the
crossfade / mu-law tail on `ftmi_wr_unfold`.

Randomness: the reference draws with torch's global generator (Categorical / uniform_);
here every draw comes from a counter-based Philox4x32-10 stream whose key is taken from
torch's CPU generator at each call (`torch.manual_seed` makes a run reproducible), or from
`seed=`.  Same distributions; the sample sequence is reproducible on any device
(oracle/wr_torch_cpu.py PhiloxSampler restates it).
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Any, Dict, Optional, Union

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from .common_layers import BatchNorm1dParams, Conv1dParams, LinearParams, Packed, presplit

_f32 = torch.float32


class ResBlock(nn.Module):
    """fatchord_version.py:14-29 (parameters)."""

    def __init__(self, dims: int) -> None:
        super().__init__()
        self.conv1 = Conv1dParams(dims, dims, 1, bias=False)
        self.conv2 = Conv1dParams(dims, dims, 1, bias=False)
        self.batch_norm1 = BatchNorm1dParams(dims)
        self.batch_norm2 = BatchNorm1dParams(dims)


class MelResNet(nn.Module):
    """fatchord_version.py:32-49 (parameters)."""

    def __init__(self, res_blocks: int, in_dims: int, compute_dims: int, res_out_dims: int,
                 pad: int) -> None:
        super().__init__()
        self.conv_in = Conv1dParams(in_dims, compute_dims, pad * 2 + 1, bias=False)
        self.batch_norm = BatchNorm1dParams(compute_dims)
        self.layers = nn.ModuleList([ResBlock(compute_dims) for _ in range(res_blocks)])
        self.conv_out = Conv1dParams(compute_dims, res_out_dims, 1, bias=True)


class Stretch2d(nn.Module):
    """fatchord_version.py:52-62: nearest-neighbour repeat along time (no parameters; the
    repeat is applied inside the kernels that read it)."""

    def __init__(self, x_scale: int, y_scale: int) -> None:
        super().__init__()
        self.x_scale, self.y_scale = x_scale, y_scale


class SmoothConv(nn.Module):
    """nn.Conv2d(1, 1, (1, 2 s + 1), padding (0, s), bias=False), weight filled with 1/k
    like the reference (:78-79)."""

    def __init__(self, scale: int) -> None:
        super().__init__()
        k = 2 * scale + 1
        self.scale = scale
        self.weight = nn.Parameter(torch.full((1, 1, 1, k), 1.0 / k))


class UpsampleNetwork(nn.Module):
    """fatchord_version.py:65-90 (parameters; compute in WaveRNN._upsample)."""

    def __init__(self, feat_dims, upsample_scales, compute_dims, res_blocks, res_out_dims, pad):
        super().__init__()
        total_scale = int(np.cumprod(upsample_scales)[-1])
        self.scales = list(upsample_scales)
        self.indent = pad * total_scale
        self.resnet = MelResNet(res_blocks, feat_dims, compute_dims, res_out_dims, pad)
        self.resnet_stretch = Stretch2d(total_scale, 1)
        self.up_layers = nn.ModuleList()
        for scale in upsample_scales:
            self.up_layers.append(Stretch2d(scale, 1))
            self.up_layers.append(SmoothConv(scale))


class GRUParams(nn.Module):
    """nn.GRU(fin, hidden, batch_first=True) parameters (one direction)."""

    def __init__(self, fin: int, hidden: int) -> None:
        super().__init__()
        self.input_size, self.hidden_size = fin, hidden
        b = 1.0 / math.sqrt(hidden)
        for name, shape in (('weight_ih_l0', (3 * hidden, fin)), ('weight_hh_l0', (3 * hidden, hidden)),
                            ('bias_ih_l0', (3 * hidden,)), ('bias_hh_l0', (3 * hidden,))):
            prm = nn.Parameter(torch.empty(*shape))
            with torch.no_grad():
                prm.uniform_(-b, b)
            self.register_parameter(name, prm)


def _fold_bn(conv_w: torch.Tensor, bn: BatchNorm1dParams):
    """conv (no bias) followed by eval BatchNorm as one conv: W' = scale W (float64
    product), bias' = shift.  Packed [N][k*Cin] like ops.conv1d takes it."""
    scale, shift = bn.folded()
    w = (conv_w.detach().double() * scale.double()[:, None, None]).float()
    return w.permute(0, 2, 1).contiguous().reshape(w.size(0), -1), shift


class WaveRNN(Packed):
    """fatchord_version.py:93-453."""

    def __init__(self, rnn_dims, fc_dims, bits, pad, upsample_factors, feat_dims, compute_dims,
                 res_out_dims, res_blocks, hop_length, sample_rate, mode='RAW'):
        super().__init__()
        self.mode = mode
        self.pad = pad
        if self.mode == 'RAW':
            self.n_classes = 2 ** bits
        elif self.mode == 'MOL':
            self.n_classes = 30
        else:
            raise RuntimeError('Unknown model mode value - ', self.mode)
        self.rnn_dims = rnn_dims
        self.aux_dims = res_out_dims // 4
        self.hop_length = hop_length
        self.sample_rate = sample_rate
        self.upsample = UpsampleNetwork(feat_dims, upsample_factors, compute_dims, res_blocks,
                                        res_out_dims, pad)
        self.I = LinearParams(feat_dims + self.aux_dims + 1, rnn_dims)
        self.rnn1 = GRUParams(rnn_dims, rnn_dims)
        self.rnn2 = GRUParams(rnn_dims + self.aux_dims, rnn_dims)
        self.fc1 = LinearParams(rnn_dims + self.aux_dims, fc_dims)
        self.fc2 = LinearParams(fc_dims + self.aux_dims, fc_dims)
        self.fc3 = LinearParams(fc_dims, self.n_classes)
        self.register_buffer('step', torch.zeros(1, dtype=torch.long))
        self.feat_dims, self.fc_dims = feat_dims, fc_dims
        self.num_params()

    # ---- packing (once per weights version) -----------------------------------------------
    def _pack(self):
        up = self.upsample
        rn = up.resnet
        conv_in = _fold_bn(rn.conv_in.weight, rn.batch_norm)
        blocks = [(_fold_bn(l.conv1.weight, l.batch_norm1), _fold_bn(l.conv2.weight, l.batch_norm2))
                  for l in rn.layers]
        w_out = rn.conv_out.weight.detach().permute(0, 2, 1).contiguous().reshape(rn.conv_out.weight.size(0), -1)
        resnet = ((conv_in[0], conv_in[1], presplit(conv_in[0])),
                  [((a[0], a[1], presplit(a[0])), (b[0], b[1], presplit(b[0]))) for a, b in blocks],
                  (w_out, rn.conv_out.bias.detach().float().contiguous(), presplit(w_out)))
        smooth = [m.weight.detach().float().reshape(-1).contiguous() for m in up.up_layers[1::2]]

        d = lambda t: t.detach().double()
        R, F, A, NM = self.rnn_dims, self.fc_dims, self.aux_dims, self.feat_dims
        WI, bI = d(self.I.weight), d(self.I.bias)
        w0, WIm, WIa = WI[:, 0], WI[:, 1:1 + NM], WI[:, 1 + NM:]
        Wih1, bih1 = d(self.rnn1.weight_ih_l0), d(self.rnn1.bias_ih_l0)
        Wih2, bih2 = d(self.rnn2.weight_ih_l0), d(self.rnn2.bias_ih_l0)
        Wih2a, Wih2b = Wih2[:, :R], Wih2[:, R:]
        Wf1, bf1 = d(self.fc1.weight), d(self.fc1.bias)
        Wf1a, Wf1b = Wf1[:, :R], Wf1[:, R:]
        Wf2, bf2 = d(self.fc2.weight), d(self.fc2.bias)
        Wf2a, Wf2b = Wf2[:, :F], Wf2[:, F:]
        dev = WI.device
        waux = torch.zeros(6 * R + 2 * F, 4 * A, dtype=torch.float64, device=dev)
        waux[:3 * R, :A] = Wih1 @ WIa
        waux[3 * R:6 * R, :A] = Wih2a @ WIa
        waux[3 * R:6 * R, A:2 * A] = Wih2b
        waux[6 * R:6 * R + F, :A] = Wf1a @ WIa
        waux[6 * R:6 * R + F, 2 * A:3 * A] = Wf1b
        waux[6 * R + F:, 3 * A:] = Wf2b
        bias = torch.cat([Wih1 @ bI + bih1, Wih2a @ bI + bih2, Wf1a @ bI + bf1, bf2])
        wm = torch.cat([Wih1 @ WIm, Wih2a @ WIm, Wf1a @ WIm], 0)
        f = lambda t: t.float().contiguous()
        waux = f(waux)
        rec = dict(
            w_hh1=f(d(self.rnn1.weight_hh_l0)), w_hh2=f(d(self.rnn2.weight_hh_l0)), w_ih2a=f(Wih2a),
            w_fc1a=f(Wf1a), w_fc2a=f(Wf2a), w_fc3=f(d(self.fc3.weight)), b_fc3=f(d(self.fc3.bias)),
            b_hh1=f(d(self.rnn1.bias_hh_l0)), b_hh2=f(d(self.rnn2.bias_hh_l0)),
            u1=f(Wih1 @ w0), u2=f(Wih2a @ w0), v1=f(Wf1a @ w0), wm=f(wm))
        return resnet, smooth, (waux, f(bias), presplit(waux)), rec

    # ---- upsampling network -----------------------------------------------------------------
    def _upsample(self, m_rows: torch.Tensor):
        """UpsampleNetwork.forward (:83-90) on (B, T, feat) rows -> (mel rows (B, (T - 2 pad)
        hop, feat), aux frames (B, T - 2 pad, res_out)); the aux stretch is implicit
        (sample g reads frame g // hop)."""
        resnet, smooth, _, _ = self.packed_weights()
        (w_in, b_in, s_in), blocks, (w_out, b_out, s_out) = resnet
        k = 2 * self.pad + 1
        T = m_rows.size(1)
        x, _ = ops.conv1d(m_rows, w_in, k, 0, bias=b_in, relu=True, T_out=T - 2 * self.pad,
                          w_split=s_in)
        for (w1, b1, s1), (w2, b2, s2) in blocks:
            h, _ = ops.conv1d(x, w1, 1, 0, bias=b1, relu=True, w_split=s1)
            x, _ = ops.conv1d(h, w2, 1, 0, bias=b2, residual=x, w_split=s2)
        aux, _ = ops.conv1d(x, w_out, 1, 0, bias=b_out, w_split=s_out)
        y = m_rows
        scales = self.upsample.scales
        for i, (s, w) in enumerate(zip(scales, smooth)):
            if i + 1 < len(scales):
                y = ops.wr_stretch_conv(y, s, w)
            else:
                W_out = y.size(1) * s - 2 * self.upsample.indent
                y = ops.wr_stretch_conv(y, s, w, W_out=W_out, crop0=self.upsample.indent)
        return y, aux

    def upsample_forward(self, mels: torch.Tensor):
        """The reference's `self.upsample(mels)` (:145 / :188): (B, feat, T) -> (mels (B, L,
        feat), aux (B, L, res_out)) with the aux stretch materialised (for tests)."""
        m, aux = self._upsample(mels.transpose(1, 2).contiguous())
        hop = int(np.prod(self.upsample.scales))
        return m, aux.repeat_interleave(hop, dim=1)

    # ---- the sample loop ---------------------------------------------------------------------
    def _run(self, m_up, frames, *, batched, L, fold_stride, B, xin=None, seed=0, want_logits=False):
        _, _, (waux, bias, waux3), rec = self.packed_weights()
        dev = m_up.device
        n_items, fpi = frames.size(0), frames.size(1)
        rows = torch.cat([frames.reshape(-1, frames.size(2)),
                          torch.zeros(1, frames.size(2), device=dev, dtype=_f32)], 0)
        cond, _ = ops.conv1d(rows.unsqueeze(0), waux, 1, 0, bias=bias, w_split=waux3)
        a = _lib.WaveRNNArgs()
        for k, v in rec.items():
            setattr(a, k, v.data_ptr())
        m_up = m_up.contiguous()
        a.cond, a.mel = cond.data_ptr(), m_up.data_ptr()
        a.bias_row, a.item_rows, a.frames_per_item = n_items * fpi, m_up.size(1), fpi
        a.hop = int(np.prod(self.upsample.scales))
        a.fold_stride, a.batched = fold_stride, int(batched)
        a.B, a.L, a.n_classes, a.mol = B, L, self.n_classes, int(self.mode == 'MOL')
        a.rnn_dims, a.fc_dims, a.feat_dims, a.aux_dims = self.rnn_dims, self.fc_dims, self.feat_dims, self.aux_dims
        a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        ws = ops.wavernn_workspace(dev)
        a.workspace = ws.data_ptr()
        self.__dict__['_ftmi_last_ws'] = ws  # diag readers (tools/wr_stamps.py)
        out = None
        if xin is not None:
            xin = xin.to(device=dev, dtype=_f32).contiguous()
            a.xin = xin.data_ptr()
            out = torch.empty(B, L, self.n_classes, device=dev, dtype=_f32)
            a.logits = out.data_ptr()
        else:
            out = torch.empty(B, L, device=dev, dtype=_f32)
            a.samples = out.data_ptr()
        R, F = self.rnn_dims, self.fc_dims
        per_step = 2.0 * (3 * R * R * 3 + F * R + F * F + self.n_classes * F + (6 * R + F) * self.feat_dims)
        # cond / ws / xin / m_up are freed on return: the caching allocator hands their blocks
        # to later allocations of this stream only, which run after the kernel (stream order)
        ops.wavernn(a, B, L, per_step * B * L, dev)
        return out

    def forward(self, x: torch.Tensor, mels: torch.Tensor) -> torch.Tensor:
        """Teacher-forced WaveRNN.forward (:132-169): x (B, L) samples, mels (B, feat, T) ->
        logits (B, L, n_classes), L = (T - 2 pad) hop."""
        if self.training:
            self.step += 1
        dev = self.step.device
        mels = torch.as_tensor(mels, device=dev, dtype=_f32)
        x = torch.as_tensor(x, device=dev, dtype=_f32)

        def run():
            m_up, frames = self._upsample(mels.transpose(1, 2).contiguous())
            if x.size(1) != m_up.size(1):
                raise ValueError(f'x has {x.size(1)} samples, the mels give {m_up.size(1)}')
            return self._run(m_up, frames, batched=False, L=m_up.size(1), fold_stride=0,
                             B=x.size(0), xin=x)
        with torch.no_grad():
            return ops.run_checked(run, dev)

    def __prepare_scriptable__(self):
        """`torch.jit.script(model)` (README.md:149-161 exports the reference this way) is not
        possible here: the compute runs in libftmi.so through ctypes, which TorchScript
        cannot call.  Fail with the reason instead of a TorchScript frontend error; the
        scripted entry point's behaviour is available eagerly (`generate`)."""
        raise RuntimeError(f'{type(self).__name__} runs on libftmi.so (HIP kernels called through '
                           'ctypes) and cannot be compiled by torch.jit.script; call generate eagerly')

    def _fold_shape(self, total_len, n_items, batched, target, overlap):
        """(B, L) of the sample loop: fold_with_overlap's fold count (:320-331) or one row
        per utterance."""
        if not batched:
            return n_items, total_len
        if n_items != 1:
            raise ValueError('batched generation folds ONE utterance (:294-341)')
        num_folds = (total_len - overlap) // (target + overlap)
        if total_len - (num_folds * (overlap + target) + overlap) != 0:
            num_folds += 1
        return num_folds, target + 2 * overlap

    def generate_samples(self, mels, batched=True, target=11000, overlap=550,
                         seed: Optional[int] = None) -> torch.Tensor:
        """The sample matrix of generate (:183-244) on the device: (B, L) fp32 sample values
        of every fold (before mu-law decoding and unfolding)."""
        dev = self.step.device
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        with torch.no_grad():
            mels = torch.as_tensor(mels).to(device=dev, dtype=_f32)
            rows = self.pad_tensor(mels.transpose(1, 2), pad=self.pad, side='both')

            def run():
                m_up, frames = self._upsample(rows)
                B, L = self._fold_shape(m_up.size(1), m_up.size(0), batched, target, overlap)
                return self._run(m_up, frames, batched=batched, L=L, fold_stride=target + overlap,
                                 B=B, seed=seed)
            return ops.run_checked(run, dev)

    def generate(self, mels, batched, target, overlap, mu_law, silent=False,
                 seed: Optional[int] = None) -> np.ndarray:
        """WaveRNN.generate (:171-265): mels (B, feat, T) (tensor or array, any device) ->
        float64 numpy wave of (T - 1) hop samples.  seed: the Philox key of the draws
        (default: drawn from torch's CPU generator)."""
        self.eval()
        mu_law = mu_law if self.mode == 'RAW' else False
        hop = self.hop_length
        T = torch.as_tensor(mels).size(-1)
        wave_len = (T - 1) * hop
        if wave_len < 20 * hop:
            raise ValueError(f'{T} mel frames: the 20-hop fade-out of the reference (:259-261) '
                             f'needs at least 21')
        smp = self.generate_samples(mels, batched, target, overlap, seed)
        with torch.no_grad():
            wav = ops.wr_unfold(smp, target, overlap, batched, mu_law, self.n_classes, wave_len,
                                20 * hop)
            out = wav.cpu().numpy()
        self.train()
        return out

    # ---- the reference's helpers ------------------------------------------------------------
    def pad_tensor(self, x, pad, side='both'):
        """:282-292 (any device)."""
        b, t, c = x.size()
        total = t + 2 * pad if side == 'both' else t + pad
        padded = torch.zeros(b, total, c, device=x.device, dtype=x.dtype)
        if side == 'before' or side == 'both':
            padded[:, pad:pad + t, :] = x
        elif side == 'after':
            padded[:, :t, :] = x
        return padded

    def fold_with_overlap(self, x, target, overlap):
        """:294-341 (data movement; generate folds implicitly inside the kernel)."""
        _, total_len, features = x.size()
        num_folds = (total_len - overlap) // (target + overlap)
        extended_len = num_folds * (overlap + target) + overlap
        remaining = total_len - extended_len
        if remaining != 0:
            num_folds += 1
            x = self.pad_tensor(x, target + 2 * overlap - remaining, side='after')
        folded = torch.zeros(num_folds, target + 2 * overlap, features, device=x.device, dtype=x.dtype)
        for i in range(num_folds):
            start = i * (target + overlap)
            folded[i] = x[:, start:start + target + 2 * overlap, :]
        return folded

    def xfade_and_unfold(self, y, target, overlap):
        """:343-406 on a (num_folds, target + 2 overlap) array of samples (float32 values, as
        generate produces them), through ftmi_wr_unfold: float64 result, no fade-out."""
        y = np.asarray(y)
        num_folds, length = y.shape
        total_len = num_folds * (length - overlap) + overlap
        t = torch.as_tensor(y, dtype=_f32, device=self.step.device)
        return ops.wr_unfold(t, length - 2 * overlap, overlap, True, False, self.n_classes,
                             total_len, 0).cpu().numpy()

    def get_step(self):
        return self.step.data.item()

    def num_params(self, print_out=False):
        parameters = sum(int(np.prod(p.size())) for p in self.parameters() if p.requires_grad) / 1_000_000
        if print_out:
            print('Trainable Parameters: %.3fM' % parameters)
        return parameters

    def load(self, path: Union[str, Path]):
        device = self.step.device
        self.load_state_dict(torch.load(path, map_location=device, weights_only=True), strict=False)

    def save(self, path: Union[str, Path]):
        torch.save(self.state_dict(), path)

    @classmethod
    def from_config(cls, config: Dict[str, Any]) -> 'WaveRNN':
        model_config = dict(config['vocoder']['model'])
        model_config['bits'] = config['dsp']['bits']
        model_config['feat_dims'] = config['dsp']['num_mels']
        model_config['hop_length'] = config['dsp']['hop_length']
        model_config['sample_rate'] = config['dsp']['sample_rate']
        return WaveRNN(**model_config)

    @classmethod
    def from_checkpoint(cls, path: Union[Path, str]) -> 'WaveRNN':
        checkpoint = torch.load(path, map_location=torch.device('cpu'), weights_only=True)
        model = WaveRNN.from_config(checkpoint['config'])
        model.load_state_dict(checkpoint['model'])
        return model
