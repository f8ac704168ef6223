"""Layers of the reference (`models/common_layers.py`, `models/forward_tacotron.py:14-71`)
re-built on libftmi.so.

Every module declares exactly the parameters / buffers of its reference counterpart, under
the same names, so ``state_dict()`` keys and shapes are identical and reference checkpoints
load with ``load_state_dict`` unchanged.  The modules hold no torch compute layers: the
math runs in HIP kernels through :mod:`forwardtacotron_amd.ops`.

Internally activations are channels-last (B, T, C) (``*_cl`` methods).  The public
``forward`` methods keep the reference's argument layout and return values so they can be
used (and tested) one layer at a time.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn

from . import ops

# --------------------------------------------------------------------------------------
# parameter holders (same tensors as nn.Conv1d / nn.BatchNorm1d / nn.Linear / nn.GRU / nn.LSTM)


def _uniform_(t: torch.Tensor, bound: float) -> None:
    with torch.no_grad():
        t.uniform_(-bound, bound)


class Conv1dParams(nn.Module):
    """Parameters of nn.Conv1d(cin, cout, k, bias=...)."""

    def __init__(self, cin: int, cout: int, k: int, bias: bool) -> None:
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = cin, cout, k
        self.weight = nn.Parameter(torch.empty(cout, cin, k))
        self.bias = nn.Parameter(torch.empty(cout)) if bias else None
        b = 1.0 / math.sqrt(cin * k)
        _uniform_(self.weight, b)
        if self.bias is not None:
            _uniform_(self.bias, b)


class BatchNorm1dParams(nn.Module):
    """Parameters and running statistics of nn.BatchNorm1d(c) (eval mode only)."""

    def __init__(self, c: int, eps: float = 1e-5) -> None:
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer('running_mean', torch.zeros(c))
        self.register_buffer('running_var', torch.ones(c))
        self.register_buffer('num_batches_tracked', torch.tensor(0, dtype=torch.long))

    def folded(self):
        """(scale, shift) with y = x*scale + shift == (x - mean)/sqrt(var + eps)*w + b."""
        invstd = 1.0 / torch.sqrt(self.running_var + self.eps)
        scale = invstd * self.weight
        shift = self.bias - self.running_mean * scale
        return scale.detach().float().contiguous(), shift.detach().float().contiguous()


class LinearParams(nn.Module):
    """Parameters of nn.Linear(fin, fout, bias=...)."""

    def __init__(self, fin: int, fout: int, bias: bool = True) -> None:
        super().__init__()
        self.in_features, self.out_features = fin, fout
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.empty(fout)) if bias else None
        b = 1.0 / math.sqrt(fin)
        _uniform_(self.weight, b)
        if self.bias is not None:
            _uniform_(self.bias, b)

    def packed_weights(self):
        """(weight, bias or None, pre-split weight) for ops.conv1d, cached on the parameter
        identity / version like Packed."""
        key = tuple((t.data_ptr(), t._version, t.device) for t in self.parameters())
        cache = self.__dict__.get('_ftmi_pack')
        if cache is None or cache[0] != key:
            with torch.no_grad():
                w = self.weight.detach().contiguous()
                b = None if self.bias is None else self.bias.detach().contiguous()
                cache = (key, (w, b, presplit(w)))
            self.__dict__['_ftmi_pack'] = cache
        return cache[1]


def pack_conv(w: torch.Tensor) -> torch.Tensor:
    """nn.Conv1d weight (N, Cin, k) -> kernel layout [N][k*Cin] (tap-major K)."""
    return w.detach().permute(0, 2, 1).contiguous().reshape(w.size(0), -1)


def presplit(w: torch.Tensor):
    """Pre-split operand of a packed weight for the default matrix path (ops.MMA): f16
    planes (f16x3), bf16 pieces (bf16x6) or None (fp32)."""
    return ops.presplit_for(w)


# --------------------------------------------------------------------------------------
# packed-weight cache: rebuilt whenever a parameter / buffer changes (load_state_dict, .to)

class Packed(nn.Module):
    """Base class: caches kernel-layout weights, keyed by the identity/version of params."""

    def _pack_key(self):
        # The (owner dict, name, tensor) list is cached: walking the module tree costs ~10 us
        # per call, which is host time on the launch path.  A parameter / buffer REPLACED in
        # any submodule (owner dict no longer holds the same object) rebuilds the list; an
        # in-place change (load_state_dict, .to, .copy_) changes data_ptr or _version.
        refs = self.__dict__.get('_ftmi_refs')
        if refs is None or any(d.get(n) is not t for d, n, t in refs):
            refs = [(d, n, t) for m in self.modules() for d in (m._parameters, m._buffers)
                    for n, t in d.items() if t is not None]
            self.__dict__['_ftmi_refs'] = refs
        return tuple((t.data_ptr(), t._version) for _, _, t in refs)

    def packed_weights(self):
        key = self._pack_key()
        cache = self.__dict__.get('_ftmi_pack')
        if cache is None or cache[0] != key:
            with torch.no_grad():
                cache = (key, self._pack())
            self.__dict__['_ftmi_pack'] = cache
        return cache[1]

    def _pack(self):  # pragma: no cover - abstract
        raise NotImplementedError


# --------------------------------------------------------------------------------------
# reference layers

class LengthRegulator(nn.Module):
    """`models/common_layers.py:7-19`: dur[dur<0]=0 (in place), repeat each frame
    int64(dur+0.5) times, zero-pad to the longest sequence."""

    def forward(self, x: torch.Tensor, dur: torch.Tensor) -> torch.Tensor:
        dur_c = dur if (dur.is_contiguous() and dur.dtype == torch.float32) else dur.float().contiguous()
        offsets, totals, _ = ops.duration_counts(dur_c, apply_fill=False)
        if dur_c is not dur:
            dur.copy_(dur_c)
        T_mel = int(totals.max().item()) if totals.numel() else 0
        index = ops.lr_index(offsets, T_mel)
        return ops.length_regulate(x.contiguous(), index)


class BatchNormConv(Packed):
    """Conv1d_s1 (pad k//2, no bias) -> (ReLU) -> BatchNorm1d(eval).
    `models/forward_tacotron.py:58-71` and `models/common_layers.py:38-52`."""

    def __init__(self, in_channels: int, out_channels: int, kernel: int, relu: bool = True) -> None:
        super().__init__()
        self.conv = Conv1dParams(in_channels, out_channels, kernel, bias=False)
        self.bnorm = BatchNorm1dParams(out_channels)
        self.relu = relu
        self.kernel = kernel

    def _pack(self):
        w = pack_conv(self.conv.weight)
        return w, self.bnorm.folded(), presplit(w)

    def forward_cl(self, x: torch.Tensor, T_out: int = 0, residual=None, maxpool=False,
                   x_split=False) -> torch.Tensor:
        w, bn, w3 = self.packed_weights()
        # bf16x6: the pre-split kernel measured slower on the maxpool (CBHG proj1) shapes
        y, _ = ops.conv1d(x, w, self.kernel, self.kernel // 2, relu=self.relu, bn=bn,
                          residual=residual, maxpool=maxpool, T_out=T_out,
                          w_split=None if (maxpool and ops.MMA == 1) else w3, x_split=x_split)
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, Cin, T) -> (B, Cout, T + 1 - k % 2), like the reference."""
        T = x.size(2)
        To = T + 2 * (self.kernel // 2) - self.kernel + 1
        y = self.forward_cl(x.transpose(1, 2).contiguous(), T_out=To)
        return y.transpose(1, 2)


class HighwayNetwork(Packed):
    """`models/common_layers.py:22-35`: y = g*relu(W1 x + b1) + (1-g)*x, g = sigmoid(W2 x + b2)."""

    def __init__(self, size: int) -> None:
        super().__init__()
        self.W1 = LinearParams(size, size)
        self.W2 = LinearParams(size, size)
        with torch.no_grad():
            self.W1.bias.zero_()

    def _pack(self):
        C = self.W1.weight.size(0)
        w1 = self.W1.weight.detach().reshape(C // 32, 32, C)
        w2 = self.W2.weight.detach().reshape(C // 32, 32, C)
        w12 = torch.stack([w1, w2], 1).reshape(2 * C, C).contiguous()
        return (w12, self.W1.bias.detach().contiguous(), self.W2.bias.detach().contiguous(),
                presplit(w12))

    def forward_cl(self, x: torch.Tensor, out=None) -> torch.Tensor:
        w12, b1, b2, w3 = self.packed_weights()
        return ops.highway(x, w12, b1, b2, out=out, w_split=w3)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        y = self.forward_cl(x.reshape(1, -1, shp[-1]).contiguous())
        return y.reshape(shp)


class BiRNN(Packed):
    """1-layer bidirectional GRU (gates r,z,n) / LSTM (gates i,f,g,o), batch_first, holding
    exactly the parameters of nn.GRU / nn.LSTM (weight_ih_l0, weight_hh_l0, bias_ih_l0,
    bias_hh_l0 and their _reverse twins)."""

    def __init__(self, fin: int, hidden: int, cell: str) -> None:
        super().__init__()
        self.cell = 0 if cell == 'gru' else 1
        self.input_size, self.hidden = fin, hidden
        # the recurrence runs alone and may spread over every CU (ops.rnn_bidir `spread`);
        # set by the owner for the decoder-side recurrences only
        self.spread = False
        gh = (3 if self.cell == 0 else 4) * hidden
        b = 1.0 / math.sqrt(hidden)
        for sfx in ('', '_reverse'):
            for name, shape in (('weight_ih_l0', (gh, fin)), ('weight_hh_l0', (gh, hidden)),
                                ('bias_ih_l0', (gh,)), ('bias_hh_l0', (gh,))):
                prm = nn.Parameter(torch.empty(*shape))
                _uniform_(prm, b)
                self.register_parameter(name + sfx, prm)

    def _pack(self):
        """W_ih both directions [2*G*H][In], input bias [2*G*H], b_hh [2*G*H], W_hh [2][G*H][H]."""
        w_ih = torch.cat([self.weight_ih_l0, self.weight_ih_l0_reverse], 0).detach().contiguous()
        b_ih = torch.cat([self.bias_ih_l0, self.bias_ih_l0_reverse], 0).detach().contiguous()
        b_hh = torch.cat([self.bias_hh_l0, self.bias_hh_l0_reverse], 0).detach().contiguous()
        w_hh = torch.stack([self.weight_hh_l0, self.weight_hh_l0_reverse], 0).detach().contiguous()
        if self.cell == 1:  # LSTM: both biases folded into the input projection
            return w_ih, (b_ih + b_hh).contiguous(), None, w_hh, presplit(w_ih)
        return w_ih, b_ih, b_hh, w_hh, presplit(w_ih)

    def forward_cl(self, x: torch.Tensor, T: Optional[int] = None, index=None, lengths=None,
                   pad_value: float = 0.0) -> torch.Tensor:
        """x: (B, T_src, In) channels-last; with index, frame t reads row index[b, t]."""
        return self.recur(self.project(x), T=T, index=index, lengths=lengths,
                          pad_value=pad_value)

    def project(self, x: torch.Tensor) -> torch.Tensor:
        """Input projections of both directions, x W_ih^T + b: (B, T_src, 2*G*H)."""
        w_ih, b_in, _, _, w3 = self.packed_weights()
        xp, _ = ops.conv1d(x, w_ih, 1, 0, bias=b_in, w_split=w3)
        return xp

    def recur(self, xp: torch.Tensor, T: Optional[int] = None, index=None, lengths=None,
              pad_value: float = 0.0) -> torch.Tensor:
        """The recurrence over `project`'s output (frame t reads row index[b, t])."""
        _, b_in, b_hh, w_hh, _ = self.packed_weights()
        return ops.rnn_bidir(self.cell, xp, self.hidden, w_hh, b_hh, T=T, index=index,
                             xp_zero=b_in if index is not None else None, lengths=lengths,
                             pad_value=pad_value, spread=self.spread)

    def forward(self, x: torch.Tensor):
        """(B, T, In) -> ((B, T, 2H), None) like nn.GRU/LSTM(batch_first=True) without h0."""
        return self.forward_cl(x.contiguous()), None


class CBHG(Packed):
    """`models/common_layers.py:55-119`: conv bank (k = 1..K) -> maxpool -> proj1 -> proj2
    + residual -> pre_highway -> highways -> bidirectional GRU."""

    def __init__(self, K: int, in_channels: int, channels: int, proj_channels: List[int],
                 num_highways: int, dropout: float = 0.5) -> None:
        super().__init__()
        self.dropout = dropout
        self.K = K
        self.channels = channels
        self.bank_kernels = list(range(1, K + 1))
        self.conv1d_bank = nn.ModuleList(
            [BatchNormConv(in_channels, channels, k) for k in self.bank_kernels])
        self.conv_project1 = BatchNormConv(K * channels, proj_channels[0], 3)
        self.conv_project2 = BatchNormConv(proj_channels[0], proj_channels[1], 3, relu=False)
        self.pre_highway = LinearParams(proj_channels[-1], channels, bias=False)
        self.highways = nn.ModuleList([HighwayNetwork(channels) for _ in range(num_highways)])
        self.rnn = GRUParamsModule(channels, channels)

    def _pack(self):
        ws = [pack_conv(c.conv.weight) for c in self.conv1d_bank]
        bank_w = torch.cat([w.reshape(-1) for w in ws]).contiguous()
        folds = [c.bnorm.folded() for c in self.conv1d_bank]
        scale = torch.cat([f[0] for f in folds]).contiguous()
        shift = torch.cat([f[1] for f in folds]).contiguous()
        w_pre = self.pre_highway.weight.detach().contiguous()
        bank3 = ops.split_bank_weights(bank_w, self.K, ws[0].size(1), self.channels)
        img = ops.bank_halves_image(bank3, self.K, ws[0].size(1), self.channels)
        return bank_w, scale, shift, w_pre, bank3, presplit(w_pre), img

    def forward_cl(self, x: torch.Tensor) -> torch.Tensor:
        """(B, T, Cin) channels-last -> (B, T, 2*channels)."""
        bank_w, scale, shift, w_pre, bank3, pre3, img = self.packed_weights()
        pooled = ops.bank_pools(x, self.K, self.channels, w_split=bank3)
        # pooled: the bank kernel applied the maxpool, and (split) stored its output as the
        # f16x3 split rows proj1 multiplies
        split = pooled and ops.SPLIT_ROWS
        xin = pooled and ops.SPLIT_BANK_IN  # x stays fp32 too: it is the proj2 residual
        bank = ops.conv_bank(ops.split_rows(x) if xin else x, bank_w, self.K, self.channels,
                             scale, shift, w_split=bank3, pool=pooled, split_out=split,
                             x_split=xin, w_image=img)
        y = self.conv_project1.forward_cl(bank, maxpool=not pooled, x_split=split)
        del bank
        y = self.conv_project2.forward_cl(y, residual=x)
        xp = self._highway_stack(y)
        if xp is not None:
            return self.rnn.recur(xp)
        h, _ = ops.conv1d(y, w_pre, 1, 0, w_split=pre3)
        h2 = torch.empty_like(h)
        for hw in self.highways:
            hw.forward_cl(h, out=h2)
            h, h2 = h2, h
        return self.rnn.forward_cl(h)

    def _stack_pack(self):
        """Fragment-major f16x3 blocks of pre_highway, the highways' w12 and the GRU's W_ih
        (the operands of ops.highway_stack), cached like every pack (rebuilt with the params)."""
        key = self._pack_key()
        cache = self.__dict__.get('_ftmi_stack')
        if cache is None or cache[0] != key:
            with torch.no_grad():
                w_pre = self.packed_weights()[3]
                hw = [m.packed_weights() for m in self.highways]
                w_ih, b_in = self.rnn.packed_weights()[:2]
                f16 = ops.split_weights_f16
                cache = (key, (f16(w_pre, frag=True), [f16(p[0], frag=True) for p in hw],
                               [p[1] for p in hw], [p[2] for p in hw], f16(w_ih, frag=True),
                               b_in, w_ih.size(0)))
            self.__dict__['_ftmi_stack'] = cache
        return cache[1]

    def spread_blocks(self, M: int) -> int:
        """Workgroups the spread CBHG tail would hold resident for M rows (0: the fused
        stack does not apply or runs the one-workgroup-per-64-rows kernel)."""
        Cp = self.channels  # the tail's input: proj2's output (common_layers.py:104-109)
        if not ops.highway_stack_ok(M, Cp, self.channels, len(self.highways), 6 * self.channels,
                                    (self.packed_weights()[5],)):
            return 0
        return ops.hs_spread_blocks(M, 6 * self.channels)

    def _highway_stack(self, y: torch.Tensor) -> Optional[torch.Tensor]:
        """pre_highway -> highways -> the GRU's input projection in one launch (the GRU input
        rows, or None where ops.highway_stack does not apply).  `allow_spread` (set per call
        by the model's co-residency check) = False keeps the stack kernel."""
        M, Cp = y.size(0) * y.size(1), y.size(2)
        n_out = 6 * self.channels
        if not ops.highway_stack_ok(M, Cp, self.channels, len(self.highways), n_out,
                                    (self.packed_weights()[5],)):
            return None
        pre_f, hw_f, b1s, b2s, ih_f, b_in, n_out = self._stack_pack()
        xp, _ = ops.highway_stack(y, pre_f, self.channels, hw_f, b1s, b2s, ih_f, b_in, n_out,
                                  spread=getattr(self, 'allow_spread', True))
        return xp

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, Cin, T) -> (B, T, 2*channels), like the reference."""
        return self.forward_cl(x.transpose(1, 2).contiguous())


class GRUParamsModule(BiRNN):
    """nn.GRU(fin, hidden, batch_first=True, bidirectional=True) parameters + HIP forward."""

    def __init__(self, fin: int, hidden: int) -> None:
        super().__init__(fin, hidden, 'gru')


class LSTMParamsModule(BiRNN):
    """nn.LSTM(fin, hidden, batch_first=True, bidirectional=True) parameters + HIP forward."""

    def __init__(self, fin: int, hidden: int) -> None:
        super().__init__(fin, hidden, 'lstm')
