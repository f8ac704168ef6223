"""TorchScript export of ForwardTacotron (reference `README.md:149-161`, the deployment path
`torch.jit.script(tts_model).generate_jit(x)`, `models/forward_tacotron.py:184-242,270-284`).

The compute of this package runs in libftmi.so (HIP kernels behind a C ABI, called through
ctypes), which TorchScript cannot compile.  So `torch.jit.script(model)` scripts a small
stand-in (`ForwardTacotron.__prepare_scriptable__` returns a `ScriptedForwardTacotron`) that
CARRIES THE MODEL: its constructor keywords and state_dict key order as a JSON string
attribute (`config`), every state_dict tensor but `step` as a `List[Tensor]` attribute
(`weights`, sharing storage with the eager model's parameters), and `step` as its own buffer
(the reference's `forward` increments it in training mode, `forward_tacotron.py:200-201`).
`torch.jit.save` writes all of it into the archive.  Its `forward` and `generate_jit` call two
operators registered in the dispatcher with `torch.library` (namespace `ftmi`, registered when
`forwardtacotron_amd` is imported):

    ftmi::ft_generate_jit(str config, Tensor[] weights, Tensor x, float alpha, float beta)
        -> (Tensor mel, Tensor mel_post, Tensor dur, Tensor pitch, Tensor energy)
    ftmi::ft_forward(str config, Tensor[] weights, Tensor x, Tensor mel, Tensor mel_len,
                     Tensor(a!) dur, Tensor pitch, Tensor energy) -> (the same five)

Their kernels (CompositeExplicitAutograd, for every device) rebuild an eager
`ForwardTacotron` on a HIP device from those arguments — cached per (config, the weight
tensors' storage and version), so a call after the first reuses the device model, its weight
packs and graphs, and an in-place update of any weight rebuilds it — and run its
`generate_jit` / `forward` on the HIP path.  So an archive made in one process runs in any
other that has imported `forwardtacotron_amd`:

    import torch, forwardtacotron_amd
    y = torch.jit.load('tts.pt').generate_jit(x)

Devices: the computation always runs on a HIP device (the weights' device when they are on
one, else the current one; no device raises).  The outputs go back to the device of `x` (CPU
in, CPU out, as the reference's CPU model returns them).  The operators are inference-only,
like this package's eager model (no autograd formula: an input that requires grad under grad
mode raises); `forward` in training mode differs from eval mode only in the `step` increment,
as in the eager model (inference numerics: no dropout, BatchNorm running statistics).
"""
from __future__ import annotations

import json
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
from torch import nn

FORMAT = 'forwardtacotron_amd.jit/1'
_KEYS = ('mel', 'mel_post', 'dur', 'pitch', 'energy')
# (config, device, (data_ptr, version, dtype, shape) per weight) -> (weights, device model):
# the entry holds the weight tensors themselves, so no other tensor can take their storage
# (and match the key) while it lives
_CACHE: 'OrderedDict[tuple, Tuple[List[torch.Tensor], nn.Module]]' = OrderedDict()
CACHE_SIZE = 2


def model_config(model) -> str:
    """The JSON `config` of a scripted ForwardTacotron: constructor keywords and the
    state_dict key order of `weights` (`step` excluded)."""
    kw = model.__dict__.get('_ctor_kwargs')
    if kw is None:
        raise RuntimeError('ForwardTacotron was built without recording its constructor keywords')
    keys = [k for k in model.state_dict() if k != 'step']
    return json.dumps({'format': FORMAT, 'kwargs': kw, 'keys': keys}, sort_keys=True)


def _compute_device(weights: List[torch.Tensor]) -> torch.device:
    if weights and weights[0].is_cuda:
        return weights[0].device
    if not torch.cuda.is_available():
        raise RuntimeError('forwardtacotron_amd computes on a HIP device; none is available')
    return torch.device('cuda', torch.cuda.current_device())


def device_model(config: str, weights: List[torch.Tensor]) -> nn.Module:
    """The eager ForwardTacotron that `config` + `weights` describe, on a HIP device, in eval
    mode (built once per weights version; see module docstring)."""
    dev = _compute_device(weights)
    key = (config, dev, tuple((w.data_ptr(), w._version, w.dtype, tuple(w.shape)) for w in weights))
    ent = _CACHE.pop(key, None)
    if ent is None:
        cfg = json.loads(config)
        if cfg.get('format') != FORMAT:
            raise RuntimeError(f'ftmi TorchScript archive of format {cfg.get("format")!r}; '
                               f'this package reads {FORMAT!r}')
        keys = cfg['keys']
        if len(keys) != len(weights):
            raise RuntimeError(f'ftmi TorchScript archive: {len(weights)} weights for '
                               f'{len(keys)} state_dict keys')
        from .forward_tacotron import ForwardTacotron
        m = ForwardTacotron(**cfg['kwargs'])
        if all(w.device == dev for w in weights):
            # the weights already live on the compute device (a scripted GPU model): build the
            # device model AROUND them — its parameters / buffers share their storage, so the
            # device holds one copy (load_state_dict + .to() made a second one)
            own = dict(m.named_parameters())
            own.update(m.named_buffers())
            for k, w in zip(keys, weights):
                t = own[k]
                if t.shape != w.shape or t.dtype != w.dtype:
                    raise RuntimeError(f'ftmi TorchScript archive: {k} is {tuple(w.shape)} '
                                       f'{w.dtype}, the model expects {tuple(t.shape)} {t.dtype}')
                t.data = w
            m = m.to(dev).eval()  # moves only `step`; the shared tensors are already there
        else:
            sd = dict(zip(keys, weights))
            sd['step'] = m.step
            m.load_state_dict(sd)
            m = m.to(dev).eval()
        ent = (list(weights), m)
        while len(_CACHE) >= CACHE_SIZE:
            _CACHE.popitem(last=False)
    _CACHE[key] = ent  # most recently used last
    return ent[1]


def clear_cache() -> None:
    """Drop the cached device models (their weight packs and HIP graphs).  Storage sharing
    has the limits of any TorchScript attribute: the scripted module holds the tensors it was
    scripted with, so re-assigning the eager model's parameters afterwards (`.to()`,
    `param.data = ...`) leaves the scripted module on the old tensors — script again after
    moving a model; in-place updates of the shared tensors ARE seen (the cache key carries
    each tensor's version)."""
    _CACHE.clear()


def _outputs(out: Dict[str, torch.Tensor], device) -> Tuple[torch.Tensor, ...]:
    return tuple(out[k].to(device) for k in _KEYS)


def _no_grad_inputs(op: str, *ts: torch.Tensor) -> None:
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        raise RuntimeError(f'ftmi::{op} is inference-only (no autograd formula): call it under '
                           'torch.no_grad() or with inputs that do not require grad')


def _generate_jit_impl(config: str, weights: List[torch.Tensor], x: torch.Tensor,
                       alpha: float, beta: float):
    m = device_model(config, weights)
    xd = x.to(m.embedding.weight.device)
    return _outputs(m.generate_jit(xd, alpha=alpha, beta=beta), x.device)


def _forward_impl(config: str, weights: List[torch.Tensor], x, mel, mel_len, dur, pitch, energy):
    _no_grad_inputs('ft_forward', mel, dur, pitch, energy)
    m = device_model(config, weights)
    dev = m.embedding.weight.device
    d = dur.to(dev)
    out = m({'x': x.to(dev), 'mel': mel.to(dev), 'mel_len': mel_len.to(dev), 'dur': d,
             'pitch': pitch.to(dev), 'energy': energy.to(dev)})
    if d.data_ptr() != dur.data_ptr():
        dur.copy_(d)  # the reference's LengthRegulator clips batch['dur'] in place
    return _outputs(out, x.device)


_LIB = torch.library.Library('ftmi', 'DEF')
_LIB.define('ft_generate_jit(str config, Tensor[] weights, Tensor x, float alpha, float beta) '
            '-> (Tensor, Tensor, Tensor, Tensor, Tensor)')
_LIB.define('ft_forward(str config, Tensor[] weights, Tensor x, Tensor mel, Tensor mel_len, '
            'Tensor(a!) dur, Tensor pitch, Tensor energy) '
            '-> (Tensor, Tensor, Tensor, Tensor, Tensor)')
_LIB.impl('ft_generate_jit', _generate_jit_impl, 'CompositeExplicitAutograd')
_LIB.impl('ft_forward', _forward_impl, 'CompositeExplicitAutograd')


class ScriptedForwardTacotron(nn.Module):
    """What `torch.jit.script(ForwardTacotron)` compiles: the reference's scriptable surface
    (`forward(batch)`, `@torch.jit.export generate_jit(x, alpha, beta)`) over the ftmi
    operators, carrying the model (see module docstring)."""

    def __init__(self, model) -> None:
        super().__init__()
        sd = model.state_dict()
        self.config: str = model_config(model)
        self.weights: List[torch.Tensor] = [sd[k] for k in json.loads(self.config)['keys']]
        self.register_buffer('step', sd['step'])  # shares the eager model's step
        self.train(model.training)

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        if self.training:
            self.step += 1
        mel, mel_post, dur, pitch, energy = torch.ops.ftmi.ft_forward(
            self.config, self.weights, batch['x'], batch['mel'], batch['mel_len'], batch['dur'],
            batch['pitch'], batch['energy'])
        return {'mel': mel, 'mel_post': mel_post, 'dur': dur, 'pitch': pitch, 'energy': energy}

    @torch.jit.export
    def generate_jit(self, x: torch.Tensor, alpha: float = 1.0,
                     beta: float = 1.0) -> Dict[str, torch.Tensor]:
        mel, mel_post, dur, pitch, energy = torch.ops.ftmi.ft_generate_jit(
            self.config, self.weights, x, alpha, beta)
        return {'mel': mel, 'mel_post': mel_post, 'dur': dur, 'pitch': pitch, 'energy': energy}
