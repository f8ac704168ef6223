"""TorchScript export of ForwardTacotron (reference `README.md:149-161`, the deployment path
`torch.jit.script(tts_model).generate_jit(x)`, `models/forward_tacotron.py:184-242,270-284`).

The compute of this package runs in libftmi.so (HIP kernels behind a C ABI, called through
ctypes), which TorchScript cannot compile.  So `torch.jit.script(model)` scripts a small
stand-in (`ForwardTacotron.__prepare_scriptable__` returns a `ScriptedForwardTacotron`)
whose `forward` and `generate_jit` call two operators registered in the dispatcher with
`torch.library` (namespace `ftmi`):

    ftmi::ft_generate_jit(int handle, Tensor x, float alpha, float beta)
        -> (Tensor mel, Tensor mel_post, Tensor dur, Tensor pitch, Tensor energy)
    ftmi::ft_forward(int handle, Tensor x, Tensor mel, Tensor mel_len, Tensor dur,
                     Tensor pitch, Tensor energy) -> (the same five)

whose kernels (CompositeExplicitAutograd, for every device) run the model's own eager
`generate_jit` / `forward` on the HIP path.  `handle` names the Python model in this
process's registry; the scripted module keeps it as an attribute, so the module (and a
`torch.jit.save` / `torch.jit.load` round trip of it) runs in the process that scripted it
— the kernels live in libftmi.so, not in the TorchScript archive.

Devices: the computation always runs on a HIP device.  A model whose weights are on the CPU
(the README's `from_checkpoint` then `torch.jit.script`) computes on a device replica made
once per weights version; the outputs go back to the device of `x` (CPU in, CPU out, as the
reference's CPU model returns them).
"""
from __future__ import annotations

import copy
import itertools
import weakref
from typing import Dict, Tuple

import torch
from torch import nn

_REGISTRY: Dict[int, 'weakref.ReferenceType'] = {}
_IDS = itertools.count(1)
_KEYS = ('mel', 'mel_post', 'dur', 'pitch', 'energy')


def register(model) -> int:
    """The handle of `model` (registered once; the registry holds a weak reference)."""
    h = model.__dict__.get('_ftmi_jit_handle')
    if h is None or h not in _REGISTRY:
        h = next(_IDS)
        _REGISTRY[h] = weakref.ref(model)
        model.__dict__['_ftmi_jit_handle'] = h
    return h


def _model(handle: int):
    ref = _REGISTRY.get(int(handle))
    m = ref() if ref is not None else None
    if m is None:
        raise RuntimeError(f'ftmi TorchScript handle {handle}: no ForwardTacotron with that handle in '
                           'this process (a scripted module runs where it was scripted: its '
                           'kernels live in libftmi.so)')
    return m


def _device_model(m):
    """m itself on a HIP device, else its replica on the current HIP device (rebuilt when the
    weights change: the model's weights key)."""
    if m.embedding.weight.is_cuda:
        return m
    if not torch.cuda.is_available():
        raise RuntimeError('forwardtacotron_amd computes on a HIP device; none is available')
    key = m._weights_key()
    ent = m.__dict__.get('_ftmi_jit_replica')
    if ent is None or ent[0] != key:
        # the per-module caches (weight packs, graphs, streams, this replica) stay behind
        saved = [(mod, {k: mod.__dict__.pop(k) for k in list(mod.__dict__) if k.startswith('_ftmi')})
                 for mod in m.modules()]
        try:
            rep = copy.deepcopy(m)
        finally:
            for mod, d in saved:
                mod.__dict__.update(d)
        ent = (key, rep.to(torch.device('cuda', torch.cuda.current_device())).eval())
        m.__dict__['_ftmi_jit_replica'] = ent
    ent[1].training = m.training
    return ent[1]


def _outputs(out: Dict[str, torch.Tensor], device) -> Tuple[torch.Tensor, ...]:
    return tuple(out[k].to(device) for k in _KEYS)


def _generate_jit_impl(handle: int, x: torch.Tensor, alpha: float, beta: float):
    m = _device_model(_model(handle))
    xd = x.to(m.embedding.weight.device)
    return _outputs(m.generate_jit(xd, alpha=alpha, beta=beta), x.device)


def _forward_impl(handle: int, x, mel, mel_len, dur, pitch, energy):
    src = _model(handle)
    m = _device_model(src)
    dev = m.embedding.weight.device
    d = dur.to(dev)
    out = m({'x': x.to(dev), 'mel': mel.to(dev), 'mel_len': mel_len.to(dev), 'dur': d,
             'pitch': pitch.to(dev), 'energy': energy.to(dev)})
    if d.data_ptr() != dur.data_ptr():
        dur.copy_(d)  # the reference's LengthRegulator clips batch['dur'] in place
    if m is not src and src.training:
        src.step.copy_(m.step.to(src.step.device))
    return _outputs(out, x.device)


_LIB = torch.library.Library('ftmi', 'DEF')
_LIB.define('ft_generate_jit(int handle, Tensor x, float alpha, float beta) '
            '-> (Tensor, Tensor, Tensor, Tensor, Tensor)')
_LIB.define('ft_forward(int handle, Tensor x, Tensor mel, Tensor mel_len, Tensor dur, '
            'Tensor pitch, Tensor energy) -> (Tensor, Tensor, Tensor, Tensor, Tensor)')
_LIB.impl('ft_generate_jit', _generate_jit_impl, 'CompositeExplicitAutograd')
_LIB.impl('ft_forward', _forward_impl, 'CompositeExplicitAutograd')


class ScriptedForwardTacotron(nn.Module):
    """What `torch.jit.script(ForwardTacotron)` compiles: the reference's scriptable surface
    (`forward(batch)`, `@torch.jit.export generate_jit(x, alpha, beta)`) over the ftmi
    operators; `handle` is the eager model's registry handle."""

    def __init__(self, model) -> None:
        super().__init__()
        self.handle = register(model)

    def forward(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        mel, mel_post, dur, pitch, energy = torch.ops.ftmi.ft_forward(
            self.handle, batch['x'], batch['mel'], batch['mel_len'], batch['dur'],
            batch['pitch'], batch['energy'])
        return {'mel': mel, 'mel_post': mel_post, 'dur': dur, 'pitch': pitch, 'energy': energy}

    @torch.jit.export
    def generate_jit(self, x: torch.Tensor, alpha: float = 1.0,
                     beta: float = 1.0) -> Dict[str, torch.Tensor]:
        mel, mel_post, dur, pitch, energy = torch.ops.ftmi.ft_generate_jit(
            self.handle, x, alpha, beta)
        return {'mel': mel, 'mel_post': mel_post, 'dur': dur, 'pitch': pitch, 'energy': energy}
