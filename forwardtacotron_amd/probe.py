"""Per-launch kernel timing with HIP events (bench.py's live roofline measurement).

Every ops.* wrapper enqueues exactly one ftmi_* entry point (one kernel; ftmi_rnn_bidir
adds a 16-byte-aligned workspace memset) on torch's current stream and reports a label
plus the launch's ALGORITHMIC work: flops (2 per multiply-add of the contraction the
reference defines) and bytes (each input read once + each output written once).  While a
KernelProbe is active the launch is bracketed by two torch.cuda.Events on that same
stream, so elapsed_time() is that kernel's device duration.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional

import torch

from ._lib import call

_ACTIVE: Optional['KernelProbe'] = None


class KernelProbe:
    def __init__(self):
        self.events = OrderedDict()  # label -> [(start, end)]
        self.meta = {}               # label -> (entry point, flops, bytes)

    def __enter__(self):
        global _ACTIVE
        self._prev, _ACTIVE = _ACTIVE, self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = self._prev
        return False

    def summary(self):
        """After a device sync: {label: dict(entry, launches, avg_ms, total_ms, flops, bytes)}."""
        out = OrderedDict()
        for label, evs in self.events.items():
            ms = []
            for s, e in evs:
                try:
                    ms.append(s.elapsed_time(e))
                except RuntimeError:  # under rocprofv3 --pmc (serialised dispatch) some
                    pass              # event pairs report no time: the run is for counters
            if not ms:
                continue
            name, flops, nbytes = self.meta[label]
            out[label] = {'entry': name, 'launches': len(ms), 'total_ms': sum(ms),
                          'avg_ms': sum(ms) / len(ms), 'flops': flops, 'bytes': nbytes}
        return out


def launch(name: str, label: str, flops: float, nbytes: float, *args) -> None:
    p = _ACTIVE
    if p is None:
        call(name, *args)
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    call(name, *args)
    e.record()
    p.events.setdefault(label, []).append((s, e))
    p.meta[label] = (name, float(flops), float(nbytes))
