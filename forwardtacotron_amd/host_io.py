"""Host transfers of generate()'s results that do not serialise the device.

`gen_forward.py:120` takes each result with `gen['mel_post'].cpu()`: a pageable copy that the
host waits for before it issues the next sentence, so the copy (28 MB per c3 batch) and the
next call's launch latency sit between two generate() calls on the device.  `PinnedD2H`
copies into page-locked buffers on a side stream ordered after the producing stream: the
next call's phoneme phase runs while the previous result drains over PCIe, and the host
waits only where it actually reads a result (`done.synchronize()`)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class PinnedD2H:
    """Ring of `depth` pinned host buffers filled by stream-ordered device->host copies.

    submit(t) queues the copy of t behind the work already issued on t's current stream
    and returns (host buffer, done event); the buffer holds t once `done` has completed.
    A slot (and its buffer) is reused `depth` submits later: a caller that reads a result
    must be finished with it by then (the copy stream itself orders the device side)."""

    def __init__(self, device, depth: int = 2) -> None:
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.depth = depth
        self.bufs: List[Optional[torch.Tensor]] = [None] * depth
        self.done: List[Optional[torch.cuda.Event]] = [None] * depth
        self.i = 0

    def submit(self, t: torch.Tensor) -> Tuple[torch.Tensor, torch.cuda.Event]:
        slot = self.i % self.depth
        self.i += 1
        buf = self.bufs[slot]
        if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
            if self.done[slot] is not None:  # the old buffer's last copy must have landed
                self.done[slot].synchronize()
            buf = self.bufs[slot] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(t.device))
        self.stream.wait_event(ready)
        with torch.cuda.stream(self.stream):
            buf.copy_(t, non_blocking=True)
        t.record_stream(self.stream)  # t's memory is not reused before the copy has read it
        done = torch.cuda.Event()
        done.record(self.stream)
        self.done[slot] = done
        return buf, done

    def fetch(self, t: torch.Tensor) -> torch.Tensor:
        """t on the host now (pinned copy, waits for it; a private copy of the ring slot):
        the drop-in for `t.cpu()`."""
        buf, done = self.submit(t)
        done.synchronize()
        return buf.clone()

    def synchronize(self) -> None:
        self.stream.synchronize()
