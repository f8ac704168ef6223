"""Batch-sharded generation over one process per GPU.

Utterances are independent in the math but the reference couples a batch through three
things; reproducing ONE reference call on the concatenation of all shards needs exactly:
  1. every shard padded to the GLOBAL phoneme length T (pad id 0)       all_reduce(MAX)
  2. the fill-2 rule (`forward_tacotron.py:254-255`, `fast_pitch.py:293-294`) decided on
     the WHOLE batch's sum of int64(trunc(dur))                        all_reduce(SUM, int64)
  3. the LengthRegulator output padded to the GLOBAL T_mel (max over all items)
                                                                       all_reduce(MAX)
Everything else is rank-local; the results are all-gathered (mel_post is
(B_global, 80, T_mel) on every rank, exactly the reference's output).  The collectives
are a few bytes, except the result gather; with the NCCL (= RCCL over xGMI) backend they
run on device tensors, with gloo on host copies.  Weights are either built identically on
every rank or broadcast once from rank 0 (`broadcast_state`).

The collective steps are plain functions of torch tensors so the protocol is testable on
CPU with gloo (tests/test_sharded.py); `generate_sharded` composes them with the HIP model.

Result collection can run on its own communicator (`gather_group`, e.g. `dist.new_group()`
made once at setup) and asynchronously (`async_gather=True`): step i's rank-0 gather then
runs on that communicator's RCCL stream while step i+1's shard-size all-gather and phoneme
phase run on the protocol's communicator and the compute stream.  On the SAME communicator
the next step's first collective would queue behind the gather.  Every rank issues the
collectives of both communicators in the same program order, the ordering RCCL needs
when communicators run concurrently.

`CollectiveTimer` times every collective of the protocol (the weights broadcast, the
shard-size all-gather, the fill-rule and T_mel all-reduces, the status all-reduce, the
result gather) for the c4 bench line.
"""
from __future__ import annotations

import contextlib
import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops


def _coll_device(group, like: torch.device) -> torch.device:
    """Tensors for collectives: the GPU for nccl (RCCL), the host for gloo."""
    backend = dist.get_backend(group)
    return like if backend == 'nccl' else torch.device('cpu')


class CollectiveTimer:
    """Per-collective time of the sharded protocol.  On a device (nccl = RCCL) HIP events
    on the issuing stream bracket each blocking collective: the RCCL stream waits for the
    start event and the issuing stream waits for the collective, so the interval is the
    collective including the wait for the slowest peer.  With gloo it is the host clock
    around the blocking call.  summary() synchronises and returns {name: {calls, total_ms,
    avg_ms}}."""

    def __init__(self) -> None:
        self._rec = []

    @contextlib.contextmanager
    def span(self, name: str, dev: torch.device):
        if dev.type == 'cuda':
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._rec.append((name, a, b))
        else:
            t0 = time.perf_counter()
            yield
            self._rec.append((name, (time.perf_counter() - t0) * 1e3, None))

    def reset(self) -> None:
        self._rec = []

    def summary(self) -> Dict[str, Dict[str, float]]:
        if any(b is not None for _, _, b in self._rec):
            torch.cuda.synchronize()
        out: Dict[str, Dict[str, float]] = {}
        for name, a, b in self._rec:
            ms = a.elapsed_time(b) if b is not None else a
            d = out.setdefault(name, {'calls': 0, 'total_ms': 0.0})
            d['calls'] += 1
            d['total_ms'] += ms
        for d in out.values():
            d['avg_ms'] = d['total_ms'] / d['calls']
        return out


def _span(timer: Optional[CollectiveTimer], name: str, dev: torch.device):
    return timer.span(name, dev) if timer is not None else contextlib.nullcontext()


def global_max(value: int, group=None, device: torch.device = torch.device('cpu'),
               timer: Optional[CollectiveTimer] = None, name: str = 'all_reduce MAX') -> int:
    dev = _coll_device(group, device)
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    with _span(timer, name, dev):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def global_sum_(t: torch.Tensor, group=None, timer: Optional[CollectiveTimer] = None,
                name: str = 'all_reduce SUM') -> torch.Tensor:
    """In-place SUM all-reduce of a small tensor (device tensor stays on device for nccl)."""
    dev = _coll_device(group, t.device)
    if dev == t.device:
        with _span(timer, name, dev):
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t
    h = t.to(dev)
    with _span(timer, name, dev):
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    t.copy_(h)
    return t


def pad_tokens(x: torch.Tensor, T: int) -> torch.Tensor:
    """Right-pad (B, t) phoneme ids with the pad id 0 to length T."""
    if x.size(1) == T:
        return x
    out = torch.zeros(x.size(0), T, dtype=x.dtype, device=x.device)
    out[:, :x.size(1)] = x
    return out


def shard_sizes(n_local: int, t_local: int, group=None,
                device: torch.device = torch.device('cpu'),
                timer: Optional[CollectiveTimer] = None):
    """ONE all-gather of (rows, phoneme length) per rank -> (rows of every rank, global T)."""
    world = dist.get_world_size(group)
    dev = _coll_device(group, device)
    mine = torch.tensor([int(n_local), int(t_local)], dtype=torch.int64, device=dev)
    allv = torch.empty(world * 2, dtype=torch.int64, device=dev)
    with _span(timer, 'shard_sizes all_gather', dev):
        dist.all_gather_into_tensor(allv, mine, group=group)
    v = allv.view(world, 2).tolist()
    return [r[0] for r in v], max(r[1] for r in v)


def _padded(t: torch.Tensor, nmax: int, dev) -> torch.Tensor:
    src = t.to(dev).contiguous()
    if src.size(0) < nmax:
        pad = torch.zeros((nmax - src.size(0),) + tuple(src.shape[1:]), dtype=src.dtype, device=dev)
        src = torch.cat([src, pad], 0)
    return src


def gather_rows(t: torch.Tensor, group=None, sizes: Optional[List[int]] = None) -> torch.Tensor:
    """All-gather along dim 0 with per-rank row counts that may differ (`sizes`: known
    counts, e.g. from shard_sizes; otherwise one extra all-gather finds them)."""
    world = dist.get_world_size(group)
    dev = _coll_device(group, t.device)
    if sizes is None:
        sizes, _ = shard_sizes(t.size(0), 0, group, t.device)
    src = _padded(t, max(sizes), dev)
    bufs = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(bufs, src, group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0).to(t.device)


class PendingRows:
    """An in-flight gather_rows_to(async_op=True).  wait() -> the concatenation on `dst`
    (None elsewhere); with nccl it orders the issuing stream after the RCCL gather without
    blocking the host."""

    def __init__(self, work, src, bufs, sizes, device) -> None:
        self._work, self._src, self._bufs, self._sizes, self._device = work, src, bufs, sizes, device

    def wait(self) -> Optional[torch.Tensor]:
        self._work.wait()
        self._src = None
        if self._bufs is None:
            return None
        return torch.cat([b[:s] for b, s in zip(self._bufs, self._sizes)], 0).to(self._device)


def gather_rows_to(t: torch.Tensor, sizes: List[int], dst: int = 0, group=None,
                   timer: Optional[CollectiveTimer] = None, async_op: bool = False):
    """Gather along dim 0 to rank `dst` only (result collection: one copy of the output,
    not one per rank); returns the concatenation on `dst`, None elsewhere (async_op: a
    PendingRows whose wait() returns that)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)  # dst is a rank WITHIN the group, like this one
    dev = _coll_device(group, t.device)
    src = _padded(t, max(sizes), dev)
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == dst else None
    # dist.gather takes the destination as a GLOBAL rank
    gdst = dst if group is None else dist.get_global_rank(group, dst)
    if async_op:
        work = dist.gather(src, bufs, dst=gdst, group=group, async_op=True)
        return PendingRows(work, src, bufs if rank == dst else None, sizes, t.device)
    with _span(timer, 'result gather to rank 0', dev):
        dist.gather(src, bufs, dst=gdst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0).to(t.device)


class GlobalBatch:
    """The batch-coupling hooks `generate(..., batch=GlobalBatch(group))` calls."""

    def __init__(self, group=None, timer: Optional[CollectiveTimer] = None) -> None:
        self.group = group
        self.timer = timer

    def duration_counts(self, dur_hat: torch.Tensor):
        """fill-2 rule on the global sum, then this shard's clip / counts / offsets."""
        s = ops.duration_trunc_sum(dur_hat)
        global_sum_(s, self.group, self.timer, 'fill_rule all_reduce SUM')
        offsets, totals, _ = ops.duration_counts_global(dur_hat, s)
        return offsets, totals

    def t_mel(self, totals: torch.Tensor) -> int:
        local = int(totals.max().item()) if totals.numel() else 0
        return global_max(local, self.group, totals.device, self.timer, 't_mel all_reduce MAX')

    def status(self, word: torch.Tensor) -> torch.Tensor:
        """The status word (ops.run_checked) OR-ed over ranks — one MAX all-reduce of its
        bits — so every rank takes the same rerun / raise decision."""
        dev = _coll_device(self.group, word.device)
        w = word.to(dev).reshape(1)
        bits = torch.cat([(w >> i) & 1 for i in range(3)])
        with _span(self.timer, 'status all_reduce MAX', dev):
            dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=self.group)
        return (bits << torch.arange(3, device=dev, dtype=bits.dtype)).sum().reshape(1).to(word.device)


def broadcast_state(model: torch.nn.Module, src: int = 0, group=None,
                    timer: Optional[CollectiveTimer] = None) -> None:
    """Copy rank `src`'s parameters and buffers to every rank: the tensors are packed into
    ONE flat buffer per dtype (98 MB fp32 for ForwardTacotron) and broadcast in one
    collective each (RCCL over xGMI with the nccl backend: one large transfer instead of
    ~330 small ones), then unpacked in place (so the packed-weight caches see new
    versions and re-pack)."""
    tensors = list(model.parameters()) + list(model.buffers())
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dt, ts in by_dtype.items():
        dev = _coll_device(group, ts[0].device)
        flat = torch.cat([t.detach().reshape(-1).to(dev) for t in ts])
        with _span(timer, 'weights broadcast', dev):
            dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class PendingResult:
    """generate_sharded(async_gather=True)'s return: wait() -> the collected dict (as the
    blocking call returns it: rank 0 for 'rank0', every rank for 'all')."""

    def __init__(self, parts: Dict[str, object], alias_mel: bool, is_none: bool) -> None:
        self._parts, self._alias, self._none = parts, alias_mel, is_none

    def wait(self) -> Optional[Dict[str, torch.Tensor]]:
        res = {k: (p.wait() if isinstance(p, PendingRows) else p) for k, p in self._parts.items()}
        if self._none:
            return None
        if self._alias:
            res['mel_post'] = res['mel']
        return res


def generate_sharded(model, x: torch.Tensor, alpha: float = 1.0,
                     pitch_function: Callable = lambda p: p,
                     energy_function: Callable = lambda e: e,
                     group=None, gather='all', gather_group=None, async_gather: bool = False,
                     timer: Optional[CollectiveTimer] = None):
    """This rank's shard x (B_local, t) of one global batch -> the reference's output for the
    whole batch.  gather: 'all' (or True) = every rank holds all rows, in rank order;
    'rank0' = result collection on rank 0 only (other ranks return None); 'none' (or False)
    = this rank's rows of it.  Shard sizes and the global phoneme length come from one
    all-gather at the start.  gather_group: the communicator of the result collection
    (default `group`; same ranks in the same order).  async_gather ('rank0'): return a
    PendingResult at once, the gather in flight on gather_group.  timer: a CollectiveTimer
    that records every blocking collective.  ForwardTacotron and FastPitch."""
    if gather is True:
        gather = 'all'
    elif gather is False:
        gather = 'none'
    if async_gather and gather != 'rank0':
        raise ValueError("async_gather needs gather='rank0'")
    sizes, T = shard_sizes(x.size(0), x.size(1), group, x.device, timer)
    x = pad_tokens(x, T)
    out = model.generate(x, alpha, pitch_function, energy_function,
                         batch=GlobalBatch(group, timer))
    if gather == 'none':
        return out
    ggroup = group if gather_group is None else gather_group
    alias = out['mel_post'] is out['mel']
    res = {}
    for k, v in out.items():
        if k == 'mel_post' and alias:
            continue
        if gather == 'rank0':
            res[k] = gather_rows_to(v, sizes, 0, ggroup, timer, async_op=async_gather)
        else:
            res[k] = gather_rows(v, ggroup, sizes)
    is_none = gather == 'rank0' and dist.get_rank(ggroup) != 0
    if async_gather:
        return PendingResult(res, alias, is_none)
    if is_none:
        return None
    if alias:
        res['mel_post'] = res['mel']
    return res
