"""Benchmark: ForwardTacotron.generate() mel-frames/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

Workload (default: BASELINE.json configs[2], "c3"): ForwardTacotron LJSpeech config, batch =
64 synthetic phoneme sequences per GPU (lengths U{50..200}, ids U{1..134}, pad 0; seed =
rank), synthetic weights (forwardtacotron_amd.synthetic, no checkpoint download), fp32-level
arithmetic (f16x3 MFMA split, range-guarded).  A step is one full `generate()` call on one
batch whose tokens are already resident in HBM (pitch / energy identity callbacks, alpha =
1).  Frames = B * T_mel of the returned mel_post (padded frames, as the reference returns
them); `valid_frames_per_s` counts only each utterance's own frames.
  --config c2            configs[1]: batch 1, 120 phonemes
  --callbacks gen_forward  the callbacks gen_forward.py:103-104 passes
                         (pitch_function = lambda x: x * amp, energy_function = lambda x: x)
  --vocoder griffinlim   configs[1] names the Griffin-Lim vocoder: a THIRD timed loop runs the
                         whole gen_forward.py sentence step (generate, mel_post.cpu(),
                         dsp.griffinlim -> numpy wav, :115-134) and reports it beside `value`
                         as `with_vocoder` (batch > 1: DSP.griffinlim_batch on the device)
  --model fast_pitch     configs[4], "c5": FastPitch, batch 64, lengths U{50..200}
  --model wavernn        the `gen_forward.py wavernn` vocoder (no BASELINE
                         number): WaveRNN.generate of one c2-length mel (821 frames, synthetic
                         log-mel values) with gen_forward's batched defaults (target 11000,
                         overlap 550, 19 folds), RAW 9 bits, mu-law; metric audio samples/s
                         (wave_len per generate() call, the float64 wave on the host); N > 1:
                         replicas only (each rank its own utterance, no collective)

Multi-GPU (c4, BASELINE.json configs[3]): rank 0 makes the synthetic weights and
broadcasts them (sharded.broadcast_state: one bucketed RCCL broadcast per dtype); the
ranks hold the shards (64 utterances each, seed = rank) of ONE global batch and run
forwardtacotron_amd.sharded.generate_sharded(gather='rank0'): global phoneme padding, the
batch-global fill-2 rule and T_mel by scalar RCCL all-reduces, mel_post gathered to rank 0
only (result collection) — the reference's output for the global batch (weak scaling:
per-GPU work fixed).  The gather runs on its own communicator and is left in flight while
the next step runs (--gather-overlap off: blocking).  Barrier + synchronize around the K
timed steps, max elapsed over ranks, value = frames of the global mel_post / that time.
`collectives` in the line: per-collective RCCL times (HIP events, max over ranks) from one
more loop with the gather blocking, the weights broadcast, and every rank's step time.

The JSON line also carries
  roofline     the dominant kernel (largest device time inside the timed steps, measured
               with HIP events on the launch stream): algorithmic FLOPs per launch / its
               average duration, against the peak of the arithmetic that kernel issues
               (f16x3 "mma=2": dense f16 MFMA / 3; bf16x6 "mma=1": / 6; fp32 MFMA), and
               `traffic` = HBM bytes per launch from the committed PMC passes;
  host_to_host the PCIe-inclusive rate: token ids H2D + generate() + mel_post D2H per step,
               as gen_forward.py:111-120 does (a second timed loop; never `value`);
  prenet_bank  the north-star kernel (fused Conv1d+ReLU+BN CBHG bank) against HBM and MFMA;
  cpu_baseline rank 0, N = 1: the torch-CPU restatement of the reference (oracle/
               ft_torch_cpu.py, the reference's ATen CPU kernels) on the same batch at all
               host threads given (CPU model, physical cores, threads used) and on 1 thread
               for the first 8 utterances;
  parity       mean / max |mel_post GPU - CPU| on that batch, and LR counts equality.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from forwardtacotron_amd import forward_tacotron as ft_module  # noqa: E402
from forwardtacotron_amd.fast_pitch import FastPitch  # noqa: E402
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402
from forwardtacotron_amd.probe import KernelProbe  # noqa: E402
from forwardtacotron_amd.sharded import (CollectiveTimer, broadcast_state,  # noqa: E402
                                         generate_sharded)
from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict, synthetic_tokens  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA == vector rate), MI355X_MICROARCH.md
# the fp32-accurate bf16x6 path (labels "mma=1") issues 6 bf16 MFMAs per fp32 product:
# its ceiling is the dense bf16 MFMA peak / 6
PEAK_BF16_TFLOPS = 2500.0  # == the dense f16 MFMA peak (same cycles per MFMA on gfx950)
PEAK_X6_TFLOPS = PEAK_BF16_TFLOPS / 6
# the default f16x3 path ("mma=2") issues 3 f16 MFMAs per fp32 product
PEAK_X3_TFLOPS = PEAK_BF16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec


PMC_PROFILE = os.path.join(ROOT, 'profiles', 'r6_pmc_traffic.json')        # c3
PMC_PROFILE_C2 = os.path.join(ROOT, 'profiles', 'r6final_c2_pmc_traffic.json')   # c2 (--config c2)
PMC_PROFILE_C5 = os.path.join(ROOT, 'profiles', 'r6c5_pmc_traffic.json')   # c5 (--model fast_pitch)
# the PMC files are a prior run of the same workload (separate FETCH_SIZE / WRITE_SIZE passes
# cannot share the timed run), taken on this tree
PMC_TREE = '16e443f (round 6: tools/gpu_r6_measure.sh pmc; MFMA-busy pass 3e61c87, GEMM kernels unchanged since)'
PMC_TREE_C2 = 'fcdfa17 (round 6 final tree: the mask-free prenet bank; FETCH_SIZE / WRITE_SIZE passes)'


def rocprof_name(label: str):
    """rocprof kernel-name prefix of a probe label (for the PMC traffic lookup)."""
    if label.startswith('rnn_bidir['):
        cell = 1 if label.startswith('rnn_bidir[lstm') else 0
        H = int(label.split('H=')[1].split(',')[0].rstrip(']'))
        B = int(label.split('B=')[1].split(',')[0])
        # rnn.hip gemv_path: B <= 4 runs the exact-fp32 GEMV recurrence for these shapes
        gemv = (os.environ.get('FTMI_RNN_GEMV', '1') != '0' and B <= 4
                and ((cell == 1 and H == 512) or (cell == 0 and H in (64, 128, 256))))
        if gemv:
            return f'rnn_gemv_kernel<{cell}, {H},'
        return f'rnn_bidir_kernel<{cell}, {H},'
    return None


def pmc_traffic(label: str, path: str = PMC_PROFILE):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes of the same
    workload (tools/profile_round.sh + tools/summarize_prof.py: FETCH_SIZE x 2 + WRITE_SIZE),
    or None."""
    pref = rocprof_name(label)
    if pref is None or not os.path.exists(path):
        return None
    ks = json.load(open(path))['kernels']
    hit = [v for k, v in ks.items() if k.startswith(pref)]
    if len(hit) != 1:
        return None
    return {'bytes_per_launch': hit[0]['hbm_bytes_per_launch'],
            'read_bytes_corrected': hit[0]['read_bytes_corrected'],
            'write_bytes': hit[0]['write_bytes'],
            'source': os.path.relpath(path, ROOT),
            'measured_on_tree': PMC_TREE_C2 if path == PMC_PROFILE_C2 else PMC_TREE,
            'note': 'a prior PMC run of this workload, not this run'}


def pmc_traffic_slab(label: str, path: str):
    """The same for a conv1d label run by the slab kernels (one kernel name for many shapes:
    the dispatch is told apart by its grid, gemm.hip launch_slab: whole XCD rounds of
    256-row tiles x 128-column tiles, 768 threads warp-specialised or 512), or None."""
    if not label.startswith('conv1d[') or not os.path.exists(path):
        return None
    f = dict(kv.split('=') for kv in label[7:-1].split(',') if '=' in kv)
    M, N = int(f['M']), int(f['N'])
    mt = -(-M // 256)
    nblk = (mt if mt < 8 else -(-mt // 8) * 8) * -(-N // 128)
    ks = json.load(open(path)).get('kernels_by_grid', {})
    hit = [(k, v) for k, v in ks.items() if k.startswith('conv_gemm_slab')
           and int(k.rsplit('|', 1)[1]) in (nblk * 768, nblk * 512)]
    if len(hit) != 1:
        return None
    k, v = hit[0]
    return {'bytes_per_launch': v['hbm_bytes_per_launch'],
            'read_bytes_corrected': v['read_bytes_corrected'], 'write_bytes': v['write_bytes'],
            'kernel_grid': k, 'source': os.path.relpath(path, ROOT),
            'measured_on_tree': PMC_TREE_C2 if path == PMC_PROFILE_C2 else PMC_TREE,
            'note': 'a prior PMC run of this workload, not this run'}


PMC_MFMA = os.path.join(ROOT, 'profiles', 'r6_pmc_mfma.json')  # tools/pmc_mfma.py


def pmc_mfma(label: str, cfg: str):
    """MFMA-busy share of the dominant kernel from the committed SQ_VALU_MFMA_BUSY_CYCLES /
    GRBM_GUI_ACTIVE pass of the same workload (tools/gpu_r5_measure.sh mfma), or None."""
    if not os.path.exists(PMC_MFMA):
        return None
    ks = json.load(open(PMC_MFMA)).get('configs', {}).get(cfg, {}).get('kernels', {})
    pref = rocprof_name(label)
    if pref is not None:
        hit = [(k, v) for k, v in ks.items() if k.startswith(pref)]
    elif label.startswith('conv1d['):
        f = dict(kv.split('=') for kv in label[7:-1].split(',') if '=' in kv)
        M, N = int(f['M']), int(f['N'])
        mt = -(-M // 256)
        nblk = (mt if mt < 8 else -(-mt // 8) * 8) * -(-N // 128)
        hit = [(k, v) for k, v in ks.items() if k.startswith('conv_gemm_slab')
               and int(k.rsplit('|', 1)[1]) in (nblk * 768, nblk * 512)]
    else:
        return None
    if len(hit) != 1 or 'mfma_busy' not in hit[0][1]:
        return None
    k, v = hit[0]
    return {'mfma_busy': v['mfma_busy'], 'kernel_grid': k,
            'definition': 'SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): '
                          'the share of the dispatch\'s active cycles an average SIMD\'s matrix '
                          'pipe was busy (16 cycles per v_mfma_f32_16x16x32_f16)',
            'source': os.path.relpath(PMC_MFMA, ROOT),
            'note': 'a separate --pmc run of this workload on this round\'s tree, not this run'}


def time_prenet_bank(model, x, reps: int = 20):
    """The prenet CBHG conv bank exactly as generate() issues it (same operand, packed
    weights, pooled / split-output choice; at c2 the one-launch halves kernel on the
    stream-order weight image; where the channel-split kernel runs, the bank + its finish
    launch), ms per call:
      warm  — `reps` calls captured in a HIP graph and replayed back to back (device time per
              call, kernel boundaries included, no host issue cost); the weights stay
              Infinity-Cache resident, as in a generate() loop;
      eager — the same calls issued from the host one by one (ctypes + argument packing);
      cold  — each call behind a 512 MiB overwrite of another buffer (the weights come from
              HBM): graph [overwrite, call] x reps minus graph [overwrite] x reps; the
              overwrite's dirty lines are still draining to HBM while the call reads;
      cold_read — each call behind a 1 GiB streaming READ of another buffer (the weights
              evicted from L2 and the 256 MB Infinity Cache by clean lines: weights from HBM,
              no write-back in flight): graph [read, call] x reps minus graph [read] x reps;
      planes — A/B in the same process: the halves kernel reading the split planes."""
    from forwardtacotron_amd import ops
    cb = model.prenet
    h = ops.embedding(x, model.embedding.weight.detach())
    bank_w, scale, shift, _, bank3, _, img = cb.packed_weights()
    pooled = ops.bank_pools(h, cb.K, cb.channels, w_split=bank3)
    if pooled or not ops._bank_halves(ops._gemm_mma(None, bank3)[0], h.size(0), h.size(1),
                                      h.size(2), cb.K, cb.channels):
        img = None  # the image serves the one-launch few-row kernel only

    def call(image=img):
        return ops.conv_bank(h, bank_w, cb.K, cb.channels, scale, shift, w_split=bank3,
                             pool=pooled, split_out=pooled and ops.SPLIT_ROWS, w_image=image)

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    for _ in range(3):
        call()
    eager = timed(lambda: [call() for _ in range(reps)]) / reps
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=x.device)
    rflush = torch.zeros(1 << 28, dtype=torch.float32, device=x.device)  # 1 GiB, read only
    graphs = {}
    bodies = [('warm', lambda: call()), ('flush', lambda: flush.fill_(1)),
              ('cold', lambda: (flush.fill_(1), call())),
              ('rflush', lambda: rflush.sum()), ('cold_read', lambda: (rflush.sum(), call()))]
    if img is not None:  # A/B: the same kernel on the split planes
        bodies += [('planes', lambda: call(None))]
    for name, body in bodies:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                body()
        g.replay()
        graphs[name] = g
    res = {'warm': timed(graphs['warm'].replay) / reps, 'eager': eager,
           'cold': (timed(graphs['cold'].replay) - timed(graphs['flush'].replay)) / reps,
           'cold_read': (timed(graphs['cold_read'].replay) - timed(graphs['rflush'].replay)) / reps,
           'weights': ('stream-order image' if img is not None
                       else 'split planes (no few-row kernel at this size)')}
    if img is not None:
        res['planes'] = timed(graphs['planes'].replay) / reps
    del graphs, flush, rflush
    return res


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dsp_kernel_table(kern):
    """The audio kernels of a probe summary against the HBM roofline: algorithmic bytes per
    launch (each input read once, each output written once) / the launch's average device
    time, as a fraction of 8 TB/s."""
    out = {}
    for lab, v in kern.items():
        if v['bytes'] <= 0 or v['avg_ms'] <= 0:
            continue
        gbs = v['bytes'] / (v['avg_ms'] / 1e3) / 1e9
        out[lab] = {'launches': v['launches'], 'avg_ms': round(v['avg_ms'], 4),
                    'algorithmic_bytes': v['bytes'], 'hbm_GBs': round(gbs, 1),
                    'hbm_frac': round(gbs / PEAK_HBM_GBS, 4),
                    'share_of_probe_ms': round(v['total_ms'] / sum(u['total_ms'] for u in kern.values()), 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--tmax', type=int, default=200)
    ap.add_argument('--tmin', type=int, default=50)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--kernels', action='store_true', help='print the per-kernel table to stderr')
    ap.add_argument('--model', choices=['forward_tacotron', 'fast_pitch', 'wavernn'],
                    default='forward_tacotron',
                    help='fast_pitch = BASELINE.json configs[4] (c5); wavernn = the vocoder (8(f))')
    ap.add_argument('--mel-frames', type=int, default=821, help='wavernn: mel length (c2: 821)')
    ap.add_argument('--config', choices=['c2', 'c3'], default=None,
                    help='c2 = BASELINE.json configs[1] (batch 1, 120 phonemes); c3 = the default')
    ap.add_argument('--callbacks', choices=['identity', 'gen_forward'], default='identity',
                    help='gen_forward: pitch_function = lambda x: x * amp, energy_function = '
                         'lambda x: x, as gen_forward.py:103-104 passes them')
    ap.add_argument('--amp', type=float, default=1.0, help='gen_forward.py --amp')
    ap.add_argument('--nnls', choices=['lbfgsb', 'fista'], default='lbfgsb',
                    help='the vocoder leg\'s mel pseudo-inverse: lbfgsb = the reference\'s util.nnls '
                         '(L-BFGS-B, its S), fista = the fast per-frame solver (another minimiser)')
    ap.add_argument('--vocoder-steps', type=int, default=0,
                    help='timed steps of the vocoder leg (0: --steps)')
    ap.add_argument('--vocoder', choices=['none', 'griffinlim'], default='none',
                    help='griffinlim: also time generate + Griffin-Lim per step (gen_forward.py)')
    ap.add_argument('--gather-overlap', choices=('auto', 'on', 'off'), default='auto',
                    help='N > 1: the rank-0 gather of step i in flight during step i + 1 (auto: '
                         'on with nccl; off in the gloo rehearsal, whose ranks share one GPU)')
    ap.add_argument('--no-host-loop', action='store_true',
                    help='skip the second (host-to-host, PCIe-inclusive) timed loop')
    args = ap.parse_args()
    if args.config == 'c2':
        args.batch, args.tmin, args.tmax = 1, 120, 120
    shape = (args.batch, args.tmin, args.tmax)
    pmc_path = {(64, 50, 200): PMC_PROFILE, (1, 120, 120): PMC_PROFILE_C2}.get(shape)
    pmc_tree = PMC_TREE_C2 if pmc_path == PMC_PROFILE_C2 else PMC_TREE

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # FTMI_BENCH_BACKEND=gloo: a rehearsal of the N > 1 path on fewer GPUs than ranks (ranks
    # share devices, collectives on host copies); the measured configuration is nccl (RCCL)
    backend = os.environ.get('FTMI_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)
    cdev = dev if backend == 'nccl' else torch.device('cpu')  # timing all-reduces
    if args.model == 'wavernn':
        bench_wavernn(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    cls = FastPitch if args.model == 'fast_pitch' else ForwardTacotron
    model = cls.from_config(default_config())
    sd = None
    if rank == 0:  # synthetic weights on rank 0; the other ranks receive them (RCCL broadcast)
        sd = synthetic_state_dict(model, seed=0, model=args.model)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dev).eval()
    bcast_timer = CollectiveTimer()
    ggroup = None
    if world > 1:
        broadcast_state(model, src=0, timer=bcast_timer)
        ggroup = dist.new_group()  # the result collection's own communicator (RCCL stream)
    x_np = synthetic_tokens(args.batch, args.tmax, seed=rank, min_len=args.tmin)
    x_host = torch.from_numpy(x_np)
    x = x_host.to(dev)

    if args.callbacks == 'gen_forward':  # gen_forward.py:103-104 (same objects every call)
        amp = args.amp
        # plain lambdas, exactly as the reference CLI passes them (not marked graph_safe):
        # generate() replays its split phoneme graph and runs them eagerly between
        cb = dict(pitch_function=lambda v: v * amp, energy_function=lambda v: v)
    else:
        cb = {}
    # auto: pipelined with RCCL (one rank per GPU).  In the gloo rehearsal the ranks share a
    # GPU and pipelining unlocks their step phase, so two processes' all-CU persistent
    # recurrences can meet on the one device (a spin timeout and compact rerun, seconds):
    # blocking there (tools/c4_overlap_diag.py)
    overlap = world > 1 and (args.gather_overlap == 'on'
                             or (args.gather_overlap == 'auto' and backend == 'nccl'))
    if world > 1:  # c4: one global batch sharded over the ranks (reference-identical result),
        # the result collected on rank 0 (SURVEY 8(e) "result collection")
        gen = lambda xx: generate_sharded(model, xx, gather='rank0', **cb)
        # timed loop: step i's rank-0 gather in flight on its own communicator while step
        # i + 1 runs; waited on after step i + 1 is issued
        gen_async = lambda xx: generate_sharded(model, xx, gather='rank0', gather_group=ggroup,
                                                async_gather=True, **cb)
    else:
        gen = lambda xx: model.generate(xx, **cb)
    for _ in range(args.warmup):
        gen(x)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    frames = 0
    out = None
    if overlap:  # the pipelined form once untimed (the gather communicator's first use)
        gen_async(x).wait()
        torch.cuda.synchronize()
    with KernelProbe() as probe:
        barrier()
        t0 = time.perf_counter()
        pending = None
        for _ in range(args.steps):
            if overlap:
                p = gen_async(x)
                o = pending.wait() if pending is not None else None
                pending = p
            else:
                o = gen(x)  # N > 1: rank 0 holds the global batch's result
            if o is not None:
                out = o
                frames += out['mel_post'].size(0) * out['mel_post'].size(2)
        if pending is not None:
            o = pending.wait()
            if o is not None:
                out = o
                frames += out['mel_post'].size(0) * out['mel_post'].size(2)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
    elapsed = t1 - t0
    kern = probe.summary()

    # c4: the communication share.  One more loop of `steps` calls with the blocking
    # rank-0 gather and every collective bracketed by HIP events (sharded.CollectiveTimer),
    # after the timed region; per-collective averages are maxed over ranks below.
    comm = None
    if world > 1:
        ctimer = CollectiveTimer()
        barrier()
        c0 = time.perf_counter()
        for _ in range(args.steps):
            generate_sharded(model, x, gather='rank0', timer=ctimer, **cb)
        torch.cuda.synchronize()
        barrier()
        comm = {'elapsed': time.perf_counter() - c0, 'per_call': ctimer.summary(),
                'broadcast': bcast_timer.summary()}

    # Second loop, PCIe-inclusive, as gen_forward.py:111-120 runs a call: token ids H2D,
    # generate(), mel_post D2H — through pinned buffers, the D2H stream-ordered on a side
    # stream (host_io.PinnedD2H) so it overlaps the next call's phoneme phase; every result
    # is on the host when the loop's clock stops.  Reported beside `value`, never as it.
    # A third loop times the serial form (pageable .cpu() per call, gen_forward.py:120).
    host_elapsed = host_serial = None
    if not args.no_host_loop:
        from forwardtacotron_amd.host_io import PinnedD2H
        d2h = PinnedD2H(dev)
        x_pin = x_host.pin_memory()
        # every slot of the pinned ring allocated untimed: a slot's first submit page-locks a
        # fresh 28 MB host buffer (c3), ~8 ms — inside the timed loop that one allocation was
        # the 5.5 % (20 steps) vs 17 % (5 steps) spread of this figure in round 4
        for _ in range(d2h.depth):
            o = gen(x_pin.to(dev, non_blocking=True))
            if o is not None:
                d2h.submit(o['mel_post'])
        d2h.synchronize()
        barrier()
        h0 = time.perf_counter()
        for _ in range(args.steps):
            o = gen(x_pin.to(dev, non_blocking=True))
            if o is not None:
                d2h.submit(o['mel_post'])
        d2h.synchronize()
        torch.cuda.synchronize()
        barrier()
        host_elapsed = time.perf_counter() - h0
        barrier()
        h0 = time.perf_counter()
        for _ in range(args.steps):
            o = gen(x_host.to(dev))
            if o is not None:
                o['mel_post'].cpu()
        torch.cuda.synchronize()
        barrier()
        host_serial = time.perf_counter() - h0
    # Third loop (--vocoder griffinlim): the whole gen_forward.py sentence step — generate,
    # mel_post.cpu(), DSP.griffinlim (HIP NNLS + 32 fast-GL iterations) -> numpy wav.
    voc = None
    if args.vocoder == 'griffinlim' and world == 1:
        from forwardtacotron_amd.dsp import DSP
        dsp = DSP.from_config(default_config())

        last = {}

        def vstep():
            o = gen(x_host.to(dev))
            m = o['mel_post']
            if m.size(0) == 1:  # as forwardtacotron_amd.gen_forward: D2H, GL from the device mel
                m.cpu()
                return dsp.griffinlim(m[0], nnls=args.nnls).cpu().numpy().shape[0]
            w, n = dsp.griffinlim_batch(m, nnls=args.nnls)
            last['wav'] = w
            w.cpu()
            return int(n.sum().item()) if torch.is_tensor(n) else int(np.sum(n))
        vstep()
        torch.cuda.synchronize()
        vsteps = args.vocoder_steps or args.steps
        v0 = time.perf_counter()
        nsamp = 0
        for _ in range(vsteps):
            nsamp += vstep()
        torch.cuda.synchronize()
        velapsed = time.perf_counter() - v0
        voc = {'name': 'griffinlim', 'nnls': args.nnls, 'steps': vsteps,
               'ms_per_step': round(velapsed / vsteps * 1e3, 3),
               'mel_frames_per_s': round(frames / args.steps * vsteps / velapsed, 1),
               'audio_samples_per_s': round(nsamp / velapsed, 1),
               'what': 'generate() + mel_post D2H + DSP.griffinlim (numpy wav out) per step, '
                       'as gen_forward.py:115-134 with the griffinlim vocoder (as forwardtacotron_'
                       'amd.gen_forward: the mel fetched to the host, Griffin-Lim started from the '
                       'device copy; the NNLS runs while the host draws the initial phases)'}
        # the HIP STFT kernels of that step (BASELINE configs[4] "+ HIP STFT", utils/dsp.py:71-103)
        # against the HBM roofline: one more step under the per-launch probe, and the analysis
        # direction (wav_to_mel: reflect pad, window, FFT, |.|, mel filterbank, log) of the
        # vocoded batch, HIP events over `reps` calls
        with KernelProbe() as vprobe:
            vstep()
            torch.cuda.synchronize()
        voc['kernels'] = dsp_kernel_table(vprobe.summary())
        # the vocoder leg's dominant audio kernel against the HBM roofline (the fused GL
        # iteration by default), with its PMC traffic from the committed passes of c5
        audio = {k: v for k, v in voc['kernels'].items()
                 if k.split('[')[0] in ('gl_iter', 'gl_stft', 'istft', 'istft_fused', 'mel_nnls',
                                        'nnls_lbfgsb', 'unit_phases', 'spec_mul')}
        if audio:
            lab, v = max(audio.items(), key=lambda kv: kv[1]['avg_ms'] * kv[1]['launches'])
            vr = {'kernel': lab, 'bound': 'hbm', 'achieved': v['hbm_GBs'], 'peak': PEAK_HBM_GBS,
                  'unit': 'GB/s', 'frac': v['hbm_frac'],
                  'algorithmic_per_launch': v['algorithmic_bytes'], 'avg_launch_ms': v['avg_ms'],
                  'launches': v['launches'], 'traffic': None,
                  'algorithmic_basis': ('gl_iter: 36 B per bin (X read + written as complex64, '
                                        'S read, tprev read + written)'
                                        if lab.startswith('gl_iter') else 'inputs + outputs once')}
            if lab.startswith('gl_iter') and args.model == 'fast_pitch' and shape == (64, 50, 200) \
                    and os.path.exists(PMC_PROFILE_C5):
                hit = json.load(open(PMC_PROFILE_C5))['kernels'].get('gl_fused_kernel<4, 32, false>')
                if hit:
                    vr['traffic'] = hit['hbm_bytes_per_launch']
                    vr['traffic_detail'] = {
                        'read_bytes_corrected': hit['read_bytes_corrected'],
                        'write_bytes': hit['write_bytes'],
                        'vs_algorithmic': round(hit['hbm_bytes_per_launch'] / v['algorithmic_bytes'], 3),
                        'source': os.path.relpath(PMC_PROFILE_C5, ROOT), 'measured_on_tree': PMC_TREE,
                        'note': 'a prior PMC run of this workload, not this run'}
            voc['roofline'] = vr
        if 'wav' in last:
            from forwardtacotron_amd.dsp import mel_spectrogram
            wav = last['wav'].contiguous()
            plan = dsp.plan(dev)
            with KernelProbe() as mprobe:
                for _ in range(10):
                    mel_spectrogram(plan, wav)
                torch.cuda.synchronize()
            voc['wav_to_mel'] = dsp_kernel_table(mprobe.summary())
            voc['wav_to_mel_what'] = (f'DSP.wav_to_mel of the vocoded batch: {wav.size(0)} rows x '
                                      f'{wav.size(1)} samples -> {plan.frames(wav.size(1))} frames '
                                      'each, one fused STFT + mel + log kernel')
    # The timed steps replay the phoneme phase as a HIP graph (forward_tacotron.GRAPH), whose
    # kernels the per-launch probe cannot see: one more generate() with the phase eager,
    # after the timed region, gives their per-kernel times (the prenet bank, --kernels).
    kern_all = kern
    from forwardtacotron_amd import fast_pitch as fp_module
    if (world == 1 and args.model == 'forward_tacotron' and ft_module.GRAPH
            and x.numel() <= ft_module.GRAPH_MAX_TOKENS):
        ft_module.GRAPH = False
        with KernelProbe() as probe_eager:
            gen(x)
            torch.cuda.synchronize()
        ft_module.GRAPH = True
        kern_all = probe_eager.summary()
    elif world == 1 and args.model == 'fast_pitch' and fp_module.FP_GRAPH:
        fp_module.FP_GRAPH = False
        with KernelProbe() as probe_eager:
            gen(x)
            torch.cuda.synchronize()
        fp_module.FP_GRAPH = True
        kern_all = probe_eager.summary()

    prenet_bank_ms = (time_prenet_bank(model, x) if world == 1 and args.model == 'forward_tacotron'
                      else None)

    if world > 1:
        rank_ms = torch.zeros(world, dtype=torch.float64, device=cdev)
        dist.all_gather_into_tensor(rank_ms, torch.tensor([elapsed / args.steps * 1e3],
                                                          dtype=torch.float64, device=cdev))
        names = ['shard_sizes all_gather', 'fill_rule all_reduce SUM', 't_mel all_reduce MAX',
                 'status all_reduce MAX', 'result gather to rank 0']
        pc = comm['per_call']
        vec = [pc.get(n, {}).get('avg_ms', 0.0) for n in names]
        vec += [pc.get(n, {}).get('total_ms', 0.0) / args.steps for n in names]
        bc = comm['broadcast'].get('weights broadcast', {'total_ms': 0.0, 'calls': 0})
        vec += [bc['total_ms'], comm['elapsed']]
        cv = torch.tensor(vec, dtype=torch.float64, device=cdev)
        dist.all_reduce(cv, op=dist.ReduceOp.MAX)
        cv = cv.tolist()
        nn = len(names)
        comm_line = {
            'per_collective': {n: {'calls_per_step': round(pc.get(n, {}).get('calls', 0) / args.steps, 2),
                                   'avg_ms': round(cv[i], 4), 'ms_per_step': round(cv[nn + i], 4)}
                               for i, n in enumerate(names)},
            'collective_ms_per_step': round(sum(cv[nn:2 * nn]), 4),
            'weights_broadcast_ms': round(cv[2 * nn], 3),
            'weights_broadcast_calls': bc['calls'],
            'ms_per_step_blocking_gather': round(cv[2 * nn + 1] / args.steps * 1e3, 3),
            'rank_ms_per_step': [round(v, 3) for v in rank_ms.tolist()],
            'gather_overlapped': overlap,
            'what': ('HIP events on the issuing stream around each blocking RCCL collective '
                     '(the interval includes the wait for the slowest peer), max over ranks, '
                     'from one extra loop of `steps` calls after the timed region with the '
                     'rank-0 gather blocking; ms_per_step_blocking_gather is that loop\'s '
                     'wall time (events included); rank_ms_per_step: each rank\'s timed loop '
                     '(ms_per_step is their max)'),
        }
        t = torch.tensor([elapsed, host_elapsed or 0.0, host_serial or 0.0], device=cdev,
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        host_elapsed = float(t[1].item()) if host_elapsed is not None else None
        host_serial = float(t[2].item()) if host_serial is not None else None

    if rank == 0:
        # dominant kernel = largest device time inside the timed region
        dom_label, dom = max(kern.items(), key=lambda kv: kv[1]['total_ms'])
        # device time per step over every kernel (the eager pass covers one step)
        total_dev_ms = sum(v['total_ms'] for v in kern_all.values()) / (
            1 if kern_all is not kern else args.steps)
        if args.kernels:
            tot_all = sum(v['total_ms'] for v in kern_all.values())
            log(f'{"kernel":60s} {"n":>4s} {"avg ms":>9s} {"share":>6s} {"TFLOP/s":>8s} {"GB/s":>8s}')
            for lab, v in sorted(kern_all.items(), key=lambda kv: -kv[1]['total_ms']):
                s = v['avg_ms'] / 1e3
                log(f'{lab:60s} {v["launches"]:4d} {v["avg_ms"]:9.3f} {v["total_ms"] / tot_all:6.1%} '
                    f'{v["flops"] / s / 1e12:8.2f} {v["bytes"] / s / 1e9:8.1f}')
        s = dom['avg_ms'] / 1e3
        if dom['flops'] > 0:
            achieved = dom['flops'] / s / 1e12
            if (rocprof_name(dom_label) or '').startswith('rnn_gemv_kernel'):
                peak, basis = PEAK_FP32_TFLOPS, ('fp32: at B <= 4 the recurrence is the exact-fp32 '
                                                 'GEMV kernel (VALU FMAs; rnn.hip gemv_path), '
                                                 'whatever mma the label requests')
            elif 'mma=2' in dom_label:
                peak, basis = PEAK_X3_TFLOPS, ('f16 dense MFMA 2.5 PF / 3 (fp32-level f16x3 split: 3 '
                                               'f16 products per fp32 product)')
            elif 'mma=1' in dom_label:
                peak, basis = PEAK_X6_TFLOPS, ('bf16 dense MFMA 2.5 PF / 6 (fp32-accurate bf16x6 '
                                               'split: 6 bf16 products per fp32 product)')
            else:
                peak, basis = PEAK_FP32_TFLOPS, 'fp32 dense MFMA'
            roof = {'kernel': dom_label, 'bound': 'mfma', 'achieved': round(achieved, 3),
                    'peak': round(peak, 1), 'unit': 'TFLOP/s',
                    'peak_basis': basis,
                    'frac': round(achieved / peak, 4),
                    'algorithmic_per_launch': dom['flops'], 'avg_launch_ms': round(dom['avg_ms'], 4),
                    'launches': dom['launches'], 'share_of_device_time': round(dom['total_ms'] / args.steps / total_dev_ms, 4),
                    'traffic': None}
            tr = (pmc_traffic(dom_label, pmc_path)
                  if pmc_path and args.model == 'forward_tacotron' and world == 1 else None)
            if tr is None and args.model == 'fast_pitch' and world == 1 and shape == (64, 50, 200):
                tr = pmc_traffic_slab(dom_label, PMC_PROFILE_C5)
            if tr is not None:
                roof['traffic'] = tr['bytes_per_launch']
                roof['traffic_detail'] = tr
            cfg = {(64, 50, 200): 'c3', (1, 120, 120): 'c2'}.get(shape) if args.model == 'forward_tacotron' \
                else ('c5' if shape == (64, 50, 200) else None)
            mb = pmc_mfma(dom_label, cfg) if cfg and world == 1 else None
            if mb is not None:
                roof['mfma_busy'] = mb['mfma_busy']
                roof['mfma_busy_detail'] = mb
        else:
            achieved = dom['bytes'] / s / 1e9
            roof = {'kernel': dom_label, 'bound': 'hbm', 'achieved': round(achieved, 1),
                    'peak': PEAK_HBM_GBS, 'unit': 'GB/s', 'frac': round(achieved / PEAK_HBM_GBS, 4),
                    'algorithmic_per_launch': dom['bytes'], 'avg_launch_ms': round(dom['avg_ms'], 4),
                    'launches': dom['launches'], 'traffic': None}

        # north-star kernel: the fused Conv1d+ReLU+BN prenet bank (K = 16), against HBM
        # (weight planes + input + output, once) and against the f16x3 MFMA ceiling
        pre = [(lab, v) for lab, v in kern_all.items() if lab.startswith('conv_bank[') and ',K=16,' in lab]
        prenet = None
        if pre:
            lab, v = pre[0]
            pb = prenet_bank_ms or {}
            ms = pb.get('warm', v['avg_ms'])
            s_ = ms / 1e3
            frac = lambda t: round(v['bytes'] / (t / 1e3) / 1e9 / PEAK_HBM_GBS, 4)  # noqa: E731
            prenet = {'kernel': lab, 'avg_launch_ms': round(ms, 4),
                      'hbm_achieved_GBs': round(v['bytes'] / s_ / 1e9, 1), 'hbm_peak_GBs': PEAK_HBM_GBS,
                      'hbm_frac': frac(ms),
                      'hbm_frac_basis': ('effective: algorithmic bytes (weight planes + input + output, '
                                         'once) / device time per call with the weight planes '
                                         'Infinity-Cache resident, as in a generate() loop'),
                      'algorithmic_bytes': v['bytes'],
                      'mfma_achieved_TFLOPs': round(v['flops'] / s_ / 1e12, 2),
                      'mfma_frac': round(v['flops'] / s_ / 1e12 / PEAK_X3_TFLOPS, 4),
                      'measured': ('HIP events around a HIP graph of 20 back-to-back calls of the '
                                   'bank as generate() issues it, after the timed steps, on the '
                                   'same embedded tokens (device time per call incl. kernel '
                                   'boundaries, no host issue cost)'
                                   if pb else 'HIP events, timed steps'),
                      'eager_single_call_ms': round(v['avg_ms'], 4)}
            if pb:
                prenet['host_issued_ms'] = round(pb['eager'], 4)
                prenet['cold_ms'] = round(pb['cold'], 4)
                prenet['hbm_frac_cold'] = frac(pb['cold'])
                prenet['cold_basis'] = ('each call behind a 512 MiB overwrite of another buffer '
                                        '(weights from HBM): graph [overwrite, call] minus graph '
                                        '[overwrite], per call')
                prenet['cold_read_ms'] = round(pb['cold_read'], 4)
                prenet['hbm_frac_cold_read'] = frac(pb['cold_read'])
                prenet['cold_read_basis'] = ('each call behind a 1 GiB streaming read of another '
                                             'buffer (weights evicted from L2 and the Infinity '
                                             'Cache by clean lines: from HBM, no dirty write-back '
                                             'competing): graph [read, call] minus graph [read], '
                                             'per call')
                prenet['weights_read'] = pb['weights']
                # PMC traffic of the bank kernel from the committed passes of this workload
                if pmc_path and os.path.exists(pmc_path) and pb['weights'] == 'stream-order image':
                    ks = json.load(open(pmc_path))['kernels']
                    # the mask-free single-sequence form (B = 1) when the PMC run has it, else
                    # the masked image kernel of earlier runs
                    hit = [ks[k_] for k_ in ('conv_bank_halves_kernel<8, 4, 0, 16, 16, true, true>',
                                             'conv_bank_halves_kernel<8, 4, 0, 16, 16, true>')
                           if k_ in ks][:1]
                    if len(hit) == 1:
                        prenet['traffic'] = hit[0]['hbm_bytes_per_launch']
                        prenet['traffic_detail'] = {
                            'read_bytes_corrected': hit[0]['read_bytes_corrected'],
                            'write_bytes': hit[0]['write_bytes'],
                            'vs_algorithmic': round(hit[0]['hbm_bytes_per_launch'] / v['bytes'], 3),
                            'what': 'FETCH_SIZE x 2 + WRITE_SIZE per launch (writes include the '
                                    'halves\' 4 MB exchange and the counters)',
                            'source': os.path.relpath(pmc_path, ROOT), 'measured_on_tree': pmc_tree,
                            'note': 'a prior PMC run of this workload, not this run'}
                if 'planes' in pb:
                    prenet['warm_ms_split_planes'] = round(pb['planes'], 4)
        value = frames / elapsed
        # valid frames: frames of the non-pad phonemes (the rest of B * T_mel is padding)
        tok = (x_np != 0) if world == 1 else None
        valid = None
        if tok is not None:
            cnt = ft_oracle_counts(out['dur'].float().cpu().numpy())
            valid = int((cnt * tok).sum())
        fp = args.model == 'fast_pitch'
        line = {
            'metric': 'mel-frames/sec at batch=64 LJSpeech shapes (%s.generate, B*T_mel per s)'
                      % ('FastPitch' if fp else 'ForwardTacotron'),
            'value': round(value, 1), 'unit': 'mel-frames/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
            'data': 'synthetic (seeded LJSpeech-shaped phoneme batches, synthetic weights)',
            'config': {'workload': (f'{"c5: FastPitch" if fp else ("c2" if args.batch == 1 else "c3") + ": ForwardTacotron"} generate, '
                                    if world == 1 else
                                    f'c4: {"FastPitch" if fp else "ForwardTacotron"} generate of one '
                                    f'global batch sharded over {world} GPUs (global padding, '
                                    f'fill rule and T_mel by RCCL all-reduce, the result gathered to '
                                    f'rank 0{" on its own communicator, pipelined with the next step" if overlap else ""}), ')
                                   + f'batch={args.batch} per GPU, '
                                   f'phoneme lengths U{{{args.tmin}..{args.tmax}}}',
                       'global_batch': args.batch * world, 'T_phonemes': int(x_np.shape[1]),
                       'T_mel': int(out['mel_post'].size(2)), 'parallelism': f'dp{world}'},
            'roofline': roof,
            'value_basis': ('tokens resident in HBM when the timed region starts, mel_post left in '
                            'HBM: the harness contract (PCIe-inclusive rates are never `value`); '
                            'SURVEY 8(d)\'s per-call figure with the token H2D and the mel_post '
                            'D2H is `host_to_host`'),
        }
        if valid is not None:
            line['valid_frames_per_step'] = valid
            line['valid_frames_per_s'] = round(valid * args.steps / elapsed, 1)
        if host_elapsed is not None:
            line['host_to_host'] = {
                'value': round(frames / host_elapsed, 1), 'unit': 'mel-frames/s',
                'ms_per_step': round(host_elapsed / args.steps * 1e3, 3),
                'vs_value': round(elapsed / host_elapsed, 4),
                'what': 'token ids H2D (pinned) + generate() + mel_post D2H per step into pinned '
                        'host buffers, the D2H stream-ordered on a side stream and overlapping the '
                        'next call (host_io.PinnedD2H); all results on the host at the clock stop '
                        '(PCIe-inclusive; `value` has the tokens resident in HBM)',
                'serial': {'value': round(frames / host_serial, 1),
                           'ms_per_step': round(host_serial / args.steps * 1e3, 3),
                           'what': 'pageable x.to(dev) + generate() + mel_post.cpu() per call, '
                                   'serialised as gen_forward.py:111-120 writes it'}}
        if args.callbacks != 'identity':
            line['config']['callbacks'] = (f'gen_forward.py:103-104: pitch_function = lambda x: x * {args.amp}, '
                                           'energy_function = lambda x: x')
        if prenet is not None:
            line['prenet_bank'] = prenet
        if world > 1:
            gb = sum(v.numel() * v.element_size() for k, v in out.items()
                     if not (k == 'mel_post' and v is out['mel']))
            comm_line['gather_bytes_per_step'] = int(gb)
            comm_line['gather_bytes_what'] = ('bytes rank 0 collects per step (mel, mel_post, dur, '
                                              'pitch, energy of the global batch)')
            line['collectives'] = comm_line
        if voc is not None:
            line['with_vocoder'] = voc
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'], line['parity'] = cpu_baseline(sd, x_np, out, args.model,
                                                                cb_kind=args.callbacks, amp=args.amp)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_wavernn(args, world, rank, dev):
    """The WaveRNN vocoder line (see the module docstring)."""
    from forwardtacotron_amd.wavernn import WaveRNN
    cfg = default_config()
    model = WaveRNN.from_config(cfg)
    sd = synthetic_state_dict(model, seed=0, model='wavernn')
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dev).eval()
    gcfg = cfg['vocoder']['generate']
    target, overlap = gcfg['target'], gcfg['overlap']
    rng = np.random.Generator(np.random.PCG64([rank, 321]))
    mels_np = (rng.normal(0.0, 1.0, (1, 80, args.mel_frames)) - 4.0).astype(np.float32)
    mels = torch.from_numpy(mels_np).to(dev)
    mu_law = cfg['dsp']['mu_law']
    gen = lambda seed: model.generate(mels, True, target, overlap, mu_law, seed=seed)
    for i in range(args.warmup):
        gen(1000 + i)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    samples = 0
    with KernelProbe() as probe:
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            wav = gen(i)
            samples += wav.shape[0]
        barrier()
        elapsed = time.perf_counter() - t0
    kern = probe.summary()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
    if rank != 0:
        return
    if args.kernels:
        for lab, v in sorted(kern.items(), key=lambda kv: -kv[1]['total_ms']):
            log(f'{lab:60s} {v["launches"]:4d} {v["avg_ms"]:9.3f}')
    dom_label, dom = max(kern.items(), key=lambda kv: kv[1]['total_ms'])
    s = dom['avg_ms'] / 1e3
    B = int(dom_label.split('B=')[1].split(',')[0])
    L = int(dom_label.split('L=')[1].split(',')[0])
    achieved = dom['flops'] / s / 1e12
    roof = {'kernel': dom_label, 'bound': 'mfma', 'achieved': round(achieved, 4),
            'peak': PEAK_FP32_TFLOPS, 'unit': 'TFLOP/s',
            'peak_basis': 'fp32 (the loop is exact fp32 FMAs on the VALU: the fp32 MFMA and vector '
                          'peaks are equal on gfx950); the loop is bound by its per-step all-to-all '
                          'hand-offs, not by either roof (DESIGN.md 5b)',
            'frac': round(achieved / PEAK_FP32_TFLOPS, 5),
            'algorithmic_per_launch': dom['flops'], 'avg_launch_ms': round(dom['avg_ms'], 3),
            'us_per_step': round(dom['avg_ms'] * 1e3 / L, 3), 'folds': B, 'steps_per_launch': L,
            'launches': dom['launches'],
            'share_of_device_time': round(dom['total_ms'] / sum(v['total_ms'] for v in kern.values()), 4),
            'traffic': None}
    line = {
        'metric': 'audio samples/s of WaveRNN.generate (gen_forward.py wavernn, batched folds)',
        'value': round(samples * world / elapsed, 1), 'unit': 'samples/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
        'data': 'synthetic (log-mel-like N(-4, 1) mels, synthetic WaveRNN weights)',
        'config': {'workload': f'WaveRNN vocoder: generate(mels (1, 80, {args.mel_frames}), batched=True, '
                               f'target={target}, overlap={overlap}, mu_law={mu_law}), RAW 9 bits',
                   'folds': B, 'steps': L, 'wave_len': int(wav.shape[0]),
                   'parallelism': f'replicas{world}' if world > 1 else 'single'},
        'roofline': roof,
        'realtime_factor': round(samples * world / elapsed / cfg['dsp']['sample_rate'], 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline_wavernn(sd, cfg, mels_np, target, overlap, B, L, samples,
                                                    args.steps)
    print(json.dumps(line), flush=True)


def cpu_baseline_wavernn(sd, cfg, mels_np, target, overlap, B, L, samples, steps):
    """The torch-CPU restatement of the reference vocoder (oracle/wr_torch_cpu.py, the
    reference's ATen kernels and its Categorical draws) on a bounded sample: the same 19
    folds for the first 300 steps (the sample loop dominates; scaled to the whole call's
    wave samples by steps / L)."""
    from oracle import wr_torch_cpu as wr
    n = min(300, L)
    sdt = wr.to_torch(sd)
    vcfg = dict(cfg['vocoder']['model'])
    info = _cpu_info()
    torch.set_num_threads(baseline_threads())
    threads = torch.get_num_threads()
    torch.manual_seed(0)
    t0 = time.perf_counter()
    wr.generate(sdt, vcfg, torch.from_numpy(mels_np), True, target, overlap, True, steps=n)
    dt = time.perf_counter() - t0
    per_call = dt * L / n  # the whole loop of one generate() call at that rate
    wave = samples / steps
    return {'value': round(wave / per_call, 1), 'unit': 'samples/s', 'cores': threads,
            'kind': 'port', 'cpu_model': info[0], 'physical_cores': info[1],
            'sample': f'{B} folds x first {n} of {L} steps of one generate() call '
                      f'({dt:.2f} s), scaled by {L}/{n}'}


def ft_oracle_counts(dur):
    from oracle import ft_oracle
    return ft_oracle.duration_counts(dur)


def _cpu_info():
    """(CPU model, physical cores of the host) for the cpu_baseline record."""
    model = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:  # pragma: no cover
        phys = None
    return model, phys


def _usable_cpus():
    """CPUs this process may run on: its affinity mask, capped by a cgroup CPU quota (the
    GPU box grants a share of the host: os.cpu_count() shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def baseline_threads():
    """BASELINE.md:48: torch.set_num_threads(<physical cores>) — capped by the CPUs the
    process is actually granted (oversubscribing a quota only slows the baseline down)."""
    _, phys = _cpu_info()
    return max(1, min(phys or 1, _usable_cpus()))


def cpu_baseline(sd, x_np, out, kind='forward_tacotron', cb_kind='identity', amp=1.0):
    """Time the torch-CPU restatement of the reference on the same batch (bounded: one call
    at the process's thread count), plus a 1-thread figure on a bounded sample of it."""
    from oracle import ft_oracle
    if kind == 'fast_pitch':
        from oracle import fp_torch_cpu as ft_torch_cpu
    else:
        from oracle import ft_torch_cpu
    cb = {}
    if cb_kind == 'gen_forward':  # gen_forward.py:103-104, plain lambdas
        cb = dict(pitch_function=lambda v: v * amp, energy_function=lambda v: v)
    sdt = ft_torch_cpu.to_torch(sd)
    xt = torch.from_numpy(x_np)
    threads_before = torch.get_num_threads()
    threads = baseline_threads()
    torch.set_num_threads(threads)
    ft_torch_cpu.generate(sdt, xt[:1, :20])  # warm the CPU kernels
    t0 = time.perf_counter()
    ref = ft_torch_cpu.generate(sdt, xt, **cb)
    dt = time.perf_counter() - t0
    frames = ref['mel_post'].size(0) * ref['mel_post'].size(2)
    # 1 thread, bounded: the first min(B, 8) utterances (about 5-10 s of CPU work)
    n1 = min(x_np.shape[0], 8)
    x1 = xt[:n1, :int((x_np[:n1] != 0).sum(1).max())]
    torch.set_num_threads(1)
    try:
        t0 = time.perf_counter()
        r1 = ft_torch_cpu.generate(sdt, x1, **cb)
        dt1 = time.perf_counter() - t0
    finally:
        torch.set_num_threads(threads_before)
    f1 = r1['mel_post'].size(0) * r1['mel_post'].size(2)
    got = out['mel_post'].float().cpu().numpy()
    r = ref['mel_post'].numpy()
    same_shape = got.shape == r.shape
    d = np.abs(got - r) if same_shape else None
    counts_equal = bool(np.array_equal(ft_oracle.duration_counts(out['dur'].cpu().numpy()),
                                       ft_oracle.duration_counts(ref['dur'].numpy())))
    cpu_model, phys = _cpu_info()
    base = {'value': round(frames / dt, 1), 'unit': 'mel-frames/s', 'cores': threads,
            'kind': 'port',
            'threads_used': threads, 'cpu_model': cpu_model, 'host_physical_cores': phys,
            'usable_cpus': _usable_cpus(), 'os_cpu_count': os.cpu_count(),
            'threads_rule': 'min(host physical cores, CPUs granted to the process: affinity '
                            'and cgroup quota) (BASELINE.md:48)',
            'value_1thread': round(f1 / dt1, 1),
            'sample': f'one generate() of the same batch ({x_np.shape[0]} x {x_np.shape[1]} phonemes, '
                      f'T_mel {r.shape[2]}) with oracle/{ft_torch_cpu.__name__.split(".")[-1]}.py '
                      f'(the reference\'s ATen CPU kernels) at {threads} threads, {dt:.2f} s; '
                      f'1 thread: the first {n1} utterances (T_mel {r1["mel_post"].size(2)}), {dt1:.2f} s'}
    parity = {'mel_post_mean_abs': float(d.mean()) if same_shape else None,
              'mel_post_max_abs': float(d.max()) if same_shape else None,
              'lr_counts_equal': counts_equal}
    return base, parity


if __name__ == '__main__':
    main()
