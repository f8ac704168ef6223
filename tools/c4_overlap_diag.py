"""Where a c4 step's time goes, pipelined vs blocking rank-0 gather (one line per rank).

    FTMI_BENCH_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29513 tools/c4_overlap_diag.py

Per step: host time of generate_sharded's issue, of the previous step's wait(), and the
status-word reruns (compact recurrences) the step took."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd import sharded as S  # noqa: E402
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402
from forwardtacotron_amd.synthetic import default_config, load_synthetic, synthetic_tokens  # noqa: E402


def main():
    rank = int(os.environ['RANK'])
    backend = os.environ.get('FTMI_BENCH_BACKEND', 'nccl')
    local = int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group(backend)
    gg = dist.new_group()
    m = load_synthetic(ForwardTacotron.from_config(default_config()), 0).to(dev).eval()
    x = torch.from_numpy(synthetic_tokens(64, 200, seed=rank, min_len=50)).to(dev)
    reruns = [0]
    orig = ops.compact_recurrences

    def counting():
        reruns[0] += 1
        return orig()
    ops.compact_recurrences = counting
    for _ in range(2):
        S.generate_sharded(m, x, gather='rank0')
        S.generate_sharded(m, x, gather='rank0', gather_group=gg, async_gather=True).wait()
    torch.cuda.synchronize()
    for mode in ('blocking', 'pipelined', 'blocking', 'pipelined'):
        dist.barrier()
        reruns[0] = 0
        issue, waits = [], []
        t0 = time.perf_counter()
        pending = None
        for _ in range(5):
            a = time.perf_counter()
            if mode == 'blocking':
                S.generate_sharded(m, x, gather='rank0')
                issue.append(time.perf_counter() - a)
                continue
            p = S.generate_sharded(m, x, gather='rank0', gather_group=gg, async_gather=True)
            b = time.perf_counter()
            issue.append(b - a)
            if pending is not None:
                pending.wait()
            waits.append(time.perf_counter() - b)
            pending = p
        if pending is not None:
            pending.wait()
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) / 5
        print(f'rank {rank} {mode:9s} {tot * 1e3:8.2f} ms/step  issue '
              f'{[round(v * 1e3, 1) for v in issue]}  wait {[round(v * 1e3, 1) for v in waits]}  '
              f'compact reruns {reruns[0]}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
