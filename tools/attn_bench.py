"""FastPitch self-attention timings at the c5 shapes, fp32 vs f16x3 kernels (HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for B, T, H, hd in [(64, 1400, 2, 128), (64, 200, 2, 128), (64, 200, 2, 64)]:
    qkv = torch.randn(B, T, 3 * H * hd, device='cuda')
    flops = 4.0 * B * H * T * T * hd
    line = f'B={B} T={T} H={H} hd={hd}:'
    outs = {}
    for m, pre in ((0, False), (2, False), (2, True)):
        ms = timed(lambda: ops.attention(qkv, H, mma=m, presplit=pre))
        outs[(m, pre)] = ops.attention(qkv, H, mma=m, presplit=pre)
        line += f'  mma={m}{"p" if pre else ""} {ms * 1e3:8.1f} us {flops / ms / 1e9:7.1f} TF/s'
    line += f'  max|f16x3 - f32| {float((outs[(0, False)] - outs[(2, True)]).abs().max()):.2e}'
    print(line, flush=True)
