"""Short-sequence attention (the phoneme side, T = 200, B = 64): attention_h3_kernel and the
transposed kernel (FTMI_ATTN_T), each with the in-kernel split and with the split pass,
for hd 64 (2 heads of 64 at d = 128) and hd 128 (2 heads at d = 256); HIP events, 20 calls,
interleaved rounds, min.  usage: python tools/attn_short_ab.py [T ...]"""
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
    return a.elapsed_time(b) / reps * 1e3


torch.manual_seed(0)
for T in ([int(a) for a in sys.argv[1:]] or (200, 300, 400)):
    for d in (128, 256):
        qkv = torch.randn(64, T, 3 * d, device='cuda')
        lens = torch.randint(T // 2, T + 1, (64,), device='cuda')
        mask = torch.arange(T, device='cuda')[None, :] >= lens[:, None]
        res = {}
        for _ in range(3):
            for at in ('0', '1'):
                os.environ['FTMI_ATTN_T'] = at
                for pre in (False, True):
                    res.setdefault((at, pre), []).append(
                        timed(lambda: ops.attention(qkv, 2, mask, mma=2, presplit=pre)))
        print(f'T={T} hd={d // 2}: ' + '  '.join(
            f'{"t3" if at == "1" else "h3"}{"+split" if pre else ""} {min(v):6.1f}'
            for (at, pre), v in res.items()) + ' us', flush=True)
