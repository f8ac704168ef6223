"""A/B of the transposed f16x3 attention kernel (FTMI_ATTN_T=1, default) against
attention_h3_kernel (FTMI_ATTN_T=0) on the c5 postnet shape (B = 64, T = 1400, 2 heads of 128,
lengths 1000..1400 in the masked run) through ftmi_attention_kv: HIP events, 20 calls back to
back, interleaved rounds, min.  usage: python tools/attn_t_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

B, T, H, d = 64, 1400, 2, 256
torch.manual_seed(0)
qkv = torch.randn(B, T, 3 * d, device='cuda')
lens = torch.randint(1000, T + 1, (B,), device='cuda')
mask = torch.arange(T, device='cuda')[None, :] >= lens[:, None]


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


res = {}
for _ in range(3):
    for m in (None, mask):
        for v in ('0', '1'):
            os.environ['FTMI_ATTN_T'] = v
            res.setdefault((m is not None, v), []).append(
                timed(lambda: ops.attention(qkv, H, m, mma=2, presplit=True)))
for masked in (False, True):
    t0, t1 = min(res[(masked, '0')]), min(res[(masked, '1')])
    print(f'attention (split pass incl.) mask={masked}: h3 {t0:7.1f} us  t3 {t1:7.1f} us  '
          f'{t0 / t1:.3f}x', flush=True)
