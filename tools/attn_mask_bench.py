"""c5 postnet self-attention (B = 64, T = 1400, 2 heads of 128) on the f16x3 kernel, with and
without a key_padding_mask (lengths U{1000..1400}), HIP events; parity of the masked output
against the fp32 kernel."""
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


torch.manual_seed(0)
B, T, H, hd = 64, 1400, 2, 128
qkv = torch.randn(B, T, 3 * H * hd, device='cuda')
lens = torch.randint(1000, T + 1, (B,), device='cuda')
mask = torch.arange(T, device='cuda')[None, :] >= lens[:, None]
t_nomask = timed(lambda: ops.attention(qkv, H, mma=2))
t_mask = timed(lambda: ops.attention(qkv, H, key_padding_mask=mask, mma=2))
err = (ops.attention(qkv, H, key_padding_mask=mask, mma=2)
       - ops.attention(qkv, H, key_padding_mask=mask, mma=0)).abs().max().item()
print(f'no mask {t_nomask * 1e3:7.1f} us | mask {t_mask * 1e3:7.1f} us | max|f16x3 - f32| {err:.2e}')
