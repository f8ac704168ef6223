"""FastPitch postnet in_proj + attention at c5 (B = 64, T = 1400, d = 256, 2 heads): the
panel projection + attention with its K / V split pass against ftmi_panel_proj_qkv +
ftmi_attention_kv (split folded into the projection); HIP events, back to back, per stage.
usage: python tools/kv_fused_ab.py"""
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


B, T, d, H = 64, 1400, 256, 2
x = torch.randn(B, T, d, device='cuda')
wf = ops.split_weights_f16(torch.randn(3 * d, d, device='cuda') / 16, frag=True)
bias = torch.randn(3 * d, device='cuda') / 10
qkv = ops.panel_proj(x, wf, 3 * d, bias=bias)
q, kv = ops.panel_proj_qkv(x, wf, d, H, bias=bias)
for _ in range(2):
    print(f'panel_proj {timed(lambda: ops.panel_proj(x, wf, 3 * d, bias=bias)):7.1f} us | '
          f'attention(split pass) {timed(lambda: ops.attention(qkv, H, presplit=True)):7.1f} us | '
          f'panel_proj_qkv {timed(lambda: ops.panel_proj_qkv(x, wf, d, H, bias=bias)):7.1f} us | '
          f'attention_kv {timed(lambda: ops.attention_kv(q, kv, H)):7.1f} us', flush=True)
