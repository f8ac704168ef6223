"""One attention shape (postnet c5: B=64, T=1400, H=2, hd=128), f16x3, a few launches —
for rocprofv3 PMC passes (tools/attn_pmc.sh).  argv[1]: presplit 0/1."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

pre = len(sys.argv) > 1 and sys.argv[1] == '1'
qkv = torch.randn(64, 1400, 3 * 256, device='cuda')
for _ in range(4):
    ops.attention(qkv, 2, mma=2, presplit=pre)
torch.cuda.synchronize()
print('done')
