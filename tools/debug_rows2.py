"""Dump the h exchange buffer of the row-owning recurrence after a 2-step GRU (H = 64)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import _lib, ops  # noqa: E402

lib = _lib.load()
lib.ftmi_set_rnn_spin_limit(2000)
H, B, T = 64, 3, 2
G = 3
rng = np.random.default_rng(0)
xp = torch.from_numpy(rng.normal(0, 1, (B, T, 2 * G * H)).astype(np.float32)).cuda()
w_hh = torch.from_numpy(rng.normal(0, 0.1, (2, G * H, H)).astype(np.float32)).cuda()
b_hh = torch.zeros(2 * G * H, device='cuda')
need = int(lib.ftmi_rnn_workspace_bytes(B, H, 0)) // 4 + 4
ws = torch.zeros(need, device='cuda', dtype=torch.int32)
st = ops.status_word('cuda'); st.zero_()
y = ops.rnn_bidir(0, xp, H, w_hh, b_hh, ws=ws)
torch.cuda.synchronize()
print('status', int(st.item()))
nchunks = 1
ctl = (10 * 32 + 2 * nchunks * 64 + 2 * nchunks * 32) * 4
w = ws.cpu().numpy().view(np.uint32)
print('err word', w[0], 'census', [w[32 * (1 + i)] for i in range(8)], 'arrive', w[9 * 32])
hx = w[ctl // 4:].view(np.uint16)
per_group = 16 * H * 2  # halves
for par in range(2):
    for g in range(2):
        base = (par * 2 + g) * per_group
        blk = hx[base:base + per_group].reshape(2 * H // 32, 64, 8)  # chunk, lane, half
        tags = blk & 1
        nz = (blk != 0).sum()
        print(f'parity {par} group {g}: nonzero halves {nz}/{blk.size}, tag1 {int(tags.sum())}')
        for c in range(blk.shape[0]):
            print('   chunk', c, 'tag1 per lane-group', [int(tags[c, 16 * q:16 * q + 16].sum()) for q in range(4)])
