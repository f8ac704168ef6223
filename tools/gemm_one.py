"""Run one GEMM-family shape repeatedly (for rocprofv3 PMC passes).
usage: python tools/gemm_one.py <shape> [--pre] [--iters N]"""
import argparse, sys
sys.path.insert(0, '.')
import torch
from forwardtacotron_amd import ops

SHAPES = {  # name: (kind, B, T, Cin, N, k, maxpool)
    'post.proj1': ('conv', 64, 1368, 2048, 256, 3, True),
    'post.gru_in': ('conv', 64, 1368, 256, 1536, 1, False),
    'lstm_in': ('conv', 64, 200, 512, 4096, 1, False),
    'post.bank': ('bank', 64, 1368, 80, 8),
    'pre.proj1': ('conv', 64, 200, 4096, 256, 3, True),
    'pred.conv': ('conv', 64, 200, 256, 256, 5, False),
    'pre.bank': ('bank', 64, 200, 256, 16),
    'fp.conv1': ('conv', 64, 1400, 256, 1024, 9, False),
}
ap = argparse.ArgumentParser()
ap.add_argument('shape')
ap.add_argument('--pre', action='store_true')
ap.add_argument('--iters', type=int, default=10)
a = ap.parse_args()
s = SHAPES[a.shape]
torch.manual_seed(0)
if s[0] == 'conv':
    _, B, T, Cin, N, k, mp = s
    x = torch.randn(B, T, Cin, device='cuda')
    w = torch.randn(N, k * Cin, device='cuda') * 0.05
    w3 = ops.presplit_for(w) if a.pre else None
    fn = lambda: ops.conv1d(x, w, k, k // 2, relu=True, maxpool=mp, w_split=w3)
else:
    _, B, T, Cin, K = s
    x = torch.randn(B, T, Cin, device='cuda')
    w = torch.randn(256 * Cin * K * (K + 1) // 2, device='cuda') * 0.05
    sc = torch.ones(K * 256, device='cuda'); sh = torch.zeros(K * 256, device='cuda')
    w3 = ops.split_bank_weights(w, K, Cin, 256) if a.pre else None
    fn = lambda: ops.conv_bank(x, w, K, 256, sc, sh, w_split=w3)
for _ in range(a.iters):
    fn()
torch.cuda.synchronize()
print('done')
