"""Column-band tile order sweep of the slab kernels (FTMI_SLAB_BAND, gemm.hip slab_tile): HIP
graph of `reps` back-to-back launches per (shape, band), min of `rounds` interleaved rounds,
plus each band's max |d| against the first (the default) (tile order never changes a result: expect 0).
usage: python tools/band_sweep.py [rounds] [shape ...]   (shapes: tools/gemm_one.py SHAPES)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

SHAPES = {  # name: (kind, B, T, Cin, N, k, maxpool) / (bank, B, T, Cin, K)
    'lstm_in': ('conv', 64, 200, 512, 4096, 1, False),
    'post.gru_in': ('conv', 64, 1368, 256, 1536, 1, False),
    'post.proj1': ('conv', 64, 1368, 2048, 256, 3, True),
    'pre.proj1': ('conv', 64, 200, 4096, 256, 3, True),
    'pred.conv': ('conv', 64, 200, 256, 256, 5, False),
    'fp.conv1': ('conv', 64, 1400, 256, 1024, 9, False),
    'post.bank': ('bank', 64, 1368, 80, 8),
    'pre.bank': ('bank', 64, 200, 256, 16),
}
BANDS = ['default', 0, 1, 2, 4, 8, 16]  # default: FTMI_SLAB_BAND unset (2)


def make(name):
    s = SHAPES[name]
    g = torch.Generator(device='cuda').manual_seed(0)
    if s[0] == 'conv':
        _, B, T, Cin, N, k, mp = s
        x = torch.randn(B, T, Cin, device='cuda', generator=g)
        w = torch.randn(N, k * Cin, device='cuda', generator=g) * 0.05
        w3 = ops.presplit_for(w, 2)
        return lambda: ops.conv1d(x, w, k, k // 2, relu=True, maxpool=mp, w_split=w3, mma=2)[0]
    _, B, T, Cin, K = s
    x = torch.randn(B, T, Cin, device='cuda', generator=g)
    w = torch.randn(256 * Cin * K * (K + 1) // 2, device='cuda', generator=g) * 0.05
    sc, sh = torch.ones(K * 256, device='cuda'), torch.zeros(K * 256, device='cuda')
    w3 = ops.split_bank_weights(w, K, Cin, 256, 2)
    pool = ops.bank_pools(x, K, 256, 2, w3)
    return lambda: ops.conv_bank(x, w, K, 256, sc, sh, mma=2, w_split=w3, pool=pool,
                                 split_out=pool and ops.SPLIT_ROWS)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    names = sys.argv[2:] or list(SHAPES)
    reps = 5
    for name in names:
        fn = make(name)
        best, ref, dmax = {}, None, {}
        for _ in range(rounds):
            for band in BANDS:
                if band == 'default':
                    os.environ.pop('FTMI_SLAB_BAND', None)
                else:
                    os.environ['FTMI_SLAB_BAND'] = str(band)
                y = fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.clone()
                dmax[band] = float((y.float() - ref.float()).abs().max())
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for _ in range(reps):
                        fn()
                gr.replay()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                a.record()
                gr.replay()
                b.record()
                torch.cuda.synchronize()
                t = a.elapsed_time(b) / reps * 1e3
                best[band] = min(best.get(band, 1e30), t)
                del gr
        print(f'{name:12s} ' + '  '.join(f'{bd} {best[bd]:7.1f}' for bd in BANDS)
              + f'  us | max|d| {max(dmax.values()):.1e}', flush=True)
    os.environ.pop('FTMI_SLAB_BAND', None)


if __name__ == '__main__':
    main()
