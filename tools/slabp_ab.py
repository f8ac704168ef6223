"""A/B of the slab kernels on the model's slab shapes: the fragment-prefetch kernel
(FTMI_SLAB_PF=1) against the previous kernel (FTMI_SLAB_PF=0, warp-specialised form for
k > 1), HIP events over back-to-back launches, interleaved rounds in one process.
usage: python tools/slabp_ab.py [rounds [ENV v0 v1]]  (default FTMI_SLAB_PF 0 1)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

SHAPES = {  # name: (kind, B, T, Cin, N, k)
    'c5.pred_k1_n128': ('conv', 64, 200, 128, 128, 1),
    'c5.pred_k1_n384': ('conv', 64, 200, 128, 384, 1),
    'c5.ffn_conv1': ('conv', 64, 1400, 256, 1024, 9),
    'c3.post_proj1': ('conv', 64, 1368, 2048, 256, 3),
    'c3.pred_conv': ('conv', 64, 200, 256, 256, 5),
    'c3.lstm_in': ('conv', 64, 200, 512, 4096, 1),
    'c3.post_gru_in': ('conv', 64, 1368, 256, 1536, 1),
    'c3.pre_bank': ('bank', 64, 200, 256, 16),
    'c3.post_bank': ('bank', 64, 1368, 80, 8),
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    env, vals = (sys.argv[2], sys.argv[3:5]) if len(sys.argv) > 4 else ('FTMI_SLAB_PF', ['0', '1'])
    torch.manual_seed(0)
    fns = {}
    only = os.environ.get('SLABP_ONLY')  # comma-separated name prefixes
    for name, s in SHAPES.items():
        if only and not any(name.startswith(o) for o in only.split(',')):
            continue
        if s[0] == 'conv':
            _, B, T, Cin, N, k = s
            x = torch.randn(B, T, Cin, device='cuda')
            w = torch.randn(N, k * Cin, device='cuda') * 0.05
            w3 = ops.presplit_for(w, 2)
            fns[name] = (lambda x=x, w=w, w3=w3, k=k: ops.conv1d(x, w, k, k // 2, relu=True, w_split=w3),
                         2.0 * B * T * N * k * Cin)
        else:
            _, B, T, Cin, K = s
            x = torch.randn(B, T, Cin, device='cuda')
            w = torch.randn(256 * Cin * K * (K + 1) // 2, device='cuda') * 0.05
            sc = torch.ones(K * 256, device='cuda')
            sh = torch.zeros(K * 256, device='cuda')
            w3 = ops.split_bank_weights(w, K, Cin, 256)
            fns[name] = (lambda x=x, w=w, w3=w3, K=K, sc=sc, sh=sh: ops.conv_bank(
                x, w, K, 256, sc, sh, w_split=w3, pool=True, split_out=True),
                2.0 * B * T * 256 * Cin * K * (K + 1) / 2)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for _ in range(rounds):
        for name, (fn, flops) in fns.items():
            for pf in vals:
                os.environ[env] = pf
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                a.record()
                for _ in range(10):
                    fn()
                b.record()
                torch.cuda.synchronize()
                res.setdefault((name, pf), []).append(a.elapsed_time(b) / 10)
    for name, (_, flops) in fns.items():
        t0, t1 = min(res[(name, vals[0])]), min(res[(name, vals[1])])
        print(f'{name:16s} {env}={vals[0]} {t0 * 1e3:8.1f} us ({flops / t0 / 1e9:6.1f} TF/s) | ={vals[1]} '
              f'{t1 * 1e3:8.1f} us ({flops / t1 / 1e9:6.1f} TF/s) | {t0 / t1:.3f}x', flush=True)


if __name__ == '__main__':
    main()
