"""Interleaved A/B of the pooled f16x3 conv bank: the walking kernel (FTMI_BANK_WALK=1,
conv_bank_walk_kernel) against the slab kernel (FTMI_BANK_WALK=0), at the c3 postnet bank
(B 64 x T_mel 1368, Cin 80, K 8, 256 columns per group, pooled, split rows out) and any
other shape given.  HIP events around 20 back-to-back calls, 5 rounds, median per call.
usage: python tools/bank_walk_ab.py [B T Cin K] (GPU box)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

F16X3_PEAK = 2.5e15 / 3  # dense f16 MFMA / 3 products per fp32 product


def main():
    B, T, Cin, K = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (64, 1368, 80, 8)
    C = 256
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, T, Cin, generator=g).cuda()
    w = (torch.randn(C * Cin * K * (K + 1) // 2, generator=g) * 0.05).cuda()
    sc = torch.rand(K * C, generator=g).cuda() + 0.5
    sh = torch.randn(K * C, generator=g).cuda() * 0.1
    w3 = ops.split_bank_weights(w, K, Cin, C, 2)
    flops = 2.0 * B * T * C * Cin * K * (K + 1) / 2
    fn = lambda: ops.conv_bank(x, w, K, C, sc, sh, mma=2, w_split=w3, pool=True, split_out=True)
    res = {'1': [], '0': []}
    outs = {}
    for r in range(6):
        for v in ('1', '0'):
            os.environ['FTMI_BANK_WALK'] = v
            for _ in range(3):
                outs[v] = fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r:  # round 0 warms both
                res[v].append(e0.elapsed_time(e1) / 20)
    same = torch.equal(outs['1'].view(torch.int32), outs['0'].view(torch.int32))
    for v, name in (('1', 'walk'), ('0', 'slab')):
        ms = statistics.median(res[v])
        print(f'{name}: B={B} T={T} Cin={Cin} K={K}: {ms * 1e3:.1f} us per call '
              f'({flops / ms / 1e9:.1f} TFLOP/s = {flops / ms / 1e-3 / F16X3_PEAK:.3f} of the f16x3 '
              f'ceiling) runs {[round(t * 1e3, 1) for t in res[v]]}')
    print(f'bit-identical: {same}; status {int(ops.status_word(x.device).item())}')


if __name__ == '__main__':
    main()
