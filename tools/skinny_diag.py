"""What binds the c2 prenet bank (skinny kernel, balanced bank schedule): the bank call
(kernel + finish) timed with FTMI_SKINNY_DIAG variants of the kernel (results invalid):
1 = no LDS A-fragment reads in the weight loop, 2 = no MFMAs, 3 = neither, 4 = L2-hot
weight loads, 7 = none of the three.  The finish kernel is the same in every variant, so
differences are the main kernel's.  usage (GPU box): python tools/skinny_diag.py [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import pack_conv  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rng = np.random.Generator(np.random.PCG64(0))
    B, T, C, K = 1, 120, 256, 16
    x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
    ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, C, C, 2)
    sc = torch.ones(K * C, device='cuda')
    sh = torch.zeros(K * C, device='cuda')
    wbytes = 4.0 * C * C * K * (K + 1) / 2
    diags = sys.argv[2].split(',') if len(sys.argv) > 2 else ['0', '1', '2', '3', '4', '7']
    for _ in range(rounds):
        for qb, last in (('0', '1'), ('0', '0'), ('1', '1'), ('1', '0')):
            os.environ['FTMI_BANK_QB'] = qb
            os.environ['FTMI_BANK_LAST'] = last
            os.environ['FTMI_SKINNY_DIAG'] = '0'
            t = timed(lambda: ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3))
            print(f'FTMI_BANK_QB={qb} FTMI_BANK_LAST={last}: bank+finish {t:6.1f} us  '
                  f'({wbytes / t / 1e3:6.0f} GB/s of weights)', flush=True)
        os.environ['FTMI_BANK_LAST'] = '0'
        os.environ['FTMI_BANK_QB'] = '0'
        for d in diags:
            if d == '0':
                continue
            os.environ['FTMI_SKINNY_DIAG'] = d
            t = timed(lambda: ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3))
            print(f'diag {d} (pairs kernel): bank+finish {t:6.1f} us', flush=True)
    os.environ['FTMI_SKINNY_DIAG'] = '0'
    os.environ.pop('FTMI_BANK_QB')


if __name__ == '__main__':
    main()
