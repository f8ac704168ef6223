"""c2 prenet bank (B = 1, T = 120, K = 16, Cin = Cout = 256) on each bank kernel: the
no-split conv_bank_cs_kernel (default), the channel-split skinny kernel + finish launch
(FTMI_BANK_CS=0), and the split kernel with the in-kernel last-arriver finish
(FTMI_BANK_LAST=1).  HIP events over back-to-back launches ('warm': the weight planes are
Infinity-Cache resident after the first launch, as in a generate() loop) and per launch
behind a 512 MiB overwrite ('cold').  Run under rocprofv3 --kernel-trace --stats for the
kernel durations.  usage: python tools/bank_cs_bench.py [T] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import pack_conv  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rng = np.random.Generator(np.random.PCG64(0))
    B, C, K = 1, 256, 16
    x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
    ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, C, C, 2)
    sc = torch.ones(K * C, device='cuda')
    sh = torch.zeros(K * C, device='cuda')
    nbytes = 4.0 * (B * T * C + C * C * K * (K + 1) / 2 + B * T * K * C)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device='cuda')
    ref = None
    for name, env in [('cs', {'FTMI_BANK_CS': '1', 'FTMI_BANK_LAST': '0'}),
                      ('split+finish', {'FTMI_BANK_CS': '0', 'FTMI_BANK_LAST': '0'}),
                      ('split+last', {'FTMI_BANK_CS': '0', 'FTMI_BANK_LAST': '1'})]:
        os.environ.update(env)
        fn = lambda: ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3)  # noqa: E731
        for _ in range(5):
            y = fn()
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        if ref is None:
            ref = got
        d = float(np.abs(got - ref).max())
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        warm = a.elapsed_time(b) / reps
        cold = 0.0
        for _ in range(10):
            flush.fill_(1)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            cold += a.elapsed_time(b) / 10
        print(f'{name:13s} T={T}: warm {warm * 1e3:6.1f} us ({nbytes / warm / 1e6:6.0f} GB/s, '
              f'{nbytes / warm / 1e6 / 8000:.1%} of HBM) | cold {cold * 1e3:6.1f} us '
              f'({nbytes / cold / 1e6:6.0f} GB/s) | max|d| vs cs {d:.2e}', flush=True)


if __name__ == '__main__':
    main()
