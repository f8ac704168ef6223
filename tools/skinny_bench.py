"""Few-row (B = 1, config c2) conv timings: the prenet bank and proj1 shapes on the skinny
kernel (2 or 1 channel chunks per block) and on the slab kernel, HIP events on torch's
stream.  usage: python tools/skinny_bench.py [skinnycpb=2 skinnycpb=1 slab]"""
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
    return a.elapsed_time(b) / reps


def main():
    rng = np.random.Generator(np.random.PCG64(0))
    B, T, C, K = 1, 120, 256, 16
    x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
    ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, C, C, 2)
    sc = torch.ones(K * C, device='cuda')
    sh = torch.zeros(K * C, device='cuda')
    bank_bytes = 4.0 * (B * T * C + C * C * K * (K + 1) / 2 + B * T * K * C)
    x1 = torch.from_numpy(rng.normal(0, 1, (B, T, K * C)).astype(np.float32)).cuda()
    w1 = pack_conv(torch.from_numpy(rng.normal(0, 0.01, (C, K * C, 3)).astype(np.float32))).cuda()
    w1s = ops.presplit_for(w1, 2)
    p1_bytes = 4.0 * (B * T * K * C + C * K * C * 3 + B * T * C)
    for name, env in [('skinny cpb=2', {'FTMI_GEMM_SKINNY': '1', 'FTMI_SKINNY_CPB': '2',
                                        'FTMI_BANK_BALANCED': '1'}),
                      ('unbalanced cpb=2', {'FTMI_GEMM_SKINNY': '1', 'FTMI_SKINNY_CPB': '2',
                                            'FTMI_BANK_BALANCED': '0'}),
                      ('skinny cpb=1', {'FTMI_GEMM_SKINNY': '1', 'FTMI_SKINNY_CPB': '1'}),
                      ('slab', {'FTMI_GEMM_SKINNY': '0'})]:
        if len(sys.argv) > 1 and name.replace(' ', '') not in sys.argv[1:]:
            continue
        os.environ.update(env)
        tb = timed(lambda: ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3))
        tp = timed(lambda: ops.conv1d(x1, w1, 3, 1, relu=True, maxpool=True, mma=2, w_split=w1s))
        print(f'{name:14s} bank {tb * 1e3:7.1f} us {bank_bytes / tb / 1e6:7.0f} GB/s | '
              f'proj1 {tp * 1e3:7.1f} us {p1_bytes / tp / 1e6:7.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
