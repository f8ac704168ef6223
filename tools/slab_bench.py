"""The f16x3 slab GEMM kernel at the c3 shapes (us per call, HIP events over 20 calls):
postnet bank / proj1 / proj2 / GRU projection, prenet bank / proj1, predictor conv, LSTM
input projection.  FTMI_SLAB_DIAG experiments change the timing (results invalid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def conv_case(name, B, T, Cin, N, k, maxpool=False, residual=False):
    x = torch.randn(B, T, Cin, device='cuda')
    w = torch.randn(N, k * Cin, device='cuda') / (k * Cin) ** 0.5
    w3 = ops.split_weights_f16(w)
    res = torch.randn(B, T, N, device='cuda') if residual else None
    sc, sh = torch.ones(N, device='cuda'), torch.zeros(N, device='cuda')
    t = timeit(lambda: ops.conv1d(x, w, k, k // 2, relu=True, bn=(sc, sh), maxpool=maxpool,
                                  residual=res, w_split=w3))
    fl = 2.0 * B * T * N * k * Cin
    print(f'{name:16s} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s', flush=True)


def bank_case(name, B, T, Cin, K, C=256):
    x = torch.randn(B, T, Cin, device='cuda')
    w = torch.cat([torch.randn(C * Cin * k, device='cuda') / (k * Cin) ** 0.5 for k in range(1, K + 1)])
    w3 = ops.split_bank_weights(w, K, Cin, C)
    sc, sh = torch.ones(K * C, device='cuda'), torch.zeros(K * C, device='cuda')
    t = timeit(lambda: ops.conv_bank(x, w, K, C, sc, sh, w_split=w3))
    fl = 2.0 * B * T * C * Cin * K * (K + 1) / 2
    print(f'{name:16s} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s', flush=True)


bank_case('post bank K8', 64, 1368, 80, 8)
conv_case('post proj1', 64, 1368, 2048, 256, 3, maxpool=True)
conv_case('post proj2', 64, 1368, 256, 80, 3, residual=True)
conv_case('post gru proj', 64, 1368, 256, 1536, 1)
bank_case('pre bank K16', 64, 200, 256, 16)
conv_case('pre proj1', 64, 200, 4096, 256, 3, maxpool=True)
conv_case('pred conv k5', 64, 200, 256, 256, 5)
conv_case('lstm proj', 64, 200, 512, 4096, 1)
