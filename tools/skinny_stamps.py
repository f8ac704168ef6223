"""Phase timeline of the skinny (batch-1) GEMM kernel on the c2 prenet bank (diagnostic build).
usage: FTMI_LIB=forwardtacotron_amd/libftmi_stamps.so python tools/skinny_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import _lib, ops  # noqa: E402
from forwardtacotron_amd.common_layers import pack_conv  # noqa: E402

lib = _lib.load()
fn = lib.ftmi_debug_skinny_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
rng = np.random.Generator(np.random.PCG64(0))
B, T, C, K = 1, 120, 256, 16
x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
w3 = ops.split_bank_weights(wp, K, C, C, 2)
sc = torch.ones(K * C, device='cuda')
sh = torch.zeros(K * C, device='cuda')
flush = torch.empty(512 << 20, dtype=torch.uint8, device='cuda')
for cold in (False, True):
    for _ in range(3):
        if cold:
            flush.zero_()  # evict the weights from L2 / MALL
        ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3)
    torch.cuda.synchronize()
    n = 4096 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert fn(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.float64)
    used = a[:, 0] > 0
    a = a[used]
    t0 = a[:, 0].min()
    w0 = a[:, :4] - t0
    w7 = a[:, 4:8] - t0
    print(f'{"cold" if cold else "warm"}: {used.sum()} blocks; cycles from the first block start')
    for name, w in (('wave0', w0), ('wave7', w7)):
        print(f'  {name}: start {np.median(w[:, 0]):8.0f} (max {w[:, 0].max():7.0f})  '
              f'slab done {np.median(w[:, 1]):8.0f}  loop done {np.median(w[:, 2]):8.0f} '
              f'(max {w[:, 2].max():7.0f})  end {np.median(w[:, 3]):8.0f} (max {w[:, 3].max():7.0f})')
    d = w0[:, 2] - w0[:, 1]
    print(f'  wave0 loop cycles: median {np.median(d):.0f} min {d.min():.0f} max {d.max():.0f}')
