"""Phase timeline of the fused Griffin-Lim iteration (gl_fused_kernel) from the diagnostic
build's s_memtime stamps (wave 0 of every workgroup), at c2 (B = 1, F = 816: 8-frame tiles)
and c5 (B = 64, F = 1400: 32-frame tiles).  s_memtime counts per XCD, so every stamp is taken
relative to its own workgroup's start; the launch-wide spread of the starts is printed too.
usage: FTMI_LIB=forwardtacotron_amd/libftmi_stamps.so python tools/gl_stamps.py [c2] [c5]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import _lib, dsp  # noqa: E402
from forwardtacotron_amd.synthetic import default_config  # noqa: E402

lib = _lib.load()
fn = lib.ftmi_debug_gl_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
D = dsp.DSP.from_config(default_config())
plan = D.plan(torch.device('cuda'))
names = ['setup', 'syn load', 'syn fft', 'syn+ola', 'wss div', 'ana fft0', 'ana fft', 'end']
for cfg in (sys.argv[1:] or ['c2', 'c5']):
    B, F = {'c2': (1, 816), 'c5': (64, 1400)}[cfg]
    rng = np.random.Generator(np.random.PCG64(0))
    S = torch.from_numpy(rng.random((B, F, 513), dtype=np.float32)).cuda()
    ph = rng.random((B, F, 513)) * 2 * np.pi
    X = torch.from_numpy(np.exp(1j * ph).astype(np.complex64)).cuda() * S
    X2, tprev = torch.empty_like(X), torch.zeros_like(X)

    def it(first):
        rc = lib.ftmi_griffinlim_iter(X.data_ptr(), X2.data_ptr(), S.data_ptr(), tprev.data_ptr(),
                                      B, F, None, 1024, 256, plan.window.data_ptr(),
                                      plan.win_sq.data_ptr(), plan.twiddle.data_ptr(),
                                      ctypes.c_float(0.99 / 1.99), int(first), dsp._stream())
        assert rc == 0, rc
    for i in range(5):
        it(i == 0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        it(False)
    b.record()
    torch.cuda.synchronize()
    nblk = B * ((F + 31) // 32 if B * ((F + 31) // 32) >= 256 else (F + 7) // 8)
    n = 4096 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert fn(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8)[:min(nblk, 4096)].astype(np.float64)
    st = st[st[:, 7] > 0]  # the workgroups that ran (a grid-stride grid is <= the tiles)
    rel = st - st[:, :1]
    print(f'{cfg}: B={B} F={F} {nblk} workgroups, {a.elapsed_time(b) / 20 * 1e3:.1f} us per '
          f'iteration (events, 20 back to back); cycles from each workgroup start, median (max):')
    print('   ' + '  '.join(f'{nm} {np.median(rel[:, i]):7.0f} ({rel[:, i].max():6.0f})'
                            for i, nm in enumerate(names)))
    # start spread per XCD (blocks are dealt round-robin: XCD = block & 7)
    for x in range(min(8, nblk)):
        s0 = st[x::8, 0]
        e = st[x::8, 7]
        print(f'   xcd {x}: {len(s0)} wgs, starts span {s0.max() - s0.min():8.0f}, '
              f'first start -> last end {e.max() - s0.min():8.0f} cycles')
