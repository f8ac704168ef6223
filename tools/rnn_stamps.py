"""Per-phase cycle breakdown of the persistent recurrence (diagnostic build).
Each phase ends in a stamp that first waits for the wave's outstanding memory operations
(s_waitcnt vmcnt(0) lgkmcnt(0)), so the build runs slower than the real kernel: the phase
split is the evidence, the real step time comes from tools/rnn_diag.py.
usage: FTMI_LIB=forwardtacotron_amd/libftmi_stamps.so python tools/rnn_stamps.py"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from forwardtacotron_amd import ops, _lib

lib = _lib.load()
fn = lib.ftmi_debug_rnn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
PH = ['xp issue', 'poll wait', 'h load', 'mfma+lds', 'cell+store', 'drain+arrive']
for cell, H, B, T in [(1, 512, 64, 1368), (0, 256, 64, 1368), (0, 128, 64, 200), (0, 64, 64, 200),
                      (1, 512, 1, 816)]:
    G = 4 if cell else 3
    xp = torch.randn(B, T, 2 * G * H, device='cuda') * 0.5
    w = torch.randn(2, G * H, H, device='cuda') / H ** 0.5
    bh = torch.randn(2 * G * H, device='cuda') * 0.1
    # the decoder LSTM and the postnet GRU run spread in the model (forward_tacotron.py)
    sp = T > 800 and B > 4 and ((cell == 1 and H == 512) or (cell == 0 and H == 256))
    for _ in range(2):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, check=True, spread=sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, check=True, spread=sp)
    dt = time.perf_counter() - t0
    nb = ops.rnn_blocks(cell, B, H) if not sp else ops.rnn_blocks(cell, B, H, 2 | ops.RNN_SPREAD)
    buf = (ctypes.c_ulonglong * (nb * 8))()
    assert fn(buf, nb * 8) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8)[:, :6].astype(np.float64)
    used = a.sum(1) > 0
    a = a[used] / T
    print(f'{"lstm" if cell else "gru"} H={H} B={B} T={T}: {dt*1e3:.2f} ms wall ({dt/T*1e6:.2f} us/step), '
          f'{used.sum()} blocks; cycles/step (mean over blocks, max):')
    for i, n in enumerate(PH):
        print(f'   {n:14s} {a[:, i].mean():9.0f} {a[:, i].max():9.0f}')
    print(f'   {"total":14s} {a.sum(1).mean():9.0f}')
