"""Phase timeline of the one-launch channel-halves bank (conv_bank_halves_kernel) on the c2
prenet bank, in the diagnostic build (s_memtime stamps), for each FTMI_BANK_HALVES_DIAG
variant (0 = the real kernel; 1 no MFMAs, 2 no A-fragment LDS reads, 4 no partner exchange:
timing only, results invalid; 'img' = the real kernel on the stream-order weight image).
s_memtime counts per XCD, so every stamp is taken relative to its own block's start.
usage: FTMI_LIB=forwardtacotron_amd/libftmi_stamps.so python tools/bank_halves_stamps.py [diag ...]"""
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
img = ops.bank_halves_image(w3, K, C, C)
sc = torch.ones(K * C, device='cuda')
sh = torch.zeros(K * C, device='cuda')
names = ['start', 'slab', 'loop w0', 'loop w7', 'reduced', 'counted', 'end w0', 'end w7']
for diag in (sys.argv[1:] or ['0', '1', '2', '4']):
    # 'img' = the image kernel; 'img:<bits>' = its timing variant <bits>
    os.environ['FTMI_BANK_HALVES_DIAG'] = diag.split(':')[1] if ':' in diag else (
        '0' if diag == 'img' else diag)
    wi = img if diag.startswith('img') else None
    for _ in range(5):
        ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3, w_image=wi)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3, w_image=wi)
    b.record()
    torch.cuda.synchronize()
    n = 4096 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert fn(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8)[:256].astype(np.float64)
    rel = st - st[:, :1]
    print(f'diag {diag}: {a.elapsed_time(b) / 20 * 1e3:.1f} us per call (events, host-issued); '
          f'cycles from each block start, median (max) over 256 blocks:')
    print('   ' + '  '.join(f'{nm} {np.median(rel[:, i]):7.0f} ({rel[:, i].max():6.0f})'
                            for i, nm in enumerate(names)))
    if os.environ.get('SLOWEST'):
        # the slowest blocks: block id, XCD (b & 7), half, unit, the pair's heavy group, phases
        order = np.argsort(-rel[:, 6:8].max(1))[:int(os.environ['SLOWEST'])]
        for blk in order:
            h, u = (blk >> 3) & 1, (blk & 7) | ((blk >> 4) << 3)
            print(f'   block {blk:3d} xcd {blk & 7} half {h} unit {u:3d} gi {u // 16:2d}: ' +
                  ' '.join(f'{rel[blk, i]:6.0f}' for i in range(1, 8)))
        fast = np.argsort(rel[:, 6:8].max(1))[:3]
        for blk in fast:
            print(f'   fast  {blk:3d} xcd {blk & 7}: ' + ' '.join(f'{rel[blk, i]:6.0f}' for i in range(1, 8)))
        ends = rel[:, 6:8].max(1)
        for xc in range(8):
            # s_memtime is one counter per XCD: absolute stamps compare within an XCD
            s0, e0 = st[xc::8, 0], st[xc::8, 6:8].max(1)
            print(f'   xcd {xc}: median block {np.median(ends[xc::8]):6.0f} max {ends[xc::8].max():6.0f}'
                  f' | starts spread {s0.max() - s0.min():6.0f}, first start -> last end '
                  f'{e0.max() - s0.min():6.0f} cycles')
    d = rel[:, 2] - rel[:, 1]
    print(f'   wave-0 loop {np.median(d):.0f} cycles (min {d.min():.0f}, max {d.max():.0f}); '
          f'longest block {rel[:, 6:8].max():.0f} cycles', flush=True)
