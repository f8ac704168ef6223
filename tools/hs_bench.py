"""Fused highway stack (ftmi_highway_stack) vs the unfused chain it replaces, at the
BASELINE shapes: c3 postnet (M = 64 x 1368, Cp = 80), c3 prenet (M = 64 x 200, Cp = 256),
c2 postnet / prenet (M = 816 / 120).  Prints us per call (HIP events, 50 calls).
usage: python tools/hs_bench.py [ncases [rows-per-workgroup ...]]  (FTMI_HS_BM A/B, fused only)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import CBHG  # noqa: E402


def timeit(fn, n=50):
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


CASES = [('c3 postnet', 64 * 1368, 80), ('c3 prenet', 64 * 200, 256),
         ('c2 postnet', 816, 80), ('c2 prenet', 120, 256)]
if len(sys.argv) > 1:  # fused only, the first argv[1] cases
    CASES = CASES[:int(sys.argv[1])]
for name, M, Cp in CASES:
    m = CBHG(K=2, in_channels=Cp, channels=256, proj_channels=[256, Cp], num_highways=4).cuda()
    w_pre, pre3 = m.packed_weights()[3], m.packed_weights()[5]
    hws = [hw.packed_weights() for hw in m.highways]
    w_ih, b_in, _, _, w3 = m.rnn.packed_weights()
    x = torch.randn(1, M, Cp, device='cuda')
    def fused():
        pre_f, hw_f, b1s, b2s, ih_f, b, n = m._stack_pack()
        ops.highway_stack(x, pre_f, 256, hw_f, b1s, b2s, ih_f, b, n)

    def unfused():
        h, _ = ops.conv1d(x, w_pre, 1, 0, w_split=pre3)
        for w12, b1, b2, s3 in hws:
            h = ops.highway(h, w12, b1, b2, w_split=s3)
        ops.conv1d(h, w_ih, 1, 0, bias=b_in, w_split=w3)

    if len(sys.argv) > 2:  # fused, per FTMI_HS_BM setting, interleaved rounds, min
        res = {}
        for _ in range(3):
            for bm in sys.argv[2:]:
                os.environ['FTMI_HS_BM'] = bm
                res.setdefault(bm, []).append(timeit(fused))
        os.environ.pop('FTMI_HS_BM')
        print(f'{name:11s} M={M:6d}: ' + '  '.join(f'bm={bm} {min(v):8.1f} us' for bm, v in res.items()),
              flush=True)
        continue
    tf = timeit(fused)
    tu = timeit(unfused) if len(sys.argv) == 1 else float('nan')
    fl = 2.0 * M * 256 * (Cp + 4 * 512 + 1536)
    print(f'{name:11s} M={M:6d}: fused {tf:8.1f} us ({fl / tf / 1e6:6.1f} TF/s)  '
          f'unfused {tu:8.1f} us  ({tu / tf:.2f}x)', flush=True)
