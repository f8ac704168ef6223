"""A/B of the c2 prenet bank's mask-free single-sequence form (conv_bank_halves_kernel<...,
NM = true>, the product path at B = 1) against the masked form (FTMI_BANK_HALVES_DIAG=2048,
any unused value: the masked kernel), in the diagnostic library: outputs must be
bit-identical, and each form is timed as a HIP graph of 20 back-to-back calls, warm, over
interleaved rounds.
usage: FTMI_LIB=forwardtacotron_amd/libftmi_stamps.so python tools/bank_nomask_ab.py [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import pack_conv  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rng = np.random.Generator(np.random.PCG64(0))
B, T, C, K = 1, 120, 256, 16
x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
w3 = ops.split_bank_weights(wp, K, C, C, 2)
img = ops.bank_halves_image(w3, K, C, C)
sc = torch.from_numpy(rng.uniform(0.5, 1.5, K * C).astype(np.float32)).cuda()
sh = torch.from_numpy(rng.normal(0, 0.1, K * C).astype(np.float32)).cuda()


def call():
    return ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3, w_image=img)


forms = {'mask-free': '0', 'masked': '2048'}
outs, graphs = {}, {}
for name, diag in forms.items():
    os.environ['FTMI_BANK_HALVES_DIAG'] = diag
    for _ in range(3):
        y = call()
    torch.cuda.synchronize()
    outs[name] = y.cpu().numpy()
    g = torch.cuda.CUDAGraph()  # the launch reads the switch at capture
    with torch.cuda.graph(g):
        for _ in range(20):
            call()
    g.replay()
    graphs[name] = g
same = np.array_equal(outs['mask-free'], outs['masked'])
print(f'bit-identical: {same} (max |d| {np.abs(outs["mask-free"] - outs["masked"]).max():.3g})')
res = {n: [] for n in forms}
for r in range(rounds):
    for n, g in graphs.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        res[n].append(a.elapsed_time(b) / 20 * 1e3)
for n, v in res.items():
    print(f'{n:10s} us per call (graph of 20, warm): ' + ' '.join(f'{t:.2f}' for t in v))
sys.exit(0 if same else 1)
