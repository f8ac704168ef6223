"""Timing experiment: the slab kernel with (FTMI_SLAB_DIAG=8) and without the f16 split of
its activations while staging (raw bits stored: results invalid).  Sizes the gain of a
pre-split activation operand.  usage: python tools/slab_split_diag.py  (GPU box)"""
import json, os, subprocess, sys

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
from forwardtacotron_amd import ops
res = {}
def t(f):
    f(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(10): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / 10
for name, B, T, Cin, N, k in [("post.proj1", 64, 1368, 2048, 256, 3), ("pre.proj1", 64, 200, 4096, 256, 3),
                              ("post.gru_in", 64, 1368, 256, 1536, 1), ("lstm_in", 64, 200, 512, 4096, 1)]:
    x = torch.randn(B, T, Cin, device="cuda"); w = torch.randn(N, k * Cin, device="cuda") * 0.05
    w3 = ops.presplit_for(w, 2)
    res[name] = t(lambda: ops.conv1d(x, w, k, k // 2, relu=True, w_split=w3, mma=2))
for name, B, T, Cin, K in [("post.bank", 64, 1368, 80, 8), ("pre.bank", 64, 200, 256, 16)]:
    x = torch.randn(B, T, Cin, device="cuda")
    w = torch.randn(256 * Cin * K * (K + 1) // 2, device="cuda") * 0.05
    sc = torch.ones(K * 256, device="cuda"); sh = torch.zeros(K * 256, device="cuda")
    w3 = ops.split_bank_weights(w, K, Cin, 256)
    res[name] = t(lambda: ops.conv_bank(x, w, K, 256, sc, sh, w_split=w3))
print(json.dumps(res))
'''
for ws in ('1', '0'):
    for diag in (0, 8):
        r = subprocess.run([sys.executable, '-c', CHILD], capture_output=True, text=True, timeout=300,
                           env={**os.environ, 'FTMI_SLAB_DIAG': str(diag), 'FTMI_GEMM_SLAB_WS': ws})
        if r.returncode != 0:
            print('FAILED', r.stderr[-2000:]); sys.exit(1)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        print(f'ws={ws} diag={diag}: ' + '  '.join(f'{k} {v * 1e3:.0f}' for k, v in res.items()), flush=True)
