"""Timing experiments on the slab GEMM kernel: FTMI_SLAB_DIAG bits (results invalid when
set): 1 = no per-step barrier, 2 = no MFMAs, 4 = no global loads in the main loop.
usage: python tools/slab_diag.py  (GPU box)"""
import json, os, subprocess, sys

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
from forwardtacotron_amd import ops
res = {}
for name, B, T, Cin, N, k, mp in [("post.proj1", 64, 1368, 2048, 256, 3, True),
                                  ("post.gru_in", 64, 1368, 256, 1536, 1, False),
                                  ("pre.proj1", 64, 200, 4096, 256, 3, True)]:
    x = torch.randn(B, T, Cin, device="cuda"); w = torch.randn(N, k * Cin, device="cuda") * 0.05
    w3 = ops.presplit_for(w, 2)
    f = lambda: ops.conv1d(x, w, k, k // 2, relu=True, maxpool=mp, w_split=w3, mma=2)
    f(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(5): f()
    e.record(); torch.cuda.synchronize()
    res[name] = s.elapsed_time(e) / 5
print(json.dumps(res))
'''
for diag in (0, 1, 2, 4, 3, 6, 7):
    r = subprocess.run([sys.executable, '-c', CHILD], env={**os.environ, 'FTMI_SLAB_DIAG': str(diag)},
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print('diag', diag, 'FAILED', r.stderr[-2000:]); sys.exit(1)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(f'diag={diag}: ' + '  '.join(f'{k} {v:.3f} ms' for k, v in res.items()), flush=True)
