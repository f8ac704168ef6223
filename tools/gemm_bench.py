"""Time the GEMM-family kernels on the c3 shapes for each matrix path / kernel variant (one
child process per variant) and report each result's error against a torch fp32 conv.
usage: python tools/gemm_bench.py [variant ...]   (variants: f32 x6b h3 slab)"""
import json, os, subprocess, sys

CHILD = r'''
import sys, json, os, torch
import torch.nn.functional as F
sys.path.insert(0, ".")
PRE = os.environ.get("PRE") == "1"
from forwardtacotron_amd import ops
torch.manual_seed(0)
def t(fn, n=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n
res = {}
def rel(y, ref):
    return float((y - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
def conv(name, B, T, Cin, N, k, maxpool=False):
    x = torch.randn(B, T, Cin, device="cuda"); w = torch.randn(N, k * Cin, device="cuda") * 0.05
    w3 = ops.presplit_for(w) if PRE else None
    f = lambda: ops.conv1d(x, w, k, k // 2, relu=True, maxpool=maxpool, w_split=w3)
    ms = t(f)
    y = f()[0]
    xi = x
    if maxpool:
        xi = torch.maximum(x, torch.cat([x[:, :1], x[:, :-1]], 1))
    W = w.view(N, k, Cin).permute(0, 2, 1)
    ref = F.relu(F.conv1d(xi.transpose(1, 2), W, padding=k // 2)).transpose(1, 2)
    res[name] = (ms, 2.0 * B * T * N * k * Cin / ms / 1e9, rel(y, ref))
def bank(name, B, T, Cin, K):
    x = torch.randn(B, T, Cin, device="cuda"); w = torch.randn(256 * Cin * K * (K + 1) // 2, device="cuda") * 0.05
    sc = torch.ones(K * 256, device="cuda"); sh = torch.zeros(K * 256, device="cuda")
    w3 = ops.split_bank_weights(w, K, Cin, 256) if PRE else None
    ms = t(lambda: ops.conv_bank(x, w, K, 256, sc, sh, w_split=w3))
    res[name] = (ms, 2.0 * B * T * 256 * Cin * K * (K + 1) / 2 / ms / 1e9, 0.0)
def hw(name, M, C):
    x = torch.randn(1, M, C, device="cuda"); w = torch.randn(2 * C, C, device="cuda") * 0.05
    b = torch.zeros(C, device="cuda")
    w3 = ops.presplit_for(w) if PRE else None
    ms = t(lambda: ops.highway(x, w, b, b, w_split=w3))
    res[name] = (ms, 2.0 * M * 2 * C * C / ms / 1e9, 0.0)
conv("post.proj1", 64, 1368, 2048, 256, 3, True)
conv("post.proj2", 64, 1368, 256, 80, 3)
bank("post.bank", 64, 1368, 80, 8)
hw("post.highway", 87552, 256)
conv("post.gru_in", 64, 1368, 256, 1536, 1)
conv("post.lin", 64, 1368, 512, 80, 1)
bank("pre.bank", 64, 200, 256, 16)
conv("pre.proj1", 64, 200, 4096, 256, 3, True)
conv("pre.proj2", 64, 200, 256, 256, 3)
conv("lstm_in", 64, 200, 512, 4096, 1)
conv("pred.conv1", 64, 200, 64, 256, 5)
conv("pred.conv", 64, 200, 256, 256, 5)
print(json.dumps(res))
'''
VARIANTS = {'f32': {'FTMI_MMA': '0'},
            'x6b': {'FTMI_MMA': '1', 'FTMI_GEMM_X6': '1', 'PRE': '1'},
            'h3': {'FTMI_MMA': '2', 'PRE': '1', 'FTMI_GEMM_SLAB': '0'},
            'slab': {'FTMI_MMA': '2', 'PRE': '1', 'FTMI_GEMM_SLAB': '1', 'FTMI_GEMM_SLAB_WS': '0'},
            'slabws': {'FTMI_MMA': '2', 'PRE': '1', 'FTMI_GEMM_SLAB': '1', 'FTMI_GEMM_SLAB_WS': '1'}}
names = sys.argv[1:] or ['h3', 'slab']
out = {}
for name in names:
    r = subprocess.run([sys.executable, '-c', CHILD], env={**os.environ, **VARIANTS[name]},
                       capture_output=True, text=True, timeout=400)
    if r.returncode != 0:
        print(name, 'FAILED', r.stderr[-3000:]); sys.exit(1)
    out[name] = json.loads(r.stdout.strip().splitlines()[-1])
shapes = list(out[names[0]])
print(f'{"shape":14s}' + ''.join(f'{v:>32s}' for v in names))
for sh in shapes:
    print(f'{sh:14s}' + ''.join(f'{out[v][sh][0]:9.3f} ms {out[v][sh][1]:7.1f} TF {out[v][sh][2]:8.1e}'
                                 for v in names))
