"""Interleaved A/B of recurrence build-time knobs that are read once per process
(FTMI_RNN_WK, FTMI_RNN_PSLEEP, ...): one child process per variant and round, us/step of the
c3 decoder recurrences (LSTM H 512 and the postnet GRU H 256, B 64, T 1368) and the
phoneme-phase GRUs.  usage (GPU box):
    python tools/rnn_env_ab.py ROUNDS "VAR=v,VAR2=w;VAR=x;..." [c3|c2]   (';' separates variants;
    c2 = the batch-1 exact-fp32 GEMV shapes, B 1, T 800)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
from forwardtacotron_amd import ops
torch.manual_seed(0)
res = {}
CASES = {"c3": [(1, 512, 64, 1368, True), (0, 256, 64, 1368, True), (0, 256, 64, 200, False)],
         "c2": [(1, 512, 1, 800, True), (0, 256, 1, 800, True), (0, 256, 1, 120, False),
                (1, 512, 2, 800, True)]}
for cell, H, B, T, spread in CASES[sys.argv[1]]:
    G = 4 if cell else 3
    xp = torch.randn(B, T, 2 * G * H, device="cuda") * 0.5
    w = torch.randn(2, G * H, H, device="cuda") / H ** 0.5
    bh = torch.randn(2 * G * H, device="cuda") * 0.1
    ws = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
    for _ in range(2):
        y = ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=spread, check=True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(5):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=spread)
    e.record(); torch.cuda.synchronize()
    res[f"{'lstm' if cell else 'gru'}{H}/B{B}/T{T}"] = round(s.elapsed_time(e) / 5 / T * 1e3, 3)
print(json.dumps(res))
'''


def main():
    rounds = int(sys.argv[1])
    cases = sys.argv[3] if len(sys.argv) > 3 else 'c3'
    variants = [dict(kv.split('=') for kv in v.split(',') if kv) for v in sys.argv[2].split(';')]
    for _ in range(rounds):
        for var in variants:
            r = subprocess.run([sys.executable, '-c', CHILD, cases], env={**os.environ, **var},
                               capture_output=True, text=True, timeout=300)
            name = ','.join(f'{k}={v}' for k, v in var.items()) or 'default'
            if r.returncode != 0:
                print(name, 'FAILED', r.stderr[-2000:], flush=True)
                sys.exit(1)
            res = json.loads(r.stdout.strip().splitlines()[-1])
            print(f'{name:40s} ' + '  '.join(f'{k} {v:.3f}' for k, v in res.items()), flush=True)


if __name__ == '__main__':
    main()
