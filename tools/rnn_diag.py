"""Timing experiments on the persistent recurrence: what each part of a step costs.
FTMI_RNN_DIAG bits (results are invalid when set; timing only): 1 = L2-hot input-projection
rows, 2 = no hand-off waits, 8 = no f16 tail split of h (head only); 16 = s_sleep between
polls (valid results).  Run on the GPU box."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
from forwardtacotron_amd import ops
res = {}
for cell, H, B, T in [(1, 512, 64, 1368), (0, 256, 64, 1368), (0, 128, 64, 200), (0, 64, 64, 200)]:
    G = 4 if cell else 3
    xp = torch.randn(B, T, 2 * G * H, device="cuda") * 0.5
    w = torch.randn(2, G * H, H, device="cuda") / H ** 0.5
    bh = torch.randn(2 * G * H, device="cuda") * 0.1
    ws = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
    for _ in range(2):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(5):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws)
    e.record(); torch.cuda.synchronize()
    res[f"{'lstm' if cell else 'gru'}{H}"] = s.elapsed_time(e) / 5 / T * 1e3
print(json.dumps(res))
'''
rows = {}
VAR = os.environ.get('DIAG_VAR', 'FTMI_RNN_DIAG')
VALS = os.environ.get('DIAG_VALS', '0 16 0 16').split()
for diag in VALS:
    env = {**os.environ, VAR: str(diag)}
    r = subprocess.run([sys.executable, '-c', CHILD], env=env, capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        print('diag', diag, 'FAILED', r.stderr[-2000:])
        sys.exit(1)
    rows[diag] = json.loads(r.stdout.strip().splitlines()[-1])
    print(f'{VAR}={diag}: ' + '  '.join(f'{k} {v:6.2f} us/step' for k, v in rows[diag].items()),
          flush=True)
