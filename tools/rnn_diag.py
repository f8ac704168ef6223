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
for cell, H, B, T in [(1, 512, 64, 1368), (0, 256, 64, 1368), (0, 128, 64, 200), (0, 64, 64, 200),
                      (1, 512, 1, 816), (0, 256, 1, 816)]:
    G = 4 if cell else 3
    xp = torch.randn(B, T, 2 * G * H, device="cuda") * 0.5
    w = torch.randn(2, G * H, H, device="cuda") / H ** 0.5
    bh = torch.randn(2 * G * H, device="cuda") * 0.1
    ws = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
    # the decoder LSTM and the postnet GRU run spread in the model (forward_tacotron.py)
    sp = T > 800 and ((cell == 1 and H == 512) or (cell == 0 and H == 256))
    for _ in range(2):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=sp)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(5):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=sp)
    e.record(); torch.cuda.synchronize()
    res[f"{'lstm' if cell else 'gru'}{H}b{B}"] = s.elapsed_time(e) / 5 / T * 1e3
    st = int(ops.status_word(xp.device).item())
    if st & 4:  # a workgroup timed out (not co-resident): the timing is not a step time
        res[f"{'lstm' if cell else 'gru'}{H}b{B}"] = -1.0
        ops.status_word(xp.device).zero_()
print(json.dumps(res))
'''
rows = {}
# variants: "VAR=val,VAR2=val2;..." (DIAG_ENVS) or the legacy single-variable sweep
if os.environ.get('DIAG_ENVS'):
    VARIANTS = [dict(kv.split('=') for kv in v.split(',') if kv) for v in os.environ['DIAG_ENVS'].split(';')]
else:
    VAR = os.environ.get('DIAG_VAR', 'FTMI_RNN_DIAG')
    VARIANTS = [{VAR: v} for v in os.environ.get('DIAG_VALS', '0 16 0 16').split()]
for var in VARIANTS:
    diag = ','.join(f'{k}={v}' for k, v in var.items())
    env = {**os.environ, **var}
    r = subprocess.run([sys.executable, '-c', CHILD], env=env, capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        print('diag', diag, 'FAILED', r.stderr[-2000:])
        sys.exit(1)
    rows[diag] = json.loads(r.stdout.strip().splitlines()[-1])
    print(f'{diag}: ' + '  '.join(f'{k} {v:6.2f} us/step' for k, v in rows[diag].items()),
          flush=True)
