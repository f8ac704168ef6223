"""A/B the recurrence kernel variants (XCD-local vs global hand-off, bf16x6 vs f32 MMA)
and print the census the XCD-local mode saw.  Run on the GPU box."""
import os, subprocess, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
from forwardtacotron_amd import ops
res = {}
for cell, H, B, T in [(1, 512, 64, 1368), (0, 256, 64, 1368), (0, 128, 64, 200), (0, 64, 64, 200), (1, 512, 1, 816)]:
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
    census = [int(ws[32 + 32 * i].item()) for i in range(8)]
    res[f"{'lstm' if cell else 'gru'}{H}_B{B}"] = {"us_per_step": s.elapsed_time(e) / 5 / T * 1e3, "census": census, "err": int(ws[0].item())}
print(json.dumps(res))
'''
for env in [{'FTMI_RNN_XCD_LOCAL': '1', 'FTMI_RNN_MMA': '1'}, {'FTMI_RNN_XCD_LOCAL': '0', 'FTMI_RNN_MMA': '1'},
            {'FTMI_RNN_XCD_LOCAL': '1', 'FTMI_RNN_MMA': '0'}]:
    r = subprocess.run([sys.executable, '-c', CHILD], env={**os.environ, **env}, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(env, 'FAILED', r.stderr[-2000:]); sys.exit(1)
    print(env)
    for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items():
        print(f'   {k:14s} {v["us_per_step"]:7.2f} us/step  census {v["census"]} err {v["err"]}')
