"""Per-phase cycle breakdown of the WaveRNN sample loop (FTMI_WR_STAMPS=1 build-free diag):
thread 0 of GRU workgroup 0 and FC workgroup 128 sum s_memtime deltas per phase."""
import os
import sys
from pathlib import Path

os.environ['FTMI_WR_STAMPS'] = '1'
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from forwardtacotron_amd.synthetic import default_config, load_synthetic  # noqa: E402
from forwardtacotron_amd.wavernn import WaveRNN  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 821
m = load_synthetic(WaveRNN.from_config(default_config()), kind='wavernn').cuda().eval()
rng = np.random.Generator(np.random.PCG64(0))
mels = torch.from_numpy((rng.normal(0, 1, (1, 80, frames)) - 4).astype(np.float32)).cuda()
for _ in range(2):
    smp = m.generate_samples(mels, True, 11000, 550, seed=1)
torch.cuda.synchronize()
B, L = smp.shape
ws = m._ftmi_last_ws.cpu().numpy().view(np.uint32)
st = ws[64:128].view(np.uint64).astype(np.float64)
gru = ['w1 matvec+mel load', 'acquire h2', 'w2 matvec + mel', 'acquire sample', 'cell1+acquire h1',
       'w3 matvec', 'cell2+publish']
fc = ['mel', 'acquire sample', 'acquire h1', 'acquire h2', 'fc1 matvec', 'fc1 fin+acq y1',
      'fc2 matvec', 'fc2 fin+acq y2', 'fc3 matvec', 'fc3 fin+draw']
print(f'B={B} L={L}')
for name, base, labels in (('GRU WG0', 0, gru), ('FC WG128', 16, fc)):
    tot = st[base:base + len(labels)].sum()
    print(f'{name}: {tot / L:.0f} cycles/step')
    for i, lab in enumerate(labels):
        print(f'  {lab:22s} {st[base + i] / L:8.0f}  {100 * st[base + i] / tot:5.1f} %')
