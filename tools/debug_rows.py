"""Debug helper for the row-owning recurrence kernel: one small GRU / LSTM against the numpy
oracle, per direction and step, with the error word and status bits."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import BiRNN  # noqa: E402
from oracle import ft_oracle as O  # noqa: E402


def run(cell, H, B, T, fin, seed=0):
    rng = np.random.default_rng(seed)
    m = BiRNN(fin, H, cell)
    G = 3 if cell == 'gru' else 4
    sd = {}
    for sfx in ('', '_reverse'):
        sd['weight_ih_l0' + sfx] = rng.normal(0, 1 / np.sqrt(fin), (G * H, fin))
        sd['weight_hh_l0' + sfx] = rng.normal(0, 1 / np.sqrt(H), (G * H, H))
        sd['bias_ih_l0' + sfx] = rng.normal(0, 0.1, G * H)
        sd['bias_hh_l0' + sfx] = rng.normal(0, 0.1, G * H)
    sd = {k: v.astype(np.float32) for k, v in sd.items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda()
    x = rng.normal(0, 1, (B, T, fin)).astype(np.float32)
    ref = (O.lstm_bidir if cell == 'lstm' else O.gru_bidir)({'r.' + k: v for k, v in sd.items()}, 'r', x, np.float32)
    st = ops.status_word('cuda')
    st.zero_()
    y = m.forward_cl(torch.from_numpy(x).cuda()).cpu().numpy()
    d = np.abs(y - ref)
    print(f'{cell} H={H} B={B} T={T} status={int(st.item())} maxerr={d.max():.3e}')
    for t in range(min(T, 4)):
        print('  t', t, 'fwd', d[:, t, :H].max(), 'bwd', d[:, T - 1 - t, H:].max())
    bad = np.argwhere(d > 1e-3)
    if len(bad):
        print('  first bad (b,t,c):', bad[:8].tolist())
        b, t, c = bad[0]
        print('  got', y[b, t, c - 2:c + 3], 'ref', ref[b, t, c - 2:c + 3])


if __name__ == '__main__':
    for args in [('gru', 64, 3, 6, 256), ('gru', 64, 16, 6, 256), ('gru', 256, 3, 6, 256), ('lstm', 512, 3, 6, 512)]:
        run(*args)
