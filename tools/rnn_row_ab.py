"""A/B of the recurrence kernels on the model's shapes: rnn_row_kernel (FTMI_RNN_ROW=1, live
sequences per group FTMI_RNN_NB or the spread choice) against rnn_bidir_kernel
(FTMI_RNN_ROW=0): us/step and max |variant - legacy| on the same inputs (both env
variables are read per call, so one process switches between them).  Run on the GPU box:
    python tools/rnn_row_ab.py [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

VARIANTS = [('legacy', {'FTMI_RNN_ROW': '0'}, False), ('row', {}, False),
            ('row_spread', {}, True), ('row_nb8', {'FTMI_RNN_NB': '8'}, False),
            ('row_nb4', {'FTMI_RNN_NB': '4'}, False)]
SHAPES = [(1, 512, 64, 1368), (0, 256, 64, 1368), (0, 128, 64, 200), (0, 256, 64, 200)]


def run(cell, H, B, T, xp, w, bh, ws, spread, reps):
    y = None
    for _ in range(2):
        y = ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=spread,
                          check=True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(reps):
        ops.rnn_bidir(cell, xp, H, w, bh if cell == 0 else None, ws=ws, spread=spread)
    e.record()
    torch.cuda.synchronize()
    return y, s.elapsed_time(e) / reps / T * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    torch.manual_seed(0)
    data = {}
    for cell, H, B, T in SHAPES:
        G = 4 if cell else 3
        data[(cell, H, B, T)] = (torch.randn(B, T, 2 * G * H, device='cuda') * 0.5,
                                 torch.randn(2, G * H, H, device='cuda') / H ** 0.5,
                                 torch.randn(2 * G * H, device='cuda') * 0.1)
    ws = torch.zeros(1 << 23, dtype=torch.int32, device='cuda')
    for _ in range(rounds):
        ref = {}
        for name, env, spread in VARIANTS:
            for k in ('FTMI_RNN_ROW', 'FTMI_RNN_NB'):
                os.environ.pop(k, None)
            os.environ.update(env)
            line = []
            for shape in SHAPES:
                cell, H, B, T = shape
                y, us = run(cell, H, B, T, *data[shape], ws, spread, 5)
                blocks = ops.rnn_blocks(cell, B, H, 2 | (ops.RNN_SPREAD if spread else 0))
                d = ''
                if name == 'legacy':
                    ref[shape] = y
                else:
                    d = f' d={float((y - ref[shape]).abs().max()):.1e}'
                line.append(f'{"lstm" if cell else "gru"}{H}/T{T} {us:5.2f}us {blocks}wg{d}')
            print(f'{name:11s} ' + '  '.join(line), flush=True)


if __name__ == '__main__':
    main()
