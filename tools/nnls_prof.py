"""The reference NNLS (device L-BFGS-B) on the bench's c2 mel: wall time, per-block iterations /
evaluations / history size, for rocprofv3 --kernel-trace --stats (which phase kernel
dominates).  usage: python tools/nnls_prof.py [seed]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import dsp as G  # noqa: E402
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402
from forwardtacotron_amd.synthetic import default_config, load_synthetic, synthetic_tokens  # noqa: E402


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    cfg = default_config()
    m = load_synthetic(ForwardTacotron.from_config(cfg), 0).cuda().eval()
    x = torch.from_numpy(synthetic_tokens(1, 120, seed=seed, min_len=120)).cuda()
    mel = m.generate(x)['mel_post']
    dsp = G.DSP.from_config(cfg)
    plan = dsp.plan(mel.device)
    torch.cuda.synchronize()
    info = []
    t0 = time.perf_counter()
    S = G._nnls_lbfgsb(plan, mel.float().contiguous(), None, True, info=info)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({'frames': int(mel.size(2)), 'seconds': round(dt, 3),
                      'blocks': [[int(a), int(b), float(f), float(g)] for a, b, f, g in info],
                      'S_sum': float(S.double().sum())}), flush=True)


if __name__ == '__main__':
    main()
