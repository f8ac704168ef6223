"""Generate the WaveRNN vocoder goldens from the reference itself (run HERE only: the
reference never travels).  Output: tests/golden/wr_*.npz + wavernn_state_dict_keys.json.

models/fatchord_version.py cannot be imported as a module in this container: its
`from utils.dsp import *` / `from utils.display import *` pull in librosa 0.7.2 and
matplotlib, which are absent.  The vocoder classes themselves only use torch / numpy, so
this script compiles the file's CLASS definitions (ResBlock, MelResNet, Stretch2d,
UpsampleNetwork, WaveRNN — the reference text, unchanged) with the names they use bound
to torch / numpy, utils/distribution.py imported normally (torch / numpy only), and
DSP.label_2_float / decode_mu_law taken the same way from utils/dsp.py's DSP class.
Nothing is stubbed: every name the executed code touches is the real library or the
reference's own function.  One compatibility alias: the reference calls
`np.cumproduct` (UpsampleNetwork :69), numpy's deprecated alias of `np.cumprod` that
numpy 2 removed; the classes see a numpy namespace where that name is numpy's own cumprod.

Cases (synthetic weights, forwardtacotron_amd/synthetic.py model='wavernn'):
  wr_upsample   UpsampleNetwork on (1, 80, 7) mels
  wr_forward    WaveRNN.forward (teacher-forced) B=2, mels (2, 80, 6): logits (2, 512, 512)
  wr_gen_raw    generate(batched=True, target=600, overlap=60, mu_law=True), RAW, seed 123
  wr_gen_unb    generate(batched=False, mu_law=False), RAW, (1, 80, 21) mels, seed 7
                (the reference's 20-hop fade-out needs >= 21 frames)
  wr_gen_mol    generate(batched=True, target=400, overlap=40), MOL mode, seed 5
  wr_fold       fold_with_overlap / xfade_and_unfold known answers
"""
from __future__ import annotations

import ast
import json
import math
import sys
import time
from pathlib import Path
from typing import Any, Dict, Union

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = Path('/root/reference')
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(REF))

from utils.distribution import sample_from_discretized_mix_logistic  # noqa: E402

from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict  # noqa: E402


def _classes(path: Path, names, ns):
    tree = ast.parse(path.read_text())
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in names]
    exec(compile(ast.Module(body=body, type_ignores=[]), str(path), 'exec'), ns)
    return ns


class _NumpyCompat:
    """numpy, plus the `cumproduct` alias (== np.cumprod) numpy 2 removed."""
    cumproduct = staticmethod(np.cumprod)

    def __getattr__(self, name):
        return getattr(np, name)


def reference_classes():
    dsp_ns = _classes(REF / 'utils' / 'dsp.py', {'DSP'}, {
        'math': math, 'np': np, 'Dict': Dict, 'Any': Any, 'Union': Union, 'Path': Path})
    ns = {'torch': torch, 'nn': nn, 'F': F, 'np': _NumpyCompat(), 'time': time, 'Path': Path,
          'Union': Union, 'Dict': Dict, 'Any': Any, 'DSP': dsp_ns['DSP'],
          'sample_from_discretized_mix_logistic': sample_from_discretized_mix_logistic}
    return _classes(REF / 'models' / 'fatchord_version.py',
                    {'ResBlock', 'MelResNet', 'Stretch2d', 'UpsampleNetwork', 'WaveRNN'}, ns)


def make_model(ns, mode='RAW'):
    cfg = default_config()
    cfg['vocoder']['model']['mode'] = mode
    m = ns['WaveRNN'].from_config(cfg)
    sd = synthetic_state_dict(m, seed=0, model='wavernn')
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.eval()


def main():
    torch.set_num_threads(8)
    ns = reference_classes()
    model = make_model(ns)
    keys = [[k, list(v.shape), str(v.dtype)] for k, v in model.state_dict().items()]
    (HERE / 'wavernn_state_dict_keys.json').write_text(json.dumps(keys))
    rng = np.random.Generator(np.random.PCG64(2024))

    def mel(B, T):
        return (rng.normal(0.0, 1.0, (B, 80, T)) - 4.0).astype(np.float32)

    with torch.no_grad():
        m = mel(1, 7)
        up, aux = model.upsample(torch.from_numpy(m))
        np.savez(HERE / 'wr_upsample.npz', mels=m, up=up.numpy(), aux=aux.numpy())

        m = mel(2, 6)
        L = (6 - 4) * 256
        x = rng.uniform(-1, 1, (2, L)).astype(np.float32)
        logits = model(torch.from_numpy(x), torch.from_numpy(m))
        np.savez(HERE / 'wr_forward.npz', mels=m, x=x, logits=logits.numpy())

    cases = [('wr_gen_raw', 'RAW', mel(1, 24), dict(batched=True, target=600, overlap=60, mu_law=True), 123),
             ('wr_gen_unb', 'RAW', mel(1, 21), dict(batched=False, target=600, overlap=60, mu_law=False), 7),
             ('wr_gen_mol', 'MOL', mel(1, 21), dict(batched=True, target=400, overlap=40, mu_law=True), 5)]
    for name, mode, m, kw, seed in cases:
        mdl = model if mode == 'RAW' else make_model(ns, mode)
        torch.manual_seed(seed)
        wav = mdl.generate(torch.from_numpy(m), silent=True, **kw)
        np.savez(HERE / f'{name}.npz', mels=m, wav=np.asarray(wav), seed=seed, mode=mode,
                 **{k: int(v) for k, v in kw.items()})
        print(name, np.asarray(wav).shape, float(np.abs(wav).mean()))

    x = torch.arange(1, 11, dtype=torch.float32).view(1, 10, 1)
    folded = model.fold_with_overlap(x, 2, 1)
    y = rng.normal(0.0, 1.0, (5, 120))
    un = model.xfade_and_unfold(y.copy(), 100, 10)
    np.savez(HERE / 'wr_fold.npz', x=x.numpy(), folded=folded.numpy(), y=y, unfolded=un)


if __name__ == '__main__':
    main()
