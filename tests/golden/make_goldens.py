"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Run in the build container only (it imports the reference from /root/reference, which does
not exist on the GPU box):

    PYTHONPATH=/root/reference python tests/golden/make_goldens.py

Weights: forwardtacotron_amd.synthetic recipe (seed 0), loaded into the reference
`models.forward_tacotron.ForwardTacotron` with load_state_dict — the fixtures store only
inputs and outputs; the weights are regenerated bit-identically from the recipe.
Every case records the reference call it pins (file:line).
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path(os.environ.get('FT_REFERENCE', '/root/reference'))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REF))

from models.common_layers import LengthRegulator  # noqa: E402  (reference)
from models.forward_tacotron import ForwardTacotron  # noqa: E402  (reference)

from forwardtacotron_amd.synthetic import default_config, load_synthetic, synthetic_tokens  # noqa: E402

torch.manual_seed(0)
torch.set_num_threads(1)


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def tie_margin(dur: np.ndarray) -> float:
    s = dur.astype(np.float32) + np.float32(0.5)
    frac = s - np.floor(s)
    return float(np.minimum(frac, 1 - frac).min())


def capture(model):
    """Forward hooks on the reference modules whose outputs the fixtures keep."""
    store = {}
    hooks = [
        model.prenet.register_forward_hook(lambda m, i, o: store.__setitem__('prenet', f32(o))),
        model.lstm.register_forward_hook(lambda m, i, o: store.__setitem__('lstm', f32(o[0]))),
        model.postnet.register_forward_hook(lambda m, i, o: store.__setitem__('postnet', f32(o))),
        model.dur_pred.register_forward_hook(lambda m, i, o: store.__setitem__('dur_raw', f32(o))),
    ]
    return store, hooks


def main():
    model = ForwardTacotron.from_config(default_config())
    load_synthetic(model, seed=0)
    model.eval()
    cases = {}
    meta = {'torch': torch.__version__, 'reference': str(REF), 'weights': 'synthetic seed 0',
            'cases': {}}

    # -- generate(): forward_tacotron.py:244-268 ------------------------------------------
    gen_cases = [
        ('gen_b1', dict(lengths=[12], seed=3), dict(alpha=1.0), True),
        ('gen_b3', dict(lengths=[23, 14, 19], seed=5), dict(alpha=1.0), False),
        ('gen_alpha', dict(lengths=[17, 9], seed=8), dict(alpha=0.8), False),
        ('gen_fill2', dict(lengths=[9, 6], seed=13), dict(alpha=1000.0), False),
        ('gen_callbacks', dict(lengths=[15, 11], seed=21),
         dict(alpha=1.2, pitch_function=lambda p: p * 2.0 + 0.1,
              energy_function=lambda e: e - 0.05), False),
    ]
    for name, tok, kw, full in gen_cases:
        x = torch.from_numpy(synthetic_tokens(len(tok['lengths']), max(tok['lengths']),
                                              seed=tok['seed'], lengths=tok['lengths']))
        store, hooks = capture(model)
        g = model.generate(x, **kw)
        for h in hooks:
            h.remove()
        d = {'x': x.numpy(), 'mel': f32(g['mel']), 'mel_post': f32(g['mel_post']),
             'dur': f32(g['dur']), 'pitch': f32(g['pitch']), 'energy': f32(g['energy']),
             'dur_raw': store['dur_raw'][..., 0], 'prenet': store['prenet']}
        if full:
            d['lstm'] = store['lstm']
            d['postnet'] = store['postnet']
        cases[name] = d
        meta['cases'][name] = {
            'pins': 'ForwardTacotron.generate models/forward_tacotron.py:244-268',
            'alpha': kw.get('alpha', 1.0),
            'callbacks': name == 'gen_callbacks',
            'T_mel': int(g['mel'].shape[-1]),
            'dur_tie_margin': tie_margin(d['dur']),
        }

    # -- generate_jit(): forward_tacotron.py:270-284 ------------------------------------
    x = torch.from_numpy(synthetic_tokens(2, 13, seed=34, lengths=[13, 10]))
    g = model.generate_jit(x, alpha=1.1, beta=0.7)
    cases['gen_jit'] = {'x': x.numpy(), 'mel': f32(g['mel']), 'mel_post': f32(g['mel_post']),
                        'dur': f32(g['dur']), 'pitch': f32(g['pitch']), 'energy': f32(g['energy'])}
    meta['cases']['gen_jit'] = {'pins': 'generate_jit models/forward_tacotron.py:270-284',
                                'alpha': 1.1, 'beta': 0.7, 'dur_tie_margin': tie_margin(f32(g['dur']))}

    # -- forward(batch): teacher forcing, packed LSTM, forward_tacotron.py:184-242 ----------
    rng = np.random.Generator(np.random.PCG64(99))
    lens = [11, 7, 9]
    xb = synthetic_tokens(3, 11, seed=55, lengths=lens)
    dur = np.zeros((3, 11), np.float32)
    for b, L in enumerate(lens):
        dur[b, :L] = rng.integers(1, 9, size=L)
    mel_len = dur.sum(1).astype(np.int64)
    mel_len[1] -= 2  # a shorter mel_len than sum(dur): packing uses mel_len, LR uses dur
    T_mel_pad = int(mel_len.max()) + 1
    mel = np.full((3, 80, T_mel_pad), -11.5129, np.float32)
    pitch = rng.normal(0, 1, (3, 11)).astype(np.float32)
    energy = rng.normal(0, 1, (3, 11)).astype(np.float32)
    batch = {'x': torch.from_numpy(xb), 'mel': torch.from_numpy(mel),
             'mel_len': torch.from_numpy(mel_len), 'dur': torch.from_numpy(dur.copy()),
             'pitch': torch.from_numpy(pitch), 'energy': torch.from_numpy(energy)}
    with torch.no_grad():
        o = model(batch)
    cases['forward'] = {'x': xb, 'mel_in': mel, 'mel_len': mel_len, 'dur_in': dur,
                        'pitch_in': pitch, 'energy_in': energy, 'mel': f32(o['mel']),
                        'mel_post': f32(o['mel_post']), 'dur': f32(o['dur']),
                        'pitch': f32(o['pitch']), 'energy': f32(o['energy'])}
    meta['cases']['forward'] = {'pins': 'ForwardTacotron.forward models/forward_tacotron.py:184-242'}

    # -- LengthRegulator known answers: common_layers.py:7-19 ----------------------------
    dur_ka = np.array([[0.49999997, 0.5, 1.5, 2.5, -0.3, 0.0, 3.4999998, 1e-8, 7.5],
                       [2.4999998, -1.5, 0.49999997, 4.0, 1.0000001, 0.7, 0.0, 0.0, 0.0]],
                      np.float32)
    xka = np.arange(2 * 9 * 4, dtype=np.float32).reshape(2, 9, 4) + 1.0
    dt = torch.from_numpy(dur_ka.copy())
    out = LengthRegulator()(torch.from_numpy(xka), dt)
    cases['lr_known'] = {'x': xka, 'dur_in': dur_ka, 'dur_out': dt.numpy(),
                         'counts': (dt + 0.5).long().numpy(), 'out': f32(out)}
    meta['cases']['lr_known'] = {'pins': 'LengthRegulator common_layers.py:7-19'}

    # -- LR on random data at a realistic size (B=4, T=50, C=512) -------------------------
    dur_r = rng.uniform(-1.0, 12.0, (4, 50)).astype(np.float32)
    x_r = rng.normal(0, 1, (4, 50, 8)).astype(np.float32)
    dt = torch.from_numpy(dur_r.copy())
    out = LengthRegulator()(torch.from_numpy(x_r), dt)
    cases['lr_random'] = {'x': x_r, 'dur_in': dur_r, 'dur_out': dt.numpy(), 'out': f32(out)}
    meta['cases']['lr_random'] = {'pins': 'LengthRegulator common_layers.py:7-19'}

    # -- checkpoint format: reference state_dict keys / shapes / dtypes (utils/checkpoints.py:16-18)
    sd_meta = [[k, list(v.shape), str(v.dtype).replace('torch.', '')] for k, v in model.state_dict().items()]
    (HERE / 'state_dict_keys.json').write_text(json.dumps(sd_meta))

    for name, arrays in cases.items():
        np.savez_compressed(HERE / f'{name}.npz', **arrays)
    (HERE / 'goldens.json').write_text(json.dumps(meta, indent=1, sort_keys=True))
    total = sum((HERE / f'{n}.npz').stat().st_size for n in cases)
    print(f'wrote {len(cases)} fixtures, {total / 1e6:.2f} MB')
    print(json.dumps(meta['cases'], indent=1))


if __name__ == '__main__':
    main()
