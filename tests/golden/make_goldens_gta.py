"""Golden fixture for the GTA batch format (forwardtacotron_amd/gta.py collate_tts), made by
running the REFERENCE's own collate_tts (`utils/dataset.py:276-315`) in the build container:

    python tests/golden/make_goldens_gta.py

utils/dataset.py cannot be imported here (it star-imports utils/dsp.py, whose librosa is
absent), so this script parses that file and executes exactly the three reference
functions pad1d / pad2d / collate_tts (unmodified, read from /root/reference at run time)
with numpy and torch; nothing of the reference is stored — the fixture holds inputs and
outputs only.  Output: tests/golden/gta_collate.npz.
"""
from __future__ import annotations

import ast
import os
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get('FT_REFERENCE', '/root/reference'))


def reference_functions():
    src = (REF / 'utils' / 'dataset.py').read_text()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ('pad1d', 'pad2d', 'collate_tts')]
    assert len(keep) == 3
    ns = {'np': np, 'torch': torch, 'List': list, 'Dict': dict, 'Union': object}
    exec(compile(ast.Module(body=keep, type_ignores=[]), str(REF / 'utils' / 'dataset.py'), 'exec'), ns)
    return ns


def items(seed=0):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i, (xl, ml) in enumerate([(17, 61), (9, 33), (13, 64)]):
        out.append({'x': rng.integers(1, 135, xl), 'mel': rng.normal(-4, 2, (80, ml)).astype(np.float32),
                    'item_id': f'LJ{i:03d}', 'x_len': xl, 'mel_len': ml,
                    'dur': rng.integers(1, 8, xl).astype(np.float64),
                    'pitch': rng.normal(0, 1, xl).astype(np.float32),
                    'energy': rng.normal(0, 1, xl).astype(np.float32)})
    return out


def main():
    ns = reference_functions()
    its = items()
    save = {}
    for i, it in enumerate(its):
        for k, v in it.items():
            if k != 'item_id':
                save[f'in{i}_{k}'] = np.asarray(v)
    for r in (1, 2, 3):
        b = ns['collate_tts'](its, r)
        for k in ('x', 'mel', 'x_len', 'mel_len', 'dur', 'pitch', 'energy'):
            save[f'r{r}_{k}'] = b[k].numpy()
        save[f'r{r}_item_id'] = np.array(b['item_id'])
    np.savez(HERE / 'gta_collate.npz', **save)
    print('wrote', HERE / 'gta_collate.npz')


if __name__ == '__main__':
    main()
