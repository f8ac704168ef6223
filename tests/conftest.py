"""Shared fixtures.  `-m gpu` tests need a HIP device and the built libftmi.so; everything
else runs on CPU (the driver runs `pytest -m "not gpu"` in the build container)."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / 'tests' / 'golden'
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP (MI355X) device and libftmi.so')
    config.addinivalue_line('markers', 'slow: full-size (BASELINE config) case')


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason='no HIP device')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    with np.load(GOLDEN / f'{name}.npz', allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope='session')
def golden_meta():
    return json.loads((GOLDEN / 'goldens.json').read_text())


def synth_sd_dict(seed: int = 0):
    """Synthetic weights as {reference key: np.ndarray}, from the key fixture."""
    from forwardtacotron_amd.synthetic import synthetic_array
    keys = json.loads((GOLDEN / 'state_dict_keys.json').read_text())
    return {k: synthetic_array(k, shape, dt, seed) for k, shape, dt in keys}


@pytest.fixture(scope='session')
def synth_sd():
    """Synthetic weights (seed 0) as {reference key: np.ndarray}, from the key fixture."""
    return synth_sd_dict(0)


@pytest.fixture(scope='session')
def gpu_model(synth_sd):
    import torch
    from forwardtacotron_amd.forward_tacotron import ForwardTacotron
    from forwardtacotron_amd.synthetic import default_config
    m = ForwardTacotron.from_config(default_config())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synth_sd.items()})
    return m.to('cuda').eval()
