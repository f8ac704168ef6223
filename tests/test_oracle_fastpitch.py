"""The FastPitch oracle (oracle/fp_oracle.py) against the reference's own outputs (golden
vectors from tests/golden/make_goldens_fastpitch.py) — parity PINNED.  CPU only."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import fp_oracle as FP

CASES = {
    'fp_gen_b1': dict(alpha=1.0),
    'fp_gen_b3': dict(alpha=1.0),
    'fp_gen_alpha': dict(alpha=0.8),
    'fp_gen_fill2': dict(alpha=1000.0),
    'fp_gen_callbacks': dict(alpha=1.2, pitch_function=lambda p: p * np.float32(2.0) + np.float32(0.1),
                             energy_function=lambda e: e - np.float32(0.05)),
}


@pytest.fixture(scope='module')
def fp_sd():
    from forwardtacotron_amd.fast_pitch import FastPitch
    from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict
    return synthetic_state_dict(FastPitch.from_config(default_config()), 0, 'fast_pitch')


def test_state_dict_matches_reference_keys(fp_sd):
    keys = json.loads((GOLDEN / 'fastpitch_state_dict_keys.json').read_text())
    assert [k for k, _, _ in keys] == list(fp_sd)
    for k, shape, _ in keys:
        assert list(fp_sd[k].shape) == shape, k


@pytest.mark.parametrize('name', list(CASES))
def test_generate(name, fp_sd):
    g = load_golden(name)
    o = FP.generate(fp_sd, g['x'], **CASES[name])
    np.testing.assert_allclose(o['dur'], g['dur'], atol=2e-5)
    np.testing.assert_array_equal(FP.duration_counts(o['dur']), FP.duration_counts(g['dur']))
    assert o['mel'].shape == g['mel'].shape
    assert np.abs(o['mel'] - g['mel']).max() < 2e-4
    np.testing.assert_allclose(o['pitch'], g['pitch'], atol=2e-5)
    np.testing.assert_allclose(o['energy'], g['energy'], atol=2e-5)
    np.testing.assert_allclose(o['postnet'], g['postnet'], atol=5e-5)


def test_forward(fp_sd):
    g = load_golden('fp_forward')
    batch = {'x': g['x'], 'mel': g['mel_in'], 'mel_len': g['mel_len'], 'dur': g['dur_in'].copy(),
             'pitch': g['pitch_in'], 'energy': g['energy_in']}
    o = FP.forward(fp_sd, batch)
    assert o['mel'].shape == g['mel'].shape
    assert np.abs(o['mel'] - g['mel']).max() < 2e-4
    np.testing.assert_allclose(o['dur'], g['dur'], atol=2e-5)
    np.testing.assert_allclose(o['pitch'], g['pitch'], atol=2e-5)


@pytest.mark.parametrize('name', ['fp_gen_b3', 'fp_gen_alpha', 'fp_gen_fill2'])
def test_torch_cpu_restatement(name, fp_sd):
    import torch
    from oracle import fp_torch_cpu as TC
    g = load_golden(name)
    o = TC.generate(TC.to_torch(fp_sd), torch.from_numpy(g['x']), alpha=CASES[name]['alpha'])
    assert np.abs(o['mel'].numpy() - g['mel']).max() < 2e-4
    np.testing.assert_array_equal(FP.duration_counts(o['dur'].numpy()), FP.duration_counts(g['dur']))
