"""The WaveRNN vocoder oracle (oracle/wr_torch_cpu.py) against goldens produced by the
reference classes themselves (tests/golden/make_goldens_wavernn.py), and the Philox4x32-10
restatement against the published Random123 known-answer vectors.  CPU only."""
from pathlib import Path

import numpy as np
import pytest
import torch

from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict
from oracle import wr_torch_cpu as wr

G = Path(__file__).resolve().parent / 'golden'


def _keys():
    import json
    return json.loads((G / 'wavernn_state_dict_keys.json').read_text())


def _sd(mode='RAW'):
    keys = _keys()
    tmpl = {}
    for k, shape, dt in keys:
        if k == 'fc3.weight' and mode == 'MOL':
            shape = [30, shape[1]]
        if k == 'fc3.bias' and mode == 'MOL':
            shape = [30]
        tmpl[k] = np.zeros(shape, dtype=np.int64 if 'int' in dt else np.float32)
    return wr.to_torch(synthetic_state_dict(tmpl, model='wavernn'))


def _cfg(mode='RAW'):
    c = dict(default_config()['vocoder']['model'])
    c['mode'] = mode
    return c


def test_upsample_matches_reference():
    g = np.load(G / 'wr_upsample.npz')
    up, aux = wr.upsample(_sd(), torch.from_numpy(g['mels']), _cfg())
    np.testing.assert_array_equal(up.numpy(), g['up'])
    np.testing.assert_array_equal(aux.numpy(), g['aux'])


def test_forward_matches_reference():
    g = np.load(G / 'wr_forward.npz')
    logits = wr.forward(_sd(), _cfg(), torch.from_numpy(g['x']), torch.from_numpy(g['mels']))
    # same ATen kernels; the reference's flattened-weight GRU sums in another order (~1e-7 rel)
    np.testing.assert_allclose(logits.numpy(), g['logits'], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize('name', ['wr_gen_raw', 'wr_gen_unb', 'wr_gen_mol'])
def test_generate_matches_reference_draws(name):
    """Seeded with the reference's seed, the 'reference' sampler consumes torch's CPU
    generator exactly like WaveRNN.generate: the waveform is the reference's."""
    g = np.load(G / f'{name}.npz')
    mode = str(g['mode'])
    torch.manual_seed(int(g['seed']))
    wav = wr.generate(_sd(mode), _cfg(mode), torch.from_numpy(g['mels']), batched=bool(g['batched']),
                      target=int(g['target']), overlap=int(g['overlap']), mu_law=bool(g['mu_law']))
    assert wav.shape == g['wav'].shape
    np.testing.assert_allclose(wav, g['wav'], rtol=0, atol=1e-12)


def test_fold_and_xfade_known_answers():
    g = np.load(G / 'wr_fold.npz')
    np.testing.assert_array_equal(wr.fold_with_overlap(torch.from_numpy(g['x']), 2, 1).numpy(), g['folded'])
    np.testing.assert_array_equal(wr.xfade_and_unfold(g['y'], 100, 10), g['unfolded'])
    # the docstring example of fold_with_overlap (:311-317): 10 steps, target 2, overlap 1
    f = wr.fold_with_overlap(torch.arange(1, 11, dtype=torch.float32).view(1, 10, 1), 2, 1)
    assert f[:3, :, 0].tolist() == [[1, 2, 3, 4], [4, 5, 6, 7], [7, 8, 9, 10]]


def test_philox_known_answers():
    """Random123 kat_vectors, philox4x32_10: (counter, key) -> output."""
    cases = [((0, 0, 0, 0), 0, (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
             ((0xffffffff,) * 4, 0xffffffffffffffff, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
             ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), 0x299f31d0a4093822,
              (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in cases:
        got = wr.philox4x32(np.array([ctr], dtype=np.uint32), key)[0]
        assert tuple(int(v) for v in got) == want


def test_philox_sampler_is_a_categorical_draw():
    """The Gumbel form argmax(logit - log(-log u)) draws class k with probability
    softmax(logit)_k (chi-square over many independent (t, b) counters)."""
    logits = torch.tensor([[2.0, 1.0, 0.0, -1.0, 0.5, 1.5, -0.5, 0.25]])
    p = torch.softmax(logits, 1)[0].double().numpy()
    s = wr.PhiloxSampler(99)
    n = 20000
    counts = np.zeros(8)
    B = 500
    for t in range(n // B):
        z = s.gumbel_scores(logits.expand(B, 8), t)
        counts += np.bincount(np.argmax(z, 1), minlength=8)
    chi2 = float(((counts - n * p) ** 2 / (n * p)).sum())
    assert chi2 < 30.0, (chi2, counts, n * p)  # 7 dof: p(chi2 > 30) ~ 1e-4


def test_generate_bounded_steps_is_prefix():
    """steps= (the CPU baseline's bounded sample) returns the first samples of the folds."""
    g = np.load(G / 'wr_gen_raw.npz')
    s = wr.PhiloxSampler(3)
    a = wr.generate(_sd(), _cfg(), torch.from_numpy(g['mels']), target=600, overlap=60,
                    sampler=s, steps=40)
    b = wr.generate(_sd(), _cfg(), torch.from_numpy(g['mels']), target=600, overlap=60,
                    sampler=s, steps=20)
    np.testing.assert_array_equal(a[:, :20], b)
