"""End-to-end parity of the HIP ForwardTacotron against the REFERENCE's golden outputs
(tests/golden, made by running /root/reference) and, at the BASELINE size (B = 64,
T = 200), against the torch-CPU restatement of the reference run on the box.

Bounds (north star: mel frames within 1e-4 fp32, LengthRegulator bit-exact):
  mean |mel_post - ref| < 1e-4, mean |mel - ref| < 1e-4, max |.| < 2e-3 (|mel| ~ 5),
  durations to 1e-5 and LengthRegulator counts identical (=> identical T_mel).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import ft_oracle as O

pytestmark = pytest.mark.gpu

MEAN_TOL, MAX_TOL = 1e-4, 2e-3


def check(out, g, mean_tol=MEAN_TOL, max_tol=MAX_TOL):
    for k in ('mel', 'mel_post'):
        got = out[k].float().cpu().numpy()
        assert got.shape == g[k].shape, (k, got.shape, g[k].shape)
        d = np.abs(got - g[k])
        assert d.mean() < mean_tol and d.max() < max_tol, (k, d.mean(), d.max())
    np.testing.assert_allclose(out['dur'].cpu().numpy(), g['dur'], atol=1e-5)
    assert np.array_equal(O.duration_counts(out['dur'].cpu().numpy()), O.duration_counts(g['dur']))
    np.testing.assert_allclose(out['pitch'].cpu().numpy(), g['pitch'], atol=1e-5)
    np.testing.assert_allclose(out['energy'].cpu().numpy(), g['energy'], atol=1e-5)


CASES = {
    'gen_b1': dict(alpha=1.0),
    'gen_b3': dict(alpha=1.0),
    'gen_alpha': dict(alpha=0.8),
    'gen_fill2': dict(alpha=1000.0),
    'gen_callbacks': dict(alpha=1.2, pitch_function=lambda p: p * 2.0 + 0.1,
                          energy_function=lambda e: e - 0.05),
}


@pytest.mark.parametrize('name', sorted(CASES))
def test_generate_matches_reference(name, gpu_model):
    g = load_golden(name)
    out = gpu_model.generate(torch.from_numpy(g['x']).cuda(), **CASES[name])
    check(out, g)


def test_generate_jit_matches_reference(gpu_model):
    g = load_golden('gen_jit')
    check(gpu_model.generate_jit(torch.from_numpy(g['x']).cuda(), alpha=1.1, beta=0.7), g)


def test_intermediates_b1(gpu_model):
    g = load_golden('gen_b1')
    x = torch.from_numpy(g['x']).cuda()
    h = gpu_model.prenet.forward_cl(gpu_model.embedding(x))
    np.testing.assert_allclose(h.cpu().numpy(), g['prenet'], atol=5e-5, rtol=1e-4)
    d = gpu_model.dur_pred.forward_bt(x)
    np.testing.assert_allclose(d.cpu().numpy(), g['dur_raw'], atol=1e-5)


def test_forward_teacher_forced(gpu_model):
    g = load_golden('forward')
    batch = {'x': torch.from_numpy(g['x']).cuda(), 'mel': torch.from_numpy(g['mel_in']).cuda(),
             'mel_len': torch.from_numpy(g['mel_len']), 'dur': torch.from_numpy(g['dur_in']).cuda(),
             'pitch': torch.from_numpy(g['pitch_in']).cuda(),
             'energy': torch.from_numpy(g['energy_in']).cuda()}
    out = gpu_model(batch)
    for k in ('dur', 'pitch', 'energy'):
        np.testing.assert_allclose(out[k].squeeze().cpu().numpy(), g[k].squeeze(), atol=1e-5)
    mel = out['mel'].cpu().numpy()
    assert np.abs(mel - g['mel']).max() / np.abs(g['mel']).max() < 2e-6
    # ill-conditioned padded frames, see tests/test_oracle.py::test_numpy_oracle_forward
    d = np.abs(out['mel_post'].cpu().numpy() - g['mel_post'])
    assert d.max() < 0.1 and d.mean() < 2e-3
    T_pack = int(g['mel_len'].max())
    assert np.all(mel[:, :, T_pack:] == np.float32(-11.5129))


def test_length_regulator_layer_api(gpu_model):
    """Reference LengthRegulator semantics: dur clipped in place, zero padding."""
    g = load_golden('lr_random')
    d = torch.from_numpy(g['dur_in']).cuda()
    y = gpu_model.lr(torch.from_numpy(g['x']).cuda(), d)
    assert np.array_equal(y.cpu().numpy(), g['out'])
    assert np.array_equal(d.cpu().numpy(), g['dur_out'])


def test_f16_range_guard_reruns_exact(gpu_model):
    """A pitch callback that drives the encoder beyond the f16 range: the f16x3 GEMMs flag
    it, generate() reruns on the exact paths, and the result equals an exact-path run."""
    from forwardtacotron_amd import ops
    g = load_golden('gen_b3')
    x = torch.from_numpy(g['x']).cuda()
    big = dict(pitch_function=lambda p: p * 0 + 1e7)
    out = gpu_model.generate(x, **big)
    assert int(ops.status_word(x.device).item()) != 0
    with ops.exact_paths():
        ref = gpu_model.generate(x, **big)
    for k in ('mel', 'mel_post', 'dur'):
        assert torch.equal(out[k], ref[k]), k
    out = gpu_model.generate(x)  # in range: the word is cleared and stays clear
    assert int(ops.status_word(x.device).item()) == 0


def test_repeated_calls_deterministic(gpu_model):
    g = load_golden('gen_b3')
    x = torch.from_numpy(g['x']).cuda()
    a = gpu_model.generate(x)['mel_post']
    b = gpu_model.generate(x)['mel_post']
    assert torch.equal(a, b)


@pytest.mark.slow
def test_baseline_size_vs_torch_cpu(gpu_model, synth_sd):
    """BASELINE c3 workload (B = 64, T = 200, lengths U{50..200}) on the GPU vs the
    torch-CPU restatement of the reference on the same inputs."""
    from forwardtacotron_amd.synthetic import synthetic_tokens
    from oracle import ft_torch_cpu as TC
    x = synthetic_tokens(64, 200, seed=0, min_len=50)
    out = gpu_model.generate(torch.from_numpy(x).cuda())
    ref = TC.generate(TC.to_torch(synth_sd), torch.from_numpy(x))
    dur_g, dur_r = out['dur'].cpu().numpy(), ref['dur'].numpy()
    np.testing.assert_allclose(dur_g, dur_r, atol=1e-4)
    assert np.array_equal(O.duration_counts(dur_g), O.duration_counts(dur_r))
    for k in ('mel', 'mel_post'):
        a, b = out[k].cpu().numpy(), ref[k].numpy()
        assert a.shape == b.shape
        d = np.abs(a - b)
        assert d.mean() < MEAN_TOL and d.max() < 5e-3, (k, d.mean(), d.max())


def test_graph_phase_matches_eager(gpu_model, monkeypatch):
    """generate() with the default callbacks replays the phoneme phase as a HIP graph:
    results identical (bit for bit) to the eager phase, across replays with new tokens of
    the same shape, and the returned dur / pitch / energy are not the graph's buffers."""
    from forwardtacotron_amd import forward_tacotron as FT
    g = load_golden('gen_b3')
    x1 = torch.from_numpy(g['x']).cuda()
    x2 = x1.clone()
    x2[x2 > 0] = (x2[x2 > 0] * 7) % 133 + 1  # other phonemes, same padding
    monkeypatch.setattr(FT, 'GRAPH', False)
    eager = [gpu_model.generate(x) for x in (x1, x2)]
    monkeypatch.setattr(FT, 'GRAPH', True)
    graph = [gpu_model.generate(x) for x in (x1, x2, x1)]
    assert graph[0]['dur'].data_ptr() != graph[2]['dur'].data_ptr()
    for e, gr in ((eager[0], graph[0]), (eager[1], graph[1]), (eager[0], graph[2])):
        for k in ('mel', 'mel_post', 'dur', 'pitch', 'energy'):
            assert torch.equal(e[k], gr[k]), k
    # the first result survived the later replays untouched
    assert torch.equal(graph[0]['dur'], eager[0]['dur'])
