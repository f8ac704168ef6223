"""WaveRNN vocoder on the GPU (csrc/wavernn.hip through the C ABI) against the oracle
(oracle/wr_torch_cpu.py, itself pinned bit-exactly against the reference classes by
tests/test_oracle_wavernn.py) and the reference goldens.

Parity bars:
  * upsampling network: rtol 1e-5 (f16x3 GEMMs for the resnet convolutions, BatchNorm
    folded into them: fp32-level);
  * teacher-forced logits (WaveRNN.forward): |diff| <= 2e-4 + 2e-5 |logit| — the sample
    loop is exact fp32 FMAs but the conditioning is re-associated (products of the linear
    layers folded in float64, tagged exchange values: <= 1 ulp each);
  * generate: the draws are the Philox stream the oracle restates.  The oracle, fed the
    GPU's own sample sequence (teacher-forced on it), recomputes every step's logits and
    Gumbel scores; every GPU choice must be the oracle's argmax or within 1e-3 of it (a
    near-tie that fp32 rounding may decide either way), with >= 99.5 % exact choices; the
    waveform equals the oracle's tail (mu-law, crossfade, fade-out) applied to the GPU
    samples to 1e-12.
"""
import numpy as np
import pytest
import torch

from forwardtacotron_amd import ops
from forwardtacotron_amd.synthetic import default_config, load_synthetic
from forwardtacotron_amd.wavernn import WaveRNN
from oracle import wr_torch_cpu as wr

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _model(mode='RAW'):
    cfg = default_config()
    cfg['vocoder']['model']['mode'] = mode
    m = WaveRNN.from_config(cfg)
    load_synthetic(m, kind='wavernn')
    return m.to(DEV).eval(), cfg


def _sd(m):
    return wr.to_torch({k: v.detach().cpu() for k, v in m.state_dict().items()})


def _cfg(cfg):
    return dict(cfg['vocoder']['model'])


def test_upsample_matches_reference():
    g = load_golden('wr_upsample')
    m, _ = _model()
    up, aux = m.upsample_forward(torch.from_numpy(g['mels']).to(DEV))
    # fp32-level: the GEMM path's summation order, scaled by each output's magnitude
    for got, ref in ((up, g['up']), (aux, g['aux'])):
        np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-5, atol=2e-6 * np.abs(ref).max())


def test_forward_logits_match_reference():
    g = load_golden('wr_forward')
    m, _ = _model()
    logits = m.forward(torch.from_numpy(g['x']), torch.from_numpy(g['mels'])).cpu().numpy()
    ref = g['logits']
    err = np.abs(logits - ref)
    assert np.all(err <= 2e-4 + 2e-5 * np.abs(ref)), (err.max(), np.abs(ref).max())
    assert err.mean() < 2e-5


def _check_draws(m, cfg, mels, seed, target, overlap, batched=True):
    smp = m.generate_samples(torch.from_numpy(mels), batched, target, overlap, seed=seed).cpu().numpy()
    trace = []
    sd = _sd(m)
    wr.generate(sd, _cfg(cfg), torch.from_numpy(mels), batched=batched, target=target,
                overlap=overlap, forced=smp, trace=trace, steps=smp.shape[1])
    sampler = wr.PhiloxSampler(seed)
    nc = m.n_classes
    exact = total = 0
    for t, logits in enumerate(trace):
        if m.mode == 'RAW':
            z = sampler.gumbel_scores(logits, t)
            idx = np.rint((smp[:, t] + 1.0) * (nc - 1) / 2.0).astype(np.int64)
            best = z.max(axis=1)
            got = z[np.arange(z.shape[0]), idx]
            assert np.all(best - got <= 1e-3), (t, (best - got).max())
            exact += int(np.sum(np.argmax(z, axis=1) == idx))
        else:
            tu, u = sampler.mol_uniforms(t, logits.size(0), nc // 3)
            x = wr.sample_mol(logits, tu, u).numpy()
            close = np.abs(x - smp[:, t]) <= 1e-4 + 1e-4 * np.abs(x)
            exact += int(close.sum())
        total += logits.size(0)
    assert exact >= 0.995 * total, (exact, total)
    return smp


def test_generate_raw_draws_match_oracle():
    g = load_golden('wr_gen_raw')
    m, cfg = _model()
    smp = _check_draws(m, cfg, g['mels'], 1234, 600, 60)
    wav = m.generate(torch.from_numpy(g['mels']), True, 600, 60, True, seed=1234)
    ref = wr.finish(smp.astype(np.float64), True, 600, 60, True, m.n_classes,
                    (g['mels'].shape[-1] - 1) * 256, 256)
    assert wav.dtype == np.float64 and wav.shape == ref.shape == g['wav'].shape
    np.testing.assert_allclose(wav, ref, rtol=0, atol=1e-12)
    # same seed -> same waveform (the stream is counter-based)
    wav2 = m.generate(torch.from_numpy(g['mels']), True, 600, 60, True, seed=1234)
    np.testing.assert_array_equal(wav, wav2)


def test_generate_unbatched_matches_oracle():
    g = load_golden('wr_gen_unb')
    m, cfg = _model()
    smp = _check_draws(m, cfg, g['mels'], 77, 600, 60, batched=False)
    wav = m.generate(torch.from_numpy(g['mels']), False, 600, 60, False, seed=77)
    ref = wr.finish(smp.astype(np.float64), False, 600, 60, False, m.n_classes,
                    (g['mels'].shape[-1] - 1) * 256, 256)
    np.testing.assert_allclose(wav, ref, rtol=0, atol=1e-12)


def test_generate_mol_matches_oracle():
    g = load_golden('wr_gen_mol')
    m, cfg = _model('MOL')
    smp = _check_draws(m, cfg, g['mels'], 5, 400, 40)
    assert np.all(np.abs(smp) <= 1.0)  # clamp(x, -1, 1) of distribution.py:125
    wav = m.generate(torch.from_numpy(g['mels']), True, 400, 40, True, seed=5)  # mu_law ignored (MOL)
    ref = wr.finish(smp.astype(np.float64), True, 400, 40, False, m.n_classes,
                    (g['mels'].shape[-1] - 1) * 256, 256)
    assert wav.shape == ref.shape == g['wav'].shape
    np.testing.assert_allclose(wav, ref, rtol=0, atol=1e-12)


def test_generate_many_folds_two_launches():
    """More than 32 folds: the loop runs in launches of <= 32 folds; fold 32 onward must
    still follow the Philox stream of its global fold index."""
    rng = np.random.Generator(np.random.PCG64(5))
    mels = (rng.normal(0, 1, (1, 80, 40)) - 4).astype(np.float32)
    m, cfg = _model()
    smp = _check_draws(m, cfg, mels, 9, 200, 20)  # (40 * 256 - 20) // 220 + 1 = 47 folds
    assert smp.shape[0] > 32


def test_xfade_and_unfold_matches_reference():
    g = load_golden('wr_fold')
    m, _ = _model()
    y = g['y'].astype(np.float32)
    got = m.xfade_and_unfold(y, 100, 10)
    np.testing.assert_allclose(got, wr.xfade_and_unfold(y.astype(np.float64), 100, 10), rtol=0, atol=1e-15)


def test_recurrence_timeout_raises():
    """A spin limit of 1 makes the co-residency barrier give up: the call must raise, not
    return a silent result."""
    g = load_golden('wr_gen_raw')
    m, _ = _model()
    lib = __import__('forwardtacotron_amd._lib', fromlist=['load']).load()
    old = lib.ftmi_set_wavernn_spin_limit(1)
    try:
        with pytest.raises(ops.RnnTimeout):
            m.generate_samples(torch.from_numpy(g['mels']), True, 600, 60, seed=1)
    finally:
        lib.ftmi_set_wavernn_spin_limit(old)
    torch.cuda.synchronize()
