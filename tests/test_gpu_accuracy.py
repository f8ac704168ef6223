"""Accuracy of the HIP path at the BASELINE sizes against a float64 truth, and the BASELINE
configs exactly as their callers run them (on the GPU box; the checkers are the torch-CPU
restatements of the reference, oracle/ft_torch_cpu.py and oracle/fp_torch_cpu.py).

fp64 truth: the reference's network in float64 (same ATen CPU kernels, weights converted),
with the LengthRegulator fed the fp32 reference's durations so both follow the same frame
counts.  The claim under test is "fp32-level": the default path (f16x3 MFMA split, step-
tagged h exchange) and the exact fp32-MFMA path are each no further from the fp64 truth
than the fp32 reference itself, within the factors below (measured margins in DESIGN.md §6).

Every measured statistic is also written to gpurun_out/accuracy_<case>.json.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ft_oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# |path - fp64| <= FACTOR * |fp32 reference - fp64| (+ FLOOR, an absolute allowance of a
# few fp32 ulps of |mel| ~ 5 for where the fp32 reference happens to be exact).
# Measured (round 2, mel_post, c3): fp32 reference mean 1.05e-5 / max 1.23e-4; default
# f16x3 path 1.03e-5 / 9.4e-5 (no worse than fp32); exact fp32-MFMA path 1.84e-5 / 1.80e-4
# (c2: 1.53e-5 / 1.02e-4 against 7.1e-6 / 4.9e-5; c2 mel max up to 3.8x) — a different
# summation order; the max over the 65 k values of c2 is the noisiest statistic.
FACTORS = {'default': (1.5, 2.0), 'exact_fp32_mfma': (3.0, 5.0)}  # (mean, max)
FLOOR = 2e-6


def _record(name, stats):
    out = os.path.join(ROOT, 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f'accuracy_{name}.json'), 'w') as f:
        json.dump(stats, f, indent=1)
    print(name, json.dumps(stats))


def _err(a, truth):
    d = np.abs(np.asarray(a, np.float64) - truth)
    return {'mean': float(d.mean()), 'max': float(d.max())}


CONFIGS = {
    'c2': dict(B=1, T=120, tmin=120),   # BASELINE configs[1]
    'c3': dict(B=64, T=200, tmin=50),   # BASELINE configs[2]
}


@pytest.mark.slow
@pytest.mark.parametrize('cfg', sorted(CONFIGS))
def test_accuracy_vs_fp64(cfg, gpu_model, synth_sd):
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.synthetic import synthetic_tokens
    from oracle import ft_torch_cpu as TC
    c = CONFIGS[cfg]
    x = synthetic_tokens(c['B'], c['T'], seed=0, min_len=c['tmin'])
    xt = torch.from_numpy(x)
    ref32 = TC.generate(TC.to_torch(synth_sd), xt)
    ref64 = TC.generate(TC.to_torch(synth_sd, torch.float64), xt, lr_dur=ref32['dur'])
    xd = xt.cuda()
    outs = {'default': gpu_model.generate(xd)}
    with ops.exact_paths():
        outs['exact_fp32_mfma'] = gpu_model.generate(xd)
    stats = {'config': cfg, 'B': c['B'], 'T': int(x.shape[1])}
    for name, o in outs.items():
        assert np.array_equal(O.duration_counts(o['dur'].cpu().numpy()),
                              O.duration_counts(ref32['dur'].numpy())), name
    for k in ('mel', 'mel_post'):
        truth = ref64[k].numpy()
        e_ref = _err(ref32[k].numpy(), truth)
        stats[k] = {'fp32_reference': e_ref}
        for name, o in outs.items():
            got = o[k].cpu().numpy()
            assert got.shape == truth.shape
            stats[k][name] = _err(got, truth)
    _record(cfg, stats)
    for k in ('mel', 'mel_post'):
        e_ref = stats[k]['fp32_reference']
        for name in outs:
            e = stats[k][name]
            f_mean, f_max = FACTORS[name]
            assert e['mean'] <= f_mean * e_ref['mean'] + FLOOR, (k, name, e, e_ref)
            assert e['max'] <= f_max * e_ref['max'] + FLOOR, (k, name, e, e_ref)


def test_c2_as_gen_forward_calls_it(gpu_model, synth_sd):
    """BASELINE c2 exactly as gen_forward.py:103-118 runs it: batch 1, 120 phonemes,
    `pitch_function = lambda x: x * args.amp`, `energy_function = lambda x: x`, the same
    callback objects on every call (so the phase is captured on the second call and
    replayed on the third) — each call against the torch-CPU reference at the north-star
    bar (mean |mel_post - ref| < 1e-4; LR counts equal)."""
    from forwardtacotron_amd.synthetic import synthetic_tokens
    from oracle import ft_torch_cpu as TC
    amp = 1.3
    pitch_function = lambda x: x * amp  # noqa: E731  (gen_forward.py:103)
    energy_function = lambda x: x       # noqa: E731  (gen_forward.py:104)
    x = torch.from_numpy(synthetic_tokens(1, 120, seed=3, min_len=120))
    ref = TC.generate(TC.to_torch(synth_sd), x, alpha=1.0, pitch_function=pitch_function,
                      energy_function=energy_function)
    stats = []
    for _ in range(3):
        out = gpu_model.generate(x=x.cuda(), alpha=1.0, pitch_function=pitch_function,
                                 energy_function=energy_function)
        m = out['mel_post'].cpu()  # gen_forward.py:120
        assert m.shape == ref['mel_post'].shape
        d = np.abs(m.numpy() - ref['mel_post'].numpy())
        stats.append({'mean': float(d.mean()), 'max': float(d.max())})
        assert d.mean() < 1e-4 and d.max() < 5e-4, stats[-1]
        assert np.array_equal(O.duration_counts(out['dur'].cpu().numpy()),
                              O.duration_counts(ref['dur'].numpy()))
        np.testing.assert_allclose(out['pitch'].cpu().numpy(), ref['pitch'].numpy(), atol=1e-5)
    _record('c2_gen_forward', {'calls': stats})


@pytest.mark.slow
def test_c5_fastpitch_full_size():
    """BASELINE c5: FastPitch, batch 64, 200 phonemes (lengths U{50..200}) against the
    torch-CPU restatement of the reference (padding masks, postnet attention at T_mel ~1.4k)."""
    from forwardtacotron_amd.fast_pitch import FastPitch
    from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict, synthetic_tokens
    from oracle import fp_oracle as FPO
    from oracle import fp_torch_cpu as FTC
    m = FastPitch.from_config(default_config())
    sd = synthetic_state_dict(m, 0, 'fast_pitch')
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    x = torch.from_numpy(synthetic_tokens(64, 200, seed=0, min_len=50))
    out = m.generate(x.cuda())
    ref = FTC.generate(FTC.to_torch(sd), x)
    assert np.array_equal(FPO.duration_counts(out['dur'].cpu().numpy()),
                          FPO.duration_counts(ref['dur'].numpy()))
    got, r = out['mel'].cpu().numpy(), ref['mel'].numpy()
    assert got.shape == r.shape
    d = np.abs(got - r)
    _record('c5', {'T_mel': int(r.shape[2]), 'mel_mean': float(d.mean()), 'mel_max': float(d.max())})
    assert d.mean() < 1e-4 and d.max() < 5e-4
