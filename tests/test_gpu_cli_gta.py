"""The §8(f) callers on the GPU: the gen_forward CLI end to end (tokens -> generate on the
HIP path -> .wav / .npy / .mel exactly as gen_forward.py:106-134 writes them) and the GTA
export (train_forward.py:33-50) over a collate_tts batch (utils/dataset.py:282-315)."""
import wave

import numpy as np
import pytest
import torch

from oracle import ft_oracle as O

pytestmark = pytest.mark.gpu


def test_cli_end_to_end(tmp_path, gpu_model, synth_sd):
    from forwardtacotron_amd import dsp as G
    from forwardtacotron_amd.gen_forward import main
    from forwardtacotron_amd.synthetic import default_config
    from oracle import dsp_oracle as D
    from oracle import ft_torch_cpu as TC
    ids = '12,40,7,88,23,5,61,19,33,2,77,45'
    outs = {}
    for voc in ('hifigan', 'melgan', 'griffinlim'):
        np.random.seed(7)  # the griffinlim vocoder draws its phases from np.random (librosa)
        (p,) = main(['--synthetic', '--input_tokens', ids, '--amp', '1.2', '--out',
                     str(tmp_path), voc])
        assert p.name.startswith('1_forward_0k_alpha1.0_amp1.2_' + voc)
        outs[voc] = p
    m = np.load(outs['hifigan'], allow_pickle=False)
    assert torch.equal(torch.load(outs['melgan'], weights_only=True), torch.from_numpy(m))
    x = torch.tensor([[int(v) for v in ids.split(',')]])
    ref = gpu_model.generate(x.cuda(), pitch_function=lambda v: v * 1.2)['mel_post'].cpu().numpy()
    assert m.shape == ref.shape == (1, 80, ref.shape[2])
    assert np.abs(m - ref).max() < 1e-5
    # the written mel against the torch-CPU restatement of the reference (gen_forward.py's
    # callbacks): the north-star bar, mean |d| < 1e-4
    cpu = TC.generate(TC.to_torch(synth_sd), x, pitch_function=lambda v: v * 1.2)['mel_post'].numpy()
    assert cpu.shape == m.shape and np.abs(m - cpu).mean() < 1e-4, np.abs(m - cpu).mean()
    # the .wav: 16-bit PCM of Griffin-Lim on the same seeded phases as the oracle's
    # librosa-0.7.2 iteration (np.random.seed(7) -> rand(513, T)), over the device NNLS
    # magnitudes (the NNLS minimiser itself is checked by its objective, test_gpu_dsp.py)
    with wave.open(str(outs['griffinlim']), 'rb') as w:
        assert w.getframerate() == 22050 and w.getsampwidth() == 2
        assert w.getnframes() == 256 * (m.shape[2] - 1)  # librosa istft length, center=True
        pcm = np.frombuffer(w.readframes(w.getnframes()), dtype='<i2').astype(np.float64) / 32767
    T = m.shape[2]
    plan = G.DSP.from_config(default_config()).plan()
    S = G.mel_to_stft(plan, torch.from_numpy(m).cuda())[0].cpu().numpy().T
    ang = np.exp(2j * np.pi * np.random.RandomState(7).rand(513, T)).astype(np.complex64)
    wref = D.griffinlim_from_stft(S, ang, n_iter=32)
    # save_wav clips to 16-bit PCM (the random-weight mel is far louder than full scale), so
    # each sample must lie between the quantised, clipped images of wref -+ the GL tolerance
    q = lambda v: np.clip(np.round(v * 32767.0), -32768, 32767) / 32767  # noqa: E731
    d = 1e-4 * np.abs(wref).max()
    lo, hi = q(wref.astype(np.float64) - d), q(wref.astype(np.float64) + d)
    assert ((pcm >= lo - 1.0 / 32767) & (pcm <= hi + 1.0 / 32767)).all()
    # the reference's `wavernn` sub-command (gen_forward.py:54-57, :125-131): batched
    # WaveRNN generation of the same mel, wave_len = (T - 1) hop
    (p,) = main(['--synthetic', '--input_tokens', ids, '--amp', '1.2', '--out', str(tmp_path),
                 'wavernn', '--voc_synthetic', '--target', '4000', '--overlap', '200'])
    assert p.name == '1_forward_0k_alpha1.0_amp1.2_wavernn.wav'
    with wave.open(str(p), 'rb') as w:
        assert w.getframerate() == 22050 and w.getnframes() == 256 * (m.shape[2] - 1)


def test_gta_export(tmp_path, gpu_model, synth_sd):
    from forwardtacotron_amd.gta import collate_tts, create_gta_features
    rng = np.random.Generator(np.random.PCG64(5))
    items = []
    for i, xl in enumerate((21, 14, 18)):
        dur = rng.integers(1, 6, xl).astype(np.float32)
        ml = int(dur.sum()) - int(rng.integers(0, 3))  # alignments may overshoot mel_len
        items.append({'x': rng.integers(1, 135, xl), 'mel': rng.normal(-4, 2, (80, ml)).astype(np.float32),
                      'item_id': f'LJ{i:03d}', 'x_len': xl, 'mel_len': ml, 'dur': dur,
                      'pitch': rng.normal(0, 1, xl).astype(np.float32),
                      'energy': rng.normal(0, 1, xl).astype(np.float32)})
    batch = collate_tts(items, r=1)
    n = create_gta_features(gpu_model, [batch], [], tmp_path)
    assert n == 3
    host = {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}
    truth = O.forward(synth_sd, {k: host[k] for k in ('x', 'mel', 'mel_len', 'dur', 'pitch', 'energy')},
                      np.float64)['mel_post']
    ref32 = O.forward(synth_sd, {k: host[k] for k in ('x', 'mel', 'mel_len', 'dur', 'pitch', 'energy')},
                      np.float32)['mel_post']
    for j, it in enumerate(items):
        g = np.load(tmp_path / f'{it["item_id"]}.npy', allow_pickle=False)
        assert g.shape == (80, it['mel_len'])
        t, r = truth[j][:, :it['mel_len']], ref32[j][:, :it['mel_len']]
        e_ref = np.abs(r - t).max()
        assert np.abs(g - t).max() <= 4 * e_ref + 1e-4, (j, np.abs(g - t).max(), e_ref)
