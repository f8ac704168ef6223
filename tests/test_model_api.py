"""The drop-in boundary on CPU: reference state_dict format, constructor / factory surface,
checkpoint round trip, and the no-CPU-fallback rule."""
import copy
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from forwardtacotron_amd.checkpoints import init_tts_model, restore_checkpoint, save_checkpoint
from forwardtacotron_amd.forward_tacotron import ForwardTacotron
from forwardtacotron_amd.synthetic import default_config, load_synthetic
from forwardtacotron_amd.text import Tokenizer, phonemes


def test_state_dict_matches_reference_exactly():
    ref = json.loads((GOLDEN / 'state_dict_keys.json').read_text())
    m = ForwardTacotron.from_config(default_config())
    got = [[k, list(v.shape), str(v.dtype).replace('torch.', '')] for k, v in m.state_dict().items()]
    assert got == ref  # same keys, order, shapes, dtypes
    assert repr(m) == 'ForwardTacotron, num params: 24509235'


def test_from_config_mutates_like_reference():
    cfg = default_config()
    ForwardTacotron.from_config(cfg)
    assert cfg['forward_tacotron']['model']['num_chars'] == len(phonemes) == 135
    assert cfg['forward_tacotron']['model']['n_mels'] == 80


def test_init_tts_model_and_errors():
    assert isinstance(init_tts_model(default_config()), ForwardTacotron)
    cfg = default_config()
    cfg['tts_model'] = 'nope'
    with pytest.raises(ValueError):
        init_tts_model(cfg)


def test_checkpoint_round_trip(tmp_path):
    m = load_synthetic(ForwardTacotron.from_config(default_config()), seed=3)
    p = tmp_path / 'latest_model.pt'
    save_checkpoint(m, None, default_config(), p)
    m2 = ForwardTacotron.from_checkpoint(p)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    m3 = ForwardTacotron.from_config(default_config())
    restore_checkpoint(m3, None, p, torch.device('cpu'))
    assert m3.get_step() == 0


def test_no_cpu_fallback():
    m = ForwardTacotron.from_config(default_config())
    with pytest.raises(RuntimeError, match='HIP device'):
        m.generate(torch.zeros(1, 5, dtype=torch.long))


def test_tokenizer_reference_vectors():
    # reference tests/test_tokenizer.py:8-14
    t = Tokenizer()
    tokens = t('_ abc{')
    assert tokens == [0, 10, 36, 52, 57]
    assert t.decode(tokens) == '_ abc'


def test_synthetic_recipe_is_deterministic():
    from forwardtacotron_amd.synthetic import synthetic_array
    a = synthetic_array('lstm.weight_hh_l0', (2048, 512), 'float32', 0)
    b = synthetic_array('lstm.weight_hh_l0', (2048, 512), 'float32', 0)
    assert np.array_equal(a, b) and a.dtype == np.float32
    assert not np.array_equal(a, synthetic_array('lstm.weight_hh_l0', (2048, 512), 'float32', 1))


def test_init_tts_model_fast_pitch():
    """utils/checkpoints.py:32-40 with tts_model: fast_pitch -> FastPitch with the reference's
    state_dict keys (CPU construction only; compute needs the GPU)."""
    import json
    from forwardtacotron_amd.checkpoints import init_tts_model
    from forwardtacotron_amd.fast_pitch import FastPitch
    from forwardtacotron_amd.synthetic import default_config
    cfg = default_config()
    cfg['tts_model'] = 'fast_pitch'
    m = init_tts_model(cfg)
    assert isinstance(m, FastPitch)
    keys = json.loads((GOLDEN / 'fastpitch_state_dict_keys.json').read_text())
    assert list(m.state_dict()) == [k for k, _, _ in keys]
    assert repr(m) == 'FastPitch, num params: 25974360'


def test_fast_pitch_cpu_raises():
    import torch
    from forwardtacotron_amd.fast_pitch import FastPitch
    from forwardtacotron_amd.synthetic import default_config
    m = FastPitch.from_config(default_config())
    with pytest.raises(RuntimeError):
        m.generate(torch.ones(1, 5, dtype=torch.long))


def test_dsp_api_surface():
    """utils/dsp.py:12-165: constructor, from_config, helpers that need no device."""
    import numpy as np
    from forwardtacotron_amd.dsp import DSP
    from forwardtacotron_amd.synthetic import default_config
    d = DSP.from_config(default_config())
    assert (d.n_mels, d.sample_rate, d.hop_length, d.n_fft) == (80, 22050, 256, 1024)
    x = np.linspace(-1, 1, 9)
    np.testing.assert_allclose(d.decode_mu_law(d.encode_mu_law(x, 512), 512, from_labels=True),
                               x, atol=0.02)
    np.testing.assert_allclose(d.label_2_float(d.float_2_label(x, 9), 9), x, atol=1e-12)
    np.testing.assert_allclose(d.denormalize(d.normalize(np.array([1e-7, 0.5]))), [1e-5, 0.5])
    with pytest.raises(RuntimeError):
        d.wav_to_mel(__import__('torch').zeros(4000))


@pytest.mark.parametrize('kind', ['fast_pitch', 'wavernn'])
def test_torchscript_export_fails_with_reason(kind):
    """The reference scripts only ForwardTacotron (README.md:149-161, the one
    @torch.jit.export); FastPitch / WaveRNN on the HIP path cannot be scripted (ctypes
    calls), and say so instead of a TorchScript frontend error."""
    from forwardtacotron_amd.checkpoints import init_tts_model
    from forwardtacotron_amd.synthetic import default_config
    from forwardtacotron_amd.wavernn import WaveRNN
    cfg = default_config()
    cfg['tts_model'] = kind if kind != 'wavernn' else 'forward_tacotron'
    m = WaveRNN.from_config(cfg) if kind == 'wavernn' else init_tts_model(cfg)
    with pytest.raises(RuntimeError, match='cannot be compiled by torch.jit.script'):
        torch.jit.script(m)


def test_torchscript_forward_tacotron(tmp_path):
    """README.md:149-161 verbatim (from_checkpoint, eval, torch.jit.script, generate_jit on a
    CPU tensor) scripts ForwardTacotron: the ScriptModule carries the constructor keywords and
    every weight (sharing the eager model's storage), its forward / generate_jit call the
    ftmi dispatcher operators with them, and a torch.jit.save / load round trip keeps all of
    it.  Without a GPU (this suite) the call reaches the operator's kernel, which refuses with
    the reason; tests/test_gpu_model.py runs it (also from a fresh process)."""
    from forwardtacotron_amd.forward_tacotron import ForwardTacotron
    from forwardtacotron_amd.synthetic import default_config
    cfg = default_config()
    path = tmp_path / 'latest_model.pt'
    torch.save({'model': ForwardTacotron.from_config(cfg).state_dict(), 'config': cfg}, path)
    # README.md:149-161
    tts_model = ForwardTacotron.from_checkpoint(path)
    tts_model.eval()
    model_script = torch.jit.script(tts_model)
    x = torch.ones((1, 5)).long()
    assert isinstance(model_script, torch.jit.ScriptModule)
    assert 'ftmi.ft_generate_jit' in model_script.generate_jit.code
    assert 'ftmi.ft_forward' in model_script.code
    sd = tts_model.state_dict()
    keys = json.loads(model_script.config)['keys']
    assert keys == [k for k in sd if k != 'step']
    for k, w in zip(keys, model_script.weights):
        assert w.data_ptr() == sd[k].data_ptr(), k  # shares the eager model's storage
    buf = tmp_path / 'scripted.pt'
    torch.jit.save(model_script, str(buf))
    loaded = torch.jit.load(str(buf))
    assert loaded.config == model_script.config
    for k, w in zip(keys, loaded.weights):
        assert torch.equal(w, sd[k]), k
    assert 'ftmi.ft_generate_jit' in loaded.generate_jit.code
    if not torch.cuda.is_available():
        for mod in (model_script, loaded):
            with pytest.raises(RuntimeError, match='computes on a HIP device'):
                mod.generate_jit(x)
    # the archive rebuilds the same eager model (CPU: construct + load_state_dict only)
    kw = json.loads(loaded.config)['kwargs']
    m2 = ForwardTacotron(**kw)
    m2.load_state_dict(dict(zip(keys, loaded.weights), step=loaded.step))
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k]), k


def test_torchscript_archive_loads_in_a_fresh_process(tmp_path):
    """a torch.jit.save'd archive is self-contained — a fresh Python
    process that imports forwardtacotron_amd (which registers the ftmi operators) loads it and
    finds the weights and the configuration (the computation itself: test_gpu_model.py)."""
    import subprocess
    import sys
    from forwardtacotron_amd.forward_tacotron import ForwardTacotron
    from forwardtacotron_amd.synthetic import default_config
    m = ForwardTacotron.from_config(default_config()).eval()
    with torch.no_grad():
        m.lin.weight.normal_()
    arc = tmp_path / 'tts.pt'
    torch.jit.save(torch.jit.script(m), str(arc))
    expect = float(m.lin.weight.double().sum())
    code = ('import json, sys, torch, forwardtacotron_amd\n'
            f'l = torch.jit.load({str(arc)!r})\n'
            'keys = json.loads(l.config)["keys"]\n'
            'w = dict(zip(keys, l.weights))\n'
            'print(len(keys), float(w["lin.weight"].double().sum()), l.step.item())\n')
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300,
                       cwd=str(GOLDEN.parent.parent))
    assert r.returncode == 0, r.stderr[-2000:]
    n, s, step = r.stdout.split()
    assert int(n) == len(m.state_dict()) - 1 and float(s) == expect and int(step) == 0


def test_torchscript_train_mode_steps():
    """The reference's forward increments step in training mode (forward_tacotron.py:200-201);
    the scripted module shares step with the eager model."""
    from forwardtacotron_amd.forward_tacotron import ForwardTacotron
    from forwardtacotron_amd.synthetic import default_config
    m = ForwardTacotron.from_config(default_config())
    s = torch.jit.script(m)
    assert s.training and 'step' in s.code
    assert s.step.data_ptr() == m.step.data_ptr()


def test_run_checked_checks_the_rerun(monkeypatch):
    """the exact-path rerun after a range bit is status-checked like the first
    pass (a timeout there raises RnnTimeout; reduce applies to it too); a clean rerun
    returns the rerun's output."""
    from forwardtacotron_amd import ops
    st = torch.zeros(1, dtype=torch.int32)
    monkeypatch.setattr(ops, 'status_word', lambda device: st)

    def pass_bits(*bits):
        calls = []

        def fn():
            calls.append(ops.forced_exact())
            st.fill_(bits[len(calls) - 1])
            return len(calls)
        return fn, calls

    fn, calls = pass_bits(1, ops.STATUS_RNN_TIMEOUT)
    with pytest.raises(ops.RnnTimeout):
        ops.run_checked(fn, 'cpu')
    assert calls == [False, True]
    fn, calls = pass_bits(2, 0)
    assert ops.run_checked(fn, 'cpu') == 2 and calls == [False, True]
    assert int(st.item()) == 2  # the word keeps the bits that caused the rerun
    fn, calls = pass_bits(0)
    assert ops.run_checked(fn, 'cpu') == 1 and calls == [False]
    # a reduce (sharded generation) sees the rerun's word as well
    seen = []
    fn, calls = pass_bits(1, 0)
    red = lambda w: (seen.append(int(w)), torch.full_like(w, ops.STATUS_RNN_TIMEOUT if len(seen) == 2 else int(w)))[1]  # noqa: E731
    with pytest.raises(ops.RnnTimeout):
        ops.run_checked(fn, 'cpu', reduce=red)
    assert seen == [1, 0]
