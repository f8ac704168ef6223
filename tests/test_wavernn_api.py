"""The WaveRNN vocoder's drop-in surface on the CPU: state_dict keys / shapes / dtypes equal
the reference's (tests/golden/wavernn_state_dict_keys.json, written from the reference
classes), the constructor / from_config keywords, and the C ABI's argument errors for the
vocoder entry points (no GPU needed: they return before any launch)."""
import ctypes
import json

import pytest
import torch

from forwardtacotron_amd import _lib
from forwardtacotron_amd.synthetic import default_config, load_synthetic
from forwardtacotron_amd.wavernn import WaveRNN

from conftest import GOLDEN


def test_state_dict_matches_reference():
    ref = json.loads((GOLDEN / 'wavernn_state_dict_keys.json').read_text())
    m = WaveRNN.from_config(default_config())
    mine = [[k, list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()]
    assert mine == ref
    assert m.n_classes == 512 and m.aux_dims == 32 and m.get_step() == 0
    assert abs(m.num_params() - sum(v.numel() for k, v in m.state_dict().items()
                                    if k != 'step' and 'running' not in k and 'num_batches' not in k) / 1e6) < 1e-9


def test_mol_mode_and_synthetic_load():
    cfg = default_config()
    cfg['vocoder']['model']['mode'] = 'MOL'
    m = load_synthetic(WaveRNN.from_config(cfg), kind='wavernn')
    assert m.n_classes == 30 and m.fc3.weight.shape == (30, 512)
    assert torch.all(m.upsample.up_layers[1].weight == 1.0 / 9)


def test_checkpoint_roundtrip(tmp_path):
    m = load_synthetic(WaveRNN.from_config(default_config()), kind='wavernn')
    cfg = default_config()
    path = tmp_path / 'voc.pt'
    torch.save({'model': m.state_dict(), 'config': cfg}, path)
    m2 = WaveRNN.from_checkpoint(path)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_generate_refuses_short_mels():
    m = WaveRNN.from_config(default_config())
    with pytest.raises(ValueError):
        m.generate(torch.zeros(1, 80, 10), True, 11000, 550, True, seed=0)


def test_abi_argument_errors():
    L = _lib.load()
    a = _lib.WaveRNNArgs()
    assert L.ftmi_wavernn(None, None) == 1001
    assert L.ftmi_wavernn(ctypes.byref(a), None) == 1001
    assert L.ftmi_wavernn_workspace_bytes() > 0
    p = ctypes.c_void_p(256)
    assert L.ftmi_wr_stretch_conv(None, 0, 1, 4, 80, 4, None, None, 0, 16, 0, None) == 1001
    assert L.ftmi_wr_stretch_conv(p, 320, 1, 4, 80, 4, p, p, 1280, 16, 1, None) == 1002  # crop past the end
    assert L.ftmi_wr_unfold(None, 1, 10, 4, 3, 1, 0, 512, 10, 0, None, None) == 1001
    assert L.ftmi_wr_unfold(p, 2, 10, 4, 2, 1, 0, 512, 10, 0, p, None) == 1002  # L != target + 2 overlap
    assert L.ftmi_wr_unfold(p, 1, 10, 10, 0, 0, 1, 500, 10, 0, p, None) == 1003  # mu-law needs 2^bits
    assert L.ftmi_wr_unfold(p, 1, 10, 10, 0, 0, 0, 512, 10, 20, p, None) == 1002  # fade longer than the wave
    # unsupported architecture (rnn_dims != 512)
    for name in ('w_hh1', 'w_hh2', 'w_ih2a', 'w_fc1a', 'w_fc2a', 'w_fc3', 'b_fc3', 'b_hh1', 'b_hh2',
                 'u1', 'u2', 'v1', 'wm', 'cond', 'mel', 'workspace', 'samples'):
        setattr(a, name, 256)
    a.B, a.L, a.hop, a.item_rows, a.frames_per_item, a.n_classes = 1, 10, 256, 10, 1, 512
    a.rnn_dims, a.fc_dims, a.feat_dims, a.aux_dims = 256, 512, 80, 32
    assert L.ftmi_wavernn(ctypes.byref(a), None) == 1003
    a.rnn_dims, a.n_classes = 512, 500
    assert L.ftmi_wavernn(ctypes.byref(a), None) == 1003
