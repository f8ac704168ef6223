"""The callers either side of the path, on CPU: the GTA batch format (collate_tts) against
the reference's own collate_tts (golden made by tests/golden/make_goldens_gta.py), and the
gen_forward CLI's output formats / names / input handling (gen_forward.py:40-136)."""
import numpy as np
import pytest
import torch

from conftest import load_golden


def _items(z):
    out = []
    for i in range(3):
        it = {k: z[f'in{i}_{k}'] for k in ('x', 'mel', 'x_len', 'mel_len', 'dur', 'pitch', 'energy')}
        it['x_len'], it['mel_len'] = int(it['x_len']), int(it['mel_len'])
        it['item_id'] = f'LJ{i:03d}'
        out.append(it)
    return out


@pytest.mark.parametrize('r', [1, 2, 3])
def test_collate_tts_matches_reference(r):
    from forwardtacotron_amd.gta import collate_tts
    z = load_golden('gta_collate')
    b = collate_tts(_items(z), r)
    for k in ('x', 'mel', 'x_len', 'mel_len', 'dur', 'pitch', 'energy'):
        got = b[k].numpy()
        assert got.dtype == z[f'r{r}_{k}'].dtype, k
        assert np.array_equal(got, z[f'r{r}_{k}']), k
    assert b['item_id'] == list(z[f'r{r}_item_id'])
    assert b['x'].dtype == torch.int64


def test_wav_name_and_formats(tmp_path):
    from forwardtacotron_amd.gen_forward import wav_name, write_output
    name = wav_name(3, 12, 1.0, 1.3, 'hifigan')
    assert name == '3_forward_12k_alpha1.0_amp1.3_hifigan'  # gen_forward.py:113
    m = torch.randn(1, 80, 37)
    p = write_output(m, name, 'hifigan', tmp_path)
    assert p.name == name + '.npy'
    assert np.array_equal(np.load(p, allow_pickle=False), m.numpy())
    p = write_output(m, 'x_melgan', 'melgan', tmp_path)
    assert p.suffix == '.mel'
    assert torch.equal(torch.load(p, weights_only=True), m)


def test_inputs(tmp_path):
    import argparse
    from forwardtacotron_amd.gen_forward import main, read_inputs
    from forwardtacotron_amd.text.tokenizer import Tokenizer
    ns = argparse.Namespace(input_tokens='5, 17,3', input_phonemes=None, input_text=None,
                            sentences=None)
    assert read_inputs(ns) == [[5, 17, 3]]
    ns.input_tokens, ns.input_phonemes = None, 'həloʊ'
    assert read_inputs(ns) == [Tokenizer()('həloʊ')]
    f = tmp_path / 's.txt'
    f.write_text('həloʊ\n\nwɜːld\n', encoding='utf-8')
    ns.input_phonemes, ns.sentences = None, str(f)
    assert len(read_inputs(ns)) == 2
    ns.input_text = 'Hello world'
    with pytest.raises(SystemExit):
        read_inputs(ns)
    with pytest.raises(SystemExit):  # wavernn needs --voc_checkpoint / --voc_synthetic
        main(['--synthetic', '--input_tokens', '1,2', 'wavernn'])


def test_raw_sentence_file_refused(tmp_path, capsys):
    """a sentences file of raw English (what the reference's sentences.txt holds)
    is refused with the reason, never tokenised as phonemes; symbols outside the phoneme
    set are reported (and dropped, as the reference Tokenizer drops them)."""
    import argparse
    from forwardtacotron_amd.gen_forward import read_inputs
    f = tmp_path / 'sentences.txt'
    f.write_text('President Trump met with other leaders at the Group of 20 conference.\n',
                 encoding='utf-8')
    ns = argparse.Namespace(input_tokens=None, input_phonemes=None, input_text=None,
                            sentences=str(f))
    with pytest.raises(SystemExit, match='raw text'):
        read_inputs(ns)
    f.write_text('həloʊ "wɜːld"\n', encoding='utf-8')
    (ids,) = read_inputs(ns)
    assert 'outside the phoneme set' in capsys.readouterr().out
    from forwardtacotron_amd.text.tokenizer import Tokenizer
    assert ids == Tokenizer()('həloʊ wɜːld')


def test_parser_grammar_matches_reference():
    """gen_forward.py:43-61: top-level options, then the vocoder sub-command; only
    `wavernn` takes --overlap / --target / --voc_checkpoint (defaults 550 / 11000)."""
    from forwardtacotron_amd.gen_forward import build_parser
    p = build_parser()
    a = p.parse_args(['--alpha', '1.5', '--amp', '0.8', 'wavernn', '--voc_checkpoint', 'v.pt',
                      '-t', '9000'])
    assert (a.vocoder, a.alpha, a.amp, a.voc_checkpoint, a.target, a.overlap) == \
        ('wavernn', 1.5, 0.8, 'v.pt', 9000, 550)
    assert p.parse_args(['griffinlim']).vocoder == 'griffinlim'
    assert p.parse_args([]).vocoder is None
    assert p.parse_args(['hifigan']).config == 'config.yaml'
    with pytest.raises(SystemExit):  # sub-command options belong to wavernn only
        p.parse_args(['griffinlim', '--target', '5'])


def test_checkpoint_from_config(tmp_path, monkeypatch):
    """gen_forward.py:68-72: no --checkpoint -> Paths(...).forward_checkpoints /
    'latest_model.pt' of the config's tts_model_id, loaded like an explicit checkpoint."""
    from forwardtacotron_amd import gen_forward as G
    from forwardtacotron_amd.checkpoints import save_checkpoint
    from forwardtacotron_amd.synthetic import default_config
    cfg = tmp_path / 'config.yaml'
    cfg.write_text("tts_model_id: 'my_tts'\ndata_path: 'data/'\n", encoding='utf-8')
    monkeypatch.chdir(tmp_path)
    path = G.checkpoint_from_config(str(cfg))
    assert path == tmp_path / 'checkpoints' / 'my_tts.forward' / 'latest_model.pt'
    model, _ = G.synthetic_tts_model()
    path.parent.mkdir(parents=True)
    save_checkpoint(model, None, default_config(), path)
    loaded = []
    monkeypatch.setattr(G, 'load_tts_model', lambda p: loaded.append(p) or G.synthetic_tts_model())
    with pytest.raises(SystemExit, match='GPU'):  # CPU container: stops at the device check
        G.main(['--config', str(cfg), '--input_tokens', '1,2', 'hifigan'])
    assert loaded == [str(path)]
    with pytest.raises(SystemExit, match='valid vocoder'):
        G.main(['--synthetic', '--input_tokens', '1,2'])


def test_checkpoint_roundtrip(tmp_path):
    """save_checkpoint -> gen_forward.load_tts_model (weights_only) restores the weights."""
    from forwardtacotron_amd.checkpoints import save_checkpoint
    from forwardtacotron_amd.gen_forward import load_tts_model, synthetic_tts_model
    m, cfg = synthetic_tts_model()
    p = tmp_path / 'latest_model.pt'
    save_checkpoint(m, None, cfg, p)
    m2, cfg2 = load_tts_model(str(p))
    assert cfg2 == cfg
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
