"""FastPitch on the GPU (csrc/transformer.hip + the GEMM family, through the C-ABI):
kernels against numpy, the model against the reference's golden vectors and the oracle.

Tolerances: attention runs on fp32 MFMA (exact fp32 products, different summation order
and an online softmax), LayerNorm accumulates in fp64, the projections / convolutions use
the fp32-accurate bf16x6 GEMM: per-kernel bounds 2e-5 relative to the output scale; the
whole model's mel within 5e-4 max / 2e-5 mean of the reference (north star: mean
|mel - ref| < 1e-4), duration counts bit-exact."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import fp_oracle as FP

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


@pytest.fixture(scope='module')
def fp_model():
    from forwardtacotron_amd.fast_pitch import FastPitch
    from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict
    m = FastPitch.from_config(default_config())
    sd = synthetic_state_dict(m, 0, 'fast_pitch')
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.cuda().eval(), sd


@pytest.mark.parametrize('C', [128, 256, 80])
def test_layernorm(C):
    from forwardtacotron_amd import ops
    rng = np.random.RandomState(C)
    x = (rng.randn(3, 37, C) * 3 + 1).astype(np.float32)
    g = rng.uniform(0.5, 1.5, C).astype(np.float32)
    b = rng.randn(C).astype(np.float32)
    ref = FP.layer_norm(x, g, b)
    np.testing.assert_allclose(host(ops.layernorm(dev(x), dev(g), dev(b))), ref, atol=2e-6, rtol=2e-6)


@pytest.mark.parametrize('mma,presplit', [(2, True), (2, False), (0, False)],
                         ids=['f16x3-presplit', 'f16x3', 'f32'])
@pytest.mark.parametrize('hd,T,masked', [(64, 37, False), (128, 200, True), (128, 33, False),
                                         (64, 129, True), (128, 1, False), (128, 1400, False)])
def test_attention(hd, T, masked, mma, presplit, monkeypatch):
    """f16x3: the transposed kernel (attention_t3_kernel, default) against the oracle, its
    pre-split and in-kernel-split forms bit-identical, likewise attention_h3_kernel's
    (FTMI_ATTN_T=0); the two kernels agree within 2e-6 (P V sums in a permuted key order)."""
    from forwardtacotron_amd import ops
    rng = np.random.RandomState(T + hd)
    B, H = 3, 2
    d = H * hd
    qkv = rng.randn(B, T, 3 * d).astype(np.float32)
    kpm = None
    if masked:
        kpm = np.zeros((B, T), bool)
        kpm[1, T - T // 3:] = True
        kpm[2, T // 2:] = True
    q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    sp = lambda t: t.reshape(B, T, H, hd).transpose(0, 2, 1, 3).astype(np.float64)
    s = (sp(q) * np.float32(np.sqrt(1.0 / hd))) @ sp(k).transpose(0, 1, 3, 2)
    if kpm is not None:
        s = np.where(kpm[:, None, None, :], -np.inf, s)
    ref = (FP.softmax(s) @ sp(v)).transpose(0, 2, 1, 3).reshape(B, T, d)
    st = ops.status_word('cuda')
    st.zero_()
    got = host(ops.attention(dev(qkv), H, dev(kpm) if kpm is not None else None, mma=mma,
                             presplit=presplit))
    np.testing.assert_allclose(got, ref, atol=2e-5, rtol=2e-5)
    assert int(st.item()) == 0
    if presplit:  # the split pass has the in-kernel split's arithmetic: identical results
        mk = dev(kpm) if kpm is not None else None
        other = host(ops.attention(dev(qkv), H, mk, mma=mma, presplit=False))
        np.testing.assert_array_equal(got, other)
        monkeypatch.setenv('FTMI_ATTN_T', '0')
        h3 = host(ops.attention(dev(qkv), H, mk, mma=mma, presplit=True))
        h3u = host(ops.attention(dev(qkv), H, mk, mma=mma, presplit=False))
        np.testing.assert_array_equal(h3, h3u)
        np.testing.assert_allclose(got, h3, atol=2e-6, rtol=2e-6)


def test_attention_f16_range_guard():
    """An attention operand beyond the f16 range sets status bit 0 on the f16x3 kernel (the
    model entry points then rerun on the fp32 kernel), and the fp32 kernel stays exact."""
    from forwardtacotron_amd import ops
    rng = np.random.RandomState(5)
    B, T, H, hd = 2, 40, 2, 64
    qkv = rng.randn(B, T, 3 * H * hd).astype(np.float32)
    qkv[1, 7, 2 * H * hd + 3] = 1e5  # one value entry
    st = ops.status_word('cuda')
    for presplit in (True, False):
        st.zero_()
        ops.attention(dev(qkv), H, mma=2, presplit=presplit)
        torch.cuda.synchronize()
        assert int(st.item()) & 1
    st.zero_()
    ops.attention(dev(qkv), H, mma=0)
    torch.cuda.synchronize()
    assert int(st.item()) == 0


def test_embedding_posenc_and_lr_posenc(fp_model):
    from forwardtacotron_amd import ops
    m, sd = fp_model
    pe = sd['postnet.pos_encoder.pe'][:, 0, :]
    sc = sd['postnet.pos_encoder.scale']
    ids = np.array([[3, 7, 0, 1], [9, 9, 2, 0]], np.int64)
    table = sd['embedding.weight']
    got = host(ops.embedding_posenc(dev(ids), dev(table), dev(pe), dev(sc)))
    np.testing.assert_array_equal(got, table[ids] + sc * pe[:4])
    x = np.random.RandomState(1).randn(2, 4, 256).astype(np.float32)
    index = np.array([[0, 0, 1, 3, 3, -1], [2, 1, 1, -1, -1, -1]], np.int32)
    got = host(ops.lr_posenc(dev(x), dev(index), dev(pe), dev(sc)))
    gathered = np.where(index[..., None] >= 0, x[np.arange(2)[:, None], np.maximum(index, 0)], 0)
    np.testing.assert_array_equal(got, gathered + sc * pe[:6])


GEN = {
    'fp_gen_b1': dict(alpha=1.0),
    'fp_gen_b3': dict(alpha=1.0),
    'fp_gen_alpha': dict(alpha=0.8),
    'fp_gen_fill2': dict(alpha=1000.0),
    'fp_gen_callbacks': dict(alpha=1.2, pitch_function=lambda p: p * 2.0 + 0.1,
                             energy_function=lambda e: e - 0.05),
}


@pytest.mark.parametrize('name', list(GEN))
def test_generate_matches_reference(name, fp_model):
    m, _ = fp_model
    g = load_golden(name)
    out = m.generate(dev(g['x']), **GEN[name])
    assert out['mel_post'] is out['mel']
    mel = host(out['mel'])
    assert mel.shape == g['mel'].shape
    d = np.abs(mel - g['mel'])
    assert d.max() < 5e-4 and d.mean() < 2e-5, (d.max(), d.mean())
    np.testing.assert_array_equal(FP.duration_counts(host(out['dur'])), FP.duration_counts(g['dur']))
    np.testing.assert_allclose(host(out['pitch']), g['pitch'], atol=5e-5)
    np.testing.assert_allclose(host(out['energy']), g['energy'], atol=5e-5)


def test_forward_matches_reference(fp_model):
    m, _ = fp_model
    g = load_golden('fp_forward')
    batch = {'x': dev(g['x']), 'mel': dev(g['mel_in']), 'mel_len': dev(g['mel_len']),
             'dur': dev(g['dur_in']), 'pitch': dev(g['pitch_in']), 'energy': dev(g['energy_in'])}
    o = m(batch)
    d = np.abs(host(o['mel']) - g['mel'])
    assert d.max() < 5e-4 and d.mean() < 2e-5
    np.testing.assert_allclose(host(o['dur']), g['dur'], atol=5e-5)


def test_batch64_against_oracle(fp_model):
    """A c5-shaped batch slice (B=8, T up to 60) against the numpy oracle."""
    from forwardtacotron_amd.synthetic import synthetic_tokens
    m, sd = fp_model
    x = synthetic_tokens(8, 60, seed=11, min_len=20)
    out = m.generate(dev(x))
    ref = FP.generate(sd, x)
    mel = host(out['mel'])
    assert mel.shape == ref['mel'].shape
    d = np.abs(mel - ref['mel'])
    assert d.mean() < 2e-5 and d.max() < 1e-3


def test_graph_phase_matches_eager(fp_model, monkeypatch):
    """generate() replays FastPitch's phoneme phase as a HIP graph (captured on the second
    call of a shape): identical (bit for bit) to the eager phase across replays with new
    tokens of the same shape; the returned dur / pitch / energy are not graph buffers; an
    unmarked callback is never captured (it runs eagerly beside the split graph)."""
    from forwardtacotron_amd import fast_pitch as FPM
    m, _ = fp_model
    g = load_golden('fp_gen_b3')
    x1 = dev(g['x'])
    x2 = x1.clone()
    x2[x2 > 0] = (x2[x2 > 0] * 7) % 133 + 1
    monkeypatch.setattr(FPM, 'FP_GRAPH', False)
    eager = [m.generate(x) for x in (x1, x2)]
    monkeypatch.setattr(FPM, 'FP_GRAPH', True)
    for k in ('_ftmi_graphs', '_ftmi_graph_seen'):
        m.__dict__.pop(k, None)
    graph = [m.generate(x) for x in (x1, x2, x1, x2)]  # eager, capture, replay, replay
    assert len(m.__dict__['_ftmi_graphs']) == 1
    assert graph[1]['dur'].data_ptr() != graph[3]['dur'].data_ptr()
    for e, gr in ((eager[0], graph[0]), (eager[1], graph[1]), (eager[0], graph[2]),
                  (eager[1], graph[3])):
        for k in ('mel', 'dur', 'pitch', 'energy'):
            assert torch.equal(e[k], gr[k]), k
    # a callback not marked graph_safe: the split graph (captured without it), the callback
    # run eagerly on every call (Python-side state it reads is seen), bit-identical to eager
    amp = [1.1]
    fn = lambda p: p * amp[0]  # noqa: E731  (not graph_safe)
    outs = []
    for a in (1.1, 1.1, 0.7, 1.3):
        amp[0] = a
        outs.append(m.generate(x1, pitch_function=fn))
    assert len(m.__dict__['_ftmi_graphs']) == 2
    assert any('split' in k for k in m.__dict__['_ftmi_graphs'])
    monkeypatch.setattr(FPM, 'FP_GRAPH', False)
    for a, o in zip((1.1, 1.1, 0.7, 1.3), outs):
        amp[0] = a
        ref = m.generate(x1, pitch_function=fn)
        for k in ('mel', 'dur', 'pitch', 'energy'):
            assert torch.equal(o[k], ref[k]), (a, k)


def test_panel_path_matches_unfused(fp_model, monkeypatch):
    """The FFT blocks' row-panel launches (ops.panel_proj: in_proj, out_proj + norm1, conv2
    + norm2) against the slab GEMM + layernorm launches (FTMI_PANEL=0).  The projections agree
    bit for bit wherever the unfused GEMM runs unsplit (test_gpu_kernels.py::test_panel_proj);
    at these row counts the unfused conv2 (K = 1024) sums split-K partials, so the bound is
    the fp32 summation-order one."""
    from forwardtacotron_amd.synthetic import synthetic_tokens
    m, _ = fp_model
    x = dev(synthetic_tokens(4, 80, seed=5, min_len=70))
    outs = {}
    for v in ('0', '1'):
        monkeypatch.setenv('FTMI_PANEL', v)
        outs[v] = {k: host(t) for k, t in m.generate(x).items() if k in ('mel', 'dur', 'pitch', 'energy')}
    d = np.abs(outs['0']['mel'] - outs['1']['mel'])
    assert d.max() < 1e-4 and d.mean() < 5e-6, (d.max(), d.mean())
    np.testing.assert_array_equal(FP.duration_counts(outs['0']['dur']), FP.duration_counts(outs['1']['dur']))
    for k in ('pitch', 'energy'):
        np.testing.assert_allclose(outs['0'][k], outs['1'][k], atol=1e-5)


@pytest.mark.parametrize('B,T,H,kpm', [(3, 500, 2, False), (2, 451, 4, True), (1, 900, 2, False)])
def test_kv_fused_in_proj_bit_identical(B, T, H, kpm):
    """ftmi_panel_proj_qkv + ftmi_attention_kv (the attention's K / V split folded into
    in_proj, FTMI_KV_FUSED) against ftmi_panel_proj + ftmi_attention with its split pass:
    bit-identical Q rows and attention outputs, with the stream's workspace reused across
    the cases (its pad keys hold earlier calls' planes)."""
    from forwardtacotron_amd import ops
    g = torch.Generator().manual_seed(B * T)
    d = 256
    x = torch.randn(B, T, d, generator=g).cuda()
    w = (torch.randn(3 * d, d, generator=g) / 16).cuda()
    b = (torch.randn(3 * d, generator=g) / 10).cuda()
    mask = None
    if kpm:
        lens = torch.randint(T // 2, T + 1, (B,), generator=g)
        mask = (torch.arange(T)[None, :] >= lens[:, None]).cuda()
    wf = ops.split_weights_f16(w, frag=True)
    qkv = ops.panel_proj(x, wf, 3 * d, bias=b)
    ref = ops.attention(qkv, H, mask, mma=2, presplit=True)
    q, kv = ops.panel_proj_qkv(x, wf, d, H, bias=b)
    got = ops.attention_kv(q, kv, H, mask)
    torch.cuda.synchronize()
    assert torch.equal(q, qkv[:, :, :d])
    assert torch.equal(got, ref)


def test_kv_workspace_after_overflow_stays_finite():
    """an overflowing call leaves inf in the reused K / V workspace (its K / V
    planes are split from out-of-range values; the call reports status bit 0 and reruns on
    the exact path).  A later call with a shorter T on the same stream must not read those
    as pad keys: the attention kernels zero keys >= T while staging the last tile."""
    from forwardtacotron_amd import ops
    g = torch.Generator().manual_seed(7)
    d, H = 256, 2
    w = (torch.randn(3 * d, d, generator=g) / 16).cuda()
    wf = ops.split_weights_f16(w, frag=True)
    st = ops.status_word('cuda')
    for B in (2, 3):  # a different B also shifts the planes' layout
        x = torch.randn(3, 300, d, generator=g).cuda() * 1e5  # K / V beyond 65504
        st.zero_()
        q, kv = ops.panel_proj_qkv(x, wf, d, H)
        ops.attention_kv(q, kv, H)
        torch.cuda.synchronize()
        assert int(st.item()) & 1
        hd, Tp = d // H, 320
        planes = kv[:4 * 3 * H * Tp * hd * 2].view(torch.float16)
        assert not torch.isfinite(planes).all()  # the workspace does hold non-finite values
        planes.view(4, -1)[:, :].fill_(float('inf'))  # and, worst case, in every pad slot
        x2 = torch.randn(B, 290, d, generator=g).cuda()
        st.zero_()
        q2, kv2 = ops.panel_proj_qkv(x2, wf, d, H)
        assert kv2.data_ptr() == kv.data_ptr()
        got = ops.attention_kv(q2, kv2, H)
        ref = ops.attention(ops.panel_proj(x2, wf, 3 * d), H, mma=2, presplit=True)
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        assert torch.isfinite(got).all()
        assert torch.equal(got, ref)
