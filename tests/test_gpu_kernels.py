"""Per-kernel parity of the HIP path (through the C-ABI) against the numpy oracle on
seeded inputs.  Integer work (LengthRegulator counts / index map / expansion) is
bit-exact; fp32 contractions are held to |err| <= ATOL + RTOL*|ref| with the bounds below
(fp32 MFMA is a k-ordered fmaf chain; the oracle is numpy sgemm: only summation order
differs)."""
import numpy as np
import pytest
import torch

from oracle import ft_oracle as O

pytestmark = pytest.mark.gpu

RTOL, ATOL = 2e-5, 2e-5


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def close(got, ref, rtol=RTOL, atol=ATOL):
    """fp32 contraction bound: |err| <= atol * max(1, rms(ref)) + rtol * |ref| (summation
    round-off grows with the output scale, i.e. with sqrt(K) * |w| * |x|)."""
    scale = max(1.0, float(np.sqrt(np.mean(np.square(ref, dtype=np.float64)))))
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=atol * scale)


@pytest.fixture
def rng():
    return np.random.Generator(np.random.PCG64(1234))


# ---------------------------------------------------------------- conv / GEMM family
# (mma, pre-split weights): fp32 MFMA, bf16x6 splitting both operands per call, bf16x6
# with the weights split once by ftmi_split_weights, f16x3 on ftmi_split_weights_f16
# planes (the model's default path)
MMA_CELLS = [(0, False, 'f32'), (1, False, 'bf16x6'), (1, True, 'bf16x6-presplit'),
             (2, True, 'f16x3')]
MMAS = pytest.mark.parametrize('mma,pre', [c[:2] for c in MMA_CELLS], ids=[c[2] for c in MMA_CELLS])
KERNELS = ('tiled', 'slab', 'skinny')


def kernel_applies(kernel, mma, M=None, N=None):
    """'skinny': the default choice (the weight-streaming skinny kernel for M <= 256 rows,
    the slab kernel above); 'slab': the f16x3 slab kernel for every eligible shape; 'tiled':
    the 128 x 128 tiled kernels only.  slab / skinny are f16x3 kernels; the skinny kernel
    takes M <= 256 rows (narrow single-group linears: M <= 1024)."""
    if kernel in ('slab', 'skinny') and mma != 2:
        return False
    if kernel == 'skinny' and M is not None and M > 256 and not (N is not None and N <= 128 and M <= 1024):
        return False
    return True


def gemm_cases(shapes, rows=lambda s: None, cols=lambda s: None, ids=None):
    """pytest params (*shape, mma, pre, kernel) of the APPLICABLE cells only (no runtime
    skips: a real skip stays visible)."""
    out = []
    for i, shape in enumerate(shapes):
        sid = ids[i] if ids else '-'.join(str(v) for v in shape)
        for mma, pre, mid in MMA_CELLS:
            for kernel in KERNELS:
                if kernel_applies(kernel, mma, rows(shape), cols(shape)):
                    out.append(pytest.param(*shape, mma, pre, kernel, id=f'{sid}-{mid}-{kernel}'))
    return out


def use_kernel(kernel, monkeypatch):
    """Route the GEMM family to `kernel` (see kernel_applies)."""
    if kernel == 'skinny':
        return
    monkeypatch.setenv('FTMI_GEMM_SKINNY', '0')
    if kernel == 'tiled':
        monkeypatch.setenv('FTMI_GEMM_SLAB_MIN', str(1 << 62))


def wsplit(w, pre, mma=1):
    from forwardtacotron_amd import ops
    return ops.presplit_for(w, mma) if pre else None


CONV_SHAPES = [
    (2, 37, 64, 256, 5, True, True, False),     # SeriesPredictor conv 1
    (3, 50, 256, 256, 5, True, True, False),    # SeriesPredictor conv 2/3
    (2, 129, 512, 80, 1, False, False, True),   # lin-like (N tail)
    (1, 7, 16, 40, 4, True, True, False),       # even k, tiny
    (2, 300, 80, 256, 8, True, True, False),    # postnet bank k=8
    (2, 60, 1024, 256, 3, True, True, True),    # long K, few tiles: split-K on the x6 path
    (3, 301, 96, 200, 7, True, True, True),     # slab kernel: ragged rows / columns, k = 7
    (2, 9, 32, 64, 16, True, False, False),     # slab kernel: k = 16 > T, every tap masked
    (4, 70, 64, 1536, 1, False, False, True),   # slab kernel, k = 1, many column tiles
    (1, 816, 1024, 80, 1, False, False, True),  # c2 lin: narrow linear, 816 rows (skinny)
    # skinny finish: split counts that leave remainders after its 4- / 8-split load batches
    (1, 40, 416, 64, 3, True, True, True),      # 7 splits (one lane per element: 4 + 3)
    (1, 33, 1280, 96, 1, False, False, True),   # 20 splits (4 lanes per element: 4 + 1)
    (1, 25, 2304, 128, 1, True, False, True),   # 36 splits (4 lanes per element: 8 + 1)
]


@pytest.mark.parametrize('B,T,Cin,N,k,relu,bn,bias,mma,pre,kernel',
                         gemm_cases(CONV_SHAPES, rows=lambda s: s[0] * s[1], cols=lambda s: s[3]))
def test_conv1d(B, T, Cin, N, k, relu, bn, bias, rng, mma, pre, kernel, monkeypatch):
    use_kernel(kernel, monkeypatch)
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    w = rng.normal(0, 1 / np.sqrt(Cin * k), (N, Cin, k)).astype(np.float32)
    b = rng.normal(0, 0.1, N).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, N).astype(np.float32)
    sh = rng.normal(0, 0.1, N).astype(np.float32)
    ref = O.conv1d(x.transpose(0, 2, 1), w, k // 2, b if bias else None)[:, :, :T]
    if relu:
        ref = np.maximum(ref, 0)
    if bn:
        ref = ref * sc[None, :, None] + sh[None, :, None]
    wp = pack_conv(torch.from_numpy(w)).cuda()
    y, _ = ops.conv1d(dev(x), wp, k, k // 2, bias=dev(b) if bias else None, relu=relu,
                      bn=(dev(sc), dev(sh)) if bn else None, mma=mma, w_split=wsplit(wp, pre, mma))
    close(host(y), ref.transpose(0, 2, 1))


@pytest.mark.parametrize('Cin,mma,pre,kernel', gemm_cases([(128,), (1024,)], rows=lambda s: 90))
def test_conv1d_maxpool_residual_transposed(rng, mma, pre, Cin, kernel, monkeypatch):
    use_kernel(kernel, monkeypatch)
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    B, T, N = 2, 45, 80
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    res = rng.normal(0, 1, (B, T, N)).astype(np.float32)
    w = rng.normal(0, 0.1, (N, Cin, 3)).astype(np.float32)
    ref = O.conv1d(O.maxpool_k2_s1_p1(x.transpose(0, 2, 1)), w, 1) + res.transpose(0, 2, 1)
    yt = torch.empty(B, N, T, device='cuda')
    wp = pack_conv(torch.from_numpy(w)).cuda()
    y, _ = ops.conv1d(dev(x), wp, 3, 1, maxpool=True, residual=dev(res), out_t=yt, mma=mma,
                      w_split=wsplit(wp, pre, mma))
    close(host(y), ref.transpose(0, 2, 1))
    close(host(yt), ref)


@pytest.mark.parametrize('kernel', ['slab', 'skinny'])
def test_conv1d_c2_proj1_maxpool(rng, kernel, monkeypatch):
    """BASELINE config c2 (B = 1, T = 120): the prenet proj1 shape (Cin = 16 x 256, k = 3,
    maxpool fused, ReLU then BN) — 64 channel splits on the skinny kernel."""
    use_kernel(kernel, monkeypatch)
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    B, T, Cin, N = 1, 120, 4096, 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    w = rng.normal(0, 1 / np.sqrt(Cin * 3), (N, Cin, 3)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, N).astype(np.float32)
    sh = rng.normal(0, 0.1, N).astype(np.float32)
    ref = np.maximum(O.conv1d(O.maxpool_k2_s1_p1(x.transpose(0, 2, 1)), w, 1), 0)
    ref = ref * sc[None, :, None] + sh[None, :, None]
    wp = pack_conv(torch.from_numpy(w)).cuda()
    y, _ = ops.conv1d(dev(x), wp, 3, 1, relu=True, bn=(dev(sc), dev(sh)), maxpool=True, mma=2,
                      w_split=wsplit(wp, True, 2))
    close(host(y), ref.transpose(0, 2, 1))


@MMAS
def test_conv1d_strided_input_view(rng, mma, pre):
    from forwardtacotron_amd import ops
    B, T, C = 2, 33, 64
    full = rng.normal(0, 1, (B, T, 2 * C)).astype(np.float32)
    w = rng.normal(0, 0.1, (48, C)).astype(np.float32)
    xt = dev(full)[:, :, C:]  # row stride 2C
    y, _ = ops.conv1d(xt, dev(w), 1, 0, mma=mma, w_split=wsplit(dev(w), pre, mma))
    close(host(y), full[:, :, C:] @ w.T)


@pytest.mark.parametrize('K,Cin,B,T,mma,pre,kernel',
                         gemm_cases([(16, 256, 2, 41), (8, 80, 2, 150), (5, 48, 3, 270),
                                     (16, 256, 1, 120), (3, 80, 2, 128)],
                                    rows=lambda s: s[2] * s[3]))
def test_conv_bank(K, Cin, B, T, rng, mma, pre, kernel, monkeypatch):
    use_kernel(kernel, monkeypatch)
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    C = 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    sc = rng.uniform(0.5, 1.5, K * C).astype(np.float32)
    sh = rng.normal(0, 0.1, K * C).astype(np.float32)
    refs = [np.maximum(O.conv1d(x.transpose(0, 2, 1), w, w.shape[2] // 2)[:, :, :T], 0) for w in ws]
    ref = np.concatenate(refs, 1) * sc[None, :, None] + sh[None, :, None]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, mma) if pre else None
    y = ops.conv_bank(dev(x), wp, K, C, dev(sc), dev(sh), mma=mma, w_split=w3)
    close(host(y), ref.transpose(0, 2, 1), rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize('K,Cin,B,T', [(16, 256, 2, 300), (8, 80, 3, 200), (8, 80, 1, 700),
                                     (3, 64, 5, 61)])
def test_conv_bank_pooled(K, Cin, B, T, rng, monkeypatch):
    """pool=True: the slab bank kernel stores the CBHG maxpool(2, 1) of its output (tiles of
    255 rows + a halo row; sequences starting inside a tile) — bit-identical to the maxpool
    of the unpooled bank, and within the fp32 bound of the oracle."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    C = 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    sc = rng.uniform(0.5, 1.5, K * C).astype(np.float32)
    sh = rng.normal(0, 0.1, K * C).astype(np.float32)
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    xd = dev(x)
    assert ops.bank_pools(xd, K, C, w_split=w3)
    y = host(ops.conv_bank(xd, wp, K, C, dev(sc), dev(sh), mma=2, w_split=w3))
    yp = host(ops.conv_bank(xd, wp, K, C, dev(sc), dev(sh), mma=2, w_split=w3, pool=True))
    ref_pool = O.maxpool_k2_s1_p1(y.transpose(0, 2, 1)).transpose(0, 2, 1)
    np.testing.assert_array_equal(yp, ref_pool)
    refs = [np.maximum(O.conv1d(x.transpose(0, 2, 1), w, w.shape[2] // 2)[:, :, :T], 0) for w in ws]
    ref = np.concatenate(refs, 1) * sc[None, :, None] + sh[None, :, None]
    close(yp, O.maxpool_k2_s1_p1(ref).transpose(0, 2, 1), rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize('K,Cin,B,T', [(8, 80, 3, 200), (8, 80, 16, 1368), (8, 96, 2, 300),
                                     (4, 48, 7, 5), (4, 48, 5, 3), (2, 16, 3, 40),
                                     (3, 64, 5, 61)])
def test_conv_bank_walk(K, Cin, B, T, rng, monkeypatch):
    """The walking bank (gemm.hip conv_bank_walk_kernel: one block per pooled row tile and
    column tile, every group over one resident slab, the epilogue from registers) gives the
    slab kernel's pooled bank bit for bit — fp32 rows and f16x3 split rows — including tiles
    that hold sequence starts, sequences shorter than the taps (T = 5, k = 4; T = 3 takes the
    slab kernel: the walk needs T >= 4) and 86 row tiles (the XCD-ordered grid); status stays
    0, and inputs or outputs beyond the f16 range set bit 0."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    C = 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    sc = dev(rng.uniform(0.5, 1.5, K * C).astype(np.float32))
    sh = dev(rng.normal(0, 0.1, K * C).astype(np.float32))
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    xd = dev(x)
    st = ops.status_word(xd.device)
    st.zero_()
    out = {}
    for walk in ('1', '0'):
        monkeypatch.setenv('FTMI_BANK_WALK', walk)
        out[walk] = [host(ops.conv_bank(xd, wp, K, C, sc, sh, mma=2, w_split=w3, pool=True,
                                        split_out=so)) for so in (False, True)]
    for a, b in zip(out['1'], out['0']):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    assert int(st.item()) == 0
    monkeypatch.setenv('FTMI_BANK_WALK', '1')
    xb = x.copy()
    xb[B - 1, T - 1, Cin - 1] = 1e5  # the last row's last channel
    ops.conv_bank(dev(xb), wp, K, C, sc, sh, mma=2, w_split=w3, pool=True)
    assert int(st.item()) & 1
    st.zero_()
    ops.conv_bank(xd, wp, K, C, sc * 1e5, sh, mma=2, w_split=w3, pool=True)  # fp32 rows: fine
    assert int(st.item()) == 0
    ops.conv_bank(xd, wp, K, C, sc * 1e5, sh, mma=2, w_split=w3, pool=True, split_out=True)
    assert int(st.item()) & 1
    st.zero_()


@pytest.mark.parametrize('K,Cin,B,T', [(16, 256, 1, 120), (16, 256, 1, 50), (8, 128, 2, 64),
                                     (4, 64, 1, 50)])
def test_conv_bank_halves(K, Cin, B, T, rng, monkeypatch):
    """The one-launch channel-halves bank (FTMI_BANK_HALVES, c2's prenet bank): bit-identical
    across repeated calls whichever half of a unit arrives last (the two halves' sums are
    added by one fp32 add: commutative), every launch leaves the unit counters zero (a bank
    of another shape on the same stream's workspace, then this one again: the same bits),
    within the fp32 bound of the channel-split kernel + finish, and status 0."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    C = 256
    x = dev(rng.normal(0, 1, (B, T, Cin)).astype(np.float32))
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    sc = dev(rng.uniform(0.5, 1.5, K * C).astype(np.float32))
    sh = dev(rng.normal(0, 0.1, K * C).astype(np.float32))
    assert ops._bank_halves(2, B, T, Cin, K, C)
    st = ops.status_word(x.device)
    st.zero_()
    a0 = host(ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3))
    other = dev(rng.normal(0, 1, (1, 100, 64)).astype(np.float32))
    ws2 = [rng.normal(0, 0.1, (C, 64, k)).astype(np.float32) for k in range(1, 5)]
    wp2 = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws2]).cuda()
    w32 = ops.split_bank_weights(wp2, 4, 64, C, 2)
    for _ in range(4):
        assert np.array_equal(host(ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3)), a0)
        ops.conv_bank(other, wp2, 4, C, sc[:4 * C], sh[:4 * C], mma=2, w_split=w32)
    # the stream-order weight image: the same bits, repeatedly
    img = ops.bank_halves_image(w3, K, Cin, C)
    assert img.numel() == ops._lib.load().ftmi_conv_bank_halves_image_bytes(Cin, K, C)
    for _ in range(2):
        yi = ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3, w_image=img)
        np.testing.assert_array_equal(host(yi), a0)
    assert int(st.item()) == 0
    key = (torch.device('cuda', torch.cuda.current_device()), torch.cuda.current_stream().cuda_stream)
    assert not ops._BANK_WS[key][:ops.BANK_COUNTERS].any()  # counters back to zero
    monkeypatch.setenv('FTMI_BANK_HALVES', '0')
    b0 = host(ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3))
    close(a0, b0, rtol=1e-5, atol=1e-5)


def test_conv_bank_halves_range_guard(rng):
    """An input beyond the f16 range sets status bit 0 on the halves bank (the model then
    reruns on the exact path)."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    K, Cin, C = 16, 256, 256
    xn = rng.normal(0, 1, (1, 120, Cin)).astype(np.float32)
    xn[0, 7, 200] = 1e5  # in the second channel half
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    st = ops.status_word('cuda')
    st.zero_()
    ops.conv_bank(dev(xn), wp, K, C, dev(np.ones(K * C, np.float32)),
                  dev(np.zeros(K * C, np.float32)), mma=2, w_split=w3)
    torch.cuda.synchronize()
    assert int(st.item()) & 1
    st.zero_()


def split_rows_host(v):
    """The f16x3 split rows of include/ftmi.h (per row C heads, then C scaled tails)."""
    h = v.astype(np.float16)
    t = ((v - h.astype(np.float32)) * np.float32(2048)).astype(np.float16)
    return np.concatenate([h, t], -1)


@pytest.mark.parametrize('K,Cin,B,T,split_k', [(16, 256, 2, 300, 0), (8, 80, 3, 200, 0),
                                               (8, 80, 1, 700, 3), (3, 64, 5, 61, 0)])
def test_split_rows_bank_to_proj1(K, Cin, B, T, split_k, rng, monkeypatch):
    """conv_bank(pool, split_out) stores the pooled bank as f16x3 split rows (bit-equal to
    splitting the fp32 pooled output on the host) and proj1 with x_split=True gives exactly
    the output of proj1 on the fp32 rows (the same head / tail feed the MFMAs), with and
    without a channel split; the C side refuses x_split where the slab kernel does not run."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd._lib import FtmiError
    from forwardtacotron_amd.common_layers import pack_conv
    C = 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    sc = dev(rng.uniform(0.5, 1.5, K * C).astype(np.float32))
    sh = dev(rng.normal(0, 0.1, K * C).astype(np.float32))
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    xd = dev(x)
    yp = ops.conv_bank(xd, wp, K, C, sc, sh, mma=2, w_split=w3, pool=True)
    ys = ops.conv_bank(xd, wp, K, C, sc, sh, mma=2, w_split=w3, pool=True, split_out=True)
    got = host(ys).view(np.float16)  # (B, T, 2*K*C) halves
    np.testing.assert_array_equal(got, split_rows_host(host(yp)))
    # the bank's own input as split rows (split_rows): the same bank output, bit for bit
    xs = ops.split_rows(xd)
    np.testing.assert_array_equal(host(xs).view(np.float16), split_rows_host(x))
    yx = ops.conv_bank(xs, wp, K, C, sc, sh, mma=2, w_split=w3, pool=True, x_split=True)
    np.testing.assert_array_equal(host(yx), host(yp))
    st = ops.status_word(xd.device)
    assert int(st.item()) == 0
    ops.split_rows(xd * 1e5)  # beyond the f16 range: the producer flags it
    assert int(st.item()) & 1
    st.zero_()
    w1 = dev(rng.normal(0, 1 / np.sqrt(3 * K * C), (256, 3 * K * C)).astype(np.float32))
    w13 = ops.split_weights_f16(w1)
    bn = (dev(rng.uniform(0.5, 1.5, 256).astype(np.float32)), dev(rng.normal(0, .1, 256).astype(np.float32)))
    if split_k:
        monkeypatch.setattr(ops, '_split_k', lambda *a: split_k)
    ref, _ = ops.conv1d(yp, w1, 3, 1, relu=True, bn=bn, mma=2, w_split=w13)
    out, _ = ops.conv1d(ys, w1, 3, 1, relu=True, bn=bn, mma=2, w_split=w13, x_split=True)
    np.testing.assert_array_equal(host(out), host(ref))
    with pytest.raises(FtmiError):  # maxpool on split rows: refused, not misread
        ops.conv1d(ys, w1, 3, 1, maxpool=True, mma=2, w_split=w13, x_split=True)
    with pytest.raises(FtmiError):  # x_split off the f16x3 path
        ops.conv1d(ys, w1, 3, 1, mma=0, x_split=True)


@pytest.mark.parametrize('schedule', ['halves', 'halves-image', 'pairs', 'groups'])
@pytest.mark.parametrize('K,Cin,B,T', [(16, 256, 1, 120), (8, 80, 1, 100), (4, 64, 2, 50),
                                     (16, 256, 2, 64), (16, 256, 1, 37), (2, 32, 1, 128),
                                     (16, 256, 1, 129), (8, 128, 1, 128), (16, 192, 3, 40)])
def test_conv_bank_skinny_schedules(K, Cin, B, T, schedule, rng, monkeypatch):
    """The weight-streaming bank at batch-1 sizes on every block schedule: the one-launch
    channel-halves kernel (conv_bank_halves_kernel, the default where it applies: M <= 128,
    Cin % 64 == 0; other shapes fall through to the next), group pairs (k, K + 1 - k) per
    block with one (unit, half) per wave, one group per block (FTMI_BANK_BALANCED=0), the
    split schedules finished by the finish launch; f16x3, against the numpy oracle.  M = 129:
    two row tiles, the second with one row.  halves-image: the halves kernel reading the
    stream-order weight image (FTMI_BANK_IMAGE), bit-identical to it reading the planes."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    monkeypatch.setenv('FTMI_BANK_HALVES', '1' if schedule.startswith('halves') else '0')
    monkeypatch.setenv('FTMI_BANK_BALANCED', '0' if schedule == 'groups' else '1')
    C = 256
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    ws = [rng.normal(0, 1 / np.sqrt(Cin * k), (C, Cin, k)).astype(np.float32) for k in range(1, K + 1)]
    sc = rng.uniform(0.5, 1.5, K * C).astype(np.float32)
    sh = rng.normal(0, 0.1, K * C).astype(np.float32)
    refs = [np.maximum(O.conv1d(x.transpose(0, 2, 1), w, w.shape[2] // 2)[:, :, :T], 0) for w in ws]
    ref = np.concatenate(refs, 1) * sc[None, :, None] + sh[None, :, None]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, Cin, C, 2)
    y = ops.conv_bank(dev(x), wp, K, C, dev(sc), dev(sh), mma=2, w_split=w3)
    close(host(y), ref.transpose(0, 2, 1), rtol=5e-5, atol=5e-5)
    if schedule == 'halves-image':
        img = ops.bank_halves_image(w3, K, Cin, C)
        if Cin % 64 == 0 and K % 2 == 0 and (K // 2) * (C // 16) % 8 == 0:
            assert img is not None
        if img is not None:
            yi = ops.conv_bank(dev(x), wp, K, C, dev(sc), dev(sh), mma=2, w_split=w3, w_image=img)
            np.testing.assert_array_equal(host(yi), host(y))


@pytest.mark.parametrize('C,B,T,mma,pre,kernel',
                         gemm_cases([(256, 3, 77), (128, 2, 300), (256, 1, 816),
                                     (160, 1, 90)]))  # skinny: 3 splits (2 + 1 in the finish)
def test_highway(rng, mma, pre, kernel, C, B, T, monkeypatch):
    from forwardtacotron_amd.common_layers import HighwayNetwork
    use_kernel(kernel, monkeypatch)
    hw = HighwayNetwork(C)
    sd = {'W1.weight': rng.normal(0, 1 / 16, (C, C)), 'W1.bias': rng.normal(0, .1, C),
          'W2.weight': rng.normal(0, 1 / 16, (C, C)), 'W2.bias': rng.normal(0, .1, C)}
    hw.load_state_dict({k: torch.from_numpy(v.astype(np.float32)) for k, v in sd.items()})
    hw = hw.cuda()
    x = rng.normal(0, 1, (B, T, C)).astype(np.float32)
    ref = O.highway({'h.' + k: v.astype(np.float32) for k, v in sd.items()}, 'h', x, np.float32)
    w12, b1, b2, _ = hw.packed_weights()
    from forwardtacotron_amd import ops
    close(host(ops.highway(dev(x), w12, b1, b2, mma=mma, w_split=wsplit(w12, pre, mma))), ref)


@pytest.mark.parametrize('B,T,Cp,L', [(2, 1600, 80, 4), (3, 77, 256, 4), (1, 40, 80, 2),
                                     (2, 300, 128, 0)])
def test_highway_stack(B, T, Cp, L, rng, monkeypatch):
    """pre_highway -> L highways -> GRU input projection in one launch
    (ftmi_highway_stack) against the numpy oracle (fp32 bound) and against the unfused
    f16x3 slab-kernel chain it replaces (conv1d, L x highway, conv1d): bit for bit where
    those launches run unsplit, else within 1e-6."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import CBHG
    monkeypatch.setenv('FTMI_GEMM_SKINNY', '0')  # the unfused chain on the slab kernel
    C = 256
    torch.manual_seed(3)
    m = CBHG(K=2, in_channels=Cp, channels=C, proj_channels=[C, Cp], num_highways=L)
    with torch.no_grad():
        for hw in m.highways:
            hw.W1.bias.normal_(0, 0.1)
    m = m.cuda()
    x = rng.normal(0, 1, (B, T, Cp)).astype(np.float32)
    w_pre, pre3 = m.packed_weights()[3], m.packed_weights()[5]
    hws = [hw.packed_weights() for hw in m.highways]
    w_ih, b_in, _, _, w3 = m.rnn.packed_weights()
    xd = dev(x)
    pre_f, hw_f, b1s, b2s, ih_f, _, n_out = m._stack_pack()
    y, h = ops.highway_stack(xd, pre_f, C, hw_f, b1s, b2s, ih_f, b_in, n_out, want_h=True)
    # numpy oracle
    ref = x.reshape(-1, Cp).astype(np.float64) @ host(w_pre).astype(np.float64).T
    for i, hw in enumerate(m.highways):
        sd = {f'h.{k}': host(v) for k, v in hw.state_dict().items()}
        ref = O.highway(sd, 'h', ref, np.float64)
    close(host(h).reshape(-1, C), ref)
    refp = ref @ host(w_ih).astype(np.float64).T + host(b_in)
    close(host(y).reshape(-1, w_ih.size(0)), refp)
    # the unfused chain
    hu, _ = ops.conv1d(xd, w_pre, 1, 0, w_split=pre3)
    for w12, b1, b2, s3 in hws:
        hu = ops.highway(hu, w12, b1, b2, w_split=s3)
    yu, _ = ops.conv1d(hu, w_ih, 1, 0, bias=b_in, w_split=w3)
    if B * T >= 3200:  # unfused launches without a split-K (whose partial sums round apart)
        np.testing.assert_array_equal(host(h), host(hu))
        np.testing.assert_array_equal(host(y), host(yu))
    else:
        close(host(h), host(hu), rtol=1e-6, atol=1e-6)
        close(host(y), host(yu), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('B,T', [(3, 333), (64, 1368)])
def test_highway_stack_rows96_bit_identical(B, T, rng, monkeypatch):
    """The 96-row workgroup form (one LDS image overwritten in place, default from 24,576
    rows) against the 64-row ping-pong form: same MFMA order and epilogue, bit for bit,
    incl. a ragged last row tile; the second case is the c3 postnet (87,552 rows)."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import CBHG
    C, Cp, L = 256, 80, 4
    torch.manual_seed(5)
    m = CBHG(K=2, in_channels=Cp, channels=C, proj_channels=[C, Cp], num_highways=L)
    with torch.no_grad():
        for hw in m.highways:
            hw.W1.bias.normal_(0, 0.1)
    m = m.cuda()
    xd = dev(rng.normal(0, 1, (B, T, Cp)).astype(np.float32))
    _, _, b_in, _, _ = m.rnn.packed_weights()
    pre_f, hw_f, b1s, b2s, ih_f, _, n_out = m._stack_pack()
    outs = []
    for bm in ('96', '64'):
        monkeypatch.setenv('FTMI_HS_BM', bm)
        y, h = ops.highway_stack(xd, pre_f, C, hw_f, b1s, b2s, ih_f, b_in, n_out, want_h=True)
        outs.append((host(y), host(h)))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('B,T,Cp,L,out', [(1, 120, 256, 4, True), (1, 816, 80, 4, True),
                                          (1, 50, 80, 2, False), (2, 64, 256, 4, True),
                                          (1, 1024, 80, 4, True), (3, 43, 80, 0, True)])
def test_highway_stack_spread_bit_identical(B, T, Cp, L, out, rng, monkeypatch):
    """The few-row CBHG tail spread over 16 workgroups per 64-row block
    (ftmi_highway_stack_spread: c2's prenet 120 and postnet 816 rows) against the
    one-workgroup-per-block kernel: the same per-accumulator order, bit for bit — the
    projection, the last highway's output, ragged row blocks, no highway layers (L = 0),
    h only (no projection) — repeatedly (the exchange counters are re-zeroed per call)."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import CBHG
    C = 256
    torch.manual_seed(7)
    m = CBHG(K=2, in_channels=Cp, channels=C, proj_channels=[C, Cp], num_highways=L)
    with torch.no_grad():
        for hw in m.highways:
            hw.W1.bias.normal_(0, 0.1)
    m = m.cuda()
    xd = dev(rng.normal(0, 1, (B, T, Cp)).astype(np.float32))
    _, b_in, _, _, _ = m.rnn.packed_weights()
    pre_f, hw_f, b1s, b2s, ih_f, _, n_out = m._stack_pack()
    st = ops.status_word('cuda')
    st.zero_()
    args = (xd, pre_f, C, hw_f, b1s, b2s) + ((ih_f, b_in, n_out) if out else (None, None, 0))
    assert ops.hs_spread_blocks(B * T, n_out if out else 0) == -(-B * T // 64) * 16
    res = []
    for sp in ('1', '1', '0'):
        monkeypatch.setenv('FTMI_HS_SPREAD', sp)
        y, h = ops.highway_stack(*args, want_h=True)
        res.append((None if y is None else host(y), host(h)))
    for r in res[:2]:
        if out:
            np.testing.assert_array_equal(r[0], res[2][0])
        np.testing.assert_array_equal(r[1], res[2][1])
    assert int(st.item()) == 0


def test_highway_stack_range_guard(rng):
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import CBHG
    m = CBHG(K=2, in_channels=80, channels=256, proj_channels=[256, 80], num_highways=2).cuda()
    pre_f, hw_f, b1s, b2s, *_ = m._stack_pack()
    x = rng.normal(0, 1, (1, 100, 80)).astype(np.float32)
    st = ops.status_word('cuda')
    for bad in (False, True):
        if bad:
            x[0, 17, 5] = 7e4
        st.zero_()
        ops.highway_stack(dev(x), pre_f, 256, hw_f, b1s, b2s, None, None, 0, want_h=True)
        assert bool(int(st.item()) & 1) == bad


PANEL_CASES = [  # (B, T, K, N, residual, ln): FFTBlock in_proj, out_proj + norm1, conv2 + norm2
    (4, 900, 256, 768, False, False),
    (4, 900, 256, 256, True, True),
    (4, 900, 1024, 256, True, True),
    (2, 333, 96, 512, True, False),  # K not a multiple of 32 (zero-padded k-step), 2 panels
    (1, 37, 256, 256, True, True),    # one partial row tile
]


@pytest.mark.parametrize('B,T,K,N,res,ln', PANEL_CASES)
def test_panel_proj(rng, monkeypatch, B, T, K, N, res, ln):
    """ftmi_panel_proj (FastPitch FFT-block projections, fast_pitch.py:56-91) vs a float64
    numpy oracle of x W^T + b (+ residual) (-> LayerNorm) within the f16x3 bound, and vs the
    unfused slab conv1d + layernorm launches bit for bit (same k-step / product / epilogue
    order) where the unfused GEMM runs unsplit, within 1e-5 where it sums split-K partials."""
    from forwardtacotron_amd import ops
    monkeypatch.setenv('FTMI_GEMM_SKINNY', '0')
    x = rng.normal(0, 1, (B, T, K)).astype(np.float32)
    w = (rng.normal(0, 1, (N, K)) / np.sqrt(K)).astype(np.float32)
    b = rng.normal(0, 0.1, N).astype(np.float32)
    r = rng.normal(0, 1, (B, T, N)).astype(np.float32) if res else None
    g = rng.normal(1, 0.2, N).astype(np.float32)
    bt = rng.normal(0, 0.2, N).astype(np.float32)
    wd = dev(w)
    lnp = (dev(g), dev(bt), 1e-5) if ln else None
    y = ops.panel_proj(dev(x), ops.split_weights_f16(wd, frag=True), N, bias=dev(b),
                       residual=dev(r) if res else None, ln=lnp)
    ref = x.reshape(-1, K).astype(np.float64) @ w.astype(np.float64).T + b
    if res:
        ref = ref + r.reshape(-1, N)
    if ln:
        mu = ref.mean(1, keepdims=True)
        ref = (ref - mu) / np.sqrt(((ref - mu) ** 2).mean(1, keepdims=True) + 1e-5) * g + bt
    close(host(y).reshape(-1, N), ref, rtol=1e-5, atol=1e-5)
    yu, _ = ops.conv1d(dev(x), wd, 1, 0, bias=dev(b), residual=dev(r) if res else None,
                       w_split=ops.split_weights_f16(wd))
    if ln:
        yu = ops.layernorm(yu, lnp[0], lnp[1], 1e-5, out=yu)
    if B * T > 256 and ops._split_k(B * T, N, K, 2, True, K) == 1:
        np.testing.assert_array_equal(host(y), host(yu))
    else:  # the unfused side sums split-K partials there (skinny kernel / slab split)
        close(host(y), host(yu), rtol=1e-5, atol=1e-5)


def test_panel_proj_in_place_and_range_guard(rng):
    """out may alias the residual (FFTBlock's norm2 step writes over h); |x| > 65504 sets
    status bit 0."""
    from forwardtacotron_amd import ops
    x = rng.normal(0, 1, (2, 300, 256)).astype(np.float32)
    w = dev((rng.normal(0, 1, (256, 256)) / 16).astype(np.float32))
    wf = ops.split_weights_f16(w, frag=True)
    r = dev(rng.normal(0, 1, (2, 300, 256)).astype(np.float32))
    ln = (torch.ones(256, device='cuda'), torch.zeros(256, device='cuda'), 1e-5)
    ref = ops.panel_proj(dev(x), wf, 256, residual=r, ln=ln)
    got = ops.panel_proj(dev(x), wf, 256, residual=r, ln=ln, out=r)
    assert got.data_ptr() == r.data_ptr()
    np.testing.assert_array_equal(host(got), host(ref))
    with pytest.raises(Exception):
        xd = dev(x)
        ops.panel_proj(xd, wf, 256, out=xd[..., :256])  # y aliasing x: refused
    st = ops.status_word('cuda')
    for bad in (False, True):
        if bad:
            x[1, 17, 5] = 7e4
        st.zero_()
        ops.panel_proj(dev(x), wf, 256)
        assert bool(int(st.item()) & 1) == bad


def test_split_weights_exact(rng):
    """The three bf16 pieces sum back to the fp32 weights exactly; K padding is zero."""
    from forwardtacotron_amd import ops
    w = (rng.normal(0, 1, (70, 1000)) * np.exp(rng.normal(0, 3, (70, 1000)))).astype(np.float32)
    p = ops.split_weights(dev(w)).double()
    assert p.shape == (3, 70, 1024)
    back = host(p[0] + p[1] + p[2])  # exact in float64
    np.testing.assert_array_equal(back[:, :1000], w.astype(np.float64))
    assert not back[:, 1000:].any()


def test_split_weights_f16_layout(rng):
    """f16x3 planes: B0 = 2^11 h, B2 = h, w s_n ~= h + 2^-11 B1 to 2^-22 relative; the
    column scale is a power of two with max|w| s_n < 16; K padding is zero."""
    from forwardtacotron_amd import ops
    N, K = 40, 300
    w = rng.normal(0, 1, (N, K)).astype(np.float32)
    w[3] *= 1000.0  # a row that needs s_n < 1
    w[5] = 0.0
    blk = host(ops.split_weights_f16(dev(w)))
    Kp = 320
    planes = blk[:3 * N * Kp * 2].view(np.float16).reshape(3, N, Kp).astype(np.float64)
    cs = blk[3 * N * Kp * 2:3 * N * Kp * 2 + 4 * N].view(np.float32).astype(np.float64)
    s = 2.0 ** -11 / cs
    assert np.all(np.log2(s) == np.round(np.log2(s))) and np.all(s <= 1.0)
    assert np.all(np.abs(w).max(1) * s < 16) and s[3] < 1.0 and s[0] == 1.0
    np.testing.assert_array_equal(planes[0], planes[2] * 2048.0)
    back = (planes[2] + planes[1] / 2048.0) / s[:, None]
    ws = w.astype(np.float64)
    assert np.all(np.abs(back[:, :K] - ws) <= 2.0 ** -22 * np.abs(ws) + 1e-30)
    assert not planes[:, :, K:].any()


def test_split_weights_f16_frag_layout(rng):
    """The fragment-major planes hold the row-major planes' elements at
    [n/16][k/32][n%16 + 16 (k/8 % 4)][k%8]; the column scales are the same."""
    from forwardtacotron_amd import ops
    N, K = 48, 80
    w = dev(rng.normal(0, 1, (N, K)).astype(np.float32))
    rm, fm = host(ops.split_weights_f16(w)), host(ops.split_weights_f16(w, frag=True))
    Kp = 96
    a = rm[:3 * N * Kp * 2].view(np.float16).reshape(3, N // 16, 16, Kp // 32, 4, 8)
    b = fm[:3 * N * Kp * 2].view(np.float16).reshape(3, N // 16, Kp // 32, 4, 16, 8)
    np.testing.assert_array_equal(a.transpose(0, 1, 3, 4, 2, 5), b)
    np.testing.assert_array_equal(rm[3 * N * Kp * 2:], fm[3 * N * Kp * 2:])


def test_f16x3_range_guard(rng):
    """An activation beyond the f16 range sets status bit 0 (the output is then invalid);
    in range it stays clear."""
    from forwardtacotron_amd import ops
    x = rng.normal(0, 1, (1, 40, 64)).astype(np.float32)
    w = dev(rng.normal(0, 0.1, (32, 64)).astype(np.float32))
    st = ops.status_word('cuda')
    st.zero_()
    ops.conv1d(dev(x), w, 1, 0, mma=2, w_split=ops.split_weights_f16(w))
    assert int(st.item()) == 0
    x[0, 7, 3] = 1e5
    ops.conv1d(dev(x), w, 1, 0, mma=2, w_split=ops.split_weights_f16(w))
    assert int(st.item()) & 1
    st.zero_()
    with ops.exact_paths():  # fp32 MFMA: no range limit, no status
        y, _ = ops.conv1d(dev(x), w, 1, 0, w_split=ops.split_weights_f16(w))
    assert int(st.item()) == 0
    close(host(y)[0], x[0] @ host(w).T)


# ---------------------------------------------------------------- recurrences
def _rnn_module(cell, fin, H, rng):
    from forwardtacotron_amd.common_layers import BiRNN
    m = BiRNN(fin, H, cell)
    G = 3 if cell == 'gru' else 4
    sd = {}
    for sfx in ('', '_reverse'):
        sd['weight_ih_l0' + sfx] = rng.normal(0, 1 / np.sqrt(fin), (G * H, fin))
        sd['weight_hh_l0' + sfx] = rng.normal(0, 1 / np.sqrt(H), (G * H, H))
        sd['bias_ih_l0' + sfx] = rng.normal(0, 0.1, G * H)
        sd['bias_hh_l0' + sfx] = rng.normal(0, 0.1, G * H)
    sd = {k: v.astype(np.float32) for k, v in sd.items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.cuda(), {'r.' + k: v for k, v in sd.items()}


RNN_MMAS = pytest.mark.parametrize('rnn_mma', [2, 1, 0], ids=['f16x3', 'bf16x6', 'f32'])
GRU_CASES = [pytest.param(H, B, T, m, id=f'{H}-{B}-{T}-{mid}')
             for H, B, T in [(64, 3, 40), (128, 2, 33), (256, 5, 60), (256, 17, 9)]
             for m, mid in ((2, 'f16x3'), (1, 'bf16x6'), (0, 'f32'))]


@pytest.mark.parametrize('H,B,T,rnn_mma', GRU_CASES)
def test_gru_bidir(H, B, T, rng, rnn_mma, monkeypatch):
    """ftmi_conv1d (input projection) + ftmi_rnn_bidir against the numpy oracle."""
    from forwardtacotron_amd import ops
    monkeypatch.setattr(ops, 'RNN_MMA', rnn_mma)
    m, sd = _rnn_module('gru', 256, H, rng)
    x = rng.normal(0, 1, (B, T, 256)).astype(np.float32)
    ref = O.gru_bidir(sd, 'r', x, np.float32)
    close(host(m.forward_cl(dev(x))), ref, rtol=1e-4, atol=1e-5)


@RNN_MMAS
def test_lstm_bidir(rng, rnn_mma, monkeypatch):
    from forwardtacotron_amd import ops
    monkeypatch.setattr(ops, 'RNN_MMA', rnn_mma)
    m, sd = _rnn_module('lstm', 512, 512, rng)
    x = rng.normal(0, 1, (3, 70, 512)).astype(np.float32)
    ref = O.lstm_bidir(sd, 'r', x, np.float32)
    close(host(m.forward_cl(dev(x))), ref, rtol=1e-4, atol=1e-5)


F16X3_SHAPES = [('lstm', 512, 1, 23), ('lstm', 512, 17, 12), ('lstm', 512, 64, 9),
                ('gru', 256, 1, 31), ('gru', 256, 64, 7), ('gru', 256, 130, 5),
                ('gru', 128, 20, 14), ('gru', 64, 64, 11), ('gru', 64, 1, 40)]
# kernel variants of rnn_bidir_kernel: the default (compute-wave h stores), the comm wave's
# h stores (FTMI_RNN_CSTORE=0), and spread (the GRU H 256: 8 units per workgroup while the
# groups fit one workgroup per CU, spread-u16 the 16-unit form with 8 live sequences per
# group); H = 64 has the default only
ROW_VARIANTS = ['default', 'comm', 'spread']
F16X3_CASES = [pytest.param(*shape, v, id=f'{shape[0]}{shape[1]}-B{shape[2]}-{v}')
               for shape in F16X3_SHAPES
               for v in ((ROW_VARIANTS + (['spread-u16'] if shape[1] == 256 else []))
                         if shape[1] >= 128 else ['default'])]


@pytest.mark.parametrize('cell,H,B,T,variant', F16X3_CASES)
def test_rnn_f16x3_kernels(cell, H, B, T, variant, rng, monkeypatch):
    """The f16x3 recurrence over batch sizes that exercise one chunk (B = 1: padded grid,
    one group per XCD), a partial chunk, whole XCDs (B = 64: 8 groups), several launches'
    worth of groups (B = 130) — against the numpy oracle, on every kernel variant.  (B <= 4
    normally takes the GEMV kernel: switched off here.)"""
    from forwardtacotron_amd import ops
    monkeypatch.setattr(ops, 'RNN_MMA', 2)
    monkeypatch.setenv('FTMI_RNN_GEMV', '0')
    monkeypatch.setenv('FTMI_RNN_CSTORE', '0' if variant == 'comm' else '1')
    monkeypatch.setenv('FTMI_RNN_U8', '0' if variant == 'spread-u16' else '1')
    fin = 512 if cell == 'lstm' else 256
    m, sd = _rnn_module(cell, fin, H, rng)
    m.spread = variant.startswith('spread')
    x = rng.normal(0, 1, (B, T, fin)).astype(np.float32)
    ref = (O.lstm_bidir if cell == 'lstm' else O.gru_bidir)(sd, 'r', x, np.float32)
    close(host(m.forward_cl(dev(x))), ref, rtol=1e-4, atol=1e-5)


GEMV_CASES = [('lstm', 512, 1, 37), ('lstm', 512, 2, 20), ('lstm', 512, 4, 15), ('gru', 256, 1, 50),
              ('gru', 256, 3, 21), ('gru', 128, 1, 33), ('gru', 128, 4, 17), ('gru', 64, 1, 40),
              ('gru', 64, 2, 25)]


@pytest.mark.parametrize('cell,H,B,T,kseg', [c + (8,) for c in GEMV_CASES] +
                         [c + (16,) for c in GEMV_CASES if c[1] >= 256])
def test_rnn_gemv(cell, H, B, T, kseg, rng, monkeypatch):
    """B <= 4: the exact-fp32 GEMV recurrence against the numpy oracle in fp64 (a tighter
    bound than the f16x3 kernels') and against the MFMA kernel; kseg: k-segments per row
    (FTMI_RNN_GEMV_KSEG, 16 for H = 512 / 256)."""
    monkeypatch.setenv('FTMI_RNN_GEMV_KSEG', str(kseg))
    fin = 512 if cell == 'lstm' else 256
    m, sd = _rnn_module(cell, fin, H, rng)
    x = rng.normal(0, 1, (B, T, fin)).astype(np.float32)
    f = O.lstm_bidir if cell == 'lstm' else O.gru_bidir
    ref = f({k: v.astype(np.float64) for k, v in sd.items()}, 'r', x.astype(np.float64), np.float64)
    got = host(m.forward_cl(dev(x)))
    close(got, ref, rtol=2e-5, atol=2e-6)
    monkeypatch.setenv('FTMI_RNN_GEMV', '0')
    close(got, host(m.forward_cl(dev(x))), rtol=1e-4, atol=1e-5)


def test_rnn_f16_weight_range_guard(rng, monkeypatch):
    """A W_hh entry beyond the f16 range sets status bit 1 on the f16x3 recurrence."""
    from forwardtacotron_amd import ops
    monkeypatch.setenv('FTMI_RNN_GEMV', '0')  # B = 2 would take the (exact) GEMV kernel
    m, sd = _rnn_module('gru', 256, 64, rng)
    with torch.no_grad():
        m.weight_hh_l0[5, 7] = 1e6
    st = ops.status_word('cuda')
    st.zero_()
    m.forward_cl(dev(rng.normal(0, 1, (2, 5, 256)).astype(np.float32)))
    assert int(st.item()) & 2


@pytest.mark.parametrize('B,variant', [(2, 'gemv'), (9, 'default'), (9, 'spread'), (40, 'spread')])
def test_lstm_through_lr_index_and_lengths(B, variant, rng, monkeypatch):
    """LSTM reading phoneme-rate projections through the LR index map == LSTM over the
    expanded sequence; with lengths it reproduces pack_padded / pad_packed semantics (B = 2:
    the GEMV kernel; B = 9 / 40: the MFMA kernel, compact and spread)."""
    from forwardtacotron_amd import ops
    m, sd = _rnn_module('lstm', 512, 512, rng)
    m.spread = variant == 'spread'
    T = 11
    x = rng.normal(0, 1, (B, T, 512)).astype(np.float32)
    dur = rng.uniform(-0.5, 5.0, (B, T)).astype(np.float32)
    xe, _ = O.length_regulator(x, dur)
    lens = np.array([xe.shape[1] - (5 * b) % 13 for b in range(B)])
    ref = O.lstm_bidir(sd, 'r', xe, np.float32, lengths=lens, pad_value=-11.5129)
    d = dev(dur)
    off, tot, _ = ops.duration_counts(d, apply_fill=False)
    idx = ops.lr_index(off, xe.shape[1])
    y = m.forward_cl(dev(x), T=xe.shape[1], index=idx, lengths=torch.from_numpy(lens),
                     pad_value=-11.5129)
    close(host(y), ref, rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------- integer / byte work
def test_duration_counts_and_lr_bit_exact():
    from conftest import load_golden
    from forwardtacotron_amd import ops
    for name in ('lr_known', 'lr_random'):
        g = load_golden(name)
        d = dev(g['dur_in'])
        off, tot, flag = ops.duration_counts(d, apply_fill=False)
        T_mel = int(tot.max())
        assert T_mel == g['out'].shape[1]
        idx = ops.lr_index(off, T_mel)
        y = ops.length_regulate(dev(g['x']), idx)
        assert np.array_equal(host(y), g['out'])
        assert np.array_equal(host(d), g['dur_out'])
        counts = O.duration_counts(g['dur_in'])
        assert np.array_equal(np.diff(host(off), axis=1), counts)


def test_fill2_rule_on_device():
    from forwardtacotron_amd import ops
    d = dev(np.array([[0.3, -2.0, 0.9], [0.2, 0.1, -0.4]], np.float32))
    off, tot, flag = ops.duration_counts(d, apply_fill=True)
    assert int(flag.item()) == 1 and np.all(host(d) == 2.0) and host(tot).tolist() == [6, 6]
    d = dev(np.array([[1.2, -2.0, 0.9]], np.float32))  # sum trunc = 1 - 2 + 0 = -1 -> fill
    ops.duration_counts(d, apply_fill=True)
    assert np.all(host(d) == 2.0)
    d = dev(np.array([[1.2, -0.5, 0.9]], np.float32))  # sum trunc = 1 -> no fill, clip
    _, tot, flag = ops.duration_counts(d, apply_fill=True)
    assert int(flag.item()) == 0 and host(d).tolist() == [[np.float32(1.2), 0.0, np.float32(0.9)]]


def test_lr_large_bit_exact(rng):
    """Full-size LengthRegulator (B = 64, T = 200, C = 512): bit-exact vs the oracle."""
    from forwardtacotron_amd import ops
    x = rng.normal(0, 1, (64, 200, 512)).astype(np.float32)
    dur = rng.uniform(-1, 14, (64, 200)).astype(np.float32)
    ref, dref = O.length_regulator(x, dur)
    d = dev(dur)
    off, tot, _ = ops.duration_counts(d, apply_fill=False)
    idx = ops.lr_index(off, int(tot.max()))
    y = ops.length_regulate(dev(x), idx)
    assert np.array_equal(host(y), ref) and np.array_equal(host(d), dref)


def test_embedding_and_oob(rng):
    from forwardtacotron_amd import ops
    table = rng.normal(0, 1, (135, 64)).astype(np.float32)
    ids = rng.integers(0, 135, (3, 17))
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    y = ops.embedding(dev(ids), dev(table), err)
    assert np.array_equal(host(y), table[ids]) and int(err.item()) == 0
    ids[0, 0] = 135
    ops.embedding(dev(ids), dev(table), err)
    assert int(err.item()) == 1


def test_series_proj_add_and_rowdot(rng):
    from forwardtacotron_amd import ops
    B, T, C = 2, 19, 512
    x = rng.normal(0, 1, (B, T, C)).astype(np.float32)
    p, e = rng.normal(0, 1, (B, 1, T)).astype(np.float32), rng.normal(0, 1, (B, 1, T)).astype(np.float32)
    wp, we = rng.normal(0, .5, (C, 1, 3)).astype(np.float32), rng.normal(0, .5, (C, 1, 3)).astype(np.float32)
    bp, be = rng.normal(0, .1, C).astype(np.float32), rng.normal(0, .1, C).astype(np.float32)
    ref = x + O.conv1d(p, wp, 1, bp).transpose(0, 2, 1) * np.float32(1.0)
    ref = ref + O.conv1d(e, we, 1, be).transpose(0, 2, 1) * np.float32(0.5)
    xd = dev(x)
    ops.series_proj_add(xd, dev(p), dev(wp.reshape(C, 3)), dev(bp), 1.0, dev(e), dev(we.reshape(C, 3)), dev(be), 0.5)
    close(host(xd), ref)
    w = rng.normal(0, 1, 128).astype(np.float32)
    b = np.array([0.3], np.float32)
    h = rng.normal(0, 1, (B, T, 128)).astype(np.float32)
    close(host(ops.rowdot(dev(h), dev(w), dev(b), 1.3)), (h @ w + b[0]) / np.float32(1.3))


# ---------------------------------------------------------------- slab kernel prefetch
# conv_gemm_slabp_kernel (FTMI_SLAB_PF=1, default) reads the fragments of step s + 1 during
# step s from swizzled, triple-buffered LDS images; its MFMAs run in the same order on the
# same operands as conv_gemm_slab_kernel (FTMI_SLAB_PF=0), so every output is BIT-identical.
SLABP_CASES = [  # B, T, Cin, N, k, residual, transposed-out
    (2, 300, 256, 256, 5, False, False),   # predictor conv
    (3, 301, 96, 200, 7, True, True),      # ragged rows / columns, residual, (B, N, T) copy
    (2, 700, 256, 1024, 9, False, False),  # FastPitch FFN conv1 (k = 9)
    (2, 9, 32, 64, 16, False, False),      # k = 16 > T: every tap masked for some rows
    (4, 70, 64, 1536, 1, False, False),    # k = 1: the slab of chunk 1 stored in the prologue
    (2, 200, 80, 256, 3, True, False),     # Cin = 80: a partial last chunk
    (1, 600, 512, 384, 2, False, False),   # even k
]


@pytest.mark.parametrize('B,T,Cin,N,k,res,tr', SLABP_CASES)
def test_slab_prefetch_bit_identical(B, T, Cin, N, k, res, tr, rng, monkeypatch):
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    monkeypatch.setenv('FTMI_GEMM_SKINNY', '0')
    x = rng.normal(0, 1, (B, T, Cin)).astype(np.float32)
    w = rng.normal(0, 1 / np.sqrt(Cin * k), (N, Cin, k)).astype(np.float32)
    b = rng.normal(0, 0.1, N).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, N).astype(np.float32)
    sh = rng.normal(0, 0.1, N).astype(np.float32)
    r = rng.normal(0, 1, (B, T, N)).astype(np.float32)
    wp = pack_conv(torch.from_numpy(w)).cuda()
    w3 = ops.presplit_for(wp, 2)
    outs = []
    for pf in ('1', '0'):
        monkeypatch.setenv('FTMI_SLAB_PF', pf)
        yt = torch.empty(B, N, T, device='cuda') if tr else None
        y, _ = ops.conv1d(dev(x), wp, k, k // 2, bias=dev(b), relu=True, bn=(dev(sc), dev(sh)),
                          residual=dev(r) if res else None, out_t=yt, mma=2, w_split=w3)
        outs.append((host(y), host(yt) if tr else None))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    if tr:
        np.testing.assert_array_equal(outs[0][1], outs[1][1])
    ref = np.maximum(O.conv1d(x.transpose(0, 2, 1), w, k // 2, b)[:, :, :T], 0)
    ref = ref * sc[None, :, None] + sh[None, :, None]
    if res:
        ref = ref + r.transpose(0, 2, 1)
    close(outs[0][0], ref.transpose(0, 2, 1))


@pytest.mark.parametrize('split_k', [1, 3])
def test_slab_prefetch_split_k_and_pooled_bank(split_k, rng, monkeypatch):
    """The prefetch kernel's split-K partials (3 splits over 8 chunks: 3 + 3 + 2) and the
    pooled bank epilogue with split-row output are bit-identical to the previous kernel's."""
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import pack_conv
    monkeypatch.setenv('FTMI_GEMM_SKINNY', '0')
    B, T, Cin, N, k = 2, 300, 256, 256, 3
    x = dev(rng.normal(0, 1, (B, T, Cin)).astype(np.float32))
    w = pack_conv(torch.from_numpy(rng.normal(0, 0.05, (N, Cin, k)).astype(np.float32))).cuda()
    w3 = ops.presplit_for(w, 2)
    K, C, Cb = 8, 256, 80
    xb = dev(rng.normal(0, 1, (B, T, Cb)).astype(np.float32))
    ws = [rng.normal(0, 1 / np.sqrt(Cb * kk), (C, Cb, kk)).astype(np.float32) for kk in range(1, K + 1)]
    wb = torch.cat([pack_conv(torch.from_numpy(v)).reshape(-1) for v in ws]).cuda()
    wb3 = ops.split_bank_weights(wb, K, Cb, C, 2)
    bsc = dev(rng.uniform(0.5, 1.5, K * C).astype(np.float32))
    bsh = dev(rng.normal(0, 0.1, K * C).astype(np.float32))
    monkeypatch.setattr(ops, '_split_k', lambda *a, **kw: split_k)
    outs = []
    for pf in ('1', '0'):
        monkeypatch.setenv('FTMI_SLAB_PF', pf)
        y, _ = ops.conv1d(x, w, k, k // 2, relu=True, mma=2, w_split=w3)
        assert ops.bank_pools(xb, K, C, w_split=wb3)
        yb = ops.conv_bank(xb, wb, K, C, bsc, bsh, mma=2, w_split=wb3, pool=True, split_out=True)
        outs.append((host(y), host(yb)))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
