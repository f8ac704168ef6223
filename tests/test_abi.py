"""The C-ABI boundary: libftmi.so loads, exports exactly what include/ftmi.h declares, and
rejects bad arguments on the host with FTMI_E_* codes (no GPU needed: these return before
any launch)."""
import ctypes
import re
from pathlib import Path

import pytest

from forwardtacotron_amd import _lib

HEADER = Path(__file__).resolve().parent.parent / 'include' / 'ftmi.h'


def declared():
    text = re.sub(r'/\*.*?\*/', '', HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r'\b(ftmi_[a-z0-9_]+)\s*\(', text)))


def test_header_matches_binding_table():
    assert declared() == sorted(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.ftmi_abi_version() == _lib.ABI_VERSION


def test_exported_symbols_are_plain_c():
    """No C++-mangled entry points: nm shows the ftmi_ names unmangled and nothing else
    global besides them (plus the HIP runtime registration hooks)."""
    import subprocess
    out = subprocess.run(['nm', '-D', '--defined-only', str(_lib.lib_path())],
                         capture_output=True, text=True, check=True).stdout
    names = {l.split()[-1] for l in out.splitlines() if ' T ' in l}
    assert set(declared()) <= names
    assert not any(n.startswith('_Z') and 'ftmi' in n for n in names)


def test_strerror():
    lib = _lib.load()
    assert b'invalid argument' in lib.ftmi_strerror(1001)
    assert lib.ftmi_strerror(0) == b'ok'


@pytest.mark.parametrize('call,code', [
    (lambda L: L.ftmi_embedding(None, 4, None, 135, 256, None, None, None), 1001),
    (lambda L: L.ftmi_conv1d(None, None), 1001),
    (lambda L: L.ftmi_conv_bank(None, 0, 1, 1, 16, None, None, 4, 8, None, None, None, 0, 1, None, None), 1001),
    (lambda L: L.ftmi_conv_bank_split(None, 0, 1, 1, 16, None, None, 4, 8, None, None, None, 0, 1, None, 0, None, 0, None), 1001),
    (lambda L: L.ftmi_conv_bank_split(ctypes.c_void_p(256), 16, 1, 1, 16, ctypes.c_void_p(256), ctypes.c_void_p(256), 4, 8, ctypes.c_void_p(256), ctypes.c_void_p(256), ctypes.c_void_p(256), 32, 2, None, 4, None, 0, None), 1001),
    # pool_out flags: unknown bit / split output rows without the pooled epilogue
    (lambda L: L.ftmi_conv_bank_split(ctypes.c_void_p(256), 16, 1, 1, 16, ctypes.c_void_p(256), ctypes.c_void_p(256), 4, 8, ctypes.c_void_p(256), ctypes.c_void_p(256), ctypes.c_void_p(256), 32, 2, None, 0, None, 8, None), 1001),
    (lambda L: L.ftmi_conv_bank_split(ctypes.c_void_p(256), 16, 1, 1, 16, ctypes.c_void_p(256), ctypes.c_void_p(256), 4, 8, ctypes.c_void_p(256), ctypes.c_void_p(256), ctypes.c_void_p(256), 32, 2, None, 0, None, 2, None), 1003),
    (lambda L: L.ftmi_highway(None, 0, 1, 32, None, None, None, None, None, 0, 1, None, None), 1001),
    (lambda L: L.ftmi_split_weights(None, 4, 4, None, None), 1001),
    (lambda L: L.ftmi_split_weights_f16(None, 4, 4, None, None), 1001),
    (lambda L: L.ftmi_rnn_bidir(0, 1, 1, 64, None, 0, 1, None, None, None, None, None, 0.0, None, 0, 2, None, None, None), 1001),
    (lambda L: L.ftmi_duration_counts(None, 1, 1, 1, 2.0, None, None, None, None), 1001),
    (lambda L: L.ftmi_lr_index(None, 1, 1, 1, None, None), 1001),
    (lambda L: L.ftmi_length_regulate(None, 0, 1, 1, 4, None, 1, None, 0, None), 1001),
    (lambda L: L.ftmi_rowdot(None, 0, 1, 4, None, None, 1.0, None, None), 1001),
    # ftmi_highway_stack: null input, C != 256, Cp % 4, n_out % 512, misaligned x
    (lambda L: L.ftmi_highway_stack(None, 80, 10, 80, 256, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(256), 256, None, None), 1001),
    (lambda L: L.ftmi_highway_stack(ctypes.c_void_p(256), 80, 10, 80, 128, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(512), 256, None, None), 1002),
    (lambda L: L.ftmi_highway_stack(ctypes.c_void_p(256), 80, 10, 78, 256, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(512), 256, None, None), 1002),
    (lambda L: L.ftmi_highway_stack(ctypes.c_void_p(256), 80, 10, 80, 256, ctypes.c_void_p(256), 0, None, None, None, ctypes.c_void_p(256), None, 500, ctypes.c_void_p(1024), 500, None, 0, None, None), 1002),
    # ftmi_highway_stack_spread: no workspace; more rows than one launch of resident workgroups
    (lambda L: L.ftmi_highway_stack_spread(ctypes.c_void_p(256), 80, 10, 80, 256, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(512), 256, None, None, None), 1001),
    (lambda L: L.ftmi_highway_stack_spread(ctypes.c_void_p(256), 80, 2000, 80, 256, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(512), 256, None, ctypes.c_void_p(1024), None), 1003),
    (lambda L: L.ftmi_highway_stack(ctypes.c_void_p(260), 80, 10, 80, 256, ctypes.c_void_p(256), 0, None, None, None, None, None, 0, None, 0, ctypes.c_void_p(512), 256, None, None), 1004),
    (lambda L: L.ftmi_split_weights_f16_frag(None, 16, 4, None, None), 1001),
    (lambda L: L.ftmi_split_weights_f16_frag(ctypes.c_void_p(256), 20, 4, ctypes.c_void_p(256), None), 1002),
    (lambda L: L.ftmi_attention(None, 0, 1, 1, 1, 64, 0, 64, 128, None, 1.0, None, 0, 2, None, None, 0, None), 1001),
    (lambda L: L.ftmi_attention(ctypes.c_void_p(256), 192, 1, 1, 1, 96, 0, 96, 192, None, 1.0, ctypes.c_void_p(256), 96, 2, None, None, 0, None), 1003),
    (lambda L: L.ftmi_attention(ctypes.c_void_p(256), 384, 1, 4, 2, 64, 0, 128, 256, None, 1.0, ctypes.c_void_p(256), 128, 2, None, ctypes.c_void_p(260), 1 << 20, None), 1004),
])
def test_argument_errors(call, code):
    assert call(_lib.load()) == code


def test_conv_shape_errors():
    lib = _lib.load()
    fake = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    a = _lib.ConvArgs()
    a.x, a.w, a.y = fake, fake, fake
    a.B, a.T, a.Cin, a.N, a.k, a.pad = 1, 8, 20, 8, 3, 1  # Cin % 16 != 0
    a.x_stride = 20
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1002
    a.Cin, a.x_stride = 16, 18  # stride not a multiple of 4 floats
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1004
    a.x_stride, a.mma = 16, 7  # unknown matrix path
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1001
    a.mma = 2  # the f16x3 path needs the pre-split planes
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1001
    a.mma, a.x_split = 0, 1  # split rows only on the f16x3 path
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1003
    a.mma, a.w_split, a.maxpool = 2, fake, 1  # ... and never under the maxpool operand
    assert lib.ftmi_conv1d(ctypes.byref(a), None) == 1003


def test_rnn_unsupported_hidden():
    lib = _lib.load()
    fake = ctypes.c_void_p(256)
    rc = lib.ftmi_rnn_bidir(0, 2, 4, 96, fake, 576, 4, None, None, fake, fake, None, 0.0, fake,
                            192, 2, None, fake, None)
    assert rc == 1003  # FTMI_E_UNSUPPORTED before any HIP call (no pending HIP error)


def test_workspace_sizes():
    lib = _lib.load()
    assert lib.ftmi_rnn_workspace_bytes(64, 512, 1) > 0
    assert lib.ftmi_rnn_workspace_bytes(0, 512, 1) == 0
    assert lib.ftmi_rnn_error_offset(64) % 4 == 0


def test_build_id_tracks_flags():
    """a build with extra compile flags carries another id than the default build
    (so _lib.load refuses it as the package library), and the default id is the sources'."""
    from forwardtacotron_amd._srchash import source_hash
    from forwardtacotron_amd.build import build_id
    assert build_id() == source_hash() == _lib.load().ftmi_build_id().decode()
    assert build_id(['-DFTMI_X=1']) != build_id()
    assert build_id(['-DFTMI_X=1']).startswith(source_hash() + '+')


def test_default_library_has_no_invalid_result_switches():
    """the timing experiments that return invalid results with status 0
    (FTMI_RNN_DIAG, FTMI_SLAB_DIAG, FTMI_SKINNY_DIAG, FTMI_BANK_HALVES_DIAG) exist only in the
    diagnostic build (-DFTMI_DIAG, libftmi_stamps.so): the product library never reads them."""
    data = (Path(_lib.__file__).parent / "libftmi.so").read_bytes()
    for name in (b'FTMI_RNN_DIAG', b'FTMI_SLAB_DIAG', b'FTMI_SKINNY_DIAG',
                 b'FTMI_BANK_HALVES_DIAG'):
        assert name not in data, name


def test_highway_stack_spread_sizes():
    """The spread CBHG tail's workgroup count and workspace: 16 workgroups per 64-row block up
    to 1024 rows, none beyond."""
    lib = _lib.load()
    assert lib.ftmi_highway_stack_spread_blocks(120) == 32
    assert lib.ftmi_highway_stack_spread_blocks(816) == 13 * 16
    assert lib.ftmi_highway_stack_spread_blocks(1025) == 0
    assert lib.ftmi_highway_stack_spread_ws_bytes(120) == 2 * 32 * 4 + 2 * 2 * 2 * 64 * 272 * 2
    assert lib.ftmi_highway_stack_spread_ws_bytes(0) == 0


@pytest.mark.gpu
def test_persistent_launch_refused_when_not_resident():
    """The persistent-launch guard (ABI 19): a spread CBHG tail of 1024 rows needs 256
    workgroups resident at once; with the CUs the check may count lowered to 8, the entry
    point returns FTMI_E_UNSUPPORTED before its counter memset or its launch (the status word
    stays clean: no spin timeout), and runs once the limit is lifted."""
    import torch
    from forwardtacotron_amd import ops
    from forwardtacotron_amd.common_layers import CBHG
    torch.manual_seed(3)
    m = CBHG(K=2, in_channels=256, channels=256, proj_channels=[256, 256], num_highways=4).cuda()
    x = torch.randn(1, 1024, 256, device='cuda')
    pre_f, hw_f, b1s, b2s, ih_f, b_in, n_out = m._stack_pack()
    assert ops.hs_spread_blocks(1024, n_out) == 256
    lib = _lib.load()
    st = ops.status_word('cuda')
    st.zero_()
    prev = lib.ftmi_set_resident_cu_limit(8)
    try:
        with pytest.raises(_lib.FtmiError, match='status 1003'):
            ops.highway_stack(x, pre_f, 256, hw_f, b1s, b2s, ih_f, b_in, n_out)
        torch.cuda.synchronize()
        assert int(st.item()) == 0
    finally:
        lib.ftmi_set_resident_cu_limit(prev)
    y, _ = ops.highway_stack(x, pre_f, 256, hw_f, b1s, b2s, ih_f, b_in, n_out)
    torch.cuda.synchronize()
    assert y is not None and torch.isfinite(y).all() and int(st.item()) == 0
