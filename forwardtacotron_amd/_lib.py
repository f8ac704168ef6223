"""ctypes binding of libftmi.so (declarations: include/ftmi.h).

The library is loaded lazily on first use.  torch is imported first so that the HIP
runtime torch ships (SONAME libamdhip64.so.7) is the one libftmi.so binds to: device
pointers and streams are then shared with torch without any interop layer.

There is no fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

from ._srchash import source_hash

_LIB_PATH = Path(os.environ.get('FTMI_LIB', Path(__file__).resolve().parent / 'libftmi.so'))
_lib = None

c_int, c_int64, c_float, c_void_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
P = c_void_p  # every device pointer travels as void*
ABI_VERSION = 19
MMA_F32, MMA_BF16X6, MMA_F16X3 = 0, 1, 2


class ConvArgs(ctypes.Structure):
    """Mirror of ftmi_conv_args (include/ftmi.h)."""
    _fields_ = [
        ('x', P), ('x_stride', c_int64), ('B', c_int), ('T', c_int), ('Cin', c_int),
        ('w', P), ('N', c_int), ('k', c_int), ('pad', c_int),
        ('bias', P), ('relu', c_int), ('bn_scale', P), ('bn_shift', P), ('maxpool', c_int),
        ('residual', P), ('res_stride', c_int64),
        ('y', P), ('y_stride', c_int64), ('yt', P), ('T_out', c_int), ('mma', c_int),
        ('split_k', c_int), ('split_ws', P), ('w_split', P), ('status', P), ('x_split', c_int),
    ]


class WaveRNNArgs(ctypes.Structure):
    """Mirror of ftmi_wavernn_args (include/ftmi.h)."""
    _fields_ = [(n, P) for n in ('w_hh1', 'w_hh2', 'w_ih2a', 'w_fc1a', 'w_fc2a', 'w_fc3', 'b_fc3',
                                 'b_hh1', 'b_hh2', 'u1', 'u2', 'v1', 'wm', 'cond', 'mel', 'xin',
                                 'samples', 'logits', 'workspace', 'status')] + [
        ('seed', ctypes.c_uint64)] + [(n, c_int) for n in (
            'bias_row', 'item_rows', 'frames_per_item', 'hop', 'fold_stride', 'batched', 'B', 'L',
            'n_classes', 'mol', 'rnn_dims', 'fc_dims', 'feat_dims', 'aux_dims')]


class NnlsArgs(ctypes.Structure):
    """Mirror of ftmi_nnls_lbfgsb_args (include/ftmi.h)."""
    _fields_ = [('mel', P)] + [(n, c_int) for n in ('B', 'F', 'n_mels', 'n_bins', 'denorm')] + [
        ('blocks', P)] + [(n, c_int) for n in ('n_blocks', 'groups', 'm', 'max_frames', 'maxiter', 'dbg_stop')] + [
        (n, P) for n in ('rowvals', 'rowptr', 'rowlo', 'bin_rows', 'bin_w', 'pinv', 'workspace', 'S',
                         'active')]


# name -> (restype, argtypes); the exact export list of include/ftmi.h
SIGNATURES = {
    'ftmi_abi_version': (c_int, []),
    'ftmi_build_id': (ctypes.c_char_p, []),
    'ftmi_strerror': (ctypes.c_char_p, [c_int]),
    'ftmi_set_resident_cu_limit': (c_int, [c_int]),
    'ftmi_embedding': (c_int, [P, c_int64, P, c_int64, c_int64, P, P, P]),
    'ftmi_conv1d': (c_int, [ctypes.POINTER(ConvArgs), P]),
    'ftmi_conv_bank': (c_int, [P, c_int64, c_int, c_int, c_int, P, P, c_int, c_int, P, P, P, c_int64,
                               c_int, P, P]),
    'ftmi_conv_bank_split': (c_int, [P, c_int64, c_int, c_int, c_int, P, P, c_int, c_int, P, P, P,
                                     c_int64, c_int, P, c_int, P, c_int, P]),
    'ftmi_conv_bank_halves_ws_floats': (c_int64, [c_int, c_int, c_int, c_int]),
    'ftmi_conv_bank_halves_image_bytes': (c_int64, [c_int, c_int, c_int]),
    'ftmi_conv_bank_halves_image': (c_int, [P, c_int, c_int, c_int, P, P]),
    'ftmi_highway': (c_int, [P, c_int64, c_int64, c_int, P, P, P, P, P, c_int64, c_int, P, P]),
    'ftmi_highway_split': (c_int, [P, c_int64, c_int64, c_int, P, P, P, P, P, c_int64, c_int, P,
                                   c_int, P, P]),
    'ftmi_highway_stack': (c_int, [P, c_int64, c_int64, c_int, c_int, P, c_int, P, P, P, P, P,
                                   c_int, P, c_int64, P, c_int64, P, P]),
    'ftmi_highway_stack_spread_ws_bytes': (c_int64, [c_int64]),
    'ftmi_highway_stack_spread_blocks': (c_int, [c_int64]),
    'ftmi_highway_stack_spread': (c_int, [P, c_int64, c_int64, c_int, c_int, P, c_int, P, P, P, P,
                                          P, c_int, P, c_int64, P, c_int64, P, P, P]),
    'ftmi_split_weights_bytes': (c_int64, [c_int64, c_int64]),
    'ftmi_split_weights': (c_int, [P, c_int64, c_int64, P, P]),
    'ftmi_split_weights_f16_bytes': (c_int64, [c_int64, c_int64]),
    'ftmi_split_rows': (c_int, [P, c_int64, c_int64, c_int, P, c_int64, P, P]),
    'ftmi_split_weights_f16': (c_int, [P, c_int64, c_int64, P, P]),
    'ftmi_split_weights_f16_frag': (c_int, [P, c_int64, c_int64, P, P]),
    'ftmi_panel_proj': (c_int, [P, c_int64, c_int64, c_int, P, c_int, P, P, c_int64, P, P,
                                c_float, P, c_int64, P, P]),
    'ftmi_rnn_workspace_bytes': (c_int64, [c_int, c_int, c_int]),
    'ftmi_rnn_error_offset': (c_int64, [c_int]),
    'ftmi_rnn_blocks': (c_int, [c_int, c_int, c_int, c_int]),
    'ftmi_set_rnn_spin_limit': (ctypes.c_uint32, [ctypes.c_uint32]),
    'ftmi_rnn_bidir': (c_int, [c_int, c_int, c_int, c_int, P, c_int64, c_int, P, P, P, P, P,
                               c_float, P, c_int64, c_int, P, P, P]),
    'ftmi_duration_counts': (c_int, [P, c_int, c_int, c_int, c_float, P, P, P, P]),
    'ftmi_duration_trunc_sum': (c_int, [P, c_int, c_int, P, P]),
    'ftmi_duration_counts_global': (c_int, [P, c_int, c_int, P, c_float, P, P, P, P]),
    'ftmi_lr_index': (c_int, [P, c_int, c_int, c_int, P, P]),
    'ftmi_length_regulate': (c_int, [P, c_int64, c_int, c_int, c_int, P, c_int, P, c_int64, P]),
    'ftmi_series_proj_add': (c_int, [P, c_int64, c_int, c_int, c_int, P, P, P, c_float, P, P, P,
                                     c_float, P]),
    'ftmi_rowdot': (c_int, [P, c_int64, c_int64, c_int, P, P, c_float, P, P]),
    'ftmi_embedding_posenc': (c_int, [P, c_int, c_int, P, c_int64, c_int, P, P, P, P, P]),
    'ftmi_lr_posenc': (c_int, [P, c_int64, c_int, c_int, c_int, P, c_int, P, P, P, c_int64, P]),
    'ftmi_layernorm': (c_int, [P, c_int64, c_int64, c_int, P, P, c_float, P, c_int64, P]),
    'ftmi_attention': (c_int, [P, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P,
                               c_float, P, c_int64, c_int, P, P, c_int64, P]),
    'ftmi_panel_proj_qkv': (c_int, [P, c_int64, c_int, c_int, c_int, P, c_int, P, c_int, P,
                                    c_int64, P, c_int64, P, P]),
    'ftmi_attention_kv': (c_int, [P, c_int64, c_int, c_int, c_int, c_int, P, c_float, P, c_int64,
                                  P, P, c_int64, P]),
    'ftmi_attention_workspace_bytes': (c_int64, [c_int, c_int, c_int, c_int]),
    'ftmi_stft': (c_int, [P, c_int64, c_int, c_int64, P, c_int, c_int, P, P, c_int, P, P, P]),
    'ftmi_mel_spectrogram': (c_int, [P, c_int64, c_int, c_int64, P, c_int, c_int, P, P, c_int, P,
                                     P, P, P, c_int, c_int, P, P]),
    'ftmi_griffinlim_stft': (c_int, [P, c_int64, c_int, c_int64, P, c_int, c_int, P, P, c_int, P,
                                     P, P, c_float, c_int, P, P]),
    'ftmi_spec_mul': (c_int, [P, P, c_int64, P, P]),
    'ftmi_unit_phases': (c_int, [P, c_int, c_int, c_int, P, P]),
    'ftmi_istft_workspace_bytes': (c_int64, [c_int, c_int, c_int]),
    'ftmi_istft': (c_int, [P, c_int, c_int, P, c_int, c_int, P, P, P, P, P, c_int64, c_int64, P]),
    'ftmi_griffinlim_iter': (c_int, [P, P, P, P, c_int, c_int, P, c_int, c_int, P, P, P, c_float,
                                     c_int, P]),
    'ftmi_istft_fused': (c_int, [P, c_int, c_int, P, c_int, c_int, P, P, P, P, c_int64, c_int64, P]),
    'ftmi_wr_stretch_conv': (c_int, [P, c_int64, c_int, c_int, c_int, c_int, P, P, c_int64, c_int,
                                     c_int, P]),
    'ftmi_wavernn_workspace_bytes': (c_int64, []),
    'ftmi_wavernn': (c_int, [ctypes.POINTER(WaveRNNArgs), P]),
    'ftmi_set_wavernn_spin_limit': (ctypes.c_uint32, [ctypes.c_uint32]),
    'ftmi_wr_unfold': (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    'ftmi_mel_nnls': (c_int, [P, c_int, c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P,
                              c_float, c_int, P, P]),
    'ftmi_nnls_lbfgsb_workspace_bytes': (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    'ftmi_nnls_lbfgsb_start': (c_int, [ctypes.POINTER(NnlsArgs), P]),
    'ftmi_nnls_lbfgsb_cycles': (c_int, [ctypes.POINTER(NnlsArgs), c_int, P]),
    'ftmi_nnls_lbfgsb_finish': (c_int, [ctypes.POINTER(NnlsArgs), P, P, P, P]),
}


class FtmiError(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB_PATH


def load():
    """Load libftmi.so and bind every exported symbol; raises if anything is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise FtmiError(f'libftmi.so not found at {_LIB_PATH}; run `python -m forwardtacotron_amd.build` '
                        '(there is no CPU fallback)')
    lib = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the export is missing
        fn.restype = res
        fn.argtypes = args
    if lib.ftmi_abi_version() != ABI_VERSION:
        raise FtmiError('libftmi.so ABI version mismatch')
    built, here = lib.ftmi_build_id().decode(), source_hash()
    if built != here and os.environ.get('FTMI_LIB') is None:
        raise FtmiError(f'{_LIB_PATH} was built from other sources (build id {built[:12]}, '
                        f'sources {here[:12]}): rebuild with `python -m forwardtacotron_amd.build`')
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    """Invoke an ftmi entry point and raise FtmiError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ftmi_strerror(rc).decode()
        raise FtmiError(f'{name} failed with status {rc}: {msg}')
