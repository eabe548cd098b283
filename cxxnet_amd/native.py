"""Loaders for the in-tree native libraries.

* ``rt()``      -> the pybind11 runtime module (config parser, NetConfig, IO, metrics).
* ``kernels()`` -> ctypes handle on ``libcxxnet_kernels.so`` (all HIP kernels, gfx950).

Both are built in-tree by ``cxxnet_amd.build``.  On a machine with a GPU the
kernel library is mandatory: a missing library raises instead of silently
falling back to another implementation.
"""
from __future__ import annotations

import ctypes
import importlib.machinery
import importlib.util
import os
import sysconfig
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
_NATIVE = os.environ.get("CXXNET_NATIVE_DIR") or os.path.join(_PKG, "_native")
if not os.path.isabs(_NATIVE):
    _NATIVE = os.path.abspath(_NATIVE)
_lock = threading.Lock()
_rt = None
_k = None


def _load_ext(name: str, path: str):
    loader = importlib.machinery.ExtensionFileLoader(name, path)
    spec = importlib.util.spec_from_file_location(name, path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def rt():
    """The native runtime module (builds it on first use if absent)."""
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                path = os.path.join(_NATIVE, "_cxxnet_rt" + sysconfig.get_config_var("EXT_SUFFIX"))
                if not os.path.exists(path):
                    from . import build
                    build.build_runtime()
                _rt = _load_ext("_cxxnet_rt", path)
    return _rt


class CxnOperand(ctypes.Structure):
    _fields_ = [
        ("ptr", ctypes.c_void_p), ("gstride", ctypes.c_long), ("nbytes", ctypes.c_long),
        ("ld", ctypes.c_int), ("rows", ctypes.c_int), ("kdim", ctypes.c_int),
        ("H", ctypes.c_int), ("W", ctypes.c_int), ("C", ctypes.c_int),
        ("Ho", ctypes.c_int), ("Wo", ctypes.c_int), ("KH", ctypes.c_int), ("KW", ctypes.c_int),
        ("stride", ctypes.c_int), ("pad_h", ctypes.c_int), ("pad_w", ctypes.c_int),
        ("dil", ctypes.c_int), ("Cg", ctypes.c_int),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_U = ctypes.c_uint

_SIGS = {
    "cxn_gemm": [ctypes.POINTER(CxnOperand), ctypes.POINTER(CxnOperand), _I, _I, _I, _I,
                 _P, _L, _I, _F, _P, _L, _I, _I, _I, _I, _I, _I, _L, _P],
    "cxn_gemm_glds_sgd": [ctypes.POINTER(CxnOperand), ctypes.POINTER(CxnOperand), _I, _F, _P, _P, _P, _F, _F, _F, _F,
                          _P, _I, _P],
    "cxn_gemm_set_group": [_I],
    "cxn_set_kernel_variant": [_I, _I],
    "cxn_gemm_glds_add": [ctypes.POINTER(CxnOperand), ctypes.POINTER(CxnOperand), _I, _I, _P, _L, _I, _P, _I, _I, _I,
                          _P],
    "cxn_gemm_glds_split": [ctypes.POINTER(CxnOperand), ctypes.POINTER(CxnOperand), _I, _I, _P, _I, _P, _I, _I, _P,
                            _I, _I, _P],
    "cxn_gemm_glds": [ctypes.POINTER(CxnOperand), ctypes.POINTER(CxnOperand), _I, _I, _P, _L, _I, _F, _P, _L, _I,
                      _I, _I, _I, _I, _I, _L, _P, _P, _L, _I, _P],
    "cxn_pad_rows": [_P, _P, _L, _I, _I, _P],
    "cxn_pad_interior": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cxn_zero": [_P, _L, _P],
    "cxn_add_rows_f32": [_P, _P, _L, _I, _I, _P],
    "cxn_conv_rowrun_fwd": [_P, _L, _P, _P, _P] + [_I] * 12 + [_P],
    "cxn_conv_fewc_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cxn_chan_reduce": [_P, _P, _P, _P, _L, _I, _I, _P],
    "cxn_bn_stats": [_P, _P, _P, _P, _L, _I, _F, _P],
    "cxn_bn_fwd": [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "cxn_bn_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "cxn_rand_fill": [_P, _L, _U, _I, _F, _F, _P],
    "cxn_prelu": [_P, _P, _P, _P, _L, _I, _U, _P, _F, _I, _P],
    "cxn_insanity": [_P, _P, _P, _P, _L, _F, _F, _I, _U, _P, _I, _P],
    "cxn_ins_pool_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _U, _P, _P],
    "cxn_ins_pool_bwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _U, _P, _P],
    "cxn_splitk_finalize": [_P, _I, _L, _P, _L, _I, _P, _I, _I, _P],
    "cxn_splitk_finalize_dropout": [_P, _I, _L, _P, _L, _I, _P, _I, _U, _P, _F, _P],
    "cxn_splitk_accumulate": [_P, _I, _L, _P, _P],
    "cxn_set_deterministic": [_I],
    "cxn_pool_bwd_tie_all": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cxn_metric_eval": [_P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "cxn_nchw_f32_to_nhwc_bf16": [_P, _P, _I, _I, _I, _I, _I, _I, _F, _P],
    "cxn_image_u8_to_nhwc_bf16": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P, _P],
    "cxn_zero_ranges": [_P, _P, _P, _I, _P],
    "cxn_jpeg_idct": [_P, _P, _P, _L, _P, _P],
    "cxn_jpeg_color": [_P, _P, _P, _I, _I, _I, _I, _P, _P],
    "cxn_nhwc_bf16_to_nchw_f32": [_P, _P, _I, _I, _I, _I, _I, _I, _P],
    "cxn_transpose": [_P, _P, _I, _I, _I, _P],
    "cxn_conv_weight_flip": [_P, _P, _I, _I, _I, _I, _I, _P],
    "cxn_conv_weight_flip_multi": [_P, _P, _P, _I, _P],
    "cxn_pool_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cxn_pool_bwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _L, _P],
    "cxn_lrn_fwd": [_P, _P, _L, _I, _I, _F, _F, _F, _P],
    "cxn_lrn_bwd": [_P, _P, _P, _L, _I, _I, _F, _F, _F, _I, _P],
    "cxn_lrn_bwd_db": [_P, _P, _P, _L, _I, _I, _F, _F, _F, _I, _P, _P, _L, _P],
    "cxn_pool_lrn_fwd": [_P, _P, _P, _P] + [_I] * 8 + [_F, _F, _F, _P],
    "cxn_lrn_pool_bwd": [_P, _P, _P, _P] + [_I] * 8 + [_F, _F, _F, _P, _P, _L, _I, _P],
    "cxn_act_fwd": [_P, _P, _P, _L, _I, _F, _P],
    "cxn_act_bwd": [_P, _P, _P, _L, _I, _F, _P],
    "cxn_dropout": [_P, _P, _L, _U, _P, _F, _P],
    "cxn_softmax": [_P, _P, _P, _I, _I, _P],
    "cxn_loss_grad": [_P, _P, _P, _I, _I, _I, _F, _I, _P],
    "cxn_colsum": [_P, _P, _L, _I, _P, _L, _P],
    "cxn_colsum_multi": [_P, _P, _P, _P, _P, _I, _P, _P],
    "cxn_concat": [_P, _P, _I, _P, _I, _L, _I, _I, _P],
    "cxn_cast_f32_bf16": [_P, _P, _L, _P],
    "cxn_add_bf16": [_P, _P, _P, _L, _P],
    "cxn_fanout_bf16": [_P, _P, _P, _P, _P, _I, _L, _P],
    "cxn_sum_bf16": [_P, _P, _P, _P, _I, _P, _L, _P, _I],
    "cxn_channel_copy": [_P, _I, _I, _P, _I, _I, _I, _L, _I, _P],
    "cxn_fused_update": [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _F, _F, _P],
    "cxn_nonfinite_check": [_P, _L, _P, _P],
    "cxn_scale_f32": [_P, _L, _F, _P],
    "cxn_add_i32": [_P, _I, _P],
    # launch-list recorder (csrc/kernels/launch_list.hip)
    "cxn_rec_begin": [],
    "cxn_rec_end": [],
    "cxn_rec_size": [_P],
    "cxn_rec_replay": [_P, _P],
    "cxn_rec_replay_many": [_P, _I, _P],
    "cxn_rec_free": [_P],
    "cxn_copy_d2d": [_P, _P, _L, _P],
    "cxn_conv_wgrad_direct": [_P, _P, _P, _P, _P, _L] + [_I] * 14 + [_F, _P],
    "cxn_conv_wgrad_rowrun": [_P, _P, _P, _P, _L] + [_I] * 12 + [_F, _P],
    "cxn_conv_rowrun_fwd2": [_P, _P, _P, _P] + [_I] * 13 + [_P],
    "cxn_conv_direct": [_P, _I, _P, _P, _P, _I, _P, _L, _P] + [_I] * 10 + [_P],
}
_RESTYPE = {"cxn_rec_end": ctypes.c_void_p, "cxn_rec_free": None, "cxn_conv_wgrad_direct": ctypes.c_long,
            "cxn_conv_wgrad_rowrun": ctypes.c_long,
            "cxn_conv_direct": ctypes.c_long}


def kernel_lib_path() -> str:
    return os.path.join(_NATIVE, "libcxxnet_kernels.so")


def kernels():
    """ctypes handle on the HIP kernel library; raises if it cannot be loaded."""
    global _k
    if _k is None:
        with _lock:
            if _k is None:
                path = kernel_lib_path()
                if not os.path.exists(path):
                    from . import build
                    build.build_kernels()
                lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                for name, args in _SIGS.items():
                    fn = getattr(lib, name)
                    fn.argtypes = args
                    fn.restype = _RESTYPE.get(name, ctypes.c_int)
                _k = lib
    return _k


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"cxxnet_amd kernel {what} failed (rc={rc})")
