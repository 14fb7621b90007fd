"""ctypes binding of ``librti.so`` (the C ABI declared in ``include/rti.h``).

The library is built in-tree (``make -C smartphone-based-rti_amd`` or
``__graft_entry__.build()``).  There is no fallback: if the library is missing
every call raises ``RTILibraryMissing``.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTI_LIBRARY", os.path.join(HERE, "librti.so"))

# ---- constants mirrored from include/rti.h (tests/test_abi.py checks they agree) ----
RTI_OK = 0
RTI_ERR_BAD_ARG = 1
RTI_ERR_UNSUPPORTED = 2
RTI_ERR_HIP = 3
RTI_ERR_SINGULAR = 4

RTI_BASIS_PTM6 = 0
RTI_BASIS_HSH16 = 1
RTI_BASIS_HSH9 = 2

RTI_F32 = 0
RTI_U8 = 1
RTI_I32 = 2
RTI_F64 = 3

RTI_COEF_PIXEL_MAJOR = 0
RTI_COEF_PLANAR = 1

RTI_OUT_EVAL_MAJOR = 0
RTI_OUT_PIXEL_MAJOR = 1

RTI_KERNEL_AUTO = 0
RTI_KERNEL_VALU = 1
RTI_KERNEL_MFMA = 2
RTI_KERNEL_TILE = 3
RTI_KERNEL_NONTEMPORAL = 0x100
RTI_KERNEL_PINV_LDS = 0x200
RTI_KERNEL_NT_STORE = 0x400
RTI_KERNEL_STAGE = 0x800
RTI_KERNEL_ROTATE = 0x10000000  # measurement variant: per-wave rotated light order (AUTO PTM-6 fp32)
RTI_PM_VALU_STREAM = 1  # rti_fit_shared_pm_plan forms (include/rti.h)
RTI_PM_MFMA_STREAM = 2
RTI_PM_BLOCK = 3
RTI_PM_DIRECT = 4
RTI_KERNEL_ONE_LAUNCH = 0x20000000  # measurement variant: AUTO without launch generations
RTI_KERNEL_ROUNDS = 0x40000000  # measurement variant: AUTO generations as rounds of one launch
RTI_KERNEL_CHUNKS_SHIFT = 12  # VALU chunks per lane in bits 12-15 (0 = AUTO)
RTI_KERNEL_TILE_PLANES_SHIFT = 16  # TILE kernel: light planes per wave and step in bits 16-19 (0 = 2)
RTI_KERNEL_TILE_DEPTH_SHIFT = 20  # TILE kernel: tiles in the LDS ring in bits 20-23 (0 = 2)
RTI_KERNEL_TILE_WAVES_SHIFT = 24  # TILE kernel: waves per workgroup in bits 24-27 (0 = 4; 8 = wide form)


class RTILibraryMissing(ImportError):
    pass


class RTIError(RuntimeError):
    def __init__(self, status, message):
        super().__init__(message)
        self.status = status


_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_double = ctypes.c_double
_c_float_p = ctypes.POINTER(ctypes.c_float)
_c_double_p = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); every symbol of include/rti.h
SIGNATURES = {
    "rti_version": (_c_int, []),
    "rti_status_string": (ctypes.c_char_p, [_c_int]),
    "rti_last_error": (ctypes.c_char_p, []),
    "rti_last_launch_count": (ctypes.c_int, []),
    "rti_rbf_last_chol_grid": (_c_i64, []),
    "rti_basis_terms": (_c_int, [_c_int]),
    "rti_device_count": (_c_int, []),
    "rti_design_matrix": (_c_int, [_c_int, _c_float_p, _c_float_p, _c_int, _c_double_p]),
    "rti_pinv": (_c_int, [_c_int, _c_float_p, _c_float_p, _c_int, _c_double, _c_double_p]),
    "rti_basis_eval": (_c_int, [_c_int, _c_double_p, _c_double_p, _c_int, _c_double_p]),
    "rti_gram_inverse": (_c_int, [_c_int, _c_float_p, _c_float_p, _c_int, _c_double, _c_double_p]),
    "rti_lsq_factors": (_c_int, [_c_int, _c_float_p, _c_float_p, _c_int, _c_double, _c_double_p, _c_double_p]),
    "rti_fit_shared": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_int, _c_i64, _c_int, _c_i64, _c_i64,
                                _c_void_p, _c_int, _c_i64, _c_int, _c_void_p]),
    "rti_fit_shared_pm": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_int, _c_i64, _c_int, _c_i64, _c_i64,
                                   _c_void_p, _c_int, _c_i64, _c_int, _c_void_p]),
    "rti_fit_shared_pm_plan": (_c_int, [_c_int, _c_int, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int]),
    "rti_q8_operator_bytes": (_c_i64, [_c_int, _c_int]),
    "rti_q8_operator": (_c_int, [_c_double_p, _c_int, _c_int, _c_void_p]),
    "rti_fit_shared_q8_max_lights": (_c_int, []),
    "rti_fit_shared_q8": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_i64, _c_int, _c_i64, _c_i64, _c_void_p,
                                   _c_int, _c_i64, _c_int, _c_void_p]),
    "rti_h16_operator_bytes": (_c_i64, [_c_int, _c_int]),
    "rti_h16_operator": (_c_int, [_c_double_p, _c_int, _c_int, _c_void_p]),
    "rti_fit_shared_h16_max_lights": (_c_int, []),
    "rti_fit_shared_h16": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_i64, _c_int, _c_i64, _c_i64, _c_void_p,
                                    _c_int, _c_i64, _c_int, _c_void_p]),
    "rti_fit_residual_blocks": (_c_i64, [_c_i64]),
    "rti_fit_residual": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_int, _c_i64, _c_int, _c_i64, _c_i64,
                                  _c_void_p, _c_int, _c_i64, _c_void_p, _c_void_p, _c_void_p]),
    "rti_fit_shared_residual_blocks": (_c_i64, [_c_i64]),
    "rti_fit_shared_residual": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_void_p, _c_int, _c_i64, _c_int,
                                         _c_i64, _c_i64, _c_void_p, _c_int, _c_i64, _c_void_p, _c_void_p, _c_int,
                                         _c_void_p]),
    "rti_fit_shared_residual_svd": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_void_p, _c_int, _c_i64,
                                             _c_int, _c_i64, _c_i64, _c_void_p, _c_int, _c_i64, _c_void_p, _c_void_p,
                                             _c_int, _c_void_p]),
    "rti_fit_perpixel_cam": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_int, _c_int, _c_int, _c_i64, _c_double,
                                      _c_double, _c_double, _c_void_p, _c_int, _c_int, _c_void_p]),
    "rti_fit_perpixel_dirs": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_i64, _c_double,
                                       _c_void_p, _c_int, _c_int, _c_void_p]),
    "rti_light_dirs": (_c_int, [_c_void_p, _c_int, _c_int, _c_int, _c_double, _c_double, _c_void_p, _c_void_p,
                                _c_void_p]),
    "rti_rbf_operator": (_c_int, [_c_float_p, _c_float_p, _c_int, _c_double_p, _c_double_p, _c_int, _c_double_p]),
    "rti_basis_operator": (_c_int, [_c_int, _c_float_p, _c_float_p, _c_int, _c_double_p, _c_double_p, _c_int, _c_double,
                                    _c_double_p]),
    "rti_apply_operator": (_c_int, [_c_void_p, _c_int, _c_int, _c_i64, _c_void_p, _c_int, _c_i64, _c_int, _c_i64,
                                    _c_i64, _c_void_p, _c_int, _c_i64, _c_i64, _c_void_p]),
    "rti_operator_split_f16": (_c_int, [_c_double_p, _c_int, _c_int, _c_i64, _c_int, _c_void_p, _c_void_p,
                                        ctypes.POINTER(ctypes.c_float)]),
    "rti_apply_operator_f16": (_c_int, [_c_void_p, _c_void_p, _c_int, ctypes.c_float, _c_int, _c_int, _c_void_p, _c_int,
                                        _c_i64, _c_int, _c_i64, _c_i64, _c_void_p, _c_int, _c_i64, _c_i64, _c_void_p]),
    "rti_rbf_perpixel": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_i64, _c_void_p, _c_int,
                                  _c_void_p, _c_int, _c_int, _c_void_p, _c_void_p]),
    "rti_rbf_perpixel_ex": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_i64, _c_void_p, _c_int,
                                     _c_void_p, _c_int, _c_int, _c_void_p, _c_void_p, _c_void_p]),
    "rti_relight": (_c_int, [_c_void_p, _c_int, _c_int, _c_i64, _c_int, _c_void_p, _c_int, _c_void_p, _c_int,
                             _c_int, _c_void_p]),
    "rti_relight_frame": (_c_int, [_c_void_p, _c_int, _c_int, _c_int, _c_i64, _c_double, _c_double, _c_void_p,
                                   _c_void_p, _c_void_p]),
}

_lock = threading.Lock()
_lib = None


def lib():
    """Load librti.so once and declare every signature."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RTILibraryMissing(
                    f"librti.so not found at {LIB_PATH}: build it with `make -C smartphone-based-rti_amd` "
                    "(or __graft_entry__.build()); there is no CPU fallback")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(status, fn_name):
    """Raise the Python exception matching an RTI status (RTI_OK passes)."""
    if status == RTI_OK:
        return
    msg = lib().rti_last_error().decode(errors="replace") or fn_name
    if status == RTI_ERR_BAD_ARG:
        raise ValueError(msg)
    if status == RTI_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if status == RTI_ERR_SINGULAR:
        import numpy as np

        raise np.linalg.LinAlgError(msg)  # what the reference's SciPy Rbf raises
    raise RTIError(status, msg)
