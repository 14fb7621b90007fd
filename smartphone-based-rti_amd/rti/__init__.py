"""rti -- MI355X-native PTM/HSH reflectance fitter (drop-in for the hot path of
bara96/Smartphone-based-RTI: analysis.py:196-411, interactive_relighting.py:11-39).

    import rti
    coef = rti.fit(I, lu, lv, basis="ptm")          # I: CUDA [N, H, W]
    img = rti.relight(coef, 0.3, -0.2)               # [H, W]

Compute runs in HIP kernels of librti.so (include/rti.h); importing this
package does not touch the GPU.
"""
from . import _lib
from ._lib import RTIError, RTILibraryMissing
from .api import (BASES, apply_operator, basis_eval, basis_id, basis_operator, basis_terms, design_matrix, fit,
                  fit_residual, fit_shared_into, fit_shared_residual_into, fit_with_residual, gram_inverse,
                  interpolate_rbf, interpolate_rbf_perpixel, light_dirs, lsq_factors, pinv, q8_operator, h16_operator, rbf_operator,
                  relight, relight_frame)

__all__ = ["BASES", "RTIError", "RTILibraryMissing", "apply_operator", "basis_eval", "basis_id", "basis_operator",
           "basis_terms", "design_matrix", "fit", "fit_residual", "fit_shared_into", "fit_shared_residual_into",
           "fit_with_residual", "gram_inverse", "interpolate_rbf", "interpolate_rbf_perpixel", "light_dirs",
           "lsq_factors", "pinv", "q8_operator", "h16_operator",
           "rbf_operator", "relight", "relight_frame", "library_path", "load"]

__version__ = "0.1.0"


def library_path():
    return _lib.LIB_PATH


def load():
    """Load librti.so now (raises RTILibraryMissing if it was not built)."""
    return _lib.lib()
