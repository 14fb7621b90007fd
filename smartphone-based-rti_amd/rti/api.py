"""Native API: ``fit()`` / ``relight()`` on CUDA (HIP) tensors through librti.so.

Every compute call goes to a HIP kernel of ``librti.so`` on the caller's
current torch stream.  Host-side work is limited to the k×N pseudo-inverse
(``rti_pinv``, also native) and argument marshalling; there is no CPU path for
the fit or the relight, and CPU tensors are rejected.

Reference mapping (bara96/Smartphone-based-RTI @ v0):
  * ``fit(mode="shared")``   — analysis.py:321-363 + :280-298, one pseudo-inverse
    for every pixel (directional lights).
  * ``fit(mode="perpixel")`` — the reference's own geometry: each pixel's light
    list from compute_intensities (analysis.py:196-246), solved per pixel.
  * ``relight()``            — analysis.py:300-315 (grid evaluation),
    analysis.py:375-411 (int32 tables), interactive_relighting.py:25-36 (clip).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L

BASES = {
    "ptm": L.RTI_BASIS_PTM6, "ptm6": L.RTI_BASIS_PTM6,
    "hsh": L.RTI_BASIS_HSH16, "hsh3": L.RTI_BASIS_HSH16, "hsh16": L.RTI_BASIS_HSH16,
    "hsh2": L.RTI_BASIS_HSH9, "hsh9": L.RTI_BASIS_HSH9,
}
_KERNELS = {"auto": L.RTI_KERNEL_AUTO, "valu": L.RTI_KERNEL_VALU, "mfma": L.RTI_KERNEL_MFMA, "tile": L.RTI_KERNEL_TILE}
_IN_DTYPES = {torch.float32: L.RTI_F32, torch.uint8: L.RTI_U8, torch.int32: L.RTI_I32}
_COEF_DTYPES = {torch.float32: L.RTI_F32, torch.float64: L.RTI_F64}
_OUT_DTYPES = {torch.float32: L.RTI_F32, torch.float64: L.RTI_F64, torch.int32: L.RTI_I32, torch.uint8: L.RTI_U8}


def basis_id(basis):
    if isinstance(basis, int):
        return basis
    try:
        return BASES[basis.lower()]
    except (KeyError, AttributeError):
        raise ValueError(f"unknown basis {basis!r}; expected one of {sorted(BASES)}") from None


def basis_terms(basis):
    return L.lib().rti_basis_terms(basis_id(basis))


def _f32_host(x, name):
    a = np.ascontiguousarray(np.asarray(x.detach().cpu() if torch.is_tensor(x) else x, dtype=np.float32).ravel())
    if a.size == 0:
        raise ValueError(f"{name} is empty")
    return a


def _fptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def design_matrix(lu, lv, basis="ptm"):
    """Host fp64 design matrix [N, k] (analysis.py:280-291 for PTM)."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    b = basis_id(basis)
    A = np.empty((lu.size, basis_terms(b)), dtype=np.float64)
    L.check(L.lib().rti_design_matrix(b, _fptr(lu), _fptr(lv), lu.size, _dptr(A)), "rti_design_matrix")
    return A


def pinv(lu, lv, basis="ptm", rcond=None):
    """Host fp64 pseudo-inverse [k, N] of the shared design (analysis.py:293-298).

    ``rcond=None`` keeps the reference's semantics (no threshold)."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    b = basis_id(basis)
    out = np.empty((basis_terms(b), lu.size), dtype=np.float64)
    rc = -1.0 if rcond is None else float(rcond)
    L.check(L.lib().rti_pinv(b, _fptr(lu), _fptr(lv), lu.size, rc, _dptr(out)), "rti_pinv")
    return out


def gram_inverse(lu, lv, basis="ptm", rcond=None):
    """Host fp64 Gram (pseudo-)inverse (AᵀA)⁺ [k, k] of the shared design (pinv = ginv·Aᵀ; the
    same SVD and rcond semantics as ``pinv``)."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    b = basis_id(basis)
    k = basis_terms(b)
    out = np.empty((k, k), dtype=np.float64)
    rc = -1.0 if rcond is None else float(rcond)
    L.check(L.lib().rti_gram_inverse(b, _fptr(lu), _fptr(lv), lu.size, rc, _dptr(out)), "rti_gram_inverse")
    return out


def lsq_factors(lu, lv, basis="ptm", rcond=None):
    """Host fp64 thin-SVD factors ``(U [N, k], W [k, k])`` of the shared design, split as the
    reference's solve is (analysis.py:295-298: ``c = uᵀL; w = c/s; a = vᵀw``): U = the orthonormal
    left singular vectors, W = V Σ⁻¹, so pinv = W·Uᵀ (rcond as ``pinv``)."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    b = basis_id(basis)
    k = basis_terms(b)
    U = np.empty((lu.size, k), dtype=np.float64)
    W = np.empty((k, k), dtype=np.float64)
    rc = -1.0 if rcond is None else float(rcond)
    L.check(L.lib().rti_lsq_factors(b, _fptr(lu), _fptr(lv), lu.size, rc, _dptr(U), _dptr(W)), "rti_lsq_factors")
    return U, W


def q8_operator(pinv64):
    """Host: the fixed-point int8-digit form of an fp64 operator [k, N] for ``rti_fit_shared_q8`` (8-bit
    stacks on the int8 matrix cores; layout in csrc/rti_q8.h).  Raises ValueError for non-finite entries."""
    pv = np.ascontiguousarray(np.asarray(pinv64, np.float64))
    k, N = pv.shape
    nb = int(L.lib().rti_q8_operator_bytes(k, N))
    if nb <= 0:
        raise ValueError(f"no q8 operator for k={k}, N={N}")
    op = np.zeros(nb, dtype=np.uint8)
    L.check(L.lib().rti_q8_operator(_dptr(pv), k, N, ctypes.c_void_p(op.ctypes.data)), "rti_q8_operator")
    return op


def h16_operator(pinv64):
    """Host: the split-fp16 form of an fp64 operator [k, N] for ``rti_fit_shared_h16`` (8-bit stacks on the
    fp16 matrix cores; layout in csrc/rti_fit_h16.hip).  Raises ValueError for non-finite entries."""
    pv = np.ascontiguousarray(np.asarray(pinv64, np.float64))
    k, N = pv.shape
    nb = int(L.lib().rti_h16_operator_bytes(k, N))
    if nb <= 0:
        raise ValueError(f"no h16 operator for k={k}, N={N}")
    op = np.zeros(nb, dtype=np.uint8)
    L.check(L.lib().rti_h16_operator(_dptr(pv), k, N, ctypes.c_void_p(op.ctypes.data)), "rti_h16_operator")
    return op


def _check_operator(op_dev, nbytes, form, k, N):
    """The kernels copy exactly rti_*_operator_bytes(k, N) bytes of the operator into LDS: one built for
    another (k, N) would be read out of range or misread, so its size must match (the C ABI cannot check
    a device buffer it is not given the size of)."""
    if op_dev.dtype != torch.uint8 or op_dev.numel() != nbytes:
        raise ValueError(f"{form} operator of {op_dev.numel()} {op_dev.dtype} elements, expected {nbytes} uint8 "
                         f"bytes for k={k}, N={N}: build it with rti.{form}_operator(pinv) for this light set")


def fit_h16_into(op_dev, I, coef, *, k, layout="pixel", flags=0):
    """Launch ``rti_fit_shared_h16`` on preallocated tensors: op_dev = h16_operator(...) on the device
    (uint8), I a contiguous uint8 CUDA [N, P] or [C, N, P] stack, coef fp32 as fit_shared_into."""
    if I.dim() == 2:
        C, (N, P) = 1, I.shape
    else:
        C, N, P = I.shape
    _check_operator(op_dev, int(L.lib().rti_h16_operator_bytes(k, N)), "h16", k, N)
    st = L.lib().rti_fit_shared_h16(_vp(op_dev), k, N, _vp(I), P, C, P, N * P, _vp(coef), _layout_id(layout),
                                    P * k, int(flags), _stream_of(I))
    L.check(st, "rti_fit_shared_h16")
    return coef


def q8_supported(I, k, N, P, kernel="q8"):
    """Whether ``rti_fit_shared_q8`` (kernel="q8") or ``rti_fit_shared_h16`` (kernel="h16") takes this contiguous
    stack of P-pixel planes (uint8, k in {6, 9, 16}, N within the kernel's LDS budget, 16-byte aligned planes)."""
    fn = L.lib().rti_fit_shared_h16_max_lights if kernel == "h16" else L.lib().rti_fit_shared_q8_max_lights
    if I.dtype != torch.uint8 or k not in (6, 9, 16) or N > int(fn()):
        return False
    return P % 16 == 0 and I.data_ptr() % 16 == 0


def fit_q8_into(op_dev, I, coef, *, k, layout="pixel", flags=0):
    """Launch ``rti_fit_shared_q8`` on preallocated tensors: op_dev = q8_operator(...) on the device (uint8),
    I a contiguous uint8 CUDA [N, P] or [C, N, P] stack, coef fp32 as fit_shared_into."""
    if I.dim() == 2:
        C, (N, P) = 1, I.shape
    else:
        C, N, P = I.shape
    _check_operator(op_dev, int(L.lib().rti_q8_operator_bytes(k, N)), "q8", k, N)
    st = L.lib().rti_fit_shared_q8(_vp(op_dev), k, N, _vp(I), P, C, P, N * P, _vp(coef), _layout_id(layout), P * k,
                                   int(flags), _stream_of(I))
    L.check(st, "rti_fit_shared_q8")
    return coef


_PM_KERNELS = ("auto", "valu", "mfma", "tile")  # the selectors rti_fit_shared_pm honours


def _fit_shared_pixel_major(I, lu, lv, b, k, rcond, cl, kernel, given_pixel_major):
    """rti.fit(mode="shared") on a pixel-major stack: ``rti_fit_shared_pm`` on the tensor's own memory.
    Integer kernel words pass through unchanged (the C entry refuses bits it does not document)."""
    if isinstance(kernel, str) and kernel not in _PM_KERNELS:
        raise NotImplementedError(f"kernel={kernel!r} does not take pixel-major stacks (rti_fit_shared_pm: "
                                  f"{', '.join(_PM_KERNELS)}); pass stack='light' with a light-major stack")
    if given_pixel_major:
        if I.dim() == 2:
            spatial, C = (I.shape[0],), 1
        elif I.dim() == 3:
            spatial, C = tuple(I.shape[:2]), 1
        elif I.dim() == 4:
            spatial, C = tuple(I.shape[1:3]), I.shape[0]
        else:
            raise ValueError("pixel-major I must be [P, N], [H, W, N] or [C, H, W, N]")
        N = I.shape[-1]
        v = I if I.stride(-1) == 1 else I.contiguous()
        if v.dim() == 3 and C == 1:
            v = v.reshape(-1, N)
        v = v.reshape(C, -1, N)
        lead4 = I.dim() == 4
    else:
        v = _pixel_major_of(I)
        C, N = v.shape[0], v.shape[2]
        spatial = tuple(I.shape[-2:]) if I.dim() >= 3 else (I.shape[-1],)
        lead4 = I.dim() == 4
    P = v.shape[1]
    if N < k:
        raise ValueError(f"shapes not aligned: {N} lights < {k} basis terms (analysis.py:298)")
    pv = pinv(lu, lv, b, rcond)
    if pv.shape[1] != N:
        raise ValueError(f"{pv.shape[1]} light directions for {N} intensity values per pixel")
    if I.dtype not in _IN_DTYPES:
        raise ValueError(f"I dtype {I.dtype} unsupported (float32, uint8 or int32)")
    coef = torch.empty((C, P, k) if cl == L.RTI_COEF_PIXEL_MAJOR else (C, k, P), dtype=torch.float32,
                       device=I.device)
    fit_shared_pm_into(torch.as_tensor(pv.astype(np.float32), device=I.device), v, coef, k=k, layout=cl,
                       kernel=kernel)
    out = coef.reshape((C,) + spatial + (k,)) if cl == L.RTI_COEF_PIXEL_MAJOR else coef.reshape((C, k) + spatial)
    return out if lead4 else out[0]


def basis_eval(lu, lv, basis="ptm"):
    """Host fp64 basis values [E, k] at (lu, lv)."""
    lu = np.ascontiguousarray(np.asarray(lu, np.float64).ravel())
    lv = np.ascontiguousarray(np.asarray(lv, np.float64).ravel())
    b = basis_id(basis)
    out = np.empty((lu.size, basis_terms(b)), np.float64)
    L.check(L.lib().rti_basis_eval(b, _dptr(lu), _dptr(lv), lu.size, _dptr(out)), "rti_basis_eval")
    return out


def _require_cuda(t, name):
    if not torch.is_tensor(t) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor: librti runs only on the GPU, there is no CPU path")


def _stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def _layout_id(layout):
    if layout in ("pixel", "pixel_major", L.RTI_COEF_PIXEL_MAJOR):
        return L.RTI_COEF_PIXEL_MAJOR
    if layout in ("planar", L.RTI_COEF_PLANAR):
        return L.RTI_COEF_PLANAR
    raise ValueError(f"unknown coefficient layout {layout!r} (expected 'pixel' or 'planar')")


def fit_shared_into(pinv_dev, I, coef, *, k, layout="pixel", kernel="auto", nontemporal=False, flags=0):
    """Launch ``rti_fit_shared`` on preallocated tensors (no allocation, graph-capturable).

    pinv_dev: CUDA fp32 [k, N]; I: CUDA [C, N, P] or [N, P] (contiguous
    light-major, fp32/u8/int32); coef: CUDA fp32 [C, P, k] / [C, k, P]."""
    if I.dim() == 2:
        C, (N, P) = 1, I.shape
    else:
        C, N, P = I.shape
    kern = _KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    if nontemporal:
        kern |= L.RTI_KERNEL_NONTEMPORAL
    kern |= int(flags)
    st = L.lib().rti_fit_shared(_vp(pinv_dev), k, N, _vp(I), _IN_DTYPES[I.dtype], P, C, P, N * P, _vp(coef),
                                _layout_id(layout), P * k, kern, _stream_of(I))
    L.check(st, "rti_fit_shared")
    return coef


def fit_shared_pm_into(pinv_dev, I, coef, *, k, layout="pixel", kernel="auto", flags=0):
    """Launch ``rti_fit_shared_pm`` (pixel-major stacks, the reference's (R, R, N) layout,
    analysis.py:217-219) on preallocated tensors: pinv_dev CUDA fp32 [k, N]; I CUDA [P, N] or [C, P, N]
    with unit light stride (any pixel / channel stride, e.g. a view of [H, W, N]); coef as
    fit_shared_into.  A broadcast (stride-0) pixel or channel dimension is materialised first: the C ABI
    reads a zero stride as "dense"."""
    I3 = I if I.dim() == 3 else I.unsqueeze(0)
    C, P, N = I3.shape
    if I3.stride(2) != 1 and N > 1:
        raise ValueError("pixel-major stack needs unit light stride (I[..., p, n] with n contiguous)")
    if (P > 1 and I3.stride(1) == 0) or (C > 1 and I3.stride(0) == 0):
        I3 = I3.contiguous()
    ps = I3.stride(1) if P > 1 else N
    cs = I3.stride(0) if C > 1 else P * ps
    kern = (_KERNELS[kernel] if isinstance(kernel, str) else int(kernel)) | int(flags)
    st = L.lib().rti_fit_shared_pm(_vp(pinv_dev), k, N, _vp(I3), _IN_DTYPES[I.dtype], P, C, ps, cs, _vp(coef),
                                   _layout_id(layout), P * k, kern, _stream_of(I))
    L.check(st, "rti_fit_shared_pm")
    return coef


def _pixel_major_of(I):
    """A light-major-shaped stack ([N, P], [N, H, W], [C, N, H, W]) that is a view of a pixel-major one
    (I.permute of the reference's [H, W, N]) -> the same data as [C, P, N] with unit light stride, else None."""
    if I.dim() < 2 or I.dim() > 4 or I.stride(1 if I.dim() == 4 else 0) != 1:
        return None  # the light dimension must be the unit-stride one
    if any(st == 0 and n > 1 for st, n in zip(I.stride(), I.shape)):
        return None  # a broadcast (expanded) dimension: not a pixel-major stack in memory
    if I.dim() == 2:
        v = I.t().unsqueeze(0)
    elif I.dim() == 3:
        N, H, W = I.shape
        if I.stride(1) != W * I.stride(2):
            return None
        v = I.permute(1, 2, 0).reshape(1, H * W, N) if H * W > 0 else None
    else:
        C, N, H, W = I.shape
        if I.stride(2) != W * I.stride(3):
            return None
        v = I.permute(0, 2, 3, 1).reshape(C, H * W, N)
    if v is None or v.data_ptr() != I.data_ptr() or v.stride(2) != 1 or v.shape[2] < 2:
        return None  # reshape copied: not a view
    return v


def fit(I, lu=None, lv=None, basis="ptm", mode="shared", rcond=None, *, cams=None, origin=(0.0, 0.0),
        layout="pixel", kernel="auto", coef_dtype=torch.float32, nontemporal=False, stack="auto"):
    """Fit per-pixel reflectance coefficients on the GPU.

    mode="shared" (the north_star path; directional lights, one (lu, lv) per light):
        I: CUDA tensor [N, H, W], [N, P] or [C, N, H, W] (light-major), fp32/u8/int32;
        with stack="pixel" the reference's own pixel-major layout instead, [H, W, N], [P, N] or
        [C, H, W, N] (analysis.py:217-219), fitted in place by ``rti_fit_shared_pm`` (no transpose).
        stack="auto" also routes a light-major-shaped VIEW of an fp32 / int32 pixel-major stack
        (``Ipm.permute(2, 0, 1)``) to that kernel instead of copying it, when kernel is one it takes
        ("auto", "valu", "mfma", "tile") and nontemporal is off; 8-bit views keep the copy + h16 path.
        lu, lv: N light directions (host or device).  Returns fp32 coefficients
        [.., H, W, k] (layout="pixel") or [.., k, H, W] (layout="planar").
        uint8 light-major stacks run the split-fp16 MFMA kernel under kernel="auto" (``rti_fit_shared_h16``:
        the operator carried to 22 significant bits, fp32 sums; within ≈1e-6 of max|c| of the fp32 stream
        that ``fit_shared_into`` / ``torch.ops.rti.fit_shared`` run on the same stack).
    mode="perpixel" (the reference's geometry, PTM only):
        either cams=[N, 3] camera positions with I light-major [N, H, W]
        (directions generated in-kernel, pixel (x, y) at origin + (x, y, 0)),
        or lu, lv, I pixel-major [H, W, N] exactly as compute_intensities returns
        them (analysis.py:217-219).  Coefficients in coef_dtype (fp32 or fp64).
    """
    _require_cuda(I, "I")
    cl = _layout_id(layout)
    if mode == "shared":
        if lu is None or lv is None:
            raise ValueError("shared mode needs lu and lv (one direction per light)")
        b = basis_id(basis)
        k = basis_terms(b)
        if stack not in ("auto", "light", "pixel"):
            raise ValueError(f"unknown stack layout {stack!r} (expected 'auto', 'light' or 'pixel')")
        if stack == "pixel":
            if nontemporal:
                raise NotImplementedError("nontemporal loads apply to light-major stacks (rti_fit_shared)")
            return _fit_shared_pixel_major(I, lu, lv, b, k, rcond, cl, kernel, True)
        # AUTO routes a pixel-major VIEW to rti_fit_shared_pm only where that kernel honours the request: fp32 /
        # int32 stacks (8-bit stacks keep the transposing copy and the h16 matrix-core fit) and the selectors and
        # options rti_fit_shared_pm takes; everything else keeps the light-major path below
        if (stack == "auto" and not I.is_contiguous() and I.dtype in (torch.float32, torch.int32)
                and kernel in _PM_KERNELS and not nontemporal and _pixel_major_of(I) is not None):
            return _fit_shared_pixel_major(I, lu, lv, b, k, rcond, cl, kernel, False)
        lead = I.shape[:-2] if I.dim() >= 3 else I.shape[:-1]
        if I.dim() == 2:
            N, P = I.shape
            C, spatial = 1, (P,)
        elif I.dim() == 3:
            N, H, W = I.shape
            C, P, spatial = 1, H * W, (H, W)
        elif I.dim() == 4:
            C, N, H, W = I.shape
            P, spatial = H * W, (H, W)
        else:
            raise ValueError("I must be [N, P], [N, H, W] or [C, N, H, W]")
        del lead
        if N < k:
            raise ValueError(f"shapes not aligned: {N} lights < {k} basis terms (analysis.py:298)")
        pv = pinv(lu, lv, b, rcond)
        if pv.shape[1] != N:
            raise ValueError(f"{pv.shape[1]} light directions for {N} intensity planes")
        Ic = I.contiguous().reshape(C, N, P)
        shape = (C, P, k) if cl == L.RTI_COEF_PIXEL_MAJOR else (C, k, P)
        coef = torch.empty(shape, dtype=torch.float32, device=I.device)
        # 8-bit stacks (the reference's V channel): AUTO runs the split-fp16 fit on the fp16 matrix cores
        # (kernel="h16"); kernel="q8" the int8 fixed-point form (exact sums); both need a finite
        # operator (a rank-deficient light set without rcond keeps the fp32 path and the reference's NaN)
        mk = "h16" if kernel == "auto" else kernel
        if mk in ("h16", "q8") and q8_supported(Ic, k, N, P, mk) and np.isfinite(pv).all():
            if mk == "h16":
                fit_h16_into(torch.as_tensor(h16_operator(pv), device=I.device), Ic, coef, k=k, layout=cl)
            else:
                fit_q8_into(torch.as_tensor(q8_operator(pv), device=I.device), Ic, coef, k=k, layout=cl)
        elif kernel in ("q8", "h16"):
            fn = L.lib().rti_fit_shared_h16_max_lights if kernel == "h16" else L.lib().rti_fit_shared_q8_max_lights
            raise NotImplementedError(f"kernel={kernel!r} needs a uint8 stack, k in (6, 9, 16), N <= {int(fn())}, "
                                      "16-pixel-aligned planes and a finite pseudo-inverse")
        else:
            pinv_dev = torch.as_tensor(pv.astype(np.float32), device=I.device)
            fit_shared_into(pinv_dev, Ic, coef, k=k, layout=cl, kernel=kernel, nontemporal=nontemporal)
        if cl == L.RTI_COEF_PIXEL_MAJOR:
            out = coef.reshape((C,) + spatial + (k,))
        else:
            out = coef.reshape((C, k) + spatial)
        return out if I.dim() == 4 else out[0]
    if mode != "perpixel":
        raise ValueError(f"unknown mode {mode!r} (expected 'shared' or 'perpixel')")
    if basis_id(basis) != L.RTI_BASIS_PTM6:
        raise NotImplementedError("per-pixel mode is the reference's PTM-6 path")
    cdt = _COEF_DTYPES.get(coef_dtype)
    if cdt is None:
        raise ValueError("coef_dtype must be torch.float32 or torch.float64")
    rc = -1.0 if rcond is None else float(rcond)
    if cams is not None:
        if I.dim() != 3:
            raise ValueError("per-pixel camera mode needs I light-major [N, H, W]")
        N, H, W = I.shape
        cams_d = torch.as_tensor(np.asarray(cams.detach().cpu() if torch.is_tensor(cams) else cams, np.float64),
                                 device=I.device).contiguous()
        if cams_d.shape != (N, 3):
            raise ValueError(f"cams must be [{N}, 3]")
        Ic = I.contiguous()
        shape = (H, W, 6) if cl == L.RTI_COEF_PIXEL_MAJOR else (6, H, W)
        coef = torch.empty(shape, dtype=coef_dtype, device=I.device)
        st = L.lib().rti_fit_perpixel_cam(_vp(cams_d), N, _vp(Ic), _IN_DTYPES[Ic.dtype], H, W, H * W,
                                          float(origin[0]), float(origin[1]), rc, _vp(coef), cdt, cl, _stream_of(I))
        L.check(st, "rti_fit_perpixel_cam")
        return coef
    if lu is None or lv is None:
        raise ValueError("per-pixel mode needs cams=[N,3] or per-pixel lu, lv [H, W, N]")
    lu_d = torch.as_tensor(lu, device=I.device).to(torch.float32).contiguous()
    lv_d = torch.as_tensor(lv, device=I.device).to(torch.float32).contiguous()
    if lu_d.shape != I.shape or lv_d.shape != I.shape:
        raise ValueError("per-pixel lu, lv and I must share the pixel-major shape [.., N]")
    N = I.shape[-1]
    spatial = tuple(I.shape[:-1])
    P = int(np.prod(spatial)) if spatial else 1
    Ic = I.contiguous()
    shape = spatial + (6,) if cl == L.RTI_COEF_PIXEL_MAJOR else (6,) + spatial
    coef = torch.empty(shape, dtype=coef_dtype, device=I.device)
    st = L.lib().rti_fit_perpixel_dirs(_vp(lu_d), _vp(lv_d), _vp(Ic), _IN_DTYPES[Ic.dtype], N, P, rc, _vp(coef), cdt,
                                       cl, _stream_of(I))
    L.check(st, "rti_fit_perpixel_dirs")
    return coef


def fit_residual(I, coef, lu, lv, basis="ptm", *, layout="pixel"):
    """Per-pixel RMS residual of a shared-direction fit (``rti_fit_residual``).

    I: the stack ``fit`` was given ([N, P], [N, H, W] or [C, N, H, W]); coef: its
    fp32 output (same layout).  Returns ``(res, rms)``: res fp32 with I's spatial
    shape (plus the leading C for 4-D stacks) = sqrt(Σ_n (I_n − A_n·coef)² / N), and
    rms fp64 [C] (or a 0-d tensor) = the RMS residual over all pixels of a channel,
    summed from per-workgroup wavefront reductions on the device."""
    _require_cuda(I, "I")
    _require_cuda(coef, "coef")
    cl = _layout_id(layout)
    b = basis_id(basis)
    k = basis_terms(b)
    if I.dim() == 2:
        (N, P), C, spatial = I.shape, 1, (I.shape[1],)
    elif I.dim() == 3:
        N, H, W = I.shape
        C, P, spatial = 1, H * W, (H, W)
    elif I.dim() == 4:
        C, N, H, W = I.shape
        P, spatial = H * W, (H, W)
    else:
        raise ValueError("I must be [N, P], [N, H, W] or [C, N, H, W]")
    if coef.dtype != torch.float32 or coef.numel() != C * P * k:
        raise ValueError(f"coef must be fp32 with {C}x{P}x{k} elements (the output of fit)")
    A = design_matrix(lu, lv, b)
    if A.shape[0] != N:
        raise ValueError(f"{A.shape[0]} light directions for {N} intensity planes")
    A_dev = torch.as_tensor(A.astype(np.float32), device=I.device).contiguous()
    Ic = I.contiguous().reshape(C, N, P)
    cc = coef.contiguous()
    res = torch.empty((C, P), dtype=torch.float32, device=I.device)
    nb = int(L.lib().rti_fit_residual_blocks(P))
    partial = torch.zeros((C, nb), dtype=torch.float64, device=I.device)
    st = L.lib().rti_fit_residual(_vp(A_dev), k, N, _vp(Ic), _IN_DTYPES[Ic.dtype], P, C, P, N * P, _vp(cc), cl,
                                  P * k, _vp(res), _vp(partial), _stream_of(I))
    L.check(st, "rti_fit_residual")
    rms = torch.sqrt(partial.sum(dim=1) / (P * N))
    res = res.reshape((C,) + spatial)
    return (res, rms) if I.dim() == 4 else (res[0], rms[0])


def _stack_shape(I):
    if I.dim() == 2:
        (N, P), C, spatial = I.shape, 1, (I.shape[1],)
    elif I.dim() == 3:
        N, H, W = I.shape
        C, P, spatial = 1, H * W, (H, W)
    elif I.dim() == 4:
        C, N, H, W = I.shape
        P, spatial = H * W, (H, W)
    else:
        raise ValueError("I must be [N, P], [N, H, W] or [C, N, H, W]")
    return C, N, P, spatial


def fit_shared_residual_into(U_dev, W_dev, I3, coef, res, partial, *, k, layout="pixel", chunks=0):
    """Launch ``rti_fit_shared_residual_svd`` on preallocated tensors (no allocation, graph-capturable).

    U_dev fp64 [N, k], W_dev fp64 [k, k] (``lsq_factors``), I3 CUDA [C, N, P] light-major, coef fp32
    [C, P, k] / [C, k, P], res fp32 [C, P] (or None), partial fp64 [C, rti_fit_shared_residual_blocks(P)]
    zeroed (or None)."""
    C, N, P = I3.shape
    cl = _layout_id(layout)
    st = L.lib().rti_fit_shared_residual_svd(_vp(U_dev), _vp(W_dev), k, N, _vp(I3), _IN_DTYPES[I3.dtype], P, C, P,
                                             N * P, _vp(coef), cl, P * k, None if res is None else _vp(res),
                                             None if partial is None else _vp(partial),
                                             int(chunks) << L.RTI_KERNEL_CHUNKS_SHIFT, _stream_of(I3))
    L.check(st, "rti_fit_shared_residual_svd")


def fit_with_residual(I, lu, lv, basis="ptm", rcond=None, *, layout="pixel", chunks=0):
    """Shared-direction fit AND per-pixel residuals in ONE pass over the stack
    (``rti_fit_shared_residual_svd``: the reference's SVD solve, analysis.py:295-298, per pixel —
    y = Uᵀ I and ‖I‖² accumulated in fp64, coefficients = V Σ⁻¹ y, residual energy ‖I‖² − ‖y‖²).

    I: CUDA [N, P], [N, H, W] or [C, N, H, W] (light-major, fp32/u8/int32).  Returns
    ``(coef, res, rms)``: coef fp32 as ``fit`` returns it (layout), res fp32 with I's spatial shape
    (leading C for 4-D stacks) = sqrt(Σ_n (I_n − A_n·coef)² / N) for the least-squares solution, and
    rms fp64 [C] (0-d for 2/3-D stacks) = the RMS residual over all pixels, summed from per-workgroup
    wavefront reductions.  An exactly rank-deficient light set (rcond=None) gives NaN coefficients AND
    NaN residuals, like the reference's division by a zero singular value."""
    _require_cuda(I, "I")
    if I.dtype not in _IN_DTYPES:
        raise ValueError(f"I dtype {I.dtype} unsupported (float32, uint8 or int32)")
    cl = _layout_id(layout)
    b = basis_id(basis)
    k = basis_terms(b)
    C, N, P, spatial = _stack_shape(I)
    if N < k:
        raise ValueError(f"shapes not aligned: {N} lights < {k} basis terms (analysis.py:298)")
    U, W = lsq_factors(lu, lv, b, rcond)
    if U.shape[0] != N:
        raise ValueError(f"{U.shape[0]} light directions for {N} intensity planes")
    dev = I.device
    U_dev = torch.as_tensor(U, device=dev).contiguous()
    W_dev = torch.as_tensor(W, device=dev).contiguous()
    Ic = I.contiguous().reshape(C, N, P)
    coef = torch.empty((C, P, k) if cl == L.RTI_COEF_PIXEL_MAJOR else (C, k, P), dtype=torch.float32, device=dev)
    res = torch.empty((C, P), dtype=torch.float32, device=dev)
    partial = torch.zeros((C, int(L.lib().rti_fit_shared_residual_blocks(P))), dtype=torch.float64, device=dev)
    fit_shared_residual_into(U_dev, W_dev, Ic, coef, res, partial, k=k, layout=cl, chunks=chunks)
    rms = torch.sqrt(partial.sum(dim=1) / (P * N))
    coef = coef.reshape((C,) + spatial + (k,)) if cl == L.RTI_COEF_PIXEL_MAJOR else coef.reshape((C, k) + spatial)
    res = res.reshape((C,) + spatial)
    return (coef, res, rms) if I.dim() == 4 else (coef[0], res[0], rms[0])


def light_dirs(cams, H, W, origin=(0.0, 0.0), device="cuda"):
    """compute_intensities' light vectors on the GPU: (lu, lv) fp32 [H, W, N]."""
    cams_d = torch.as_tensor(np.asarray(cams.detach().cpu() if torch.is_tensor(cams) else cams, np.float64),
                             device=device).contiguous()
    _require_cuda(cams_d, "cams")
    N = cams_d.shape[0]
    lu = torch.empty((H, W, N), dtype=torch.float32, device=cams_d.device)
    lv = torch.empty_like(lu)
    st = L.lib().rti_light_dirs(_vp(cams_d), N, H, W, float(origin[0]), float(origin[1]), _vp(lu), _vp(lv),
                                _stream_of(cams_d))
    L.check(st, "rti_light_dirs")
    return lu, lv


def relight(coef, lu, lv, basis="ptm", *, layout="pixel", out_dtype=torch.float32, out_layout="eval"):
    """Evaluate coefficient maps at light directions on the GPU.

    coef: CUDA fp32/fp64, [H, W, k] / [P, k] (layout="pixel") or [k, H, W] /
    [k, P] (layout="planar").  lu, lv: scalars or E directions.
    Returns [E, H, W] (out_layout="eval") or [H, W, E] (out_layout="pixel"),
    squeezed to [H, W] for a single scalar direction.  out_dtype int32 gives
    the reference's truncated tables, uint8 its clipped display values."""
    _require_cuda(coef, "coef")
    b = basis_id(basis)
    k = basis_terms(b)
    cl = _layout_id(layout)
    cdt = _COEF_DTYPES.get(coef.dtype)
    if cdt is None:
        raise ValueError("coef must be float32 or float64")
    odt = _OUT_DTYPES.get(out_dtype)
    if odt is None:
        raise ValueError("out_dtype must be float32, float64, int32 or uint8")
    if cl == L.RTI_COEF_PIXEL_MAJOR:
        if coef.shape[-1] != k:
            raise ValueError(f"coef last dim {coef.shape[-1]} != {k} terms")
        spatial = tuple(coef.shape[:-1])
    else:
        if coef.shape[0] != k:
            raise ValueError(f"coef first dim {coef.shape[0]} != {k} terms")
        spatial = tuple(coef.shape[1:])
    P = int(np.prod(spatial))
    scalar = np.ndim(lu) == 0 and np.ndim(lv) == 0
    luv = np.stack([np.asarray(lu, np.float64).ravel(), np.asarray(lv, np.float64).ravel()], -1)
    E = luv.shape[0]
    luv_d = torch.as_tensor(np.ascontiguousarray(luv), device=coef.device)
    ol = L.RTI_OUT_EVAL_MAJOR if out_layout == "eval" else L.RTI_OUT_PIXEL_MAJOR
    shape = (E,) + spatial if ol == L.RTI_OUT_EVAL_MAJOR else spatial + (E,)
    out = torch.empty(shape, dtype=out_dtype, device=coef.device)
    c = coef.contiguous()
    st = L.lib().rti_relight(_vp(c), cdt, b, P, cl, _vp(luv_d), E, _vp(out), odt, ol, _stream_of(c))
    L.check(st, "rti_relight")
    if scalar:
        return out[0] if ol == L.RTI_OUT_EVAL_MAJOR else out[..., 0]
    return out


def relight_frame(src, hsv, lu=None, lv=None, basis="ptm", *, layout="pixel", out=None):
    """One relighting_event image on the GPU (interactive_relighting.py:31-38):
    V = clip(value, 0, 255) written into the HSV ROI's V channel, then OpenCV's 8-bit
    HSV -> BGR conversion, in one launch.

    src: CUDA int32 [H, W] table image (the cursor's interpolation_results[ly][lx]), or
    fp32/fp64 coefficient maps ([H, W, k] layout="pixel" / [k, H, W] "planar") evaluated at
    (lu, lv) and truncated to int32 like the reference's tables.
    hsv: CUDA uint8 [H, W, 3].  Returns (or fills ``out``) CUDA uint8 [H, W, 3] BGR."""
    _require_cuda(src, "src")
    _require_cuda(hsv, "hsv")
    if hsv.dtype != torch.uint8 or hsv.shape[-1] != 3:
        raise ValueError("hsv must be uint8 [..., 3]")
    spatial = tuple(hsv.shape[:-1])
    P = int(np.prod(spatial))
    if src.dtype == torch.int32:
        if int(src.numel()) != P:
            raise ValueError(f"table image has {src.numel()} pixels, hsv has {P}")
        sdt, b, cl, u, v = L.RTI_I32, L.RTI_BASIS_PTM6, L.RTI_COEF_PIXEL_MAJOR, 0.0, 0.0
    else:
        sdt = _COEF_DTYPES.get(src.dtype)
        if sdt is None:
            raise ValueError("src must be an int32 table image or float32/float64 coefficients")
        if lu is None or lv is None:
            raise ValueError("coefficient maps need a light direction (lu, lv)")
        b = basis_id(basis)
        k = basis_terms(b)
        cl = _layout_id(layout)
        if int(src.numel()) != P * k:
            raise ValueError(f"coefficients {tuple(src.shape)} do not match {k} terms x {P} pixels")
        u, v = float(lu), float(lv)
    h = hsv.contiguous()
    c = src.contiguous()
    if out is None:
        out = torch.empty(spatial + (3,), dtype=torch.uint8, device=hsv.device)
    elif out.dtype != torch.uint8 or int(out.numel()) != 3 * P or not out.is_contiguous():
        raise ValueError("out must be a contiguous uint8 tensor with 3 bytes per pixel")
    if out.data_ptr() == h.data_ptr():
        raise ValueError("out may not alias hsv")
    st = L.lib().rti_relight_frame(_vp(c), sdt, b, cl, P, u, v, _vp(h), _vp(out), _stream_of(h))
    L.check(st, "rti_relight_frame")
    return out


# ---- light operators (RBF, fused PTM/HSH fit + evaluation) ----------------------------------

def _query(qu, qv):
    qu = np.ascontiguousarray(np.asarray(qu, np.float64).ravel())
    qv = np.ascontiguousarray(np.asarray(qv, np.float64).ravel())
    if qu.size != qv.size or qu.size == 0:
        raise ValueError("query directions: qu and qv must be non-empty and of equal length")
    return qu, qv


def rbf_operator(lu, lv, qu, qv):
    """Host fp64 linear-RBF operator opT[N, E] (SciPy Rbf 'linear', analysis.py:249-260).

    Raises numpy.linalg.LinAlgError for a singular system, as SciPy does."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    qu, qv = _query(qu, qv)
    out = np.empty((lu.size, qu.size), np.float64)
    L.check(L.lib().rti_rbf_operator(_fptr(lu), _fptr(lv), lu.size, _dptr(qu), _dptr(qv), qu.size, _dptr(out)),
            "rti_rbf_operator")
    return out


def basis_operator(lu, lv, qu, qv, basis="ptm", rcond=None):
    """Host fp64 operator opT[N, E] = (B(q) · pinv)ᵀ: fit and evaluation fused (analysis.py:293-315)."""
    lu, lv = _f32_host(lu, "lu"), _f32_host(lv, "lv")
    if lu.size != lv.size:
        raise ValueError("lu and lv differ in length")
    qu, qv = _query(qu, qv)
    out = np.empty((lu.size, qu.size), np.float64)
    rc = -1.0 if rcond is None else float(rcond)
    L.check(L.lib().rti_basis_operator(basis_id(basis), _fptr(lu), _fptr(lv), lu.size, _dptr(qu), _dptr(qv),
                                       qu.size, rc, _dptr(out)), "rti_basis_operator")
    return out


def split_operator_f16(opT, device):
    """Host split of an fp64 operator opT[N, E] for rti_apply_operator_f16: fp16 halves
    hi, lo [E, Kp] on ``device`` (M·s = hi + lo, Kp = N rounded up to 16) and 1/s."""
    op = np.ascontiguousarray(opT.detach().cpu().numpy() if torch.is_tensor(opT) else opT, np.float64)
    if op.ndim != 2:
        raise ValueError("operator must be [N, E]")
    N, E = op.shape
    Kp = max(16, (N + 15) // 16 * 16)
    hi = np.empty((E, Kp), np.uint16)
    lo = np.empty((E, Kp), np.uint16)
    inv = ctypes.c_float()
    L.check(L.lib().rti_operator_split_f16(_dptr(op), N, E, E, Kp, hi.ctypes.data_as(ctypes.c_void_p),
                                           lo.ctypes.data_as(ctypes.c_void_p), ctypes.byref(inv)),
            "rti_operator_split_f16")
    return (torch.from_numpy(hi).to(device), torch.from_numpy(lo).to(device), Kp, float(inv.value))


def apply_operator(opT, I, out_dtype=torch.float32, precision="auto"):
    """out[.., E, H, W] = Σ_n opT[n, e] · I[.., n, H, W] on the GPU (MFMA).

    opT: [N, E] operator (host array or tensor).  I: CUDA [N, H, W], [N, P] or
    [C, N, H, W], fp32/u8/int32, light-major.
    precision: "split16" (AUTO for N <= 256) = the fp64 operator split into two fp16
    halves on v_mfma_f32_32x32x16_f16 (22-bit operator, fp32 accumulation);
    "fp32" = the operator rounded to fp32 on v_mfma_f32_16x16x4_f32."""
    _require_cuda(I, "I")
    odt = _OUT_DTYPES.get(out_dtype)
    if odt is None:
        raise ValueError("out_dtype must be float32, float64, int32 or uint8")
    if precision not in ("auto", "split16", "fp32"):
        raise ValueError("precision must be 'auto', 'split16' or 'fp32'")
    N, E = tuple(opT.shape)
    if I.dim() == 2:
        C, spatial = 1, (I.shape[1],)
    elif I.dim() == 3:
        C, spatial = 1, tuple(I.shape[1:])
    elif I.dim() == 4:
        C, spatial = I.shape[0], tuple(I.shape[2:])
    else:
        raise ValueError("I must be [N, P], [N, H, W] or [C, N, H, W]")
    n_img = I.shape[-3] if I.dim() >= 3 else I.shape[0]
    if n_img != N:
        raise ValueError(f"operator has {N} lights, I has {n_img}")
    P = int(np.prod(spatial))
    Ic = I.contiguous()
    out = torch.empty((C, E) + spatial, dtype=out_dtype, device=I.device)
    if precision == "split16" or (precision == "auto" and N <= 256):
        hi, lo, Kp, inv = split_operator_f16(opT, I.device)
        st = L.lib().rti_apply_operator_f16(_vp(hi), _vp(lo), Kp, inv, E, N, _vp(Ic), _IN_DTYPES[Ic.dtype], P, C, P,
                                            N * P, _vp(out), odt, P, E * P, _stream_of(I))
        L.check(st, "rti_apply_operator_f16")
    else:
        op = torch.as_tensor(opT, device=I.device).to(torch.float32).contiguous()
        st = L.lib().rti_apply_operator(_vp(op), E, N, E, _vp(Ic), _IN_DTYPES[Ic.dtype], P, C, P, N * P, _vp(out),
                                        odt, P, E * P, _stream_of(I))
        L.check(st, "rti_apply_operator")
    return out if I.dim() == 4 else out[0]


def interpolate_rbf(I, lu, lv, qu, qv, out_dtype=torch.float32):
    """Linear-RBF interpolation of every pixel at (qu, qv) for a SHARED light set -> [.., E, H, W]."""
    return apply_operator(rbf_operator(lu, lv, qu, qv), I, out_dtype=out_dtype)


def interpolate_rbf_perpixel(I, lu, lv, qu, qv, out_dtype=torch.float64, out_layout="pixel", stats=None):
    """Per-pixel linear RBF (the reference's default with per-pixel light lists) on the GPU.

    I, lu, lv: pixel-major [.., N] (compute_intensities' layout), on any device.
    Returns [.., E] (out_layout="pixel") or [E, ..] ("eval").  Raises
    numpy.linalg.LinAlgError if any pixel's system is singular, as SciPy does.
    stats: a dict receives "fallback_px", the pixels (81 <= N <= 256) re-solved by the fp64 fallback."""
    _require_cuda(I, "I")
    dev = I.device
    odt = _OUT_DTYPES.get(out_dtype)
    if odt is None:
        raise ValueError("out_dtype must be float32, float64, int32 or uint8")
    lu_d = torch.as_tensor(lu, device=dev).to(torch.float32).contiguous()
    lv_d = torch.as_tensor(lv, device=dev).to(torch.float32).contiguous()
    if lu_d.shape != I.shape or lv_d.shape != I.shape:
        raise ValueError("per-pixel lu, lv and I must share the pixel-major shape [.., N]")
    N = I.shape[-1]
    spatial = tuple(I.shape[:-1])
    P = int(np.prod(spatial)) if spatial else 1
    qu, qv = _query(qu, qv)
    luv = torch.as_tensor(np.ascontiguousarray(np.stack([qu, qv], -1)), device=dev)
    E = qu.size
    ol = L.RTI_OUT_PIXEL_MAJOR if out_layout == "pixel" else L.RTI_OUT_EVAL_MAJOR
    out = torch.empty(spatial + (E,) if ol == L.RTI_OUT_PIXEL_MAJOR else (E,) + spatial, dtype=out_dtype, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    Ic = I.contiguous()
    fb = torch.zeros(1, dtype=torch.int32, device=dev)
    st = L.lib().rti_rbf_perpixel_ex(_vp(lu_d), _vp(lv_d), _vp(Ic), _IN_DTYPES[Ic.dtype], N, P, _vp(luv), E,
                                     _vp(out), odt, ol, _vp(status), _vp(fb), _stream_of(I))
    L.check(st, "rti_rbf_perpixel")
    if stats is not None:
        stats["fallback_px"] = int(fb.item())
    if int(status.item()) == L.RTI_ERR_SINGULAR:
        raise np.linalg.LinAlgError("Matrix is singular.")
    return out
