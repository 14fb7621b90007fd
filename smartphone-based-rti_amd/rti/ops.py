"""PyTorch custom ops over the C ABI: ``torch.ops.rti.fit_shared`` / ``fit_shared_residual`` /
``fit_residual`` / ``relight``.

They let the fit and relight kernels sit inside torch programs (and
``torch.library`` fake-tensor tracing) while the compute stays in librti's
HIP kernels on the current stream.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import api


def _same_device(**tensors):
    """Every tensor on one device: a pointer from another GPU must not reach a kernel launched
    on this GPU's stream."""
    devs = {name: t.device for name, t in tensors.items()}
    if len(set(devs.values())) > 1:
        raise ValueError("tensors on different devices: " + ", ".join(f"{n}={d}" for n, d in devs.items()))


def _in_dtype(I):
    if I.dtype not in api._IN_DTYPES:
        raise ValueError(f"I dtype {I.dtype} unsupported (float32, uint8 or int32)")


@torch.library.custom_op("rti::fit_shared", mutates_args=())
def fit_shared(pinv: torch.Tensor, I: torch.Tensor, planar: bool = False, kernel: int = 0) -> torch.Tensor:
    """coef = pinv (fp32 [k, N]) applied to I (CUDA [N, P] or [C, N, P]) -> [C?, P, k] or [C?, k, P]."""
    api._require_cuda(I, "I")
    api._require_cuda(pinv, "pinv")
    if pinv.dtype != torch.float32:
        raise ValueError("pinv must be float32")
    _same_device(pinv=pinv, I=I)
    _in_dtype(I)
    k = pinv.shape[0]
    I3 = I.contiguous() if I.dim() == 3 else I.contiguous().unsqueeze(0)
    C, N, P = I3.shape
    if pinv.shape[1] != N:
        raise ValueError(f"pinv is [{k}, {pinv.shape[1]}] but I has {N} lights")
    shape = (C, k, P) if planar else (C, P, k)
    coef = torch.empty(shape, dtype=torch.float32, device=I.device)
    api.fit_shared_into(pinv.contiguous(), I3, coef, k=k, layout="planar" if planar else "pixel", kernel=kernel)
    return coef if I.dim() == 3 else coef[0]


@fit_shared.register_fake
def _(pinv, I, planar=False, kernel=0):
    k = pinv.shape[0]
    P = I.shape[-1]
    shape = (k, P) if planar else (P, k)
    if I.dim() == 3:
        shape = (I.shape[0],) + shape
    return I.new_empty(shape, dtype=torch.float32)


@torch.library.custom_op("rti::fit_shared_residual", mutates_args=())
def fit_shared_residual(U: torch.Tensor, W: torch.Tensor, I: torch.Tensor, planar: bool = False,
                        chunks: int = 0) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """The north_star fit with per-pixel residuals in ONE pass over the stack
    (``rti_fit_shared_residual_svd``; the reference's solve, analysis.py:293-298, as y = Uᵀ I,
    coef = W y with the thin SVD A = U Σ Vᵀ, W = V Σ⁻¹).

    U fp64 [N, k], W fp64 [k, k] (``rti.lsq_factors``), I CUDA [N, P] or [C, N, P] (fp32/u8/int32) ->
    ``(coef, res, partial)``: coef fp32 [C?, P, k] (or [C?, k, P] if planar), res fp32 [C?, P] =
    sqrt(Σ_n (I_n − A_n·coef)² / N), partial fp64 [C?, rti_fit_shared_residual_blocks(P)] = each
    workgroup's residual energy from wavefront reductions (sum / (P·N) = mean squared residual)."""
    api._require_cuda(I, "I")
    api._require_cuda(U, "U")
    api._require_cuda(W, "W")
    if U.dtype != torch.float64 or W.dtype != torch.float64:
        raise ValueError("U and W must be float64 (rti.lsq_factors)")
    _same_device(U=U, W=W, I=I)
    _in_dtype(I)
    I3 = I.contiguous() if I.dim() == 3 else I.contiguous().unsqueeze(0)
    C, N, P = I3.shape
    k = U.shape[1]
    if U.shape[0] != N or W.shape != (k, k):
        raise ValueError(f"U must be [{N}, k] and W [k, k]; got {tuple(U.shape)} and {tuple(W.shape)}")
    if N < k:
        raise ValueError(f"shapes not aligned: {N} lights < {k} basis terms (analysis.py:298)")
    coef = torch.empty((C, k, P) if planar else (C, P, k), dtype=torch.float32, device=I.device)
    res = torch.empty((C, P), dtype=torch.float32, device=I.device)
    partial = torch.zeros((C, int(L.lib().rti_fit_shared_residual_blocks(P))), dtype=torch.float64, device=I.device)
    api.fit_shared_residual_into(U.contiguous(), W.contiguous(), I3, coef, res, partial, k=k,
                                 layout="planar" if planar else "pixel", chunks=chunks)
    if I.dim() == 2:
        return coef[0], res[0], partial[0]
    return coef, res, partial


@fit_shared_residual.register_fake
def _(U, W, I, planar=False, chunks=0):
    k = U.shape[1]
    P = I.shape[-1]
    lead = (I.shape[0],) if I.dim() == 3 else ()
    nb = (P + 255) // 256  # rti_fit_shared_residual_blocks(P): one slot per 256-pixel workgroup span
    return (I.new_empty(lead + ((k, P) if planar else (P, k)), dtype=torch.float32),
            I.new_empty(lead + (P,), dtype=torch.float32),
            I.new_empty(lead + (nb,), dtype=torch.float64))


@torch.library.custom_op("rti::fit_residual", mutates_args=())
def fit_residual(A: torch.Tensor, I: torch.Tensor, coef: torch.Tensor) -> torch.Tensor:
    """Per-pixel RMS residual of coef (fp32 [P, k], fit_shared's pixel-major output) against
    I (CUDA [N, P]) under the fp32 design matrix A [N, k] -> fp32 [P]."""
    api._require_cuda(I, "I")
    api._require_cuda(A, "A")
    api._require_cuda(coef, "coef")
    if A.dtype != torch.float32 or coef.dtype != torch.float32:
        raise ValueError("A and coef must be float32")
    _same_device(A=A, I=I, coef=coef)
    _in_dtype(I)
    if I.dim() != 2:
        raise ValueError("I must be [N, P]")
    N, P = I.shape
    k = A.shape[1]
    if A.shape[0] != N or coef.shape != (P, k):
        raise ValueError(f"A must be [{N}, k] and coef [{P}, k]")
    Ic, Ac, cc = I.contiguous(), A.contiguous(), coef.contiguous()
    res = torch.empty(P, dtype=torch.float32, device=I.device)
    st = L.lib().rti_fit_residual(api._vp(Ac), k, N, api._vp(Ic), api._IN_DTYPES[Ic.dtype], P, 1, P, N * P,
                                  api._vp(cc), L.RTI_COEF_PIXEL_MAJOR, P * k, api._vp(res), None,
                                  api._stream_of(I))
    L.check(st, "rti_fit_residual")
    return res


@fit_residual.register_fake
def _(A, I, coef):
    return I.new_empty((I.shape[-1],), dtype=torch.float32)


@torch.library.custom_op("rti::relight", mutates_args=())
def relight(coef: torch.Tensor, luv: torch.Tensor, basis: int = L.RTI_BASIS_PTM6) -> torch.Tensor:
    """coef CUDA [P, k] (fp32/fp64), luv [E, 2] -> [E, P] in coef's dtype."""
    lu = luv[:, 0].detach().cpu().double().numpy()
    lv = luv[:, 1].detach().cpu().double().numpy()
    return api.relight(coef, lu, lv, basis=basis, out_dtype=coef.dtype)


@relight.register_fake
def _(coef, luv, basis=L.RTI_BASIS_PTM6):
    return coef.new_empty((luv.shape[0], coef.shape[0]))
