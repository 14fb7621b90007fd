"""The reference's own edge light sets through EVERY HIP solver.

tests/golden/ptm_edge.npz holds what analysis.py:_interpolate_PTM (SVD without rcond, :293-298)
returned for: an exact N = 6 fit, N = 200 lights, near-collinear lights (lv ≈ lu/2, cond(A) = 1.1e8:
the reference returns finite coefficients of order 3e8), and exactly rank-deficient lights (all
lv = 0: NaN).  Each solver is held to the reference's coefficients per pixel
(|Δ| <= tol · max_k |c_ref,k|) and reports its error:

* shared fp32 fit (rti_fit_shared: host fp64 Jacobi pinv, fp32 stream)         tol 1e-4 (the fp32 bar)
* one-pass fit + residual, SVD form (rti_fit_shared_residual_svd, fit_with_residual) tol 1e-6
* one-pass fit + residual, Gram form (rti_fit_shared_residual, (AᵀA)⁺ Aᵀ I)      tol 1e-4 (cond² loss)
* per-pixel, explicit light vectors (rti_fit_perpixel_dirs) fp64 and fp32 out     tol 1e-6
* per-pixel, light vectors from camera positions (rti_fit_perpixel_cam)            tol 1e-6

The per-pixel kernels solve the normal equations by Cholesky and send the pixels whose pivots show an
ill-conditioned A to a Givens-QR refine pass: the near-collinear case takes that path (the normal
equations alone are 6.5e-3 off there)."""
import ctypes

import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden
from rti import _lib as L

pytestmark = pytest.mark.gpu

CASES = ["exact6", "nearcollinear", "n200"]
P = 1031  # ragged: a partial last workgroup / wave / 4-pixel lane


def edge(case):
    e = golden("ptm_edge.npz")
    return e[f"{case}_lu"], e[f"{case}_lv"], e[f"{case}_I"], e[f"{case}_coef"]


def report(name, case, err):
    print(f"{name}[{case}]: max |Δ| / max|c_ref| = {err:.3g}")


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8])
def test_shared_fp32_fit(cuda, case, in_dtype):
    lu, lv, I, ref = edge(case)
    Id = torch.as_tensor(np.tile(I.astype(np.float32)[:, None], (1, P)), device=cuda).to(in_dtype)
    coef = rti.fit(Id, lu, lv).cpu().numpy()
    assert np.isfinite(coef).all()
    err, ok = coef_close(coef, np.broadcast_to(ref, coef.shape), rtol=1e-4)
    report("shared fp32", case, err)
    assert ok, err


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_fit_with_residual_svd_form(cuda, case, layout):
    lu, lv, I, ref = edge(case)
    Inp = np.tile(I.astype(np.float64)[:, None], (1, P))
    coef, res, rms = rti.fit_with_residual(torch.as_tensor(Inp, dtype=torch.float32, device=cuda), lu, lv,
                                           layout=layout)
    c = coef.cpu().numpy()
    c = c.T if layout == "planar" else c
    err, ok = coef_close(c, np.broadcast_to(ref, c.shape), rtol=1e-6)
    report("fit_with_residual (SVD form)", case, err)
    assert ok, err
    A = o.ptm_design(lu, lv)
    ref_r, _ = o.fit_residual(Inp[:, :1], A, ref[None, :])  # the reference's coefficients' own residual
    got = res.cpu().numpy()
    assert np.isfinite(got).all()
    assert np.abs(got - ref_r[0]).max() <= 1e-4 + 1e-6 * ref_r[0], (got.max(), ref_r[0])
    assert abs(float(rms) - ref_r[0]) <= 1e-4 + 1e-6 * ref_r[0]


@pytest.mark.parametrize("case", CASES)
def test_fit_with_residual_gram_form(cuda, case):
    """The Gram form (coefficients = (AᵀA)⁺ AᵀI) squares cond(A); kept as an ABI entry and reported."""
    lu, lv, I, ref = edge(case)
    N = I.size
    Id = torch.as_tensor(np.tile(I.astype(np.float32)[:, None], (1, P)), device=cuda)
    A64 = torch.as_tensor(rti.design_matrix(lu, lv), device=cuda).contiguous()
    G = torch.as_tensor(rti.gram_inverse(lu, lv), device=cuda).contiguous()
    coef = torch.empty((P, 6), device=cuda)
    res = torch.empty(P, device=cuda)
    s = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = L.lib().rti_fit_shared_residual(vp(A64), vp(G), 6, N, vp(Id), L.RTI_F32, P, 1, P, N * P, vp(coef),
                                         L.RTI_COEF_PIXEL_MAJOR, P * 6, vp(res), None, 0, s)
    L.check(st, "rti_fit_shared_residual")
    c = coef.cpu().numpy()
    err, ok = coef_close(c, np.broadcast_to(ref, c.shape), rtol=1e-4)
    report("fit_shared_residual (Gram form)", case, err)
    assert ok, err


def pixel_major(case, reps):
    lu, lv, I, ref = edge(case)
    t = lambda a, dt: np.ascontiguousarray(np.tile(a.astype(dt)[None, :], (reps, 1)))  # noqa: E731
    return t(lu, np.float32), t(lv, np.float32), t(I, np.int32), ref


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cdt", [torch.float64, torch.float32])
@pytest.mark.parametrize("in_dtype", [torch.int32, torch.float32])
def test_perpixel_dirs(cuda, case, cdt, in_dtype):
    """interpolate_intensities' exact input (pixel-major lx, ly, I; analysis.py:341-363)."""
    lu, lv, I, ref = pixel_major(case, P)
    dev = lambda a, dt=None: torch.as_tensor(a, device=cuda) if dt is None else torch.as_tensor(a, device=cuda).to(dt)  # noqa: E731,E501
    coef = rti.fit(dev(I, in_dtype), dev(lu), dev(lv), mode="perpixel", coef_dtype=cdt).cpu().numpy()
    err, ok = coef_close(coef, np.broadcast_to(ref, coef.shape), rtol=1e-6)
    report(f"perpixel dirs {cdt}", case, err)
    assert ok, err


def cams_for(lu, lv, px, py, dist):
    """Camera positions that put light n at direction ≈ (lu_n, lv_n) from pixel (px, py) (analysis.py:228)."""
    lu = lu.astype(np.float64)
    lv = lv.astype(np.float64)
    lw = np.sqrt(np.maximum(1.0 - lu * lu - lv * lv, 0.0))
    return np.stack([px + dist * lu, py + dist * lv, dist * lw], -1)


def design_xx(lu, lv):
    """The PTM rows the kernels form: fp32 x*x monomials (the reference's powf differs by an ulp on ≈1
    in 1200 inputs, which cond(A) = 1e8 would amplify)."""
    lu = np.asarray(lu, np.float32)
    lv = np.asarray(lv, np.float32)
    return np.stack([(lu * lu), (lv * lv), (lu * lv), lu, lv, np.ones_like(lu)], -1).astype(np.float64)


@pytest.mark.parametrize("case", CASES)
def test_perpixel_cam(cuda, case):
    """Light vectors generated in-kernel from camera positions (compute_intensities fused into the fit):
    pixel (2, 1) of a 5 × 7 ROI sees the case's light set, the others nearby ones; every pixel is held to
    the fp64 SVD of its own design (the oracle's light vectors, bit-exact with rti_light_dirs)."""
    lu0, lv0, I, ref = edge(case)
    H, W = 5, 7
    cams = cams_for(lu0, lv0, 2.0, 1.0, 40.0)
    N = cams.shape[0]
    rng = np.random.default_rng(7)
    Ist = (I[:, None, None] + rng.integers(-3, 4, size=(N, H, W))).astype(np.float32)
    coef = rti.fit(torch.as_tensor(Ist, device=cuda), mode="perpixel", cams=cams,
                   coef_dtype=torch.float64).cpu().numpy()
    ys, xs = np.mgrid[0:H, 0:W]
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    glu, glv = rti.light_dirs(cams, H, W, device=cuda)
    assert np.array_equal(glu.cpu().numpy().reshape(-1, N), lu) and np.array_equal(glv.cpu().numpy().reshape(-1, N), lv)
    refs = np.stack([o.svd_solve(design_xx(lu[p], lv[p]), Ist.reshape(N, -1)[:, p].astype(np.float64))
                     for p in range(H * W)])
    err, ok = coef_close(coef.reshape(-1, 6), refs, rtol=1e-6)
    report("perpixel cam", case, err)
    assert ok, err
    if case == "nearcollinear":
        c = np.linalg.cond(design_xx(lu[1 * W + 2], lv[1 * W + 2]))
        assert c > 1e6, c  # the case really exercises the ill-conditioned (refine) path


def test_perpixel_singular_and_rcond(cuda):
    e = golden("ptm_edge.npz")
    lu, lv, I = (np.ascontiguousarray(np.tile(e[f"singular_{n}"][None, :], (64, 1))) for n in ("lu", "lv", "I"))
    d = lambda a: torch.as_tensor(a, device=cuda)  # noqa: E731
    coef = rti.fit(d(I), d(lu), d(lv), mode="perpixel", coef_dtype=torch.float64).cpu().numpy()
    assert np.isnan(coef).all()  # the reference's division by a zero singular value
    coef = rti.fit(d(I), d(lu), d(lv), mode="perpixel", rcond=1e-10, coef_dtype=torch.float64).cpu().numpy()
    assert np.isnan(coef).all()  # per-pixel rcond: a pivot below rcond counts as singular (include/rti.h)


def test_fit_with_residual_rank_deficient_nan_reaches_residuals(cuda):
    """No rcond: NaN coefficients AND NaN residuals / RMS (not a clamped 0 that reads as a perfect fit)."""
    e = golden("ptm_edge.npz")
    I = torch.as_tensor(np.tile(e["singular_I"].astype(np.float32)[:, None], (1, 300)), device=cuda)
    coef, res, rms = rti.fit_with_residual(I, e["singular_lu"], e["singular_lv"])
    assert torch.isnan(coef).all() and torch.isnan(res).all() and np.isnan(float(rms))
    coef, res, rms = rti.fit_with_residual(I, e["singular_lu"], e["singular_lv"], rcond=1e-10)
    assert torch.isfinite(coef).all() and torch.isfinite(res).all() and np.isfinite(float(rms))


def test_perpixel_all_pixels_ill_conditioned(cuda):
    """Every pixel through the refine pass (a whole ROI of near-collinear light sets): still the
    reference's coefficients, over many workgroups."""
    lu, lv, I, ref = pixel_major("nearcollinear", 70_001)
    d = lambda a: torch.as_tensor(a, device=cuda)  # noqa: E731
    coef = rti.fit(d(I), d(lu), d(lv), mode="perpixel", coef_dtype=torch.float64).cpu().numpy()
    err, ok = coef_close(coef, np.broadcast_to(ref, coef.shape), rtol=1e-6)
    report("perpixel dirs, all refined", "nearcollinear", err)
    assert ok, err


@pytest.mark.parametrize("var", ["0", "1", "2", "3", "4", "5"])
def test_perpixel_cam_variants(cuda, monkeypatch, var):
    """Every exactness variant of the fused per-pixel fit (RTI_PERPIXEL_VARIANT, rti_perpixel.hip: two or one
    Newton steps with the refine pass, the in-place group fix-up at 6 / 5 / 4 waves per SIMD, and 5 = every
    group fixed up, which drives the subtract-and-replace path on any input) against the fp64 SVD of each
    pixel's own design with the reference's light vectors, on a 48 × 40 ROI plus the near-collinear golden
    pixel (the QR refine)."""
    monkeypatch.setenv("RTI_PERPIXEL_VARIANT", var)
    for case, (H, W) in (("n200", (48, 40)), ("nearcollinear", (5, 7))):
        lu0, lv0, I, _ = edge(case)
        cams = cams_for(lu0, lv0, 2.0, 1.0, 40.0)
        N = cams.shape[0]
        rng = np.random.default_rng(11)
        Ist = (I[:, None, None] + rng.integers(-3, 4, size=(N, H, W))).astype(np.float32)
        coef = rti.fit(torch.as_tensor(Ist, device=cuda), mode="perpixel", cams=cams,
                       coef_dtype=torch.float64).cpu().numpy().reshape(-1, 6)
        ys, xs = np.mgrid[0:H, 0:W]
        px = np.unique(np.r_[np.random.default_rng(3).integers(0, H * W, 64), 0, H * W - 1, 1 * W + 2])
        lu, lv = o.light_dirs_for_pixels(cams, xs.ravel()[px], ys.ravel()[px])
        refs = np.stack([o.svd_solve(design_xx(lu[i], lv[i]), Ist.reshape(N, -1)[:, p].astype(np.float64))
                         for i, p in enumerate(px)])
        err, ok = coef_close(coef[px], refs, rtol=1e-6)
        report(f"perpixel cam variant {var}", case, err)
        assert ok, (case, err)
