"""Pin the CPU oracle against golden vectors produced by the reference itself.

tests/golden/make_goldens.py ran the reference's own analysis.py functions
(bara96/Smartphone-based-RTI @ v0) on seeded inputs; these tests require the
oracle's restatement to reproduce them.  No GPU needed.
"""
import numpy as np
import pytest

import rti_oracle as o
from conftest import coef_close, golden


def test_shared_coefficients_match_reference():
    d = golden("ptm_shared_256x256_N20.npz")
    lu, lv, I, ref = d["lu"], d["lv"], d["I"], d["coef"]
    coef = o.fit_shared(I.astype(np.float64), o.pinv_shared("ptm", lu, lv)).reshape(ref.shape)
    err, ok = coef_close(coef, ref, rtol=1e-12)
    assert ok, err


def test_single_pixel_svd_restatement_is_reference_exact():
    d = golden("ptm_shared_256x256_N20.npz")
    lu, lv, I, ref = d["lu"], d["lv"], d["I"], d["coef"]
    for y, x in [(0, 0), (31, 200), (255, 255)]:
        a = o.ptm_fit_pixel(lu, lv, I[:, y, x].astype(np.int32))
        assert np.allclose(a, ref[y, x], rtol=0, atol=1e-10)


def test_grid_evaluation_bit_exact():
    d = golden("ptm_shared_256x256_N20.npz")
    lu, lv, I = d["lu"], d["lv"], d["I"]
    xf = o.grid_axis()
    assert xf.shape == (100,) and xf[0] == -1.0 and xf[-1] == 0.98
    for (y, x), g in zip(d["grid_px"], d["grid"]):
        assert np.array_equal(o.interpolate_ptm(lu, lv, xf, I[:, y, x].astype(np.int32)), g)


def test_compute_intensities_bit_exact():
    d = golden("ptm_perpixel_32x32_N50.npz")
    data = [(d["frames"][i], d["cams"][i]) for i in range(len(d["cams"]))]
    lx, ly, inten = o.compute_intensities(data, roi=32)
    assert lx.dtype == np.float32 and inten.dtype == np.int32
    assert np.array_equal(lx, d["lx"]) and np.array_equal(ly, d["ly"]) and np.array_equal(inten, d["I"])


def test_perpixel_fit_interpolate_prepare_match_reference():
    d = golden("ptm_perpixel_32x32_N50.npz")
    lx, ly, inten, ref = d["lx"], d["ly"], d["I"], d["coef"]
    coef = o.fit_perpixel(lx.reshape(-1, 50), ly.reshape(-1, 50), inten.reshape(-1, 50)).reshape(ref.shape)
    err, ok = coef_close(coef, ref, rtol=1e-12)
    assert ok, err
    r = int(d["roi_grid"])
    grid = o.interpolate_intensities_ptm((lx[:r, :r], ly[:r, :r], inten[:r, :r]))
    assert np.array_equal(grid, d["grid"])
    assert np.array_equal(o.prepare_images_data(grid), d["tables"])


def test_edge_cases_match_reference():
    e = golden("ptm_edge.npz")
    for name in ("exact6", "n200"):
        a = o.ptm_fit_pixel(e[f"{name}_lu"], e[f"{name}_lv"], e[f"{name}_I"])
        err, ok = coef_close(a[None], e[f"{name}_coef"][None], rtol=1e-9)
        assert ok, (name, err)
    # exactly rank deficient: the reference divides by a zero singular value -> NaN
    with np.errstate(all="ignore"):
        a = o.ptm_fit_pixel(e["singular_lu"], e["singular_lv"], e["singular_I"])
    assert np.isnan(e["singular_coef"]).all() and not np.isfinite(a).all()
    # near-collinear: finite, huge garbage on both sides
    a = o.ptm_fit_pixel(e["nearcollinear_lu"], e["nearcollinear_lv"], e["nearcollinear_I"])
    assert np.isfinite(a).all() and np.abs(e["nearcollinear_coef"]).max() > 1e6
    # N < 6 raises ValueError in the reference
    assert str(e["n5_raises"]) == "ValueError"
    with pytest.raises(ValueError):
        o.ptm_fit_pixel(e["exact6_lu"][:5], e["exact6_lv"][:5], e["exact6_I"][:5])


def test_error_messages_match_reference():
    e = golden("ptm_edge.npz")
    with pytest.raises(Exception) as ex:
        o.compute_intensities([])
    assert str(ex.value) == str(e["msg_compute_intensities"])
    with pytest.raises(Exception) as ex:
        o.interpolate_intensities_ptm((1, 2))
    assert str(ex.value) == str(e["msg_interpolate_intensities"])
    with pytest.raises(Exception) as ex:
        o.prepare_images_data([])
    assert str(ex.value) == str(e["msg_prepare_images_data"])


def test_relight_lookup_mapping_matches_reference():
    rows = golden("relight_lookup.npz")["rows"]
    for x, y, h, w, lx, ly, ix, iy in rows:
        got = o.draw_light_roi_position(int(x), int(y), (int(h), int(w)), to_light_vector=True)
        assert got == (lx, ly)
        assert o.table_index(got[0]) == ix and o.table_index(got[1]) == iy


def test_hsh_basis_is_orthonormal_on_hemisphere():
    # Build-defined HSH (no reference counterpart): check ∫_Ω H_i H_j dω = δ_ij.
    n_t, n_p = 400, 800
    th = (np.arange(n_t) + 0.5) / n_t * (np.pi / 2)
    ph = (np.arange(n_p) + 0.5) / n_p * 2 * np.pi
    T, Ph = np.meshgrid(th, ph, indexing="ij")
    lu, lv = np.sin(T) * np.cos(Ph), np.sin(T) * np.sin(Ph)
    B = o.hsh_basis(lu.ravel(), lv.ravel())
    w = (np.sin(T) * (np.pi / 2 / n_t) * (2 * np.pi / n_p)).ravel()
    G = (B * w[:, None]).T @ B
    assert np.allclose(G, np.eye(16), atol=2e-3)


def test_rbf_restatement_matches_scipy_goldens():
    d = golden("rbf_shared_4px_N20.npz")
    yi, xi = np.mgrid[-1:1:0.02, -1:1:0.02]
    xi, yi = np.around(xi, 2), np.around(yi, 2)
    for p in range(4):
        g = o.rbf_linear(d["lu"], d["lv"], d["I"][p], xi, yi)
        assert np.abs(g - d["grid"][p]).max() < 1e-9
    op = o.rbf_operator(d["lu"], d["lv"], xi.ravel(), yi.ravel())
    assert np.abs((op.T @ d["I"].T.astype(np.float64)).T.reshape(-1, 100, 100) - d["grid"]).max() < 1e-9


def test_rbf_perpixel_default_path_matches_reference():
    d = golden("rbf_perpixel_4x4_N50.npz")
    grid = o.interpolate_intensities_rbf((d["lx"], d["ly"], d["I"]))
    assert np.abs(grid - d["grid"]).max() < 1e-8
    t = o.prepare_images_data(grid)
    near = np.abs(d["grid"] - np.round(d["grid"])) < 1e-6
    assert not ((t != d["tables"]) & ~np.transpose(near, (2, 3, 0, 1))).any()
    assert str(d["singular_raises"]) == "LinAlgError"
    with pytest.raises(np.linalg.LinAlgError):
        o.rbf_linear(d["singular_lx"][0, 0], d["singular_ly"][0, 0], d["I"][0, 0], [0.0], [0.0])


def test_hsv2bgr_known_answers():
    """OpenCV's documented 8-bit HSV (hue range 180) primaries and greys (cvtColor COLOR_HSV2BGR)."""
    hsv = np.array([[0, 255, 255], [60, 255, 255], [120, 255, 255], [30, 255, 255], [90, 255, 255],
                    [150, 255, 255], [0, 0, 128], [77, 0, 200], [0, 0, 0], [0, 255, 0]], np.uint8)
    bgr = np.array([[0, 0, 255], [0, 255, 0], [255, 0, 0], [0, 255, 255], [255, 255, 0],
                    [255, 0, 255], [128, 128, 128], [200, 200, 200], [0, 0, 0], [0, 0, 0]], np.uint8)
    assert np.array_equal(o.hsv2bgr_u8(hsv), bgr)
    # V substitution + clip as relighting_event does (interactive_relighting.py:33-38)
    img = o.relighting_event_image(np.array([[300, -4]], np.int32), np.array([[[0, 0, 9], [0, 0, 9]]], np.uint8))
    assert np.array_equal(img, np.array([[[255] * 3, [0] * 3]], np.uint8))


def test_fit_residual_oracle_identity():
    """The residual restatement against the normal-equation identity
    ‖I − A c‖² = ‖I‖² − cᵀAᵀI (exact for the least-squares c), in fp64 on the golden stack."""
    d = golden("ptm_shared_256x256_N20.npz")
    I = np.asarray(d["I"], np.float64).reshape(d["I"].shape[0], -1)
    A = o.design("ptm", d["lu"], d["lv"])
    coef = o.fit_shared(I, o.pinv_shared("ptm", d["lu"], d["lv"]))
    res, ss = o.fit_residual(I, A, coef)
    ident = (I * I).sum(0) - np.einsum("pk,nk,np->p", coef, A, I)
    np.testing.assert_allclose(res * res * I.shape[0], ident, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ss, ident.sum(), rtol=1e-9)
    # the reference's golden coefficients explain the stack equally well
    res_g, _ = o.fit_residual(I, A, np.asarray(d["coef"]).reshape(-1, 6))
    np.testing.assert_allclose(res_g, res, rtol=1e-6, atol=1e-9)
