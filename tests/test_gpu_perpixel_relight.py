"""GPU parity of the reference-faithful per-pixel path (light vectors, per-pixel
PTM solve), the relight evaluator and the reference-signature adapters,
against the reference's golden vectors and the oracle."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden, relight_close
from rti import compat

pytestmark = pytest.mark.gpu


def test_light_dirs_match_reference(cuda):
    d = golden("ptm_perpixel_32x32_N50.npz")
    lu, lv = rti.light_dirs(d["cams"], 32, 32, device=cuda)
    lu, lv = lu.cpu().numpy(), lv.cpu().numpy()
    # separately rounded fp64 ops (no contraction) rounded to fp32: bit-identical to the reference
    assert np.array_equal(lu, d["lx"]) and np.array_equal(lv, d["ly"])


@pytest.mark.parametrize("coef_dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("in_dtype", [torch.int32, torch.float32, torch.uint8])
def test_perpixel_dirs_match_reference(cuda, coef_dtype, in_dtype):
    d = golden("ptm_perpixel_32x32_N50.npz")
    lx = torch.as_tensor(d["lx"], device=cuda)
    ly = torch.as_tensor(d["ly"], device=cuda)
    I = torch.as_tensor(d["I"]).to(cuda).to(in_dtype)
    coef = rti.fit(I, lx, ly, mode="perpixel", coef_dtype=coef_dtype).cpu().numpy()
    # fp64 path: the reference's design rows use glibc powf for lu**2 (1-ulp off x*x in ~1/1200
    # inputs), which moves its coefficients by up to ~4e-8 relative; fp32 path: the 1e-4 criterion
    err, ok = coef_close(coef, d["coef"], rtol=1e-4 if coef_dtype == torch.float32 else 1e-6)
    assert ok, err


@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_perpixel_cam_matches_reference(cuda, layout):
    d = golden("ptm_perpixel_32x32_N50.npz")
    I = torch.as_tensor(np.ascontiguousarray(d["frames"]), device=cuda)  # [N, H, W] uint8, light-major
    coef = rti.fit(I, cams=d["cams"], mode="perpixel", coef_dtype=torch.float64, layout=layout).cpu().numpy()
    if layout == "planar":
        coef = np.moveaxis(coef, 0, -1)
    err, ok = coef_close(coef, d["coef"], rtol=1e-6)
    assert ok, err


def test_perpixel_cam_origin_offset_vs_oracle(cuda):
    rng = np.random.default_rng(5)
    N, H, W = 40, 24, 40
    cams = np.stack([rng.uniform(-200, 400, N), rng.uniform(-200, 400, N), rng.uniform(150, 400, N)], -1)
    frames = rng.integers(0, 256, (N, H, W)).astype(np.uint8)
    x0, y0 = 13.0, -7.0
    ys, xs = np.mgrid[0:H, 0:W]
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel() + x0, ys.ravel() + y0)
    ref = o.fit_perpixel(lu, lv, frames.reshape(N, -1).T).reshape(H, W, 6)
    coef = rti.fit(torch.as_tensor(frames, device=cuda), cams=cams, origin=(x0, y0), mode="perpixel",
                   coef_dtype=torch.float64).cpu().numpy()
    err, ok = coef_close(coef, ref, rtol=1e-6)
    assert ok, err


def test_perpixel_singular_gives_nan(cuda):
    e = golden("ptm_edge.npz")
    n = len(e["singular_lu"])
    lu = torch.as_tensor(np.tile(e["singular_lu"], (4, 1)), device=cuda)
    lv = torch.as_tensor(np.tile(e["singular_lv"], (4, 1)), device=cuda)
    I = torch.as_tensor(np.tile(e["singular_I"], (4, 1)), device=cuda)
    coef = rti.fit(I, lu, lv, mode="perpixel", coef_dtype=torch.float64).cpu().numpy()
    assert coef.shape == (4, 6) and np.isnan(coef).all()
    assert n >= 6


@pytest.mark.parametrize("basis", ["ptm", "hsh", "hsh9"])
@pytest.mark.parametrize("cdt", [torch.float32, torch.float64])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_relight_vs_oracle(cuda, basis, cdt, layout):
    k = rti.basis_terms(basis)
    rng = np.random.default_rng(1)
    coef = rng.uniform(-50, 50, (37, 29, k))
    coef[..., 0 if basis != "ptm" else 5] += 150
    lu, lv = o.synth_dirs(70, 8, radius=1.0)
    B = rti.basis_eval(lu, lv, basis)
    ref = np.einsum("ek,hwk->ehw", B, coef)
    c = torch.as_tensor(coef if layout == "pixel" else np.moveaxis(coef, -1, 0).copy(), device=cuda, dtype=cdt)
    out = rti.relight(c, lu.astype(np.float64), lv.astype(np.float64), basis=basis, layout=layout,
                      out_dtype=cdt).cpu().numpy()
    err, ok = relight_close(out, ref, rtol=1e-6 if cdt == torch.float32 else 1e-12)
    assert ok, err
    outp = rti.relight(c, lu.astype(np.float64), lv.astype(np.float64), basis=basis, layout=layout,
                       out_dtype=cdt, out_layout="pixel").cpu().numpy()
    assert np.array_equal(np.moveaxis(outp, -1, 0), out)


def test_relight_f64_grid_bit_exact_with_reference(cuda):
    d = golden("ptm_shared_256x256_N20.npz")
    px = d["grid_px"]
    coef = torch.as_tensor(d["coef"][px[:, 0], px[:, 1]], device=cuda)  # reference's coefficients
    xf = o.grid_axis()
    out = rti.relight(coef, np.tile(xf, 100), np.repeat(xf, 100), out_dtype=torch.float64, out_layout="pixel")
    assert np.array_equal(out.cpu().numpy().reshape(-1, 100, 100), o.ptm_eval_grid(d["coef"][px[:, 0], px[:, 1]], xf))
    err, ok = relight_close(out.cpu().numpy().reshape(-1, 100, 100), d["grid"], rtol=1e-12)
    assert ok, err


def test_relight_int_semantics(cuda):
    coef = np.zeros((1, 8, 6))
    coef[0, :, 5] = [-3.7, -0.5, 0.0, 0.99, 254.6, 255.0, 300.2, np.nan]
    c = torch.as_tensor(coef, device=cuda)
    i32 = rti.relight(c, 0.0, 0.0, out_dtype=torch.int32).cpu().numpy()
    assert i32.tolist() == [[-3, 0, 0, 0, 254, 255, 300, np.iinfo(np.int32).min]]
    u8 = rti.relight(c, 0.0, 0.0, out_dtype=torch.uint8).cpu().numpy()
    assert u8.tolist() == [[0, 0, 0, 0, 254, 255, 255, 0]]


# ---- reference-signature adapters -------------------------------------------------------

def test_compat_compute_intensities(cuda):
    d = golden("ptm_perpixel_32x32_N50.npz")
    data = [(d["frames"][i], d["cams"][i]) for i in range(len(d["cams"]))]
    lx, ly, inten = compat.compute_intensities(data)
    assert lx.dtype == np.float32 and inten.dtype == np.int32 and lx.shape == (32, 32, 50)
    assert np.array_equal(lx, d["lx"]) and np.array_equal(ly, d["ly"])
    assert np.array_equal(inten, d["I"])
    with pytest.raises(Exception, match="results are empty"):
        compat.compute_intensities([])


def test_compat_interpolate_and_prepare(cuda):
    d = golden("ptm_perpixel_32x32_N50.npz")
    r = int(d["roi_grid"])
    data = (d["lx"][:r, :r], d["ly"][:r, :r], d["I"][:r, :r])
    grid = compat.interpolate_intensities(data, interpolate_PTM=True)
    assert grid.shape == d["grid"].shape and grid.dtype == np.float64
    err, ok = relight_close(grid, d["grid"], rtol=1e-6)  # coefficients within ~4e-8 (powf ulps)
    assert ok, err
    tables = compat.prepare_images_data(grid)
    ref_t = d["tables"]
    # int32 truncation could only differ where the reference value sits within 1e-4 of an integer
    # (fp64 Cholesky normal equations vs the reference's SVD: coefficients agree to ~4e-8 relative);
    # 33 of this golden's values do, and none flips — held at zero like the cams path
    # (test_compat_compute_end_to_end), the kernels being deterministic.
    diff = tables != ref_t
    near = np.abs(np.transpose(d["grid"], (2, 3, 0, 1)) - np.round(np.transpose(d["grid"], (2, 3, 0, 1)))) < 1e-4
    flips = int(diff.sum())
    print(f"per-pixel PTM int32 tables: {flips} of {diff.size} entries differ from the reference "
          f"({int(near.sum())} reference values lie within 1e-4 of an integer)")
    assert int(near.sum()) > 0  # the golden does exercise near-integer truncations
    assert flips == 0
    assert np.array_equal(compat.prepare_images_data(d["grid"]), ref_t)
    one = compat.interpolate_intensities(data, interpolate_PTM=True, first_only=True)
    assert one.shape == (1, 1, 100, 100)
    with pytest.raises(Exception, match="empty or invalid"):
        compat.interpolate_intensities((1, 2), interpolate_PTM=True)


def test_compat_interpolate_ptm_single_pixel(cuda):
    d = golden("ptm_shared_256x256_N20.npz")
    xf = o.grid_axis()
    for (y, x), g in zip(d["grid_px"], d["grid"]):
        out = compat._interpolate_PTM(d["lu"], d["lv"], xf, d["I"][:, y, x].astype(np.int32))
        err, ok = relight_close(out, g, rtol=1e-6)
        assert ok, err
    with pytest.raises(ValueError):
        compat._interpolate_PTM(d["lu"][:5], d["lv"][:5], xf, np.arange(5))


def test_relight_tables_and_lookup(cuda):
    d = golden("ptm_perpixel_32x32_N50.npz")
    r = int(d["roi_grid"])
    coef = torch.as_tensor(d["coef"][:r, :r], device=cuda)  # the reference's own coefficients
    tables = compat.relight_tables(coef).cpu().numpy()
    assert np.array_equal(tables, d["tables"])
    rows = golden("relight_lookup.npz")["rows"]
    for x, y, h, w, lx, ly, ix, iy in rows[:20]:
        img = compat.relight_lookup(tables, int(x), int(y), (int(h), int(w)))
        ref = np.clip(d["tables"][int(iy), int(ix)], 0, 255)
        assert np.array_equal(img, ref)
    u8 = compat.relight_at_cursor(coef, 200, 100, (400, 400)).cpu().numpy()
    lxy = o.draw_light_roi_position(200, 100, (400, 400), to_light_vector=True)
    L = o.relight(d["coef"][:r, :r], "ptm", lxy[0], lxy[1]).reshape(r, r)
    assert np.array_equal(u8, np.clip(np.trunc(L), 0, 255).astype(np.uint8))


@pytest.mark.parametrize("ptm", [True, False])
def test_compat_compute_end_to_end(cuda, tmp_path, ptm):
    """analysis.compute(from_storage=True) steps 2-4: frames .pbz2 -> GPU -> tables .pickle."""
    from rti import io as rio

    d = golden("ptm_perpixel_32x32_N50.npz")
    data = [(d["frames"][i][:4, :4].copy(), d["cams"][i]) for i in range(len(d["cams"]))]
    rio.write_on_file(data, str(tmp_path / "frames_results_coin9"))
    tables = compat.compute("coin9", from_storage=True, interpolate_PTM=ptm, assets_dir=str(tmp_path))
    assert tables.shape == (100, 100, 4, 4) and tables.dtype == np.int32
    back = rio.read_tables(str(tmp_path / "interpolation_results_coin9"))
    assert np.array_equal(back, tables)
    if ptm:
        ref_grid = d["grid"]  # the reference's own PTM grids for these 4x4 pixels
        ref_t = d["tables"]
    else:
        r = golden("rbf_perpixel_4x4_N50.npz")
        ref_grid, ref_t = r["grid"], r["tables"]
    near = np.abs(ref_grid - np.round(ref_grid)) < 1e-4
    diff = tables != ref_t
    print(f"compute({'PTM' if ptm else 'RBF'}) tables: {int(diff.sum())} of {diff.size} entries differ "
          f"from the reference")
    assert not (diff & ~np.transpose(near, (2, 3, 0, 1))).any()
    if ptm:
        # the fused per-pixel fit's light vectors are bit-exact (rti_perpixel.hip light_dir_fast + refine), so
        # the int32 tables equal the reference's entry for entry
        assert not diff.any(), int(diff.sum())


@pytest.mark.parametrize("basis", ["ptm", "hsh9", "hsh"])
@pytest.mark.parametrize("cdt", [torch.float32, torch.float64])
def test_relight_staged_rows_bit_identical_to_planar(cuda, basis, cdt):
    """Pixel-major maps go through the LDS-staged coalesced row loads (whole 256-pixel wave chunks),
    planar maps through per-lane loads; both evaluate the same products in the same order, so over a
    large image (thousands of workgroups, a partial last chunk) the outputs are bit-identical —
    for relight (several evals, every output type) and for the interactive frame."""
    k = rti.basis_terms(basis)
    P = 1_000_037
    g = torch.Generator(device=cuda).manual_seed(11)
    coef = (torch.rand((P, k), generator=g, device=cuda, dtype=torch.float64) * 120 - 60).to(cdt)
    coef[:, 0 if basis != "ptm" else 5] += 140
    planar = coef.T.contiguous()
    lu, lv = np.array([0.1, -0.7, 0.55]), np.array([0.2, 0.3, -0.6])
    for odt in (cdt, torch.int32, torch.uint8):
        a = rti.relight(coef, lu, lv, basis=basis, out_dtype=odt)
        b = rti.relight(planar, lu, lv, basis=basis, layout="planar", out_dtype=odt)
        assert torch.equal(a, b), odt
    hsv = torch.randint(0, 256, (P, 3), generator=g, device=cuda, dtype=torch.uint8)
    fa = rti.relight_frame(coef, hsv, 0.3, -0.25, basis=basis)
    fb = rti.relight_frame(planar, hsv, 0.3, -0.25, basis=basis, layout="planar")
    assert torch.equal(fa, fb)


@pytest.mark.parametrize("H,W,N", [(32, 32, 50), (300, 257, 100)])
def test_perpixel_cam_light_vectors_bit_exact(cuda, H, W, N):
    """fit_perpixel_cam generates compute_intensities' light vectors in-kernel (rsq + Newton, with pixels
    near an fp32 rounding midpoint sent to the exact refine pass): its coefficients equal those of
    fit_perpixel_dirs fed the bit-exact rti_light_dirs output — bit for bit on every pixel the refine pass
    did not redo (those few are re-solved by QR, within 1e-12)."""
    if N == 50:
        d = golden("ptm_perpixel_32x32_N50.npz")
        cams, frames = d["cams"], np.ascontiguousarray(d["frames"])
    else:
        rng = np.random.default_rng(3)
        cams = np.stack([rng.uniform(-300, 600, N), rng.uniform(-300, 600, N), rng.uniform(100, 500, N)], -1)
        frames = rng.integers(0, 256, (N, H, W)).astype(np.uint8)
    I = torch.as_tensor(frames, device=cuda)
    a = rti.fit(I, cams=cams, mode="perpixel", coef_dtype=torch.float64)
    lu, lv = rti.light_dirs(cams, H, W, device=cuda)
    b = rti.fit(I.permute(1, 2, 0).contiguous(), lu, lv, mode="perpixel", coef_dtype=torch.float64)
    same = (a == b).all(-1)
    frac = float(same.double().mean())
    err, ok = coef_close(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-12)
    print(f"cam vs dirs {H}x{W}x{N}: {frac:.6f} of pixels bit-identical, the rest within {err:.2g}")
    assert ok, err
    assert frac >= 0.999, frac
