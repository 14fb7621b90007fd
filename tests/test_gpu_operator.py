"""GPU parity of the light-operator path (rti_apply_operator): the reference's
default linear-RBF interpolation (SciPy Rbf goldens) and the fused PTM/HSH
fit + grid evaluation, against the oracle."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import golden, relight_close
from rti import compat

pytestmark = pytest.mark.gpu


def grid_q():
    xf = o.grid_axis()
    return np.tile(xf, 100), np.repeat(xf, 100)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("in_dtype", [torch.int32, torch.float32, torch.uint8])
def test_rbf_grid_matches_scipy_golden(cuda, out_dtype, in_dtype):
    d = golden("rbf_shared_4px_N20.npz")
    qu, qv = grid_q()
    I = torch.as_tensor(np.ascontiguousarray(d["I"].T)).to(cuda).to(in_dtype)  # [N, 4 px]
    out = rti.interpolate_rbf(I, d["lu"], d["lv"], qu, qv, out_dtype=out_dtype).cpu().numpy()
    got = out.T.reshape(-1, 100, 100)
    err, ok = relight_close(got, d["grid"])
    assert ok, err


def test_compat_interpolate_rbf_single_pixel(cuda):
    d = golden("rbf_shared_4px_N20.npz")
    yi, xi = np.mgrid[-1:1:0.02, -1:1:0.02]
    xi, yi = np.around(xi, 2), np.around(yi, 2)
    for p in range(4):
        g = compat._interpolate_RBF(d["lu"], d["lv"], xi, yi, d["I"][p])
        assert g.shape == (100, 100) and g.dtype == np.float64
        err, ok = relight_close(g, d["grid"][p])
        assert ok, err


def test_compat_interpolate_intensities_default_rbf(cuda):
    d = golden("rbf_shared_4px_N20.npz")
    N = len(d["lu"])
    lx = np.broadcast_to(d["lu"], (2, 2, N)).copy()
    ly = np.broadcast_to(d["lv"], (2, 2, N)).copy()
    inten = d["I"].reshape(2, 2, N)
    grid = compat.interpolate_intensities((lx, ly, inten))  # default = RBF (analysis.py:321)
    assert grid.shape == (2, 2, 100, 100)
    err, ok = relight_close(grid.reshape(4, 100, 100), d["grid"])
    assert ok, err
    tables = compat.prepare_images_data(grid)
    ref_t = np.transpose(d["grid"].reshape(2, 2, 100, 100), (2, 3, 0, 1)).astype(np.int32)
    near = np.abs(np.transpose(d["grid"].reshape(2, 2, 100, 100), (2, 3, 0, 1)) % 1.0)
    near = np.minimum(near, 1 - near) < 1e-3
    assert not ((tables != ref_t) & ~near).any()
    fused = compat.rbf_tables(torch.as_tensor(np.ascontiguousarray(d["I"].T.reshape(N, 2, 2)), device=cuda),
                              d["lu"], d["lv"]).cpu().numpy()
    assert not ((fused != ref_t) & ~near).any()



def test_rbf_singular_raises_linalgerror(cuda):
    lu = np.array([0.1, 0.1, 0.5, -0.2], np.float32)
    lv = np.array([0.2, 0.2, 0.0, 0.3], np.float32)
    with pytest.raises(np.linalg.LinAlgError):
        rti.rbf_operator(lu, lv, [0.0], [0.0])


@pytest.mark.parametrize("precision", ["split16", "fp32"])
@pytest.mark.parametrize("hw,n,E", [((1, 1), 6, 1), ((3, 5), 7, 3), ((17, 33), 13, 100), ((64, 65), 37, 257),
                                    ((31, 128), 50, 1000), ((8, 8), 256, 70), ((9, 41), 129, 33)])
def test_operator_ragged_vs_oracle(cuda, hw, n, E, precision):
    h, w = hw
    lu, lv = o.synth_dirs(n, n)
    I = o.synth_intensities(h, w, lu, lv, seed=h + w)
    rng = np.random.default_rng(E)
    qu, qv = rng.uniform(-1, 1, E), rng.uniform(-1, 1, E)
    op = rti.basis_operator(lu, lv, qu, qv, "ptm")  # fused fit + evaluation
    out = rti.apply_operator(op, torch.as_tensor(I, device=cuda), precision=precision).cpu().numpy()
    coef = o.fit_shared(I, o.pinv_shared("ptm", lu, lv))
    ref = o.relight(coef, "ptm", qu, qv).reshape(E, h, w)
    err, ok = relight_close(out, ref, rtol=1e-5)
    assert ok, err


@pytest.mark.parametrize("n", [257, 300, 512, 513, 700, 1100])
def test_operator_many_lights(cuda, n):
    """Above 256 lights AUTO applies the fp32 operator (v_mfma_f32_16x16x4_f32): the tile is staged once to
    N = 512, beyond that the light chunks are restaged per row tile.  Fused PTM fit + evaluation and the
    shared-light RBF interpolation (analysis.py:249-260, the reference has no light cap) against the oracle."""
    h, w, E = 9, 37, 300
    lu, lv = o.synth_dirs(n, n)
    I = o.synth_intensities(h, w, lu, lv, seed=n)
    rng = np.random.default_rng(n)
    qu, qv = rng.uniform(-1, 1, E), rng.uniform(-1, 1, E)
    out = rti.apply_operator(rti.basis_operator(lu, lv, qu, qv, "ptm"), torch.as_tensor(I, device=cuda))
    ref = o.relight(o.fit_shared(I, o.pinv_shared("ptm", lu, lv)), "ptm", qu, qv).reshape(E, h, w)
    err, ok = relight_close(out.cpu().numpy(), ref, rtol=1e-5)
    assert ok, err
    sub = np.moveaxis(np.round(I[:, :2, :2]).astype(np.int32), 0, -1)  # 4 pixels [y][x][n], compat's layout
    lx = np.broadcast_to(lu, (2, 2, n)).copy()
    ly = np.broadcast_to(lv, (2, 2, n)).copy()
    gu, gv = grid_q()
    ref = np.stack([o.rbf_linear(lu, lv, sub[y, x], gu, gv) for y in range(2) for x in range(2)])
    got = compat.interpolate_intensities((lx, ly, sub)).reshape(4, -1)
    # the fp32 operator's bound: |err| <= 1e-5 · Σ_n |M_en| |I_n| (M = Φ A⁻¹ grows with cond(A))
    op = rti.rbf_operator(lu, lv, gu, gv)
    bound = 1e-5 * (np.abs(sub.reshape(4, n)) @ np.abs(op))
    err = np.abs(got - ref)
    assert (err <= np.maximum(bound, 1e-9)).all(), float((err / np.maximum(bound, 1e-9)).max())


@pytest.mark.parametrize("precision", ["split16", "fp32"])
def test_operator_channels_and_int_outputs(cuda, precision):
    lu, lv = o.synth_dirs(30, 2)
    planes = np.stack([o.synth_intensities(20, 24, lu, lv, seed=s) for s in (1, 2, 3)])  # [3, N, H, W]
    qu, qv = grid_q()
    op = rti.rbf_operator(lu, lv, qu[:500], qv[:500])
    I = torch.as_tensor(planes, device=cuda)
    f = rti.apply_operator(op, I, out_dtype=torch.float64, precision=precision).cpu().numpy()
    assert f.shape == (3, 500, 20, 24)
    ref = np.einsum("ne,cnhw->cehw", op, planes.astype(np.float64))
    err, ok = relight_close(f, ref)
    assert ok, err
    i32 = rti.apply_operator(op, I, out_dtype=torch.int32, precision=precision).cpu().numpy()
    u8 = rti.apply_operator(op, I, out_dtype=torch.uint8, precision=precision).cpu().numpy()
    frac = np.abs(ref - np.round(ref)) > 1e-3
    assert np.array_equal(i32[frac], np.trunc(ref[frac]).astype(np.int32))
    assert np.array_equal(u8[frac], np.clip(np.trunc(ref[frac]), 0, 255).astype(np.uint8))


@pytest.mark.parametrize("kind", ["fractional", "large", "int32", "nonfinite"])
def test_split16_non_fp16_inputs(cuda, kind):
    """The split-fp16 path stages remainders for inputs not exact in fp16 and scales tiles whose
    values reach 2^15, so any fp32/int32 stack keeps fp32-level accuracy."""
    rng = np.random.default_rng(7)
    n, P, E = 40, 1000, 300
    lu, lv = o.synth_dirs(n, 3)
    qu, qv = rng.uniform(-1, 1, E), rng.uniform(-1, 1, E)
    op = rti.rbf_operator(lu, lv, qu, qv)
    if kind == "fractional":
        I = rng.uniform(0, 255, (n, P)).astype(np.float32)
    elif kind == "large":
        I = (rng.uniform(0, 1, (n, P)) * np.where(np.arange(P) < 500, 1e6, 3.0)).astype(np.float32)
    elif kind == "int32":
        I = rng.integers(-2**30, 2**30, (n, P)).astype(np.int32)
    else:
        I = rng.uniform(0, 255, (n, P)).astype(np.float32)
        I[3, 700] = np.inf
    ref = op.T @ I.astype(np.float64)
    out = rti.apply_operator(op, torch.as_tensor(I, device=cuda), out_dtype=torch.float64,
                             precision="split16").cpu().numpy()
    if kind == "nonfinite":
        tile = (np.arange(P) >= 640) & (np.arange(P) < 768)  # the 128-pixel tile holding the inf
        assert not np.isfinite(out[:, 700]).all()
        ok = ~tile
        scale = np.abs(op).sum(0)[:, None] * np.abs(I[:, ok]).max(0)[None, :]
        assert (np.abs(out[:, ok] - ref[:, ok]) <= 1e-5 * np.maximum(scale, 255)).all()
        return
    # fp32-level: |err| <= 1e-5 * Σ_n |M_en| |I_np| (the fp32 path's bound)
    bound = 1e-5 * (np.abs(op).T @ np.abs(I.astype(np.float64)))
    err = np.abs(out - ref)
    assert (err <= np.maximum(bound, 1e-9)).all(), float((err / np.maximum(bound, 1e-9)).max())


@pytest.mark.parametrize("out_dtype", [torch.float64, torch.float32])
def test_rbf_perpixel_matches_reference_default_path(cuda, out_dtype):
    d = golden("rbf_perpixel_4x4_N50.npz")
    I = torch.as_tensor(d["I"], device=cuda)
    qu, qv = grid_q()
    out = rti.interpolate_rbf_perpixel(I, d["lx"], d["ly"], qu, qv, out_dtype=out_dtype).cpu().numpy()
    err, ok = relight_close(out.reshape(4, 4, 100, 100), d["grid"], rtol=1e-9 if out_dtype == torch.float64 else 1e-6)
    assert ok, err
    ev = rti.interpolate_rbf_perpixel(I, d["lx"], d["ly"], qu, qv, out_dtype=torch.int32, out_layout="eval")
    near = np.abs(d["grid"] - np.round(d["grid"])) < 1e-6
    t = ev.cpu().numpy().reshape(100, 100, 4, 4)
    assert not ((t != d["tables"]) & ~np.transpose(near, (2, 3, 0, 1))).any()


def test_compat_default_interpolation_perpixel(cuda):
    d = golden("rbf_perpixel_4x4_N50.npz")
    grid = compat.interpolate_intensities((d["lx"], d["ly"], d["I"]))  # interpolate_PTM=False: the default
    assert grid.shape == (4, 4, 100, 100) and grid.dtype == np.float64
    err, ok = relight_close(grid, d["grid"], rtol=1e-9)
    assert ok, err
    one = compat.interpolate_intensities((d["lx"], d["ly"], d["I"]), first_only=True)
    assert one.shape == (1, 1, 100, 100)
    with pytest.raises(np.linalg.LinAlgError):
        compat.interpolate_intensities((d["singular_lx"], d["singular_ly"], d["I"][:1, :1]))


@pytest.mark.parametrize("n", [2, 6, 37, 64, 65, 80, 81, 100, 127, 128, 129, 160, 200, 248, 249, 255, 256,
                               257, 300, 400, 512, 568, 569, 1100, 1800, 2557, 3000, 3500, 4089, 4090, 5000])
def test_rbf_perpixel_sizes_vs_oracle(cuda, n):
    """Every solver of rti_rbf_perpixel: fp64 register Gauss-Jordan (N <= 80) and the register-blocked
    fp32 Gauss-Jordan inverse + fp64 refinement on the full 16x16 block grid (N <= 128), the
    lower-triangle block grid (N <= 248) and the full 32x32 grid (N <= 256) (SURVEY §6 timed the
    reference at N = 200), and above 256 lights the blocked fp64 Cholesky (panels of 32 lights to N = 568,
    16 to 1022, 8 to 1704, 4 to 2556, 2 to 3408, 1 to 4089; above that the same solver with only the diagonal
    block in LDS and the panel solved in place in global memory — the reference takes N = frames/8 with no cap,
    analysis.py:120,152), each with the reference's per-pixel geometry, against SciPy's fp64 solve restated
    in the oracle.  (N > 1800 runs on 4 pixels: each pixel is one workgroup's seconds of work; 3500 and 4089
    take the one-column panel, 4090 and 5000 the global-panel form.)"""
    ys, xs = np.mgrid[0:3, 0:5] if n <= 1800 else np.mgrid[0:2, 0:2]
    rng = np.random.default_rng(n)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())  # [15, n] float32
    npx = xs.size
    inten = rng.integers(0, 256, (npx, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 300), rng.uniform(-1, 1, 300)
    out = rti.interpolate_rbf_perpixel(torch.as_tensor(inten, device=cuda), lu, lv, qu, qv).cpu().numpy()
    ref = np.stack([o.rbf_linear(lu[p], lv[p], inten[p], qu, qv) for p in range(npx)])
    err, ok = relight_close(out, ref, rtol=1e-8)
    assert ok, err


@pytest.mark.parametrize("n", [129, 130, 146, 177, 193, 194, 200, 256, 300, 449, 641, 642, 660, 706, 1000])
def test_rbf_perpixel_llt_matches_right_looking(cuda, monkeypatch, n):
    """r06: 129 <= N <= 1022 runs the left-looking matrix-core Cholesky (rbf_solve_llt; two 4-wave pixels per CU up
    to 641 lights, one 8-wave pixel per CU above); RTI_RBF_CHOL_OLD=1 keeps r05's solvers (the fp32 Gauss-Jordan
    inverses + refinement up to 256, the right-looking rbf_solve_chol above).  Both agree with SciPy's fp64 solve
    (the oracle) at 1e-8 of max(|f|, 255) on the same pixels, and with each other.  The padding trim's cases
    (n = N − 1 padded to a multiple of 64): one real column in the last block column and three padding row groups
    (130, 194), two / three real sub-panels (146, 177), no padding (129, 193, 449, 641), and the 8-wave form with
    padding row groups and two real sub-panels (660), three and one real column (706), one and three (1000)."""
    ys, xs = np.mgrid[0:2, 0:3]
    rng = np.random.default_rng(1000 + n)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    inten = rng.integers(0, 256, (xs.size, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 200), rng.uniform(-1, 1, 200)
    I = torch.as_tensor(inten, device=cuda)
    new = rti.interpolate_rbf_perpixel(I, lu, lv, qu, qv).cpu().numpy()
    monkeypatch.setenv("RTI_RBF_CHOL_OLD", "1")
    old = rti.interpolate_rbf_perpixel(I, lu, lv, qu, qv).cpu().numpy()
    ref = np.stack([o.rbf_linear(lu[p], lv[p], inten[p], qu, qv) for p in range(xs.size)])
    for got in (new, old):
        err, ok = relight_close(got, ref, rtol=1e-8)
        assert ok, err
    err, ok = relight_close(new, old, rtol=1e-8)
    assert ok, err


@pytest.mark.parametrize("budget_slots", [0, 2])
def test_rbf_perpixel_gp_small_workspace_budget(cuda, monkeypatch, budget_slots):
    """Above 4089 lights the Cholesky slots (≈ 4·N² bytes each) are sized from the device's free memory, not a
    fixed 48 GiB: a budget below one slot still runs ONE workgroup striding over every pixel, and a budget of
    two slots runs two (RTI_RBF_GP_WS_BYTES lowers the budget).  Same results as the oracle either way."""
    n = 4090
    ld = (n + 31) // 32 * 32
    slot = 8 * ((ld * (ld + 1) // 2 + 31) // 32 * 32 + 6 * ld)  # chol_slot_doubles_gp(n) * 8 bytes
    monkeypatch.setenv("RTI_RBF_GP_WS_BYTES", str(budget_slots * slot + slot // 2 if budget_slots else 1))
    ys, xs = np.mgrid[0:1, 0:3]
    rng = np.random.default_rng(77)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    npx = xs.size
    inten = rng.integers(0, 256, (npx, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 64), rng.uniform(-1, 1, 64)
    out = rti.interpolate_rbf_perpixel(torch.as_tensor(inten, device=cuda), lu, lv, qu, qv).cpu().numpy()
    grid = int(rti._lib.lib().rti_rbf_last_chol_grid())
    assert grid == max(1, min(budget_slots, npx)), grid
    ref = np.stack([o.rbf_linear(lu[p], lv[p], inten[p], qu, qv) for p in range(npx)])
    err, ok = relight_close(out, ref, rtol=1e-8)
    assert ok, err


@pytest.mark.parametrize("n", [81, 128, 129, 200, 256, 257, 400, 600, 4100])
def test_rbf_perpixel_large_n_repeated_node_raises(cuda, n):
    """A repeated light direction makes A exactly singular: SciPy raises LinAlgError; so do the
    block Gauss-Jordan and the blocked Cholesky solvers (LDS and global panels); N above 32768 lights
    (a 2.4-hour capture at 30 fps: a 4.3 GB fp64 slot per workgroup) is refused (RTI_ERR_UNSUPPORTED)."""
    ys, xs = np.mgrid[0:2, 0:2]
    rng = np.random.default_rng(n)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    lu[2, 7], lv[2, 7] = lu[2, 3], lv[2, 3]
    inten = rng.integers(0, 256, (4, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 50), rng.uniform(-1, 1, 50)
    with pytest.raises(np.linalg.LinAlgError):
        rti.interpolate_rbf_perpixel(torch.as_tensor(inten, device=cuda), lu, lv, qu, qv)
    with pytest.raises(NotImplementedError):
        rti.interpolate_rbf_perpixel(torch.zeros((1, 32769), dtype=torch.int32, device=cuda),
                                     np.zeros((1, 32769), np.float32), np.zeros((1, 32769), np.float32), qu, qv)


@pytest.mark.parametrize("n", [100, 200, 256, 300])
@pytest.mark.parametrize("d", [1e-5, 1e-6, 1e-7])
def test_rbf_perpixel_near_repeated_nodes_fp64_fallback(cuda, n, d):
    """Nearly repeated light directions (cond(A) ~ 1e7 .. 2e9): SciPy's fp64 LU still solves them, the
    fp32 Gauss-Jordan inverse cannot (non-positive pivot, or a refinement that contracts too slowly).
    Such pixels are flagged and solved again by the fp64 partial-pivoting fallback; the other pixels
    of the same launch keep the fast path.  Parity with the oracle at 1e-7 of max(|f|, 255) (both
    solvers are fp64 with errors ~ cond * eps)."""
    ys, xs = np.mgrid[0:2, 0:2]
    rng = np.random.default_rng(n)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    lu[2, 7], lv[2, 7] = np.float32(lu[2, 3] + d), lv[2, 3]
    inten = rng.integers(0, 256, (4, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 200), rng.uniform(-1, 1, 200)
    stats = {}
    out = rti.interpolate_rbf_perpixel(torch.as_tensor(inten, device=cuda), lu, lv, qu, qv, stats=stats).cpu().numpy()
    assert stats["fallback_px"] <= 1  # only the perturbed pixel may need it (N >= 129: the Cholesky, no fallback)
    for p in range(4):
        ref = o.rbf_linear(lu[p], lv[p], inten[p], qu, qv)
        err, ok = relight_close(out[p], ref, rtol=1e-7 if p == 2 else 1e-8)
        assert ok, (p, err)


@pytest.mark.parametrize("n", [100, 138, 139, 200])
@pytest.mark.parametrize("solver", ["gj", "llt"])
def test_rbf_perpixel_fallback_many_pixels(cuda, monkeypatch, n, solver):
    """Every pixel of the launch nearly repeats a light direction: (nearly) all go to the fp64 fallback,
    whose list spreads them over the grid (more pixels than workgroups: each takes several), with [A | b]
    in LDS up to N = 138 and in a global slot above; the count comes back as stats["fallback_px"].  Since r06
    the fp64 left-looking Cholesky solves N >= 129 without any fallback ("llt": count 0); "gj" keeps r05's fp32
    Gauss-Jordan inverses + fallback for those N (RTI_RBF_LLT_MIN_N=257, the measurement switch)."""
    if solver == "llt" and n < 129:
        pytest.skip("N <= 128 is the register Gauss-Jordan inverse's range")
    if solver == "gj":
        monkeypatch.setenv("RTI_RBF_LLT_MIN_N", "257")
    P = 300
    rng = np.random.default_rng(n + 1)
    ys, xs = np.divmod(np.arange(P), 20)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs, ys)
    lu[:, 7], lv[:, 7] = lu[:, 3] + np.float32(1e-6), lv[:, 3]
    inten = rng.integers(0, 256, (P, n)).astype(np.int32)
    qu, qv = rng.uniform(-1, 1, 64), rng.uniform(-1, 1, 64)
    stats = {}
    out = rti.interpolate_rbf_perpixel(torch.as_tensor(inten, device=cuda), lu, lv, qu, qv, stats=stats).cpu().numpy()
    # how many pixels the fp32 inverse gives up on depends on N and the geometry (N = 100: 295 of 300, more than
    # the 256 workgroups, so some take two list entries; N = 138: 127)
    if solver == "llt":
        assert stats["fallback_px"] == 0
    else:
        assert (257 if n == 100 else 1) <= stats["fallback_px"] <= P
    for p in list(range(0, P, 37)) + [P - 1]:
        ref = o.rbf_linear(lu[p], lv[p], inten[p], qu, qv)
        err, ok = relight_close(out[p], ref, rtol=1e-6)  # cond(A) ~ 1e9..1e10: both fp64 solves err ~ cond·eps
        assert ok, (p, err)


def test_rbf_perpixel_query_on_a_node(cuda):
    """A grid query that coincides exactly with a light direction (distance 0 in the evaluation sweep)
    gives the node's own value: finite, and equal to the oracle's (the sweep biases ‖q − x‖² by 1e-300
    instead of clamping every term)."""
    ys, xs = np.mgrid[0:2, 0:2]
    n = 40
    rng = np.random.default_rng(5)
    cams = np.stack([rng.uniform(-100, 100, n), rng.uniform(-100, 100, n), rng.uniform(60, 150, n)], -1)
    lu, lv = o.light_dirs_for_pixels(cams, xs.ravel(), ys.ravel())
    lu[:, 5], lv[:, 5] = np.float32(0.5), np.float32(-0.5)  # exactly on the reference's 0.02 grid
    inten = rng.integers(0, 256, (4, n)).astype(np.int32)
    xf = np.around(np.arange(-1, 1, 0.02), 2)
    qu, qv = np.tile(xf, 100), np.repeat(xf, 100)
    for m in (n, 100, 200):  # fp64 register GJ, and the block solvers
        if m != n:
            extra = o.light_dirs_for_pixels(np.stack([rng.uniform(-100, 100, m - n), rng.uniform(-100, 100, m - n),
                                                      rng.uniform(60, 150, m - n)], -1), xs.ravel(), ys.ravel())
            lum, lvm = np.concatenate([lu, extra[0]], 1), np.concatenate([lv, extra[1]], 1)
            im = np.concatenate([inten, rng.integers(0, 256, (4, m - n)).astype(np.int32)], 1)
        else:
            lum, lvm, im = lu, lv, inten
        out = rti.interpolate_rbf_perpixel(torch.as_tensor(im, device=cuda), lum, lvm, qu, qv).cpu().numpy()
        assert np.isfinite(out).all()
        on = np.flatnonzero((qu == 0.5) & (qv == -0.5))
        for p in range(4):
            ref = o.rbf_linear(lum[p], lvm[p], im[p], qu, qv)
            err, ok = relight_close(out[p], ref, rtol=1e-8)
            assert ok, (m, p, err)
            assert abs(out[p][on[0]] - im[p][5]) < 1e-6


def test_rbf_perpixel_large_roi_past_65535_tiles(cuda):
    """A 2100 x 2100 ROI (4.41 M pixels: more 64-pixel tiles than one launch's grid-y holds) is
    evaluated in pixel-range launches; pixels on both sides of the 4.19 M boundary match the oracle."""
    H = W = 2100
    n = 20
    rng = np.random.default_rng(21)
    cams = np.stack([rng.uniform(-600, 2700, n), rng.uniform(-600, 2700, n), rng.uniform(300, 900, n)], -1)
    lu, lv = rti.light_dirs(cams, H, W, device=cuda)
    g = torch.Generator(device=cuda).manual_seed(3)
    inten = torch.randint(0, 256, (H, W, n), generator=g, device=cuda, dtype=torch.int32)
    qu, qv = rng.uniform(-1, 1, 12), rng.uniform(-1, 1, 12)
    out = rti.interpolate_rbf_perpixel(inten, lu, lv, qu, qv)
    P = H * W
    idx = np.concatenate([[0, 1, 65535 * 64 - 1, 65535 * 64, 65535 * 64 + 1, P - 1],
                          rng.integers(0, P, 40)])
    lu_h = lu.reshape(P, n)[idx].cpu().numpy()
    lv_h = lv.reshape(P, n)[idx].cpu().numpy()
    i_h = inten.reshape(P, n)[idx].cpu().numpy()
    got = out.reshape(P, -1)[idx].cpu().numpy()
    for k in range(len(idx)):
        ref = o.rbf_linear(lu_h[k], lv_h[k], i_h[k], qu, qv)
        err, ok = relight_close(got[k], ref, rtol=1e-8)
        assert ok, (int(idx[k]), err)
