"""GPU parity of the shared-direction fit (rti_fit_shared) against the oracle
and the reference's golden coefficients.  Tolerance:
|c - c_ref| <= 1e-4 * max_k |c_ref,k| per pixel, fp32 arithmetic."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden

pytestmark = pytest.mark.gpu

KERNELS = ["valu", "mfma", "tile"]


def to_dev(a, dev, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dev, dtype)


@pytest.mark.parametrize("kernel", KERNELS)
def test_golden_256x256_N20(cuda, kernel):
    d = golden("ptm_shared_256x256_N20.npz")
    I = to_dev(d["I"], cuda)  # [20, 256, 256] light-major
    coef = rti.fit(I, d["lu"], d["lv"], kernel=kernel).cpu().numpy()
    err, ok = coef_close(coef, d["coef"])
    assert ok, err


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8, torch.int32])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_dtypes_layouts(cuda, kernel, in_dtype, layout):
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"]).to(cuda).to(in_dtype)
    coef = rti.fit(I, d["lu"], d["lv"], kernel=kernel, layout=layout).cpu().numpy()
    if layout == "planar":
        coef = np.moveaxis(coef, 0, -1)
    err, ok = coef_close(coef, d["coef"])
    assert ok, err


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("hw,n", [((1, 1), 6), ((3, 5), 7), ((17, 33), 13), ((64, 65), 37), ((31, 128), 50),
                                  ((8, 8), 200)])
def test_ragged_shapes_vs_oracle(cuda, kernel, hw, n):
    h, w = hw
    lu, lv = o.synth_dirs(n, n)
    I = o.synth_intensities(h, w, lu, lv, seed=h * 1000 + w)
    ref = o.fit_shared(I, o.pinv_shared("ptm", lu, lv)).reshape(h, w, 6)
    coef = rti.fit(to_dev(I, cuda), lu, lv, kernel=kernel).cpu().numpy()
    err, ok = coef_close(coef, ref)
    assert ok, err


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("basis,k", [("hsh", 16), ("hsh9", 9)])
def test_hsh_vs_oracle(cuda, kernel, basis, k):
    lu, lv = o.synth_dirs(60, 11)
    I = o.synth_intensities(48, 40, lu, lv, seed=3, basis="hsh")
    A = o.design("hsh", lu, lv)[:, :k]
    ref = (np.linalg.pinv(A) @ I.reshape(60, -1).astype(np.float64)).T.reshape(48, 40, k)
    coef = rti.fit(to_dev(I, cuda), lu, lv, basis=basis, kernel=kernel).cpu().numpy()
    err, ok = coef_close(coef, ref)
    assert ok, err


@pytest.mark.parametrize("kernel", KERNELS)
def test_rgb_channels(cuda, kernel):
    lu, lv = o.synth_dirs(40, 4)
    planes = [o.synth_intensities(32, 48, lu, lv, seed=s) for s in (1, 2, 3)]
    I = np.stack(planes)  # [3, N, H, W]
    pv = o.pinv_shared("ptm", lu, lv)
    coef = rti.fit(to_dev(I, cuda), lu, lv, kernel=kernel).cpu().numpy()
    assert coef.shape == (3, 32, 48, 6)
    for c in range(3):
        err, ok = coef_close(coef[c], o.fit_shared(planes[c], pv).reshape(32, 48, 6))
        assert ok, (c, err)


@pytest.mark.parametrize("flags", [0x100, 0x200, 0x300, 0x400, 0x800, 0x900, 0xB00, 0xF00])
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("basis,n", [("ptm", 37), ("hsh", 53), ("hsh9", 20)])
def test_tuning_variants(cuda, flags, kernel, basis, n):
    lu, lv = o.synth_dirs(n, 21)
    I = o.synth_intensities(40, 36, lu, lv, seed=9, basis="hsh" if basis != "ptm" else "ptm")
    k = rti.basis_terms(basis)
    A = o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k]
    ref = (np.linalg.pinv(A) @ I.reshape(n, -1).astype(np.float64)).T.reshape(40, 36, k)
    Id = to_dev(I, cuda).reshape(n, -1)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    for layout in ("pixel", "planar"):
        coef = torch.empty((1, 40 * 36, k) if layout == "pixel" else (1, k, 40 * 36), device=cuda)
        rti.fit_shared_into(pv, Id[None], coef, k=k, layout=layout, kernel=kernel, flags=flags)
        got = coef[0].cpu().numpy()
        got = got.reshape(40, 36, k) if layout == "pixel" else np.moveaxis(got.reshape(k, 40, 36), 0, -1)
        err, ok = coef_close(got, ref)
        assert ok, (layout, err)


def test_rank_deficient_gives_nonfinite(cuda):
    e = golden("ptm_edge.npz")
    I = to_dev(np.tile(e["singular_I"].astype(np.float32)[:, None], (1, 64)), cuda)
    coef = rti.fit(I, e["singular_lu"], e["singular_lv"]).cpu().numpy()
    assert not np.isfinite(coef).all()
    coef = rti.fit(I, e["singular_lu"], e["singular_lv"], rcond=1e-10).cpu().numpy()
    assert np.isfinite(coef).all()


def test_edge_goldens_single_pixels(cuda):
    e = golden("ptm_edge.npz")
    for name in ("exact6", "n200"):
        I = to_dev(e[f"{name}_I"].astype(np.float32)[:, None], cuda)
        coef = rti.fit(I, e[f"{name}_lu"], e[f"{name}_lv"]).cpu().numpy()
        err, ok = coef_close(coef, e[f"{name}_coef"][None])
        assert ok, (name, err)


def test_too_few_lights_raises(cuda):
    lu, lv = o.synth_dirs(5, 1)
    with pytest.raises(ValueError):
        rti.fit(torch.zeros((5, 4, 4), device=cuda), lu, lv)


def test_custom_op_matches_api(cuda):
    from rti import ops  # noqa: F401  registers torch.ops.rti.*

    d = golden("ptm_shared_256x256_N20.npz")
    I = to_dev(d["I"], cuda).reshape(20, -1)
    pv = torch.as_tensor(rti.pinv(d["lu"], d["lv"]).astype(np.float32), device=cuda)
    coef = torch.ops.rti.fit_shared(pv, I).cpu().numpy().reshape(d["coef"].shape)
    err, ok = coef_close(coef, d["coef"])
    assert ok, err


@pytest.mark.slow
@pytest.mark.parametrize("kernel,layout", [(k, "planar") for k in KERNELS] + [("auto", "pixel")])
def test_full_size_4k_n100_properties(cuda, kernel, layout):
    """BASELINE configs[2] size (3840x2160, N=100): sampled fp64 parity, exact recovery, linearity.
    ("auto", "pixel") is bench.py's headline path exactly: fit_shared_valu as 4 launch generations with
    LDS-staged pixel-major stores."""
    H, W, N = 2160, 3840, 100
    lu, lv = o.synth_dirs(N, 2)
    g = torch.Generator(device=cuda).manual_seed(0)
    a_true = torch.rand((6, H * W), generator=g, device=cuda, dtype=torch.float32) * 100 - 50
    B = o.ptm_design(lu, lv)  # [N, 6] fp64
    # noise-free stack built element-wise in fp32 (no library GEMM involved)
    I = torch.empty((N, H * W), device=cuda, dtype=torch.float32)
    for n in range(N):
        row = torch.zeros(H * W, device=cuda, dtype=torch.float32)
        for j in range(6):
            row.add_(a_true[j], alpha=float(B[n, j]))
        I[n] = row
    def fit6(stack):  # [6, P] whatever the layout
        c = rti.fit(stack.reshape(N, H, W), lu, lv, kernel=kernel, layout=layout)
        return c.reshape(6, -1) if layout == "planar" else c.reshape(-1, 6).T

    coef = fit6(I)
    if kernel == "auto":
        assert int(rti._lib.lib().rti_last_launch_count()) == 4  # the bench's 4 launch generations
    # sampled pixels against the fp64 oracle on the same fp32 stack
    idx = torch.randint(0, H * W, (4096,), generator=g, device=cuda)
    ref = o.fit_shared(I[:, idx].cpu().numpy(), o.pinv_shared("ptm", lu, lv))
    err, ok = coef_close(coef[:, idx].T.cpu().numpy(), ref)
    assert ok, err
    # exact recovery of the generating coefficients (up to fp32 rounding of the stack)
    scale = a_true.abs().amax(0).clamp_min(1.0)
    assert float(((coef - a_true).abs() / scale).max()) < 1e-4
    # linearity: fit(2I + 3) = 2 fit(I) + 3 pinv·1
    coef2 = fit6(2 * I + 3)
    c3 = torch.as_tensor(o.pinv_shared("ptm", lu, lv).sum(1) * 3, device=cuda, dtype=torch.float32)[:, None]
    assert float(((coef2 - 2 * coef - c3).abs() / (2 * scale)).max()) < 1e-4


@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_auto_hsh_large_image(cuda, layout):
    """AUTO on an HSH-16 fp32 stack big enough for the LDS-tiled MFMA kernel (>= 1024 tiles):
    2 channels x 1100 x 1000 px x 23 lights (a partial tile and a partial light step), sampled
    pixels against the fp64 oracle."""
    C, H, W, N = 2, 1100, 1000, 23
    lu, lv = o.synth_dirs(N, 5)
    g = torch.Generator(device=cuda).manual_seed(3)
    I = torch.randint(0, 256, (C, N, H, W), generator=g, device=cuda).float()
    coef = rti.fit(I, lu, lv, basis="hsh", layout=layout)
    pinv64 = np.linalg.pinv(o.design("hsh", lu, lv))
    idx = torch.randint(0, H * W, (4096,), generator=g, device=cuda)
    for c in range(C):
        ref = (pinv64 @ I[c].reshape(N, -1)[:, idx].cpu().numpy().astype(np.float64)).T
        got = coef[c].reshape(H * W, 16)[idx] if layout == "pixel" else coef[c].reshape(16, H * W)[:, idx].T
        err, ok = coef_close(got.cpu().numpy(), ref)
        assert ok, (c, err)


@pytest.mark.parametrize("rc,sp", [(1, 1), (2, 1), (4, 1), (8, 1), (1, 2), (2, 2), (4, 2), (8, 2)])
@pytest.mark.parametrize("basis,n", [("hsh", 29), ("hsh9", 10), ("ptm", 37), ("hsh9", 200)])
@pytest.mark.parametrize("nt", [0, 0x100])
@pytest.mark.parametrize("depth", [2, 3, 4])
def test_lds_tile_variants(cuda, rc, sp, basis, n, nt, depth):
    """MFMA kernel on the LDS tile (RTI_KERNEL_TILE): tile widths 256·rc, 4·sp planes per step with
    light counts that leave a partial last step, register-staged (depth 2) and DMA-ring (3, 4)
    staging, pixel counts around tile multiples (partial tiles, lanes past the image), two
    channels, both coefficient layouts."""
    k = rti.basis_terms(basis)
    lu, lv = o.synth_dirs(n, 17)
    pinv64 = np.linalg.pinv(o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k])
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    R = 256 * rc
    flags = nt | (rc << rti._lib.RTI_KERNEL_CHUNKS_SHIFT) | (sp << rti._lib.RTI_KERNEL_TILE_PLANES_SHIFT) | \
        (depth << rti._lib.RTI_KERNEL_TILE_DEPTH_SHIFT)
    for P in (4, R - 4, R, R + 4, 3 * R + 260):
        rng = np.random.default_rng(P + n)
        I = rng.integers(0, 256, size=(2, n, P)).astype(np.float32)
        ref = np.einsum("kn,cnp->cpk", pinv64, I.astype(np.float64))
        for layout in ("pixel", "planar"):
            coef = torch.full((2, P, k) if layout == "pixel" else (2, k, P), float("nan"), device=cuda)
            rti.fit_shared_into(pv, torch.as_tensor(I, device=cuda), coef, k=k, layout=layout, kernel="tile",
                                flags=flags)
            got = coef.cpu().numpy()
            if layout == "planar":
                got = np.moveaxis(got, 1, 2)
            for c in range(2):
                err, ok = coef_close(got[c], ref[c])
                assert ok, (P, layout, c, err)


@pytest.mark.parametrize("chunks", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("basis,n", [("ptm", 23), ("hsh9", 17), ("hsh", 29)])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8, torch.int32])
def test_wide_lane_chunks(cuda, chunks, basis, n, in_dtype):
    """VALU kernel with `chunks` 1 KiB runs per lane and plane (RTI_KERNEL_CHUNKS): pixel counts
    around whole-wave multiples (partial last wave, lanes with only some chunks in range),
    two channels, both coefficient layouts."""
    k = rti.basis_terms(basis)
    lu, lv = o.synth_dirs(n, 31)
    A = o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k]
    pinv64 = np.linalg.pinv(A)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    wave_px = 64 * 4 * chunks
    for P in (4, wave_px - 4, wave_px, wave_px + 4, 3 * wave_px + 260, 5 * wave_px + 1024 * 3 + 8):
        rng = np.random.default_rng(P + n)
        I = rng.integers(0, 256, size=(2, n, P)).astype(np.float32)
        ref = np.einsum("kn,cnp->cpk", pinv64, I.astype(np.float64))
        Id = torch.as_tensor(I, device=cuda).to(in_dtype)
        for layout in ("pixel", "planar"):
            coef = torch.full((2, P, k) if layout == "pixel" else (2, k, P), float("nan"), device=cuda)
            rti.fit_shared_into(pv, Id, coef, k=k, layout=layout, kernel="valu",
                                flags=0x100 | (chunks << rti._lib.RTI_KERNEL_CHUNKS_SHIFT))
            got = coef.cpu().numpy()
            if layout == "planar":
                got = np.moveaxis(got, 1, 2)
            for c in range(2):
                err, ok = coef_close(got[c], ref[c])
                assert ok, (P, layout, c, err)


@pytest.mark.parametrize("rc,depth", [(4, 2), (4, 3), (8, 2), (8, 3), (8, 1), (15, 1)])
@pytest.mark.parametrize("basis,n", [("hsh", 29), ("hsh", 200), ("hsh9", 10), ("ptm", 37), ("hsh", 16), ("hsh", 24)])
def test_lds_tile_wide_workgroup(cuda, rc, depth, basis, n):
    """The 8-wave tile kernel (RTI_KERNEL_TILE_WAVES(8)): one plane per wave and step, plane loads
    1 (depth 2) or 2 (depth 3) steps ahead, or one LDS tile (depth 1, rc 8 or 15 -> 16 chunks);
    light counts giving 1, 2, 3 (odd) and 25 steps and a partial last step, pixel counts around tile
    multiples, two channels, both layouts."""
    rc_eff = 16 if rc >= 12 else rc
    k = rti.basis_terms(basis)
    lu, lv = o.synth_dirs(n, 19)
    pinv64 = np.linalg.pinv(o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k])
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    R = 256 * rc_eff
    L = rti._lib
    flags = 0x100 | (rc << L.RTI_KERNEL_CHUNKS_SHIFT) | (depth << L.RTI_KERNEL_TILE_DEPTH_SHIFT) | \
        (8 << L.RTI_KERNEL_TILE_WAVES_SHIFT)
    for P in (4, R - 4, R, 3 * R + 260):
        rng = np.random.default_rng(P + n + rc)
        I = rng.integers(0, 256, size=(2, n, P)).astype(np.float32)
        ref = np.einsum("kn,cnp->cpk", pinv64, I.astype(np.float64))
        for layout in ("pixel", "planar"):
            coef = torch.full((2, P, k) if layout == "pixel" else (2, k, P), float("nan"), device=cuda)
            rti.fit_shared_into(pv, torch.as_tensor(I, device=cuda), coef, k=k, layout=layout, kernel="tile",
                                flags=flags)
            got = coef.cpu().numpy()
            if layout == "planar":
                got = np.moveaxis(got, 1, 2)
            for c in range(2):
                err, ok = coef_close(got[c], ref[c])
                assert ok, (P, layout, c, err)


@pytest.mark.parametrize("basis,N,C,layout", [("ptm", 100, 1, "pixel"), ("ptm", 100, 2, "planar"),
                                              ("hsh", 40, 1, "pixel"), ("hsh", 40, 2, "planar")])
def test_launch_generations_bit_identical(cuda, basis, N, C, layout):
    """AUTO issues large fits as consecutive launches over pixel ranges (rti_fit.hip, launch
    generations); every pixel's arithmetic is the one-launch kernel's, so the coefficients must be
    bit-identical to RTI_KERNEL_ONE_LAUNCH's, over a ragged pixel count (partial last wave / tile)."""
    from rti import _lib as L

    H, W = 2150, 2100  # P = 4 515 000: PTM-6 splits into 5 launches per channel, HSH-16 into 5 tile ranges
    P = H * W
    k = rti.basis_terms(basis)
    g = torch.Generator(device=cuda).manual_seed(7)
    I = torch.randint(0, 256, (C, N, P), generator=g, device=cuda).to(torch.float32)
    lu, lv = o.synth_dirs(N, 3)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    shape = (C, P, k) if layout == "pixel" else (C, k, P)
    a = torch.full(shape, float("nan"), device=cuda)
    b = torch.full(shape, float("nan"), device=cuda)
    rti.fit_shared_into(pv, I, a, k=k, layout=layout)
    assert int(L.lib().rti_last_launch_count()) > 1  # the call was split into launch generations
    rti.fit_shared_into(pv, I, b, k=k, layout=layout, flags=L.RTI_KERNEL_ONE_LAUNCH)
    assert int(L.lib().rti_last_launch_count()) == 1
    torch.cuda.synchronize()
    assert not torch.isnan(a).any()
    assert torch.equal(a, b)
    # the same generations as rounds of one launch (RTI_KERNEL_ROUNDS: the VALU rounds kernel for PTM-6, the
    # tile stream for HSH-16): same per-pixel arithmetic, so the same bits
    r = torch.full(shape, float("nan"), device=cuda)
    rti.fit_shared_into(pv, I, r, k=k, layout=layout, flags=L.RTI_KERNEL_ROUNDS)
    assert int(L.lib().rti_last_launch_count()) == 1
    torch.cuda.synchronize()
    assert torch.equal(r, b)
    if k == 16:  # AUTO's non-temporal LDS-staged whole-line stores against the plain per-lane stores of TILE
        s = torch.full(shape, float("nan"), device=cuda)
        rti.fit_shared_into(pv, I, s, k=k, layout=layout, kernel="tile",
                            flags=(15 << L.RTI_KERNEL_CHUNKS_SHIFT) | (1 << L.RTI_KERNEL_TILE_DEPTH_SHIFT)
                            | (8 << L.RTI_KERNEL_TILE_WAVES_SHIFT) | L.RTI_KERNEL_NONTEMPORAL)
        torch.cuda.synchronize()
        assert torch.equal(s, b)
    # and against the fp64 oracle on sampled pixels of the last channel (parts' boundaries included)
    px = np.unique(np.concatenate([np.random.default_rng(5).integers(0, P, 512), [0, P - 1, P // 5, P // 5 - 1]]))
    ref = o.fit_shared(I[-1][:, torch.as_tensor(px, device=cuda)].cpu().numpy(), o.pinv_shared(basis, lu, lv))
    got = (a[-1][px] if layout == "pixel" else a[-1][:, px].T).double().cpu().numpy()
    err, ok = coef_close(got, ref)
    assert ok, err


@pytest.mark.parametrize("P", [1024 * 37, 1024 * 37 + 16 * 5, 4096 * 600 + 48])
def test_u8_staged_pixel_major_matches_planar(cuda, P):
    """8-bit stacks (the reference's V channel, analysis.py:219): AUTO's 16-pixel lanes leave their
    pixel-major coefficients through the LDS slab in four 256-pixel steps (whole 1024-pixel chunks; the
    partial chunk stores directly).  Same accumulators as the planar layout's direct stores, so the two
    must agree bit for bit, and with the fp64 oracle."""
    N = 40
    lu, lv = o.synth_dirs(N, 5)
    g = torch.Generator(device=cuda).manual_seed(P)
    I = torch.randint(0, 256, (N, P), generator=g, device=cuda).to(torch.uint8)
    pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
    a = torch.full((1, P, 6), float("nan"), device=cuda)
    b = torch.full((1, 6, P), float("nan"), device=cuda)
    rti.fit_shared_into(pv, I, a, k=6, layout="pixel")
    rti.fit_shared_into(pv, I, b, k=6, layout="planar")
    assert torch.equal(a[0], b[0].T)
    idx = np.unique(np.concatenate([np.random.default_rng(1).integers(0, P, 300), [0, 255, 256, 1023, P - 1]]))
    ref = o.fit_shared(I[:, torch.as_tensor(idx, device=cuda)].cpu().numpy(), o.pinv_shared("ptm", lu, lv))
    err, ok = coef_close(a[0][idx].double().cpu().numpy(), ref)
    assert ok, err
