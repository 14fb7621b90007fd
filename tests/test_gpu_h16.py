"""GPU parity of the 8-bit fit on the fp16 matrix cores (rti_fit_shared_h16, AUTO for uint8 stacks in
rti.fit, rti_fit_h16.hip): the reference's golden coefficients, the fp64 oracle over every supported basis,
light counts around the 32-light steps and the LDS limit, ragged pixel counts (partial tiles and streams),
channels, both layouts, exact extremes, and the ABI's refusals.

Tolerance: the operator is split as w·s = hi + lo in fp16 (22 significant bits) and the sums are fp32, the
accuracy of the fp32 stream; coefficients are held to the SURVEY §8(c) bar, 1e-4 of max_k |c_ref,k| per
pixel, and in practice land near 1e-6 (printed)."""
import ctypes

import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden
from rti import _lib as L

pytestmark = pytest.mark.gpu


def test_golden_256x256_N20(cuda):
    d = golden("ptm_shared_256x256_N20.npz")
    I = np.asarray(d["I"]).astype(np.uint8)
    assert np.array_equal(I, d["I"])  # the golden stack is integer 0..255
    coef = rti.fit(torch.as_tensor(I, device=cuda), d["lu"], d["lv"]).cpu().numpy()  # AUTO = h16 on uint8
    err, ok = coef_close(coef, d["coef"], rtol=1e-5)  # the reference's own coefficients (analysis.py:293-298)
    print(f"h16 vs reference golden: {err:.3g}")
    assert ok, err


@pytest.mark.parametrize("basis", ["ptm", "hsh9", "hsh"])
@pytest.mark.parametrize("N", [16, 31, 32, 33, 100, 200])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_vs_oracle(cuda, basis, N, layout):
    k = rti.basis_terms(basis)
    if N < k:
        pytest.skip("N < k")
    lu, lv = o.synth_dirs(N, N + k)
    rng = np.random.default_rng(N * 37 + k)
    worst = 0.0
    for P in (16, 2048, 2064, 3 * 2048 + 16 * 7):
        I = rng.integers(0, 256, size=(2, N, P), dtype=np.uint8)
        coef = rti.fit(torch.as_tensor(I, device=cuda)[..., None], lu, lv, basis=basis, layout=layout,
                       kernel="h16").cpu().numpy()
        pv = np.linalg.pinv(o.design("ptm" if basis == "ptm" else "hsh", lu, lv)[:, :k])
        for c in range(2):
            got = coef[c].reshape(P, k) if layout == "pixel" else coef[c].reshape(k, P).T
            err, ok = coef_close(got, (pv @ I[c].astype(np.float64)).T)
            worst = max(worst, err)
            assert ok, (P, c, err)
    print(f"h16 {basis} N={N} {layout}: max rel {worst:.3g}")


def test_max_lights_and_extremes(cuda):
    Nmax = int(L.lib().rti_fit_shared_h16_max_lights())
    assert Nmax >= 256
    lu, lv = o.synth_dirs(Nmax, 5)
    pv = o.pinv_shared("hsh", lu, lv)
    for fill in (0, 255, None):
        I = (np.full((Nmax, 4096), fill, np.uint8) if fill is not None
             else np.random.default_rng(2).integers(0, 256, (Nmax, 4096), dtype=np.uint8))
        coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv, basis="hsh", kernel="h16").cpu().numpy()
        ref = (pv @ I.astype(np.float64)).T
        if fill == 0:
            assert not coef.any()
        else:
            err, ok = coef_close(coef, ref)
            assert ok, (fill, err)


def test_auto_is_h16_and_matches_q8(cuda):
    """AUTO on uint8 equals kernel="h16" bit for bit, and agrees with the exact-sum q8 form and the fp64 oracle."""
    lu, lv = o.synth_dirs(100, 2)
    I = torch.as_tensor(o.synth_intensities(216, 384, lu, lv, seed=3), device=cuda).round().clamp(0, 255)
    a = rti.fit(I.to(torch.uint8), lu, lv)
    assert torch.equal(a, rti.fit(I.to(torch.uint8), lu, lv, kernel="h16"))
    q = rti.fit(I.to(torch.uint8), lu, lv, kernel="q8")
    ref = o.fit_shared(I.reshape(100, -1).double().cpu().numpy(), o.pinv_shared("ptm", lu, lv)).reshape(a.shape)
    ea, ok = coef_close(a.cpu().numpy(), ref)
    eq, _ = coef_close(q.cpu().numpy(), ref)
    print(f"u8 4K-slice: h16 {ea:.3g}, q8 {eq:.3g} (max rel to fp64)")
    assert ok and ea <= 1e-5, ea


def test_tile_streams_bit_identical(cuda):
    """AUTO lets every workgroup stream several interleaved tiles through one load pipeline; the result equals
    one cold tile per workgroup (RTI_KERNEL_CHUNKS(1)), 3 tiles per workgroup, batched groups and both tile
    geometries (2048 pixels one workgroup per CU, 1024 pixels two) bit for bit (ragged P: a partial last tile
    and a short last stream, 3 channels, HSH-16 and PTM-6)."""
    for k, N in ((16, 200), (6, 100)):
        C, P = 3, 2048 * 1050 + 16 * 5
        lu, lv = o.synth_dirs(N, 4)
        pv = o.pinv_shared("hsh" if k == 16 else "ptm", lu, lv)
        op = torch.as_tensor(rti.h16_operator(pv), device=cuda)
        g = torch.Generator(device=cuda).manual_seed(5)
        I = torch.randint(0, 256, (C, N, P), generator=g, device=cuda, dtype=torch.uint8)
        outs = []
        W = L.RTI_KERNEL_TILE_WAVES_SHIFT  # geometry: 1 = 2048 px / 8 waves, 2 = 1024 px (AUTO k <= 9), 3 = 2048 / 16
        for flags in (0, 1 << L.RTI_KERNEL_CHUNKS_SHIFT, 3 << L.RTI_KERNEL_CHUNKS_SHIFT,
                      4 << L.RTI_KERNEL_TILE_DEPTH_SHIFT, 8 << L.RTI_KERNEL_TILE_DEPTH_SHIFT,  # batched groups
                      1 << W, 2 << W, (2 << W) | (1 << L.RTI_KERNEL_CHUNKS_SHIFT), (1 << W) | (3 << L.RTI_KERNEL_CHUNKS_SHIFT),
                      3 << W, (3 << W) | (3 << L.RTI_KERNEL_CHUNKS_SHIFT)):  # 3: 2048 pixels on 16 waves (r05)
            coef = torch.full((C, P, k), float("nan"), device=cuda)
            rti.api.fit_h16_into(op, I, coef, k=k, flags=flags)
            outs.append(coef)
        a = outs[0]
        assert not torch.isnan(a).any() and all(torch.equal(a, b) for b in outs[1:])
        idx = torch.as_tensor(np.unique(np.r_[np.random.default_rng(1).integers(0, P, 512), 0, P - 1]), device=cuda)
        for c in range(C):
            err, ok = coef_close(a[c][idx].cpu().numpy(), (pv @ I[c][:, idx].double().cpu().numpy()).T)
            assert ok, (k, c, err)


def test_fallbacks_keep_reference_semantics(cuda):
    """Where h16 does not apply rti.fit keeps the fp32 stream: P % 16 != 0, N above the LDS limit, and an
    exactly rank-deficient light set (NaN like the reference; the h16 operator refuses non-finite weights)."""
    e = golden("ptm_edge.npz")
    I = torch.as_tensor(np.tile(e["singular_I"].astype(np.uint8)[:, None], (1, 64)), device=cuda)
    assert torch.isnan(rti.fit(I, e["singular_lu"], e["singular_lv"])).all()
    with pytest.raises(NotImplementedError):
        rti.fit(I, e["singular_lu"], e["singular_lv"], kernel="h16")
    lu, lv = o.synth_dirs(30, 1)
    I = np.random.default_rng(0).integers(0, 256, (30, 37), dtype=np.uint8)  # P % 16 != 0
    coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv).cpu().numpy()
    err, ok = coef_close(coef, o.fit_shared(I.astype(np.float64), o.pinv_shared("ptm", lu, lv)))
    assert ok, err
    Nbig = int(L.lib().rti_fit_shared_h16_max_lights()) + 1
    lu, lv = o.synth_dirs(Nbig, 2)
    I = np.random.default_rng(1).integers(0, 256, (Nbig, 64), dtype=np.uint8)
    coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv).cpu().numpy()
    err, ok = coef_close(coef, o.fit_shared(I.astype(np.float64), o.pinv_shared("ptm", lu, lv)))
    assert ok, err


def test_abi_errors(cuda):
    lib = L.lib()
    lu, lv = o.synth_dirs(20, 1)
    op = torch.as_tensor(rti.h16_operator(o.pinv_shared("ptm", lu, lv)), device=cuda)
    I = torch.zeros((20, 48), dtype=torch.uint8, device=cuda)
    coef = torch.empty((48, 6), device=cuda)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
    assert lib.rti_fit_shared_h16(vp(op), 7, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_UNSUPPORTED
    assert lib.rti_fit_shared_h16(vp(op), 6, 20, vp(I), 40, 1, 40, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_UNSUPPORTED
    assert lib.rti_fit_shared_h16(vp(op), 6, 5, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_BAD_ARG
    assert lib.rti_fit_shared_h16(None, 6, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_BAD_ARG
    assert lib.rti_fit_shared_h16(vp(op), 6, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_OK
    with pytest.raises(ValueError):
        rti.h16_operator(np.full((6, 20), np.nan))


@pytest.mark.parametrize("basis", ["ptm", "hsh9", "hsh"])
def test_geometries_at_max_lights(cuda, basis):
    """At the largest N the LDS takes, the 1024-pixel tile (forced: one workgroup per CU fits there, two do
    not) and the 2048-pixel tile give the same bits as AUTO, with a partial last tile of each geometry."""
    Nmax = int(L.lib().rti_fit_shared_h16_max_lights())
    k = rti.basis_terms(basis)
    lu, lv = o.synth_dirs(Nmax, 6)
    pv = np.linalg.pinv(o.design("ptm" if basis == "ptm" else "hsh", lu, lv)[:, :k])  # HSH-9: the first 9 terms
    op = torch.as_tensor(rti.h16_operator(pv), device=cuda)
    P = 2048 * 3 + 1024 + 48
    I = torch.randint(0, 256, (Nmax, P), generator=torch.Generator(device=cuda).manual_seed(7), device=cuda,
                      dtype=torch.uint8)
    outs = []
    for geom in (0, 1, 2, 3):
        coef = torch.full((1, P, k), float("nan"), device=cuda)
        rti.api.fit_h16_into(op, I, coef, k=k, flags=geom << L.RTI_KERNEL_TILE_WAVES_SHIFT)
        outs.append(coef)
    assert not torch.isnan(outs[0]).any() and all(torch.equal(outs[0], c) for c in outs[1:])
    err, ok = coef_close(outs[0][0].cpu().numpy(), (pv @ I.double().cpu().numpy()).T)
    assert ok, err
