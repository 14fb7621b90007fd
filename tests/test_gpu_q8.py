"""GPU parity of the 8-bit fit on the int8 matrix cores (rti_fit_shared_q8, rti.fit(kernel="q8"); AUTO for
uint8 stacks is the split-fp16 form, tests/test_gpu_h16.py): the reference's golden coefficients, the fp64 oracle over every supported basis, light counts
around the 64-light steps and the LDS limit, ragged pixel counts (partial tiles), two channels, both
layouts, launch generations, and the fallbacks (fp32 path) where q8 does not apply.

Tolerance: the q8 operator's quantization bound is 2^-28·max_n|pinv|·Σ_n I_n (rti_q8.h), far below fp32
rounding; coefficients are held to 1e-6 of max_k |c_ref,k| per pixel (the fp32 stream's bar is 1e-4)."""
import ctypes

import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden
from rti import _lib as L

pytestmark = pytest.mark.gpu


def fit_u8(I_np, lu, lv, basis, cuda, **kw):
    return rti.fit(torch.as_tensor(I_np, device=cuda), lu, lv, basis=basis, **kw)


def q8_close(got, pv, I):
    """The q8 contract (rti_q8.h): |c_i − (pinv·I)_i| <= 2^-28·max_n|pinv_in|·Σ_n I_n + one fp32 rounding.
    got [P, k], pv [k, N] fp64, I [N, P] -> max error relative to max_k |c_ref,k| (reported)."""
    ref = (pv @ I.astype(np.float64)).T
    bound = 2.0 ** -28 * np.abs(pv).max(1)[None, :] * I.sum(0).astype(np.float64)[:, None] + 2.0 ** -24 * np.abs(ref)
    diff = np.abs(np.asarray(got, np.float64) - ref)
    assert (diff <= bound * 1.001 + 1e-30).all(), float((diff / (bound + 1e-30)).max())
    return float((diff / np.maximum(np.abs(ref).max(-1, keepdims=True), 1e-30)).max())


def test_golden_256x256_N20(cuda):
    d = golden("ptm_shared_256x256_N20.npz")
    I = np.asarray(d["I"]).astype(np.uint8)
    assert np.array_equal(I, d["I"])  # the golden stack is integer 0..255
    coef = fit_u8(I, d["lu"], d["lv"], "ptm", cuda, kernel="q8").cpu().numpy()
    err, ok = coef_close(coef, d["coef"], rtol=1e-6)  # the reference's own coefficients (analysis.py:293-298)
    print(f"q8 vs reference golden: {err:.3g}")
    assert ok, err


@pytest.mark.parametrize("basis", ["ptm", "hsh9", "hsh"])
@pytest.mark.parametrize("N", [16, 63, 64, 65, 100, 200])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_vs_oracle(cuda, basis, N, layout):
    k = rti.basis_terms(basis)
    if N < k:
        pytest.skip("N < k")
    lu, lv = o.synth_dirs(N, N + k)
    rng = np.random.default_rng(N * 31 + k)
    for P in (16, 1024, 1040, 3 * 1024 + 16 * 7):
        I = rng.integers(0, 256, size=(2, N, P), dtype=np.uint8)
        coef = rti.fit(torch.as_tensor(I, device=cuda)[..., None], lu, lv, basis=basis, layout=layout,
                       kernel="q8").cpu().numpy()
        pv = np.linalg.pinv(o.design("ptm" if basis == "ptm" else "hsh", lu, lv)[:, :k])
        for c in range(2):
            got = coef[c].reshape(P, k) if layout == "pixel" else coef[c].reshape(k, P).T
            err = q8_close(got, pv, I[c])  # the documented quantization bound, per coefficient
            assert err <= (1e-6 if N > k else 1e-5), (P, c, err)  # N = k: a square, less well-conditioned solve


def test_max_lights_and_extremes(cuda):
    Nmax = int(L.lib().rti_fit_shared_q8_max_lights())
    assert Nmax >= 256
    lu, lv = o.synth_dirs(Nmax, 5)
    pv = o.pinv_shared("hsh", lu, lv)
    for fill in (0, 255, None):
        I = (np.full((Nmax, 2048), fill, np.uint8) if fill is not None
             else np.random.default_rng(2).integers(0, 256, (Nmax, 2048), dtype=np.uint8))
        coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv, basis="hsh", kernel="q8").cpu().numpy()
        ref = (pv @ I.astype(np.float64)).T
        if fill == 0:
            assert not coef.any()
        else:
            err, ok = coef_close(coef, ref, rtol=1e-6)
            assert ok, (fill, err)


def test_q8_matches_fp32_stream_and_is_used(cuda):
    """kernel="q8" on uint8 runs rti_fit_shared_q8 and agrees with the fp32 stream on the same stack within the
    fp32 stream's own rounding, and is closer to fp64 than it."""
    lu, lv = o.synth_dirs(100, 2)
    I = torch.as_tensor(o.synth_intensities(216, 384, lu, lv, seed=3), device=cuda).round().clamp(0, 255)
    a = rti.fit(I.to(torch.uint8), lu, lv, kernel="q8")
    b = rti.fit(I.to(torch.uint8), lu, lv, kernel="valu")
    c = rti.fit(I, lu, lv)
    err, ok = coef_close(a.cpu().numpy(), c.cpu().numpy(), rtol=1e-5)
    assert ok, err
    assert torch.equal(b, rti.fit(I.to(torch.uint8), lu, lv, kernel="valu"))
    ref = o.fit_shared(I.reshape(100, -1).double().cpu().numpy(), o.pinv_shared("ptm", lu, lv)).reshape(a.shape)
    ea, _ = coef_close(a.cpu().numpy(), ref)
    eb, _ = coef_close(b.cpu().numpy(), ref)
    print(f"u8 4K-slice: q8 {ea:.3g} vs fp32 VALU stream {eb:.3g} (max rel to fp64)")
    assert ea <= 1e-6 and ea <= eb


def test_tile_streams_bit_identical(cuda):
    """AUTO lets every workgroup stream several consecutive 1024-pixel tiles through one load pipeline; the
    result equals one cold tile per workgroup (RTI_KERNEL_CHUNKS(1)) and 3 tiles per workgroup bit for bit
    (ragged P: a partial last tile and a short last stream, 3 channels, HSH-16 and PTM-6)."""
    for k, N in ((16, 200), (6, 100)):
        C, P = 3, 1024 * 2100 + 16 * 5
        lu, lv = o.synth_dirs(N, 4)
        pv = o.pinv_shared("hsh" if k == 16 else "ptm", lu, lv)
        op = torch.as_tensor(rti.q8_operator(pv), device=cuda)
        g = torch.Generator(device=cuda).manual_seed(5)
        I = torch.randint(0, 256, (C, N, P), generator=g, device=cuda, dtype=torch.uint8)
        outs = []
        for flags in (0, 1 << L.RTI_KERNEL_CHUNKS_SHIFT, 3 << L.RTI_KERNEL_CHUNKS_SHIFT,
                      L.RTI_KERNEL_STAGE, L.RTI_KERNEL_STAGE | (2 << L.RTI_KERNEL_TILE_DEPTH_SHIFT)):
            coef = torch.full((C, P, k), float("nan"), device=cuda)
            rti.api.fit_q8_into(op, I, coef, k=k, flags=flags)
            outs.append(coef)
        a = outs[0]
        # (+ the LDS-staged pixel-major stores, and 2 launch generations of them: the same values)
        assert not torch.isnan(a).any() and all(torch.equal(a, b) for b in outs[1:])
        idx = torch.as_tensor(np.unique(np.r_[np.random.default_rng(1).integers(0, P, 512), 0, P - 1]), device=cuda)
        for c in range(C):
            err = q8_close(a[c][idx].cpu().numpy(), pv, I[c][:, idx].cpu().numpy())
            assert err <= 1e-6, (k, c, err)


def test_fallbacks_keep_reference_semantics(cuda):
    """Where q8 does not apply rti.fit keeps the fp32 stream: P % 16 != 0, N above the LDS limit, and an
    exactly rank-deficient light set (NaN like the reference; the q8 operator refuses non-finite weights)."""
    e = golden("ptm_edge.npz")
    I = torch.as_tensor(np.tile(e["singular_I"].astype(np.uint8)[:, None], (1, 64)), device=cuda)
    assert torch.isnan(rti.fit(I, e["singular_lu"], e["singular_lv"])).all()
    with pytest.raises(NotImplementedError):
        rti.fit(I, e["singular_lu"], e["singular_lv"], kernel="q8")
    lu, lv = o.synth_dirs(30, 1)
    I = np.random.default_rng(0).integers(0, 256, (30, 37), dtype=np.uint8)  # P % 16 != 0
    coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv).cpu().numpy()
    err, ok = coef_close(coef, o.fit_shared(I.astype(np.float64), o.pinv_shared("ptm", lu, lv)))
    assert ok, err
    Nbig = int(L.lib().rti_fit_shared_q8_max_lights()) + 1
    lu, lv = o.synth_dirs(Nbig, 2)
    I = np.random.default_rng(1).integers(0, 256, (Nbig, 64), dtype=np.uint8)
    coef = rti.fit(torch.as_tensor(I, device=cuda), lu, lv).cpu().numpy()
    err, ok = coef_close(coef, o.fit_shared(I.astype(np.float64), o.pinv_shared("ptm", lu, lv)))
    assert ok, err


def test_abi_errors(cuda):
    lib = L.lib()
    lu, lv = o.synth_dirs(20, 1)
    op = torch.as_tensor(rti.q8_operator(o.pinv_shared("ptm", lu, lv)), device=cuda)
    I = torch.zeros((20, 48), dtype=torch.uint8, device=cuda)
    coef = torch.empty((48, 6), device=cuda)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
    assert lib.rti_fit_shared_q8(vp(op), 7, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_UNSUPPORTED
    assert lib.rti_fit_shared_q8(vp(op), 6, 20, vp(I), 40, 1, 40, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_UNSUPPORTED
    assert lib.rti_fit_shared_q8(vp(op), 6, 5, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_BAD_ARG
    assert lib.rti_fit_shared_q8(None, 6, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_ERR_BAD_ARG
    assert lib.rti_fit_shared_q8(vp(op), 6, 20, vp(I), 48, 1, 48, 0, vp(coef), 0, 0, 0, s) == L.RTI_OK
