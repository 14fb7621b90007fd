"""GPU parity of the one-pass fit + residual kernel (rti_fit_shared_residual_svd, the form
rti.fit_with_residual uses; the Gram form rti_fit_shared_residual in the generations test and
test_gpu_edge_solvers.py) against the oracle and the reference's golden coefficients.

The kernel accumulates Uᵀ I and ‖I‖² in fp64, so its coefficients
are held to 1e-6 of max_k |c_ref| per pixel (100× inside the SURVEY §8(c) 1e-4 bar) and its
residuals — of the exact least-squares solution, compared with oracle.fit_residual evaluated on
the fp64 reference coefficients — to |res − res_ref| <= 1e-4 + 1e-6·res_ref (intensity units)."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden

pytestmark = pytest.mark.gpu


def to_dev(a, dev, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dev, dtype)


def check(coef, res, rms, I_np, basis, lu, lv, k, ctol=1e-6):
    """coef [P, k] fp32, res [P], I_np [N, P] -> asserts against the fp64 oracle."""
    A = o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k]
    ref_c = (np.linalg.pinv(A) @ np.asarray(I_np, np.float64)).T
    err, ok = coef_close(np.asarray(coef), ref_c, rtol=ctol)
    assert ok, ("coef", err)
    ref_r, ss = o.fit_residual(I_np, A, ref_c)
    got = np.asarray(res).reshape(-1)
    bad = np.abs(got - ref_r) > 1e-4 + 1e-6 * ref_r
    assert not bad.any(), ("res", np.abs(got - ref_r).max())
    if rms is not None:
        ref_rms = np.sqrt(ss / I_np.size)
        assert abs(float(rms) - ref_rms) <= 1e-9 * ref_rms + 1e-9, (float(rms), ref_rms)


@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8, torch.int32])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_golden_256x256_N20(cuda, in_dtype, layout):
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"]).to(cuda).to(in_dtype)
    coef, res, rms = rti.fit_with_residual(I, d["lu"], d["lv"], layout=layout)
    c = coef.cpu().numpy()
    c = np.moveaxis(c, 0, -1) if layout == "planar" else c
    err, ok = coef_close(c, d["coef"], rtol=1e-6)  # the reference's own coefficients (analysis.py:293-298)
    assert ok, err
    check(c.reshape(-1, 6), res.cpu().numpy(), rms, np.asarray(d["I"], np.float64).reshape(20, -1), "ptm",
          d["lu"], d["lv"], 6)


@pytest.mark.parametrize("chunks", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("basis,n", [("ptm", 23), ("hsh9", 17), ("hsh", 29)])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8])
def test_chunks_ragged(cuda, chunks, basis, n, in_dtype):
    """Every chunks-per-lane variant over pixel counts around whole-wave multiples (partial last
    wave, lanes with only some chunks in range, P % 4 != 0 -> one-pixel lanes), 2 channels, both
    coefficient layouts."""
    k = rti.basis_terms(basis)
    lu, lv = o.synth_dirs(n, 31)
    wave_px = 64 * 4 * max(chunks, 1)
    for P in (3, 4, wave_px - 4, wave_px + 4, 3 * wave_px + 260, 5 * wave_px + 1024 * 3 + 8, 4099):
        rng = np.random.default_rng(P + n)
        I = rng.integers(0, 256, size=(2, n, P)).astype(np.float32)
        Id = torch.as_tensor(I, device=cuda).to(in_dtype)[..., None]  # [C, N, P, 1]
        for layout in ("pixel", "planar"):
            coef, res, rms = rti.fit_with_residual(Id, lu, lv, basis=basis, layout=layout, chunks=chunks)
            for c in range(2):
                cc = coef[c].cpu().numpy()
                cc = cc.reshape(P, k) if layout == "pixel" else cc.reshape(k, P).T
                check(cc, res[c].cpu().numpy(), rms[c], I[c], basis, lu, lv, k)


def test_exact_data_zero_residual_and_noise_level(cuda):
    n, h, w, sigma = 64, 64, 64, 3.0
    lu, lv = o.synth_dirs(n, 11)
    a = o.synth_coef_fields(h, w, 11).reshape(-1, 6)
    I = (o.design("ptm", lu, lv) @ a.T).astype(np.float32)  # [N, P]
    coef, res, rms = rti.fit_with_residual(to_dev(I, cuda), lu, lv)
    assert res.abs().max().item() < 1e-4 and float(rms) < 1e-5
    noise = np.random.default_rng(0).normal(0, sigma, I.shape).astype(np.float32)
    coef, res, rms = rti.fit_with_residual(to_dev(I + noise, cuda), lu, lv)
    expect = sigma * np.sqrt((n - 6) / n)
    assert abs(float(rms) - expect) < 0.02 * expect


def test_rank_deficient_and_rcond(cuda):
    e = golden("ptm_edge.npz")
    I = to_dev(np.tile(e["singular_I"].astype(np.float32)[:, None], (1, 64)), cuda)
    coef, _, _ = rti.fit_with_residual(I, e["singular_lu"], e["singular_lv"])
    assert not np.isfinite(coef.cpu().numpy()).all()  # the reference divides by a zero singular value
    coef, res, _ = rti.fit_with_residual(I, e["singular_lu"], e["singular_lv"], rcond=1e-10)
    ref = o.fit_shared(np.tile(e["singular_I"].astype(np.float64)[:, None], (1, 64)),
                       o.pinv_shared("ptm", e["singular_lu"], e["singular_lv"], rcond=1e-10))
    err, ok = coef_close(coef.cpu().numpy(), ref, rtol=1e-6)
    assert ok, err
    assert np.isfinite(res.cpu().numpy()).all()


def test_matches_two_pass(cuda):
    """One pass vs rti_fit_shared + rti_fit_residual on the same stack."""
    lu, lv = o.synth_dirs(40, 4)
    I = to_dev(o.synth_intensities(96, 80, lu, lv, seed=2), cuda)
    coef1, res1, rms1 = rti.fit_with_residual(I, lu, lv)
    coef2 = rti.fit(I, lu, lv)
    res2, rms2 = rti.fit_residual(I, coef2, lu, lv)
    err, ok = coef_close(coef1.cpu().numpy(), coef2.cpu().numpy())
    assert ok, err
    assert torch.allclose(res1, res2, atol=1e-3, rtol=1e-4)
    assert abs(float(rms1) - float(rms2)) < 1e-4 * float(rms2)


def test_bad_args(cuda):
    lu, lv = o.synth_dirs(10, 1)
    with pytest.raises(ValueError):
        rti.fit_with_residual(torch.zeros((5, 4, 4), device=cuda), lu[:5], lv[:5])
    with pytest.raises(ValueError):
        rti.fit_with_residual(torch.zeros((10, 4, 4), device=cuda), lu[:9], lv[:9])
    with pytest.raises(ValueError):
        rti.fit_with_residual(torch.zeros((10, 4, 4)), lu, lv)
    with pytest.raises(ValueError):
        rti.fit_with_residual(torch.zeros((10, 4, 4), device=cuda, dtype=torch.float64), lu, lv)


@pytest.mark.slow
def test_full_size_4k_n100(cuda):
    """BASELINE configs[2] size: sampled fp64 parity of coefficients and residuals, exact-data
    recovery, and the noise level of the workgroup residual energy."""
    n, h, w = 100, 2160, 3840
    P = h * w
    lu, lv = o.synth_dirs(n, 2)
    A = o.design("ptm", lu, lv)
    g = torch.Generator(device=cuda).manual_seed(1)
    a = torch.rand((6, P), generator=g, device=cuda) * 100 - 50
    I = torch.zeros((n, P), device=cuda)
    for j in range(6):
        for i in range(n):
            I[i].add_(a[j], alpha=float(A[i, j]))  # element-wise: no library GEMM
    coef, res, rms = rti.fit_with_residual(I, lu, lv, layout="planar")
    assert res.max().item() < 1e-3
    I.add_(torch.randn(I.shape, generator=g, device=cuda) * 2.0).round_()
    coef, res, rms = rti.fit_with_residual(I, lu, lv, layout="planar")
    idx = torch.randint(0, P, (4096,), generator=g, device=cuda)
    check(coef[:, idx].T.cpu().numpy(), res[idx].cpu().numpy(), None, I[:, idx].double().cpu().numpy(), "ptm", lu,
          lv, 6)
    mean_sq = torch.mean(res.double() ** 2).item()
    assert abs(float(rms) ** 2 - mean_sq) <= 1e-6 * mean_sq
    expect = np.sqrt(4.0 + 1.0 / 12.0) * np.sqrt((n - 6) / n)  # N(0, 2²) noise + rounding
    assert abs(float(rms) - expect) < 0.02 * expect


@pytest.mark.parametrize("form", ["svd", "gram"])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_launch_generations_bit_identical(cuda, layout, form):
    """AUTO issues a large fit + residual call as consecutive launches over pixel ranges of whole
    workgroups (launch generations, rti_fitres.hip); coefficients, residuals and the per-workgroup
    residual energies must equal RTI_KERNEL_ONE_LAUNCH's bit for bit, over a ragged pixel count and 2
    channels, and match the fp64 oracle on sampled pixels.  Both runs pin 3 chunks per lane: the slot
    layout of partial[] follows the chunks per lane, which AUTO picks from the CU count."""
    import ctypes

    from rti import _lib as L

    H, W, N, C, k = 2150, 2100, 100, 2, 6  # P = 4 515 000: 3 chunks per lane, 3 launches per channel
    P = H * W
    lu, lv = o.synth_dirs(N, 9)
    g = torch.Generator(device=cuda).manual_seed(11)
    I = torch.randint(0, 256, (C, N, P), generator=g, device=cuda).to(torch.float32)
    if form == "gram":
        A64 = torch.as_tensor(rti.design_matrix(lu, lv, "ptm"), device=cuda).contiguous()
        G = torch.as_tensor(rti.gram_inverse(lu, lv, "ptm"), device=cuda).contiguous()
        fn = L.lib().rti_fit_shared_residual
    else:
        U, Wf = rti.lsq_factors(lu, lv, "ptm")
        A64 = torch.as_tensor(U, device=cuda).contiguous()
        G = torch.as_tensor(Wf, device=cuda).contiguous()
        fn = L.lib().rti_fit_shared_residual_svd
    lib = L.lib()
    nb = int(lib.rti_fit_shared_residual_blocks(P))
    s = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    outs = []
    for flags in (0, L.RTI_KERNEL_ONE_LAUNCH):
        coef = torch.full((C, P, k) if layout == "pixel" else (C, k, P), float("nan"), device=cuda)
        res = torch.full((C, P), float("nan"), device=cuda)
        part = torch.zeros((C, nb), dtype=torch.float64, device=cuda)
        st = fn(vp(A64), vp(G), k, N, vp(I), L.RTI_F32, P, C, P, N * P, vp(coef), rti.api._layout_id(layout), P * k,
                vp(res), vp(part), flags | (3 << L.RTI_KERNEL_CHUNKS_SHIFT), s)
        L.check(st, "rti_fit_shared_residual")
        outs.append((coef, res, part, int(lib.rti_last_launch_count())))
    torch.cuda.synchronize()
    (ca, ra, pa, la), (cb, rb, pb, lb) = outs
    assert la > 1 and lb == 1, (la, lb)
    assert not torch.isnan(ca).any() and not torch.isnan(ra).any()
    assert torch.equal(ca, cb) and torch.equal(ra, rb) and torch.equal(pa, pb)
    px = np.unique(np.concatenate([np.random.default_rng(3).integers(0, P, 256), [0, P - 1, P // 3, P // 3 - 1]]))
    idx = torch.as_tensor(px, device=cuda)
    for c in range(C):
        cc = ca[c][idx] if layout == "pixel" else ca[c][:, idx].T
        check(cc.cpu().numpy(), ra[c][idx].cpu().numpy(), None, I[c][:, idx].double().cpu().numpy(), "ptm", lu, lv, k)


@pytest.mark.parametrize("planar", [False, True])
def test_torch_op_fit_shared_residual(cuda, planar):
    """torch.ops.rti.fit_shared_residual(U, W, I) -> (coef, res, partial): the same call as
    rti.fit_with_residual, against the reference's golden coefficients and the fp64 oracle, plus the
    fake-tensor registration (torch.library.opcheck: schema, fake vs real shapes/dtypes)."""
    from rti import ops  # noqa: F401  registers torch.ops.rti.*

    d = golden("ptm_shared_256x256_N20.npz")
    N = 20
    I = torch.as_tensor(d["I"], device=cuda).to(torch.float32).reshape(N, -1)
    U, W = (torch.as_tensor(a, device=cuda) for a in rti.lsq_factors(d["lu"], d["lv"]))
    coef, res, partial = torch.ops.rti.fit_shared_residual(U, W, I, planar)
    c = coef.T.cpu().numpy() if planar else coef.cpu().numpy()
    err, ok = coef_close(c.reshape(d["coef"].shape), d["coef"], rtol=1e-6)  # analysis.py:293-298
    assert ok, err
    c2, r2, rms2 = rti.fit_with_residual(I, d["lu"], d["lv"], layout="planar" if planar else "pixel")
    assert torch.equal(coef, c2) and torch.equal(res, r2)
    P = I.shape[1]
    assert partial.shape == (int(rti._lib.lib().rti_fit_shared_residual_blocks(P)),)
    assert abs(float(torch.sqrt(partial.sum() / (P * N))) - float(rms2)) <= 1e-12 * float(rms2)
    check(c, res.cpu().numpy(), float(rms2), np.asarray(d["I"], np.float64).reshape(N, -1), "ptm", d["lu"], d["lv"], 6)
    # 3-D (channels) form and the fake kernel
    I3 = torch.stack([I, I.flip(1)])
    coef3, res3, part3 = torch.ops.rti.fit_shared_residual(U, W, I3, planar)
    assert torch.equal(coef3[0], coef) and torch.equal(res3[0], res)
    torch.library.opcheck(torch.ops.rti.fit_shared_residual.default, (U, W, I3, planar, 0),
                          test_utils=("test_schema", "test_faketensor"))
    with pytest.raises(ValueError):
        torch.ops.rti.fit_shared_residual(U.float(), W, I, planar)
