"""GPU parity of the per-pixel fit residual (rti_fit_residual) against the oracle.

The residual is compared on the GPU's own coefficients (cast to fp64), so the test
isolates the residual kernel's fp32 arithmetic.  Tolerance: per pixel
|res − res_ref| <= 1e-3 + 1e-4·res_ref (intensity units; the prediction Σ A·c ≈ 255
carries ≈1e-5 fp32 rounding per term), channel RMS to the same 1e-3 + 1e-4 relative."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import golden

pytestmark = pytest.mark.gpu


def to_dev(a, dev, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dev, dtype)


def check(res, rms, I_np, A, coef_np):
    ref, ss = o.fit_residual(I_np, A, coef_np)
    got = res.cpu().numpy().reshape(-1)
    assert np.all(np.abs(got - ref) <= 1e-3 + 1e-4 * ref), np.abs(got - ref).max()
    ref_rms = np.sqrt(ss / I_np.size)
    assert abs(float(rms) - ref_rms) <= 1e-4 * ref_rms + 1e-3, (float(rms), ref_rms)


@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8, torch.int32])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_golden_stack(cuda, in_dtype, layout):
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"]).to(cuda).to(in_dtype)
    coef = rti.fit(I, d["lu"], d["lv"], layout=layout)
    res, rms = rti.fit_residual(I, coef, d["lu"], d["lv"], layout=layout)
    assert res.shape == I.shape[1:]
    c = coef.cpu().numpy()
    c = np.moveaxis(c, 0, -1) if layout == "planar" else c
    check(res, rms, np.asarray(d["I"], np.float64).reshape(I.shape[0], -1), o.design("ptm", d["lu"], d["lv"]),
          c.reshape(-1, 6))


@pytest.mark.parametrize("hw,n", [((1, 1), 6), ((3, 5), 7), ((17, 33), 13), ((64, 65), 37), ((8, 8), 200)])
def test_ragged_shapes(cuda, hw, n):
    h, w = hw
    lu, lv = o.synth_dirs(n, n)
    I = o.synth_intensities(h, w, lu, lv, seed=h * 1000 + w)
    Id = to_dev(I, cuda)
    coef = rti.fit(Id, lu, lv)
    res, rms = rti.fit_residual(Id, coef, lu, lv)
    check(res, rms, I.reshape(n, -1), o.design("ptm", lu, lv), coef.cpu().numpy().reshape(-1, 6))


def test_rgb_hsh16(cuda):
    n, h, w = 40, 24, 36
    lu, lv = o.synth_dirs(n, 7)
    I = np.stack([o.synth_intensities(h, w, lu, lv, seed=s, basis="hsh") for s in range(3)])
    Id = to_dev(I, cuda)
    coef = rti.fit(Id, lu, lv, basis="hsh")
    res, rms = rti.fit_residual(Id, coef, lu, lv, basis="hsh")
    assert res.shape == (3, h, w) and rms.shape == (3,)
    A = o.design("hsh", lu, lv)
    for c in range(3):
        check(res[c], rms[c], I[c].reshape(n, -1), A, coef[c].cpu().numpy().reshape(-1, 16))


def test_noise_free_is_zero_and_noise_level(cuda):
    """Exact basis data leaves no residual; i.i.d. N(0, σ²) noise leaves RMS ≈ σ·sqrt((N−k)/N)."""
    n, h, w, sigma = 64, 64, 64, 3.0
    lu, lv = o.synth_dirs(n, 11)
    a = o.synth_coef_fields(h, w, 11).reshape(-1, 6)
    I = (o.design("ptm", lu, lv) @ a.T).astype(np.float32)  # [N, P]
    Id = to_dev(I, cuda)
    res, rms = rti.fit_residual(Id, rti.fit(Id, lu, lv), lu, lv)
    assert res.abs().max().item() < 2e-3 and float(rms) < 1e-3
    noise = np.random.default_rng(0).normal(0, sigma, I.shape).astype(np.float32)
    Id = to_dev(I + noise, cuda)
    res, rms = rti.fit_residual(Id, rti.fit(Id, lu, lv), lu, lv)
    expect = sigma * np.sqrt((n - 6) / n)
    assert abs(float(rms) - expect) < 0.02 * expect


def test_bad_args(cuda):
    lu, lv = o.synth_dirs(10, 1)
    I = torch.zeros((10, 4, 4), device=cuda)
    coef = rti.fit(I, lu, lv)
    with pytest.raises(ValueError):
        rti.fit_residual(I, coef[..., :5].contiguous(), lu, lv)
    with pytest.raises(ValueError):
        rti.fit_residual(I, coef, lu[:9], lv[:9])
    with pytest.raises(ValueError):
        rti.fit_residual(I.cpu(), coef, lu, lv)


def test_full_size_4k_n100(cuda):
    """BASELINE configs[2] size, through size-independent properties: exact basis data
    leaves ≈0 everywhere; with N(0, 2²) noise the channel RMS equals sqrt(mean(res²)) and
    2·sqrt((N−k)/N)."""
    n, h, w = 100, 2160, 3840
    lu, lv = o.synth_dirs(n, 2)
    A = torch.as_tensor(o.design("ptm", lu, lv).astype(np.float32), device=cuda)
    a = torch.rand((h * w, 6), device=cuda) * 60.0
    I = torch.zeros((n, h * w), device=cuda)
    for i in range(6):
        I.addcmul_(A[:, i:i + 1], a[:, i].unsqueeze(0))  # element-wise: no library GEMM
    coef = rti.fit(I, lu, lv)
    res, rms = rti.fit_residual(I, coef, lu, lv)
    assert res.abs().max().item() < 5e-3
    I += torch.randn_like(I) * 2.0
    coef = rti.fit(I, lu, lv)
    res, rms = rti.fit_residual(I, coef, lu, lv)
    mean_sq = torch.mean(res.double() ** 2).item()
    assert abs(float(rms) ** 2 - mean_sq) <= 1e-6 * mean_sq
    expect = 2.0 * np.sqrt((n - 6) / n)
    assert abs(float(rms) - expect) < 0.01 * expect


def test_custom_op_matches_api(cuda):
    from rti import ops  # noqa: F401  registers torch.ops.rti.*
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"]).to(cuda).to(torch.float32)
    coef = rti.fit(I, d["lu"], d["lv"])
    res, _ = rti.fit_residual(I, coef, d["lu"], d["lv"])
    A = torch.as_tensor(rti.design_matrix(d["lu"], d["lv"]).astype(np.float32), device=cuda)
    N = I.shape[0]
    got = torch.ops.rti.fit_residual(A, I.reshape(N, -1), coef.reshape(-1, 6))
    assert torch.equal(got, res.reshape(-1))


@pytest.mark.parametrize("layout", ["pixel", "planar"])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.uint8])
def test_wide_lane_path_ragged(cuda, layout, in_dtype):
    """The PTM-6 4-chunks-per-lane residual path (taken when P·C >= 2.048 M) with a ragged pixel
    count (P % 4096 != 0: a partial last wave whose lanes hold only some chunks), 3 channels,
    both coefficient layouts, 8-bit and fp32 stacks — per pixel against the oracle."""
    n, C, P = 12, 3, 700001 * 4
    lu, lv = o.synth_dirs(n, 41)
    g = torch.Generator(device=cuda).manual_seed(5)
    I = torch.randint(0, 256, (C, n, P), generator=g, device=cuda).to(in_dtype)
    coef = rti.fit(I.reshape(C, n, P // 4, 4), lu, lv, layout=layout)
    res, rms = rti.fit_residual(I.reshape(C, n, P // 4, 4), coef, lu, lv, layout=layout)
    A = o.design("ptm", lu, lv)
    idx = np.concatenate([np.arange(4096), np.arange(P - 8192, P)])  # the start and the ragged tail
    for c in range(C):
        cc = coef[c].reshape(P, 6) if layout == "pixel" else coef[c].reshape(6, P).T
        Ic = I[c][:, idx].double().cpu().numpy()
        ref, _ = o.fit_residual(Ic, A, cc[idx].cpu().numpy())
        got = res[c].reshape(P)[idx].cpu().numpy()
        assert np.all(np.abs(got - ref) <= 1e-3 + 1e-4 * ref), (c, np.abs(got - ref).max())
        _, ss = o.fit_residual(I[c].double().cpu().numpy(), A, cc.cpu().numpy())
        ref_rms = np.sqrt(ss / (n * P))
        assert abs(float(rms[c]) - ref_rms) <= 1e-4 * ref_rms + 1e-3, (c, float(rms[c]), ref_rms)
