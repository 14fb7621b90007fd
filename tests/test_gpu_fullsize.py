"""GPU parity at the full BASELINE.json sizes, through size-independent properties plus sampled
fp64 oracle checks (the oracle cannot fit a whole 4K stack in seconds):

  configs[1]  1920×1080 px × 50 lights PTM-6, AUTO kernel (4 chunks per lane)
  configs[3]  3840×2160 RGB × 200 lights HSH-16, AUTO LDS-tiled MFMA kernel: 4.98e9 stack
              elements, so channel 2 sits past 2^31 elements (64-bit offsets)
  configs[4]  4K PTM-6 maps × 1000 (lu, lv) evaluations, fp32 / int32 / uint8 outputs

configs[2] (4K × 100 PTM) is test_gpu_fit.py::test_full_size_4k_n100_properties.  Tolerances are
SURVEY §8(c): coefficients |Δ| <= 1e-4·max_k|c_ref|, relight |Δ| <= 1e-4·max(|L_ref|, 255)."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def basis_stack(a, B, dtype=torch.float32):
    """I[N, P] = B[N, k] · a[k, P], element-wise on the device (no library GEMM)."""
    N, k = B.shape
    I = torch.zeros((N, a.shape[1]), device=a.device, dtype=dtype)
    for n in range(N):
        for j in range(k):
            I[n].add_(a[j], alpha=float(B[n, j]))
    return I


def smooth_fields(k, H, W, dev, seed, const_col, base, amp, side):
    g = torch.Generator(device=dev).manual_seed(seed)
    yy = torch.linspace(0, 1, H, device=dev)[:, None]
    xx = torch.linspace(0, 1, W, device=dev)[None, :]
    a = torch.empty((k, H * W), device=dev)
    for j in range(k):
        f1, f2, p1, p2 = (torch.rand(4, generator=g, device=dev) * 6).tolist()
        s = (torch.sin(2 * np.pi * f1 * xx + p1) * torch.cos(2 * np.pi * f2 * yy + p2)).reshape(-1)
        a[j] = base + amp * s if j == const_col else side * s
    return a


def check_sampled(coef_pk, I_np_cols, pinv64):
    ref = o.fit_shared(I_np_cols, pinv64)
    err, ok = coef_close(coef_pk, ref)
    assert ok, err
    return err


def test_config1_1080p_n50_ptm():
    """configs[1]: sampled fp64 parity (with noise), exact recovery (noise-free) and linearity."""
    dev = torch.device("cuda", 0)
    H, W, N = 1080, 1920, 50
    P = H * W
    lu, lv = o.synth_dirs(N, 1)
    B = o.ptm_design(lu, lv)
    a = smooth_fields(6, H, W, dev, 7, 5, 130.0, 70.0, 60.0)
    I = basis_stack(a, B)
    coef = rti.fit(I.reshape(N, H, W), lu, lv).reshape(P, 6)  # AUTO: VALU stream, 4 chunks per lane
    scale = a.abs().amax(0).clamp_min(1.0)
    assert float(((coef.T - a).abs() / scale).max()) < 1e-4
    pv = o.pinv_shared("ptm", lu, lv)
    I.add_(torch.randn(I.shape, device=dev) * 2.0).round_().clamp_(0, 255)
    coef = rti.fit(I.reshape(N, H, W), lu, lv).reshape(P, 6)
    idx = torch.randint(0, P, (4096,), device=dev)
    idx = torch.cat([idx, torch.arange(P - 2048, P, device=dev)])
    check_sampled(coef[idx].cpu().numpy(), I[:, idx].cpu().numpy(), pv)
    coef2 = rti.fit((2 * I + 3).reshape(N, H, W), lu, lv).reshape(P, 6)
    c3 = torch.as_tensor(pv.sum(1) * 3, device=dev, dtype=torch.float32)
    s2 = coef.abs().amax(1, keepdim=True).clamp_min(1.0)
    assert float(((coef2 - 2 * coef - c3) / (2 * s2)).abs().max()) < 1e-4


def test_config3_4k_rgb_n200_hsh16():
    """configs[3]: C = 3 × N = 200 × 8.29 M px = 4.98e9 elements (channel 2 starts at 3.3e9 > 2^31).
    Sampled fp64 parity in every channel including the last pixels of the last channel, exact
    recovery of the generating HSH-16 coefficients, and linearity fit(2I + 3) = 2·fit(I) + 3·pinv·1."""
    dev = torch.device("cuda", 0)
    H, W, N, C = 2160, 3840, 200, 3
    P = H * W
    lu, lv = o.synth_dirs(N, 3)
    B = o.design("hsh", lu, lv)
    pinv64 = np.linalg.pinv(B)
    I = torch.empty((C, N, P), device=dev)
    fields = []
    for c in range(C):
        a = smooth_fields(16, H, W, dev, 11 + c, 0, 250.0, 120.0, 40.0)
        I[c] = basis_stack(a, B)
        fields.append(a)
    assert I.numel() > 2 ** 32 and 2 * N * P > 2 ** 31
    coef = rti.fit(I.reshape(C, N, H, W), lu, lv, basis="hsh")  # AUTO: LDS-tiled MFMA kernel
    coef = coef.reshape(C, P, 16)
    for c in range(C):  # exact recovery, the whole image of every channel
        scale = fields[c].abs().amax(0).clamp_min(1.0)
        assert float(((coef[c].T - fields[c]).abs() / scale).max()) < 1e-4, c
    del fields
    g = torch.Generator(device=dev).manual_seed(5)
    I.add_(torch.randn(I.shape, generator=g, device=dev) * 2.0).round_().clamp_(0, 255)
    coef = rti.fit(I.reshape(C, N, H, W), lu, lv, basis="hsh").reshape(C, P, 16)
    idx = torch.cat([torch.randint(0, P, (2048,), generator=g, device=dev), torch.arange(P - 1024, P, device=dev)])
    for c in range(C):
        check_sampled(coef[c][idx].cpu().numpy(), I[c][:, idx].cpu().numpy(), pinv64)
    coef_a = coef.clone()
    I.mul_(2).add_(3)
    coef2 = rti.fit(I.reshape(C, N, H, W), lu, lv, basis="hsh").reshape(C, P, 16)
    c3 = torch.as_tensor(pinv64.sum(1) * 3, device=dev, dtype=torch.float32)
    for c in range(C):
        s2 = coef_a[c].abs().amax(1, keepdim=True).clamp_min(1.0)
        assert float(((coef2[c] - 2 * coef_a[c] - c3) / (2 * s2)).abs().max()) < 1e-4, c


def test_config4_4k_relight_1000_evals():
    """configs[4]: 4K PTM-6 maps at 1000 random (lu, lv) in the unit disk, one launch per eval (the
    interactive semantics) into fp32 with sampled pixels against the fp64 oracle per eval; the same
    1000 evals in ONE launch to uint8 [1000][P] (8.3 GB) sampled; int32 over whole rows for 16 evals."""
    dev = torch.device("cuda", 0)
    H, W, E = 2160, 3840, 1000
    P = H * W
    g = torch.Generator(device=dev).manual_seed(4)
    coef = (torch.rand((P, 6), generator=g, device=dev) * 100 - 50).contiguous()
    coef[:, 5] += 130
    rng = np.random.default_rng(4)
    r = np.sqrt(rng.random(E))
    th = 2 * np.pi * rng.random(E)
    lu, lv = r * np.cos(th), r * np.sin(th)
    idx = torch.cat([torch.randint(0, P, (512,), generator=g, device=dev), torch.arange(P - 256, P, device=dev)])
    cs = coef[idx].cpu().numpy()
    worst = 0.0
    outs = []
    for e in range(E):
        img = rti.relight(coef, float(lu[e]), float(lv[e]))
        outs.append(img[idx])
    got = torch.stack(outs).cpu().numpy()  # [E, n]
    ref = o.relight(cs, "ptm", lu, lv)  # [E, n] fp64
    worst = float((np.abs(got - ref) / np.maximum(np.abs(ref), 255)).max())
    assert worst <= 1e-4, worst
    u8 = rti.relight(coef, lu, lv, out_dtype=torch.uint8)  # [E, P]
    assert u8.shape == (E, P)
    gu = u8.reshape(E, P)[:, idx].cpu().numpy().astype(np.int64)
    ru = np.clip(np.trunc(ref), 0, 255)
    near = np.abs(ref - np.round(ref)) < 1e-3  # fp32 evaluation vs fp64 truncation at integers
    assert not ((gu != ru) & ~near).any()
    del u8
    rows = slice(0, 4 * W)
    for e in range(0, E, E // 16):
        i32 = rti.relight(coef, float(lu[e]), float(lv[e]), out_dtype=torch.int32).reshape(P)[rows].cpu().numpy()
        rf = o.relight(coef[rows].cpu().numpy(), "ptm", lu[e], lv[e])[0]
        near = np.abs(rf - np.round(rf)) < 1e-3
        assert not ((i32 != np.trunc(rf)) & ~near).any(), e


def _u8_checks(I8, lu, lv, basis, k, idx_per_c):
    """AUTO on an 8-bit stack (the reference's V channel, analysis.py:219) runs the split-fp16 fit
    (rti_fit_shared_h16): the whole map against the fp32 stream on the same values (fit_shared_into, the
    kernel test_gpu_fit / test_config3 pin), sampled pixels against the fp64 oracle, and linearity."""
    dev = I8.device
    C, N, P = I8.shape
    pinv64 = o.pinv_shared(basis, lu, lv) if basis == "ptm" else np.linalg.pinv(o.design("hsh", lu, lv))
    coef = rti.fit(I8.reshape(C, N, 1, P), lu, lv, basis=basis).reshape(C, P, k)  # AUTO -> h16 for uint8
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    for c in range(C):
        ref32 = rti.fit_shared_into(pv, I8[c].float(), torch.empty((P, k), device=dev), k=k, kernel="auto")
        s = ref32.abs().amax(1, keepdim=True).clamp_min(1.0)
        assert float(((coef[c] - ref32) / s).abs().max()) < 1e-5, c
        del ref32
        idx = idx_per_c[c]
        check_sampled(coef[c][idx].cpu().numpy(), I8[c][:, idx].float().cpu().numpy(), pinv64)
    return coef, pinv64


def test_config2_4k_n100_u8_h16():
    """configs[2] on the reference's own 8-bit intensities: 4K × 100 uint8 through rti.fit's AUTO (the h16
    fit, 1024-pixel tiles two per CU): whole-map agreement with the fp32 stream, sampled fp64 parity
    including the last pixels, and fit(2I + 3) = 2·fit(I) + 3·pinv·1 on I <= 126 (2I + 3 stays 8-bit)."""
    dev = torch.device("cuda", 0)
    H, W, N = 2160, 3840, 100
    P = H * W
    lu, lv = o.synth_dirs(N, 2)
    g = torch.Generator(device=dev).manual_seed(21)
    I8 = torch.randint(0, 127, (1, N, P), generator=g, device=dev, dtype=torch.uint8)
    idx = torch.cat([torch.randint(0, P, (4096,), generator=g, device=dev), torch.arange(P - 2048, P, device=dev)])
    coef, pinv64 = _u8_checks(I8, lu, lv, "ptm", 6, [idx])
    coef2 = rti.fit((2 * I8 + 3).reshape(1, N, 1, P), lu, lv).reshape(1, P, 6)
    c3 = torch.as_tensor(pinv64.sum(1) * 3, device=dev, dtype=torch.float32)
    s2 = coef[0].abs().amax(1, keepdim=True).clamp_min(1.0)
    assert float(((coef2[0] - 2 * coef[0] - c3) / (2 * s2)).abs().max()) < 1e-4


def test_config3_4k_rgb_n200_u8_h16():
    """configs[3] with 8-bit channels: 3 × 200 × 8.29 M = 4.98e9 bytes, past 2^32, through the h16 fit
    (2048-pixel tiles, HSH-16): whole maps against the fp32 stream channel by channel, sampled fp64 parity
    in every channel including the last pixels of the last channel (offsets past 2^32 bytes)."""
    dev = torch.device("cuda", 0)
    H, W, N, C = 2160, 3840, 200, 3
    P = H * W
    lu, lv = o.synth_dirs(N, 3)
    g = torch.Generator(device=dev).manual_seed(33)
    I8 = torch.randint(0, 256, (C, N, P), generator=g, device=dev, dtype=torch.uint8)
    assert I8.numel() > 2 ** 32
    idx = [torch.cat([torch.randint(0, P, (2048,), generator=g, device=dev), torch.arange(P - 1024, P, device=dev)])
           for _ in range(C)]
    _u8_checks(I8, lu, lv, "hsh", 16, idx)


def test_config3_4k_rgb_n200_hsh16_pixel_major():
    """configs[3] in the reference's pixel-major layout ([C][P][N], analysis.py:217-219): AUTO for k = 16 is
    the direct form (rti_fit_shared_pm: the stack straight into v_mfma_f32_16x16x4_f32 operands, non-temporal
    coefficient bursts); the MFMA stream (bounded LDS-DMA ring) runs too.  Whole maps against the light-major
    fit of the same values, sampled fp64 parity including the last pixels of the last channel."""
    dev = torch.device("cuda", 0)
    H, W, N, C = 2160, 3840, 200, 3
    P = H * W
    lu, lv = o.synth_dirs(N, 3)
    pinv64 = np.linalg.pinv(o.design("hsh", lu, lv))
    assert rti._lib.lib().rti_fit_shared_pm_plan(16, N, rti._lib.RTI_F32, P, C, 0, 0, 0) // 10 ** 8 == \
        rti._lib.RTI_PM_DIRECT
    g = torch.Generator(device=dev).manual_seed(41)
    Ipm = torch.randint(0, 256, (C, P, N), generator=g, device=dev, dtype=torch.uint8).float()  # 19.9 GB
    coef = rti.fit(Ipm.reshape(C, H, W, N), lu, lv, basis="hsh", stack="pixel").reshape(C, P, 16)
    pv = torch.as_tensor(rti.pinv(lu, lv, "hsh").astype(np.float32), device=dev)
    direct = rti.api.fit_shared_pm_into(pv, Ipm, torch.empty((C, P, 16), device=dev), k=16, kernel="mfma")
    s = coef.abs().amax(-1, keepdim=True).clamp_min(1.0)
    assert float(((direct - coef) / s).abs().max()) < 1e-5
    del direct
    for c in range(C):
        lm = rti.fit_shared_into(pv, Ipm[c].T.contiguous(), torch.empty((P, 16), device=dev), k=16)
        s = lm.abs().amax(1, keepdim=True).clamp_min(1.0)
        assert float(((coef[c] - lm) / s).abs().max()) < 1e-5, c
        del lm
        idx = torch.cat([torch.randint(0, P, (2048,), generator=g, device=dev), torch.arange(P - 1024, P, device=dev)])
        check_sampled(coef[c][idx].cpu().numpy(), Ipm[c][idx].T.cpu().numpy(), pinv64)
