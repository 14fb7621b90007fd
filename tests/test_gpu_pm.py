"""GPU parity of the shared fit on PIXEL-major stacks (rti_fit_shared_pm), the reference's own
(R, R, N) layout (analysis.py:217-219), against the reference's golden coefficients and the fp64
oracle.  Tolerance: |c - c_ref| <= 1e-4 * max_k |c_ref,k| per pixel."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import coef_close, golden

pytestmark = pytest.mark.gpu

L = rti._lib


def test_golden_256x256_N20_pixel_major(cuda):
    """The reference's golden stack handed over in its own layout ([y][x][n]), as the reference's
    compute_intensities builds it, and as a permuted view of that layout."""
    d = golden("ptm_shared_256x256_N20.npz")
    Ipm = torch.as_tensor(np.ascontiguousarray(np.moveaxis(d["I"], 0, -1))).to(cuda, torch.float32)  # [256, 256, 20]
    plan = L.lib().rti_fit_shared_pm_plan(6, 20, L.RTI_F32, 256 * 256, 1, 0, 0, 0)
    assert plan // 10**8 == L.RTI_PM_VALU_STREAM, plan  # AUTO for PTM-6: the packed-FMA stream
    plan = L.lib().rti_fit_shared_pm_plan(6, 20, L.RTI_F32, 256 * 256, 1, 0, 0, L.RTI_KERNEL_STAGE)
    assert plan // 10**8 == L.RTI_PM_DIRECT, plan  # AUTO | STAGE: straight to registers
    plan = L.lib().rti_fit_shared_pm_plan(16, 20, L.RTI_F32, 256 * 256, 1, 0, 0, 0)
    assert plan // 10**8 == L.RTI_PM_DIRECT, plan  # AUTO for HSH-16: the direct form (non-temporal bursts)
    for layout in ("pixel", "planar"):
        coef = rti.fit(Ipm, d["lu"], d["lv"], stack="pixel", layout=layout).cpu().numpy()
        if layout == "planar":
            coef = np.moveaxis(coef, 0, -1)
        err, ok = coef_close(coef, d["coef"])
        assert ok, (layout, err)
        got = torch.empty((256 * 256, 6) if layout == "pixel" else (6, 256 * 256), device=cuda)
        pv = torch.as_tensor(rti.pinv(d["lu"], d["lv"], "ptm").astype(np.float32), device=cuda)
        rti.api.fit_shared_pm_into(pv, Ipm.reshape(-1, 20), got, k=6, layout=layout, flags=L.RTI_KERNEL_STAGE)
        got = got.cpu().numpy() if layout == "pixel" else got.T.cpu().numpy()
        err, ok = coef_close(got.reshape(256, 256, 6), d["coef"])
        assert ok, ("stage", layout, err)
    # the plan AUTO ran when round 4's uncommitted edit faulted: the MFMA stream, 8 waves, 19-KiB
    # rings, one-group units, interleaved; now reachable as RTI_KERNEL_MFMA, its DMAs bounded by descriptors
    fl = L.RTI_KERNEL_MFMA | (8 << L.RTI_KERNEL_TILE_WAVES_SHIFT)
    assert L.lib().rti_fit_shared_pm_plan(6, 20, L.RTI_F32, 256 * 256, 1, 0, 0, fl) == \
        L.RTI_PM_MFMA_STREAM * 10**8 + 19 * 1000 + 8
    pv = torch.as_tensor(rti.pinv(d["lu"], d["lv"], "ptm").astype(np.float32), device=cuda)
    got = rti.api.fit_shared_pm_into(pv, Ipm.reshape(-1, 20), torch.empty((256 * 256, 6), device=cuda), k=6,
                                     kernel="mfma", flags=8 << L.RTI_KERNEL_TILE_WAVES_SHIFT)
    err, ok = coef_close(got.cpu().numpy().reshape(256, 256, 6), d["coef"])
    assert ok, ("mfma stream w8", err)
    # a light-major-shaped VIEW of the pixel-major stack goes to the same kernel without a copy
    view = Ipm.permute(2, 0, 1)
    assert not view.is_contiguous()
    coef = rti.fit(view, d["lu"], d["lv"]).cpu().numpy()
    err, ok = coef_close(coef, d["coef"])
    assert ok, err
    # ... and agrees with the light-major fit of the same values
    lm = rti.fit(view.contiguous(), d["lu"], d["lv"]).cpu().numpy()
    err, ok = coef_close(coef, lm)
    assert ok, err


def _ref(I_cpn, pinv64):
    return np.einsum("kn,cpn->cpk", pinv64, I_cpn.astype(np.float64))


@pytest.mark.parametrize("basis", ["ptm", "hsh9", "hsh"])
@pytest.mark.parametrize("N", [16, 17, 18, 20, 36, 50, 64, 100, 112, 128, 150, 200, 208, 252, 256, 260])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.int32, torch.uint8])
def test_pm_shapes_vs_fp64(cuda, basis, N, in_dtype):
    """Every light-count class (N % 16 partial chunks, N % 4 in {0, 1, 2}: b128 / b64 / b32 LDS reads; the
    direct form's 16-light step buckets 2/4/7/8/13/16 at and between their edges, and N = 260 past them),
    pixel counts around block multiples (a partial last block), two channels, both coefficient layouts,
    fp32 / int32 stacks (DMA + MFMA) and uint8 (one lane per pixel)."""
    k = rti.basis_terms(basis)
    if N < k:
        pytest.skip("N < k")
    lu, lv = o.synth_dirs(N, 11)
    pinv64 = np.linalg.pinv(o.design("hsh" if basis != "ptm" else "ptm", lu, lv)[:, :k])
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=cuda)
    for P in (4, 16, 20, 68, 1000, 4100):
        if (P * N) % 4 and in_dtype != torch.uint8:
            P += 1  # keep this case on the DMA kernel (P·N % 4 == 0); test_pm_lane_fallback covers the rest
        rng = np.random.default_rng(P * 7 + N)
        I = rng.integers(0, 256, size=(2, P, N)).astype(np.float32)
        ref = _ref(I, pinv64)
        Id = torch.as_tensor(I, device=cuda).to(in_dtype)
        for layout in ("pixel", "planar"):
            for flags in (0, L.RTI_KERNEL_STAGE):  # AUTO, and the direct form for every k
                coef = torch.full((2, P, k) if layout == "pixel" else (2, k, P), float("nan"), device=cuda)
                rti.api.fit_shared_pm_into(pv, Id, coef, k=k, layout=layout, flags=flags)
                got = coef.cpu().numpy()
                if layout == "planar":
                    got = np.moveaxis(got, 1, 2)
                for c in range(2):
                    err, ok = coef_close(got[c], ref[c])
                    assert ok, (P, layout, flags, c, err)


@pytest.mark.parametrize("kern,g,w", [("tile", 1, 1), ("tile", 1, 4), ("tile", 2, 2), ("tile", 2, 5), ("tile", 4, 1),
                                      ("tile", 4, 3), ("mfma", 0, 1), ("mfma", 0, 2), ("mfma", 0, 3), ("mfma", 0, 4),
                                      ("mfma", 0, 6), ("mfma", 0, 8), ("mfma_contig", 0, 8), ("mfma_contig", 0, 3),
                                      ("mfma", 2, 8), ("mfma", 3, 4), ("mfma_contig", 2, 6),
                                      ("auto", 0, 6), ("auto", 0, 5), ("auto", 0, 4), ("auto", 0, 3), ("auto", 0, 2),
                                      ("auto", 0, 1),
                                      ("auto_stage", 0, 12), ("auto_stage", 0, 8), ("auto_stage", 0, 4),
                                      ("auto_stage", 2, 4)])
@pytest.mark.parametrize("N", [20, 100, 33, 200])
def test_pm_block_plans(cuda, kern, g, w, N):
    """kernel="tile" (the double-buffered block form): RTI_KERNEL_CHUNKS(G) / TILE_WAVES(W) = 16, 32 and
    64-pixel blocks at 1 to 5 waves per workgroup; kernel="mfma" (the streaming ring, AUTO's form) at 1 to 8
    waves per workgroup (ring sizes from 18 to 150 KiB, so the ring wraps inside groups at every N), units of
    1-3 groups (CHUNKS), interleaved or contiguous: the same coefficients (every pixel covered exactly once)."""
    k = 6
    lu, lv = o.synth_dirs(N, 5)
    pinv64 = np.linalg.pinv(o.design("ptm", lu, lv))
    pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
    P = 37 * 64 + 16  # partial block for every G
    flags = (g << L.RTI_KERNEL_CHUNKS_SHIFT) | (w << L.RTI_KERNEL_TILE_WAVES_SHIFT)
    if kern == "mfma_contig":  # each wave one contiguous run of units instead of interleaved units
        kern, flags = "mfma", flags | L.RTI_KERNEL_ROTATE
    if kern == "auto_stage":  # the direct form: W waves per CU, CHUNKS(g) launch generations
        kern, flags = "auto", flags | L.RTI_KERNEL_STAGE
    if not L.lib().rti_fit_shared_pm_plan(k, N, L.RTI_F32, P, 3, 0, 0, flags | rti.api._KERNELS[kern]):
        pytest.skip("plan does not fit the LDS")
    rng = np.random.default_rng(g * 10 + w + N)
    I = rng.integers(0, 256, size=(3, P, N)).astype(np.float32)
    coef = torch.full((3, P, k), float("nan"), device=cuda)
    rti.api.fit_shared_pm_into(pv, torch.as_tensor(I, device=cuda), coef, k=k, kernel=kern, flags=flags)
    ref = _ref(I, pinv64)
    got = coef.cpu().numpy()
    for c in range(3):
        err, ok = coef_close(got[c], ref[c])
        assert ok, (c, err)


def test_pm_lane_fallback(cuda):
    """Shapes the DMA kernel does not take run one lane per pixel: P·N % 4 != 0, a pixel stride > N
    (a light slice of a wider stack), N past the LDS budget, and kernel="valu" forcing it."""
    k = 6
    cases = [(3, 1001, 50, 50), (1, 777, 13, 16), (2, 300, 1100, 1100), (1, 4096, 100, 100)]
    for C, P, N, ps in cases:
        lu, lv = o.synth_dirs(N, 3)
        pinv64 = np.linalg.pinv(o.design("ptm", lu, lv))
        pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
        rng = np.random.default_rng(P + N)
        full = rng.integers(0, 256, size=(C, P, ps)).astype(np.float32)
        Id = torch.as_tensor(full, device=cuda)[:, :, :N]
        coef = torch.full((C, P, k), float("nan"), device=cuda)
        kern = "valu" if N == 100 else "auto"
        rti.api.fit_shared_pm_into(pv, Id, coef, k=k, kernel=kern)
        ref = _ref(full[:, :, :N], pinv64)
        got = coef.cpu().numpy()
        for c in range(C):
            err, ok = coef_close(got[c], ref[c])
            assert ok, (C, P, N, ps, c, err)
    # the MFMA kernel refuses what it cannot take instead of falling back
    lu, lv = o.synth_dirs(13, 3)
    pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
    with pytest.raises(NotImplementedError):
        rti.api.fit_shared_pm_into(pv, torch.zeros((777, 13), device=cuda), torch.empty((777, 6), device=cuda), k=6,
                                   kernel="mfma")


@pytest.mark.parametrize("N,flags", [(21, 0), (20, 0), (20, L.RTI_KERNEL_STAGE), (100, L.RTI_KERNEL_STAGE),
                                     (104, L.RTI_KERNEL_STAGE)])
def test_pm_nan_stays_in_its_pixel(cuda, N, flags):
    """A NaN intensity makes its own pixel's coefficients NaN (0·NaN in the reference's matmul) and no
    other pixel's: the masked tail chunk (LDS forms) and the out-of-range lights of the last 16-light step
    (direct form) must not bring in the next pixel's values."""
    P = 64
    lu, lv = o.synth_dirs(N, 2)
    pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
    I = torch.full((P, N), 7.0, device=cuda)
    I[5, 0] = float("nan")
    I[6, 0] = float("inf")
    I[40, N - 1] = float("nan")
    coef = rti.api.fit_shared_pm_into(pv, I, torch.empty((P, 6), device=cuda), k=6, flags=flags).cpu().numpy()
    bad = ~np.isfinite(coef).all(-1)
    assert bad[5] and bad[6] and bad[40] and bad.sum() == 3


@pytest.mark.slow
def test_pm_full_size_4k_n100(cuda):
    """BASELINE configs[2] size (3840x2160, N=100) in the reference's pixel-major layout: sampled fp64
    parity, exact recovery of noise-free generating coefficients, agreement with the light-major fit."""
    H, W, N = 2160, 3840, 100
    P = H * W
    lu, lv = o.synth_dirs(N, 2)
    g = torch.Generator(device=cuda).manual_seed(0)
    a_true = torch.rand((P, 6), generator=g, device=cuda, dtype=torch.float32) * 100 - 50
    B = torch.as_tensor(o.ptm_design(lu, lv), device=cuda, dtype=torch.float32)  # [N, 6]
    Ipm = torch.empty((P, N), device=cuda, dtype=torch.float32)
    for n in range(N):  # element-wise fp32 (no library GEMM)
        col = torch.zeros(P, device=cuda, dtype=torch.float32)
        for j in range(6):
            col.add_(a_true[:, j], alpha=float(B[n, j]))
        Ipm[:, n] = col
    coef = rti.fit(Ipm.reshape(H, W, N), lu, lv, stack="pixel").reshape(P, 6)
    idx = torch.randint(0, P, (4096,), generator=g, device=cuda)
    ref = o.fit_shared(Ipm[idx].T.cpu().numpy(), o.pinv_shared("ptm", lu, lv))
    err, ok = coef_close(coef[idx].cpu().numpy(), ref)
    assert ok, err
    scale = a_true.abs().amax(1, keepdim=True).clamp_min(1.0)
    assert float(((coef - a_true).abs() / scale).max()) < 1e-4
    lm = rti.fit(Ipm.T.contiguous().reshape(N, H, W), lu, lv).reshape(P, 6)
    assert float(((coef - lm).abs() / scale).max()) < 1e-5


@pytest.mark.parametrize("N", [17, 20, 36, 50, 100])
def test_pm_generations_many_blocks_per_wave(cuda, N):
    """The VALU generations form (AUTO, k <= 9) with several 64-pixel blocks parked per wave (a ragged pixel
    count: a partial last block), two channels, both layouts, and 1, 3 or 7 launches per channel
    (RTI_KERNEL_CHUNKS forces the extra generations; the 4K full-size test runs AUTO's own 4), units of 1, 2
    and 4 blocks (N % 4), interleaved (AUTO) or one contiguous run per wave (RTI_KERNEL_ROTATE): every
    coefficient bit-identical whatever the split (a pixel's arithmetic does not depend on it)."""
    P, C = next(p for p in range(300_001, 300_005) if p * N % 4 == 0), 2  # (P·N % 4 == 0: the DMA forms)
    lu, lv = o.synth_dirs(N, 13)
    pinv64 = np.linalg.pinv(o.design("ptm", lu, lv))
    pv = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=cuda)
    rng = np.random.default_rng(N)
    I = rng.integers(0, 256, size=(C, P, N)).astype(np.float32)
    Id = torch.as_tensor(I, device=cuda)
    assert L.lib().rti_fit_shared_pm_plan(6, N, L.RTI_F32, P, C, 0, 0, 0) // 10**8 == L.RTI_PM_VALU_STREAM
    ref = _ref(I, pinv64)
    for layout in ("pixel", "planar"):
        outs = []
        for gens, contig in ((0, 0), (3, 0), (7, 0), (0, L.RTI_KERNEL_ROTATE), (5, L.RTI_KERNEL_ROTATE)):
            coef = torch.full((C, P, 6) if layout == "pixel" else (C, 6, P), float("nan"), device=cuda)
            rti.api.fit_shared_pm_into(pv, Id, coef, k=6, layout=layout,
                                       flags=(gens << L.RTI_KERNEL_CHUNKS_SHIFT) | contig)
            assert L.lib().rti_last_launch_count() == C * max(gens, 1), gens  # the generations form ran
            outs.append(coef.cpu().numpy())
        got = outs[0] if layout == "pixel" else np.moveaxis(outs[0], 1, 2)
        for c in range(C):
            err, ok = coef_close(got[c], ref[c])
            assert ok, (layout, c, err)
        assert all(np.array_equal(outs[0], x) for x in outs[1:]), layout


def test_pm_broadcast_stack_and_routing(cuda):
    """a broadcast (stride-0) pixel-major stack is materialised, not read as dense by the C ABI;
    stack="auto" sends a pixel-major view to rti_fit_shared_pm only for fp32 / int32 stacks and the kernels
    it takes, and an explicit stack="pixel" refuses the rest."""
    H, W, N = 24, 40, 20
    lu, lv = o.synth_dirs(N, 4)
    pinv64 = np.linalg.pinv(o.design("ptm", lu, lv))
    rng = np.random.default_rng(3)
    one = torch.as_tensor(rng.integers(0, 256, size=(H, W, N)).astype(np.float32), device=cuda)
    ref = _ref(one.reshape(1, -1, N).cpu().numpy(), pinv64)[0].reshape(H, W, 6)
    rgb = one.unsqueeze(0).expand(3, H, W, N)  # three channels sharing one stack (channel stride 0)
    assert rgb.stride(0) == 0
    coef = rti.fit(rgb, lu, lv, stack="pixel").cpu().numpy()
    for c in range(3):
        err, ok = coef_close(coef[c], ref)
        assert ok, (c, err)
    row = one[0, 0].reshape(1, 1, N).expand(H, W, N)  # every pixel the same row (pixel strides 0)
    coef = rti.fit(row, lu, lv, stack="pixel").cpu().numpy()
    err, ok = coef_close(coef, np.broadcast_to(ref[0, 0], (H, W, 6)))
    assert ok, err
    assert rti.api._pixel_major_of(rgb.permute(0, 3, 1, 2)) is None  # never routed as a pm view
    coef = rti.fit(rgb.permute(0, 3, 1, 2), lu, lv).cpu().numpy()  # auto: the light-major copy
    for c in range(3):
        assert coef_close(coef[c], ref)[1]
    # 8-bit views keep the copy + h16 path; explicit pm with a kernel it does not take raises
    u8 = one.to(torch.uint8)
    coef = rti.fit(u8.permute(2, 0, 1), lu, lv).cpu().numpy()
    assert coef_close(coef, ref, rtol=1e-4)[1]
    with pytest.raises(NotImplementedError):
        rti.fit(one, lu, lv, stack="pixel", kernel="h16")
    with pytest.raises(NotImplementedError):
        rti.fit(one, lu, lv, stack="pixel", nontemporal=True)
