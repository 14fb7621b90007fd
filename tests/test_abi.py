"""C ABI checks that need no GPU: librti.so loads, exports every symbol of
include/rti.h, its constants match the Python mirror, and the host half
(design matrix, pseudo-inverse, basis) agrees with the oracle."""
import os
import re

import numpy as np
import pytest

import rti
import rti_oracle as o
from conftest import ROOT, golden
from rti import _lib as L

HEADER = os.path.join(ROOT, "include", "rti.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rti_[a-z0-9_]+)\s*\(", src)))


def header_defines():
    return dict((m.group(1), int(m.group(2), 0))
                for m in re.finditer(r"#define\s+(RTI_[A-Z0-9_]+)\s+(0x[0-9a-fA-F]+|\d+)", open(HEADER).read()))


def test_library_exports_every_header_symbol():
    lib = rti.load()
    names = header_functions()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(L.SIGNATURES), "Python signature table out of sync with include/rti.h"


def test_constants_match_header():
    for name, value in header_defines().items():
        assert getattr(L, name) == value, name


def test_info_functions():
    lib = rti.load()
    assert lib.rti_version() == 100
    assert lib.rti_status_string(0) == b"ok"
    assert lib.rti_basis_terms(L.RTI_BASIS_PTM6) == 6
    assert lib.rti_basis_terms(L.RTI_BASIS_HSH16) == 16
    assert lib.rti_basis_terms(L.RTI_BASIS_HSH9) == 9
    assert lib.rti_basis_terms(99) == -1


def test_pinv_matches_oracle_and_reference_goldens():
    d = golden("ptm_shared_256x256_N20.npz")
    pv = rti.pinv(d["lu"], d["lv"])
    ref = o.pinv_shared("ptm", d["lu"], d["lv"])
    assert np.abs(pv - ref).max() <= 1e-13 * np.abs(ref).max()
    # applied to the golden intensities, the host pinv reproduces the reference's coefficients
    I = d["I"].astype(np.float64).reshape(20, -1)
    coef = (pv @ I).T.reshape(d["coef"].shape)
    scale = np.abs(d["coef"]).max(-1, keepdims=True)
    assert (np.abs(coef - d["coef"]) / scale).max() < 1e-12


@pytest.mark.parametrize("basis,k", [("hsh", 16), ("hsh9", 9)])
def test_hsh_design_and_pinv_match_oracle(basis, k):
    lu, lv = o.synth_dirs(120, 7)
    A = rti.design_matrix(lu, lv, basis)
    A0 = o.design("hsh", lu, lv)[:, :k]
    assert A.shape == (120, k)
    assert np.abs(A - A0).max() < 1e-13
    pv = rti.pinv(lu, lv, basis)
    assert np.abs(pv - np.linalg.pinv(A0)).max() < 1e-11 * np.abs(pv).max()


def test_ptm_design_uses_float32_monomials():
    lu, lv = o.synth_dirs(50, 3)
    A = rti.design_matrix(lu, lv)
    A0 = o.ptm_design(lu, lv)
    # the reference forms lu**2 with glibc powf (1-ulp differences from x*x are allowed)
    assert np.abs(A - A0).max() <= 2 * np.finfo(np.float32).eps
    assert np.array_equal(A[:, 2:], A0[:, 2:])


def test_pinv_rank_deficient_and_rcond():
    e = golden("ptm_edge.npz")
    pv = rti.pinv(e["singular_lu"], e["singular_lv"])
    assert not np.isfinite(pv).all()  # reference semantics: division by a zero singular value
    pv = rti.pinv(e["singular_lu"], e["singular_lv"], rcond=1e-10)
    assert np.isfinite(pv).all()
    A = o.ptm_design(e["singular_lu"], e["singular_lv"])
    assert np.abs(pv - np.linalg.pinv(A, rcond=1e-10)).max() < 1e-10 * np.abs(pv).max()


def test_bad_arguments_raise_like_reference():
    lu, lv = o.synth_dirs(5, 1)
    with pytest.raises(ValueError):
        rti.pinv(lu, lv)  # N < 6: the reference raises ValueError (analysis.py:298)
    with pytest.raises(ValueError):
        rti.pinv(lu, lv[:4])
    with pytest.raises(ValueError):
        rti.basis_id("rbf")


def test_fit_rejects_cpu_tensors():
    import torch

    I = torch.zeros((8, 4, 4))
    lu, lv = o.synth_dirs(8, 1)
    with pytest.raises(ValueError, match="CUDA"):
        rti.fit(I, lu, lv)
    with pytest.raises(ValueError, match="CUDA"):
        rti.relight(torch.zeros((4, 4, 6)), 0.1, 0.2)


def test_basis_eval_matches_oracle():
    lu, lv = o.synth_dirs(64, 9, radius=1.0)
    lu = lu.astype(np.float64)
    lv = lv.astype(np.float64)
    B = rti.basis_eval(lu, lv, "hsh")
    assert np.abs(B - o.hsh_basis(lu, lv)).max() < 1e-13
    P = rti.basis_eval(lu, lv, "ptm")
    assert np.array_equal(P, np.stack([lu * lu, lv * lv, lu * lv, lu, lv, np.ones_like(lu)], -1))


@pytest.mark.parametrize("case", ["exact6", "nearcollinear", "n200"])
def test_lsq_factors_reproduce_reference_edge_goldens(case):
    """rti_lsq_factors splits the reference's solve (analysis.py:295-298) as U (orthonormal) and
    W = V Σ⁻¹: W·(Uᵀ I) gives the reference's own coefficients for its edge light sets, including the
    near-collinear one (cond(A) = 1.1e8) where the normal equations lose 6.5e-3."""
    e = golden("ptm_edge.npz")
    U, W = rti.lsq_factors(e[f"{case}_lu"], e[f"{case}_lv"])
    assert np.abs(U.T @ U - np.eye(6)).max() < 1e-14
    ref = e[f"{case}_coef"]
    got = W @ (U.T @ e[f"{case}_I"].astype(np.float64))
    assert np.abs(got - ref).max() <= 1e-7 * np.abs(ref).max()
    pv = rti.pinv(e[f"{case}_lu"], e[f"{case}_lv"])
    assert np.abs(W @ U.T - pv).max() <= 1e-9 * np.abs(pv).max()


def test_lsq_factors_rank_deficient_and_rcond():
    e = golden("ptm_edge.npz")
    U, W = rti.lsq_factors(e["singular_lu"], e["singular_lv"])
    assert np.isnan(W @ (U.T @ e["singular_I"].astype(np.float64))).all()  # the reference's NaN
    U, W = rti.lsq_factors(e["singular_lu"], e["singular_lv"], rcond=1e-10)
    A = o.ptm_design(e["singular_lu"], e["singular_lv"])
    ref = np.linalg.pinv(A, rcond=1e-10)
    assert np.abs(W @ U.T - ref).max() < 1e-10 * np.abs(ref).max()
    with pytest.raises(ValueError):
        rti.lsq_factors(e["singular_lu"][:5], e["singular_lv"][:5])


def _q8_decode(op, k, N):
    """Read rti_q8_operator's buffer back (layout of csrc/rti_q8.h): digits [4, k, N], scale [k], corr [k, 4]."""
    T = (N + 63) // 64
    frag = op[: T * 4 * 64 * 16].view(np.int8).reshape(T, 4, 64, 16)
    scale = op[T * 4096: T * 4096 + 128].view(np.float64)
    corr = op[T * 4096 + 128: T * 4096 + 128 + 256].view(np.int32).reshape(16, 4)
    light = lambda g, e: 8 * g + e if e < 8 else 32 + 8 * g + (e - 8)  # noqa: E731
    dig = np.zeros((4, 16, T * 64), np.int64)
    for lane in range(64):
        i, g = lane & 15, lane >> 4
        for e in range(16):
            dig[:, i, np.arange(T) * 64 + light(g, e)] = frag[:, :, lane, e].T
    assert not dig[:, k:].any() and not dig[:, :, N:].any()  # padding rows / lights are zero
    return dig[:, :k, :N], scale[:k], corr[:k]


@pytest.mark.parametrize("basis,N", [("ptm", 20), ("ptm", 100), ("hsh", 200), ("hsh9", 65), ("ptm", 6)])
def test_q8_operator_fixed_point_digits(basis, N):
    """rti_q8_operator (host): four balanced int8 digits per weight reconstruct the 27-bit fixed-point
    operator, the sign-flip corrections are 128·Σ digits, and the exact integer evaluation the kernel does
    (int32 digit sums of x − 128, fp64 combination) reproduces pinv·I to the 2^-28 quantization bound."""
    lu, lv = o.synth_dirs(N, 7)
    pv = rti.pinv(lu, lv, basis)
    k = pv.shape[0]
    op = rti.q8_operator(pv)
    assert op.size == rti._lib.lib().rti_q8_operator_bytes(k, N)
    dig, scale, corr = _q8_decode(op, k, N)
    assert dig[1:].min() >= -64 and dig[1:].max() <= 63 and np.abs(dig[0]).max() <= 64
    W = ((dig[0] * 128 + dig[1]) * 128 + dig[2]) * 128 + dig[3]
    m = np.abs(pv).max(1)
    assert np.allclose(scale, m * 2.0 ** -27, rtol=0, atol=0)
    assert np.abs(W * scale[:, None] - pv).max() <= m.max() * 2.0 ** -28 * 1.0000001
    assert np.array_equal(corr, 128 * dig.sum(-1).T)
    I = np.random.default_rng(N).integers(0, 256, (N, 777))
    acc = np.einsum("jin,np->jip", dig, I - 128)
    s = acc + corr.T[:, :, None]
    c = (((s[0] * 128 + s[1]) * 128 + s[2]) * 128 + s[3]) * scale[:, None]
    ref = pv @ I
    bound = 2.0 ** -28 * m[:, None] * I.sum(0)[None, :]
    assert (np.abs(c - ref) <= bound * 1.0000001 + 1e-12 * np.abs(ref)).all()


def test_q8_operator_rejects_non_finite():
    e = golden("ptm_edge.npz")
    with pytest.raises(ValueError, match="non-finite"):
        rti.q8_operator(rti.pinv(e["singular_lu"], e["singular_lv"]))


@pytest.mark.parametrize("basis,N", [("ptm", 20), ("ptm", 100), ("hsh", 200), ("hsh9", 33)])
def test_h16_operator_split_fp16(basis, N):
    """rti_h16_operator (host): per coefficient row a power-of-two scale s with max|w·s| in [2^14, 2^15), the
    weights split as w·s = hi + lo in fp16 (22 significant bits: |hi + lo − w·s| <= 2^-22·max|w·s|), rows
    >= k and lights >= N zero, inv_s = 1/s; and the product the kernel forms (exact fp16 intensities, fp32-like
    sums) reproduces pinv·I."""
    lu, lv = o.synth_dirs(N, 9)
    pv = rti.pinv(lu, lv, basis)
    k = pv.shape[0]
    op = rti.h16_operator(pv)
    assert op.size == rti._lib.lib().rti_h16_operator_bytes(k, N)
    Np = (N + 31) // 32 * 32
    hi = op[:16 * Np * 2].view(np.float16).reshape(16, Np).astype(np.float64)
    lo = op[16 * Np * 2:32 * Np * 2].view(np.float16).reshape(16, Np).astype(np.float64)
    inv_s = op[32 * Np * 2:].view(np.float32).astype(np.float64)
    assert not hi[k:].any() and not lo[k:].any() and not hi[:, N:].any() and not lo[:, N:].any()
    s = 1.0 / inv_s[:k]
    assert np.array_equal(np.log2(s), np.round(np.log2(s)))  # powers of two
    ws = pv * s[:, None]
    mx = np.abs(ws).max(1)
    assert (mx >= 2.0 ** 14).all() and (mx < 2.0 ** 15).all()
    assert (np.abs(hi[:k, :N] + lo[:k, :N] - ws) <= 2.0 ** -22 * mx[:, None]).all()
    I = np.random.default_rng(N).integers(0, 256, (N, 555)).astype(np.float64)
    c = ((hi[:k, :N] + lo[:k, :N]) @ I) * inv_s[:k, None]
    ref = pv @ I
    assert (np.abs(c - ref) <= 2.0 ** -21 * np.abs(pv).max(1)[:, None] * I.sum(0)[None, :]).all()


def test_h16_operator_rejects_non_finite():
    e = golden("ptm_edge.npz")
    with pytest.raises(ValueError, match="non-finite"):
        rti.h16_operator(rti.pinv(e["singular_lu"], e["singular_lv"]))


def test_entry_points_refuse_unknown_kernel_bits():
    """Every entry point that takes a kernel-selection word refuses bits it does not document with
    RTI_ERR_BAD_ARG before it touches a pointer (no flag may return RTI_OK with the
    coefficients unwritten).  The pointers here are never dereferenced: the check comes first."""
    import ctypes

    lib = rti.load()
    p = ctypes.c_void_p(4096)
    calls = {
        "rti_fit_shared": lambda kern: lib.rti_fit_shared(p, 6, 20, p, L.RTI_F32, 64, 1, 0, 0, p, 0, 0, kern, None),
        "rti_fit_shared_pm": lambda kern: lib.rti_fit_shared_pm(p, 6, 20, p, L.RTI_F32, 64, 1, 0, 0, p, 0, 0, kern,
                                                                None),
        "rti_fit_shared_q8": lambda kern: lib.rti_fit_shared_q8(p, 6, 20, p, 64, 1, 0, 0, p, 0, 0, kern, None),
        "rti_fit_shared_h16": lambda kern: lib.rti_fit_shared_h16(p, 6, 20, p, 64, 1, 0, 0, p, 0, 0, kern, None),
        "rti_fit_shared_residual": lambda kern: lib.rti_fit_shared_residual(p, p, 6, 20, p, L.RTI_F32, 64, 1, 0, 0, p,
                                                                            0, 0, p, p, kern, None),
        "rti_fit_shared_residual_svd": lambda kern: lib.rti_fit_shared_residual_svd(p, p, 6, 20, p, L.RTI_F32, 64, 1, 0,
                                                                                    0, p, 0, 0, p, p, kern, None),
    }
    # the bits each entry documents (include/rti.h); every other single bit must be refused
    chunks, planes = 0xF << L.RTI_KERNEL_CHUNKS_SHIFT, 0xF << L.RTI_KERNEL_TILE_PLANES_SHIFT
    depth, waves = 0xF << L.RTI_KERNEL_TILE_DEPTH_SHIFT, 0xF << L.RTI_KERNEL_TILE_WAVES_SHIFT
    allowed = {
        "rti_fit_shared": 0xFF | L.RTI_KERNEL_NONTEMPORAL | L.RTI_KERNEL_PINV_LDS | L.RTI_KERNEL_NT_STORE
        | L.RTI_KERNEL_STAGE | L.RTI_KERNEL_ROTATE | L.RTI_KERNEL_ROUNDS | L.RTI_KERNEL_ONE_LAUNCH | chunks | planes
        | depth | waves,
        "rti_fit_shared_pm": 0xFF | L.RTI_KERNEL_STAGE | L.RTI_KERNEL_NT_STORE | L.RTI_KERNEL_ROTATE | chunks | waves,
        "rti_fit_shared_q8": L.RTI_KERNEL_STAGE | chunks | depth,
        "rti_fit_shared_h16": chunks | depth | waves,
        "rti_fit_shared_residual": L.RTI_KERNEL_ONE_LAUNCH | chunks,
        "rti_fit_shared_residual_svd": L.RTI_KERNEL_ONE_LAUNCH | chunks,
    }
    for name, call in calls.items():
        for bit in range(8, 32):
            flag = ctypes.c_int(1 << bit).value
            if allowed[name] & (1 << bit):
                continue
            assert call(flag) == L.RTI_ERR_BAD_ARG, (name, hex(1 << bit))
            assert b"kernel bits" in lib.rti_last_error(), name
        # selectors past the ones the entry documents
        top = L.RTI_KERNEL_TILE if allowed[name] & 0xFF else L.RTI_KERNEL_AUTO
        assert call(top + 1) == L.RTI_ERR_BAD_ARG, name
    # the retired pixel-major measurement modes (r04: "no stores" / "no arithmetic" / SGPR weights)
    for flag in (L.RTI_KERNEL_ONE_LAUNCH, L.RTI_KERNEL_ROUNDS, L.RTI_KERNEL_PINV_LDS):
        assert calls["rti_fit_shared_pm"](flag) == L.RTI_ERR_BAD_ARG
        assert lib.rti_fit_shared_pm_plan(6, 20, L.RTI_F32, 64, 1, 0, 0, flag) == 0
