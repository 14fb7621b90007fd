"""GPU parity of the interactive relight frame (rti_relight_frame: interactive_relighting.py:31-38):
clip + V substitution + OpenCV 8-bit HSV -> BGR, bit-exact against the oracle's restatement,
exhaustively over every (H, S, V) byte triple, and consistent with rti_relight's int32 tables."""
import numpy as np
import pytest
import torch

import rti
import rti_oracle as o
from conftest import golden
from rti import compat

pytestmark = pytest.mark.gpu


def test_every_hsv_triple_bit_exact(cuda):
    # 256 x 256 (H, S) image, one launch per V-table value; table values beyond [0, 255]
    # exercise the clip (interactive_relighting.py:35-36), including INT32_MIN (a NaN pixel).
    hs = np.stack(np.meshgrid(np.arange(256), np.arange(256), indexing="ij"), -1).astype(np.uint8)
    hsv = np.concatenate([hs, np.zeros((256, 256, 1), np.uint8)], -1)
    hsv_d = torch.as_tensor(hsv, device=cuda)
    vals = list(range(256)) + [-7, 0, 256, 1000, np.iinfo(np.int32).min, np.iinfo(np.int32).max]
    outs = []
    for v in vals:
        t = torch.full((256, 256), int(v), dtype=torch.int32, device=cuda)
        outs.append(rti.relight_frame(t, hsv_d))
    got = torch.stack(outs).cpu().numpy()
    for i, v in enumerate(vals):
        ref = o.relighting_event_image(np.full((256, 256), v, np.int32), hsv)
        assert np.array_equal(got[i], ref), (v, np.argwhere(got[i] != ref)[:5])


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (7, 13), (64, 64), (400, 400)])
def test_ragged_sizes_and_offsets(cuda, shape):
    rng = np.random.default_rng(1)
    H, W = shape
    hsv = rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
    tab = rng.integers(-50, 300, (H, W)).astype(np.int32)
    ref = o.relighting_event_image(tab, hsv)
    got = rti.relight_frame(torch.as_tensor(tab, device=cuda), torch.as_tensor(hsv, device=cuda)).cpu().numpy()
    assert np.array_equal(got, ref)
    # misaligned (odd byte offset) views take the byte path
    buf = torch.zeros(H * W * 3 + 1, dtype=torch.uint8, device=cuda)
    hv = buf[1:].view(H, W, 3)
    hv.copy_(torch.as_tensor(hsv))
    got = rti.relight_frame(torch.as_tensor(tab, device=cuda), hv).cpu().numpy()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("coef_dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("layout", ["pixel", "planar"])
def test_coefficients_match_table_path(cuda, coef_dtype, layout):
    """Frame from coefficients at (lu, lv) == frame from rti_relight's int32 table at (lu, lv)."""
    d = golden("ptm_perpixel_32x32_N50.npz")
    coef = torch.as_tensor(d["coef"], device=cuda).to(coef_dtype)  # [32, 32, 6]
    if layout == "planar":
        coef = coef.permute(2, 0, 1).contiguous()
    rng = np.random.default_rng(2)
    hsv = torch.as_tensor(rng.integers(0, 256, (32, 32, 3)).astype(np.uint8), device=cuda)
    for lu, lv in [(0.0, 0.0), (-1.0, 0.98), (0.34, -0.72), (0.5, 0.5)]:
        tab = rti.relight(coef, lu, lv, layout=layout, out_dtype=torch.int32)
        a = rti.relight_frame(coef, hsv, lu, lv, layout=layout).cpu().numpy()
        b = rti.relight_frame(tab, hsv).cpu().numpy()
        assert np.array_equal(a, b)
        assert np.array_equal(a, o.relighting_event_image(tab.cpu().numpy(), hsv.cpu().numpy()))


@pytest.mark.parametrize("basis", ["hsh", "hsh9"])
def test_hsh_coefficients(cuda, basis):
    k = rti.basis_terms(basis)
    rng = np.random.default_rng(3)
    coef = torch.as_tensor(rng.normal(0, 60, (20, 24, k)).astype(np.float32), device=cuda)
    hsv = torch.as_tensor(rng.integers(0, 256, (20, 24, 3)).astype(np.uint8), device=cuda)
    tab = rti.relight(coef, 0.2, -0.3, basis=basis, out_dtype=torch.int32)
    a = rti.relight_frame(coef, hsv, 0.2, -0.3, basis=basis).cpu().numpy()
    assert np.array_equal(a, o.relighting_event_image(tab.cpu().numpy(), hsv.cpu().numpy()))


def test_session_matches_reference_event(cuda):
    """RelightingSession.relighting_event == the reference's event on its own int32 tables, and the
    coefficient-backed session (quantize=True) gives the same images as the tables made from them."""
    d = golden("ptm_perpixel_32x32_N50.npz")
    coef64 = torch.as_tensor(d["coef"], device=cuda)
    tables = compat.relight_tables(coef64)  # [100, 100, 32, 32] int32 (GPU, fp64: bit-exact to the reference)
    tables_np = tables.cpu().numpy()
    rng = np.random.default_rng(4)
    hsv = rng.integers(0, 256, (32, 32, 3)).astype(np.uint8)
    shape = (180, 240)
    s_tab = compat.RelightingSession(hsv, shape, interpolation_results=tables_np, device=cuda)
    s_coef = compat.RelightingSession(hsv, shape, coef=coef64, device=cuda)
    for x, y in [(0, 0), (120, 90), (239, 179), (17, 160), (230, 5)]:
        ref = o.relighting_event_image(o.relight_lookup(tables_np, x, y, shape), hsv)
        assert np.array_equal(s_tab.relighting_event(None, x, y), ref), (x, y)
        assert np.array_equal(s_coef.relighting_event(None, x, y), ref), (x, y)
    s_cont = compat.RelightingSession(hsv, shape, coef=coef64, quantize=False, device=cuda)
    lx, ly = s_cont.light(77, 33)
    tab = rti.relight(coef64, lx, ly, out_dtype=torch.int32).cpu().numpy()
    assert np.array_equal(s_cont.relighting_event(None, 77, 33), o.relighting_event_image(tab, hsv))


def test_bad_args(cuda):
    hsv = torch.zeros((4, 4, 3), dtype=torch.uint8, device=cuda)
    with pytest.raises(ValueError):
        rti.relight_frame(torch.zeros((4, 5), dtype=torch.int32, device=cuda), hsv)
    with pytest.raises(ValueError):
        rti.relight_frame(torch.zeros((4, 4, 6), device=cuda), hsv)  # no (lu, lv)
    with pytest.raises(ValueError):
        rti.relight_frame(torch.zeros((4, 4, 6), device=cuda), hsv, 0.1, 0.2, basis="hsh")
