"""The ctypes stubs INTEGRATION.md §2 shows a reference maintainer are run as written (the code blocks
are extracted from the document, "<this repo>" substituted) and checked against the package API."""
import os
import re

import numpy as np
import pytest
import torch

import rti
import rti_oracle as o

from conftest import ROOT, coef_close, golden

pytestmark = pytest.mark.gpu


def _stub_namespace():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. The C ABI directly"):text.index("## 3. Multi-GPU")]
    code = "\n".join(re.findall(r"```python\n(.*?)```", sec, re.S)).replace("<this repo>", ROOT)
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


def test_stub_ptm_fit_and_residual(cuda):
    ns = _stub_namespace()
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"].astype(np.float32), device=cuda)  # [N, H, W]
    coef = ns["ptm_fit"](I, d["lu"], d["lv"]).cpu().numpy()
    err, ok = coef_close(coef.reshape(-1, 6), d["coef"].reshape(-1, 6))
    assert ok, err
    coef2, res, rms = ns["ptm_fit_with_residual"](I, d["lu"], d["lv"])
    err, ok = coef_close(coef2.cpu().numpy().reshape(-1, 6), d["coef"].reshape(-1, 6))
    assert ok, err
    assert np.isfinite(rms) and res.shape == I.shape[1:]


def test_stub_ptm_fit_pixel_major(cuda):
    """The reference's own (R, R, N) stack handed to rti_fit_shared_pm by the stub, no transpose."""
    ns = _stub_namespace()
    d = golden("ptm_shared_256x256_N20.npz")
    Ipm = torch.as_tensor(np.ascontiguousarray(np.moveaxis(d["I"], 0, -1)).astype(np.float32), device=cuda)
    pv = torch.as_tensor(rti.pinv(d["lu"], d["lv"], "ptm").astype(np.float32), device=cuda)
    coef = ns["ptm_fit_pixel_major"](Ipm, pv).cpu().numpy()
    err, ok = coef_close(coef.reshape(-1, 6), d["coef"].reshape(-1, 6))
    assert ok, err


def test_stub_ptm_fit_u8(cuda):
    ns = _stub_namespace()
    d = golden("ptm_shared_256x256_N20.npz")
    I = torch.as_tensor(d["I"], device=cuda).to(torch.uint8)  # the golden stack is integer 0..255
    assert torch.equal(I.float(), torch.as_tensor(d["I"].astype(np.float32), device=cuda))
    coef = ns["ptm_fit_u8"](I, d["lu"], d["lv"]).cpu().numpy()
    err, ok = coef_close(coef.reshape(-1, 6), d["coef"].reshape(-1, 6))
    assert ok, err


def test_stub_rbf_tables(cuda):
    ns = _stub_namespace()
    d = golden("rbf_perpixel_4x4_N50.npz")
    tables = ns["rbf_tables"](d["lx"], d["ly"], d["I"]).cpu().numpy()
    ref = d["tables"]
    near = np.abs(np.transpose(d["grid"], (2, 3, 0, 1)) - np.round(np.transpose(d["grid"], (2, 3, 0, 1)))) < 1e-6
    assert tables.shape == ref.shape
    assert not ((tables != ref) & ~near).any()
