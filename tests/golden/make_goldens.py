#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE's own functions.

Runs only in the build container, where the reference is mounted read-only at
``/root/reference`` (it never travels to the GPU box).  The reference's
``analysis.py`` imports ``cv2`` and ``Utils/email_utils.py`` imports ``dotenv``;
neither is installed here and the PTM / RBF / intensity / lookup functions used
below never call them, so both are replaced by EMPTY modules at import time (any
attribute access on them would raise).  Nothing from the reference is copied:
this script only calls its functions and stores inputs and outputs as ``.npz``.

Usage:  python tests/golden/make_goldens.py [--ref /root/reference] [--out tests/golden]
"""
from __future__ import annotations

import argparse
import io
import os
import sys
import types
import contextlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference(ref):
    sys.dont_write_bytecode = True
    for name in ("cv2", "dotenv"):
        sys.modules.setdefault(name, types.ModuleType(name))

    def _not_available(*_a, **_k):
        raise RuntimeError("dotenv is not installed; the e-mail path is never exercised here")

    # email_utils does `from dotenv import load_dotenv` at import time; the name must exist.
    sys.modules["dotenv"].load_dotenv = _not_available
    import matplotlib

    matplotlib.use("Agg")
    sys.path.insert(0, ref)
    import analysis  # noqa: E402  (reference module)
    from Utils import utilities  # noqa: E402

    return analysis, utilities


def quiet(fn, *a, **kw):
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        return fn(*a, **kw)


def coefs_via_ref(analysis, lu, lv, inten):
    """Exact PTM coefficients through the reference's own _interpolate_PTM with xy_fine=[0,1,-1]."""
    G = analysis._interpolate_PTM(x_coarse=lu, y_coarse=lv, xy_fine=np.array([0.0, 1.0, -1.0]),
                                  intensity_values=inten)
    a5 = G[0, 0]
    a0 = (G[0, 1] + G[0, 2]) / 2 - a5
    a3 = (G[0, 1] - G[0, 2]) / 2
    a1 = (G[1, 0] + G[2, 0]) / 2 - a5
    a4 = (G[1, 0] - G[2, 0]) / 2
    a2 = G[1, 1] - a0 - a1 - a3 - a4 - a5
    return np.array([a0, a1, a2, a3, a4, a5]), G


def disk_dirs(rng, n, radius=0.9):
    r = radius * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    return (r * np.cos(th)).astype(np.float32), (r * np.sin(th)).astype(np.float32)


def smooth_ptm_image(rng, h, w, lu, lv, noise=2.0):
    yy = np.linspace(0, 1, h)[:, None]
    xx = np.linspace(0, 1, w)[None, :]
    a = np.empty((h, w, 6))
    for j in range(6):
        f1, f2 = rng.uniform(0.5, 3.0, 2)
        p1, p2 = rng.uniform(0, 2 * np.pi, 2)
        s = np.sin(2 * np.pi * f1 * xx + p1) * np.cos(2 * np.pi * f2 * yy + p2)
        a[:, :, j] = 130 + 70 * s if j == 5 else 60 * s
    lu64, lv64 = lu.astype(np.float64), lv.astype(np.float64)
    B = np.stack([lu64 * lu64, lv64 * lv64, lu64 * lv64, lu64, lv64, np.ones_like(lu64)], -1)
    I = np.einsum("nk,hwk->nhw", B, a) + rng.normal(0, noise, (len(lu), h, w))
    return np.clip(np.round(I), 0, 255).astype(np.uint8)  # light-major [N, H, W]


def meta():
    import scipy

    return np.array(f"numpy {np.__version__}; scipy {scipy.__version__}; reference bara96/Smartphone-based-RTI@v0")


def gen_shared(analysis, out, h=256, w=256, n=20, seed=0):
    """Config 1 (BASELINE.json configs[0]): shared directions, 256x256, N=20."""
    rng = np.random.default_rng(seed)
    lu, lv = disk_dirs(rng, n)
    I = smooth_ptm_image(rng, h, w, lu, lv)
    coef = np.empty((h, w, 6))
    for y in range(h):
        for x in range(w):
            coef[y, x], _ = coefs_via_ref(analysis, lu, lv, I[:, y, x].astype(np.int32))
    # full 100x100 grids for a few pixels through the reference's default grid
    xi = np.around(np.mgrid[-1:1:0.02, -1:1:0.02][1], decimals=2)[0]
    px = np.array([[0, 0], [17, 200], [128, 64], [255, 255]])
    grids = np.stack([analysis._interpolate_PTM(lu, lv, xi, I[:, y, x].astype(np.int32)) for y, x in px])
    np.savez_compressed(os.path.join(out, f"ptm_shared_{h}x{w}_N{n}.npz"), lu=lu, lv=lv, I=I, coef=coef,
                        grid_px=px, grid=grids, meta=meta())


def gen_perpixel(analysis, out, roi=32, n=50, seed=1, roi_grid=4):
    """Reference-faithful per-pixel geometry: compute_intensities -> per-pixel PTM -> grid -> tables."""
    rng = np.random.default_rng(seed)
    # cameras on a hemisphere above the ROI centre (ROI-index units, analysis.py:228)
    th = np.arccos(rng.uniform(0.35, 0.95, n))
    ph = rng.uniform(0, 2 * np.pi, n)
    rad = rng.uniform(2.0, 3.0, n) * roi
    c = roi / 2.0
    cams = np.stack([c + rad * np.sin(th) * np.cos(ph), c + rad * np.sin(th) * np.sin(ph), rad * np.cos(th)], -1)
    frames = rng.integers(0, 256, (n, roi, roi)).astype(np.uint8)
    # smooth-ish: add a shading term so the fit has structure
    data = [(frames[i], cams[i]) for i in range(n)]
    analysis.cst.ROI_DIAMETER = roi
    try:
        lx, ly, inten = quiet(analysis.compute_intensities, data)
        coef = np.empty((roi, roi, 6))
        for y in range(roi):
            for x in range(roi):
                coef[y, x], _ = coefs_via_ref(analysis, lx[y][x], ly[y][x], inten[y][x])
        analysis.cst.ROI_DIAMETER = roi_grid
        sub = (lx[:roi_grid, :roi_grid], ly[:roi_grid, :roi_grid], inten[:roi_grid, :roi_grid])
        grid = quiet(analysis.interpolate_intensities, sub, interpolate_PTM=True)
        grid = np.array(grid)
        tables = quiet(analysis.prepare_images_data, grid)
        tables = np.array(tables)
    finally:
        analysis.cst.ROI_DIAMETER = 400
    np.savez_compressed(os.path.join(out, f"ptm_perpixel_{roi}x{roi}_N{n}.npz"), cams=cams, frames=frames,
                        lx=lx, ly=ly, I=inten, coef=coef, grid=grid, tables=tables, roi_grid=roi_grid,
                        meta=meta())


def gen_edge(analysis, out, seed=2):
    rng = np.random.default_rng(seed)
    cases = {}
    # (a) N = 6: exact interpolation
    lu, lv = disk_dirs(rng, 6)
    I = rng.integers(0, 256, 6).astype(np.int32)
    cases["exact6"] = (lu, lv, I)
    # (b) near-collinear lights: lv = 0.5 lu + 1e-4 jitter (finite but ill-conditioned)
    lu = rng.uniform(-0.9, 0.9, 30).astype(np.float32)
    lv = (0.5 * lu + 1e-4 * rng.standard_normal(30)).astype(np.float32)
    cases["nearcollinear"] = (lu, lv, rng.integers(0, 256, 30).astype(np.int32))
    # (c) exactly rank deficient: every light on lv = 0
    lu = rng.uniform(-0.9, 0.9, 20).astype(np.float32)
    lv = np.zeros(20, np.float32)
    cases["singular"] = (lu, lv, rng.integers(0, 256, 20).astype(np.int32))
    # (d) well-conditioned with N = 200
    lu, lv = disk_dirs(rng, 200)
    cases["n200"] = (lu, lv, rng.integers(0, 256, 200).astype(np.int32))
    arrays = {}
    for name, (lu, lv, I) in cases.items():
        with np.errstate(all="ignore"):
            coef, G = coefs_via_ref(analysis, lu, lv, I)
        arrays[f"{name}_lu"], arrays[f"{name}_lv"], arrays[f"{name}_I"] = lu, lv, I
        arrays[f"{name}_coef"], arrays[f"{name}_G3"] = coef, G
    # (e) N < 6 raises ValueError in the reference (analysis.py:298)
    lu, lv = disk_dirs(rng, 5)
    try:
        coefs_via_ref(analysis, lu, lv, np.arange(5, dtype=np.int32))
        raised = ""
    except Exception as e:  # record the exception type name
        raised = type(e).__name__
    arrays["n5_raises"] = np.array(raised)
    # empty / invalid input messages (analysis.py:205-206, 332-333, 384-385)
    msgs = {}
    for fname, arg in (("compute_intensities", []), ("interpolate_intensities", (1, 2)),
                       ("prepare_images_data", [])):
        try:
            quiet(getattr(analysis, fname), arg)
        except Exception as e:
            msgs[fname] = str(e)
    for k, v in msgs.items():
        arrays[f"msg_{k}"] = np.array(v)
    np.savez_compressed(os.path.join(out, "ptm_edge.npz"), meta=meta(), **arrays)


def gen_rbf(analysis, out, n=20, npx=4, seed=3):
    """Linear RBF grids (the reference's default method) for the 'next' row."""
    rng = np.random.default_rng(seed)
    lu, lv = disk_dirs(rng, n)
    I = rng.integers(0, 256, (npx, n)).astype(np.int32)
    yi, xi = np.mgrid[-1:1:0.02, -1:1:0.02]
    yi = np.around(yi, decimals=2)
    xi = np.around(xi, decimals=2)
    grids = np.stack([analysis._interpolate_RBF(lu, lv, xi, yi, I[p]) for p in range(npx)])
    np.savez_compressed(os.path.join(out, f"rbf_shared_{npx}px_N{n}.npz"), lu=lu, lv=lv, I=I, grid=grids,
                        meta=meta())


def gen_rbf_perpixel(analysis, out, roi=4, seed=5):
    """The reference's DEFAULT path: interpolate_intensities(interpolate_PTM=False) on per-pixel
    light vectors from compute_intensities, then prepare_images_data."""
    p = np.load(os.path.join(out, "ptm_perpixel_32x32_N50.npz"))
    lx, ly, inten = p["lx"][:roi, :roi], p["ly"][:roi, :roi], p["I"][:roi, :roi]
    analysis.cst.ROI_DIAMETER = roi
    try:
        grid = np.array(quiet(analysis.interpolate_intensities, (lx, ly, inten), interpolate_PTM=False))
        tables = np.array(quiet(analysis.prepare_images_data, grid))
    finally:
        analysis.cst.ROI_DIAMETER = 400
    # a repeated light direction makes SciPy's linear system singular
    lx2 = lx[:1, :1].copy()
    ly2 = ly[:1, :1].copy()
    lx2[0, 0, 1], ly2[0, 0, 1] = lx2[0, 0, 0], ly2[0, 0, 0]
    analysis.cst.ROI_DIAMETER = 1
    try:
        quiet(analysis.interpolate_intensities, (lx2, ly2, inten[:1, :1]), interpolate_PTM=False)
        raised = ""
    except Exception as e:
        raised = type(e).__name__
    finally:
        analysis.cst.ROI_DIAMETER = 400
    np.savez_compressed(os.path.join(out, f"rbf_perpixel_{roi}x{roi}_N{lx.shape[-1]}.npz"), lx=lx, ly=ly, I=inten,
                        grid=grid, tables=tables, singular_lx=lx2, singular_ly=ly2, singular_raises=np.array(raised),
                        meta=meta())


def gen_lookup(utilities, out, seed=4):
    """Cursor -> (lx, ly) -> table index (Utils/utilities.py:357-381, interactive_relighting.py:25-26)."""
    rng = np.random.default_rng(seed)
    rows = []
    for h, w in ((400, 400), (399, 401), (100, 300)):
        xs = list(rng.integers(0, w + 1, 40)) + [0, w, w - 1, w // 2]
        ys = list(rng.integers(0, h + 1, 40)) + [0, h, h - 1, h // 2]
        for x, y in zip(xs, ys):
            lx, ly = utilities.draw_light_roi_position(int(x), int(y), (h, w), to_light_vector=True)
            rows.append((x, y, h, w, lx, ly, round((1 + lx) / 2 * 100), round((1 + ly) / 2 * 100)))
    np.savez_compressed(os.path.join(out, "relight_lookup.npz"), rows=np.array(rows, dtype=np.float64),
                        meta=meta())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    if not os.path.isdir(args.ref):
        print(f"reference not present at {args.ref}; nothing to do")
        return 0
    analysis, utilities = import_reference(args.ref)
    os.makedirs(args.out, exist_ok=True)
    jobs = {
        "shared": lambda: gen_shared(analysis, args.out),
        "perpixel": lambda: gen_perpixel(analysis, args.out),
        "edge": lambda: gen_edge(analysis, args.out),
        "rbf": lambda: gen_rbf(analysis, args.out),
        "rbf_perpixel": lambda: gen_rbf_perpixel(analysis, args.out),
        "lookup": lambda: gen_lookup(utilities, args.out),
    }
    for name, job in jobs.items():
        if args.only and name not in args.only.split(","):
            continue
        print("generating", name, flush=True)
        job()
    return 0


if __name__ == "__main__":
    sys.exit(main())
