"""Reference-signature adapters (bara96/Smartphone-based-RTI @ v0, analysis.py).

Same names, argument meaning, return layout and error behaviour as the
reference's hot-path functions, with the compute done by librti's HIP kernels:

==============================  ===========================================  ==============================
reference                       file:line                                    HIP path used here
==============================  ===========================================  ==============================
compute_intensities             analysis.py:196-246                          rti_light_dirs
_interpolate_PTM                analysis.py:263-317                          rti_fit_perpixel_dirs (P=1) + rti_relight
_interpolate_RBF                analysis.py:249-260                          rti_rbf_operator + rti_apply_operator
interpolate_intensities (PTM)   analysis.py:321-372                          rti_fit_perpixel_dirs + rti_relight (pixel-major)
interpolate_intensities (RBF)   analysis.py:321-372 (default method)         rti_rbf_perpixel, or the shared operator
prepare_images_data             analysis.py:375-411                          layout adapter (torch); native: relight_tables
relighting_event lookup         interactive_relighting.py:11-39              table lookup + clip (host, one image)
relighting_event image          interactive_relighting.py:31-38              RelightingSession: rti_relight_frame
compute (steps 2-4 + save)      analysis.py:414-482 (from_storage=True)      compute_tables: fused GPU pipeline
==============================  ===========================================  ==============================

Inputs may be NumPy arrays (as in the reference) or tensors; outputs are NumPy
arrays with the reference's dtypes.  The reference returns nested lists; here
the same indexing ([y][x][ly][lx], [ly][lx][y][x]) works on ndarrays.
Differences, by design:
  * the ROI size is the data's size, not ``constants.ROI_DIAMETER``;
  * the RBF branch (``interpolate_PTM=False``, the reference's default) uses one
    shared operator when every pixel sees the same light directions, else one
    fp64 LU solve per pixel (rti_rbf_perpixel);
  * the debug plots of ``first_only=True`` are not drawn (first pixel only is kept).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import api

INTERPOLATION_PARAM = 0.02  # constants.py:11


def _device(device=None):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("rti.compat needs a HIP device (librti has no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def grid_axis(step=INTERPOLATION_PARAM):
    """``np.around(np.mgrid[-1:1:step, -1:1:step], 2)`` axis (analysis.py:345-347, :390-393)."""
    _, xi = np.mgrid[-1:1:step, -1:1:step]
    return np.around(xi, decimals=2)[0]


def _grid_luv(xy_fine):
    xf = np.asarray(xy_fine, np.float64).ravel()
    lu = np.tile(xf, xf.size)          # e = v*G + u  ->  (lu = xf[u], lv = xf[v])
    lv = np.repeat(xf, xf.size)
    return xf.size, lu, lv


def compute_intensities(data, first_only=False, origin=(0.0, 0.0), device=None):
    """analysis.py:196-246: list of (V uint8[R,R], camera f64[3]) -> (lx f32, ly f32, I int32), each [R,R,N]."""
    if data is None or len(data) <= 0:
        raise Exception("Error computing intensities: results are empty")
    dev = _device(device)
    frames = [np.asarray(f) for f, _ in data]
    cams = np.stack([np.asarray(c, np.float64).ravel()[:3] for _, c in data])
    R = frames[0].shape[0]
    if first_only:
        R = 1
    lu, lv = api.light_dirs(cams, R, R, origin=origin, device=dev)
    inten = np.stack([f[:R, :R] for f in frames], axis=-1).astype(np.int32)
    torch.cuda.synchronize(dev)
    return lu.cpu().numpy(), lv.cpu().numpy(), inten


def _perpixel_coefs(lx, ly, inten, dev):
    lx_t = torch.as_tensor(np.ascontiguousarray(lx, np.float32), device=dev)
    ly_t = torch.as_tensor(np.ascontiguousarray(ly, np.float32), device=dev)
    it = np.asarray(inten)
    if it.dtype not in (np.float32, np.int32, np.uint8):
        it = it.astype(np.int32)
    I_t = torch.as_tensor(np.ascontiguousarray(it), device=dev)
    return api.fit(I_t, lx_t, ly_t, basis="ptm", mode="perpixel", coef_dtype=torch.float64)


def _interpolate_PTM(x_coarse, y_coarse, xy_fine, intensity_values, device=None):
    """analysis.py:263-317: one pixel's PTM fit evaluated on xy_fine × xy_fine -> f64 [G, G] ([lv][lu])."""
    dev = _device(device)
    n = len(intensity_values)
    if n < 6:
        raise ValueError(f"shapes not aligned: {n} lights < 6 PTM terms")
    coef = _perpixel_coefs(np.asarray(x_coarse).reshape(1, n), np.asarray(y_coarse).reshape(1, n),
                           np.asarray(intensity_values).reshape(1, n), dev)
    G, lu, lv = _grid_luv(xy_fine)
    out = api.relight(coef, lu, lv, basis="ptm", out_dtype=torch.float64, out_layout="pixel")
    return out.reshape(G, G).cpu().numpy()


def _interpolate_RBF(x_coarse, y_coarse, x_fine, y_fine, intensity_values, device=None):
    """analysis.py:249-260: SciPy Rbf(x, y, I, function='linear')(x_fine, y_fine) for one pixel, f64.

    A singular node set (e.g. repeated directions) raises numpy.linalg.LinAlgError like SciPy."""
    dev = _device(device)
    xf = np.asarray(x_fine, np.float64)
    op = api.rbf_operator(x_coarse, y_coarse, xf.ravel(), np.asarray(y_fine, np.float64).ravel())
    it = np.asarray(intensity_values)
    if it.dtype not in (np.float32, np.int32, np.uint8):
        it = it.astype(np.int32)
    I = torch.as_tensor(np.ascontiguousarray(it.reshape(-1, 1)), device=dev)
    out = api.apply_operator(op, I, out_dtype=torch.float64)
    return out.reshape(xf.shape).cpu().numpy()


def _shared_directions(lx, ly):
    """True when every pixel holds the same light list (directional lights)."""
    return bool((lx == lx[:1, :1]).all() and (ly == ly[:1, :1]).all())


def interpolate_intensities(data, interpolate_PTM=False, first_only=False, device=None):
    """analysis.py:321-372 -> ndarray [R, R, G, G] f64 indexed [y][x][ly][lx]."""
    if data is None or len(data) != 3:
        raise Exception("Error computing interpolation: results are empty or invalid")
    lx, ly, inten = (np.asarray(d) for d in data)
    R = 1 if first_only else lx.shape[0]
    lx, ly, inten = lx[:R, :R], ly[:R, :R], inten[:R, :R]
    if not interpolate_PTM:
        return _interpolate_rbf_roi(lx, ly, inten, device)
    if lx.shape[-1] < 6:
        raise ValueError(f"shapes not aligned: {lx.shape[-1]} lights < 6 PTM terms")
    dev = _device(device)
    coef = _perpixel_coefs(lx, ly, inten, dev)
    G, lu, lv = _grid_luv(grid_axis())
    out = api.relight(coef, lu, lv, basis="ptm", out_dtype=torch.float64, out_layout="pixel")
    return out.reshape(R, R, G, G).cpu().numpy()


def _interpolate_rbf_roi(lx, ly, inten, device):
    """RBF branch of interpolate_intensities (analysis.py:360-363).

    Shared light list (directional lights): one operator for all pixels (MFMA).
    Per-pixel light lists (the reference's geometry): one fp64 solve per pixel."""
    dev = _device(device)
    R, N = lx.shape[0], lx.shape[-1]
    G, qu, qv = _grid_luv(grid_axis())
    if not _shared_directions(lx, ly):
        it = inten if inten.dtype in (np.float32, np.int32, np.uint8) else inten.astype(np.int32)
        I = torch.as_tensor(np.ascontiguousarray(it), device=dev)
        out = api.interpolate_rbf_perpixel(I, lx, ly, qu, qv, out_dtype=torch.float64)
        return out.reshape(R, R, G, G).cpu().numpy()
    op = api.rbf_operator(lx[0, 0], ly[0, 0], qu, qv)
    it = inten if inten.dtype in (np.float32, np.int32, np.uint8) else inten.astype(np.int32)
    I = torch.as_tensor(np.ascontiguousarray(it.reshape(R * R, N).T), device=dev)  # light-major [N, P]
    out = api.apply_operator(op, I, out_dtype=torch.float64)  # [E, P]
    return out.T.reshape(R, R, G, G).cpu().numpy()


def rbf_tables(I, lu, lv, step=INTERPOLATION_PARAM):
    """Native fused RBF path: light-major stack [N, H, W] -> int32 tables [G, G, H, W]
    (interpolate_intensities(RBF) + prepare_images_data in one operator launch)."""
    G, qu, qv = _grid_luv(grid_axis(step))
    out = api.apply_operator(api.rbf_operator(lu, lv, qu, qv), I, out_dtype=torch.int32)
    return out.reshape((G, G) + tuple(out.shape[1:]))


def prepare_images_data(data, first_only=False, device=None):
    """analysis.py:375-411: [y][x][ly][lx] f64 -> [ly][lx][y][x] int32 (C truncation; NaN -> INT32_MIN)."""
    if data is None or len(data) <= 0:
        raise Exception("Error preparing images: results are empty")
    dev = _device(device)
    d = torch.as_tensor(np.asarray(data, np.float64), device=dev)
    if first_only:
        d = d[:1, :1]
    t = d.permute(2, 3, 0, 1).contiguous()
    ok = (t >= -2147483648.0) & (t < 2147483648.0)
    out = torch.where(ok, torch.trunc(torch.where(ok, t, torch.zeros_like(t))),
                      torch.full_like(t, -2147483648.0)).to(torch.int32)
    return out.cpu().numpy()


def relight_tables(coef, step=INTERPOLATION_PARAM, layout="pixel"):
    """Native fused replacement of interpolate_intensities + prepare_images_data:
    coefficient maps [H, W, 6] (fp64 for bit-faithful grids) -> int32 [G, G, H, W]."""
    G, lu, lv = _grid_luv(grid_axis(step))
    out = api.relight(coef, lu, lv, basis="ptm", layout=layout, out_dtype=torch.int32, out_layout="eval")
    spatial = out.shape[1:]
    return out.reshape((G, G) + tuple(spatial))


def draw_light_roi_position(given_x, given_y, shape, to_light_vector=False):
    """Cursor <-> light-vector mapping (Utils/utilities.py:357-381)."""
    h, w = shape
    if to_light_vector:
        lx = round(2 * (given_x / w) - 1, 2)
        ly = round(2 * (given_y / h) - 1, 2)
        if lx >= 0.99:
            lx = 0.98
        if ly >= 0.99:
            ly = 0.98
        return lx, ly
    return int(2 * (1 + given_x) * 100), int(2 * (1 + given_y) * 100)


def table_index(l):
    """interactive_relighting.py:25-26."""
    return round((1 + l) / 2 * 100)


def relight_lookup(tables, x, y, shape):
    """relighting_event's table lookup + clip (interactive_relighting.py:22-36) -> int32 image [R, R].

    The reference clips the looked-up table IN PLACE (:35-36); this returns a
    clipped copy and leaves ``tables`` unchanged."""
    lx, ly = draw_light_roi_position(x, y, shape, to_light_vector=True)
    vals = np.array(tables[table_index(ly)][table_index(lx)], copy=True)
    vals[vals > 255] = 255
    vals[vals <= 0] = 0
    return vals


def relight_at_cursor(coef, x, y, shape, basis="ptm"):
    """Continuous relighting: cursor -> (lx, ly) -> uint8 V image from coefficients."""
    lx, ly = draw_light_roi_position(x, y, shape, to_light_vector=True)
    return api.relight(coef, lx, ly, basis=basis, out_dtype=torch.uint8)


class RelightingSession:
    """interactive_relighting.compute()'s state plus relighting_event (interactive_relighting.py:11-39,
    78-124) without the OpenCV windows: the HSV ROI (get_ROI(..., hsv=True)) and either the
    reference's int32 tables ``interpolation_results[ly][lx]`` or coefficient maps stay on the
    device, and every event is one rti_relight_frame launch (clip + V substitution +
    HSV -> BGR).

    light_shape: (h, w) of the light-position window the cursor moves in (draw_light, :55-56).
    With coefficients, ``quantize=True`` evaluates at the 0.02 grid point the reference's table
    lookup would pick (same image as a table made from the same fp64 coefficients);
    ``quantize=False`` relights continuously at the cursor's (lx, ly)."""

    def __init__(self, roi_hsv, light_shape, interpolation_results=None, coef=None, basis="ptm", layout="pixel",
                 quantize=True, device=None):
        if (interpolation_results is None) == (coef is None):
            raise ValueError("give exactly one of interpolation_results (int32 tables) or coef (coefficient maps)")
        self.dev = _device(device)
        self.hsv = torch.as_tensor(np.ascontiguousarray(roi_hsv, np.uint8)).to(self.dev)
        self.shape = tuple(light_shape)[:2]
        self.tables = interpolation_results
        self.coef = None if coef is None else torch.as_tensor(coef).to(self.dev)
        self.basis, self.layout, self.quantize = basis, layout, quantize
        self.axis = grid_axis()
        self.out = torch.empty(self.hsv.shape, dtype=torch.uint8, device=self.dev)
        self._table_dev = None

    def light(self, x, y):
        """draw_light (interactive_relighting.py:42-61) minus the drawing: cursor -> (lx, ly)."""
        return draw_light_roi_position(x, y, self.shape, to_light_vector=True)

    def frame(self, x, y):
        """Device uint8 [R, R, 3] BGR image for a cursor position (no host copy)."""
        lx, ly = self.light(x, y)
        iy, ix = table_index(ly), table_index(lx)
        if self.coef is None:
            t = np.ascontiguousarray(self.tables[iy][ix], np.int32)
            if self._table_dev is None or self._table_dev.shape != t.shape:
                self._table_dev = torch.empty(t.shape, dtype=torch.int32, device=self.dev)
            self._table_dev.copy_(torch.from_numpy(t))
            return api.relight_frame(self._table_dev, self.hsv, out=self.out)
        lu, lv = (self.axis[ix], self.axis[iy]) if self.quantize else (lx, ly)
        return api.relight_frame(self.coef, self.hsv, lu, lv, basis=self.basis, layout=self.layout, out=self.out)

    def relighting_event(self, event, x, y, flags=None, param=None):
        """interactive_relighting.py:11-39: returns the BGR image the reference passes to imshow.

        Unlike the reference, the table is not clipped in place (a copy is clipped on the GPU)."""
        return self.frame(x, y).cpu().numpy()


def compute_tables(results_frames, interpolate_PTM=False, first_only=False, origin=(0.0, 0.0), device=None):
    """Steps 2-4 of analysis.compute (analysis.py:465-472) fused on the GPU.

    results_frames: the reference's list of (V uint8[R,R], camera f64[3]).  Returns the
    int32 tables [G, G, R, R] ([ly][lx][y][x]) that prepare_images_data would produce.
    PTM: light vectors + per-pixel fit in one kernel, then the 100×100 grid in one relight
    launch (fp64, reference op order).  RBF (the default): light vectors, then one
    per-pixel fp64 solve + evaluation launch writing the tables directly."""
    if results_frames is None or len(results_frames) <= 0:
        raise Exception("Error computing intensities: results are empty")
    dev = _device(device)
    frames = np.stack([np.asarray(f) for f, _ in results_frames])
    cams = np.stack([np.asarray(c, np.float64).ravel()[:3] for _, c in results_frames])
    R = 1 if first_only else frames.shape[1]
    frames = np.ascontiguousarray(frames[:, :R, :R])
    G, qu, qv = _grid_luv(grid_axis())
    if interpolate_PTM:
        I = torch.as_tensor(frames, device=dev)  # light-major [N, R, R] uint8
        coef = api.fit(I, cams=cams, origin=origin, mode="perpixel", coef_dtype=torch.float64)
        out = api.relight(coef, qu, qv, basis="ptm", out_dtype=torch.int32, out_layout="eval")
    else:
        lu, lv = api.light_dirs(cams, R, R, origin=origin, device=dev)
        I = torch.as_tensor(np.ascontiguousarray(np.moveaxis(frames, 0, -1)), device=dev)  # [R, R, N]
        out = api.interpolate_rbf_perpixel(I, lu, lv, qu, qv, out_dtype=torch.int32, out_layout="eval")
    return out.reshape(G, G, R, R).cpu().numpy()


def compute(video_name="coin1", from_storage=True, storage_filepath=None, interpolate_PTM=False, debug=False,
            assets_dir="assets"):
    """analysis.compute (analysis.py:414-482) for stored frames: read the frames dataset,
    run steps 2-4 on the GPU and write the relight tables the reference's
    interactive_relighting.compute() loads.  Video sync / frame extraction and the e-mail
    notification are host-side features out of scope."""
    from . import io as rio

    if not from_storage:
        raise NotImplementedError("frame extraction from video stays on the host (out of scope)")
    frames_path = storage_filepath or os.path.join(assets_dir, f"frames_results_{video_name}")
    results_frames = rio.read_from_file(frames_path)
    tables = compute_tables(results_frames, interpolate_PTM=interpolate_PTM, first_only=debug)
    if not debug:
        rio.write_tables(tables, os.path.join(assets_dir, f"interpolation_results_{video_name}"))
    return tables
