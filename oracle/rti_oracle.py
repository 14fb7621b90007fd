"""CPU oracle for the RTI fit/relight hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``smartphone-based-rti_amd/rti``) never imports it and fails
loudly when the HIP library is missing.

This is a NumPy restatement of the reference's algorithm
(bara96/Smartphone-based-RTI @ v0, ``/root/reference``).  Every function cites
the reference file:line it follows.

Parity pinning: the PTM functions below are checked against golden vectors in
``tests/golden/*.npz`` that ``tests/golden/make_goldens.py`` produced by
importing the reference's own ``analysis.py`` in the build container (with
NumPy 2.2.6 / SciPy 1.15.3).  The HSH-16 basis has no reference counterpart
(SURVEY.md §0 fact 1): it is build-defined and its parity is against this
file's own fp64 least-squares ("parity unpinned by the reference" for HSH).
"""
from __future__ import annotations

import math

import numpy as np

# constants.py:10-11
ROI_DIAMETER = 400
INTERPOLATION_PARAM = 0.02

PTM_K = 6
HSH_K = 16


# ----------------------------------------------------------------------------
# Light vectors (analysis.py:196-246, compute_intensities)
# ----------------------------------------------------------------------------
def compute_intensities(data, roi=ROI_DIAMETER):
    """Restates ``compute_intensities`` (analysis.py:196-246).

    ``data`` is a list of ``(intensities uint8[R,R], camera_position f64[3])``.
    For frame i and ROI pixel (x, y): ``l = (cam_i - (x,y,0)) / |cam_i - (x,y,0)|``
    (analysis.py:228-229), keep l[0], l[1] as float32 (analysis.py:217-218,230-231)
    and the intensity as int32 (analysis.py:219,232).  Output is pixel-major
    ``[R, R, N]`` (index ``[y][x][i]``).
    """
    if data is None or len(data) <= 0:
        raise Exception("Error computing intensities: results are empty")
    n = len(data)
    ys, xs = np.mgrid[0:roi, 0:roi]
    lx = np.empty((roi, roi, n), dtype=np.float32)
    ly = np.empty((roi, roi, n), dtype=np.float32)
    inten = np.empty((roi, roi, n), dtype=np.int32)
    for i, (frame, cam) in enumerate(data):
        cam = np.asarray(cam, dtype=np.float64)
        dx = cam[0] - xs
        dy = cam[1] - ys
        dz = cam[2] - 0.0
        # np.linalg.norm of a 3-vector == sqrt(dx*dx + dy*dy + dz*dz)
        nrm = np.sqrt(dx * dx + dy * dy + dz * dz)
        lx[:, :, i] = dx / nrm
        ly[:, :, i] = dy / nrm
        inten[:, :, i] = np.asarray(frame)[:roi, :roi]
    return lx, ly, inten


def light_dirs_for_pixels(cams, xs, ys):
    """(lu, lv) float32 for pixels (xs, ys) and cameras cams[N,3] -> [len(xs), N].

    Same arithmetic as analysis.py:228-231 (fp64, rounded to float32)."""
    cams = np.asarray(cams, dtype=np.float64)
    dx = cams[None, :, 0] - np.asarray(xs, np.float64)[:, None]
    dy = cams[None, :, 1] - np.asarray(ys, np.float64)[:, None]
    dz = cams[None, :, 2] - 0.0
    nrm = np.sqrt(dx * dx + dy * dy + dz * dz)
    return (dx / nrm).astype(np.float32), (dy / nrm).astype(np.float32)


# ----------------------------------------------------------------------------
# PTM basis / solve (analysis.py:263-317, _interpolate_PTM)
# ----------------------------------------------------------------------------
def ptm_design(lu, lv):
    """Design matrix rows ``(lu², lv², lu·lv, lu, lv, 1.)`` (analysis.py:282-291).

    The reference takes float32 ``lu, lv`` (pixels_lx is float32), so the
    monomials are float32 products, then ``np.array`` of the tuples upcasts to
    float64 (the trailing ``1.`` is a Python float).
    """
    lu = np.asarray(lu, dtype=np.float32)
    lv = np.asarray(lv, dtype=np.float32)
    cols = [_pow2_f32(lu), _pow2_f32(lv), lu * lv, lu, lv, np.ones_like(lu)]
    return np.stack([c.astype(np.float64) for c in cols], axis=-1)


def _pow2_f32(x):
    """``lu ** 2`` on a NumPy float32 SCALAR, as analysis.py:285 evaluates it.

    NumPy's scalar power calls C ``powf``, which on glibc is not always the
    correctly rounded square (≈1 in 1200 inputs differ from ``x*x`` by 1 ulp),
    so the element-wise array square would not reproduce the reference's design
    matrix bit for bit."""
    flat = [v ** 2 for v in np.asarray(x, np.float32).ravel()]
    return np.array(flat, dtype=np.float32).reshape(np.shape(x))


def svd_solve(A, L):
    """Min-norm LS without rcond, exactly as analysis.py:295-298.

    ``u, s, v = svd(A)``; ``c = uᵀL``; ``w = c[:len(s)] / s``; ``a = vᵀw``.
    Raises ValueError for N < k (shape mismatch at analysis.py:298)."""
    A = np.asarray(A, dtype=np.float64)
    L = np.asarray(L)
    if A.shape[0] < A.shape[1]:
        raise ValueError("shapes not aligned: fewer lights than basis terms")
    u, s, v = np.linalg.svd(A)
    c = np.dot(u.T, L)
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.divide(c[: len(s)], s)
    return np.dot(v.T, w)


def ptm_fit_pixel(lu, lv, intensity):
    """Coefficients ``a[6]`` of one pixel (analysis.py:280-298)."""
    return svd_solve(ptm_design(lu, lv), np.asarray(intensity))


def ptm_eval_grid(a, xy_fine):
    """Grid evaluation of analysis.py:300-315, vectorised with the same op order.

    ``results[v][u] = a0*lu**2 + a1*lv**2 + a2*(lu*lv) + a3*lu + a4*lv + a5``
    summed left to right; element-wise NumPy ops round each op like the loop.
    ``a`` may be ``[..., 6]``; the result is ``[..., G, G]`` indexed [lv][lu]."""
    a = np.asarray(a, dtype=np.float64)
    xf = np.asarray(xy_fine, dtype=np.float64)
    lu = xf[None, :]
    lv = xf[:, None]
    a = a[..., None, None, :]
    l0 = a[..., 0] * (lu ** 2)
    l1 = a[..., 1] * (lv ** 2)
    l2 = a[..., 2] * (lu * lv)
    l3 = a[..., 3] * lu
    l4 = a[..., 4] * lv
    return l0 + l1 + l2 + l3 + l4 + a[..., 5]


def interpolate_ptm(x_coarse, y_coarse, xy_fine, intensity_values):
    """Restates ``_interpolate_PTM`` (analysis.py:263-317): fit + grid eval."""
    return ptm_eval_grid(ptm_fit_pixel(x_coarse, y_coarse, intensity_values), xy_fine)


def grid_axis(step=INTERPOLATION_PARAM):
    """``xi[0]`` of analysis.py:345-347: ``np.around(mgrid[-1:1:step], 2)``."""
    _, xi = np.mgrid[-1:1:step, -1:1:step]
    return np.around(xi, decimals=2)[0]


def interpolate_intensities_ptm(data, roi=None):
    """PTM branch of ``interpolate_intensities`` (analysis.py:321-372).

    Returns an ndarray ``[R, R, G, G]`` f64 indexed ``[y][x][ly][lx]``."""
    if data is None or len(data) != 3:
        raise Exception("Error computing interpolation: results are empty or invalid")
    lx, ly, inten = data
    R = lx.shape[0] if roi is None else roi
    xf = grid_axis()
    out = np.empty((R, R, len(xf), len(xf)))
    for y in range(R):
        for x in range(R):
            out[y, x] = interpolate_ptm(lx[y][x], ly[y][x], xf, inten[y][x])
    return out


def prepare_images_data(data):
    """Restates ``prepare_images_data`` (analysis.py:375-411).

    ``[y][x][ly][lx]`` f64 -> ``[ly][lx][y][x]`` int32 with C truncation toward
    zero (the element assignment into an int32 array at analysis.py:407)."""
    if data is None or len(data) <= 0:
        raise Exception("Error preparing images: results are empty")
    d = np.asarray(data, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        return np.ascontiguousarray(np.transpose(d, (2, 3, 0, 1))).astype(np.int32)


def coefs_from_3x3(G):
    """Recover PTM a[6] from the reference's grid at ``xy_fine=[0,1,-1]``.

    SURVEY §8(c): G[v][u] = L(lu=xf[u], lv=xf[v])."""
    G = np.asarray(G, dtype=np.float64)
    a5 = G[..., 0, 0]
    a0 = (G[..., 0, 1] + G[..., 0, 2]) / 2 - a5
    a3 = (G[..., 0, 1] - G[..., 0, 2]) / 2
    a1 = (G[..., 1, 0] + G[..., 2, 0]) / 2 - a5
    a4 = (G[..., 1, 0] - G[..., 2, 0]) / 2
    a2 = G[..., 1, 1] - a0 - a1 - a3 - a4 - a5
    return np.stack([a0, a1, a2, a3, a4, a5], axis=-1)


# ----------------------------------------------------------------------------
# HSH-16 (build-defined; no reference counterpart)
# ----------------------------------------------------------------------------
def _assoc_legendre_no_cs(l, m, t):
    """P_l^m(t) without the Condon-Shortley phase, l <= 3, via scipy-free recursion."""
    # P_m^m = (2m-1)!! (1-t^2)^{m/2}
    pmm = np.ones_like(t)
    somx2 = np.sqrt(np.clip((1.0 - t) * (1.0 + t), 0.0, None))
    fact = 1.0
    for _ in range(m):
        pmm = pmm * fact * somx2
        fact += 2.0
    if l == m:
        return pmm
    pmmp1 = t * (2 * m + 1) * pmm
    if l == m + 1:
        return pmmp1
    pll = None
    for ll in range(m + 2, l + 1):
        pll = (t * (2 * ll - 1) * pmmp1 - (ll + m - 1) * pmm) / (ll - m)
        pmm, pmmp1 = pmmp1, pll
    return pll


def hsh_basis(lu, lv, order=3):
    """Hemispherical harmonics (Gautron et al. 2004), l = 0..order, (order+1)² terms.

    θ from lw = sqrt(max(0, 1 - lu² - lv²)), φ = atan2(lv, lu), t = 2·cosθ − 1.
    H_l^0 = K_l^0 P_l^0(t); H_l^{+m} = √2 K_l^m cos(mφ) P_l^m(t);
    H_l^{-m} = √2 K_l^m sin(mφ) P_l^m(t);  K_l^m = sqrt((2l+1)/(2π) (l-m)!/(l+m)!).
    Column index l² + l + m.  Returns fp64 ``[..., (order+1)²]``."""
    lu = np.asarray(lu, dtype=np.float64)
    lv = np.asarray(lv, dtype=np.float64)
    lw = np.sqrt(np.clip(1.0 - lu * lu - lv * lv, 0.0, None))
    phi = np.arctan2(lv, lu)
    t = 2.0 * lw - 1.0
    cols = []
    for l in range(order + 1):
        for m in range(-l, l + 1):
            am = abs(m)
            K = math.sqrt((2 * l + 1) / (2 * math.pi) * math.factorial(l - am) / math.factorial(l + am))
            P = _assoc_legendre_no_cs(l, am, t)
            if m == 0:
                cols.append(K * P)
            elif m > 0:
                cols.append(math.sqrt(2.0) * K * np.cos(am * phi) * P)
            else:
                cols.append(math.sqrt(2.0) * K * np.sin(am * phi) * P)
    return np.stack(cols, axis=-1)


def design(basis, lu, lv):
    if basis == "ptm":
        return ptm_design(lu, lv)
    if basis == "hsh":
        return hsh_basis(np.asarray(lu, np.float32), np.asarray(lv, np.float32))
    raise ValueError(f"unknown basis {basis!r}")


# ----------------------------------------------------------------------------
# Shared-direction fit (the north_star restatement of analysis.py:321-363)
# ----------------------------------------------------------------------------
def pinv_shared(basis, lu, lv, rcond=None):
    """fp64 pseudo-inverse [k][N] of the shared design matrix.

    rcond=None reproduces the reference's SVD solve with no threshold
    (analysis.py:295-298): a = V diag(1/s) Uᵀ L, so pinv = V diag(1/s) Uᵀ."""
    A = design(basis, lu, lv)
    if A.shape[0] < A.shape[1]:
        raise ValueError("shapes not aligned: fewer lights than basis terms")
    u, s, vh = np.linalg.svd(A, full_matrices=False)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / s
        if rcond is not None:
            inv = np.where(s > rcond * s.max(), inv, 0.0)
        return (vh.T * inv[None, :]) @ u.T


def fit_shared(I_np, pinv):
    """coef[P, k] = I[N, P]ᵀ · pinvᵀ for a light-major intensity stack, fp64."""
    I_np = np.asarray(I_np, dtype=np.float64).reshape(I_np.shape[0], -1)
    return (np.asarray(pinv, np.float64) @ I_np).T


def fit_shared_f32(I_np, pinv):
    """The CPU baseline form: fp64 pinv, fp32 matmul on (N, P)."""
    I2 = I_np.reshape(I_np.shape[0], -1)
    return (np.asarray(pinv, np.float32) @ I2).T


def fit_residual(I_np, A, coef):
    """Per-pixel RMS residual of a shared fit and the residual energy (test oracle of
    rti_fit_residual; the reference solves the same least squares, analysis.py:280-298,
    but never reports the residual).  I_np: [N, P] light-major; A: [N, k]; coef: [P, k].
    Returns (res[P] = sqrt(Σ_n r² / N), ss_total = Σ_p Σ_n r²), fp64."""
    I2 = np.asarray(I_np, np.float64).reshape(I_np.shape[0], -1)
    r = I2 - np.asarray(A, np.float64) @ np.asarray(coef, np.float64).reshape(I2.shape[1], -1).T
    ss = (r * r).sum(axis=0)
    return np.sqrt(ss / I2.shape[0]), float(ss.sum())


def fit_perpixel(lu, lv, inten, basis="ptm"):
    """Per-pixel fit with each pixel's own (lu, lv) list (analysis.py:350-359).

    lu, lv, inten: ``[P, N]``.  fp64 batched SVD with reference semantics."""
    A = design(basis, lu, lv)  # [P, N, k]
    L = np.asarray(inten, dtype=np.float64)
    if A.shape[-2] < A.shape[-1]:
        raise ValueError("shapes not aligned: fewer lights than basis terms")
    u, s, vh = np.linalg.svd(A, full_matrices=False)
    c = np.einsum("pnk,pn->pk", u, L)
    with np.errstate(divide="ignore", invalid="ignore"):
        w = c / s
    return np.einsum("pkj,pk->pj", vh, w)


def relight(coef, basis, lu, lv):
    """L = Σ_k coef[..., k] · b_k(lu, lv) for each (lu, lv) -> [E, P] fp64."""
    B = design(basis, np.atleast_1d(lu), np.atleast_1d(lv))  # [E, k]
    c = np.asarray(coef, np.float64).reshape(-1, B.shape[-1])
    return B @ c.T


# ----------------------------------------------------------------------------
# Linear RBF (analysis.py:249-260: SciPy Rbf(x, y, I, function='linear'))
# ----------------------------------------------------------------------------
def rbf_linear(x_coarse, y_coarse, intensity_values, x_fine, y_fine):
    """Restates SciPy's Rbf with function='linear', smooth=0, norm='euclidean' as the
    reference calls it (analysis.py:259-260): nodes are float64 copies of the float32
    light vectors, A_ij = ‖x_i − x_j‖, w = scipy.linalg.solve(A, I) (LU with partial
    pivoting; an exactly singular A raises LinAlgError), and
    f(q) = Σ_j w_j ‖q − x_j‖ (cdist · nodes)."""
    import scipy.linalg  # the solver SciPy's Rbf itself uses (LAPACK gesv)

    X = np.stack([np.asarray(x_coarse, np.float64).ravel(), np.asarray(y_coarse, np.float64).ravel()], -1)
    A = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    w = scipy.linalg.solve(A, np.asarray(intensity_values, np.float64).ravel())
    xf = np.asarray(x_fine, np.float64)
    Q = np.stack([xf.ravel(), np.asarray(y_fine, np.float64).ravel()], -1)
    D = np.sqrt(((Q[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    return (D @ w).reshape(xf.shape)


def rbf_operator(lu, lv, qu, qv):
    """Shared-node linear-RBF operator opT[N, E] with out = opTᵀ · I (M = Φ A⁻¹, fp64)."""
    X = np.stack([np.asarray(lu, np.float64), np.asarray(lv, np.float64)], -1)
    A = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    Q = np.stack([np.asarray(qu, np.float64), np.asarray(qv, np.float64)], -1)
    Phi = np.sqrt(((Q[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    return np.linalg.solve(A, Phi.T)  # A symmetric: A⁻¹ Φᵀ = (Φ A⁻¹)ᵀ


def interpolate_intensities_rbf(data):
    """RBF (default) branch of interpolate_intensities (analysis.py:321-372) -> [R, R, G, G] f64."""
    if data is None or len(data) != 3:
        raise Exception("Error computing interpolation: results are empty or invalid")
    lx, ly, inten = data
    R = lx.shape[0]
    _, xi = np.mgrid[-1:1:INTERPOLATION_PARAM, -1:1:INTERPOLATION_PARAM]
    yi, _ = np.mgrid[-1:1:INTERPOLATION_PARAM, -1:1:INTERPOLATION_PARAM]
    xi, yi = np.around(xi, 2), np.around(yi, 2)
    out = np.empty((R, R) + xi.shape)
    for y in range(R):
        for x in range(R):
            out[y, x] = rbf_linear(lx[y][x], ly[y][x], inten[y][x], xi, yi)
    return out


# ----------------------------------------------------------------------------
# Relight lookup (interactive_relighting.py:11-39, Utils/utilities.py:357-381)
# ----------------------------------------------------------------------------
def draw_light_roi_position(given_x, given_y, shape, to_light_vector=False):
    """Restates Utils/utilities.py:357-381."""
    h, w = shape
    if to_light_vector:
        lx = round(2 * (given_x / w) - 1, 2)
        ly = round(2 * (given_y / h) - 1, 2)
        if lx >= 0.99:
            lx = 0.98
        if ly >= 0.99:
            ly = 0.98
        return lx, ly
    x = int(2 * (1 + given_x) * 100)
    y = int(2 * (1 + given_y) * 100)
    return x, y


def table_index(l):
    """interactive_relighting.py:25-26: ``round((1 + l) / 2 * 100)``."""
    return round((1 + l) / 2 * 100)


def relight_lookup(table, x, y, shape):
    """interactive_relighting.py:22-36: cursor -> table[int_ly][int_lx] clipped.

    Returns the clipped int32 V-channel image (the reference clips in place)."""
    lx, ly = draw_light_roi_position(x, y, shape, to_light_vector=True)
    vals = np.array(table[table_index(ly)][table_index(lx)], copy=True)
    vals[vals > 255] = 255
    vals[vals <= 0] = 0
    return vals


def hsv2bgr_u8(hsv):
    """cv2.cvtColor(img, cv2.COLOR_HSV2BGR) for uint8 images, as called at
    interactive_relighting.py:38 (OpenCV >= 4.2, README.md:46; OpenCV is not installed
    here, so this restates its published HSV2RGB_b / HSV2RGB_native scalar algorithm,
    hue range 180): s, v = S/255, V/255 and h = H·(6/180) in float32; sector = floor(h)
    (h - 6 when h >= 6); tab = (v, v(1-s), v(1-s·f), v(1-s(1-f))); (b, g, r) by the
    sector table {{1,3,0},{1,0,2},{3,0,1},{0,2,1},{0,1,3},{2,1,0}}; each channel
    saturate_cast<uchar>(x·255) = round half to even, clamp.  s == 0 -> b = g = r = v.
    Parity against OpenCV itself is unpinned; the known-answer tests pin the primaries."""
    a = np.asarray(hsv, np.uint8)
    f32 = np.float32
    H = a[..., 0].astype(f32)
    S = a[..., 1].astype(f32) * (f32(1.0) / f32(255.0))
    V = a[..., 2].astype(f32) * (f32(1.0) / f32(255.0))
    h = H * (f32(6.0) / f32(180.0))
    h = np.where(h >= f32(6.0), h - f32(6.0), h).astype(f32)
    sector = np.floor(h).astype(np.int32)
    fr = (h - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    fr = np.where(bad, f32(0.0), fr).astype(f32)
    one = f32(1.0)
    tab = np.stack([V, V * (one - S), V * (one - S * fr), V * (one - S * (one - fr))], -1).astype(f32)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sd[sector]  # [..., 3]
    bgr = np.take_along_axis(tab, idx, axis=-1)
    bgr = np.where((S == 0)[..., None], V[..., None], bgr).astype(f32)
    return np.clip(np.rint(bgr * f32(255.0)), 0, 255).astype(np.uint8)


def relighting_event_image(values, roi_hsv):
    """interactive_relighting.py:31-38 without the window: clip the selected int32 table
    image in place semantics (values > 255 -> 255, values <= 0 -> 0), write it into the HSV
    ROI's V channel and convert HSV -> BGR."""
    v = np.array(values, copy=True)
    v[v > 255] = 255
    v[v <= 0] = 0
    img = np.array(roi_hsv, np.uint8, copy=True)
    img[:, :, 2] = v
    return hsv2bgr_u8(img)


# ----------------------------------------------------------------------------
# Synthetic inputs (SURVEY §8(d) recipe)
# ----------------------------------------------------------------------------
def synth_dirs(n, seed, radius=0.9):
    """lu, lv ~ U(disk r <= radius), float32."""
    rng = np.random.default_rng(seed)
    r = radius * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    return (r * np.cos(th)).astype(np.float32), (r * np.sin(th)).astype(np.float32)


def synth_coef_fields(h, w, seed, basis="ptm"):
    """Smooth random coefficient fields [H, W, k] (a5 in [60,200], |a0..a4| <= 60)."""
    rng = np.random.default_rng(seed + 1000)
    k = PTM_K if basis == "ptm" else HSH_K
    yy = np.linspace(0, 1, h)[:, None]
    xx = np.linspace(0, 1, w)[None, :]
    out = np.empty((h, w, k))
    for j in range(k):
        f1, f2 = rng.uniform(0.5, 3.0, 2)
        p1, p2 = rng.uniform(0, 2 * np.pi, 2)
        s = np.sin(2 * np.pi * f1 * xx + p1) * np.cos(2 * np.pi * f2 * yy + p2)
        if basis == "ptm":
            out[:, :, j] = 130 + 70 * s if j == 5 else 60 * s
        else:
            out[:, :, j] = 250 + 120 * s if j == 0 else 40 * s
    return out


def synth_intensities(h, w, lu, lv, seed, basis="ptm", noise=2.0):
    """I[N, H, W] float32 = clip(round(basis·a + N(0, noise)), 0, 255)."""
    a = synth_coef_fields(h, w, seed, basis)
    B = design(basis, lu, lv)  # [N, k]
    rng = np.random.default_rng(seed + 2000)
    I = np.einsum("nk,hwk->nhw", B, a) + rng.normal(0, noise, (len(lu), h, w))
    return np.clip(np.round(I), 0, 255).astype(np.float32)
