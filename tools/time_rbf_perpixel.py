"""Split the per-pixel RBF time into solve (E=1) and evaluation (E=10^4) on a 400x400 ROI."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rti  # noqa: E402

dev = torch.device("cuda", 0)
for N in (50, 100):
    P = 400 * 400
    rng = np.random.default_rng(0)
    cams = np.stack([rng.uniform(-600, 1000, N), rng.uniform(-600, 1000, N), rng.uniform(300, 900, N)], -1)
    lu, lv = rti.light_dirs(cams, 400, 400, device=dev)
    I = torch.as_tensor(rng.integers(0, 256, (400, 400, N)).astype(np.int32), device=dev)
    xf = np.around(np.arange(-1, 1, 0.02), 2)
    grid = np.stack([np.tile(xf, 100), np.repeat(xf, 100)])  # the reference's 100x100 grid, row-major
    for E in (1, 100, 10000, "grid"):
        q = grid if E == "grid" else rng.uniform(-1, 1, (2, E))
        rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.int32, out_layout="eval")
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.int32, out_layout="eval")
        torch.cuda.synchronize()
        print(f"N={N} E={E}: {(time.perf_counter() - t) / 3 * 1e3:.1f} ms", flush=True)
    for lay in ("pixel",):
        q = grid
        rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.int32, out_layout=lay)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.int32, out_layout=lay)
        torch.cuda.synchronize()
        print(f"N={N} E=grid layout={lay}: {(time.perf_counter() - t) / 3 * 1e3:.1f} ms", flush=True)
