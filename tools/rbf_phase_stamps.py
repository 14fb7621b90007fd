"""Per-phase wall-clock split of the per-pixel RBF kernel (probe build with -DRBF_TIMING).

    RTI_LIBRARY=tools/probe/librti_timing.so python tools/rbf_phase_stamps.py
Phases per block (first 256 blocks, 100 MHz wall clock): load+build A, LU, first solve,
refinement (with sweep count), evaluation."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rti  # noqa: E402
from rti import _lib  # noqa: E402

dev = torch.device("cuda", 0)
L = _lib.lib()
L.rti_rbf_probe_stamps.argtypes = [ctypes.c_void_p]
for N, E in ((50, 10000), (100, 10000)):
    rng = np.random.default_rng(0)
    cams = np.stack([rng.uniform(-600, 1000, N), rng.uniform(-600, 1000, N), rng.uniform(300, 900, N)], -1)
    lu, lv = rti.light_dirs(cams, 400, 400, device=dev)
    I = torch.as_tensor(rng.integers(0, 256, (400, 400, N)).astype(np.int32), device=dev)
    q = rng.uniform(-1, 1, (2, E))
    rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.int32, out_layout="eval")
    torch.cuda.synchronize()
    st = np.zeros((256, 8), np.int64)
    assert L.rti_rbf_probe_stamps(st.ctypes.data) == 0
    t = st[:, [5, 0, 1, 2, 3, 4]].astype(np.float64) * 10e-3  # us (100 MHz)
    d = np.diff(t, axis=1)
    names = ["load+A", "LU", "solve0", "refine", "eval"]
    print(f"N={N} E={E}: " + ", ".join(f"{n} {np.median(d[:, i]):.1f}us" for i, n in enumerate(names))
          + f", sweeps median {np.median(st[:, 7]):.0f} max {st[:, 7].max()}", flush=True)
