#!/usr/bin/env python3
"""The blocked Cholesky RBF solver (rti_rbf.hip rbf_solve_chol, N > 256) in one process: the solve of a
400x400 ROI (E = 1 query) with reference-geometry light vectors, median of 5 HIP-event timings, and 64
sampled pixels of a 100-query evaluation against the fp64 oracle (max |f − f_ref| / max(|f_ref|, 255)), and a
hash of the whole fp64 evaluation (runs under RTI_RBF_CHOL_LA=0 / 1 must print the same one).

  python tools/sweep_chol.py [N ...]"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("RTI_PKG_DIR", os.path.join(ROOT, "smartphone-based-rti_amd")))  # A/B builds
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rti  # noqa: E402
import rti_oracle as o  # noqa: E402

dev = torch.device("cuda", 0)
ns = [int(a) for a in sys.argv[1:]] or [300, 400, 600]
q = np.random.default_rng(0).uniform(-1, 1, (2, 100))
for N in ns:
    rng = np.random.default_rng(N)
    cams = np.stack([rng.uniform(-600, 1000, N), rng.uniform(-600, 1000, N), rng.uniform(300, 900, N)], -1)
    lu, lv = rti.light_dirs(cams, 400, 400, device=dev)
    I = torch.as_tensor(rng.integers(0, 256, (400, 400, N)).astype(np.int32), device=dev)
    idx = np.random.default_rng(1).choice(400 * 400, 64, replace=False)
    luh, lvh = lu.cpu().numpy().reshape(-1, N)[idx], lv.cpu().numpy().reshape(-1, N)[idx]
    ih = I.cpu().numpy().reshape(-1, N)[idx].astype(np.float64)
    refs = [o.rbf_linear(luh[k], lvh[k], ih[k], q[0], q[1]) for k in range(len(idx))]
    solve = lambda: rti.interpolate_rbf_perpixel(I, lu, lv, [0.0], [0.0], out_dtype=torch.float64,  # noqa: E731
                                                 out_layout="eval")
    solve()
    torch.cuda.synchronize()
    ms = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        solve()
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    out = rti.interpolate_rbf_perpixel(I, lu, lv, q[0], q[1], out_dtype=torch.float64, out_layout="eval")
    got = out.cpu().numpy().reshape(q.shape[1], -1)[:, idx].T
    worst = max(float(np.abs(got[k] - refs[k]).max() / max(np.abs(refs[k]).max(), 255.0)) for k in range(len(idx)))
    sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"N": N, "solve_ms": round(float(np.median(ms)), 3), "max_rel_vs_oracle": worst,
                      "la": os.environ.get("RTI_RBF_CHOL_LA", "1"), "sha": sha}), flush=True)
