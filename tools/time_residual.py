#!/usr/bin/env python3
"""Time rti_fit_residual at BASELINE configs[2] (3840x2160, N=100, PTM-6, fp32) with HIP
events on the launch stream; algorithmic bytes per launch = 4·P·N (stack) + 4·P·k (coef)
+ 4·P (res) -> fraction of the 8 TB/s HBM peak.  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
import rti  # noqa: E402


def main(steps=20, warmup=5):
    dev = torch.device("cuda", 0)
    n, h, w, k = 100, 2160, 3840, 6
    P = h * w
    rng = np.random.default_rng(2)
    r = np.sqrt(rng.uniform(0, 0.81, n))
    t = rng.uniform(0, 2 * np.pi, n)
    lu, lv = (r * np.cos(t)).astype(np.float32), (r * np.sin(t)).astype(np.float32)
    I = torch.rand((n, P), device=dev) * 255.0
    coef = rti.fit(I, lu, lv)
    A = torch.as_tensor(rti.design_matrix(lu, lv).astype(np.float32), device=dev)
    res = torch.empty(P, device=dev)
    nb = int(rti._lib.lib().rti_fit_residual_blocks(P))
    partial = torch.zeros(nb, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev)
    import ctypes
    args = [ctypes.c_void_p(A.data_ptr()), k, n, ctypes.c_void_p(I.data_ptr()), 0, P, 1, P, n * P,
            ctypes.c_void_p(coef.data_ptr()), 0, P * k, ctypes.c_void_p(res.data_ptr()),
            ctypes.c_void_p(partial.data_ptr()), ctypes.c_void_p(s.cuda_stream)]
    lib = rti._lib.lib()
    for _ in range(warmup):
        rti._lib.check(lib.rti_fit_residual(*args), "rti_fit_residual")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record(s)
        lib.rti_fit_residual(*args)
        b.record(s)
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    alg = 4.0 * P * n + 4.0 * P * k + 4.0 * P
    gbs = alg / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": "fit_residual_k<6,4,4,float>", "config": "3840x2160 N=100 PTM-6 fp32",
                      "median_ms": round(ms, 4), "alg_bytes": alg, "achieved_GBs": round(gbs, 1),
                      "frac_of_8TBs": round(gbs / 8000.0, 4)}))


if __name__ == "__main__":
    main()
