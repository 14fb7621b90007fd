#!/usr/bin/env python3
"""Launch generations for the residual pass (rti_fit_residual): the c3 stack's residuals as ONE call
against the same pixels as 2 / 4 / 8 consecutive calls over pixel ranges (pointer offsets, the plane
stride kept at P), interleaved in one process with shuffled order, HIP events per step; plus the
fit in AUTO and one-launch form as the reference point.  Checks the split residuals are bit-identical.

  python tools/probe_residual_split.py [--rounds 40]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _, H, W, N, C, basis, _ = bench.CONFIGS[args.config]
    P, k = H * W, rti.basis_terms(basis)
    L = rti._lib
    lib = L.lib()
    lu, lv = bench.synth_dirs(N, 2)
    I = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev)
    A32 = torch.as_tensor(rti.design_matrix(lu, lv, basis), device=dev).float().contiguous()
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    coef = torch.empty((C, P, k), device=dev)
    res = torch.empty((C, P), device=dev)
    stream = torch.cuda.current_stream(dev)
    s = ctypes.c_void_p(stream.cuda_stream)
    vp = lambda t, off=0: ctypes.c_void_p(t.data_ptr() + off)  # noqa: E731

    def fit(flags):
        return lambda: L.check(lib.rti_fit_shared(vp(pv), k, N, vp(I), L.RTI_F32, P, C, P, N * P, vp(coef),
                                                  L.RTI_COEF_PIXEL_MAJOR, P * k, flags, s), "fit")

    def resid(parts):
        bounds = [(P * i // parts) // 4096 * 4096 for i in range(parts)] + [P]

        def f():
            for c in range(C):
                for a0, a1 in zip(bounds[:-1], bounds[1:]):
                    L.check(lib.rti_fit_residual(vp(A32), k, N, vp(I, 4 * (c * N * P + a0)), L.RTI_F32, a1 - a0, 1, P,
                                                 N * P, vp(coef, 4 * (c * P + a0) * k), L.RTI_COEF_PIXEL_MAJOR, 0,
                                                 vp(res, 4 * (c * P + a0)), None, s), "resid")
        return f

    fit(0)()
    variants = [("fit AUTO", fit(0)), ("fit ONE_LAUNCH", fit(L.RTI_KERNEL_ONE_LAUNCH))]
    variants += [(f"residual {p} call(s)", resid(p)) for p in (1, 2, 4, 8)]
    outs = {}
    for n, f in variants:
        for _ in range(3):
            f()
        if n.startswith("residual"):
            torch.cuda.synchronize()
            outs[n] = res.clone()
    for n, r in outs.items():
        print(f"{n}: bit-identical to one call: {torch.equal(r, outs['residual 1 call(s)'])}", flush=True)
    byts = {"fit": 4.0 * P * C * (N + k), "residual": 4.0 * P * C * (N + k + 1)}
    ev = {n: [] for n, _ in variants}
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for i in rng.permutation(len(variants)):
            n, f = variants[i]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            f()
            b.record(stream)
            ev[n].append((a, b))
    torch.cuda.synchronize()
    for n, _ in variants:
        ms = np.array([a.elapsed_time(b) for a, b in ev[n]])
        bb = byts[n.split()[0]]
        print(f"{n:22s} median {np.median(ms):.4f} ms  min {ms.min():.4f}  {bb / np.median(ms) / 1e6:.0f} GB/s = "
              f"{bb / np.median(ms) / 8e9:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
