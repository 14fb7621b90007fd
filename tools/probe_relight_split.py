#!/usr/bin/env python3
"""Launch generations for the relight stream (c5): one 4K PTM-6 relight as ONE rti_relight launch
against the same pixels as 2 / 4 consecutive launches over pixel ranges, with 3 coefficient-map sets
rotated so every launch streams its maps from HBM (bench c5 "cold").  Windows of 30 steps timed with
HIP events, shuffled order, one process.

  python tools/probe_relight_split.py [--rounds 30]
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

import rti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = rti._lib
    lib = L.lib()
    P, k, sets, win = 2160 * 3840, 6, 3, 30
    coefs = [torch.rand((P, k), device=dev) * 100 for _ in range(sets)]
    outs = [torch.empty(P, device=dev) for _ in range(sets)]
    luv = torch.tensor([0.3, -0.2], dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    s = ctypes.c_void_p(stream.cuda_stream)

    def relight(parts):
        bounds = [(P * i // parts) // 1024 * 1024 for i in range(parts)] + [P]

        def f(i):
            c, o = coefs[i % sets], outs[i % sets]
            for a0, a1 in zip(bounds[:-1], bounds[1:]):
                L.check(lib.rti_relight(ctypes.c_void_p(c.data_ptr() + 4 * k * a0), L.RTI_F32, L.RTI_BASIS_PTM6,
                                        a1 - a0, L.RTI_COEF_PIXEL_MAJOR, ctypes.c_void_p(luv.data_ptr()), 1,
                                        ctypes.c_void_p(o.data_ptr() + 4 * a0), L.RTI_F32, L.RTI_OUT_EVAL_MAJOR, s),
                        "relight")
        return f

    variants = [(f"relight {p} launch(es)", relight(p)) for p in (1, 2, 4)]
    ref = None
    for n, f in variants:
        for i in range(6):
            f(i)
        torch.cuda.synchronize()
        got = outs[5 % sets].clone()
        ref = got if ref is None else ref
        print(f"{n}: bit-identical to one launch: {torch.equal(got, ref)}", flush=True)
    ev = {n: [] for n, _ in variants}
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for j in rng.permutation(len(variants)):
            n, f = variants[j]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for i in range(win):
                f(i)
            b.record(stream)
            ev[n].append((a, b))
    torch.cuda.synchronize()
    byts = 4.0 * P * (k + 1)
    for n, _ in variants:
        ms = np.array([a.elapsed_time(b) for a, b in ev[n]]) / win
        print(f"{n:22s} median {np.median(ms) * 1e3:.2f} us  min {ms.min() * 1e3:.2f}  "
              f"{byts / np.median(ms) / 8e9:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
