#!/usr/bin/env python3
"""Interleaved A/B of rti_fit_perpixel_cam exactness variants (RTI_PERPIXEL_VARIANT, read per call) on the
c6 workload (4K x 100 lights, bench.py's synthetic cameras and stack) in ONE process: every round runs each
variant once, HIP events around the call (fit + refine launches); median / min per variant, and every
variant's coefficients against the first's.

  python tools/sweep_perpixel.py [--variants 0,1,2,3] [--rounds 20]
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
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _, H, W, N, C, basis, desc = bench.CONFIGS["c6"]
    P = H * W
    cams = torch.as_tensor(bench.synth_cams(N, 6, H, W), device=dev).contiguous()
    lu, lv = bench.synth_dirs(N, seed=2)
    I = bench.synth_stack(H, W, N, 1, "ptm", lu, lv, seed=1000, device=dev)[0]
    L = rti._lib
    fn = L.lib().rti_fit_perpixel_cam
    stream = torch.cuda.current_stream(dev)
    variants = [int(v) for v in args.variants.split(",")]
    coefs = {v: torch.empty((P, 6), dtype=torch.float32, device=dev) for v in variants}

    def run(v):
        os.environ["RTI_PERPIXEL_VARIANT"] = str(v)
        st = fn(ctypes.c_void_p(cams.data_ptr()), N, ctypes.c_void_p(I.data_ptr()), L.RTI_F32, H, W, P, 0.0, 0.0,
                -1.0, ctypes.c_void_p(coefs[v].data_ptr()), L.RTI_F32, L.RTI_COEF_PIXEL_MAJOR,
                ctypes.c_void_p(stream.cuda_stream))
        L.check(st, "rti_fit_perpixel_cam")

    for v in variants:
        for _ in range(2):
            run(v)
    torch.cuda.synchronize()
    ref = coefs[variants[0]].double()
    scale = ref.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            run(v)
            b.record(stream)
            times[v].append((a, b))
    torch.cuda.synchronize()
    for v in variants:
        ms = np.array([a.elapsed_time(b) for a, b in times[v]])
        rel = float(((coefs[v].double() - ref).abs() / scale).max())
        same = bool(torch.equal(coefs[v], coefs[variants[0]]))
        print(f"variant {v}: median {np.median(ms):.4f} ms  min {ms.min():.4f} ms  vs variant {variants[0]}: "
              f"max rel {rel:.2e}, bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
