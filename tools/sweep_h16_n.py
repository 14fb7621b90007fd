#!/usr/bin/env python3
"""The 8-bit shared fit (rti_fit_shared_h16) at one image size over several light counts, interleaved in ONE
process, HIP events per launch, median of --rounds: does a light count that leaves the last 32-light step
mostly empty (N = 100: 3 full steps + 4 lights) cost like the next multiple of 32?

  python tools/sweep_h16_n.py [--hw 2160x3840] [--basis ptm] [--ns 64,96,100,112,128] [--rounds 20]
"""
import argparse
import json
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
    ap.add_argument("--hw", default="2160x3840")
    ap.add_argument("--basis", default="ptm")
    ap.add_argument("--ns", default="64,96,100,112,128")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--geom", default="0", help="RTI_KERNEL_TILE_WAVES values: 0 AUTO, 1 2048-px, 2 1024-px tiles")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    H, W = (int(x) for x in args.hw.split("x"))
    P, k = H * W, rti.basis_terms(args.basis)
    runs = []
    geoms = [int(x) for x in args.geom.split(",")]
    for N in [int(x) for x in args.ns.split(",")]:
        lu, lv = bench.synth_dirs(N, 2)
        I8 = bench.synth_stack(H, W, N, 1, args.basis, lu, lv, 1000, dev).clamp(0, 255).to(torch.uint8)
        op = torch.as_tensor(rti.api.h16_operator(rti.pinv(lu, lv, args.basis)), device=dev)
        coef = torch.empty((1, P, k), device=dev)
        for gm in geoms:
            fl = gm << rti._lib.RTI_KERNEL_TILE_WAVES_SHIFT
            runs.append(((N, gm), lambda op=op, I8=I8, coef=coef, fl=fl: rti.api.fit_h16_into(op, I8, coef, k=k,
                                                                                           layout="pixel", flags=fl)))
    for _, fn in runs:
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    times = {key: [] for key, _ in runs}
    for _ in range(args.rounds):
        for key, fn in runs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            times[key].append((a, b))
        torch.cuda.synchronize()
    res = {}
    for (N, gm), _ in runs:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[(N, gm)]]))
        alg = 1.0 * P * N + 4.0 * P * k
        gbs = alg / (ms * 1e-3) / 1e9
        res[f"{N}_g{gm}"] = {"median_ms": ms, "GBps": gbs, "frac_8TBps": gbs / 8000.0, "us_per_light": 1e3 * ms / N}
        print(f"N={N:4d} geom={gm} {ms:.4f} ms  {gbs:.0f} GB/s ({gbs / 8000:.3f})  {1e3 * ms / N:.3f} us per light",
              flush=True)
    print(json.dumps({"hw": [H, W], "basis": args.basis, "results": res}))


if __name__ == "__main__":
    main()
