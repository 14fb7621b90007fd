#!/usr/bin/env python3
"""Launch generations for the 8-bit h16 fit (measurement): the AUTO launch against the same stack fitted as G
consecutive pixel ranges, one rti_fit_shared_h16 launch each (so every launch is about one round of resident
workgroups and their per-tile store bursts restart in step), interleaved in one process, HIP events per
step, median of --rounds, each checked bit-identical to the AUTO launch.

  python tools/probe_h16_gens.py --config c3|c2|c4 [--gens 1,2,4,8,16] [--rounds 20]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("RTI_PKG_DIR", os.path.join(ROOT, "smartphone-based-rti_amd")))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--gens", default="1,2,4,8,16")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = rti._lib
    lib = L.lib()
    _, H, W, N, C, basis, _ = bench.CONFIGS[args.config]
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I8 = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev).clamp(0, 255).to(torch.uint8).contiguous()
    op = torch.as_tensor(rti.api.h16_operator(rti.pinv(lu, lv, basis)), device=dev)
    coef = torch.empty((C, P, k), device=dev)
    ref = torch.empty((C, P, k), device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    vp = ctypes.c_void_p

    def gens(G):
        bounds = [min(P, (P * g // G + 1023) // 1024 * 1024) for g in range(G + 1)]
        bounds[-1] = P

        def run():
            for g in range(G):
                p0, p1 = bounds[g], bounds[g + 1]
                if p1 <= p0:
                    continue
                st = lib.rti_fit_shared_h16(vp(op.data_ptr()), k, N, vp(I8.data_ptr() + p0), ctypes.c_int64(p1 - p0), C,
                                            ctypes.c_int64(P), ctypes.c_int64(N * P), vp(coef.data_ptr() + 4 * p0 * k),
                                            0, ctypes.c_int64(P * k), 0, s)
                assert st == 0, st
        return run

    variants = [(f"gens{G}", gens(G)) for G in [int(x) for x in args.gens.split(",")]]
    rti.api.fit_h16_into(op, I8, ref, k=k, layout="pixel")
    same = {}
    for name, fn in variants:
        coef.fill_(float("nan"))
        fn()
        torch.cuda.synchronize()
        same[name] = bool(torch.equal(coef, ref))
    stream = torch.cuda.current_stream(dev)
    times = {name: [] for name, _ in variants}
    for _ in range(args.rounds):
        for name, fn in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            times[name].append((a, b))
        torch.cuda.synchronize()
    alg = 1.0 * P * N * C + 4.0 * P * k * C
    for name, _ in variants:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[name]]))
        gbs = alg / (ms * 1e-3) / 1e9
        print(f"{args.config} {name:8s} {ms:.4f} ms  {gbs:.0f} GB/s ({gbs / 8000:.3f} of 8 TB/s)  same {same[name]}",
              flush=True)


if __name__ == "__main__":
    main()
