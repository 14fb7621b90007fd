#!/usr/bin/env python3
"""The 8-bit shared fit (rti_fit_shared_h16) variants interleaved in ONE process, HIP events per launch, median
of --rounds: tile geometry (RTI_KERNEL_TILE_WAVES 1/2: 2048 / 1024 pixels) × tiles per workgroup
(RTI_KERNEL_CHUNKS) × 16-pixel groups batched per transposed-read/MFMA round (RTI_KERNEL_TILE_DEPTH 1/4/8), each
checked bit-identical to the AUTO launch.  (Earlier r04 runs of this tool
also timed a three-stage load pipeline, since removed: profiles/r04s_h16_depth_sweep_*.)

  python tools/sweep_h16.py --config c2|c3|c4 [--rounds 20] [--tpw 0,8,16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("RTI_PKG_DIR", os.path.join(ROOT, "smartphone-based-rti_amd")))  # A/B builds
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--tpw", default="0")
    ap.add_argument("--batches", default="1,4,8")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = rti._lib
    _, H, W, N, C, basis, _ = bench.CONFIGS[args.config]
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I8 = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev).clamp(0, 255).to(torch.uint8)
    op = torch.as_tensor(rti.api.h16_operator(rti.pinv(lu, lv, basis)), device=dev)
    coef = torch.empty((C, P, k), device=dev)
    ref = torch.empty((C, P, k), device=dev)
    variants = []
    geoms = {1: "2048px", 2: "1024px", 3: "2048px16w"}
    for half in (1, 2, 3):  # RTI_KERNEL_TILE_WAVES: 1 = 2048-pixel tiles (one workgroup per CU), 2 = 1024 (two), 3 = 2048 on 16 waves
        for tpw in [int(x) for x in args.tpw.split(",")]:
            for cb in [int(x) for x in args.batches.split(",") if x]:  # groups batched per step (TILE_DEPTH)
                fl = (tpw << L.RTI_KERNEL_CHUNKS_SHIFT) | (cb << L.RTI_KERNEL_TILE_DEPTH_SHIFT) | \
                     (half << L.RTI_KERNEL_TILE_WAVES_SHIFT)
                variants.append((f"h16_{geoms[half]}_tpw{tpw or 'auto'}_batch{cb}",
                                 lambda fl=fl: rti.api.fit_h16_into(op, I8, coef, k=k, layout="pixel", flags=fl)))
    probe = os.path.join(ROOT, "tools", "probe", "libh16_probe.so")
    if C == 1 and os.path.exists(probe):  # tools/probe/h16_probe.hip: the library kernel with its stores dropped
        import ctypes
        plib = ctypes.CDLL(probe)
        vp = ctypes.c_void_p

        def pr(mode):
            st = plib.h16_probe(vp(op.data_ptr()), k, N, vp(I8.data_ptr()), ctypes.c_int64(P), vp(coef.data_ptr()),
                                mode, vp(torch.cuda.current_stream(dev).cuda_stream))
            assert st == 0, st
        variants.append(("probe_h16_perlane", lambda: pr(0)))  # the r04 per-lane coefficient stores
        variants.append(("probe_h16_nostores", lambda: pr(1)))
        variants.append(("probe_h16_nt_stores", lambda: pr(2)))
        if k == 6:
            variants.append(("probe_h16_staged", lambda: pr(3)))
            variants.append(("probe_h16_staged_nt", lambda: pr(4)))
            variants.append(("probe_h16_loads_park", lambda: pr(5)))  # no stores, no transposed reads / MFMAs
            variants.append(("probe_h16_loads_only", lambda: pr(6)))  # ... and no LDS parking
    rti.api.fit_h16_into(op, I8, ref, k=k, layout="pixel")
    same = {}
    for name, fn in variants:
        coef.fill_(float("nan"))
        fn()
        torch.cuda.synchronize()
        same[name] = bool(torch.equal(coef, ref)) if name not in ("probe_h16_nostores", "probe_h16_loads_park",
                                                                   "probe_h16_loads_only") else None
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
    res = {}
    for name, _ in variants:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[name]]))
        gbs = alg / (ms * 1e-3) / 1e9
        res[name] = {"median_ms": ms, "GBps": gbs, "frac_8TBps": gbs / 8000.0, "bit_identical": same[name]}
        print(f"{name:24s} {ms:.4f} ms  {gbs:.0f} GB/s ({gbs / 8000:.3f} of 8 TB/s)  same {same[name]}", flush=True)
    print(json.dumps({"config": args.config, "alg_bytes": alg, "results": res}))


if __name__ == "__main__":
    main()
