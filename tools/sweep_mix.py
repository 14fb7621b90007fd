#!/usr/bin/env python3
"""Mixed read/write HBM ceiling of the shared fits, interleaved in ONE process:
the AUTO fit next to tools/probe/mix_probe.hip's arithmetic-free kernels of the same data flow
(reads in the fit's shape, the fit's coefficient bytes in 1-KiB stores), with the stores placed
after the sweep (the fits' shape), spread over the sweep (an ideal pipeline), left out (the read
ceiling) or alone (the write ceiling).

  python tools/sweep_mix.py --config c3|c4 [--rounds 20]
"""
import argparse
import ctypes
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

PLACES = {0: "reads only", 1: "stores after sweep", 2: "stores spread", 3: "stores only", 4: "stores after, nt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "pm", "u8"],
                    help="pm: 1-KiB-per-instruction streams over the c3 stack's bytes (LDS-DMA vs registers)")
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _, H, W, N, C, basis, _ = bench.CONFIGS["c3" if args.config in ("pm", "u8") else args.config]
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    h16op = torch.as_tensor(rti.api.h16_operator(rti.pinv(lu, lv, basis)), device=dev) if args.config == "u8" else None
    coef = torch.empty((C, P, k), device=dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libmix_probe.so"))
    lib.probe_mix_px.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.probe_mix_tile.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    ip, op = ctypes.c_void_p(I.data_ptr()), ctypes.c_void_p(coef.data_ptr())
    variants = [("fit_auto", lambda: rti.fit_shared_into(pv, I, coef, k=k, layout="pixel", kernel="auto"))]
    if args.config == "u8":  # the c3 stack as uint8: P bytes per plane = P/4 words, 16 pixels per 16-B lane chunk
        I8 = I.to(torch.uint8)
        i8 = ctypes.c_void_p(I8.data_ptr())
        variants = [("fit_h16_auto", lambda: rti.api.fit_h16_into(h16op, I8, coef, k=k, layout="pixel"))]
        for nc, launches in ((2, 1), (4, 1), (2, 4), (4, 4)):  # (the probe needs P % (256·nc) == 0, N % (8/nc) == 0)
            for place in (0, 1):
                variants.append((f"mix_u8_nc{nc}_L{launches}_p{place}",
                                 (lambda nc=nc, launches=launches, place=place:
                                  lib.probe_mix_px(i8, N, P // 4, op, nc, 24, place, launches, sp))))
    elif args.config == "pm":
        lib.probe_pm_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        nbytes = (I.numel() * 4) // (1024 * 256 * 8) * (1024 * 256 * 8)
        for dma in (2, 1, 0):  # 2: LDS-DMA in bursts of 6 KiB (wait 6, refill 6), the fits' shape
            for order in (1, 0):
                for waves in (8, 4):
                    for depth in (8, 16):
                        if dma == 2 and depth < 8:
                            continue
                        variants.append((f"pm_read_{['reg', 'dma', 'dmaburst6'][dma]}_{'slab' if order else 'runs'}_w{waves}_d{depth}",
                                         (lambda dma=dma, order=order, waves=waves, depth=depth:
                                          lib.probe_pm_read(ip, nbytes, op, dma, order, waves, depth, sp))))
    elif args.config == "c3":
        for nc, launches in ((4, 4), (8, 4), (4, 1)):
            for place in PLACES:
                variants.append((f"mix_px_nc{nc}_L{launches}_p{place}",
                                 (lambda nc=nc, launches=launches, place=place:
                                  lib.probe_mix_px(ip, N, P, op, nc, k, place, launches, sp))))
    else:
        for parts in (2, 1):
            for place in PLACES:
                variants.append((f"mix_tile_rc16_parts{parts}_p{place}",
                                 (lambda parts=parts, place=place:
                                  lib.probe_mix_tile(ip, N, P, C, op, k, place, parts, sp))))
    for name, fn in variants:
        for _ in range(3):
            r = fn()
            assert r is None or torch.is_tensor(r) or r == 0, (name, r)
    torch.cuda.synchronize()
    times = {name: [] for name, _ in variants}
    for _ in range(args.rounds):
        for name, fn in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            times[name].append((a, b))
        torch.cuda.synchronize()
    rbytes, wbytes = (1.0 if args.config == "u8" else 4.0) * P * N * C, 4.0 * P * k * C
    res = {}
    for name, _ in variants:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[name]]))
        place = int(name[-1]) if name.startswith("mix") else 1
        byts = (rbytes if place != 3 else 0.0) + (wbytes if place != 0 else 0.0)
        if name.startswith("pm_read"):
            place, byts = 0, float(nbytes)
        res[name] = {"median_ms": ms, "bytes": byts, "TBps": byts / ms / 1e9, "frac_8TBps": byts / ms / 1e9 / 8.0}
        print(f"{name:28s} {PLACES.get(place, ''):20s} {ms:.4f} ms  {byts / ms / 1e9:.2f} TB/s  "
              f"({byts / ms / 1e9 / 8.0:.3f} of 8 TB/s)", flush=True)
    print(json.dumps({"config": args.config, "P": P, "N": N, "C": C, "k": k, "read_bytes": rbytes,
                      "write_bytes": wbytes, "results": res}))


if __name__ == "__main__":
    main()
