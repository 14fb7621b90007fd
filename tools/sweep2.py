#!/usr/bin/env python3
"""Interleaved A/B timing of the fit_probe2 variants (tools/probe/fit_probe2.hip) against
the library's AUTO fit, in one process: every round runs each variant once with HIP
events around the launch; median / min per variant.  Store variants are checked against
the library's coefficients (max |diff|) so a variant worth promoting is also correct.

  python tools/sweep2.py [--config c3] [--rounds 30] [--variants 4801:0,4811:2048,...]
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

DEFAULT = ("40801:0,40800:0,80801:0,80800:0,160401:0,160400:0,160801:0,160800:0,161601:0,161600:0,"
           "160811:1024,320801:0,320800:0,321601:0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--variants", default=DEFAULT)
    ap.add_argument("--spin", type=int, default=20000, help="grid-barrier spin bound (iterations of s_sleep 2)")
    ap.add_argument("--pad", type=int, default=0, help="light-plane stride = P + pad floats (probe variants)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _, H, W, N, C, basis, desc = bench.CONFIGS[args.config]
    k = rti.basis_terms(basis)
    assert k == 6 and C == 1
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    ls = P + args.pad
    Ip = I.reshape(N, P)
    if args.pad:
        Ip = torch.empty((N, ls), device=dev)
        Ip[:, :P].copy_(I.reshape(N, P))
    ref = torch.empty((C, P, k), device=dev)
    out = torch.empty((C, P, k), device=dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libfit_probe2.so"))
    lib.probe2_fit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.probe2_gb.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    lib.probe2_gb.restype = ctypes.c_longlong
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    arrivals = [0]
    stream = torch.cuda.current_stream(dev)
    variants = [("auto", None, None)]
    for v in args.variants.split(","):
        a, g = v.split(":")
        if a.startswith("gb"):  # gb<PXL>x<U>: grid-barrier rounds
            px, u = a[2:].split("x")
            variants.append((f"{a}_g{g}", ("gb", int(px), int(u)), int(g)))
        else:
            variants.append((f"v{a}_g{g}", int(a), int(g)))

    def launch(var, grid):
        if var is None:
            rti.fit_shared_into(pv, I, ref, k=k, layout="pixel", kernel="auto")
            return 0
        if isinstance(var, tuple):
            n = lib.probe2_gb(ctypes.c_void_p(pv.data_ptr()), ctypes.c_void_p(Ip.data_ptr()), N, P, ls,
                              ctypes.c_void_p(out.data_ptr()), var[1], var[2], grid, ctypes.c_void_p(ctr.data_ptr()),
                              arrivals[0], args.spin, ctypes.c_void_p(stream.cuda_stream))
            if n < 0:
                return int(-n)
            arrivals[0] += n
            return 0
        return lib.probe2_fit(ctypes.c_void_p(pv.data_ptr()), ctypes.c_void_p(Ip.data_ptr()), N, P, ls,
                              ctypes.c_void_p(out.data_ptr()), var, grid, ctypes.c_void_p(stream.cuda_stream))

    check = {}
    for name, var, grid in variants:
        out.fill_(float("nan"))
        rc = launch(var, grid)
        torch.cuda.synchronize()
        if rc:
            print(f"{name}: rc={rc}", flush=True)
            continue
        if var is not None and (isinstance(var, tuple) or var % 10 == 1):
            check[name] = float((out - ref).abs().max())
    variants = [v for v in variants if v[0] in check or v[1] is None or (not isinstance(v[1], tuple) and v[1] % 10 == 0)]
    for name, var, grid in variants:
        for _ in range(3):
            launch(var, grid)
    torch.cuda.synchronize()
    times = {name: [] for name, *_ in variants}
    for _ in range(args.rounds):
        for name, var, grid in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            launch(var, grid)
            b.record(stream)
            times[name].append((a, b))
    torch.cuda.synchronize()
    alg = 4.0 * P * N + 4.0 * P * k
    res = {}
    for name, var, grid in variants:
        ms = np.array([a.elapsed_time(b) for a, b in times[name]])
        gbs = alg / (np.median(ms) * 1e-3) / 1e9
        res[name] = {"median_ms": float(np.median(ms)), "min_ms": float(ms.min()), "GBps": gbs,
                     "maxdiff": check.get(name)}
        print(f"{name:16s} median {np.median(ms):.4f} ms  min {ms.min():.4f} ms  {gbs:.0f} GB/s "
              f"({gbs / 80:.1f}%)  maxdiff {check.get(name)}", flush=True)
    print(json.dumps({"config": args.config, "pad": args.pad, "results": res}))


if __name__ == "__main__":
    main()
