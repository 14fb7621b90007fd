#!/usr/bin/env python3
"""Launch generations for the RBF table operator (c7, rti_apply_operator_f16): the 400x400 ROI's
10^4 int32 tables as ONE launch against the same pixels as 2 / 3 / 4 / 5 consecutive launches over
pixel ranges (stack and table pointers offset, the plane / row strides kept at P), interleaved in one
process with shuffled order, HIP events per step.  Checks the split tables are bit-identical.

  python tools/probe_operator_split.py [--rounds 30]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    args = ap.parse_args()
    bargs = bench.parse_args(["--config", "c7", "--no-cpu"])
    cfg = bench.CONFIGS["c7"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.Ctx(bargs, cfg[1], 0, 1, dev)
    wl = bench.OperatorWorkload(bargs, cfg, ctx)
    L, lib, P, N, E = wl.L, wl.lib, wl.P, wl.N, wl.E
    stream = torch.cuda.current_stream(dev)
    vp = lambda t, off=0: ctypes.c_void_p(t.data_ptr() + off)  # noqa: E731

    def parts_fn(parts):
        bounds = [(P * i // parts) // 128 * 128 for i in range(parts)] + [P]

        def f():
            for a0, a1 in zip(bounds[:-1], bounds[1:]):
                st = lib.rti_apply_operator_f16(vp(wl.hi), vp(wl.lo), wl.Kp, wl.inv, E, N, vp(wl.I, 4 * a0),
                                                L.RTI_F32, a1 - a0, 1, P, N * P, vp(wl.out, 4 * a0), L.RTI_I32, P,
                                                E * P, wl.stream)
                L.check(st, "rti_apply_operator_f16")
        return f

    variants = [(f"operator {p} launch(es)", parts_fn(p)) for p in (1, 2)]
    plib = os.path.join(ROOT, "tools", "probe", "libop_probe.so")
    if os.path.exists(plib):  # explicit row split gy: launches of T tiles x gy row groups (one generation ~ 512 WGs)
        probe = ctypes.CDLL(plib)
        probe.probe_op.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]

        def gen_fn(T, gy):
            def f():
                for a0 in range(0, P, 128 * T):
                    np_ = min(P - a0, 128 * T)
                    assert probe.probe_op(vp(wl.hi), vp(wl.lo), wl.Kp, wl.inv, E, N, vp(wl.I), P, a0, np_, gy,
                                          vp(wl.out), wl.stream) == 0
            return f
        for T, gy in ((1250, 2), (1250, 1), (256, 2), (512, 1), (128, 4), (250, 2), (625, 2)):
            variants.append((f"probe T={T} gy={gy}", gen_fn(T, gy)))
    ref = None
    for n, f in variants:
        wl.out.zero_()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        got = wl.out.clone()
        ref = got if ref is None else ref
        print(f"{n}: bit-identical to one launch: {torch.equal(got, ref)}", flush=True)
        del got
    ev = {n: [] for n, _ in variants}
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for j in rng.permutation(len(variants)):
            n, f = variants[j]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            f()
            b.record(stream)
            ev[n].append((a, b))
    torch.cuda.synchronize()
    for n, _ in variants:
        ms = np.array([a.elapsed_time(b) for a, b in ev[n]])
        print(f"{n:22s} median {np.median(ms):.4f} ms  min {ms.min():.4f}  "
              f"{wl.alg_bytes / np.median(ms) / 8e9:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
