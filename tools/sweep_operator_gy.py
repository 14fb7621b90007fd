#!/usr/bin/env python3
"""Interleaved A/B of the RBF table operator's E-split (c7, rti_apply_operator_f16): grid.y = the number of
row-block sweeps each 128-pixel tile is split over (RTI_OP_GY, read per call; AUTO = 2 at c7), in ONE process,
bench.py's OperatorWorkload step timed with HIP events; tables checked bit-identical to the first variant.

  python tools/sweep_operator_gy.py [--gy auto,1,4,8,16] [--rounds 20]
"""
import argparse
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
    ap.add_argument("--gy", default="auto,1,4,8,16")
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    bargs = bench.parse_args(["--config", "c7", "--no-cpu"])
    cfg = bench.CONFIGS["c7"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.Ctx(bargs, cfg[1], 0, 1, dev)
    wl = bench.OperatorWorkload(bargs, cfg, ctx)
    stream = torch.cuda.current_stream(dev)
    variants = args.gy.split(",")

    def run(v):  # "auto", a grid.y, "plain" (plain instead of non-temporal table stores) or "xcd" (r06: XCD-
        # contiguous tile order, RTI_OP_XCD=1)
        os.environ.pop("RTI_OP_PLAIN_STORES", None)
        os.environ.pop("RTI_OP_XCD", None)
        if v in ("auto", "plain", "xcd"):
            os.environ.pop("RTI_OP_GY", None)
            if v == "plain":
                os.environ["RTI_OP_PLAIN_STORES"] = "1"
            if v == "xcd":
                os.environ["RTI_OP_XCD"] = "1"
        else:
            os.environ["RTI_OP_GY"] = v
        wl.step(0)

    ref = None
    same = {}
    for v in variants:
        run(v)
        torch.cuda.synchronize()
        out = wl.out.clone() if ref is None else wl.out
        if ref is None:
            ref = out
        same[v] = bool(torch.equal(wl.out, ref))
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
        print(f"gy {v:>5s}: median {np.median(ms):.4f} ms  min {ms.min():.4f} ms  "
              f"{wl.alg_bytes / (np.median(ms) * 1e-3) / 8e12:.3f} of 8 TB/s  same tables {same[v]}", flush=True)


if __name__ == "__main__":
    main()
