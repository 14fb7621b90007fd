#!/usr/bin/env python3
"""c7 write-pattern probe: the int32 table stores of rti_apply_operator_f16 without compute
(tools/probe/store_probe.hip) timed next to the real c7 launch, interleaved in one process.

  python tools/sweep_store.py [--rounds 10] [--variants 0,1,2,3,4]
"""
import argparse
import ctypes
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--gy", type=int, default=1, help="variants 0-4: row-block split; 5-7: pixel segments")
    ap.add_argument("--segs", type=int, default=32, help="pixel segments of the row-sweep variants 5-7")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c7"]
    ns = types.SimpleNamespace(op_precision="split16", weak=False, config="c7")
    w = bench.OperatorWorkload(ns, cfg, bench.Ctx(ns, cfg[1], 0, 1, dev))
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libstore_probe.so"))
    lib.probe_store_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p]
    stream = torch.cuda.current_stream(dev)
    sink = torch.empty((w.E, w.P), dtype=torch.int32, device=dev)
    runs = [("c7_kernel", None)] + [(f"store_v{v}", int(v)) for v in args.variants.split(",")]

    def launch(v):
        if v is None:
            w.step(0)
        else:
            assert lib.probe_store_rows(ctypes.c_void_p(sink.data_ptr()), w.E, w.P, v, args.segs if v >= 5 else args.gy,
                                        ctypes.c_void_p(stream.cuda_stream)) == 0

    for name, v in runs:
        launch(v)
    torch.cuda.synchronize()
    times = {name: [] for name, _ in runs}
    for _ in range(args.rounds):
        for name, v in runs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            launch(v)
            b.record(stream)
            times[name].append((a, b))
    torch.cuda.synchronize()
    byts = 4.0 * w.E * w.P
    for name, _ in runs:
        ms = np.array([a.elapsed_time(b) for a, b in times[name]])
        gbs = byts / (np.median(ms) * 1e-3) / 1e9
        print(f"{name:12s} median {np.median(ms):.4f} ms  min {ms.min():.4f} ms  table write rate {gbs:.0f} GB/s "
              f"({gbs / 80:.1f}%)", flush=True)


if __name__ == "__main__":
    main()
