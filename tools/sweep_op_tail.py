#!/usr/bin/env python3
"""Does the c7 table operator (rti_apply_operator_f16, E = 10⁴ int32 tables, N = 100) lose time to a partial
last round of workgroups?  c7's 400² image is 1250 tiles of 128 pixels = 2.44 rounds of 512 resident
workgroups; this times pixel counts of whole and partial rounds (HIP events, one process, median of
--rounds, the split-fp16 launch only — the operator is split once outside the timed region) and reports
table bytes per second.

  python tools/sweep_op_tail.py [--tiles 1024,1250,1280,1536] [--rounds 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rti  # noqa: E402
from rti import _lib as L  # noqa: E402
from rti.api import _vp, _stream_of, split_operator_f16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1024,1250,1280,1536")
    ap.add_argument("--rounds", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    E, N = 10000, 100
    rng = np.random.default_rng(0)
    opT = rng.standard_normal((N, E)) * 0.05
    hi, lo, Kp, inv = split_operator_f16(opT, dev)
    runs = []
    for t in [int(x) for x in args.tiles.split(",")]:
        P = 128 * t
        I = torch.as_tensor(rng.integers(0, 256, (N, P)).astype(np.float32), device=dev)
        out = torch.empty((E, P), dtype=torch.int32, device=dev)

        def fn(I=I, out=out, P=P):
            st = L.lib().rti_apply_operator_f16(_vp(hi), _vp(lo), Kp, inv, E, N, _vp(I), L.RTI_F32, P, 1, P, N * P,
                                                _vp(out), L.RTI_I32, P, E * P, _stream_of(I))
            L.check(st, "rti_apply_operator_f16")
        runs.append((t, P, fn))
    for _, _, fn in runs:
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    times = {t: [] for t, _, _ in runs}
    for _ in range(args.rounds):
        for t, _, fn in runs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            times[t].append((a, b))
        torch.cuda.synchronize()
    for t, P, _ in runs:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[t]]))
        alg = 4.0 * E * P + 4.0 * N * P
        print(f"tiles={t:5d} ({t / 512:.2f} rounds of 512)  P={P}  {ms:.4f} ms  {alg / ms / 1e9:.3f} TB/s  "
              f"{1e3 * ms / t:.3f} us per tile", flush=True)


if __name__ == "__main__":
    main()
