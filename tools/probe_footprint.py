#!/usr/bin/env python3
"""Does the stack's address-space footprint slow the HBM stream?  (c4 question: the HSH-16 stack is
19.9 GB, the c3 PTM stack 3.3 GB, and c4's reads run ≈5 % below c3's per byte.)

Same bytes, same kernel, different footprints, interleaved in ONE process (HIP events per launch):
  c3 shape (P = 4K, N = 100, PTM-6 AUTO) with light_stride = P (3.3 GB), 2P, 6P (20 GB) and P + 1 MiB;
  c4 shape (C = 3, N = 200, HSH-16 AUTO) as one launch vs three one-channel launches, and one channel alone.

  python tools/probe_footprint.py [--rounds 20]
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
from rti import _lib as L  # noqa: E402


def vp(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--only", default="", help="comma-separated variant-name prefixes")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    pr = torch.cuda.get_device_properties(dev)
    print(f"device: {pr.name} {pr.gcnArchName} CUs {pr.multi_processor_count} mem {pr.total_memory >> 30} GiB", flush=True)
    lib = L.lib()
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    H, W = 2160, 3840
    P = H * W
    # one 20 GB arena: fp32 [6P * 100 + slack]
    N3 = 100
    arena = torch.empty(6 * P * N3 + (1 << 20) * N3, dtype=torch.float32, device=dev)
    arena.uniform_(0, 255)
    lu, lv = bench.synth_dirs(N3, 2)
    pv6 = torch.as_tensor(rti.pinv(lu, lv, "ptm").astype(np.float32), device=dev)
    coef6 = torch.empty((P, 6), device=dev)
    N4, C4 = 200, 3
    lu4, lv4 = bench.synth_dirs(N4, 2)
    pv16 = torch.as_tensor(rti.pinv(lu4, lv4, "hsh16").astype(np.float32), device=dev)
    coef16 = torch.empty((C4, P, 16), device=dev)
    auto = 0
    ROT = 0x10000000  # rti.h RTI_KERNEL_ROTATE
    ONE = 0x20000000  # rti.h RTI_KERNEL_ONE_LAUNCH

    def c3(stride, kern=0):
        def f():
            st = lib.rti_fit_shared(vp(pv6), 6, N3, vp(arena), 0, P, 1, stride, N3 * stride, vp(coef6), 0, P * 6,
                                    kern, sp)
            assert st == 0, st
        return f

    def c4_one(kern=ONE):
        def f():
            st = lib.rti_fit_shared(vp(pv16), 16, N4, vp(arena), 0, P, C4, P, N4 * P, vp(coef16), 0, P * 16, kern, sp)
            assert st == 0, st
        return f

    def c3_rows(rows, kern=0):  # a row shard of the 4K image (8-GPU strong scaling: 270 / 540 / 1080 rows)
        def f():
            st = lib.rti_fit_shared(vp(pv6), 6, N3, vp(arena), 0, rows * W, 1, rows * W, N3 * rows * W, vp(coef6), 0,
                                    0, kern, sp)
            assert st == 0, st
        return f

    def c4_split():
        for c in range(C4):
            st = lib.rti_fit_shared(vp(pv16), 16, N4, ctypes.c_void_p(arena.data_ptr() + 4 * c * N4 * P), 0, P, 1, P,
                                    N4 * P, ctypes.c_void_p(coef16.data_ptr() + 4 * c * P * 16), 0, P * 16, ONE, sp)
            assert st == 0, st

    def c4_pad():
        st = lib.rti_fit_shared(vp(pv16), 16, N4, vp(arena), 0, P, C4, P, N4 * P + (1 << 18), vp(coef16), 0, P * 16,
                                ONE, sp)
        assert st == 0, st

    def c4_ch0():
        st = lib.rti_fit_shared(vp(pv16), 16, N4, vp(arena), 0, P, 1, P, N4 * P, vp(coef16), 0, P * 16, ONE, sp)
        assert st == 0, st

    def c3_parts(parts, kern=0):  # the image's pixels as `parts` consecutive launches (one plane stride P)
        bounds = [(P * i // parts) // 1024 * 1024 for i in range(parts)] + [P]

        def f():
            for a0, a1 in zip(bounds[:-1], bounds[1:]):
                st = lib.rti_fit_shared(vp(pv6), 6, N3, ctypes.c_void_p(arena.data_ptr() + 4 * a0), 0, a1 - a0, 1, P,
                                        N3 * P, ctypes.c_void_p(coef6.data_ptr() + 4 * 6 * a0), 0, 0, kern | ONE, sp)
                assert st == 0, st
        return f

    def c4_parts(tiles_per_launch):  # every channel as launches of `tiles_per_launch` 4096-pixel tiles
        step = 4096 * tiles_per_launch

        def f():
            for c in range(C4):
                for a0 in range(0, P, step):
                    a1 = min(P, a0 + step)
                    st = lib.rti_fit_shared(vp(pv16), 16, N4, ctypes.c_void_p(arena.data_ptr() + 4 * (c * N4 * P + a0)),
                                            0, a1 - a0, 1, P, N4 * P,
                                            ctypes.c_void_p(coef16.data_ptr() + 4 * 16 * (c * P + a0)), 0, 0, ONE, sp)
                    assert st == 0, st
        return f

    b3 = 4.0 * P * N3 + 4.0 * P * 6
    b4 = (4.0 * P * N4 + 4.0 * P * 16) * C4
    br = lambda rows: 4.0 * rows * W * (N3 + 6)  # noqa: E731
    variants = [("c3 AUTO", c3(P), b3), ("c3 ONE_LAUNCH", c3(P, ONE), b3), ("c4 AUTO", c4_one(0), b4),
                ("c4 ONE_LAUNCH", c4_one(ONE), b4),
                ("rows1080 AUTO", c3_rows(1080), br(1080)), ("rows1080 ONE_LAUNCH", c3_rows(1080, ONE), br(1080)),
                ("rows540 AUTO", c3_rows(540), br(540)), ("rows540 ONE_LAUNCH", c3_rows(540, ONE), br(540)),
                ("rows270 AUTO", c3_rows(270), br(270)), ("rows270 ONE_LAUNCH", c3_rows(270, ONE), br(270)),
                ("c3 stride P (3.3 GB)", c3(P, ONE), b3), ("c3 stride P+1MiB", c3(P + (1 << 18), ONE), b3),
                ("c3 stride P+4KiB", c3(P + 1024, ONE), b3), ("c3 stride P+64KiB", c3(P + (1 << 14), ONE), b3),
                ("c3 stride P+2KiB", c3(P + 512, ONE), b3), ("c3 stride P+256B", c3(P + 64, ONE), b3),
                ("c3 stride 6P (20 GB)", c3(6 * P, ONE), b3),
                ("c3 rotated lights", c3(P, ROT | ONE), b3), ("c3 rotated lights P+4KiB", c3(P + 1024, ROT | ONE), b3),
                ("c4 one launch C=3", c4_one(), b4), ("c4 three C=1 launches", c4_split, b4),
                ("c4 C=3 cstride+1MiB", c4_pad, b4), ("c4 channel 0 only", c4_ch0, b4 / C4),
                ("c3 2 launches", c3_parts(2), b3), ("c3 4 launches", c3_parts(4), b3),
                ("c3 3 launches", c3_parts(3), b3), ("c3 5 launches", c3_parts(5), b3),
                ("c3 6 launches", c3_parts(6), b3), ("c3 8 launches", c3_parts(8), b3),
                ("c3 8 launches NC8", c3_parts(8, 8 << 12), b3), ("c3 4 launches NC4", c3_parts(4, 4 << 12), b3),
                ("c3 2 launches NC8", c3_parts(2, 8 << 12), b3), ("c3 4 launches NC8", c3_parts(4, 8 << 12), b3),
                ("c3 8 launches NC4", c3_parts(8, 4 << 12), b3), ("c3 8 launches NC2", c3_parts(8, 2 << 12), b3),
                ("c3 16 launches NC2", c3_parts(16, 2 << 12), b3), ("c3 1 launch NC4", c3_parts(1, 4 << 12), b3),
                ("c4 1350-tile launches", c4_parts(1350), b4), ("c4 768-tile launches", c4_parts(768), b4),
                ("c4 675-tile launches", c4_parts(675), b4),
                ("c4 1012-tile launches", c4_parts(1013), b4), ("c4 512-tile launches", c4_parts(512), b4),
                ("c4 256-tile launches", c4_parts(256), b4)]
    if args.only:
        variants = [v for v in variants if v[0].startswith(tuple(args.only.split(",")))]
    for _, f, _ in variants:
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    ev = {n: [] for n, _, _ in variants}
    rng = np.random.default_rng(0)
    for _ in range(args.rounds):
        for i in rng.permutation(len(variants)):  # shuffled order every round
            n, f, _ = variants[i]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            f()
            b.record(stream)
            ev[n].append((a, b))
    torch.cuda.synchronize()
    for n, _, byts in variants:
        ms = np.array([a.elapsed_time(b) for a, b in ev[n]])
        print(f"{n:26s} median {np.median(ms):.4f} ms  min {ms.min():.4f}  "
              f"{byts / np.median(ms) / 1e6:.0f} GB/s = {byts / np.median(ms) / 8e9:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
