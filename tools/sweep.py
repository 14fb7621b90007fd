#!/usr/bin/env python3
"""Interleaved A/B timing of fit-kernel variants in ONE process (methodology
rule 24): every round runs each variant once, HIP events around each launch;
reports median / min kernel time and GB/s (algorithmic bytes) per variant,
plus the pure read-stream ceiling from tools/probe/libhbm_probe.so.

  python tools/sweep.py [--config c3] [--rounds 30]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--variants", default="valu:pixel,valu:pixel:nt,valu:pixel:nt+lds,valu:pixel:nt+stage,"
                    "valu:pixel:nt+lds+stage,valu:pixel:nt+stage+nts,valu:pixel:nt+lds+stage+nts,"
                    "valu:planar:nt,valu:planar:nt+nts,valu:planar:nt+lds+nts,valu:planar:nt+lds,"
                    "mfma:planar:nt,mfma:pixel:nt")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--store-windows", default="", help="PTM-6 store probe wrapping its stores inside W MiB (list)")
    ap.add_argument("--rows", type=int, default=0, help="override the config's H (row-shard sizes: 2160/G)")
    ap.add_argument("--in-dtype", default="f32", choices=["f32", "u8", "i32"], help="intensity stack type")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _, H, W, N, C, basis, desc = bench.CONFIGS[args.config]
    H = args.rows or H
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev)
    if args.in_dtype != "f32":  # integer-valued 0..255 stacks, as the reference's V channel
        I = I.to(torch.uint8 if args.in_dtype == "u8" else torch.int32)
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    op_dev = torch.as_tensor(rti.q8_operator(rti.pinv(lu, lv, basis)), device=dev) if args.in_dtype == "u8" else None
    h16_dev = torch.as_tensor(rti.api.h16_operator(rti.pinv(lu, lv, basis)), device=dev) \
        if args.in_dtype == "u8" else None
    coefs = {"pixel": torch.empty((C, P, k), device=dev), "planar": torch.empty((C, k, P), device=dev)}
    variants = []
    for v in args.variants.split(","):
        parts = v.split(":")
        opts = parts[2].split("+") if len(parts) > 2 else []
        fl = (rti._lib.RTI_KERNEL_NONTEMPORAL if "nt" in opts else 0) | \
             (rti._lib.RTI_KERNEL_PINV_LDS if "lds" in opts else 0) | \
             (rti._lib.RTI_KERNEL_NT_STORE if "nts" in opts else 0) | (rti._lib.RTI_KERNEL_STAGE if "stage" in opts else 0) | \
             (rti._lib.RTI_KERNEL_ONE_LAUNCH if "one" in opts else 0) | \
             (rti._lib.RTI_KERNEL_ROUNDS if "rounds" in opts else 0)
        for o in opts:  # c<n>: chunks per lane (rti.h RTI_KERNEL_CHUNKS)
            if o[:1] == "c" and o[1:].isdigit():
                fl |= int(o[1:]) << 12
            if o[:1] == "t" and o[1:].isdigit():  # t<sp>: TILE kernel planes per wave and step
                fl |= int(o[1:]) << 16
            if o[:1] == "d" and o[1:].isdigit():  # d<n>: TILE kernel LDS ring depth
                fl |= int(o[1:]) << 20
            if o[:1] == "w" and o[1:].isdigit():  # w<n>: TILE kernel waves per workgroup
                fl |= int(o[1:]) << 24
        variants.append((v, parts[0], parts[1], fl))
    probe = None
    plib = os.path.join(ROOT, "tools", "probe", "libhbm_probe.so")
    tlib = os.path.join(ROOT, "tools", "probe", "libtile_probe.so")
    if os.path.exists(tlib) and k == 16 and not args.no_probe:
        # the probe includes rti_fit.hip and resolves librti's host helpers (rti::fail, ...) from it
        ctypes.CDLL(os.path.join(ROOT, "smartphone-based-rti_amd", "rti", "librti.so"),
                    mode=os.RTLD_NOW | os.RTLD_GLOBAL)
        tprobe = ctypes.CDLL(tlib)
        tprobe.probe_tile_nostore.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        variants.append(("probe_tile_nostore", "ptile", "0", 0))
    if os.path.exists(plib) and not args.no_probe:
        probe = ctypes.CDLL(plib)
        probe.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p]
        probe.probe_fit6.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        sink = torch.zeros(1, device=dev)
        for pvnt in (0, 1, 2, 3, 4):  # C channels = C*N light planes of one [C*N][P] stack
            variants.append((f"probe_read_v{pvnt}", "probe", str(pvnt), 0))
        probe.probe_store.argtypes = probe.probe_fit6.argtypes
        probe.probe_write.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        variants.append(("probe_write_coef_bytes", "pwrite", "0", 0))
        if k == 6 and C == 1:
            for pvnt, nm in ((1, "nostore"),):
                variants.append((f"probe_fit6_{nm}", "pfit", str(pvnt), 0))
            for pvnt, nm in ((0, "plain"), (4, "win64K")):
                variants.append((f"probe_store_{nm}", "pstore", str(pvnt), 0))
            for mib in filter(None, args.store_windows.split(",")):
                variants.append((f"probe_store_win{mib}M", "pstore", str(100 + int(mib)), 0))
            probe.probe_persist.argtypes = probe.probe_fit6.argtypes
            for v in (1256, 1512, 2256, 2512, 3256, 1768, 2384):
                variants.append((f"probe_persist_F{v // 1000}_wg{v % 1000}", "ppersist", str(v), 0))
    stream = torch.cuda.current_stream(dev)
    times = {name: [] for name, *_ in variants}

    def launch(kern, layout, fl):
        if kern == "probe":
            probe.probe_read(ctypes.c_void_p(I.data_ptr()), N * C, P, ctypes.c_void_p(sink.data_ptr()), int(layout),
                             ctypes.c_void_p(stream.cuda_stream))
        elif kern == "ptile":
            tprobe.probe_tile_nostore(ctypes.c_void_p(pv.data_ptr()), k, N, ctypes.c_void_p(I.data_ptr()), P, C,
                                      ctypes.c_void_p(coefs["pixel"].data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        elif kern == "pwrite":
            probe.probe_write(ctypes.c_void_p(coefs["pixel"].data_ptr()), 4 * P * k * C,
                              ctypes.c_void_p(stream.cuda_stream))
        elif kern == "ppersist":
            probe.probe_persist(ctypes.c_void_p(pv.data_ptr()), ctypes.c_void_p(I.data_ptr()), N, P,
                                ctypes.c_void_p(coefs["pixel"].data_ptr()), int(layout),
                                ctypes.c_void_p(stream.cuda_stream))
        elif kern == "pstore":
            tgt = coefs["planar"] if layout in ("5", "8") else coefs["pixel"]
            probe.probe_store(ctypes.c_void_p(pv.data_ptr()), ctypes.c_void_p(I.data_ptr()), N, P,
                              ctypes.c_void_p(tgt.data_ptr()), int(layout), ctypes.c_void_p(stream.cuda_stream))
        elif kern == "pfit":
            probe.probe_fit6(ctypes.c_void_p(pv.data_ptr()), ctypes.c_void_p(I.data_ptr()), N, P,
                             ctypes.c_void_p(coefs["pixel"].data_ptr()), int(layout), ctypes.c_void_p(stream.cuda_stream))
        elif kern == "h16":
            rti.api.fit_h16_into(h16_dev, I, coefs[layout], k=k, layout=layout, flags=fl)
        elif kern == "q8":
            rti.api.fit_q8_into(op_dev, I, coefs[layout], k=k, layout=layout, flags=fl)
        else:
            rti.fit_shared_into(pv, I, coefs[layout], k=k, layout=layout, kernel=kern, flags=fl)

    agree = {}  # every library variant's coefficients against the first library variant's
    ref = None
    for name, kern, layout, fl in variants:  # warm-up
        for _ in range(3):
            launch(kern, layout, fl)
        if kern in ("valu", "mfma", "tile", "auto", "q8", "h16"):
            got = coefs[layout] if layout == "pixel" else coefs[layout].transpose(1, 2)
            got = got.double()
            if ref is None:
                ref = got.clone()
            scale = ref.abs().amax(-1, keepdim=True).clamp_min(1e-30)
            agree[name] = float(((got - ref).abs() / scale).max())
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, kern, layout, fl in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            launch(kern, layout, fl)
            b.record(stream)
            times[name].append((a, b))
    torch.cuda.synchronize()
    es = I.element_size()
    alg = es * P * N * C + 4.0 * P * k * C
    res = {}
    for name, *rest in variants:
        ms = np.array([a.elapsed_time(b) for a, b in times[name]])
        byts = 4.0 * P * N * C if name.startswith(("probe_read", "probe_tile_nostore")) else \
            (4.0 * P * k * C if name.startswith("probe_write") else alg)
        res[name] = {"median_ms": float(np.median(ms)), "min_ms": float(ms.min()),
                     "GBps_median": byts / (np.median(ms) * 1e-3) / 1e9}
        if name in agree:
            res[name]["max_rel_vs_first"] = agree[name]
        print(f"{name:24s} median {np.median(ms):.4f} ms  min {ms.min():.4f} ms  "
              f"{res[name]['GBps_median']:.0f} GB/s ({res[name]['GBps_median'] / 80:.1f}% of 8 TB/s)"
              + (f"  rel {agree[name]:.1e}" if name in agree else ""), flush=True)
    print(json.dumps({"config": args.config, "results": res}))


if __name__ == "__main__":
    main()
