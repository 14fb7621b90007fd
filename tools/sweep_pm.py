#!/usr/bin/env python3
"""Pixel-major shared fit (rti_fit_shared_pm) variants next to the light-major AUTO fit of the same
values, interleaved in ONE process (HIP events per launch, median of --rounds): the VALU generations
form (AUTO for k <= 9) at W waves per CU, forced generation counts and contiguous runs, the MFMA stream
("mfma") and block form ("tile"), the direct form, and (tools/probe/libpm_probe.so, when built) the
generations kernel with its stores dropped.

  python tools/sweep_pm.py --config c3|c4|c2 [--rounds 20] [--waves 2,3,4,6,8] [--blocks 1,2,4]
"""
import argparse
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
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--waves", default="2,3,4,6,8")
    ap.add_argument("--blocks", default="1,2")
    ap.add_argument("--in-dtype", default="f32", choices=["f32", "i32"])
    ap.add_argument("--gens", default="6,8,12", help="VALU generations: launches per channel forced (CHUNKS)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = rti._lib
    _, H, W, N, C, basis, _ = bench.CONFIGS[args.config]
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = bench.synth_dirs(N, 2)
    I = bench.synth_stack(H, W, N, C, basis, lu, lv, 1000, dev)
    if args.in_dtype == "i32":
        I = I.to(torch.int32)
    Ipm = I.transpose(1, 2).contiguous()  # [C, P, N]
    pv = torch.as_tensor(rti.pinv(lu, lv, basis).astype(np.float32), device=dev)
    coef = torch.empty((C, P, k), device=dev)
    ref = torch.empty((C, P, k), device=dev)
    variants = [("light_major_auto", lambda: rti.fit_shared_into(pv, I, ref, k=k, layout="pixel", kernel="auto"))]
    for w in [int(x) for x in args.waves.split(",") if x]:
        fl = w << L.RTI_KERNEL_TILE_WAVES_SHIFT
        plan = L.lib().rti_fit_shared_pm_plan(k, N, rti.api._IN_DTYPES[I.dtype], P, C, N, P * N, fl | L.RTI_KERNEL_MFMA)
        if plan:
            variants.append((f"pm_stream_w{w}_ring{plan % 100000000 // 1000}K",
                             lambda fl=fl: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="mfma", flags=fl)))
        if plan and w == 8:
            for u in (2, 4):
                flu = fl | (u << L.RTI_KERNEL_CHUNKS_SHIFT)
                variants.append((f"pm_stream_w{w}_unit{u}",
                                 lambda flu=flu: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="mfma", flags=flu)))
            fln = fl | L.RTI_KERNEL_NT_STORE
            variants.append((f"pm_stream_w{w}_nts",
                             lambda fln=fln: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="mfma", flags=fln)))
            flc = fl | L.RTI_KERNEL_ROTATE
            variants.append((f"pm_stream_w{w}_contiguous",
                             lambda flc=flc: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="mfma", flags=flc)))
    for g in [int(x) for x in args.blocks.split(",") if x]:
        fl = g << L.RTI_KERNEL_CHUNKS_SHIFT
        plan = L.lib().rti_fit_shared_pm_plan(k, N, rti.api._IN_DTYPES[I.dtype], P, C, N, P * N, fl | L.RTI_KERNEL_TILE)
        if plan:
            variants.append((f"pm_block_{plan % 100000000 // 1000}px_w{plan % 1000}",
                             lambda fl=fl: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="tile", flags=fl)))
    direct = [(f"pm_direct_{w}wpc", w << L.RTI_KERNEL_TILE_WAVES_SHIFT) for w in (4, 8, 12)]
    direct += [(f"pm_direct_gens{g}", g << L.RTI_KERNEL_CHUNKS_SHIFT) for g in (2, 4, 6, 11, 15)]
    direct += [(f"pm_direct_gens{g}_12wpc", (g << L.RTI_KERNEL_CHUNKS_SHIFT) | (12 << 24)) for g in (7, 14)]
    direct += [("pm_direct_nts", L.RTI_KERNEL_NT_STORE), ("pm_direct_nts_12wpc", L.RTI_KERNEL_NT_STORE | (12 << 24))]
    for name, fl in direct:
        fl |= L.RTI_KERNEL_STAGE  # the direct form for every k
        plan = L.lib().rti_fit_shared_pm_plan(k, N, rti.api._IN_DTYPES[I.dtype], P, C, N, P * N, fl)
        if plan // 100000000 == L.RTI_PM_DIRECT:
            variants.append((name, lambda fl=fl: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="auto", flags=fl)))
    for w in (6, 5, 4):
        fl = w << L.RTI_KERNEL_TILE_WAVES_SHIFT
        plan = L.lib().rti_fit_shared_pm_plan(k, N, rti.api._IN_DTYPES[I.dtype], P, C, N, P * N, fl)
        if plan // 100000000 == L.RTI_PM_VALU_STREAM:
            variants.append((f"pm_vgen_w{w}_ring{plan % 100000000 // 1000}K",
                             lambda fl=fl: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="auto", flags=fl)))
    if k <= 9:  # more (smaller) launch generations than AUTO's
        for g in [int(x) for x in args.gens.split(",") if x]:
            fl = g << L.RTI_KERNEL_CHUNKS_SHIFT
            variants.append((f"pm_vgen_gens{g}",
                             lambda fl=fl: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="auto", flags=fl)))
    variants.append(("pm_auto", lambda: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="auto")))
    if k <= 9:  # each wave one contiguous run of blocks instead of interleaved units
        variants.append(("pm_vgen_contig", lambda: rti.api.fit_shared_pm_into(pv, Ipm, coef, k=k, kernel="auto",
                                                                            flags=L.RTI_KERNEL_ROTATE)))
    probe = os.path.join(ROOT, "tools", "probe", "libpm_probe.so")
    if k == 6 and C == 1 and N % 4 == 0 and I.dtype == torch.float32 and os.path.exists(probe):
        # tools/probe/pm_probe.hip: the library's generation kernel built with its stores dropped
        import ctypes
        plib = ctypes.CDLL(probe)
        vp = ctypes.c_void_p

        def pr(mode):
            st = plib.pm_probe_vgen(vp(pv.data_ptr()), N, vp(Ipm.data_ptr()), ctypes.c_int64(P), vp(coef.data_ptr()),
                                    0, 0, mode, vp(torch.cuda.current_stream(dev).cuda_stream))
            assert st == 0, st
        variants.append(("probe_vgen_same", lambda: pr(0)))
        variants.append(("probe_vgen_nostores", lambda: pr(1)))
        variants.append(("probe_vgen_contig_nostores", lambda: pr(3)))
    if k == 16 and I.dtype == torch.float32 and os.path.exists(probe):
        # tools/probe/pm_probe.hip: the library's direct form at HSH-16 with its burst stores dropped
        import ctypes
        plib = ctypes.CDLL(probe)
        vp = ctypes.c_void_p

        def prd(mode):
            st = plib.pm_probe_direct(vp(pv.data_ptr()), N, vp(Ipm.data_ptr()), ctypes.c_int64(P), C,
                                      vp(coef.data_ptr()), mode, vp(torch.cuda.current_stream(dev).cuda_stream))
            assert st == 0, st
        for name, mode in (("same", 0), ("nostores", 1), ("nts", 4), ("phase20", 2), ("phase20_nts", 6),
                           ("phase10x2", 8), ("phase10x2_nts", 12), ("phase20_nostores", 3)):
            variants.append((f"probe_direct_{name}", lambda mode=mode: prd(mode)))
    agree = {}
    for name, fn in variants:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if name not in ("light_major_auto", "probe_vgen_nostores", "probe_vgen_contig_nostores",
                        "probe_direct_nostores", "probe_direct_phase20_nostores"):
            scale = ref.abs().amax(-1, keepdim=True).clamp_min(1e-30)
            agree[name] = float(((coef - ref).abs() / scale).max())
            coef.fill_(float("nan"))
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
    alg = 4.0 * P * N * C + 4.0 * P * k * C
    res = {}
    for name, _ in variants:
        ms = float(np.median([a.elapsed_time(b) for a, b in times[name]]))
        gbs = alg / (ms * 1e-3) / 1e9
        res[name] = {"median_ms": ms, "GBps": gbs, "frac_8TBps": gbs / 8000.0, "max_rel_vs_light": agree.get(name)}
        print(f"{name:28s} {ms:.4f} ms  {gbs:.0f} GB/s ({gbs / 8000:.3f} of 8 TB/s)"
              + (f"  rel {agree[name]:.1e}" if name in agree else ""), flush=True)
    print(json.dumps({"config": args.config, "alg_bytes": alg, "results": res}))


if __name__ == "__main__":
    main()
