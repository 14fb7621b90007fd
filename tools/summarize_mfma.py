#!/usr/bin/env python3
"""Summarise a matrix-core utilisation pass for one kernel.

Counters (one --pmc pass): SQ_VALU_MFMA_BUSY_CYCLES (cycles a SIMD's matrix core is busy,
summed over the chip) and GRBM_GUI_ACTIVE (GPU active clock, summed over the 8 XCDs, so
÷8 is the per-XCD kernel clock count; MI355X_MICROARCH.md, "DVFS give-back").

  mfma_busy_frac    = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 × 256 CUs × 4 SIMDs)
  expected_busy     = n_mfma × cycles_per_mfma   (the kernel's MFMA count, from its tiling)
  effective_clock   = GRBM_GUI_ACTIVE/8 / kernel duration

The expected-vs-counted ratio checks the normalisation; the busy fraction is the
"MFMA utilisation against gfx950 peak" that BASELINE.json's north_star asks for.

  python tools/summarize_mfma.py --trace DIR --pmc DIR --kernel REGEX --key WORKLOAD
        --n-mfma N --cycles-per-mfma C [--out profiles/mfma.json]
"""
import argparse
import json
import os
import re

from summarize_prof import rows

CUS, SIMDS_PER_CU, XCDS = 256, 4, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--n-mfma", type=float, required=True)
    ap.add_argument("--cycles-per-mfma", type=float, required=True)
    ap.add_argument("--out", default="profiles/mfma.json")
    args = ap.parse_args()
    rx = re.compile(args.kernel)
    s = {"kernel_regex": args.kernel, "n_mfma_per_launch": args.n_mfma,
         "cycles_per_mfma": args.cycles_per_mfma}
    if args.trace:
        tr = [r for r in rows(args.trace, "kernel_trace.csv") if rx.search(r["Kernel_Name"])]
        if tr:
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
            s["kernel"] = tr[0]["Kernel_Name"]
            s["launches"] = len(durs)
            s["avg_duration_ns"] = sum(durs) / len(durs)
    by = {}
    for r in rows(args.pmc, "counter_collection.csv"):
        if rx.search(r["Kernel_Name"]):
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for name, vals in by.items():
        s[name + "_avg"] = sum(vals) / len(vals)
    busy, gui = s.get("SQ_VALU_MFMA_BUSY_CYCLES_avg"), s.get("GRBM_GUI_ACTIVE_avg")
    if busy is not None and gui:
        per_xcd = gui / XCDS
        s["mfma_busy_frac"] = busy / (per_xcd * CUS * SIMDS_PER_CU)
        s["expected_busy_cycles"] = args.n_mfma * args.cycles_per_mfma
        s["counted_over_expected"] = busy / s["expected_busy_cycles"]
        if "avg_duration_ns" in s:
            s["effective_clock_ghz_profiled"] = per_xcd / s["avg_duration_ns"]
    data = {}
    if os.path.exists(args.out):
        with open(args.out) as fh:
            data = json.load(fh)
    data[args.key] = s
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps(s, indent=1))


if __name__ == "__main__":
    main()
