#!/usr/bin/env python3
"""Summarise rocprofv3 output for one kernel: average duration from the
kernel-trace pass and HBM traffic per launch from separate FETCH_SIZE and
WRITE_SIZE --pmc passes, with the gfx950 correction of MI355X_MICROARCH.md
§HBM (FETCH_SIZE reports half of a wide coalesced read stream: ×2;
units are KiB: ×1024).

  python tools/summarize_prof.py --trace DIR --fetch DIR --write DIR --kernel REGEX
        --key WORKLOAD --alg-bytes B (per bench step) [--launches-per-step L] [--out profiles/traffic.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_sources / sources_sha16: the provenance bench.py checks)


def rows(d, suffix):
    out = []
    for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--alg-bytes", type=float, required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--launches-per-step", type=int, default=1,
                    help="kernel launches per bench step (launch generations): per-step figures = per-launch x L")
    args = ap.parse_args()
    rx = re.compile(args.kernel)
    L = args.launches_per_step
    summary = {"kernel_regex": args.kernel, "alg_bytes_per_launch": args.alg_bytes / L, "launches_per_step": L,
               "alg_bytes_per_step": args.alg_bytes}
    if args.trace:
        trace = [r for r in rows(args.trace, "kernel_trace.csv") if rx.search(r["Kernel_Name"])]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
        if durs:
            summary["launches"] = len(durs)
            summary["avg_duration_ns"] = sum(durs) / len(durs)
            # provenance (bench.py load_traffic): the profiled kernel's symbol (most launches) and a hash of the
            # source files that define it; bench reports this traffic only while those files are unchanged
            names = collections.Counter(r["Kernel_Name"] for r in trace)
            summary["kernel_symbol"] = names.most_common(1)[0][0]
    files = bench.kernel_sources(args.kernel)
    if files:
        summary["sources"] = files
        summary["src_sha16"] = bench.sources_sha16(files)
    for name, d, corr in (("FETCH_SIZE", args.fetch, 2.0), ("WRITE_SIZE", args.write, 1.0)):
        if not d:
            continue
        vals = [float(r["Counter_Value"]) for r in rows(d, "counter_collection.csv")
                if rx.search(r["Kernel_Name"]) and r["Counter_Name"] == name]
        if vals:
            summary[name + "_KiB_raw_avg"] = sum(vals) / len(vals)
            summary[name + "_bytes_corrected"] = sum(vals) / len(vals) * 1024 * corr
    if "FETCH_SIZE_bytes_corrected" in summary and "WRITE_SIZE_bytes_corrected" in summary:
        summary["traffic_bytes_per_launch"] = summary["FETCH_SIZE_bytes_corrected"] + \
            summary["WRITE_SIZE_bytes_corrected"]
        summary["traffic_bytes_per_step"] = summary["traffic_bytes_per_launch"] * L
        summary["traffic_over_alg"] = summary["traffic_bytes_per_step"] / args.alg_bytes
    data = {}
    if os.path.exists(args.out):
        with open(args.out) as fh:
            data = json.load(fh)
    data[args.key] = summary
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
