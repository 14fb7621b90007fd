#!/usr/bin/env python3
"""Median per-dispatch counter values of tools/pmc_sq.sh passes: python3 tools/summarize_sq.py KEY [KEY ...]"""
import csv
import glob
import os
import statistics
import sys

for key in sys.argv[1:]:
    vals = {}
    for f in glob.glob(os.path.join("gpurun_out", f"pmcsq_{key}", "*", "*counter_collection.csv")):
        per = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per.setdefault((row["Counter_Name"], row["Dispatch_Id"]), 0.0)
                per[(row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
        for (name, _), v in per.items():
            vals.setdefault(name, []).append(v)
    med = {k: statistics.median(v) for k, v in vals.items()}
    print(key)
    for k in sorted(med):
        print(f"  {k:28s} {med[k]:.4g}")
    w = med.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in med:
                print(f"  {k} / WAVE_CYCLES = {med[k] / w:.3f}")
