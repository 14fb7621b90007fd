#!/usr/bin/env python3
"""Merge the PMC traffic entries a GPU run wrote (gpurun_out/traffic.json, tools/pmc_pass.sh) into
profiles/traffic.json, stamping each with the commit its kernel sources were measured at: the entry's
src_sha16 must equal the hash of the same files in this tree (else the entry is refused), and `commit`
is this tree's HEAD (with "+dirty" when those files differ from HEAD).

  python tools/merge_traffic.py [gpurun_out/traffic.json] [profiles/traffic.json]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "traffic.json")
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "traffic.json")
    new = json.load(open(src))
    data = json.load(open(dst)) if os.path.exists(dst) else {}
    head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                          text=True).stdout.strip()
    for key, e in new.items():
        files = e.get("sources")
        if not files or bench.sources_sha16(files) != e.get("src_sha16"):
            print(f"refused {key}: its kernel sources changed since the PMC pass")
            continue
        dirty = subprocess.run(["git", "diff", "--quiet", "HEAD", "--"] + files, cwd=ROOT).returncode != 0
        e["commit"] = head + ("+dirty" if dirty else "")
        data[key] = e
        print(f"merged {key}: {e.get('kernel_symbol', '?')[:80]} traffic/alg {e.get('traffic_over_alg')}")
    with open(dst, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
