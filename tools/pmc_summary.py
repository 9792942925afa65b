#!/usr/bin/env python3
"""Condense rocprofv3 CSV output (tools/profile.sh) into per-kernel averages.

    python tools/pmc_summary.py gpurun_out prof_r01 > profiles/r01_summary.md

Applies the gfx950 corrections of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB)
reports half the bytes of a wide coalesced streaming read -> ×2; WRITE_SIZE
(KiB) is exact for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def kernel_key(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    base, tag = sys.argv[1], sys.argv[2]
    out = {}
    kt = find(os.path.join(base, f"{tag}_kt"), "*kernel_stats.csv")
    if kt:
        for r in rows(kt):
            out.setdefault(kernel_key(r["Name"]), {}).update(
                calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), total_ns=float(r["TotalDurationNs"]),
                pct=float(r["Percentage"]))
    for name in ("fetch", "write", "sq", "cyc", "waits", "waits2"):
        cc = find(os.path.join(base, f"{tag}_{name}"), "*counter_collection.csv")
        if not cc:
            continue
        acc = defaultdict(lambda: defaultdict(list))
        for r in rows(cc):
            acc[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in acc.items():
            for cn, vals in d.items():
                out.setdefault(k, {})[cn] = sum(vals) / len(vals)
                out[k][cn + "_sum"] = sum(vals)
                out[k][cn + "_n"] = len(vals)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
