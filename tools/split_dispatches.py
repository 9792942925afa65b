#!/usr/bin/env python3
"""Per-step view of a split-interior kernel trace (rocprofv3 --kernel-trace):
the headline's step is two concurrent half-launches + one seam-band launch of
bit_pair_kernel, so rocprof's per-dispatch average mixes them.  This groups
the dispatches by grid size (halves vs seam band) and measures the step period
from consecutive half-launch starts on one stream.

    python tools/split_dispatches.py gpurun_out/prof_r05u_k8split_kt > profiles/r05u_k8split_dispatches.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "bit_pair_kernel"   # (the k = 16 headline: bit_chain_kernel)
rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
by_grid = defaultdict(list)
for r in rows:
    by_grid[int(r["Grid_Size_X"])].append(r)
out = {"trace": os.path.relpath(path), "dispatches": len(rows), "by_grid_size": {}}
for g, rs in sorted(by_grid.items(), key=lambda kv: -len(kv[1])):
    dur = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
    out["by_grid_size"][g] = {"calls": len(rs), "median_us": dur[len(dur) // 2] / 1e3,
                              "mean_us": sum(dur) / len(dur) / 1e3}
# step period: per stream, the gaps between consecutive starts of the big (half) launches
big = [r for r in rows if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 200_000]
per_stream = defaultdict(list)
for r in big:
    per_stream[r["Stream_Id"]].append(int(r["Start_Timestamp"]))
gaps = []
for st, ts in per_stream.items():
    ts.sort()
    gaps += [(b - a) / 1e3 for a, b in zip(ts, ts[1:]) if b - a < 5_000_000]
if gaps:
    out["half_launch_start_to_start_us"] = {"median": statistics.median(gaps), "n": len(gaps)}
# the point of the split: a half-launch starts while the OTHER stream's half of the
# previous step is still running — how long the two overlap after that start
streams = sorted(per_stream, key=lambda st: -len(per_stream[st]))[:2]
if len(streams) == 2:
    spans = {st: sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in big if r["Stream_Id"] == st)
             for st in streams}
    ov = []
    for a, b in ((streams[0], streams[1]), (streams[1], streams[0])):
        for s0, _ in spans[a]:
            running = [e for (s1, e) in spans[b] if s1 < s0 < e]
            if running:
                ov.append((max(running) - s0) / 1e3)
    if ov:
        out["overlap_after_start_us"] = {"median": statistics.median(ov), "n": len(ov),
                                         "note": "time the other stream's half keeps running after a half starts"}
out["note"] = ("the step = two half-launches on two streams (side by side) + the seam band on the halo stream; "
               "a half-launch lasts about one step period because the halves share the chip")
print(json.dumps(out, indent=1))
