#!/usr/bin/env python3
"""profiles/traffic.json from a tools/profile.sh run (PMC passes of bench.py).

    python tools/make_traffic.py gpurun_out prof_r01 bit131072_k8 [kernel-substring] [--per-step D] [--out PATH]

--per-step D: every k-step dispatches the kernel D times (the split interior:
two half-launches + the seam band, D = 3); the record is then per STEP = the
counter's sum over all dispatches ÷ (dispatches / D), the unit bench.py's
roofline uses for a split slab.

HBM bytes per launch of the stencil kernel = (2·FETCH_SIZE + WRITE_SIZE) KiB,
the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the
bytes of wide coalesced streaming reads; WRITE_SIZE is exact for them).
"""
import json
import os
import subprocess
import sys

argv = sys.argv[1:]
per_step = 0
if "--per-step" in argv:
    i = argv.index("--per-step")
    per_step = int(argv[i + 1])
    del argv[i:i + 2]
out_path = None
if "--out" in argv:   # (default: profiles/traffic.json)
    i = argv.index("--out")
    out_path = argv[i + 1]
    del argv[i:i + 2]
base, tag, key = argv[0], argv[1], argv[2]
sub = argv[3] if len(argv) > 3 else "pipe_kernel"
here = os.path.dirname(os.path.abspath(__file__))
summ = json.loads(subprocess.run([sys.executable, os.path.join(here, "pmc_summary.py"), base, tag],
                                 capture_output=True, text=True, check=True).stdout)
name = [k for k in summ if sub in k][0]
k = summ[name]
if per_step:   # per step: sums over the dispatches of whole steps
    for cn in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"):
        if cn + "_sum" in k:
            k[cn] = k[cn + "_sum"] / (k[cn + "_n"] / per_step)
path = out_path or os.path.join(os.path.dirname(here), "profiles", "traffic.json")
data = json.load(open(path)) if os.path.exists(path) else {}
data[key] = {
    "kernel": name, "profile": tag,
    "fetch_kib_raw": k["FETCH_SIZE"], "write_kib": k["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024,
    "valu_insts_per_launch": k.get("SQ_INSTS_VALU"), "avg_ns": k.get("avg_ns"),
    "clock_ghz": (k["GRBM_GUI_ACTIVE"] / 8 / (k["avg_ns"] * 1e-9) / 1e9)
    if ("GRBM_GUI_ACTIVE" in k and not per_step) else None,
}
if per_step:
    data[key]["dispatches_per_step"] = per_step
    data[key]["note"] = ("per k-step: counter sums over all dispatches of the kernel / (dispatches / "
                         f"{per_step}); avg_ns is the per-dispatch kernel-trace average")
json.dump(data, open(path, "w"), indent=1)
print(json.dumps(data[key], indent=1))
