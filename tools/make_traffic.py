#!/usr/bin/env python3
"""profiles/traffic.json from a tools/profile.sh run (PMC passes of bench.py).

    python tools/make_traffic.py gpurun_out prof_r01 bit131072_k8 [kernel-substring]

HBM bytes per launch of the stencil kernel = (2·FETCH_SIZE + WRITE_SIZE) KiB,
the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the
bytes of wide coalesced streaming reads; WRITE_SIZE is exact for them).
"""
import json
import os
import subprocess
import sys

base, tag, key = sys.argv[1], sys.argv[2], sys.argv[3]
sub = sys.argv[4] if len(sys.argv) > 4 else "pipe_kernel"
here = os.path.dirname(os.path.abspath(__file__))
summ = json.loads(subprocess.run([sys.executable, os.path.join(here, "pmc_summary.py"), base, tag],
                                 capture_output=True, text=True, check=True).stdout)
name = [k for k in summ if sub in k][0]
k = summ[name]
path = os.path.join(os.path.dirname(here), "profiles", "traffic.json")
data = json.load(open(path)) if os.path.exists(path) else {}
data[key] = {
    "kernel": name, "profile": tag,
    "fetch_kib_raw": k["FETCH_SIZE"], "write_kib": k["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024,
    "valu_insts_per_launch": k.get("SQ_INSTS_VALU"), "avg_ns": k.get("avg_ns"),
    "clock_ghz": (k["GRBM_GUI_ACTIVE"] / 8 / (k["avg_ns"] * 1e-9) / 1e9) if "GRBM_GUI_ACTIVE" in k else None,
}
json.dump(data, open(path, "w"), indent=1)
print(json.dumps(data[key], indent=1))
