#!/usr/bin/env python3
"""Chunk-policy / depth sweep of the stencil kernels on one GPU (GCUPS, kernel time).

    python tools/tune.py [--layout bit|byte] [--n 131072] [--gens 400] [--reps 2] [--spec K:CHUNK ...]

CHUNK is GOL_OPT_CHUNK_ROWS (r > 0 rows; -r rounds of resident waves; -(100+r)
guided) or 'd' for the library default (of the spec's split); an optional third
field K:CHUNK:S sets GOL_OPT_INTERIOR_SPLIT = S (1 .. 4; default: the context's,
2 for bit k = 8; '-' keeps it) and a fourth K:CHUNK:S:C the byte layout's
GOL_OPT_BYTE_CORE = C (1 default, 2 one wave per strip, 3 the chain kernel, 4 the pair-wave chain).  Every spec runs on one board per k in
round-robin repetitions and the fastest repetition is kept, so box drift hits
all specs alike.  Compile-time kernel variants are compared with
tools/ab_libs.sh over libgolhip_<name>.so builds (tools/build_variants.sh).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--layout", default="bit", choices=["bit", "byte"])
p.add_argument("--n", type=int, default=None, help="grid side (default 131072 bit, 32768 byte)")
p.add_argument("--gens", type=int, default=400)
p.add_argument("--reps", type=int, default=2)
p.add_argument("--spec", action="append")
a = p.parse_args()
n = a.n or (131072 if a.layout == "bit" else 32768)
bpc = 0.25 if a.layout == "bit" else 2.0
specs = a.spec or (["1:d", "4:d", "8:d"] if a.layout == "bit" else ["28:d"])
best, engines, allg = {}, {}, {}
for rep in range(a.reps):
    for sp in specs:
        k, chunk, *rest = sp.split(":")
        k = int(k)
        if k not in engines:
            for e, *_ in engines.values():
                e.close()
            engines.clear()
            e = gh.Engine(n, n, layout=a.layout, tblock_k=k)
            e.initialize_board("stream", 1)
            e.step(4 * k)
            e.sync()
            engines[k] = (e, e.get_option(gh.OPT_CHUNK_ROWS), e.get_option(gh.OPT_INTERIOR_SPLIT))
        e, default_chunk, default_split = engines[k]
        split = int(rest[0]) if rest and rest[0] != "-" else default_split
        e.set_option(gh.OPT_INTERIOR_SPLIT, split)
        if a.layout == "byte":
            e.set_option(gh.OPT_BYTE_CORE, int(rest[1]) if len(rest) > 1 else 1)
        if chunk == "d":   # the bit k = 8 default follows the split (-1 split, -104 unsplit)
            chunk = default_chunk if (split == default_split or a.layout != "bit" or k != 8) else (
                -1 if split >= 2 else -104)
        e.set_option(gh.OPT_CHUNK_ROWS, int(chunk))
        e.step(2 * k)
        e.sync()
        steps = max(2, a.gens // k)
        # split: the parts of a step run side by side, so summed per-launch times exceed
        # the step; take the batch's event span instead (gol_sync, as bench.py does)
        events = split < 2
        e.set_option(gh.OPT_KERNEL_TIMING, 1 if events else 0)
        e.kernel_time(reset=True)
        t = time.perf_counter()
        e.step(steps * k)
        dev_ms = e.sync()
        dt = time.perf_counter() - t
        kms, nl = e.kernel_time(reset=True)
        e.set_option(gh.OPT_KERNEL_TIMING, 0)
        per = (kms if events else dev_ms) / steps   # device ms per step
        rec = {"layout": a.layout, "spec": sp, "gcups": n * n * steps * k / dt / 1e9, "kernel_ms": per,
               "alg_GBps": bpc * n * n / (per * 1e-3) / 1e9, "rep": rep}
        allg.setdefault(sp, []).append(rec["gcups"])
        if sp not in best or rec["gcups"] > best[sp]["gcups"]:
            best[sp] = rec
for e, *_ in engines.values():
    e.close()
for sp in specs:
    g = sorted(allg[sp])
    best[sp]["median_gcups"] = g[len(g) // 2]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in best[sp].items()}), flush=True)
