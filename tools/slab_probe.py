#!/usr/bin/env python3
"""Multi-slab rehearsal on one GPU (the PEER transport of config 5): GCUPS of S
row slabs of H rows × n columns in ONE context, per overlap mode and chunk
policy, against one slab of the same size.

    python tools/slab_probe.py [--slabs 1,2,8] [--h 131072] [--n 131072] [--k 8]
                               [--spec OVERLAP:CHUNK[:SPLIT] ...] [--gens 320] [--reps 2]

OVERLAP 1 = interior kernel under the halo exchange + boundary bands (default),
0 = one kernel per slab after the exchange; CHUNK = GOL_OPT_CHUNK_ROWS or 'd'
(the default of the spec's split); SPLIT = GOL_OPT_INTERIOR_SPLIT (default: the
context's).
One JSON line per (slabs, spec, rep).
"""
import argparse
import json
import os
import sys
import time

# two streams per slab: give each its own hardware queue (bench.py does the same)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--slabs", default="1,2,8")
p.add_argument("--h", type=int, default=131072, help="rows per slab")
p.add_argument("--total", type=int, default=0, help="if > 0: total rows, split over the slabs (h = total / S)")
p.add_argument("--n", type=int, default=131072)
p.add_argument("--k", type=int, default=8)
p.add_argument("--gens", type=int, default=320)
p.add_argument("--reps", type=int, default=2)
p.add_argument("--spec", action="append")
a = p.parse_args()
specs = a.spec or ["1:d"]
for S in [int(x) for x in a.slabs.split(",")]:
    rows = a.total if a.total > 0 else S * a.h
    with gh.Engine(rows, a.n, n_gpus=S, layout="bit", tblock_k=a.k) as e:
        e.set_option(gh.OPT_SCHEDULE_TRIAL, 0)
        default_split = e.get_option(gh.OPT_INTERIOR_SPLIT)
        default_chunk = e.get_option(gh.OPT_CHUNK_ROWS)
        e.initialize_board("stream", 1)
        e.step(40 * a.k)   # past the clock ramp
        e.sync()
        for rep in range(a.reps):
            for sp in specs:
                ov, chunk, *rest = sp.split(":")
                e.set_option(gh.OPT_OVERLAP, int(ov))
                split = int(rest[0]) if rest else default_split
                e.set_option(gh.OPT_INTERIOR_SPLIT, split)
                if chunk == "d":   # the k = 8 default follows the split (-1 split, -104 unsplit)
                    chunk = default_chunk if (split == default_split or a.k != 8) else (-1 if split >= 2 else -104)
                e.set_option(gh.OPT_CHUNK_ROWS, int(chunk))
                e.step(4 * a.k)
                e.sync()
                steps = max(2, a.gens // a.k)
                t = time.perf_counter()
                e.step(steps * a.k)
                e.sync()
                dt = time.perf_counter() - t
                print(json.dumps({"slabs": S, "spec": sp, "split": e.get_option(gh.OPT_INTERIOR_SPLIT), "rep": rep, "gcups": round(rows * a.n * steps * a.k / dt / 1e9, 1),
                                  "ms_per_step": round(dt * 1e3 / steps, 3),
                                  "rows": rows}), flush=True)
