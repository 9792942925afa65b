#!/usr/bin/env python3
"""Sweep kernel geometry on one GPU: GCUPS per (layout, k, words/lane, chunk rows)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--layout", default="bit")
p.add_argument("--n", type=int, default=131072)
p.add_argument("--ks", default="1,2,3,4,5,6,8")
p.add_argument("--wpls", default="4,8")
p.add_argument("--chunks", default="64,128,256,512")
p.add_argument("--gens", type=int, default=96)
p.add_argument("--reps", type=int, default=3)
a = p.parse_args()
rows = cols = a.n
bpc = 0.25 if a.layout == "bit" else 2.0
for k in map(int, a.ks.split(",")):
    e = gh.Engine(rows, cols, layout=a.layout, tblock_k=k)
    e.initialize_board("stream", 1)
    t_w = time.perf_counter()   # bring the clock / caches to steady state before the first config
    while time.perf_counter() - t_w < 1.5:
        e.step(8 * k)
        e.sync()
    for wpl in (map(int, a.wpls.split(",")) if a.layout == "bit" else [4]):
        if a.layout == "bit":
            e.set_option(gh.OPT_WORDS_PER_LANE, wpl)
        for ch in map(int, a.chunks.split(",")):
            e.set_option(gh.OPT_CHUNK_ROWS, ch)
            steps = max(2, a.gens // k)
            e.step(4 * k)
            e.sync()
            best = None
            for rep in range(a.reps):   # interleaving-free repeats; keep the fastest
                e.set_option(gh.OPT_KERNEL_TIMING, 1)
                e.kernel_time(reset=True)
                t = time.perf_counter()
                e.step(steps * k)
                e.sync()
                dt_r = time.perf_counter() - t
                kms_r, n_r = e.kernel_time(reset=True)
                e.set_option(gh.OPT_KERNEL_TIMING, 0)
                if best is None or dt_r < best[0]:
                    best = (dt_r, kms_r, n_r)
            dt, kms, n = best
            gcups = rows * cols * steps * k / dt / 1e9
            per = kms / n
            hbm = bpc * rows * cols / (per * 1e-3) / 1e9
            print(json.dumps({"layout": a.layout, "k": k, "wpl": wpl, "chunk": ch, "gcups": round(gcups, 1),
                              "kernel_ms": round(per, 4), "alg_GBps": round(hbm, 1),
                              "kernel_gcups": round(rows * cols * k / (per * 1e-3) / 1e9, 1)}), flush=True)
    e.close()
