#!/usr/bin/env python3
"""Per-wave start/end times of one bytebit launch (diagnostic build only).

    GOL_LIB=mpi_amd/libgolhip_stamps.so python tools/bb_stamps.py [--k 28] [--chunk -1]

The diagnostic build (GOL_BB_STAMPS=1 stamps and gol_debug_bb_stamps) lives in
commit 967c846's gol_kernels.hip, not in the product source:
    git show 967c846:mpi_amd/csrc/gol_kernels.hip > /tmp/k.hip && tools/build_variants.sh ...

Prints, for the last launch of a 32768² byte board, the distribution of item
durations and end times relative to the launch's first start (100-MHz
s_memrealtime ticks -> µs): how much of the launch the slowest waves add.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=28)
p.add_argument("--n", type=int, default=32768)
p.add_argument("--chunk", type=int, default=None)
a = p.parse_args()
L = gh.load()
L.gol_debug_bb_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
e = gh.Engine(a.n, a.n, layout="byte", tblock_k=a.k)
e.initialize_board("stream", 1)
if a.chunk is not None:
    e.set_option(gh.OPT_CHUNK_ROWS, a.chunk)
e.step(40 * a.k)
e.sync()
for rep in range(3):
    e.step(a.k)
    e.sync()
    buf = (ctypes.c_ulonglong * (3 * 8192))()
    assert L.gol_debug_bb_stamps(buf, 3 * 8192) == 0
    s = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3).astype(np.int64)
    s = s[s[:, 1] > 0]
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) / 100.0
    end = (s[:, 1] - t0) / 100.0
    dur = end - start
    span = end.max()
    q = lambda x, p: float(np.percentile(x, p))
    print(json.dumps({"k": a.k, "rep": rep, "items": int(len(s)), "launch_us": span,
                      "start_us_p50_p99_max": [q(start, 50), q(start, 99), float(start.max())],
                      "dur_us_min_p10_p50_p90_max": [float(dur.min()), q(dur, 10), q(dur, 50), q(dur, 90), float(dur.max())],
                      "end_us_p10_p50_p90": [q(end, 10), q(end, 50), q(end, 90)],
                      "mean_end_frac": float(end.mean() / span)}), flush=True)
    if rep == 2:   # where the slow items are: by XCD (block % 8), by strip, by band decile
        blk = s[:, 2]
        idx = np.nonzero(np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3)[:, 1] > 0)[0]
        nstrips = int(round(len(s) / max(1, (idx // 1).size and (idx.max() + 1) / len(s))))
        by_xcd = [round(float(dur[blk % 8 == x].mean()), 1) for x in range(8)]
        strip_of = idx % 17 if a.k >= 20 else idx
        by_strip = [round(float(dur[strip_of == t].mean()), 1) for t in range(17)]
        band = idx // 17
        dec = np.minimum(9, band * 10 // max(1, band.max() + 1))
        by_band = [round(float(dur[dec == d].mean()), 1) for d in range(10)]
        print(json.dumps({"k": a.k, "dur_mean_by_xcd": by_xcd, "dur_mean_by_strip": by_strip,
                          "dur_mean_by_band_decile": by_band}), flush=True)
e.close()
