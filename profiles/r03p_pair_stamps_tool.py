#!/usr/bin/env python3
"""Slot utilisation of one k=8 pair-kernel launch (diagnostic build with per-item clocks).

    GOL_LIB=mpi_amd/libgolhip_pstamps.so python tools/pair_stamps.py [--chunk -6]
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
p.add_argument("--chunk", type=int, default=-6)
a = p.parse_args()
L = gh.load()
L.gol_debug_pair_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 131072
e = gh.Engine(n, n, layout="bit", tblock_k=8)
e.initialize_board("stream", 1)
e.step(8 * 300)
e.sync()
for chunk in [a.chunk]:
    e.set_option(gh.OPT_CHUNK_ROWS, chunk)
    e.step(8 * 100)
    e.sync()
    for rep in range(2):
        e.step(8)
        e.sync()
        buf = (ctypes.c_ulonglong * (3 * 65536))()
        assert L.gol_debug_pair_stamps(buf, 3 * 65536) == 0
        s = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3).astype(np.int64)
        s = s[s[:, 1] > 0]
        t0 = s[:, 0].min()
        start = (s[:, 0] - t0) / 100.0
        end = (s[:, 1] - t0) / 100.0
        dur = end - start
        span = float(end.max())
        slots = 4096
        util = float(dur.sum() / (slots * span))
        # running items over time (10-us bins)
        edges = np.arange(0, span + 10, 10.0)
        run = [int(((start < t1) & (end > t0_)).sum()) for t0_, t1 in zip(edges[:-1], edges[1:])]
        q = lambda x, pc: round(float(np.percentile(x, pc)), 1)
        print(json.dumps({"chunk": chunk, "rep": rep, "items": int(len(s)), "launch_us": round(span, 1),
                          "slot_utilisation": round(util, 4), "dur_us_p10_p50_p90_max": [q(dur, 10), q(dur, 50), q(dur, 90), round(float(dur.max()), 1)],
                          "last_start_us": round(float(start.max()), 1), "running_per_10us_head": run[:6],
                          "running_per_10us_tail": run[-12:]}), flush=True)
        e.set_option(gh.OPT_CHUNK_ROWS, chunk)
e.close()
