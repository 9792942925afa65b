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
        idx = np.nonzero(np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3)[:, 1] > 0)[0]
        ns = 33
        strip = idx % ns
        band = idx // ns
        nb = band.max() + 1
        edge_s = (strip == 0) | (strip == ns - 1)
        edge_b = (band == 0) | (band == nb - 1)
        late = end >= np.percentile(end, 95)
        print(json.dumps({"dur_edge_strip": round(float(dur[edge_s].mean()), 1), "dur_interior": round(float(dur[~edge_s & ~edge_b].mean()), 1),
                          "dur_edge_band": round(float(dur[edge_b].mean()), 1),
                          "late5pct_edge_strip_frac": round(float(edge_s[late].mean()), 3), "edge_strip_frac": round(float(edge_s.mean()), 3),
                          "late5pct_band_min": int(band[late].min()), "late5pct_start_us_min": round(float(start[late].min()), 1),
                          "late5pct_dur_mean": round(float(dur[late].mean()), 1)}), flush=True)
        hw = s[:, 2] & 0xffffffff
        xcc = (s[:, 2] >> 32) & 0xf
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        slot = key * 16 + (hw & 15)
        us, invs = np.unique(slot, return_inverse=True)
        last_end = np.zeros(len(us)); n_it = np.bincount(invs); first_start = np.full(len(us), 1e9)
        np.maximum.at(last_end, invs, end); np.minimum.at(first_start, invs, start)
        busy_s = np.bincount(invs, weights=dur)
        gaps = (last_end - first_start) - busy_s
        xcc_end = [round(float(end[xcc == x].max()), 1) for x in range(8)]
        xcc_mean = [round(float(dur[xcc == x].mean()), 1) for x in range(8)]
        print(json.dumps({"slots": int(len(us)), "items_per_slot_hist": np.bincount(n_it).tolist(),
                          "slot_last_end_p0_p10_p50_p90_p100": [round(float(np.percentile(last_end, q)), 1) for q in (0, 10, 50, 90, 100)],
                          "slot_gap_us_mean_max": [round(float(gaps.mean()), 2), round(float(gaps.max()), 2)],
                          "xcc_last_end": xcc_end, "xcc_mean_dur": xcc_mean}), flush=True)
        uk, inv = np.unique(key, return_inverse=True)
        mean_d = np.bincount(inv, weights=dur) / np.bincount(inv)
        busy = np.bincount(inv, weights=dur)
        cnt = np.bincount(inv)
        cu_key = key // 4
        ucu, invc = np.unique(cu_key, return_inverse=True)
        cu_mean = np.bincount(invc, weights=dur) / np.bincount(invc)
        print(json.dumps({"simd_groups": int(len(uk)), "cu_groups": int(len(ucu)),
                          "simd_mean_dur_p0_p10_p50_p90_p100": [round(float(np.percentile(mean_d, q)), 1) for q in (0, 10, 50, 90, 100)],
                          "cu_mean_dur_p0_p10_p50_p90_p100": [round(float(np.percentile(cu_mean, q)), 1) for q in (0, 10, 50, 90, 100)],
                          "simd_items_min_max": [int(cnt.min()), int(cnt.max())],
                          "simd_busy_us_p0_p50_p100": [round(float(np.percentile(busy, q)), 1) for q in (0, 50, 100)],
                          "se_mean_dur": [round(float(dur[se == x].mean()), 1) if (se == x).any() else None for x in range(8)]}), flush=True)
        print(json.dumps({"chunk": chunk, "rep": rep, "items": int(len(s)), "launch_us": round(span, 1),
                          "slot_utilisation": round(util, 4), "dur_us_p10_p50_p90_max": [q(dur, 10), q(dur, 50), q(dur, 90), round(float(dur.max()), 1)],
                          "last_start_us": round(float(start.max()), 1), "running_per_10us_head": run[:6],
                          "running_per_10us_tail": run[-12:]}), flush=True)
        e.set_option(gh.OPT_CHUNK_ROWS, chunk)
e.close()
