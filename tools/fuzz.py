#!/usr/bin/env python3
"""Randomised parity fuzzing of every kernel/option combination against the
oracle (test infrastructure; run on the GPU box, not part of `pytest -m gpu`).

    python tools/fuzz.py [--cases 400] [--seed 1] [--max-cells 4000000]

Each case draws a board shape, layout, boundary (dead / serial-compat /
mesh-compat), k, number of slabs, chunk policy, byte-core, interior-split and overlap switches and a generation count, runs it through libgolhip.so
and compares bit-exactly with oracle/golcpu — the board, a random window
(download, device-formatted `.gol` text, parse round trip), the popcount and
an async window snapshot taken after a random k-step while later steps run.
Prints one line per failure and a JSON summary; exit status 1 on any mismatch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402
from oracle import golcpu as g  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--cases", type=int, default=400)
p.add_argument("--seed", type=int, default=1)
p.add_argument("--max-cells", type=int, default=4_000_000)
p.add_argument("--only", type=str, default=None,
               help="A:B — draw every case (same random stream) but run only cases A..B, twice, verbosely")
p.add_argument("--bit-k", type=str, default=None, help="comma list: the bit layout's k values (default 1..8)")
p.add_argument("--byte-k", type=str, default=None,
               help="comma list: the byte layout's k values (default 1..8, 12, 16, ..., 32)")
p.add_argument("--byte-cores", type=str, default=None,
               help="comma list: GOL_OPT_BYTE_CORE values drawn for byte k > 8 (default 1; a core without a "
                    "kernel at that depth runs the default one)")
p.add_argument("--gens-max", type=int, default=40, help="generation counts drawn from 1..this")
p.add_argument("--rccl-shim", default=None,
               help="path of tests/shim/libfake_rccl.so: fuzz the one-process-per-rank transport instead "
                    "(ranks as threads on one GPU)")
a = p.parse_args()
rng = np.random.default_rng(a.seed)


def fuzz_rccl_shim():
    """Random world sizes / layouts / k / uneven steps through gol_create_rank."""
    import ctypes
    import threading
    ctypes.CDLL(a.rccl_shim, mode=ctypes.RTLD_GLOBAL)
    fails = 0
    for case in range(a.cases):
        world = int(rng.integers(2, 9))
        layout = str(rng.choice(["bit", "byte"]))
        k = int(rng.choice((SHIM_BYTE_K if layout == "byte" else SHIM_BIT_K)))
        boundary = str(rng.choice(["dead", "serial_compat"]))
        rows = int(rng.integers(max(world * k, 2 * world), max(world * k, 2 * world) + 300))
        cols = int(rng.integers(2, 5000))
        gens = int(rng.integers(1, a.gens_max + 1))
        steps, d = [], 0
        while d < gens:
            steps.append(int(rng.integers(1, gens - d + 1)))
            d += steps[-1]
        overlap = int(rng.random() < 0.8)
        b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
        split = int(np.random.default_rng([a.seed, case, 12]).choice([1, 2, 2, 3, 4]))   # (own stream)
        mode = g.DEAD
        if boundary == "serial_compat":
            b0[-1, :] = 0
            b0[:, -1] = 0
            mode = g.SERIAL_COMPAT
        uid = gh.unique_id()
        parts, errs = [None] * world, []

        def worker(r):
            try:
                with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout=layout, tblock_k=k,
                               boundary=boundary) as e:
                    e.set_option(gh.OPT_OVERLAP, overlap)
                    e.set_option(gh.OPT_INTERIOR_SPLIT, split)
                    e.upload(b0)
                    for st in steps:
                        e.step(st)
                    r0, n = gh.slab_plan(rows, world, r)
                    parts[r] = (r0, e.download_window(r0, 0, n, cols))
            except Exception as ex:   # noqa: BLE001
                errs.append((r, repr(ex)))

        ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        desc = dict(world=world, split=split, rows=rows, cols=cols, layout=layout, k=k, boundary=boundary, steps=steps,
                    overlap=overlap)
        if errs or any(t.is_alive() for t in ts):
            print("ERROR", case, desc, errs, flush=True)
            fails += 1
            break   # a hung rank thread keeps its barrier: stop here
        got = np.zeros_like(b0)
        for r0, w in parts:
            got[r0:r0 + w.shape[0]] = w
        bad = int((got != g.run(b0, gens, mode)).sum())
        if bad:
            fails += 1
            print("MISMATCH", case, bad, desc, flush=True)
        if case % 25 == 0:
            print(f"case {case}: {fails} failures", flush=True)
    print(json.dumps({"mode": "rccl-shim", "cases": a.cases, "failures": fails, "seed": a.seed}))
    sys.exit(1 if fails else 0)


# the shim mode's depths (--bit-k / --byte-k override them)
SHIM_BYTE_K = [int(x) for x in a.byte_k.split(",")] if a.byte_k else [1, 2, 3, 5, 8, 12, 16, 24, 28]
SHIM_BIT_K = [int(x) for x in a.bit_k.split(",")] if a.bit_k else list(range(1, 9))
if a.rccl_shim:
    fuzz_rccl_shim()

BYTE_K = [int(x) for x in a.byte_k.split(",")] if a.byte_k else [1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 20, 24, 28, 32]
BYTE_CORES = [int(x) for x in a.byte_cores.split(",")] if a.byte_cores else [1]
BIT_K = [int(x) for x in a.bit_k.split(",")] if a.bit_k else list(range(1, 9))
CHUNKS = [None, 8, 37, 256, -1, -2, -3, -102, -103]
fails, done, t0 = 0, 0, time.time()
only = tuple(int(x) for x in a.only.split(":")) if a.only else None
for case in range(a.cases):
    layout = str(rng.choice(["bit", "byte"]))
    boundary = str(rng.choice(["dead", "dead", "serial_compat", "mesh_compat"]))
    if boundary == "mesh_compat":   # any layout and k: the reversed-block board of gol_runtime.cpp
        k = int(rng.choice(BYTE_K if layout == "byte" else BIT_K))
        m = int(rng.integers(1, 6))
        cols = m * int(rng.integers(2, 700))
    else:
        k = int(rng.choice(BYTE_K if layout == "byte" else BIT_K))
        m = 1
        # (9000-40000: the folded strips of the k=8 pair kernel, >= 16257 columns, and of the bytebit
        # kernel, >= 4033 columns)
        cols = int(rng.choice([rng.integers(1, 300), rng.integers(300, 5000), rng.integers(5000, 9000),
                               rng.integers(9000, 40000)]))
    rows = int(rng.integers(1, max(2, min(3000, a.max_cells // max(cols, 1)))))
    if boundary != "dead" and (rows < 2 or cols < 2):
        continue
    slabs = int(rng.integers(1, 5))
    if boundary == "mesh_compat":
        rows = cols
    if slabs > 1 and rows // slabs < max(k, 1):
        slabs = 1
    gens = int(rng.integers(1, a.gens_max + 1))
    chunk = CHUNKS[int(rng.integers(len(CHUNKS)))]
    core = int(rng.random() < 0.85) if (layout == "byte" and k <= 8) else (
        int(rng.choice(BYTE_CORES)) if (layout == "byte" and a.byte_cores) else 1)   # (default: the old stream)
    b0 = (rng.random((rows, cols)) < rng.uniform(0.1, 0.6)).astype(np.uint8)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    # sometimes start from the device-side glibc initialisation instead of an upload
    init = None
    if rng.random() < 0.3:
        if boundary == "dead":
            init = ("stream", int(rng.integers(0, 1 << 31)))
            b0 = g.init_dead(rows, cols, init[1])
        elif boundary == "serial_compat" and rows == cols:
            init = ("serial", g.SERIAL_SEED)
            b0 = g.init_serial(rows)
        elif boundary == "mesh_compat" and (layout == "byte" or (cols // m) % 32 == 0):
            init = ("mesh", 0)
            b0 = g.init_mesh(rows, m)
    mode = {"dead": g.DEAD, "serial_compat": g.SERIAL_COMPAT, "mesh_compat": g.MESH_COMPAT}[boundary]
    desc = dict(rows=rows, cols=cols, layout=layout, boundary=boundary, m=m, k=k, slabs=slabs, gens=gens,
                chunk=chunk, core=core, init=init)
    steps, done_g = [], 0
    while done_g < gens:   # uneven step sizes exercise partial blocks
        steps.append(int(rng.integers(1, gens - done_g + 1)))
        done_g += steps[-1]
    desc["steps"] = steps
    # the split interior (GOL_OPT_INTERIOR_SPLIT) from a stream of its own, so the cases
    # above stay what earlier seeds drew
    split = int(np.random.default_rng([a.seed, case, 12]).choice([1, 2, 2, 3, 4]))
    desc["split"] = split
    # overlap on/off and an async window snapshot after a random k-step (streams of their own)
    xr = np.random.default_rng([a.seed, case, 13])
    overlap = int(xr.random() < 0.8)
    snap_i = int(xr.integers(0, len(steps)))
    sr0, sc0 = int(xr.integers(0, rows)), int(xr.integers(0, cols))
    sh, sw = int(xr.integers(1, min(rows - sr0, 64) + 1)), int(xr.integers(1, min(cols - sc0, 256) + 1))
    desc["overlap"], desc["snap"] = overlap, (snap_i, sr0, sc0, sh, sw)
    if only and not (only[0] <= case <= only[1]):
        continue

    def run_case():
        with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, boundary=boundary, mesh_m=m, tblock_k=k) as e:
            if chunk is not None:
                e.set_option(gh.OPT_CHUNK_ROWS, chunk)
            if layout == "byte":
                e.set_option(gh.OPT_BYTE_CORE, core)
            e.set_option(gh.OPT_INTERIOR_SPLIT, split)
            e.set_option(gh.OPT_OVERLAP, overlap)
            if init:
                e.initialize_board(*init)
            else:
                e.upload(b0)
            snap = None
            for i, st in enumerate(steps):
                e.step(st)
                if i == snap_i:   # filled at the next sync, while later steps are already enqueued
                    snap = e.download_window_async(sr0, sc0, sh, sw)
            full = e.download()
            # I/O paths on a random window: download, device text format, parse back, popcount
            r0, c0 = int(io_rng.integers(0, rows)), int(io_rng.integers(0, cols))
            h, w = int(io_rng.integers(1, rows - r0 + 1)), int(io_rng.integers(1, cols - c0 + 1))
            win = e.download_window(r0, c0, h, w)
            txt = e.format_text(r0, c0, h, w)
            io = {"win": (r0, c0, win), "txt": txt, "pop": e.popcount()}
            e.parse_text(r0, c0, h, w, txt)   # identity round trip
            io["reparsed"] = e.download()
            io["snap"] = snap
            return full, io

    io_rng = np.random.default_rng([a.seed, case])

    def expect_text(board):   # writeBoardToFile's body: "v\t" per cell, "\n" per row
        t = np.empty((board.shape[0], 2 * board.shape[1] + 1), np.uint8)
        t[:, 0:-1:2] = np.where(board != 0, ord("1"), ord("0"))
        t[:, 1:-1:2] = ord("\t")
        t[:, -1] = ord("\n")
        return t.tobytes()

    try:
        got, io = run_case()
        want = g.run(b0, gens, mode, m) if boundary == "mesh_compat" else g.run(b0, gens, mode)
        bad = int((got != want).sum())
        r0, c0, win = io["win"]
        wref = want[r0:r0 + win.shape[0], c0:c0 + win.shape[1]]
        g_snap = sum(steps[:snap_i + 1])
        at_snap = g.run(b0, g_snap, mode, m) if boundary == "mesh_compat" else g.run(b0, g_snap, mode)
        snap_ok = (io["snap"] == at_snap[sr0:sr0 + sh, sc0:sc0 + sw]).all()
        if not (win == wref).all() or io["txt"] != expect_text(wref) or io["pop"] != int(want.sum()) \
                or not (io["reparsed"] == want).all() or not snap_ok:
            bad = max(bad, 1)
            print("IO MISMATCH", case, desc, (r0, c0, win.shape), flush=True)
        if only:
            again, _ = run_case()
            diff = np.argwhere(got != want)
            print(f"case {case}: {bad} bad, rerun {int((again != want).sum())} bad, runs differ "
                  f"{int((again != got).sum())}; first bad {diff[:5].tolist()} rows {sorted(set(diff[:, 0].tolist()))[:20]}",
                  desc, flush=True)
    except gh.GolError as ex:
        print("ERROR", case, desc, ex, flush=True)
        fails += 1
        continue
    done += 1
    if bad:
        fails += 1
        print("MISMATCH", case, bad, desc, flush=True)
    if case % 50 == 0:
        print(f"case {case}: {done} ok-or-checked, {fails} failures, {time.time() - t0:.0f} s", flush=True)
print(json.dumps({"cases_run": done, "failures": fails, "seed": a.seed, "seconds": time.time() - t0}))
sys.exit(1 if fails else 0)
