#!/usr/bin/env python3
"""Soak test (GPU box, outside the suite): long runs of mid-size boards through
the default schedule (split interior at k = 8, 1-3 slabs) with random step
depths, async window snapshots between steps and option toggles, compared
bit-exactly with the oracle every segment.  Test infrastructure: the oracle is
the checker only.

    python tools/soak.py [--minutes 4] [--seed 7]
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
p.add_argument("--minutes", type=float, default=4.0)
p.add_argument("--seed", type=int, default=7)
a = p.parse_args()
rng = np.random.default_rng(a.seed)
t_end = time.time() + 60 * a.minutes
runs = fails = segs = 0
while time.time() < t_end:
    slabs = int(rng.integers(1, 4))
    k = int(rng.choice([8, 8, 8, 5, 3]))
    rows = int(rng.integers(600, 2400)) * slabs
    cols = int(rng.choice([2100, 4096, 9000, 17000]))
    b = (rng.random((rows, cols)) < rng.uniform(0.2, 0.5)).astype(np.uint8)
    with gh.Engine(rows, cols, n_gpus=slabs, layout="bit", tblock_k=k) as e:
        e.upload(b)
        split0 = e.get_option(gh.OPT_INTERIOR_SPLIT)
        for seg in range(int(rng.integers(3, 7))):
            steps = [int(rng.choice([k, k, k, 1, 2, k - 1 or 1])) for _ in range(int(rng.integers(5, 40)))]
            snaps, done = [], 0
            for st in steps:
                e.step(st)
                done += st
                if rng.random() < 0.15:
                    r0, c0 = int(rng.integers(0, rows - 8)), int(rng.integers(0, cols - 64))
                    snaps.append((done, r0, c0, e.download_window_async(r0, c0, 8, 64)))
            got = e.download()
            want, at = b, 0
            for d0, r0, c0, w in snaps:   # the oracle walks the same generations
                want = g.run_dead_fast(want, d0 - at)
                at = d0
                if not (w == want[r0:r0 + 8, c0:c0 + 64]).all():
                    fails += 1
                    print("SNAPSHOT MISMATCH", dict(rows=rows, cols=cols, slabs=slabs, k=k, seg=seg, gen=d0), flush=True)
            want = g.run_dead_fast(want, done - at)
            if not (got == want).all():
                fails += 1
                print("MISMATCH", dict(rows=rows, cols=cols, slabs=slabs, k=k, seg=seg,
                                       cells=int((got != want).sum())), flush=True)
            b = want
            segs += 1
            if rng.random() < 0.3:   # toggle the split (synchronises the context)
                e.set_option(gh.OPT_INTERIOR_SPLIT, 1 if e.get_option(gh.OPT_INTERIOR_SPLIT) > 1 else max(2, split0))
    runs += 1
    if runs % 10 == 0:
        print(f"{runs} runs, {segs} segments, {fails} failures", flush=True)
print(json.dumps({"runs": runs, "segments": segs, "failures": fails, "seed": a.seed, "minutes": a.minutes}))
sys.exit(1 if fails else 0)
