#!/usr/bin/env python3
"""Reproduce the fuzz mismatch (byte SWAR k=3, 2 slabs, 1129x1917, uneven steps)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402
from oracle import golcpu as g  # noqa: E402

rng = np.random.default_rng(3)
rows, cols = 1129, 1917
b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
want = {n: g.run(b0, n, g.DEAD) for n in (1, 2, 3, 5, 6, 20)}


def run(steps, slabs, k, core=0, chunk=None, layout="byte", overlap=1):
    with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
        if layout == "byte":
            e.set_option(gh.OPT_BYTE_CORE, core)
        e.set_option(gh.OPT_OVERLAP, overlap)
        if chunk is not None:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
        e.upload(b0)
        for s in steps:
            e.step(s)
        got = e.download()
    ref = want[sum(steps)] if sum(steps) in want else g.run(b0, sum(steps), g.DEAD)
    bad = np.argwhere(got != ref)
    return len(bad), (bad[:3].tolist() if len(bad) else [])


for layout in ("byte", "bit"):
    for slabs in (1, 2):
        for k in (3,):
            for steps in ([20], [3] * 6 + [2], [2, 3, 3, 3, 3, 3, 3], [1, 2, 3, 1, 3, 3, 2, 3, 2], [1] * 20, [2] * 10):
                for overlap in (1, 0):
                    n, where = run(steps, slabs, k, layout=layout, overlap=overlap)
                    if n:
                        print(f"FAIL layout={layout} slabs={slabs} k={k} steps={steps} overlap={overlap}: {n} cells, "
                              f"e.g. {where}", flush=True)
print("repro done", flush=True)
