#!/usr/bin/env python3
"""Parity of the k=8 work-queue chunk plans against the static plan (GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

codes = [-3230, -3231, -3232, -3233, -3460, -3461, -3463, -3011]
rng = np.random.default_rng(7)
for rows, cols, slabs in [(300, 9000, 1), (4096, 8192, 1), (2048, 131072, 2), (5000, 3000, 3)]:
    b0 = (rng.random((rows, cols)) < 0.33).astype(np.uint8)
    ref = None
    for code in [None] + codes:
        with gh.Engine(rows, cols, n_gpus=slabs, layout="bit", tblock_k=8) as e:
            if code is not None:
                e.set_option(gh.OPT_CHUNK_ROWS, code)
            e.upload(b0)
            e.step(8 * 7)
            e.step(8 * 5)
            got = e.download()
        if ref is None:
            ref = got
        else:
            assert (got == ref).all(), (rows, cols, slabs, code, int((got != ref).sum()))
    print("ok", rows, cols, slabs, flush=True)
n = 131072
res = {}
for code in [None, -3230, -3461, -3233]:
    with gh.Engine(n, n, layout="bit", tblock_k=8) as e:
        e.initialize_board("stream", 1)
        if code is not None:
            e.set_option(gh.OPT_CHUNK_ROWS, code)
        e.step(8 * 20)
        wins = [e.download_window(r, c, 192, 192) for r, c in [(0, 0), (65000, 70000), (n - 192, n - 192), (131072 // 2 - 96, 5000), (1000, n - 192)]]
        res[code] = (e.popcount(), wins)
base = res[None]
for code, (pc, wins) in res.items():
    assert pc == base[0], (code, pc, base[0])
    for a, b in zip(wins, base[1]):
        assert (a == b).all(), code
print("ok 131072 full size", base[0], flush=True)
