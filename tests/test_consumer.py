"""The reference's consumer, gol_visualization.py, reads the driver's output
unchanged (north_star: "so gol_visualization.py still consumes the results
unchanged").

tests/golden/gol_sets/ holds small snapshot sets written by mpi_amd/bin/gol on
an MI355X (serial mode with 1 and 2 parts, MPI mode P=4 on 2 parts, dead mode
on 3 parts).  This CPU test runs /root/reference/gol_visualization.py BY PATH
on each set (matplotlib Agg, pcolor/pause recorded instead of drawn) and checks
that it loads every iteration and that the parts tile the whole board.  It is
skipped where /root/reference is absent (the GPU box).  The cells themselves
are checked against the oracle from the same files (the consumer's own
str->bool conversion makes every parsed cell True under numpy 2).
"""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import golcpu as g

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETS = os.path.join(ROOT, "tests", "golden", "gol_sets")
CONSUMER = "/root/reference/gol_visualization.py"

RUNNER = r"""
import json, runpy, sys
import matplotlib
matplotlib.use("Agg")
import matplotlib.pyplot as plt
boards = []
plt.pcolor = lambda b, *a, **k: boards.append([list(b.shape), int(b.sum())])
plt.pause = lambda *a, **k: None
plt.show = lambda *a, **k: None
sys.argv = ["gol_visualization.py", sys.argv[1]]
runpy.run_path(CONSUMER, run_name="__main__")
print("BOARDS" + json.dumps(boards))
"""


def main_file(d):
    return [f for f in glob.glob(os.path.join(d, "*.gol")) if "_" not in os.path.basename(f)][0]


def set_dirs():
    return sorted(glob.glob(os.path.join(SETS, "*")))


@pytest.mark.skipif(not os.path.exists(CONSUMER), reason="the reference consumer is only in the build container")
@pytest.mark.parametrize("d", set_dirs(), ids=os.path.basename)
def test_reference_consumer_reads_driver_output(d):
    mf = main_file(d)
    rows, cols, gap, iters, parts = map(int, open(mf).read().split())
    code = RUNNER.replace("CONSUMER", repr(CONSUMER))
    r = subprocess.run([sys.executable, "-c", code, mf], cwd=d, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, MPLBACKEND="Agg"))
    assert r.returncode == 0, r.stderr[-2000:]
    boards = __import__("json").loads(r.stdout.split("BOARDS", 1)[1])
    assert len(boards) == iters // gap + 1
    for shape, live in boards:
        assert shape == [rows, cols]
        assert live == rows * cols   # every cell was assigned by some part (numpy 2: '0' -> True)


@pytest.mark.parametrize("d", set_dirs(), ids=os.path.basename)
def test_driver_sets_match_oracle(d):
    """The same files, parsed with integer tokens, against the oracle run of
    the convention each set was written with."""
    mf = main_file(d)
    name = mf[:-4]
    rows, cols, gap, iters, parts = map(int, open(mf).read().split())
    kind = os.path.basename(d)
    if kind.startswith("serial"):
        b, mode, m = g.init_serial(rows), g.SERIAL_COMPAT, 1
    elif kind.startswith("mpi"):
        b, mode, m = g.init_mesh(rows, 2), g.MESH_COMPAT, 2
    else:
        b, mode, m = g.init_dead(rows, cols, 1), g.DEAD, 1
    for it in range(0, iters + 1, gap):
        if it:
            b = g.run(b, gap, mode, m)
        got = np.full((rows, cols), 7, np.uint8)
        for p in range(parts):
            lines = open(f"{name}_{it}_{p}.gol").read().splitlines()
            x0, x1 = map(int, lines[0].split())
            y0, y1 = map(int, lines[1].split())
            cells = np.array([[int(t) for t in ln.split()] for ln in lines[2:]], np.uint8)
            got[x0:x1 + 1, y0:y1 + 1] = cells   # the consumer's inclusive slicing (gol_visualization.py:33)
        assert (got == b).all(), (kind, it)
