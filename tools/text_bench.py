#!/usr/bin/env python3
"""Throughput of the device-side `.gol` snapshot text path.

    python tools/text_bench.py [--n 16384] [--layout bit] [--dir /tmp]

Times, for one n×n board initialised on the device:
  write : gol_write_text of the whole board to /dev/null (format on device,
          D2H through pinned buffers, write(2)) and to a file under --dir;
  read  : gol_read_text of that file back into the board (resume path);
  ref   : the reference's writeBoardToFile loop shape (an fprintf-style
          per-cell "%d\\t" of main.cpp:117-126) restated in numpy for scale.
Text bytes per board = n·(2n+1).  One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_amd import golhip as gh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=16384)
p.add_argument("--layout", default="bit")
p.add_argument("--dir", default="/tmp")
a = p.parse_args()
n = a.n
nbytes = n * (2 * n + 1)
with gh.Engine(n, n, layout=a.layout, tblock_k=1) as e:
    e.initialize_board("stream", 1)
    e.sync()
    lib = e.lib
    for target in ("/dev/null", os.path.join(a.dir, f"text_bench_{os.getpid()}.gol")):
        fd = os.open(target, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        t = time.perf_counter()
        e._chk(lib.gol_write_text(e._c, 0, 0, n, n, fd), "gol_write_text")
        os.fsync(fd) if target != "/dev/null" else None
        dt = time.perf_counter() - t
        os.close(fd)
        print(json.dumps({"op": "write", "target": target, "n": n, "layout": a.layout, "bytes": nbytes,
                          "seconds": dt, "GBps": nbytes / dt / 1e9}), flush=True)
    live = e.popcount()
    fd = os.open(target, os.O_RDONLY)
    t = time.perf_counter()
    e._chk(lib.gol_read_text(e._c, 0, 0, n, n, fd), "gol_read_text")
    e.sync()
    dt = time.perf_counter() - t
    os.close(fd)
    assert e.popcount() == live
    print(json.dumps({"op": "read", "source": target, "n": n, "bytes": nbytes, "seconds": dt,
                      "GBps": nbytes / dt / 1e9}), flush=True)
    os.unlink(target)
