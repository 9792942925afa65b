"""bench.py's own N>1 code path on CPU: two ranks under torch.distributed
(gloo), exactly as the driver's `torch.distributed.run --nproc-per-node N
bench.py --gpus N` launches it, with the GPU engine replaced by a stand-in.

What runs for real: bench.main() — process-group set-up, the RCCL unique-id
broadcast, the clock-settle loop whose continue flag rank 0 broadcasts (every
rank must take the same number of steps, each of which exchanges halos on the
GPU), the barriers around the timed steps, the max-over-ranks time, the
per-rank light-cone verification and its all-reduce, and the single JSON line
of rank 0.  The stand-in engine (test infrastructure) keeps the whole grid on
every rank and steps it with the oracle, and records the calls bench makes.
"""
import io
import json
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeEngine:
    """Whole-grid stand-in for golhip.Engine in rank mode (dead boundary)."""

    def __init__(self, rows, cols, *, rank=0, world=1, device=0, uid=None, layout="bit", tblock_k=1, **kw):
        from oracle import golcpu as g
        assert world == 2 and uid == bytes(range(128)) and device == rank, (world, device, rank)
        self.g, self.rows, self.cols, self.k = g, rows, cols, tblock_k
        self.board = np.zeros((rows, cols), np.uint8)
        self.opts, self.steps, self.launches = {}, 0, 0
        _FakeEngine.instances.append(self)

    instances = []

    def set_option(self, opt, value):
        self.opts[opt] = value

    def get_option(self, opt):
        return self.opts.get(opt, -6)

    def initialize_board(self, mode="stream", seed=1):
        self.board = self.g.init_dead(self.rows, self.cols, seed)

    def step(self, generations=1):
        self.board = self.g.run(self.board, generations, self.g.DEAD)
        self.steps += generations
        self.launches += (generations + self.k - 1) // self.k

    def sync(self):
        return 1.0

    def download_window(self, r0, c0, h, w):
        return self.board[r0:r0 + h, c0:c0 + w].copy()

    def kernel_time(self, reset=False):
        n = self.launches
        if reset:
            self.launches = 0
        return 0.5 * n, n

    def popcount(self):
        return int(self.board.sum())

    def close(self):
        pass


def _rank(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    golhip.Engine = _FakeEngine
    golhip.unique_id = lambda: bytes(range(128))
    mpi_amd.golhip = golhip
    import bench
    sys.argv = ["bench.py", "--gpus", str(world), "--rows", "256", "--cols", "160", "-k", "2", "--steps", "3",
                "--warmup", "1", "--settle-s", "0.2", "--no-secondary"]
    out = io.StringIO()
    real = sys.stdout
    sys.stdout = out
    try:
        bench.main()
    finally:
        sys.stdout = real
    e = _FakeEngine.instances[0]
    q.put((rank, out.getvalue(), e.steps))


def test_bench_main_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, s)) for r, o, s in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lines = [ln for ln in res[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1 and res[1][0].strip() == ""   # rank 0 prints the one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["rows"] == 512 and d["config"]["parallelism"] == "row-slabs x2 (rccl halos)"
    assert d["verified"] is True and d["cpu_baseline"] is None
    # both ranks took the same steps (settle flag broadcast): settle + warm-up + timed
    assert res[0][1] == res[1][1] and res[0][1] >= (1 + 3) * 2
