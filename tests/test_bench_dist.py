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
        assert world == 1 or (world == 2 and uid == bytes(range(128)) and device == rank), (world, device, rank)
        self.g, self.rows, self.cols, self.k, self.world = g, rows, cols, tblock_k, world
        self.board = np.zeros((rows, cols), np.uint8)
        self.opts, self.steps, self.launches, self.comm_steps = {}, 0, 0, 0
        _FakeEngine.instances.append(self)

    instances = []
    corrupt_halo = bool(os.environ.get("GOL_FAKE_CORRUPT_HALO"))

    def set_option(self, opt, value):
        self.opts[opt] = value

    def comm_time(self, reset=False):
        """(exchange ms, bands ms, k-steps): 0.1 / 0.2 ms per k-step stepped since the last reset."""
        n = self.comm_steps
        if reset:
            self.comm_steps = 0
        return 0.1 * n, 0.2 * n, n

    def get_option(self, opt):
        return self.opts.get(opt, -6)

    def initialize_board(self, mode="stream", seed=1):
        self.board = self.g.init_dead(self.rows, self.cols, seed)

    def step(self, generations=1):
        left = generations
        while left > 0:   # k generations per step, as the library's halo exchange moves k rows
            kk = min(self.k, left)
            new = self.g.run(self.board, kk, self.g.DEAD)
            if _FakeEngine.corrupt_halo and self.world > 1:
                # rank 1's top halo arrives with its row next to the seam flipped
                # (a garbage halo row): slab 1 is stepped from that padded copy
                H = self.rows // self.world
                lo, hi = H, 2 * H
                pad = self.board[lo - kk:min(self.rows, hi + kk)].copy()
                pad[kk - 1] ^= 1
                new[lo:hi] = self.g.run(pad, kk, self.g.DEAD)[kk:kk + H]
            self.board = new
            left -= kk
        self.steps += generations
        self.launches += (generations + self.k - 1) // self.k
        self.comm_steps += (generations + self.k - 1) // self.k

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


def _rank(rank, world, port, q, corrupt=False, split=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    _FakeEngine.corrupt_halo = corrupt
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    golhip.Engine = _SplitFakeEngine if split else _FakeEngine
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


def _run_world2(corrupt=False, split=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, corrupt, split)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, s)) for r, o, s in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lines = [ln for ln in res[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1 and res[1][0].strip() == ""   # rank 0 prints the one JSON line
    return json.loads(lines[0]), res


def test_bench_main_world2_gloo():
    d, res = _run_world2()
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["rows"] == 512 and d["config"]["parallelism"] == "row-slabs x2 (rccl halos)"
    assert d["verified"] is True and d["cpu_baseline"] is None
    # both ranks took the same steps on the headline board (warm-up + timed; the settle steps ran on the twin)
    assert res[0][1] == res[1][1] and res[0][1] >= (1 + 3) * 2
    # one window per rank (mid-slab) and one across the seam, all verified
    kinds = sorted("seam" in v for v in d["verify"])
    assert kinds == [False, False, True] and all(v["ok"] for v in d["verify"])
    seam = next(v for v in d["verify"] if "seam" in v)
    assert seam["seam"] == 256 and seam["ranks"] == [0, 1] and seam["window"][0] == 224
    check_halo_fields(d["halo"], world=2, steps=3)


def check_halo_fields(h, world, steps):
    """The N>1 line's halo diagnostic: present, per rank, and self-consistent."""
    assert h is not None and len(h["per_rank"]) == world
    assert sorted(r["rank"] for r in h["per_rank"]) == list(range(world))
    assert abs(h["exposed_ms_per_step"] - (h["step_ms"] - h["step_ms_no_halo"])) < 1e-9
    assert abs(h["efficiency_vs_no_halo"] - h["step_ms_no_halo"] / h["step_ms"]) < 1e-9
    assert abs(h["comm_ms_per_step"] - (h["exchange_ms_per_step"] + h["bands_ms_per_step"])) < 1e-9
    assert h["step_ms"] == min(h["windows_ms_per_step"]["with_halo"])
    assert h["step_ms_no_halo"] == min(h["windows_ms_per_step"]["no_halo"])
    for r in h["per_rank"]:
        assert r["steps_timed"] == 2 * (steps + 2)   # 2 rounds of (warm 2 + steps) real k-steps
        assert abs(r["bands_ms_per_step"] - 0.2) < 1e-9 and abs(r["exchange_ms_per_step"] - 0.1) < 1e-9


def test_bench_main_world2_detects_corrupt_halo():
    """A halo row that arrives wrong (here: rank 1's row next to the seam,
    flipped at every k-step) must flip `verified` to false: the seam window
    catches it while both mid-slab windows still pass."""
    d, _ = _run_world2(corrupt=True)
    assert d["verified"] is False
    seam = [v for v in d["verify"] if "seam" in v]
    slab = [v for v in d["verify"] if "seam" not in v]
    assert len(seam) == 1 and seam[0]["ok"] is False
    assert len(slab) == 2 and all(v["ok"] for v in slab)


def test_bench_main_single_rank(monkeypatch, capsys):
    """bench.main() at N=1 with the stand-in engine: the headline board, the
    twin the clock settles on (timed afterwards as `aged_board`), one JSON line
    with the contract keys and a verified window."""
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    monkeypatch.setattr(golhip, "Engine", _FakeEngine)
    monkeypatch.setattr(mpi_amd, "golhip", golhip)
    import bench
    for key in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(key, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--rows", "200", "--cols", "160", "-k", "2", "--steps", "3",
                                      "--warmup", "1", "--settle-s", "0.05", "--no-secondary", "--no-cpu-baseline"])
    _FakeEngine.instances.clear()
    bench.main()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["verified"] is True and len(d["verify"]) == 1
    assert d["aged_board"]["value"] > 0 and d["config4_1000gen"] is None   # (config 4 needs the full grid)
    assert d["settle"]["on_second_board"] is True and "seeded grid" in d["board"]
    eng, twin = _FakeEngine.instances[:2]
    assert eng.steps == (1 + 3) * 2          # warm-up + timed only: the headline board is the seeded grid
    assert twin.steps > eng.steps            # the settle steps ran on the twin


class _SplitFakeEngine(_FakeEngine):
    """The stand-in with the split interior on: two timed launches per step."""

    def get_option(self, opt):
        from mpi_amd import golhip
        if opt == golhip.OPT_INTERIOR_SPLIT:
            return 2
        return super().get_option(opt)

    def step(self, generations=1):
        super().step(generations)
        self.launches += (generations + self.k - 1) // self.k


def test_bench_main_split_interior_roofline(monkeypatch, capsys):
    """Under the split interior (the k = 8 default) the roofline's unit is the
    step: two concurrent half-launches per step, so the time per launch is the
    batch's device time ÷ steps (not ÷ launches) and the bytes are the whole
    slab's; the stream count for the twin check is three per slab."""
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    monkeypatch.setattr(golhip, "Engine", _SplitFakeEngine)
    monkeypatch.setattr(mpi_amd, "golhip", golhip)
    import bench
    for key in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(key, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--rows", "200", "--cols", "160", "-k", "2", "--steps", "3",
                                      "--warmup", "1", "--settle-s", "0.05", "--no-secondary", "--no-cpu-baseline",
                                      "--no-aged"])
    _FakeEngine.instances.clear()
    bench.main()
    d = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.strip()][-1])
    rf = d["roofline"]
    assert rf["interior_split"] is True and d["config"]["interior_split"] == 2
    assert rf["launches"] == 6 and abs(rf["kernel_avg_ms"] - 1.0 / 3) < 1e-9   # sync() = 1.0 ms per batch
    assert rf["hbm"]["bytes_per_launch"] == 0.25 * 200 * 160
    assert abs(rf["hbm"]["achieved"] - 0.25 * 200 * 160 / (1.0e-3 / 3) / 1e9) < 1e-9
    assert "split interior" in rf["timing"] and d["settle"]["on_second_board"] is True


def test_bench_main_world2_split_roofline():
    """Rank mode under the split interior: each rank's step is two half-launches
    (+ bands and seam band), so the roofline takes the whole slab's bytes per
    step; the seam windows still verify."""
    d, _ = _run_world2(split=True)
    rf = d["roofline"]
    assert d["verified"] is True and rf["interior_split"] is True and rf["launches"] == 6
    assert rf["hbm"]["bytes_per_launch"] == 0.25 * 256 * 160   # rows per rank x cols, bands included


class _ProbeFakeEngine(_FakeEngine):
    """The stand-in with the clock probe and the async window copy: the copy is
    the window as of the steps enqueued so far (the library copies it behind
    them), so steps enqueued later (the clock batch) must not reach it."""

    def clock_start(self, max_ms):
        self.probe_from = self.steps

    def clock_stop(self):
        self.probe_steps = self.steps - self.probe_from
        return 2300.0, 1.0

    def download_window_async(self, r0, c0, h, w):
        return self.download_window(r0, c0, h, w)


def test_bench_clock_batch_after_timed_steps(monkeypatch, capsys):
    """The clock is read over the same K steps run again after the timed ones
    (the probe's wave would cost the timed steps a round's tail): the headline
    board takes warm-up + timed + clock-batch steps, the window verified is the
    one at the timed steps' end (grabbed before the clock batch), and the line
    carries the clock and that batch's time."""
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    monkeypatch.setattr(golhip, "Engine", _ProbeFakeEngine)
    monkeypatch.setattr(mpi_amd, "golhip", golhip)
    import bench
    for key in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(key, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--rows", "200", "--cols", "160", "-k", "2", "--steps", "3",
                                      "--warmup", "1", "--settle-s", "0.05", "--no-secondary", "--no-cpu-baseline"])
    _FakeEngine.instances.clear()
    bench.main()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    d = json.loads(lines[-1])
    eng = _FakeEngine.instances[0]
    assert eng.steps == (1 + 3 + 3) * 2 and eng.probe_steps == 3 * 2   # warm-up, timed, then the clock batch
    assert d["verified"] is True and d["verify"][0]["generations"] == (1 + 3) * 2
    assert d["clock"]["sclk_mhz"] == 2300.0 and d["clock"]["probe_batch_ms_per_step"] > 0
    assert d["aged_board"]["sclk_mhz"] == 2300.0


def _rank_probe(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import mpi_amd
    from mpi_amd import golhip
    golhip.Engine = _ProbeFakeEngine
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
    q.put((rank, out.getvalue(), e.probe_steps))


def test_bench_world2_clock_batch():
    """N = 2 with the probe: every rank runs the clock batch (its steps exchange
    halos), the seam window is taken before it and verifies."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_probe, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, s)) for r, o, s in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = json.loads([ln for ln in res[0][0].splitlines() if ln.strip()][0])
    assert res[0][1] == res[1][1] == 3 * 2
    assert d["verified"] is True and any("seam" in v for v in d["verify"])
    assert d["clock"]["sclk_mhz"] == 2300.0
