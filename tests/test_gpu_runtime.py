"""Runtime features of the C ABI (GPU): the asynchronous window copy, the
clock probe, the bounded kernel-timing ring, the non-blocking k=8 schedule
trial, the retired options, and REAL RCCL through the library's own binding
(a 1-rank communicator sending halo-sized messages to itself — the pool's
boxes have one GPU, and RCCL refuses two ranks on one device)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def test_rccl_selftest_real(gh):
    """ncclCommInitRank(1 rank) + grouped ncclSend/ncclRecv to self of two
    8-row halos of the 131072-column bit board (8 × 16512 B), 50 groups."""
    us, msg = gh.rccl_selftest(0, 8 * 16512, 50)
    assert msg.startswith("ok"), msg
    assert 0 < us < 10000, us


def test_rccl_selftest_beside_torch():
    """The same in a process that imported torch.distributed first, as bench.py's
    ranks do: torch's own librccl / HIP runtime are then in the process, and the
    library must bind to them (same sonames) and still move the bytes."""
    code = ("import torch.distributed, sys; sys.path.insert(0, %r); from mpi_amd import golhip; "
            "us, msg = golhip.rccl_selftest(0, 65536, 10); print(msg)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ok:" in r.stdout, r.stdout


@pytest.mark.parametrize("layout,slabs,boundary", [("bit", 1, "dead"), ("byte", 1, "dead"), ("bit", 3, "dead"),
                                                    ("byte", 2, "mesh_compat")])
def test_window_async_is_a_snapshot(gh, layout, slabs, boundary):
    """A window copied asynchronously after step A holds generation A even
    though more steps are enqueued before the sync."""
    rng = np.random.default_rng(5 + slabs)
    rows, cols, m = 300, 4100 if boundary == "dead" else 4096, 1 if boundary == "dead" else 4
    b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
    mode = g.DEAD if boundary == "dead" else g.MESH_COMPAT
    with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, boundary=boundary, mesh_m=m, tblock_k=4) as e:
        e.upload(b0)
        e.step(8)
        w1 = e.download_window_async(40, 1000, 200, 3000)
        full = e.download_window_async(0, 0, rows, cols)
        e.step(12)
        w2 = e.download_window_async(0, 3, rows, cols - 3)
        e.sync()
        now = e.download()
    g8, g20 = g.run(b0, 8, mode, m), g.run(b0, 20, mode, m)
    assert (full == g8).all() and (w1 == g8[40:240, 1000:4000]).all()
    assert (w2 == g20[:, 3:]).all() and (now == g20).all()


def test_clock_probe(gh):
    with gh.Engine(8192, 65536, layout="bit", tblock_k=8) as e:
        e.initialize_board("stream", 1)
        e.clock_start(5000.0)
        e.step(8 * 200)
        e.sync()
        mhz, span = e.clock_stop()
    assert 300 < mhz < 3500, mhz
    assert 0.1 < span < 5000, span
    with gh.Engine(64, 64, layout="bit") as e:   # bounded by max_ms with nothing else running
        e.clock_start(20.0)
        mhz, span = e.clock_stop()
        assert span < 1000


def test_kernel_timing_ring_and_launch_count(gh):
    """More timed launches than the event ring holds (1024) in one batch: the
    oldest pairs are harvested on the way; every launch is counted.  Without
    timing the launches are still counted (on the host)."""
    with gh.Engine(64, 256, layout="bit", tblock_k=1) as e:
        e.set_option(gh.OPT_KERNEL_TIMING, 1)
        e.initialize_board("stream", 1)
        e.step(2500)
        ms, n = e.kernel_time(reset=True)
        assert n == 2500 and ms > 0
        e.set_option(gh.OPT_KERNEL_TIMING, 0)
        e.step(37)
        ms, n = e.kernel_time(reset=True)
        assert n == 37 and ms == 0


def test_schedule_trial_nonblocking(gh):
    """The trial never waits on the host: 440 k-steps are enqueued in one
    gol_step while the trial runs inside them; the pick is made once its
    events complete (here: at the sync) and reported by GOL_OPT_SCHEDULE_TRIAL
    = 2.  Turning the trial off keeps the default."""
    rng = np.random.default_rng(3)
    b0 = (rng.random((256, 4096)) < 0.35).astype(np.uint8)
    ref = g.run_dead_fast(b0, 8 * 440)
    for slabs in (1, 3):
        with gh.Engine(256, 4096, n_gpus=slabs, layout="bit", tblock_k=8) as e:
            assert e.get_option(gh.OPT_SCHEDULE_TRIAL) == 1
            e.upload(b0)
            e.step(8 * 440)
            e.sync()
            assert e.get_option(gh.OPT_SCHEDULE_TRIAL) == 2
            # the split interior is the default only where its streams fit the hardware queues
            cand = (-1, -2, -3) if e.get_option(gh.OPT_INTERIOR_SPLIT) >= 2 else (-104, -6, -3)
            assert e.get_option(gh.OPT_CHUNK_ROWS) in cand
            assert (e.download() == ref).all()
    with gh.Engine(256, 4096, layout="bit", tblock_k=8) as e:
        e.set_option(gh.OPT_SCHEDULE_TRIAL, 0)
        e.upload(b0)
        e.step(8 * 440)
        assert e.get_option(gh.OPT_CHUNK_ROWS) == -1 and e.get_option(gh.OPT_SCHEDULE_TRIAL) == 0
        assert (e.download() == ref).all()


def test_retired_options(gh):
    """0.1's option keys stay accepted (no-ops); chunk 0 (the retired work
    queue) is GOL_EUNSUPPORTED with a message."""
    with gh.Engine(64, 64, layout="bit") as e:
        e.set_option(gh.OPT_WORDS_PER_LANE, 4)
        e.set_option(gh.OPT_SPLIT, 0)
        assert e.get_option(gh.OPT_WORDS_PER_LANE) == 2 and e.get_option(gh.OPT_SPLIT) == 1
        with pytest.raises(gh.GolError) as ei:
            e.set_option(gh.OPT_CHUNK_ROWS, 0)
        assert ei.value.code == -5 and "retired" in str(ei.value)
    assert gh.version().startswith("golhip 0.3")


def test_window_async_dropped_reference(gh):
    """The caller may drop the returned array before the sync that fills it:
    the binding keeps it alive until then (the library writes into it)."""
    with gh.Engine(512, 4096, layout="byte", tblock_k=1) as e:
        e.initialize_board("stream", 1)
        for _ in range(20):
            e.download_window_async(0, 0, 512, 4096)   # result discarded at once
            e.step(1)
        e.sync()
        keep = e.download_window_async(100, 100, 64, 64)
        e.sync()
        assert (keep == e.download_window(100, 100, 64, 64)).all()


def test_caller_policy_set_during_trial_stays(gh):
    """A chunk policy the caller sets while the trial is running (or waiting
    for its events) is kept: the trial's pick never overrides it."""
    rng = np.random.default_rng(11)
    b0 = (rng.random((256, 4096)) < 0.35).astype(np.uint8)
    with gh.Engine(256, 4096, layout="bit", tblock_k=8) as e:
        e.upload(b0)
        e.step(8 * 410)              # the trial runs from k-step 400
        e.set_option(gh.OPT_CHUNK_ROWS, 64)
        e.step(8 * 30)
        e.sync()
        assert e.get_option(gh.OPT_CHUNK_ROWS) == 64
        assert (e.download() == g.run_dead_fast(b0, 8 * 440)).all()


def test_window_copy_during_probe_does_not_wait_for_it(gh):
    """A window copy while the clock probe runs (started with a 30-s limit)
    returns at once with the right cells: window copies use the pooled staging
    and stream syncs only.  A copy that would need a new staging allocation,
    the snapshot-text path and re-initialisation refuse (GOL_ESTATE) instead of
    waiting for the probe; after the probe they work."""
    import time
    ref = g.run_dead_fast(g.init_dead(512, 4096, 1), 160)
    for layout in ("bit", "byte"):
        with gh.Engine(512, 4096, layout=layout, tblock_k=8) as e:
            e.initialize_board("stream", 1)          # (an upload would pool a whole-board buffer)
            e.download_window(0, 0, 64, 64)          # pools a staging buffer of this size
            e.step(160)
            e.clock_start(30000.0)
            try:
                t = time.perf_counter()
                w = e.download_window(200, 1000, 64, 64)
                dt = time.perf_counter() - t
                assert dt < 1.0, dt
                assert (w == ref[200:264, 1000:1064]).all()
                with pytest.raises(gh.GolError) as ei:   # 512 x 4096 has no pooled staging yet
                    e.download_window(0, 0, 512, 4096)
                assert ei.value.code == -6 and "probe" in str(ei.value)
                with pytest.raises(gh.GolError) as ei:
                    e.format_text(0, 0, 4, 16)
                assert ei.value.code == -6
                with pytest.raises(gh.GolError) as ei:
                    e.initialize_board("stream", 1)
                assert ei.value.code == -6
            finally:
                mhz, span = e.clock_stop()
            assert span < 20000, span
            assert (e.download() == ref).all()


def test_failed_async_copy_leaves_no_pending_write(gh):
    """gol_download_window_async over two slabs whose second piece cannot get
    staging (probe running, nothing pooled): GOL_ESTATE, and the next sync
    writes nothing into the caller's buffer (no pending entry survives)."""
    import ctypes
    rng = np.random.default_rng(19)
    b0 = (rng.random((256, 2048)) < 0.35).astype(np.uint8)
    with gh.Engine(256, 2048, n_gpus=2, layout="bit", tblock_k=4) as e:
        e.upload(b0)
        e.download_window(0, 0, 128, 2048)        # pools one buffer (slab 0's 128 rows)
        e.clock_start(30000.0)
        try:
            buf = np.full((200, 2048), 0xAB, np.uint8)
            rc = e.lib.gol_download_window_async(e._c, 20, 0, 200, 2048,
                                                 buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 2048)
            assert rc == -6, rc
        finally:
            e.clock_stop()
        e.step(4)
        e.sync()
        assert (buf == 0xAB).all()
        assert (e.download() == g.run_dead_fast(b0, 4)).all()


def test_kernel_timing_ring_three_slabs(gh):
    """The timing ring with 3 slabs (a slab count that does not divide the
    1024-pair ring): past the wrap every pair is (re)made on its slab's device."""
    rng = np.random.default_rng(23)
    b0 = (rng.random((96, 1024)) < 0.35).astype(np.uint8)
    with gh.Engine(96, 1024, n_gpus=3, layout="bit", tblock_k=2) as e:
        e.set_option(gh.OPT_KERNEL_TIMING, 1)
        e.upload(b0)
        e.step(2 * 700)   # 700 steps x 3 timed interior launches = 2100 > 1024
        ms, n = e.kernel_time(reset=True)
        assert n == 2100 and ms > 0
        assert (e.download() == g.run_dead_fast(b0, 1400)).all()


def test_one_probe_per_device(gh):
    """The probe stream is one per device for the whole process: while one
    context's probe runs, another context's gol_clock_start is refused
    (GOL_ESTATE) instead of queueing behind it (its span would include the
    wait); once the first stops, the second can start, and a context destroyed
    with its probe running releases the device's probe.  (Destroying a context
    while ANOTHER context's probe runs still waits for that probe: hipFree
    waits for the device.)"""
    with gh.Engine(64, 256, layout="bit") as a, gh.Engine(64, 256, layout="bit") as b:
        a.clock_start(30000.0)
        try:
            with pytest.raises(gh.GolError) as ei:
                b.clock_start(1000.0)
            assert ei.value.code == -6 and "another context" in str(ei.value)
        finally:
            a.clock_stop()
        c = gh.Engine(64, 256, layout="bit")
        c.clock_start(50.0)
        c.close()   # its own probe was running: stopped, waited for and released here
        b.clock_start(50.0)
        mhz, span = b.clock_stop()
        assert span < 1000
        a.clock_start(50.0)
        a.clock_stop()


def test_staging_pool_reuses_slots(gh):
    """Window copies of growing sizes: an idle pooled pair too small for the
    next copy is freed and its slot reused (the pool does not grow by one
    pinned pair per size), and every copy is right."""
    rng = np.random.default_rng(29)
    b0 = (rng.random((600, 3000)) < 0.35).astype(np.uint8)
    for layout in ("bit", "byte"):
        with gh.Engine(600, 3000, layout=layout, n_gpus=2, tblock_k=2) as e:
            e.upload(b0)
            for h in (8, 40, 100, 250, 600, 30):
                w = e.download_window(0, 7, h, 2900)
                assert (w == b0[:h, 7:2907]).all(), (layout, h)
                keep = e.download_window_async(600 - h, 0, h, 3000)
                e.sync()
                assert (keep == b0[600 - h:]).all(), (layout, h)
            e.step(4)
            assert (e.download() == g.run_dead_fast(b0, 4)).all()
