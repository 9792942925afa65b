"""The runtime's real step schedule, recorded (GOL_OPT_SCHED_TRACE) and
checked for races by happens-before (tests/sched_race.py): every board access
of one stream must be ordered by stream order, events or host syncs against
every conflicting access of another.  Unlike a parity test this does not
depend on timing: an unordered pair is reported even when the run happened
to come out right.  Shapes: one slab and several (peer halos), the interior
split into 1-4 parts, overlap on and off, uneven step depths (the short
blocks that move band and seam geometry), window copies mid-run."""
import numpy as np
import pytest

from sched_race import READ, WRITE, find_races

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def run_traced(gh, rows, cols, slabs, layout, k, split, steps, overlap=1, chunk=None):
    with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
        e.initialize_board("stream", 7)
        e.set_option(gh.OPT_OVERLAP, overlap)
        e.set_option(gh.OPT_INTERIOR_SPLIT, split)
        if chunk is not None:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
        e.set_option(gh.OPT_SCHED_TRACE, 1)
        for i, st in enumerate(steps):
            e.step(st)
            if i == len(steps) // 2:   # a window copy behind the steps enqueued so far
                e.download_window_async(rows // 2 - 3, 0, 6, min(cols, 64))
            if i == len(steps) // 2 + 1:   # and a window upload (synchronous) two steps on
                e.upload_window(rows // 3, 0, np.ones((5, min(cols, 40)), np.uint8))
        e.sync()
        ops = e.sched_trace()
        e.set_option(gh.OPT_SCHED_TRACE, 0)
    return ops


CASES = [  # rows, cols, slabs, layout, k, split, steps, overlap
    (2116, 47, 2, "bit", 5, 4, [14, 11, 5, 1, 5, 2, 9, 1, 1, 13], 1),   # the fuzz case (moved cuts)
    (2116, 47, 2, "bit", 5, 3, [14, 11, 5, 1, 5, 2, 9, 1, 1, 13], 1),
    (4096, 2100, 1, "bit", 8, 2, [8, 8, 3, 8, 1, 8, 8, 5, 8], 1),
    (4096, 2100, 1, "bit", 8, 4, [8, 8, 3, 8, 1, 8, 8, 5, 8], 1),
    (3 * 1200, 2100, 3, "bit", 8, 2, [8, 3, 8, 8, 1, 8, 6, 8], 1),
    (3 * 1200, 2100, 3, "bit", 8, 3, [8, 3, 8, 8, 1, 8, 6, 8], 1),
    (3 * 1200, 2100, 3, "bit", 8, 2, [8, 3, 8, 8, 1, 8], 0),
    (2 * 1500, 300, 2, "bit", 3, 4, [3, 1, 3, 2, 3, 3, 1], 1),
    (2 * 2600, 4100, 2, "byte", 32, 2, [32, 7, 32, 1, 32], 1),
    (2 * 700, 4100, 2, "byte", 8, 1, [8, 5, 8, 8, 2, 8], 1),
]


@pytest.mark.parametrize("rows,cols,slabs,layout,k,split,steps,overlap", CASES)
def test_step_schedule_has_no_race(gh, rows, cols, slabs, layout, k, split, steps, overlap):
    ops = run_traced(gh, rows, cols, slabs, layout, k, split, steps, overlap)
    writes = int((ops[:, 0] == WRITE).sum())
    assert writes >= len(steps) * slabs and int((ops[:, 0] == READ).sum()) >= writes
    races = find_races(ops)
    assert not races, "\n".join(r[2] for r in races)


def test_trace_off_records_nothing(gh):
    with gh.Engine(512, 256, n_gpus=2, layout="bit", tblock_k=4) as e:
        e.initialize_board("stream", 1)
        e.step(9)
        e.sync()
        assert e.get_option(gh.OPT_SCHED_TRACE) == 0 and len(e.sched_trace()) == 0


def test_checker_sees_the_real_edges(gh):
    """Control: the same recorded schedule with its event waits removed must
    show races — the check above passes because of the runtime's edges, not
    because it saw nothing."""
    from sched_race import WAIT
    ops = run_traced(gh, 2116, 47, 2, "bit", 5, 4, [5, 5, 1, 5], 1)
    assert not find_races(ops)
    assert find_races(ops[ops[:, 0] != WAIT])


@pytest.mark.parametrize("slabs", [1, 2])
def test_schedule_with_the_k8_trial_has_no_race(gh, slabs):
    """440 k-steps at k = 8 (the schedule trial runs: its marks join the comm
    and part streams into the compute stream), one short step inside the
    trial, the default split."""
    rows, cols = 1200 * slabs, 2100
    with gh.Engine(rows, cols, n_gpus=slabs, layout="bit", tblock_k=8) as e:
        e.initialize_board("stream", 5)
        e.set_option(gh.OPT_SCHED_TRACE, 1)
        for i in range(440):
            e.step(3 if i == 410 else 8)
        e.sync()
        ops = e.sched_trace()
        assert e.get_option(gh.OPT_SCHEDULE_TRIAL) == 2
    races = find_races(ops)
    assert not races, "\n".join(r[2] for r in races)
