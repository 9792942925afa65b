"""The happens-before checker of tests/sched_race.py on synthetic schedules
(CPU): it must flag unordered conflicting accesses and accept the orderings
HIP guarantees (stream order, event record -> wait, host syncs)."""
from sched_race import EVENT_SYNC, READ, RECORD, STREAM_SYNC, WAIT, WRITE, find_races

S1, S2, S3, E1, E2 = 0x10, 0x20, 0x30, 0x100, 0x200


def op(kind, st=0, ev=0, slab=0, buf=0, r0=0, r1=0):
    return [kind, st, ev, slab, buf, r0, r1]


def test_unordered_write_read_is_a_race():
    races = find_races([op(WRITE, S1, r0=0, r1=10), op(READ, S2, r0=5, r1=15)])
    assert len(races) == 1 and races[0][:2] == (0, 1)


def test_event_edge_orders():
    assert not find_races([op(WRITE, S1, r0=0, r1=10), op(RECORD, S1, E1), op(WAIT, S2, E1),
                           op(READ, S2, r0=5, r1=15)])


def test_record_before_the_write_does_not_order_it():
    assert find_races([op(RECORD, S1, E1), op(WRITE, S1, r0=0, r1=10), op(WAIT, S2, E1),
                       op(READ, S2, r0=5, r1=15)])


def test_wait_uses_the_latest_record():
    # E1 re-recorded after the write: a wait enqueued after that re-record orders the read
    assert not find_races([op(RECORD, S1, E1), op(WRITE, S1, r0=0, r1=10), op(RECORD, S1, E1),
                           op(WAIT, S2, E1), op(READ, S2, r0=0, r1=1)])


def test_host_syncs_order():
    assert not find_races([op(WRITE, S1, r0=0, r1=10), op(STREAM_SYNC, S1), op(WRITE, S2, r0=0, r1=10)])
    assert not find_races([op(WRITE, S1, r0=0, r1=10), op(RECORD, S1, E2), op(EVENT_SYNC, ev=E2),
                           op(READ, S3, r0=9, r1=11)])
    # a sync of another stream orders nothing
    assert find_races([op(WRITE, S1, r0=0, r1=10), op(STREAM_SYNC, S3), op(WRITE, S2, r0=0, r1=10)])


def test_disjoint_rows_buffers_slabs_and_reads_only():
    assert not find_races([op(WRITE, S1, r0=0, r1=10), op(WRITE, S2, r0=10, r1=20)])
    assert not find_races([op(WRITE, S1, buf=0, r0=0, r1=10), op(WRITE, S2, buf=1, r0=0, r1=10)])
    assert not find_races([op(WRITE, S1, slab=0, r0=0, r1=10), op(WRITE, S2, slab=1, r0=0, r1=10)])
    assert not find_races([op(READ, S1, r0=0, r1=10), op(READ, S2, r0=0, r1=10)])


def test_transitive_order_through_a_third_stream():
    assert not find_races([op(WRITE, S1, r0=0, r1=4), op(RECORD, S1, E1), op(WAIT, S3, E1), op(RECORD, S3, E2),
                           op(WAIT, S2, E2), op(WRITE, S2, r0=2, r1=3)])


def test_moving_cut_pattern():
    """The pattern of the round-5 split bug: part j+1 of step t-1 reads rows
    from the cut on, part j of step t (another stream) writes up to a cut that
    moved up; both only wait for the seam band's event, so the checker flags
    the write-after-read."""
    ops = [op(READ, S2, buf=0, r0=791, r1=900),     # part 3, step t-1, input buffer 0
           op(RECORD, S1, E1),                      # seam bands of t-1 (comm stream S1)
           op(WAIT, S3, E1),
           op(WRITE, S3, buf=0, r0=600, r1=792)]    # part 2, step t, output = buffer 0
    races = find_races(ops)
    assert len(races) == 1 and "write" in races[0][2]
