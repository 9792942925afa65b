"""Happens-before check of a recorded schedule (GOL_OPT_SCHED_TRACE,
gol_sched_trace): finds two accesses of the same board rows, at least one a
write, that the streams' order, the event edges and the host syncs leave
unordered — a race whatever the timing, found from the enqueue order alone.

Model (HIP semantics on non-blocking streams): work on one stream runs in
order; hipEventRecord(e, s) captures everything enqueued on s so far;
hipStreamWaitEvent(t, e) makes later work on t wait for e's most recent
record; a host-side stream or event sync orders everything enqueued after it
behind what it waited for.  Vector clocks per stream carry these edges.
"""
import numpy as np

RECORD, WAIT, STREAM_SYNC, EVENT_SYNC, READ, WRITE = 1, 2, 3, 4, 5, 6


def _join(a: dict, b: dict) -> None:
    for k, v in b.items():
        if a.get(k, 0) < v:
            a[k] = v


def find_races(ops, limit: int = 20):
    """ops: (n, 7) int array (kind, stream, event, slab, buffer, row0, row1).
    Returns up to `limit` races as (earlier op index, later op index, text)."""
    ops = np.asarray(ops, np.int64).reshape(-1, 7)
    vcs, events, host = {}, {}, {}
    # per (slab, buffer): per stream, the accesses in enqueue order (epoch, row0, row1, write, op index)
    hist = {}
    races = []
    for i, (kind, st, ev, slab, buf, r0, r1) in enumerate(ops.tolist()):
        if kind in (RECORD, WAIT, READ, WRITE):
            vc = vcs.setdefault(st, {})
            _join(vc, host)
        if kind == RECORD:
            events[ev] = dict(vc)
        elif kind == WAIT:
            _join(vc, events.get(ev, {}))
        elif kind == STREAM_SYNC:
            _join(host, vcs.get(st, {}))
        elif kind == EVENT_SYNC:
            _join(host, events.get(ev, {}))
        elif kind in (READ, WRITE):
            if r1 <= r0:
                continue
            vc[st] = vc.get(st, 0) + 1
            write = kind == WRITE
            per_stream = hist.setdefault((slab, buf), {})
            for other, acc in per_stream.items():
                if other == st:
                    continue
                seen = vc.get(other, 0)
                for epoch, a0, a1, aw, j in reversed(acc):
                    if epoch <= seen:
                        break   # this one and every earlier one on `other` are ordered before us
                    if (aw or write) and a0 < r1 and r0 < a1 and len(races) < limit:
                        races.append((j, i, f"slab {slab} buffer {buf}: {'write' if aw else 'read'} rows "
                                            f"[{a0},{a1}) on stream {other:#x} (op {j}) and "
                                            f"{'write' if write else 'read'} rows [{r0},{r1}) on stream "
                                            f"{st:#x} (op {i}) are unordered"))
            per_stream.setdefault(st, []).append((vc[st], r0, r1, write, i))
    return races
