"""Runs the library's RCCL transport (one gol_ctx per rank, halos by
ncclSend/ncclRecv) with every rank as a host thread on ONE GPU, over
tests/shim/libfake_rccl.so (see its header), and checks the gathered slabs
bit-exactly against the oracle.  Test infrastructure: started in a fresh
process by tests/test_gpu_rccl_shim.py, because the shim must be in the global
symbol scope before libgolhip.so first resolves RCCL.

    python tests/rccl_shim_check.py <libfake_rccl.so> [--config5]
"""
import ctypes
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)

import numpy as np  # noqa: E402

from mpi_amd import golhip as gh  # noqa: E402
from oracle import golcpu as g  # noqa: E402


def run_ranks(world, rows, cols, layout, k, gens, boundary, b0, overlap=1, steps=None):
    uid = gh.unique_id()
    out = [None] * world
    errs = []

    def worker(r):
        try:
            e = gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout=layout, tblock_k=k,
                          boundary=boundary)
            try:
                e.set_option(gh.OPT_OVERLAP, overlap)
                e.upload(b0)
                for st in (steps or [gens]):
                    e.step(st)
                e.sync()
                row0, n = gh.slab_plan(rows, world, r)
                out[r] = (row0, e.download_window(row0, 0, n, cols))
            finally:
                e.close()
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    if any(t.is_alive() for t in ts):
        raise SystemExit(f"rank threads hung (world={world})")
    if errs:
        raise SystemExit(f"rank errors: {errs}")
    got = np.zeros((rows, cols), np.uint8)
    for row0, w in out:
        got[row0:row0 + w.shape[0]] = w
    return got


def config5():
    """BASELINE config 5 through the RCCL transport: 8 rank contexts (threads,
    all on this GPU, halos over the shim) of 131072 rows × 131072 columns each,
    device init of the global srand(1) stream, uneven k-steps; every rank
    checks light-cone windows at its top and bottom slab edges (the rows its
    halo exchange feeds) and across its middle (the seam band of the split
    interior, the k = 8 default) against the oracle."""
    world, H, cols, k = 8, 131072, 131072, 8
    rows = world * H
    steps = [8, 3, 8, 8, 5, 8, 8]
    gens = sum(steps)
    uid = gh.unique_id()
    got, errs = {}, []

    def worker(r):
        try:
            with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout="bit", tblock_k=k) as e:
                e.initialize_board("stream", 1)
                for st in steps:
                    e.step(st)
                e.sync()
                # the slab's top and bottom edges (its halos) and its middle (the split interior's seam band)
                for r0, c0 in ((r * H, (r * 7919) % (cols - 64)), ((r + 1) * H - 64, (r * 104729) % (cols - 64)),
                               (r * H + H // 2 - 32, (r * 15485863) % (cols - 64))):
                    got[(r0, c0)] = e.download_window(r0, c0, 64, 64)
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    if errs or any(t.is_alive() for t in ts):
        raise SystemExit(f"config-5 ranks failed: {errs}")
    from concurrent.futures import ThreadPoolExecutor
    wins = sorted(got)
    with ThreadPoolExecutor(12) as ex:
        want = list(ex.map(lambda rc: g.lightcone(rows, cols, gens, rc[0], rc[1], 64, 64), wins))
    bad = [(rc, int((got[rc] != w).sum())) for rc, w in zip(wins, want) if (got[rc] != w).any()]
    print(f"config5 world={world} {rows}x{cols} bit k={k} steps={steps}: {len(wins)} windows, "
          f"{'ok' if not bad else bad}", flush=True)
    if bad:
        raise SystemExit(1)
    print("rccl shim config5 ok")


def trial(override=None, split=False):
    """The k=8 schedule trial in RCCL mode: the ranks agree on one policy (an
    ncclAllReduce MAX of their medians at the same k-step on every rank), so
    every rank must report the same GOL_OPT_CHUNK_ROWS once the trial is over
    (GOL_OPT_SCHEDULE_TRIAL reads 2).  A short k-step in the middle of the
    trial restarts it.  The board is checked against one slab in one context.
    override (a step index): rank 3 alone sets GOL_OPT_CHUNK_ROWS = 64 before
    that step, while the trial records (402: before the short step, so the
    restart must not leave rank 3 out; 415: in the restarted recording); it
    must still join the agreement (no hang) and then keep its own policy, the
    others the agreed one.  split: rank 3 instead turns the split interior off
    (GOL_OPT_INTERIOR_SPLIT = 1) at that step — the option that moves the k = 8
    default and candidates; it must not take rank 3 out of the agreement
    either, and rank 3 keeps a policy of the unsplit candidates."""
    world, rows_per, cols, k = 8, 192, 4096, 8
    rows = world * rows_per
    steps = [k] * 405 + [3] + [k] * 62
    with gh.Engine(rows, cols, layout="bit", tblock_k=k) as e:
        e.initialize_board("stream", 1)
        for st in steps:
            e.step(st)
        want = e.download()
    uid = gh.unique_id()
    res, errs = [None] * world, []

    def worker(r):
        try:
            with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout="bit", tblock_k=k) as e:
                e.initialize_board("stream", 1)
                for i, st in enumerate(steps):
                    if override is not None and r == 3 and i == override:
                        if split:
                            e.set_option(gh.OPT_INTERIOR_SPLIT, 1)
                        else:
                            e.set_option(gh.OPT_CHUNK_ROWS, 64)
                    e.step(st)
                e.sync()
                res[r] = (e.get_option(gh.OPT_CHUNK_ROWS), e.get_option(gh.OPT_SCHEDULE_TRIAL),
                          e.download_window(r * rows_per, 0, rows_per, cols))
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    if errs or any(t.is_alive() for t in ts):
        raise SystemExit(f"trial ranks failed: {errs}")
    policies = [p for p, _, _ in res]
    states = [t for _, t, _ in res]
    bad = int((np.concatenate([b for _, _, b in res]) != want).sum())
    print(f"trial world={world} {rows}x{cols} bit k={k} override at {override}: policies {policies}, "
          f"trial states {states}, {'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
    agreed = [p for r, p in enumerate(policies) if not (override is not None and r == 3)]
    if bad or len(set(agreed)) != 1 or agreed[0] not in (-1, -2, -3) or set(states) != {2}:
        raise SystemExit(1)
    if override is not None and policies[3] not in ((-104, -6, -3) if split else (64,)):
        raise SystemExit(1)
    print("rccl shim trial ok")


def sched():
    """Each rank's recorded step schedule (GOL_OPT_SCHED_TRACE) through the RCCL
    transport, checked for races by happens-before (tests/sched_race.py): the
    exchange's sends and receives, the boundary bands, seam bands and interior
    parts of every rank, split 1-3, uneven depths, a window copy mid-run."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from sched_race import find_races
    cases = [(3, 3 * 1200, 2100, "bit", 8, 2, [8, 3, 8, 8, 1, 8, 6, 8]),
             (3, 3 * 1200, 2100, "bit", 8, 3, [8, 3, 8, 8, 1, 8, 6, 8]),
             (2, 2 * 1100, 300, "bit", 5, 1, [5, 2, 5, 5, 1, 5]),
             (4, 4 * 2600, 4100, "byte", 32, 2, [32, 7, 32, 1, 32])]
    for world, rows, cols, layout, k, split, steps in cases:
        uid = gh.unique_id()
        found, errs = [None] * world, []

        def worker(r):
            try:
                with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout=layout, tblock_k=k) as e:
                    e.initialize_board("stream", 3)
                    e.set_option(gh.OPT_INTERIOR_SPLIT, split)
                    e.set_option(gh.OPT_SCHED_TRACE, 1)
                    r0, n = gh.slab_plan(rows, world, r)
                    for i, st in enumerate(steps):
                        e.step(st)
                        if i == len(steps) // 2:
                            e.download_window_async(r0 + n // 2 - 3, 0, 6, 64)
                    e.sync()
                    ops = e.sched_trace()
                    found[r] = (len(ops), find_races(ops))
            except Exception as ex:   # noqa: BLE001
                errs.append((r, repr(ex)))

        ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        if errs or any(t.is_alive() for t in ts):
            raise SystemExit(f"sched ranks failed: {errs}")
        bad = [(r, races) for r, (_, races) in enumerate(found) if races]
        print(f"sched world={world} {layout} k={k} split={split}: ops {[n for n, _ in found]}, "
              f"{'no race' if not bad else bad}", flush=True)
        if bad:
            raise SystemExit(1)
    print("rccl shim sched ok")


def main():
    if "--sched" in sys.argv:
        sched()
        return
    if "--config5" in sys.argv:
        config5()
        return
    if "--trial" in sys.argv:
        trial(override=int(sys.argv[sys.argv.index("--override") + 1]) if "--override" in sys.argv else None,
              split="--split" in sys.argv)
        return
    rng = np.random.default_rng(2024)
    cases = [
        # world, rows, cols, layout, k, gens, boundary, overlap
        (2, 64, 300, "bit", 1, 9, "dead", 1),
        (2, 97, 1000, "bit", 8, 37, "dead", 1),
        (3, 120, 4099, "bit", 4, 29, "dead", 1),
        (4, 200, 700, "bit", 8, 40, "serial_compat", 1),
        (4, 64, 130, "bit", 3, 20, "dead", 0),
        (2, 90, 5000, "byte", 8, 41, "dead", 1),
        (3, 150, 4100, "byte", 16, 50, "dead", 1),
        (2, 80, 333, "byte", 2, 11, "serial_compat", 1),
        (8, 256, 512, "bit", 8, 24, "dead", 1),
    ]
    for world, rows, cols, layout, k, gens, boundary, overlap in cases:
        b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
        mode = g.DEAD
        if boundary == "serial_compat":
            b0[-1, :] = 0
            b0[:, -1] = 0
            mode = g.SERIAL_COMPAT
        want = g.run(b0, gens, mode)
        got = run_ranks(world, rows, cols, layout, k, gens, boundary, b0, overlap)
        bad = int((got != want).sum())
        print(f"world={world} {rows}x{cols} {layout} k={k} gens={gens} {boundary} overlap={overlap}: "
              f"{'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
        if bad:
            raise SystemExit(1)
    # uneven steps: a deeper step after a short one sends rows the previous
    # step's interior kernel wrote (gol_runtime.cpp exchange(), "grow")
    for world, layout, k in [(2, "bit", 8), (3, "byte", 28), (4, "bit", 3)]:
        rows, cols = 60 * world + 7, 2100
        b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
        steps = [1, k, 2, k, k, 1, 3, k]
        want = g.run(b0, sum(steps), g.DEAD)
        got = run_ranks(world, rows, cols, layout, k, sum(steps), "dead", b0, 1, steps)
        bad = int((got != want).sum())
        print(f"world={world} {rows}x{cols} {layout} k={k} uneven steps {steps}: "
              f"{'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
        if bad:
            raise SystemExit(1)

    # bench-shaped: 4 ranks of 2048 x 16384 (bit, k=8, device init of the global
    # srand(1) stream) against the same grid as one slab in one context
    world, rows_per, cols, k, gens = 4, 2048, 16384, 8, 64
    rows = world * rows_per
    with gh.Engine(rows, cols, layout="bit", tblock_k=k) as e:
        e.initialize_board("stream", 1)
        e.step(gens)
        want = e.download()
    uid = gh.unique_id()
    parts, errs = [None] * world, []

    def worker(r):
        try:
            with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout="bit", tblock_k=k) as e:
                e.initialize_board("stream", 1)
                e.step(gens)
                parts[r] = e.download_window(r * rows_per, 0, rows_per, cols)
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    if errs or any(t.is_alive() for t in ts):
        raise SystemExit(f"bench-shaped ranks failed: {errs}")
    bad = int((np.concatenate(parts) != want).sum())
    print(f"world={world} {rows}x{cols} bit k={k} gens={gens} device init vs one slab: "
          f"{'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
    if bad:
        raise SystemExit(1)
    print("rccl shim transport ok")


if __name__ == "__main__":
    main()
