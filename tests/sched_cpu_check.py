#!/usr/bin/env python3
"""Random step schedules of the REAL runtime code, recorded on the CPU
(libgolhip's host code over tests/fake_hip: GOL_LIB=tests/fake_hip/
libgolhip_fakehip.so) and race-checked by happens-before (sched_race.py).
Run by tests/test_sched_cpu.py in a subprocess (the library choice is made at
import).  Results of the fake launches are meaningless; the schedule is real.

    GOL_LIB=tests/fake_hip/libgolhip_fakehip.so python tests/sched_cpu_check.py [cases] [seed]
"""
import ctypes
import os
import sys
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
# RCCL mode: the in-process RCCL stand-in built for the host (tests/shim over the HIP
# stand-in) goes into the global scope first, where the runtime looks for RCCL
if os.environ.get("GOL_RCCL_SHIM"):
    ctypes.CDLL(os.environ["GOL_LIB"], mode=ctypes.RTLD_GLOBAL)
    ctypes.CDLL(os.environ["GOL_RCCL_SHIM"], mode=ctypes.RTLD_GLOBAL)
from mpi_amd import golhip as gh  # noqa: E402
from sched_race import WAIT, find_races  # noqa: E402


def scenario(rng):
    slabs = int(rng.integers(1, 5))
    layout = str(rng.choice(["bit", "bit", "byte"]))
    k = int(rng.choice([16, 8, 8, 5, 3, 1] if layout == "bit" else [48, 32, 28, 8, 1]))
    split = int(rng.integers(1, 5))
    rows = slabs * int(rng.integers(max(2 * k + 1, 40), 32 * k * split + 300))
    cols = int(rng.integers(33, 3000))
    steps = [int(rng.choice([k, k, k, 1, max(1, k - 1), max(1, k // 2)])) for _ in range(int(rng.integers(3, 24)))]
    return dict(slabs=slabs, layout=layout, k=k, split=split, rows=rows, cols=cols, steps=steps,
                overlap=int(rng.random() < 0.8), snaps=[int(rng.integers(0, len(steps))) for _ in range(2)],
                toggle=int(rng.integers(-1, len(steps))))


def run(sc):
    with gh.Engine(sc["rows"], sc["cols"], n_gpus=sc["slabs"], layout=sc["layout"], tblock_k=sc["k"]) as e:
        e.upload(np.zeros((sc["rows"], sc["cols"]), np.uint8))
        e.set_option(gh.OPT_OVERLAP, sc["overlap"])
        e.set_option(gh.OPT_INTERIOR_SPLIT, sc["split"])
        e.set_option(gh.OPT_SCHED_TRACE, 1)
        ops = []
        for i, st in enumerate(sc["steps"]):
            e.step(st)
            if i in sc["snaps"]:
                e.download_window_async(sc["rows"] // 2, 0, min(4, sc["rows"] // 2), min(sc["cols"], 40))
            if i == sc["toggle"]:   # (synchronises: the record so far is checked on its own)
                e.sync()
                ops.append(e.sched_trace())
                e.set_option(gh.OPT_INTERIOR_SPLIT, 1 + sc["split"] % 4)
        e.sync()
        ops.append(e.sched_trace())
    return ops


def run_ranks(rng):
    """One RCCL-mode world (ranks as threads over the stand-in): every rank's
    own schedule (exchange sends/receives, bands, seam bands, parts)."""
    world = int(rng.integers(2, 5))
    layout = str(rng.choice(["bit", "bit", "byte"]))
    k = int(rng.choice([16, 8, 8, 5, 1] if layout == "bit" else [48, 32, 8, 1]))
    split = int(rng.integers(1, 4))
    rows = world * int(rng.integers(max(2 * k + 1, 40), 32 * k * split + 200))
    cols = int(rng.integers(33, 2000))
    steps = [int(rng.choice([k, k, 1, max(1, k - 1)])) for _ in range(int(rng.integers(3, 16)))]
    uid = gh.unique_id()
    out, errs = [None] * world, []

    def worker(r):
        try:
            with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout=layout, tblock_k=k) as e:
                e.upload(np.zeros((rows, cols), np.uint8))
                e.set_option(gh.OPT_INTERIOR_SPLIT, split)
                e.set_option(gh.OPT_SCHED_TRACE, 1)
                for i, st in enumerate(steps):
                    e.step(st)
                    if i == len(steps) // 2:
                        r0, n = gh.slab_plan(rows, world, r)
                        e.download_window_async(r0 + n // 2, 0, 2, min(cols, 40))
                e.sync()
                out[r] = e.sched_trace()
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    if errs or any(t.is_alive() for t in ts):
        raise SystemExit(f"rank threads failed: {errs}")
    return dict(world=world, layout=layout, k=k, split=split, rows=rows, cols=cols, steps=steps), out


def main_rccl(cases, rng):
    bad = 0
    for i in range(cases):
        sc, traces = run_ranks(rng)
        for r, ops in enumerate(traces):
            races = find_races(ops)
            if races:
                bad += 1
                print("RACE", i, r, sc, races[0][2], flush=True)
    print(f"sched cpu rccl: {cases} worlds, {bad} ranks with races", flush=True)
    if bad:
        raise SystemExit(1)
    print("sched cpu rccl ok")


def trial_agreement(override):
    """The k = 8 schedule trial's state machine in RCCL mode (8 ranks as threads):
    every rank reaches the ncclAllReduce agreement (no hang), all keep one policy;
    override = (step, what): rank 3 alone changes an option mid-trial and still
    joins the agreement, keeping its own setting afterwards (a split change: the
    unsplit default -104, never a pick from the medians of the trial's candidates)."""
    world, rows_per, cols, k = 8, 192, 256, 8
    rows = world * rows_per
    steps = [k] * 405 + [3] + [k] * 62
    uid = gh.unique_id()
    res, errs = [None] * world, []

    def worker(r):
        try:
            with gh.Engine(rows, cols, rank=r, world=world, device=0, uid=uid, layout="bit", tblock_k=k) as e:
                for i, st in enumerate(steps):
                    if override and r == 3 and i == override[0]:
                        if override[1] == "chunk":
                            e.set_option(gh.OPT_CHUNK_ROWS, 64)
                        elif override[1] == "split":
                            e.set_option(gh.OPT_INTERIOR_SPLIT, 1)
                        else:
                            e.set_option(gh.OPT_SCHEDULE_TRIAL, 0)
                    e.step(st)
                e.sync()
                res[r] = (e.get_option(gh.OPT_CHUNK_ROWS), e.get_option(gh.OPT_SCHEDULE_TRIAL))
        except Exception as ex:   # noqa: BLE001
            errs.append((r, repr(ex)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    if errs or any(t.is_alive() for t in ts):
        raise SystemExit(f"trial ranks failed or hung: {errs}")
    others = {res[r] for r in range(world) if not (override and r == 3)}
    print(f"trial override {override}: {res}", flush=True)
    if len(others) != 1 or next(iter(others))[1] != 2 or next(iter(others))[0] not in (-1, -2, -3):
        raise SystemExit(1)
    if override and override[1] == "chunk" and res[3][0] != 64:
        raise SystemExit(1)
    if override and override[1] == "split" and res[3][0] != -104:   # the unsplit default, not a pick
        raise SystemExit(1)


def main():
    if os.environ.get("GOL_RCCL_SHIM") and "--trial" in sys.argv:
        for ov in (None, (402, "chunk"), (415, "chunk"), (410, "split"), (410, "trial")):
            trial_agreement(ov)
        print("sched cpu trial ok")
        return
    if os.environ.get("GOL_RCCL_SHIM"):
        main_rccl(int(sys.argv[1]) if len(sys.argv) > 1 else 50,
                  np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1))
        return
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    bad = checked = 0
    for i in range(cases):
        sc = scenario(rng)
        for ops in run(sc):
            checked += len(ops)
            races = find_races(ops)
            if races:
                bad += 1
                print("RACE", i, sc, races[0][2], flush=True)
    # control: the headline shape's schedule without its event waits must race
    sc = dict(slabs=2, layout="bit", k=8, split=2, rows=2400, cols=300, steps=[8, 3, 8, 8], overlap=1, snaps=[],
              toggle=-1)
    ops = run(sc)[-1]
    control = len(find_races(ops[ops[:, 0] != WAIT]))
    print(f"sched cpu: {cases} scenarios, {checked} ops, {bad} with races; control (waits stripped) {control} races",
          flush=True)
    if bad or control == 0:
        raise SystemExit(1)
    print("sched cpu ok")


if __name__ == "__main__":
    main()
