#!/usr/bin/env python3
"""Real RCCL between two processes on ONE GPU (test infrastructure).

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"),
so each rank process sets its own NCCL_HOSTID: RCCL then takes them for two
hosts and moves the halos through its network transport (sockets on the
loopback interface, staged through host memory) — slower than xGMI, but the
library's RCCL-mode path runs for real: gol_create_rank over a real
communicator, exchange() with ncclSend/ncclRecv of both neighbours in one
group, the boundary and seam bands, the schedule trial's ncclAllReduce.

    python tests/rccl_real2_check.py            (parent: spawns the 2 ranks, checks)
    python tests/rccl_real2_check.py --cases N [--seed S]
                                                (random worlds 2-4, layouts, depths, boundaries)
    python tests/rccl_real2_check.py rank R DIR (a rank; the parent starts these)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS, COLS, K = 2 * 1200, 4096, 8
STEPS = [8] * 402 + [3] + [8] * 40 + [5, 8]   # through the k = 8 trial (restarted by the short step)


def rank_main(r, d):
    import json

    import numpy as np
    sys.path.insert(0, ROOT)
    from mpi_amd import golhip as gh
    case = json.load(open(os.path.join(d, "case.json"))) if os.path.exists(os.path.join(d, "case.json")) else None
    uid_path = os.path.join(d, "uid.bin")
    if r == 0:
        uid = gh.unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(uid_path + ".tmp", uid_path)
    else:
        t0 = time.time()
        while not os.path.exists(uid_path):
            if time.time() - t0 > 60:
                raise SystemExit("rank 1: no unique id from rank 0")
            time.sleep(0.05)
        uid = open(uid_path, "rb").read()
    if case:   # a random case: upload the board, step, download the slab
        W, rows, cols = case["world"], case["rows"], case["cols"]
        b0 = np.load(os.path.join(d, "b0.npy"))
        with gh.Engine(rows, cols, rank=r, world=W, device=0, uid=uid, layout=case["layout"], tblock_k=case["k"],
                       boundary=case["boundary"]) as e:
            e.set_option(gh.OPT_INTERIOR_SPLIT, case["split"])
            e.upload(b0)
            for st in case["steps"]:
                e.step(st)
            e.sync()
            r0, n = gh.slab_plan(rows, W, r)
            np.save(os.path.join(d, f"slab{r}.npy"), e.download_window(r0, 0, n, cols))
        return
    with gh.Engine(ROWS, COLS, rank=r, world=2, device=0, uid=uid, layout="bit", tblock_k=K) as e:
        e.initialize_board("stream", 1)
        for st in STEPS:
            e.step(st)
        e.sync()
        r0, n = gh.slab_plan(ROWS, 2, r)
        np.save(os.path.join(d, f"slab{r}.npy"), e.download_window(r0, 0, n, COLS))
        with open(os.path.join(d, f"state{r}.txt"), "w") as f:
            f.write(f"{e.get_option(gh.OPT_CHUNK_ROWS)} {e.get_option(gh.OPT_SCHEDULE_TRIAL)} "
                    f"{e.get_option(gh.OPT_INTERIOR_SPLIT)}\n")
    print(f"rank {r} done", flush=True)


def _spawn(d, world):
    procs = []
    for r in range(world):
        env = dict(os.environ, NCCL_HOSTID=f"golhip-rank{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   NCCL_P2P_DISABLE="1", NCCL_SHM_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "rank", str(r), d], env=env))
    return [p.wait(timeout=240) for p in procs]


def random_cases(n, seed):
    """Random worlds 2-4 through real RCCL against the oracle."""
    import json
    import tempfile

    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import golcpu as g
    rng = np.random.default_rng(seed)
    fails = 0
    for i in range(n):
        world = int(rng.integers(2, 5))
        layout = str(rng.choice(["bit", "byte"]))
        k = int(rng.choice([8, 8, 5, 3, 1] if layout == "bit" else [32, 28, 8, 1]))
        boundary = str(rng.choice(["dead", "serial_compat"]))
        rows = world * int(rng.integers(max(2 * k, 8) + 1, 700))
        cols = int(rng.integers(40, 3000))
        gens = int(rng.integers(1, 3 * k + 10))
        steps, done = [], 0
        while done < gens:
            steps.append(int(rng.integers(1, gens - done + 1)))
            done += steps[-1]
        b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
        mode = g.DEAD
        if boundary == "serial_compat":
            b0[-1, :] = 0
            b0[:, -1] = 0
            mode = g.SERIAL_COMPAT
        case = dict(world=world, rows=rows, cols=cols, layout=layout, k=k, boundary=boundary, steps=steps,
                    split=int(rng.choice([1, 2, 3])))
        with tempfile.TemporaryDirectory() as d:
            json.dump(case, open(os.path.join(d, "case.json"), "w"))
            np.save(os.path.join(d, "b0.npy"), b0)
            rc = _spawn(d, world)
            if any(rc):
                print("ERROR", i, case, rc, flush=True)
                fails += 1
                continue
            got = np.concatenate([np.load(os.path.join(d, f"slab{r}.npy")) for r in range(world)])
        bad = int((got != g.run(b0, sum(steps), mode)).sum())
        print(f"case {i}: {case} {'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
        fails += bad > 0
    print(f"real rccl random cases: {n}, failures {fails}")
    if fails:
        raise SystemExit(1)
    print("real rccl cases ok")


def parent():
    import tempfile

    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import golcpu as g
    with tempfile.TemporaryDirectory() as d:
        rc = _spawn(d, 2)
        if any(rc):
            raise SystemExit(f"rank exit codes {rc}")
        got = np.concatenate([np.load(os.path.join(d, f"slab{r}.npy")) for r in range(2)])
        states = [open(os.path.join(d, f"state{r}.txt")).read().split() for r in range(2)]
    want = g.run_dead_fast(g.init_dead(ROWS, COLS, 1), sum(STEPS))
    bad = int((got != want).sum())
    print(f"real rccl world=2 on one GPU (net transport): {ROWS}x{COLS} bit k={K}, {sum(STEPS)} generations, "
          f"states {states}, {'ok' if bad == 0 else f'{bad} cells differ'}", flush=True)
    if bad or states[0] != states[1] or states[0][1] != "2":
        raise SystemExit(1)
    print("real rccl 2-rank ok")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "rank":
        rank_main(int(sys.argv[2]), sys.argv[3])
    elif "--cases" in sys.argv:
        random_cases(int(sys.argv[sys.argv.index("--cases") + 1]),
                     int(sys.argv[sys.argv.index("--seed") + 1]) if "--seed" in sys.argv else 1)
    else:
        parent()
