#!/usr/bin/env python3
"""bench.py — GCUPS of the MI355X Game-of-Life engine (BASELINE.json's metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload bit131072|byte32768] [-k K]

One step = one pass of the hot path over the grid: ONE fused launch of
`k` generations (plus, for N>1, one k-row halo exchange over RCCL).  The timed
region is exactly K steps, bracketed by a barrier and a device sync on both
sides; the time is the max over ranks.  Inputs (the glibc-seeded board) are
generated on the device before timing, so they are resident in HBM.

Workloads (BASELINE.json configs):
  bit131072  (default) config 4/5: bit-packed 131072×131072 per GPU, dead
             boundary, srand(1) row-major stream; N>1 = weak-scaling row slabs
             (global grid N·131072 × 131072), halos by RCCL send/recv.
  byte32768  config 3: byte-per-cell 32768×32768 per GPU (byte board in HBM,
             bit-sliced core in registers, k=28 generations per pass).

For N>1 the driver launches this file under torch.distributed.run; ranks find
each other through torch.distributed (gloo, control plane only: barrier, max
of the timings, broadcast of the RCCL unique id); the halo rows go over the
library's own RCCL communicator.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md (spec)
VALU_PEAK = 256 * 4 * 32 * 2.4e9   # lane-ops/s: 256 CU × 4 SIMD-32 × 2.4 GHz

WORKLOADS = {
    "bit131072": dict(layout="bit", rows=131072, cols=131072, bytes_per_cell=0.25),
    "byte32768": dict(layout="byte", rows=32768, cols=32768, bytes_per_cell=2.0),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default: 1000 generations)")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", default="bit131072", choices=sorted(WORKLOADS))
    p.add_argument("-k", "--tblock-k", type=int, default=None, help="generations fused per launch")
    p.add_argument("--rows", type=int, default=None, help="rows per GPU (override)")
    p.add_argument("--cols", type=int, default=None)
    p.add_argument("--wpl", type=int, default=None, help="bit layout: words per lane (1,2,4)")
    p.add_argument("--chunk", type=int, default=None, help="rows per wave chunk")
    p.add_argument("--single-process", action="store_true",
                   help="N slabs in this process (peer copies) instead of one rank per GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the short runs of the other BASELINE configs reported beside the metric")
    return p.parse_args()


# ---------------------------------------------------------------- cpu baseline

def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def serial_baseline() -> dict | None:
    """main_serial.cpp (BASELINE config 1: 1024², 100 generations) on one core:
    the unmodified reference program (oracle/_ref/gol_serial), wall time of the
    whole run (it has no timer of its own; init and its generation-0 .gol write
    are included, ≈10 % at this size)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "gol_serial")
    if not os.path.exists(exe):
        return None
    n, gens = 1024, 100
    tmp = tempfile.mkdtemp(prefix="golser")
    try:
        t = time.perf_counter()
        r = subprocess.run([exe, str(n), str(n), "100000", str(gens)], cwd=tmp, capture_output=True, text=True,
                           timeout=120)
        dt = time.perf_counter() - t
        if r.returncode != 0:
            return None
        return {"value": n * n * gens / dt / 1e9, "unit": "GCUPS", "cores": 1, "kind": "reference",
                "sample": f"main_serial.cpp (reference, g++ -O2) {n}x{n}, {gens} generations, wall time incl. "
                          f"init + gen-0 write", "seconds": dt}
    except Exception as e:
        log("serial cpu baseline failed:", e)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_baseline() -> dict:
    """The reference's own CPU path on this host's cores, bounded to ~10-30 s.

    Prefers the real main.cpp (oracle/_ref/gol_mpi, built from /root/reference
    by oracle/Makefile) under mpirun; falls back to the oracle's bool**-layout
    restatement of main.cpp:79-103 on one core."""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    budget = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    cores = max(1, min(ncpu, budget, 16))
    exe = os.path.join(ROOT, "oracle", "_ref", "gol_mpi")
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    n = 16384
    if os.path.exists(exe) and os.path.exists(mpirun):
        P = max(p for p in (1, 4, 16) if p <= cores)   # √P | 16384 (main.cpp:195)
        gens = 4 * P
        tmp = tempfile.mkdtemp(prefix="golcpu")
        try:
            r = subprocess.run([mpirun, "-np", str(P), exe, str(n), str(n), "100000", str(gens), "tf"],
                               cwd=tmp, capture_output=True, text=True, timeout=240)
            row = open(os.path.join(tmp, "tf_compact.csv")).read().strip().splitlines()[-1].split(",")
            nosetup_us = float(row[6])   # "nosetup single" (rank 0), main.cpp:313,362
            if r.returncode == 0 and nosetup_us > 0:
                return {"value": n * n * gens / (nosetup_us * 1e-6) / 1e9, "unit": "GCUPS", "cores": P,
                        "kind": "reference",
                        "sample": f"main.cpp (reference, g++ -O2, MPICH) mpirun -np {P}, {n}x{n}, {gens} "
                                  f"generations, rank-0 'nosetup' time (main.cpp:313)",
                        "cpu_model": _cpu_model(), "seconds": nosetup_us * 1e-6}
        except Exception as e:   # fall through to the port
            log("reference cpu baseline failed:", e)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    from oracle import golcpu
    L, gens = 4096, 20
    t = time.perf_counter()
    golcpu.ref_shaped_run(L, gens, 1)
    dt = time.perf_counter() - t
    return {"value": L * L * gens / dt / 1e9, "unit": "GCUPS", "cores": 1, "kind": "port",
            "sample": f"oracle restatement of main.cpp:79-103 (bool** layout), {L}x{L}, {gens} generations, "
                      f"1 thread", "cpu_model": _cpu_model(), "seconds": dt}


# ---------------------------------------------------------------- other configs

def secondary_configs(gh, headline: str) -> dict:
    """The other single-GPU BASELINE configs, measured briefly beside the
    headline (not part of `value`): the byte-per-cell board (config 3, k=28) and
    the unfused k=1 bit sweep (the HBM-bound regime).  Same timing rules:
    device-resident input, warm-up, wall time around synchronised steps."""
    out = {}
    runs = [("byte32768_k28", "byte", 32768, 28, 36, 2.0), ("bit131072_k1", "bit", 131072, 1, 100, 0.25)]
    for name, layout, n, k, steps, bpc in runs:
        if headline.startswith(name.split("_")[0]) and name != "bit131072_k1":
            continue
        try:
            with gh.Engine(n, n, layout=layout, tblock_k=k) as e:
                e.initialize_board("stream", 1)
                e.step(3 * k)
                e.sync()
                e.set_option(gh.OPT_KERNEL_TIMING, 1)
                e.kernel_time(reset=True)
                t = time.perf_counter()
                e.step(steps * k)
                e.sync()
                dt = time.perf_counter() - t
                kms, nl = e.kernel_time(reset=True)
            per = kms / max(nl, 1) * 1e-3
            out[name] = {"value": n * n * steps * k / dt / 1e9, "unit": "GCUPS", "generations": steps * k,
                         "gens_per_step": k, "layout": layout, "cells": n * n,
                         "hbm_GBps_algorithmic": bpc * n * n / per / 1e9 if per > 0 else None,
                         "hbm_frac": bpc * n * n / per / HBM_PEAK if per > 0 else None}
        except Exception as ex:   # never let a side measurement break the contract line
            out[name] = {"error": repr(ex)}
    return out


# ---------------------------------------------------------------- main

def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_amd import golhip as gh

    wl = dict(WORKLOADS[args.workload])
    rows_per = args.rows or wl["rows"]
    cols = args.cols or wl["cols"]
    k = args.tblock_k or (8 if wl["layout"] == "bit" else 28)   # byte: the bit-sliced core, 28 gens/pass
    steps = args.steps if args.steps is not None else max(1, round(1000 / k))
    n_total = world if world > 1 else args.gpus
    rows = rows_per * n_total

    if world > 1:
        uid = [gh.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        # GOL_DEVICE_MOD=m maps ranks onto m devices (rehearsal of the RCCL path on fewer GPUs)
        dev = local % int(os.environ["GOL_DEVICE_MOD"]) if os.environ.get("GOL_DEVICE_MOD") else local
        eng = gh.Engine(rows, cols, rank=rank, world=world, device=dev, uid=uid[0], layout=wl["layout"],
                        tblock_k=k)
    else:
        eng = gh.Engine(rows, cols, n_gpus=args.gpus if args.single_process else 1, layout=wl["layout"],
                        tblock_k=k)
        if args.gpus > 1 and not args.single_process:
            raise SystemExit("--gpus N>1 is launched by torch.distributed.run (or pass --single-process)")
    if args.wpl:
        eng.set_option(gh.OPT_WORDS_PER_LANE, args.wpl)
    if args.chunk:
        eng.set_option(gh.OPT_CHUNK_ROWS, args.chunk)

    t_init = time.perf_counter()
    eng.initialize_board("stream", 1)
    eng.sync()
    t_init = time.perf_counter() - t_init
    eng.step(args.warmup * k)
    eng.sync()
    eng.set_option(gh.OPT_KERNEL_TIMING, 1)
    eng.kernel_time(reset=True)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    eng.sync()
    t0 = time.perf_counter()
    eng.step(steps * k)
    dev_ms = eng.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms, launches = eng.kernel_time(reset=True)
    live = eng.popcount()
    if dist is not None:
        import torch
        t = torch.tensor([live], dtype=torch.int64)
        dist.all_reduce(t)
        live = int(t.item())

    gens = steps * k
    cells = rows * cols
    value = cells * gens / elapsed / 1e9

    # roofline of the dominant kernel (the pipelined stencil), per launch:
    # algorithmic bytes = one read + one write of the local grid = bytes_per_cell × cells
    local_rows = rows_per if (world > 1) else rows
    if world > 1 or args.single_process and args.gpus > 1:
        local_rows = max(1, rows_per - 2 * k)   # timed launches are the interior ones
    launch_bytes = wl["bytes_per_cell"] * local_rows * cols
    avg_launch_s = (kernel_ms / max(launches, 1)) * 1e-3
    achieved = launch_bytes / avg_launch_s if avg_launch_s > 0 else 0.0
    traffic, tr_rec = None, None
    tr_key = f"{args.workload}_k{k}"
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath) and not (args.wpl or args.chunk or args.rows or args.cols):
        try:
            tr_rec = json.load(open(tpath)).get(tr_key)
            if tr_rec:
                traffic = tr_rec["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic, tr_rec = None, None
    valu = None
    if tr_rec is not None and tr_rec.get("valu_insts_per_launch") and avg_launch_s > 0:
        lane_ops = tr_rec["valu_insts_per_launch"] * 64 / avg_launch_s
        measured = None
        probe = os.path.join(ROOT, "profiles", "r01_valu_probe.jsonl")
        if os.path.exists(probe):
            for ln in open(probe):
                try:
                    rec = json.loads(ln)
                except ValueError:
                    continue
                if rec.get("probe", "").startswith("v_xor_b32"):
                    measured = rec["Tlane_ops"] * 1e12
        valu = {"achieved": lane_ops / 1e12, "peak": VALU_PEAK / 1e12, "unit": "Tlane-op/s",
                "frac": lane_ops / VALU_PEAK,
                "peak_measured": measured / 1e12 if measured else None,
                "frac_of_measured": lane_ops / measured if measured else None,
                "ops_per_cell_update": tr_rec["valu_insts_per_launch"] * 64 / (local_rows * cols * k),
                "source": f"SQ_INSTS_VALU from profiles/traffic.json[{tr_key}]"}
    copy_peak = None   # best STREAM-style copy on this GPU model (tools/hbm_probe.hip, committed profile)
    cpath = os.path.join(ROOT, "profiles", "r01d_hbm_probe.jsonl")
    if os.path.exists(cpath):
        for ln in open(cpath):
            try:
                rec = json.loads(ln)
            except ValueError:
                continue
            if "copy" in rec.get("probe", "") and rec.get("GBps"):
                copy_peak = max(copy_peak or 0.0, rec["GBps"])
    roofline = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "traffic_GBps": traffic / avg_launch_s / 1e9 if (traffic and avg_launch_s > 0) else None,
                "copy_calibration_GBps": copy_peak,
                "frac_of_copy": (achieved / 1e9 / copy_peak) if copy_peak else None,
                "effective_GBps": value * 1e9 * wl["bytes_per_cell"] / 1e9,   # bytes a k=1 sweep would move
                "effective_frac": value * 1e9 * wl["bytes_per_cell"] / HBM_PEAK,
                "frac": achieved / HBM_PEAK, "traffic": traffic, "valu": valu,
                "kernel": (f"bytebit_pipe_kernel<k={k}>" if wl["layout"] == "byte" and k in (4, 8, 12, 16, 20, 24, 28, 32)
                           else f"{wl['layout']}_pipe_kernel<k={k}>"),
                "kernel_avg_ms": avg_launch_s * 1e3, "launches": launches,
                "bytes_per_launch": launch_bytes,
                "note": f"algorithmic bytes {wl['bytes_per_cell']} B/cell per launch = "
                        f"{wl['bytes_per_cell'] / k:.4g} B per cell-update at k={k}"}

    result = {
        "metric": "cell updates/sec (GCUPS) at 1/2/4/8 MI355X; % of HBM bandwidth roofline",
        "value": value,
        "unit": "GCUPS",
        "n_gpus": n_total,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if wl["layout"] == "bit" else "u8",
        "data": "synthetic (glibc srand(1) rand()%3==0 stream, generated on device)",
        "config": {"workload": f"{args.workload}: {wl['layout']}-packed {rows_per}x{cols} per GPU, "
                               f"{k} generations fused per step, dead boundary",
                   "rows": rows, "cols": cols, "generations": gens, "gens_per_step": k,
                   "parallelism": f"row-slabs x{n_total}" + (" (rccl halos)" if world > 1 else ""),
                   "global_cells": cells},
        "roofline": roofline,
        "device_ms": dev_ms,
        "init_s": t_init,
        "live_cells": live,
    }
    eng.close()
    if world == 1 and not args.single_process and not args.no_secondary:
        result["secondary"] = secondary_configs(gh, args.workload)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline()
        cb["serial"] = serial_baseline()
        result["cpu_baseline"] = cb
        result["speedup_vs_cpu"] = value / cb["value"] if cb["value"] else None
    elif rank == 0:
        result["cpu_baseline"] = None
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
