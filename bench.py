#!/usr/bin/env python3
"""bench.py — GCUPS of the MI355X Game-of-Life engine (BASELINE.json's metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload bit131072|byte32768] [-k K]

One step = one pass of the hot path over the grid: ONE fused launch of
`k` generations (plus, for N>1, one k-row halo exchange).  The timed region is
exactly K steps, bracketed by a barrier and a device sync on both sides; the
time is the max over ranks.  Inputs (the glibc-seeded board) are generated on
the device before timing, so they are resident in HBM.

Workloads (BASELINE.json configs):
  bit131072  (default) config 4/5: bit-packed 131072×131072 per GPU, dead
             boundary, srand(1) row-major stream; N>1 = weak-scaling row slabs
             (global grid N·131072 × 131072), halos by RCCL send/recv.
  byte32768  config 3: byte-per-cell 32768×32768 per GPU (byte board in HBM,
             bit-sliced core in registers, k=32 generations per pass).

The board: the timed steps are generations W·k .. (W+K)·k of the seeded grid
itself (BASELINE config 4's srand(1) row-major stream, main.cpp:68-77).  The
clock settle phase runs on a TWIN board; right after the headline the twin
(aged by the settle phase) is timed the same way (`aged_board`), and a third
board runs config 4 in full, 1000 generations from generation 0
(`config4_1000gen`).

After the timed region every rank checks one light-cone window of its board
against an independent CPU computation (numpy, bit-parallel 8-neighbour
counter) started from a cone copied asynchronously just before the warm-up;
for N>1 ranks one more window straddles every slab seam (its cone halves held
by the two ranks, gathered over gloo): `verify` lists them, `verified` is
their AND.

Clock discipline: an MI355X that idled runs this kernel at
≈1.97 GHz and needs ≈0.25 s of load to reach ≈2.38 GHz, and even 5 ms of idle
before the timed steps costs 8 %.  So the settle phase (--settle-s, default 1)
is one synchronised calibration block and then one batch of steps on the twin,
the cone copies and the W warm-up steps of the headline board enqueued back to
back; the hosts meet at the barrier while the GPU still runs them.  `clock` in
the line is the shader clock of the timed steps (a one-wave
s_memtime/s_memrealtime probe beside them).

For N>1 the driver launches this file under torch.distributed.run; ranks find
each other through torch.distributed (gloo, control plane only: barrier, max
of the timings, broadcast of the RCCL unique id); the halo rows go over the
library's own RCCL communicator.  Started as `python bench.py --gpus N`
without a launcher, it starts the N rank processes itself (same environment)
before anything touches the GPU.  `--single-process --gpus N` instead holds N
slabs in one process (peer copies; all on one device when only one is
visible: the config-5 rehearsal on one MI355X).
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

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's default: 4).  Streams beyond them share a
# queue in order, and a launch queued behind the clock probe's long-lived wave
# on a shared queue waits until the probe ends.  This run holds up to three
# contexts (one stream each; --single-process: two per slab) and the probe's
# stream.  Set before anything loads the HIP runtime.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

PROBE_MAX_MS = 5000.0   # the clock probe ends by itself after this (a timed window takes < 0.2 s)
HBM_PEAK = 8.0e12                   # B/s, MI355X spec (MI355X_MICROARCH.md)
VALU_PEAK = 256 * 4 * 32 * 2.4e9    # lane-ops/s: 256 CU × 4 SIMD × 32 lanes/clk (wave64 in 2 clk) × 2.4 GHz
# What the k=8 pair kernel's instruction mix can issue: full-rate
# issue measured at ≈63 T lane-op/s (three-VGPR v_bitop3, tools/valu_probe.hip,
# profiles/r02k_cross_probe.jsonl); on 4-word lane groups, per word-update 1
# of the 10.0 instructions (half a DPP lane move and half a v_alignbit) issues
# at half rate (profiles/r04f_k8_pmc_summary.json: 6.71e8 VALU per launch).
FULL_RATE_MEASURED = 63.0e12
PAIR_HALF_RATE_SHARE = 1.0 / 10.0

WORKLOADS = {
    # k = 16 (round 6): the chain of two pair waves per strip, 16 generations per HBM
    # pass — the k = 8 pair kernel's rate per clock at the clock half the HBM traffic
    # leaves the power-limited chip
    "bit131072": dict(layout="bit", rows=131072, cols=131072, bytes_per_cell=0.25, k=16),
    "byte32768": dict(layout="byte", rows=32768, cols=32768, bytes_per_cell=2.0, k=48),
}
# fused depths from which the bit-sliced kernels are issue-bound, not HBM-bound;
# the byte board streams 2 B/cell per launch and stays HBM-bound at every depth
# measured (k = 20, 24, 28 take the same 0.46-0.49 ms per launch at 32768²,
# profiles/r03o_bbring_ab.jsonl, profiles/r03o_byte_waits_pmc.json)
VALU_BOUND_FROM = {"bit": 5, "byte": 10 ** 9}
BYTEBIT_K = (4, 8, 12, 16, 20, 24, 28, 32, 48, 64)   # byte board: fused depths of the bit-sliced core
# the byte board's chain kernel (a workgroup of waves per strip splitting the k
# generations; k = 48 and 64 only): its name, and columns stored per strip
CHAIN_KERNEL = {48: ("bytebit_coop_kernel<1,12,4,4>", 1920), 64: ("bytebit_coop_kernel<1,16,4,3>", 1920)}


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
    p.add_argument("--chunk", type=int, default=None, help="GOL_OPT_CHUNK_ROWS override")
    p.add_argument("--interior-split", type=int, default=None, choices=(1, 2, 3, 4),
                   help="GOL_OPT_INTERIOR_SPLIT override (diagnostic: the k = 8 default is 2)")
    p.add_argument("--same-device", action="store_true",
                   help="diagnostic: N ranks on GPU 0 with real RCCL over its socket transport (one NCCL_HOSTID "
                        "per rank) — the N>1 path rehearsed on one GPU; the rate is not a scaling number")
    p.add_argument("--single-process", action="store_true",
                   help="N slabs in this process (peer copies) instead of one rank per GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-gens", type=int, default=1000, help="generations of the main.cpp baseline (config 2)")
    p.add_argument("--cpu-host-ranks", action="store_true",
                   help="also run the CPU baseline at P from the host's physical cores (ignores the cgroup quota)")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the short runs of the other BASELINE configs reported beside the metric")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--settle-s", type=float, default=1.0,
                   help="untimed seconds of steps before the warm-up (GPU clock ramp)")
    p.add_argument("--no-clock", action="store_true", help="no clock probe beside the timed steps")
    p.add_argument("--no-aged", action="store_true", help="skip the aged-board run beside the headline")
    p.add_argument("--no-config4", action="store_true",
                   help="skip the 1000-generation run of the seeded grid (config4_1000gen) beside the headline")
    p.add_argument("--launch-events", action="store_true",
                   help="an event pair around every timed launch (gol_kernel_time) instead of one pair around the "
                        "whole timed batch: the kernel's own duration, but ~8 µs of event packets between launches "
                        "(-0.8 %% GCUPS, profiles/r03k_timing.jsonl)")
    p.add_argument("--aged-board", action="store_true",
                   help="diagnostic (round 3's headline): run the settle phase on the headline board itself, so "
                        "the timed steps run on a board the settle phase has aged, not on the seeded grid")
    p.add_argument("--rank-timeout", type=float, default=900.0,
                   help="N>1 started without a launcher: seconds before every rank is stopped and the ranks "
                        "still running are named")
    p.add_argument("--idle-before-timed-ms", type=float, default=0.0,
                   help="diagnostic: leave the GPU idle this long between the warm-up and the timed steps "
                        "(shows the DVFS ramp; never used for the contract line)")
    p.add_argument("--no-halo-diag", action="store_true",
                   help="N>1: skip the halo diagnostic (comm-stream device time per step, and the same steps "
                        "with the exchange skipped: the interior-only step time and efficiency_vs_no_halo)")
    return p.parse_args()


# ---------------------------------------------------------------- verification

def life_cpu(board: np.ndarray, gens: int) -> np.ndarray:
    """Dead-boundary B3/S23 of a 0/1 board, bit-parallel on the host: rows of
    uint64 words, the 8 neighbour planes summed into a 4-bit counter by half
    adders, next = (n == 3) | (alive & n == 2) (main.cpp:79-90).  Independent of
    the device kernels' 9-sum circuit and of oracle/."""
    rows, cols = board.shape
    nw = (cols + 63) // 64
    pad = np.zeros((rows, nw * 64), np.uint8)
    pad[:, :cols] = board
    x = np.packbits(pad.reshape(rows, nw, 64)[:, :, ::-1], axis=2).view(">u8").reshape(rows, nw).astype(np.uint64)
    colmask = np.full(nw, ~np.uint64(0), np.uint64)
    if cols % 64:
        colmask[-1] = np.uint64((1 << (cols % 64)) - 1)
    one, s63 = np.uint64(1), np.uint64(63)

    def west(a):   # cell c sees column c-1 (bit b of word w = column 64w + b)
        r = a << one
        r[:, 1:] |= a[:, :-1] >> s63
        return r

    def east(a):
        r = a >> one
        r[:, :-1] |= a[:, 1:] << s63
        return r

    def north(a):  # cell r sees row r-1
        r = np.zeros_like(a)
        r[1:] = a[:-1]
        return r

    def south(a):
        r = np.zeros_like(a)
        r[:-1] = a[1:]
        return r

    for _ in range(gens):
        w, e = west(x), east(x)
        planes = [w, e, north(x), south(x), north(w), north(e), south(w), south(e)]
        c0 = np.zeros_like(x)
        c1 = np.zeros_like(x)
        c2 = np.zeros_like(x)
        for p in planes:   # ripple half adders: (c2 c1 c0) += p, saturating bit c2 = "4 or more"
            t0 = c0 & p
            c0 ^= p
            t1 = c1 & t0
            c1 ^= t0
            c2 |= t1
        x = (~c2 & c1 & (c0 | x)) & colmask   # n == 3, or n == 2 and alive
    bits = np.unpackbits(x.astype(">u8").view(np.uint8).reshape(rows, nw, 8), axis=2).reshape(rows, nw, 64)
    return bits[:, :, ::-1].reshape(rows, nw * 64)[:, :cols].astype(np.uint8)


class Verifier:
    """Light-cone check of one h×w window: the cone of the window (grown by the
    generations to come, clipped at the grid edge, which is dead) is copied
    from the device behind the steps enqueued so far — asynchronously, so the
    GPU never idles for it (gol_download_window_async; it lands at the next
    sync) — and after the run the window is compared with life_cpu."""

    def __init__(self, eng, rows, cols, r0, c0, gens, h=64, w=64, row_lo=0, row_hi=None):
        self.r0, self.c0, self.h, self.w, self.gens = r0, c0, h, w, gens
        row_hi = rows if row_hi is None else row_hi
        self.R0, self.C0 = max(row_lo, r0 - gens), max(0, c0 - gens)
        self.R1, self.C1 = min(row_hi, r0 + h + gens), min(cols, c0 + w + gens)
        take = getattr(eng, "download_window_async", None) or eng.download_window
        self.cone = take(self.R0, self.C0, self.R1 - self.R0, self.C1 - self.C0)
        self.got = None

    def grab(self, eng):
        """Copy the window now (behind the steps enqueued so far, asynchronously),
        so more steps (the clock batch) can follow before check()."""
        take = getattr(eng, "download_window_async", None) or eng.download_window
        self.got = take(self.r0, self.c0, self.h, self.w)

    def check(self, eng) -> dict:
        if self.got is not None:
            eng.sync()   # (an async grab lands at the engine's next sync)
        got = self.got if self.got is not None else eng.download_window(self.r0, self.c0, self.h, self.w)
        t = time.perf_counter()
        ref = life_cpu(self.cone, self.gens)[self.r0 - self.R0:self.r0 - self.R0 + self.h,
                                             self.c0 - self.C0:self.c0 - self.C0 + self.w]
        return {"window": [self.r0, self.c0, self.h, self.w], "generations": self.gens,
                "ok": bool((got == ref).all()), "live": int(got.sum()), "cpu_s": round(time.perf_counter() - t, 2)}


class MeshSeamVerifier:
    """Light-cone check across one of main.cpp's swapped column seams (mesh-
    compat m): block cy's left ghost column holds the LAST
    column of block cy+1 (main.cpp:51-54), so the last w/2 columns of block
    cy+1 followed by the first w/2 of block cy form a strip with plain
    adjacency inside it (dead beyond block cy+1's first and block cy's last
    column are more than `gens` away).  The cone is that strip grown by gens at
    both outer ends, taken as two logical column pieces; life_cpu steps the
    concatenation."""

    def __init__(self, eng, n, L, r0, cy, gens, h=64, w=64):
        self.r0, self.h, self.w, self.gens, self.n = r0, h, w, gens, n
        self.R0, self.R1 = max(0, r0 - gens), min(n, r0 + h + gens)
        hw = w // 2
        self.a0 = (cy + 2) * L - hw          # window piece A: last hw columns of block cy+1
        self.b0 = cy * L                     # window piece B: first hw columns of block cy
        self.A0 = max((cy + 1) * L, self.a0 - gens)
        self.B1 = min((cy + 1) * L, self.b0 + hw + gens)
        take = getattr(eng, "download_window_async", None) or eng.download_window
        nr = self.R1 - self.R0
        self.ca = take(self.R0, self.A0, nr, (cy + 2) * L - self.A0)
        self.cb = take(self.R0, self.b0, nr, self.B1 - self.b0)
        self.got = None

    def grab(self, eng):   # (as Verifier.grab)
        take = getattr(eng, "download_window_async", None) or eng.download_window
        hw = self.w // 2
        self.got = (take(self.r0, self.a0, self.h, hw), take(self.r0, self.b0, self.h, hw))

    def check(self, eng) -> dict:
        hw = self.w // 2
        if self.got is not None:
            eng.sync()
        parts = self.got or (eng.download_window(self.r0, self.a0, self.h, hw),
                             eng.download_window(self.r0, self.b0, self.h, hw))
        got = np.hstack(parts)
        t = time.perf_counter()
        cone = np.hstack([self.ca, self.cb])
        x0 = self.a0 - self.A0
        ref = life_cpu(cone, self.gens)[self.r0 - self.R0:self.r0 - self.R0 + self.h, x0:x0 + self.w]
        return {"window": [self.r0, [self.a0, self.b0], self.h, self.w], "generations": self.gens,
                "ok": bool((got == ref).all()), "live": int(got.sum()), "cpu_s": round(time.perf_counter() - t, 2)}


# ---------------------------------------------------------------- cpu baseline

def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def gpu_info() -> dict | None:
    """The first GPU agent as rocminfo reports it (name, compute units, max
    clock): the line's box, for comparing runs across the pool's boxes."""
    exe = shutil.which("rocminfo") or "/opt/rocm/bin/rocminfo"
    try:
        out = subprocess.run([exe], capture_output=True, text=True, timeout=30).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    info, cur = None, {}
    for ln in out.splitlines():
        ln = ln.strip()
        if ln.startswith("Agent ") and cur.get("gpu"):
            break
        if ln.startswith("Agent "):
            cur = {}
        key, _, val = ln.partition(":")
        key, val = key.strip(), val.strip()
        if key == "Name" and "name" not in cur:
            cur["name"] = val
        elif key == "Marketing Name":
            cur["marketing_name"] = val
        elif key == "Device Type":
            cur["gpu"] = val == "GPU"
        elif key == "Compute Unit":
            cur["compute_units"] = int(val) if val.isdigit() else val
        elif key.startswith("Max Clock Freq"):
            cur["max_clock_mhz"] = int(val.split()[0]) if val.split() and val.split()[0].isdigit() else val
    if cur.get("gpu"):
        info = {k: v for k, v in cur.items() if k != "gpu"}
    return info


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


def physical_cores() -> int:
    """Distinct (socket, core) pairs in /proc/cpuinfo: cores, not SMT threads."""
    pairs, phys = set(), None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("physical id"):
                phys = ln.split(":", 1)[1].strip()
            elif ln.startswith("core id"):
                pairs.add((phys, ln.split(":", 1)[1].strip()))
    except OSError:
        pass
    return len(pairs) or (os.cpu_count() or 1)


def mesh_ranks(cores: int, n: int = 16384) -> int:
    """Largest P = m² <= cores with m | n (main.cpp:194-200 accepts only those)."""
    return max(m * m for m in range(1, 1 + int(cores ** 0.5)) if n % m == 0)


def run_mpi_reference(P: int, gens: int, n: int = 16384) -> dict | None:
    """The unmodified reference main.cpp (oracle/_ref/gol_mpi, built from
    /root/reference by oracle/Makefile) under mpirun -np P, n², its own rank-0
    "nosetup" time (main.cpp:313)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "gol_mpi")
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    if not (os.path.exists(exe) and os.path.exists(mpirun)):
        return None
    tmp = tempfile.mkdtemp(prefix="golcpu")
    try:
        r = subprocess.run([mpirun, "-np", str(P), exe, str(n), str(n), "100000", str(gens), "tf"],
                           cwd=tmp, capture_output=True, text=True, timeout=900)
        row = open(os.path.join(tmp, "tf_compact.csv")).read().strip().splitlines()[-1].split(",")
        nosetup_us = float(row[6])   # "nosetup single" (rank 0), main.cpp:313,362
        if r.returncode != 0 or nosetup_us <= 0:
            return None
        return dict(value=n * n * gens / (nosetup_us * 1e-6) / 1e9, unit="GCUPS", cores=P, kind="reference",
                    sample=f"BASELINE config 2: main.cpp (reference, g++ -O2, MPICH) mpirun -np {P}, "
                           f"{n}x{n}, {gens} generations, rank-0 'nosetup' time (main.cpp:313)",
                    seconds=nosetup_us * 1e-6)
    except Exception as e:
        log(f"reference cpu baseline (P={P}) failed:", e)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_quota() -> float | None:
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max or
    v1 cfs quota), None when unlimited or unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_baseline(gens: int, host_ranks: bool = False) -> dict:
    """BASELINE config 2 on this host's cores: the reference
    main.cpp under mpirun, 16384², `gens` generations.  P = the largest square
    with √P | 16384 (main.cpp:194-200) that is <= the cores this process can
    actually run on at once: the physical cores (SMT threads not counted), the
    affinity set, the cgroup CPU quota and the per-GPU share of the box
    (OMP_NUM_THREADS there).  On the MI355X box the cgroup and the share allow
    16 of the 128 physical cores (2 × EPYC 9575F, 256 threads); P = 64 on 16
    CPUs of quota ran at half the speed of P = 16 (4.15 vs 8.30 GCUPS,
    profiles/r03b_bench_full.json), so the oversubscribed run is not the
    baseline.  --cpu-host-ranks adds the P of the physical cores as `host`
    beside it (for boxes without a quota).  Falls back to the oracle's
    bool**-layout restatement on one core."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    phys = physical_cores()
    quota = cpu_quota()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    usable = min(x for x in (phys, affinity, quota, share) if x)
    info = {"nproc": nproc, "affinity_threads": affinity, "physical_cores": phys, "cgroup_cpu_quota": quota,
            "cpu_share": share, "usable_cores": usable, "cpu_model": _cpu_model()}
    run = run_mpi_reference(mesh_ranks(max(1, int(usable))), gens)
    if run:
        out = dict(info, **run)
        P_host = mesh_ranks(max(1, min(phys, affinity)))
        if host_ranks and P_host != run["cores"]:
            out["host"] = run_mpi_reference(P_host, gens)
        return out
    from oracle import golcpu
    L, g = 4096, 20
    t = time.perf_counter()
    golcpu.ref_shaped_run(L, g, 1)
    dt = time.perf_counter() - t
    return dict(info, value=L * L * g / dt / 1e9, unit="GCUPS", cores=1, kind="port",
                sample=f"oracle restatement of main.cpp:79-103 (bool** layout), {L}x{L}, {g} generations, 1 thread",
                seconds=dt)


# ---------------------------------------------------------------- other configs

def timed_run(gh, eng, gens_total, k):
    """Wall time of `gens_total` generations after a sync and the device time
    per k-step from one event pair around the batch (gol_sync)."""
    eng.set_option(gh.OPT_KERNEL_TIMING, 0)
    eng.kernel_time(reset=True)   # synchronises
    t = time.perf_counter()
    eng.step(gens_total)
    dev_ms = eng.sync()
    dt = time.perf_counter() - t
    eng.kernel_time(reset=True)
    # per k-step (a split interior runs two concurrent half-launches per step)
    return dt, dev_ms / max(1, -(-gens_total // k)) * 1e-3


def clock_batch(eng, gens_total):
    """The shader clock of an identical batch run right after a timed one (the
    one-wave probe beside it), and that batch's wall time.  Timed batches run
    without the probe: its wave takes VGPRs on one SIMD of one CU, so that CU
    holds one 256-VGPR workgroup fewer, its XCD (workgroups are dealt round-robin
    over the 8 XCDs) gets one item more than it can start, and a one-round plan
    ends a round late — 1.5-2.3 % of the headline (profiles/r06w_probe_ab.jsonl),
    40 % of a one-workgroup-per-CU kernel (bytepair_chain_kernel)."""
    eng.kernel_time(reset=True)   # synchronises
    eng.clock_start(PROBE_MAX_MS)
    t = time.perf_counter()
    eng.step(gens_total)
    eng.sync()
    dt = time.perf_counter() - t
    mhz = eng.clock_stop()[0]
    eng.kernel_time(reset=True)
    return mhz, dt


SECONDARY = [  # name, layout, n, k, timed steps, algorithmic B/cell per launch, boundary, mesh m
    # the HBM-bound k = 1 kernels first.  bit k = 1 runs 0.686-0.693 of HBM on the
    # driver's lines and ≈0.700 in a process's later contexts (this build and round
    # 3's alike, profiles/r06an_k1_r03_ab.jsonl): the first 131072² boards a process
    # allocates stream 2 % slower, whichever build; measuring the secondaries before
    # the headline changes nothing (profiles/r06ab_order_ab.jsonl)
    ("bit131072_k1", "bit", 131072, 1, 300, 0.25, "dead", 1),
    ("byte32768_k1", "byte", 32768, 1, 100, 2.0, "dead", 1),
    ("bit131072_k8", "bit", 131072, 8, 40, 0.25, "dead", 1),
    ("byte32768_k48", "byte", 32768, 48, 21, 2.0, "dead", 1),
    ("byte32768_k32", "byte", 32768, 32, 31, 2.0, "dead", 1),
    ("byte16384_k1", "byte", 16384, 1, 200, 2.0, "dead", 1),
    ("mesh16384_m4_k1", "byte", 16384, 1, 200, 2.0, "mesh_compat", 4),
    ("mesh16384_m4_k28", "byte", 16384, 28, 36, 2.0, "mesh_compat", 4),
]


def secondary_configs(gh, headline: str, verify: bool = True, probe: bool = False) -> dict:
    """The other single-GPU configurations, measured briefly beside the
    headline (not part of `value`): the byte-per-cell board (config 3) at k=32
    (fused) and k=1 (one generation per pass, the literal config), the unfused
    k=1 bit sweep (the HBM-bound regime) and main.cpp's P=16 semantics (config
    2's rule with its swapped column halos, mesh-compat m=4) at 16384², k=1 and
    k=28.  Same timing rules: device-resident input, warm-up, wall time around
    synchronised steps; hbm_frac from the kernels' own hipEvent time.  Each run
    is verified: a 64×64 window (dead-boundary runs: across a strip seam of the
    bytebit / bit kernels; mesh runs: across the block edge at column 3·4096,
    where the swapped halos act) against life_cpu, from a cone copied behind
    the warm-up.  `sclk_mhz`: the clock of the timed batch (the same one-wave
    probe as the headline's), so a box effect can be told from a regression."""
    out = {}
    for name, layout, n, k, steps, bpc, boundary, m in SECONDARY:
        if name.startswith(headline) and k == WORKLOADS[headline]["k"]:
            continue
        try:
            with gh.Engine(n, n, layout=layout, tblock_k=k, boundary=boundary, mesh_m=m) as e:
                e.initialize_board("mesh" if m > 1 else "stream", 0 if m > 1 else 1)
                make = None
                if verify and m == 1:
                    # byte: strip seams at multiples of 1920 (k = 48, 64: the chain kernel) / 1984
                    # (k >= 20) / 3968 (k <= 16) columns
                    w = CHAIN_KERNEL[k][1] if k in CHAIN_KERNEL else (1984 if k >= 20 else 3968 // 2)
                    c0 = (5 * w - 32 if k >= 20 else 3968 * 2 - 32) if layout == "byte" else 7 * 62 * 64 - 30
                    make = lambda: Verifier(e, n, n, n // 2 + 13, c0, steps * k)
                elif verify:
                    make = lambda: MeshSeamVerifier(e, n, n // m, n // 2 + 5, 2, steps * k)
                if make:   # allocate the staging of the async cone copy up front (discarded)
                    warm = make()
                    e.sync()
                    del warm
                # warm-up as long as the timed run, then the cone behind it: the timed
                # steps start a host round trip after the warm-up (no idle gap, §5)
                e.step(max(steps, 3) * k)
                v = make() if make else None
                dt, per = timed_run(gh, e, steps * k, k)
                if v:
                    v.grab(e)
                mhz = clock_batch(e, steps * k)[0] if probe else None
                chk = v.check(e) if v else None
            out[name] = {"value": n * n * steps * k / dt / 1e9, "unit": "GCUPS", "generations": steps * k,
                         "gens_per_step": k, "layout": layout, "boundary": boundary, "cells": n * n,
                         "hbm_GBps_algorithmic": bpc * n * n / per / 1e9 if per > 0 else None,
                         "hbm_frac": bpc * n * n / per / HBM_PEAK if per > 0 else None,
                         "kernel_ms": per * 1e3, "kernel_ms_unit": "device time per k-step",
                         "sclk_mhz": round(mhz, 1) if mhz else None,
                         "verified": chk["ok"] if chk else None, "verify": chk}
        except Exception as ex:   # never let a side measurement break the contract line
            out[name] = {"error": repr(ex)}
    return out


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def best_copy_GBps():
    """Best STREAM-style copy measured on this GPU model (tools/hbm_probe.hip,
    committed under profiles/)."""
    best, src = None, None
    for name in ("r02l_hbm_probe_pitch.jsonl", "r02_hbm_probe.jsonl", "r01d_hbm_probe.jsonl"):
        path = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(path):
            continue
        for ln in open(path):
            try:
                rec = json.loads(ln)
            except ValueError:
                continue
            if "copy" in rec.get("probe", "") and rec.get("GBps") and rec["GBps"] > (best or 0.0):
                best, src = rec["GBps"], name
    return best, src


# ---------------------------------------------------------------- main

def spawn_ranks(n: int, argv: list[str], script: str | None = None, timeout: float | None = 900.0) -> int:
    """`bench.py --gpus N` started directly (no torch.distributed.run): start N
    rank processes of `script` (default: this file) with the launcher's
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free
    MASTER_PORT) and relay their output: rank 0's JSON line to stdout,
    everything else to stderr with a "[rank r] " prefix.  This process never
    touches the GPU (it imports no HIP code), so the ranks are plain children —
    no exec after a HIP call.  If one rank fails the others are stopped; if the
    deadline (`timeout` seconds, --rank-timeout) passes first, every rank is
    stopped and the ranks still running are named (a stuck RCCL group, a peer
    that died after ncclCommInitRank).  Returns the exit code: the first
    failing rank's, 124 at the deadline, else 0."""
    import socket
    import threading
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0")
    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv),
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r)), text=True,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE)
             for r in range(n)]
    lock = threading.Lock()

    def relay(r, f, is_out):   # rank 0's JSON line to stdout, anything else to stderr, prefixed
        for ln in f:
            with lock:
                if is_out and r == 0 and ln.lstrip().startswith("{"):
                    sys.stdout.write(ln)
                    sys.stdout.flush()
                else:
                    sys.stderr.write(f"[rank {r}] {ln}" if ln.endswith("\n") else f"[rank {r}] {ln}\n")
                    sys.stderr.flush()

    ths = [threading.Thread(target=relay, args=(r, f, f is p.stdout), daemon=True)
           for r, p in enumerate(procs) for f in (p.stdout, p.stderr)]
    for th in ths:
        th.start()
    t0, rc = time.monotonic(), 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0][1]
                log(f"[bench] rank {bad[0][0]} exited with status {rc}: stopping the other ranks")
                break
            if timeout and time.monotonic() - t0 > timeout:
                rc = 124
                alive = [r for r, p in enumerate(procs) if p.poll() is None]
                log(f"[bench] rank deadline of {timeout:g} s expired; still running: ranks {alive} "
                    f"(stopping them)")
                break
            time.sleep(0.2)
        else:
            bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode]
            if bad:
                rc = bad[0][1]
                log(f"[bench] rank {bad[0][0]} exited with status {rc}")
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for th in ths:
            th.join(timeout=30)
    return rc


class SeamCheck:
    """N>1: light-cone check of one h×w window straddling every slab seam
    (global row j·H, j = 1..N-1) — the rows the halo exchange feeds (the
    ghost-row exchange of main.cpp:58-61 inside the loop of main.cpp:291-305).
    The seam's cone is held by two ranks: each copies the cone rows it holds
    asynchronously before the warm-up (gol_download_window_async), and after
    the timed steps its rows of the final window; the pieces are gathered over
    the control-plane group (gloo) and rank j checks seam j with life_cpu.  A
    wrong halo at any step reaches the window, so `verified` cannot be true
    with garbage halos."""

    def __init__(self, eng, rank, world, rows_per, cols, c0, gens, h=64, w=64):
        self.rank, self.world, self.rows_per, self.gens, self.h, self.w = rank, world, rows_per, gens, h, w
        self.lo, self.hi, self.rows = rank * rows_per, (rank + 1) * rows_per, world * rows_per
        self.c0 = c0
        self.C0, self.C1 = max(0, c0 - gens), min(cols, c0 + w + gens)
        self.seams = [j * rows_per for j in range(1, world)]
        take = getattr(eng, "download_window_async", None) or eng.download_window
        self.cone = {}
        for s in self.seams:
            a, b = max(self.cone_rows(s)[0], self.lo), min(self.cone_rows(s)[1], self.hi)
            if a < b:
                self.cone[s] = (a, take(a, self.C0, b - a, self.C1 - self.C0))

    def cone_rows(self, s):
        return max(0, s - self.h // 2 - self.gens), min(self.rows, s + self.h // 2 + self.gens)

    def pieces(self, eng) -> dict:
        """After the run: this rank's cone rows and final window rows of every seam."""
        out = {}
        for s in self.seams:
            a, b = max(s - self.h // 2, self.lo), min(s + self.h // 2, self.hi)
            win = (a, eng.download_window(a, self.c0, b - a, self.w)) if a < b else None
            out[s] = (self.cone.get(s), win)
        return out

    def check(self, s, parts) -> dict:
        R0, R1 = self.cone_rows(s)
        r0 = s - self.h // 2
        cone = np.zeros((R1 - R0, self.C1 - self.C0), np.uint8)
        got = np.zeros((self.h, self.w), np.uint8)
        have_c = np.zeros(R1 - R0, bool)
        have_w = np.zeros(self.h, bool)
        for part in parts:
            c, wn = part.get(s, (None, None))
            if c is not None:
                cone[c[0] - R0:c[0] - R0 + len(c[1])] = c[1]
                have_c[c[0] - R0:c[0] - R0 + len(c[1])] = True
            if wn is not None:
                got[wn[0] - r0:wn[0] - r0 + len(wn[1])] = wn[1]
                have_w[wn[0] - r0:wn[0] - r0 + len(wn[1])] = True
        t = time.perf_counter()
        x0 = self.c0 - self.C0
        ref = life_cpu(cone, self.gens)[r0 - R0:r0 - R0 + self.h, x0:x0 + self.w]
        ok = bool(have_c.all() and have_w.all() and (got == ref).all())
        return {"seam": s, "ranks": [s // self.rows_per - 1, s // self.rows_per],
                "window": [r0, self.c0, self.h, self.w], "generations": self.gens, "ok": ok,
                "live": int(got.sum()), "cpu_s": round(time.perf_counter() - t, 2)}


def halo_diagnostic(eng, gh, steps, k, dist, world, rank, rounds=2):
    """Why an N>1 line runs at the efficiency it does, measured after the
    timed steps and their verification (so `value` is untouched): per rank, the
    comm stream's device time per k-step — the halo exchange (ncclSend/Recv,
    main.cpp:36-65's distr_borders) and the boundary + seam bands — from
    hipEvents on that stream (GOL_OPT_COMM_TIMING); and the same slabs stepped
    with the exchange skipped (GOL_OPT_HALO_EXCHANGE = 0: the bands and interior
    launches as before, no rows moved, results at the seams wrong — it comes
    last), interleaved with real steps, the best of `rounds` each: the
    interior-only step time.  exposed = step time − interior-only step time (what
    the exchange adds to a step), efficiency_vs_no_halo = their ratio."""
    import torch

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def window(halo: bool):
        eng.set_option(gh.OPT_HALO_EXCHANGE, 1 if halo else 0)
        eng.step(2 * k)   # (untimed: the clock after the host-side verification)
        eng.sync()
        if dist is not None:
            dist.barrier()
        t = time.perf_counter()
        eng.step(steps * k)
        eng.sync()
        if dist is not None:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t) / steps * 1e3

    with_halo, without = [], []
    ex = bd = 0.0
    n = 0
    for _ in range(rounds):
        eng.set_option(gh.OPT_COMM_TIMING, 1)   # (the real steps only)
        eng.comm_time(reset=True)
        with_halo.append(window(True))
        e1, b1, n1 = eng.comm_time(reset=True)
        ex, bd, n = ex + e1, bd + b1, n + n1
        eng.set_option(gh.OPT_COMM_TIMING, 0)
        without.append(window(False))
    eng.set_option(gh.OPT_HALO_EXCHANGE, 1)
    mine = {"rank": rank, "exchange_ms_per_step": ex / max(n, 1), "bands_ms_per_step": bd / max(n, 1),
            "steps_timed": n}
    per_rank = [mine]
    if dist is not None:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    step_ms, step0_ms = min(with_halo), min(without)
    exch = max(r["exchange_ms_per_step"] for r in per_rank)
    bands = max(r["bands_ms_per_step"] for r in per_rank)
    exposed = step_ms - step0_ms
    return {"step_ms": step_ms, "step_ms_no_halo": step0_ms, "exposed_ms_per_step": exposed,
            "efficiency_vs_no_halo": step0_ms / step_ms if step_ms > 0 else None,
            "exchange_ms_per_step": exch, "bands_ms_per_step": bands, "comm_ms_per_step": exch + bands,
            "comm_hidden_frac": (max(0.0, min(1.0, 1.0 - exposed / exch)) if exch > 0 else None),
            "windows_ms_per_step": {"with_halo": with_halo, "no_halo": without}, "per_rank": per_rank,
            "note": "after the timed steps: comm-stream device time per k-step from hipEvents (exchange = the "
                    "ncclSend/Recv group or peer copies; bands = boundary + seam band kernels), max over ranks; "
                    "the same slabs with the exchange skipped (GOL_OPT_HALO_EXCHANGE = 0, wrong seams, run "
                    "last) give the interior-only step; best of %d interleaved windows of %d k-steps each" % (
                        rounds, steps)}


def timed_window(eng, steps, k, launch_events, gh, gens=None):
    """Enqueue `steps` k-steps (or exactly `gens` generations) behind a sync,
    wall-time them, and return (seconds, device ms of the batch, launches)."""
    eng.set_option(gh.OPT_KERNEL_TIMING, 1 if launch_events else 0)
    eng.kernel_time(reset=True)
    t = time.perf_counter()
    eng.step(gens if gens is not None else steps * k)
    dev = eng.sync()
    t = time.perf_counter() - t
    ms, n = eng.kernel_time(reset=True)
    if not launch_events:
        ms = dev
    return t, ms, n


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and not args.single_process:
        # one process per GPU, as torch.distributed.run would start them
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], timeout=args.rank_timeout))
    rank = int(os.environ.get("RANK", "0"))
    try:
        run(args, world, rank)
    except Exception as ex:
        if world > 1:   # name the rank: the launcher interleaves every rank's stderr
            import traceback
            for ln in traceback.format_exc().splitlines():
                log(f"[rank {rank}] {ln}")
            log(f"[rank {rank}] fatal: {ex!r}")
            sys.exit(1)
        raise


def run(args, world, rank):
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device and world > 1:
        # rehearsal of the N>1 path on one GPU with REAL RCCL: every rank on device 0,
        # each under its own NCCL_HOSTID (RCCL refuses two ranks on one device of one
        # host), so the halos move over RCCL's socket transport on the loopback
        # interface (tests/rccl_real2_check.py); correctness, not speed
        local = 0
        os.environ.update(NCCL_HOSTID=f"golhip-bench-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                          NCCL_P2P_DISABLE="1", NCCL_SHM_DISABLE="1")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_amd import golhip as gh

    wl = dict(WORKLOADS[args.workload])
    rows_per = args.rows or wl["rows"]
    cols = args.cols or wl["cols"]
    k = args.tblock_k or wl["k"]
    steps = args.steps if args.steps is not None else max(1, round(1000 / k))
    n_total = world if world > 1 else args.gpus
    rows = rows_per * n_total
    single = world == 1 and not args.single_process

    def engine():
        """A context of the run's shape (rank mode: its own RCCL communicator)."""
        if world > 1:
            uid = [gh.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            e = gh.Engine(rows, cols, rank=rank, world=world, device=local, uid=uid[0], layout=wl["layout"],
                          tblock_k=k)
        else:
            e = gh.Engine(rows, cols, n_gpus=args.gpus if args.single_process else 1, layout=wl["layout"],
                          tblock_k=k)
        if args.interior_split:
            e.set_option(gh.OPT_INTERIOR_SPLIT, args.interior_split)
        if args.chunk:
            e.set_option(gh.OPT_CHUNK_ROWS, args.chunk)
        return e

    # The headline's board: the seeded grid of BASELINE config 4 (srand(1)
    # row-major, main.cpp:68-77), untouched until the warm-up — the timed steps
    # are generations W·k .. (W+K)·k of it.  The clock settles on a TWIN board
    # (same seed) first; right after the headline the twin, aged by the settle
    # phase, is timed the same way (`aged_board`), and a third board runs
    # config 4 in full: 1000 generations from generation 0 (`config4_1000gen`).
    eng = engine()
    t_init = time.perf_counter()
    eng.initialize_board("stream", 1)
    eng.sync()
    t_init = time.perf_counter() - t_init
    twin = None
    # The twin needs its own streams, and every stream wants a hardware queue of
    # its own (GPU_MAX_HW_QUEUES = 24 here): two 8-slab contexts in one process
    # (--single-process --gpus 8: 2 x 16 streams + the probe's) ran the headline
    # board at 92-107 k against 141-145 k without the twin
    # (profiles/r05g_sp8_bench.jsonl).  So a multi-slab context settles on its own
    # board when a twin's streams would not fit.
    # streams per slab: comm + comp, + one per further part under the split interior (the k = 8 default)
    # (a lone unsplit slab runs on one stream)
    n_split = eng.get_option(gh.OPT_INTERIOR_SPLIT)
    per_slab = 1 + n_split if n_split >= 2 else 2
    multi = args.single_process and args.gpus > 1
    streams = per_slab * (args.gpus if multi else 1) if (multi or world > 1 or n_split >= 2) else 1
    twin_fits = 2 * streams + 1 <= int(os.environ.get("GPU_MAX_HW_QUEUES", "24"))
    if not args.aged_board and twin_fits:
        twin = engine()
        twin.initialize_board("stream", 1)
        twin.sync()
    settler = twin or eng
    c4 = None
    if single and not args.no_config4 and args.workload == "bit131072" and not (args.rows or args.cols):
        c4 = engine()
        c4.initialize_board("stream", 1)
        c4.sync()

    # clock settle (untimed).  An MI355X that idled runs this kernel at
    # ≈1.97 GHz and needs ≈0.25 s of back-to-back load to reach ≈2.38 GHz;
    # 5 ms of idle before the timed steps already costs 8 %, 50 ms 14 %
    # (profiles/r03e_steps.jsonl, profiles/r03g_idle_gap.jsonl).  So: one
    # calibration block (25 steps, synchronised, clock-probed) on the twin,
    # then the rest of --settle-s on the twin, the verification cones of the
    # headline board (copied asynchronously) and its W warm-up steps are
    # enqueued back to back and the hosts meet at the barrier while the GPU
    # still runs them.  The k=8 schedule trial (gol_runtime.cpp) runs inside
    # the twin's settle steps without host waits; its pick is copied to the
    # headline board before the timed steps.  (Not under rocprofv3: its
    # tracing serialises dispatches, so the probe would hold the stencil
    # launches back until its own time limit.)
    profiled = any(key.startswith("ROCPROFILER_") for key in os.environ)
    probe_ok = hasattr(eng, "clock_start") and not args.no_clock and not profiled
    t_settle, settle_steps, first_block, tb = time.perf_counter(), 0, None, 0.0
    if args.settle_s > 0:
        if probe_ok:
            settler.clock_start(PROBE_MAX_MS)
        tb = time.perf_counter()
        settler.step(25 * k)
        settler.sync()
        tb = time.perf_counter() - tb
        if probe_ok:
            first_block = round(settler.clock_stop()[0])
        settle_steps = 25
    # verification windows (the cones are taken from the headline board just
    # before its warm-up): one light-cone window per rank (one slab, and rank
    # mode: mid-slab, across the split interior's seam band; several slabs in
    # one process: across the first slab seam) and, for N>1 ranks, one across
    # every slab seam (SeamCheck)
    gens_v = (args.warmup + steps) * k
    cone = seams = None
    if not args.no_verify:
        lo, hi = (rank * rows_per, (rank + 1) * rows_per) if world > 1 else (0, rows)
        if world > 1:
            r0 = lo + rows_per // 2 - 32
        elif n_total > 1:
            r0 = rows_per - 32
        else:
            r0 = rows // 2 - 32
        cone = dict(rows=rows, cols=cols, r0=r0, c0=cols // 3, gens=gens_v, row_lo=lo, row_hi=hi)
        seam_c0 = max(0, min(cols // 3 + 101, cols - 64))   # (its own columns: a 64-cell stretch of each seam)
        # the same copy once here, discarded: it allocates the library's staging
        # buffers (allocations can wait for the whole device) before the run-up
        warm = Verifier(eng, **cone)
        if world > 1:
            warm_s = SeamCheck(eng, rank, world, rows_per, cols, seam_c0, gens_v, w=min(64, cols))
        eng.sync()
        del warm
        if world > 1:
            del warm_s
    more = 0
    if args.settle_s > 0:
        more = max(0, int(round((args.settle_s - tb) / max(tb, 1e-6)))) * 25   # steps, from the calibration block
        if dist is not None:   # every rank takes the same steps (each one exchanges halos)
            import torch
            n = torch.tensor([more], dtype=torch.int64)
            dist.broadcast(n, src=0)
            more = int(n.item())
        settler.step(more * k)
        settle_steps += more
    if twin is not None and world > 1:
        # two RCCL communicators must not run at once (their kernels can block
        # each other): the twin's settle steps drain before the headline board moves
        twin.sync()
    verifier = Verifier(eng, **cone) if cone else None
    if cone and world > 1:
        seams = SeamCheck(eng, rank, world, rows_per, cols, seam_c0, gens_v, w=min(64, cols))
    eng.set_option(gh.OPT_KERNEL_TIMING, 1 if args.launch_events else 0)
    eng.step(args.warmup * k)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()   # the hosts meet while the GPUs still run the settle and warm-up steps
    if twin is not None:
        twin.sync()
    eng.sync()
    t_settle = time.perf_counter() - t_settle
    if twin is not None and args.chunk is None:   # the schedule the twin's trial kept
        policy = twin.get_option(gh.OPT_CHUNK_ROWS)
        eng.set_option(gh.OPT_CHUNK_ROWS, policy)
        if c4 is not None:
            c4.set_option(gh.OPT_CHUNK_ROWS, policy)
    eng.kernel_time(reset=True)   # (already synchronised) the warm-up launches are not counted
    if args.idle_before_timed_ms > 0:
        time.sleep(args.idle_before_timed_ms * 1e-3)
    probe = probe_ok
    t0 = time.perf_counter()
    eng.step(steps * k)
    dev_ms = eng.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms, launches = eng.kernel_time(reset=True)
    if not args.launch_events:   # one event pair around the whole timed batch (gol_sync): launches + gaps
        kernel_ms = dev_ms
    live = eng.popcount()
    if verifier:
        verifier.grab(eng)
    my_pieces = seams.pieces(eng) if seams is not None else None
    clock = None
    if probe:   # the clock: the same K steps again on the headline board, the probe beside them
        mhz, t_probe = clock_batch(eng, steps * k)
        if dist is not None:
            import torch
            t = torch.tensor([t_probe], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_probe = float(t.item())
        clock = {"sclk_mhz": round(mhz, 1), "first_settle_block_mhz": first_block,
                 "probe_batch_ms_per_step": round(t_probe * 1e3 / steps, 4),
                 "source": "in-kernel s_memtime / s_memrealtime (100 MHz) of a one-wave probe (gol_clock_start/"
                           "stop) beside the same K steps run again on the headline board right after the "
                           "timed ones; the timed steps run without it: its wave takes VGPRs on one SIMD, so "
                           "its CU holds one workgroup fewer and a one-round plan ends a round late on that "
                           "XCD (1.5-2.3 % of the headline, profiles/r06w_probe_ab.jsonl)"}
    aged_line = c4_line = None
    if single and twin is not None and not args.no_aged:   # enqueued within a host round trip of the headline's end
        ta, ams, an = timed_window(twin, steps, k, args.launch_events, gh)
        amhz = clock_batch(twin, steps * k)[0] if probe else None
        aged_line = {"value": rows * cols * steps * k / ta / 1e9, "unit": "GCUPS",
                     "generations": [(settle_steps + args.warmup) * k, (settle_steps + args.warmup + steps) * k],
                     "kernel_avg_ms": ams / max(an, 1), "sclk_mhz": round(amhz, 1) if amhz else None,
                     "live_cells": twin.popcount(),
                     "note": "the same K timed steps on the twin board the settle phase aged (the headline "
                             "before round 4), run right after the headline; a young random soup switches more "
                             "bits per instruction, so under this load the chip clocks lower on the seeded grid"}
    if c4 is not None:
        # exactly 1000 generations: whole k-steps and, for k = 16, a last 8-deep one
        c4_gens = 1000
        c4_steps = -(-c4_gens // k)
        vc4 = Verifier(c4, rows, cols, rows // 8 * 5 - 32, cols // 5, c4_gens) if not args.no_verify else None
        tc, cms, cn = timed_window(c4, c4_steps, k, args.launch_events, gh, gens=c4_gens)
        if vc4:
            vc4.grab(c4)
        cmhz = clock_batch(c4, c4_steps * k)[0] if probe else None
        chk = vc4.check(c4) if vc4 else None
        c4_line = {"value": rows * cols * c4_gens / tc / 1e9, "unit": "GCUPS",
                   "generations": [0, c4_gens], "steps": c4_steps, "ms_per_step": tc * 1e3 / c4_steps,
                   "kernel_avg_ms": cms / max(cn, 1), "sclk_mhz": round(cmhz, 1) if cmhz else None,
                   "live_cells": c4.popcount(), "verified": chk["ok"] if chk else None, "verify": chk,
                   "note": "BASELINE config 4 in full: 1000 generations of the seeded 131072x131072 grid from "
                           "generation 0, timed right after the headline (GPU hot, inputs resident)"}
        c4.close()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    verify = [verifier.check(eng)] if verifier else []
    if seams is not None:
        parts = [None] * world
        dist.all_gather_object(parts, my_pieces)
        mine = [seams.check(s, parts) for s in seams.seams if s == rank * rows_per]
        allv = [None] * world
        dist.all_gather_object(allv, verify + mine)
        verify = [v for vs in allv for v in vs]
    if dist is not None:
        import torch
        t = torch.tensor([live], dtype=torch.int64)
        dist.all_reduce(t)
        live = int(t[0].item())
    all_ok = all(v["ok"] for v in verify) if verify else None
    chunk_policy = eng.get_option(gh.OPT_CHUNK_ROWS)
    # N > 1 (ranks, or several slabs in one process): the halo diagnostic, after
    # verification (its no-exchange steps leave the seams wrong)
    halo = None
    if (world > 1 or (args.single_process and args.gpus > 1)) and not args.no_halo_diag:
        halo = halo_diagnostic(eng, gh, steps, k, dist, world, rank)

    gen_timed = steps * k
    cells = rows * cols
    value = cells * gen_timed / elapsed / 1e9
    if clock and clock.get("sclk_mhz"):
        # boxes of the pool run this load at 1.9-2.4 GHz (power-limited on a young board):
        # the rate per GPU and GHz compares builds across boxes
        clock["gcups_per_gpu_per_ghz"] = round(value / n_total / (clock["sclk_mhz"] / 1e3), 1)

    # roofline of the dominant kernel (the pipelined stencil), per launch:
    # algorithmic bytes = one read + one write of the local grid = bytes_per_cell × cells
    local_rows = rows_per if world > 1 else rows
    if world > 1 or (args.single_process and args.gpus > 1):
        local_rows = max(1, rows_per - 2 * k)   # timed launches are the interior ones, one per slab
    launch_bytes = wl["bytes_per_cell"] * local_rows * cols
    avg_launch_s = (kernel_ms / max(launches, 1)) * 1e-3
    shared = world == 1 and args.single_process and args.gpus > 1
    if shared:
        # several slabs per device run their launches concurrently, so one
        # launch's events span the others' work too: the roofline takes the
        # step time and the bytes of every slab's launch instead
        launch_bytes = wl["bytes_per_cell"] * rows * cols
        avg_launch_s = elapsed / steps
    # the split interior (GOL_OPT_INTERIOR_SPLIT = 2, the k = 8 default): each
    # step is two concurrent half-launches + a seam band, so the roofline's
    # unit is the step (all of the slab's bytes over the time per step) and
    # the PMC record is the per-step one (tools/make_traffic.py --per-step 3)
    n_parts = round(launches / max(steps, 1))
    split = (not shared and eng.get_option(gh.OPT_INTERIOR_SPLIT) >= 2 and n_parts >= 2)
    if split:
        avg_launch_s = (elapsed if args.launch_events else dev_ms * 1e-3) / steps
        local_rows = rows_per   # (a rank's step: its boundary bands and seam band included)
        launch_bytes = wl["bytes_per_cell"] * local_rows * cols
    achieved = launch_bytes / avg_launch_s if avg_launch_s > 0 else 0.0
    tr_key = f"{args.workload}_k{k}" + (("_split" if n_parts == 2 else f"_split{n_parts}") if split else "")
    traffic_json = load_json(os.path.join(ROOT, "profiles", "traffic.json")) or {}
    tr_rec = traffic_json.get(tr_key) if not (args.chunk or args.rows or args.cols) else None
    traffic = tr_rec.get("hbm_bytes_per_launch") if tr_rec else None
    if traffic:
        traffic *= (rows if shared else local_rows) / rows_per
    copy_peak, copy_src = best_copy_GBps()
    hbm = {"achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
           "traffic_GBps": traffic / avg_launch_s / 1e9 if (traffic and avg_launch_s > 0) else None,
           "copy_calibration_GBps": copy_peak, "copy_calibration_source": copy_src,
           "frac_of_copy": (achieved / 1e9 / copy_peak) if copy_peak else None,
           "bytes_per_launch": launch_bytes,
           "note": f"algorithmic bytes {wl['bytes_per_cell']} B/cell per launch = "
                   f"{wl['bytes_per_cell'] / k:.4g} B per cell-update at k={k}"}
    valu = None
    if tr_rec and tr_rec.get("valu_insts_per_launch") and avg_launch_s > 0:
        insts = tr_rec["valu_insts_per_launch"] * (rows if shared else local_rows) / rows_per
        lane_ops = insts * 64 / avg_launch_s
        valu = {"achieved": lane_ops / 1e12, "peak": VALU_PEAK / 1e12, "unit": "Tlane-op/s",
                "frac": lane_ops / VALU_PEAK,
                "insts_per_launch": insts,
                "lane_insts_per_cell_update": insts * 64 / ((rows if shared else local_rows) * cols * k),
                "source": f"SQ_INSTS_VALU per launch from profiles/traffic.json[{tr_key}] "
                          f"({tr_rec.get('profile')}), time per launch measured here"}
        if wl["layout"] == "bit" and k in (8, 16, 32):   # the pair kernel's mix (its chains: the same stages)
            ceiling = FULL_RATE_MEASURED / (1.0 + PAIR_HALF_RATE_SHARE)
            valu["mix_ceiling"] = {"Tlane_op": ceiling / 1e12, "frac": lane_ops / ceiling,
                                   "basis": "measured full-rate issue (63 T lane-op/s) with 1 of 10.0 "
                                            "instructions per word-update at half rate (DESIGN.md §3)"}
        if clock and clock.get("sclk_mhz"):
            # the spec peak assumes 2.4 GHz; the timed steps ran at the probe's clock
            valu["frac_at_measured_clock"] = lane_ops / (VALU_PEAK * clock["sclk_mhz"] / 2400.0)
    valu_bound = k >= VALU_BOUND_FROM[wl["layout"]] and valu is not None
    kname = (CHAIN_KERNEL[k][0] if wl["layout"] == "byte" and k in CHAIN_KERNEL
             else f"bytebit_pipe_kernel<{1 if k >= 20 else 2},{k}>" if wl["layout"] == "byte" and k in BYTEBIT_K
             else "bit_pair_kernel<8,1,4,4>" if wl["layout"] == "bit" and k == 8
             else f"bit_chain_kernel<{k // 8}> ({k // 8} bit_pair_kernel<8,1,4,4> waves per strip)"
             if wl["layout"] == "bit" and k in (16, 32)
             else f"{wl['layout']}_pipe_kernel<k={k}>")
    if valu_bound:
        roofline = {"bound": "valu", "achieved": valu["achieved"], "peak": valu["peak"], "unit": valu["unit"],
                    "frac": valu["frac"], "traffic": traffic, "hbm": hbm, "valu": valu}
    else:
        roofline = {"bound": "hbm", "achieved": hbm["achieved"], "peak": hbm["peak"], "unit": "GB/s",
                    "frac": hbm["frac"], "traffic": traffic, "hbm": hbm, "valu": valu}
    roofline.update({"kernel": kname, "kernel_avg_ms": avg_launch_s * 1e3, "launches": launches,
                     "clock_mhz": clock["sclk_mhz"] if clock else None,
                     "interior_split": split,
                     "dispatches_per_step": (n_parts + n_parts - 1) if split else 1,
                     "timing": ("step time over all slabs' concurrent launches (several slabs per device)" if shared
                                else "hipEvents around the whole timed batch on the launch stream (gol_sync), per "
                                     "step: two concurrent half-launches + the seam band (split interior)" if split
                                else "hipEvents around the whole timed batch on the launch stream (gol_sync), "
                                     "over the launches: inter-launch gaps included" if not args.launch_events
                                else "hipEvents around every timed stencil launch on its own stream, inside the "
                                     "timed region (gol_kernel_time)")})

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
                   "rows": rows, "cols": cols, "generations": gen_timed, "gens_per_step": k,
                   "parallelism": f"row-slabs x{n_total}" + ((" (rccl halos, all ranks on GPU 0: --same-device "
                                                              "rehearsal)" if args.same_device else " (rccl halos)")
                                                             if world > 1 else
                                                             " (one process, peer copies)" if n_total > 1 else ""),
                   "chunk_policy": chunk_policy, "global_cells": cells,
                   "interior_split": eng.get_option(gh.OPT_INTERIOR_SPLIT)},
        "roofline": roofline,
        "verified": all_ok,
        "verify": verify,
        "board": ("the seeded grid (srand(1) row-major, main.cpp:68-77): the timed steps are its generations "
                  f"{args.warmup * k}..{(args.warmup + steps) * k}; the clock settled on a twin board"
                  if twin is not None else "aged by the settle phase (" + (
                      "--aged-board)" if args.aged_board else "a twin context's streams would exceed the "
                      "hardware queues)")),
        "clock": clock if clock else {"skipped": "under rocprofv3" if profiled else "--no-clock"},
        "aged_board": aged_line,
        "config4_1000gen": c4_line,
        "halo": halo,
        "device_ms": dev_ms,
        "settle": {"seconds": t_settle, "steps": settle_steps, "on_second_board": bool(twin)},
        "init_s": t_init,
        "live_cells": live,
    }
    eng.close()
    if twin:
        twin.close()
    if world == 1 and not args.single_process and not args.no_secondary:
        result["secondary"] = secondary_configs(gh, args.workload, probe=probe_ok)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args.cpu_gens, args.cpu_host_ranks)
        cb["serial"] = serial_baseline()
        result["cpu_baseline"] = cb
        result["speedup_vs_cpu"] = value / cb["value"] if cb["value"] else None
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        result["gpu"] = gpu_info()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
