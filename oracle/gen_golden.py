"""Generate tests/golden/ from the reference itself — TEST INFRASTRUCTURE ONLY.

Runs in the build container only (needs /root/reference and MPICH in /opt/conda):

    make -C oracle ref && python oracle/gen_golden.py
    python oracle/gen_golden.py --config2     # BASELINE config 2 in full (≈5 min on 8 CPUs)
    python oracle/gen_golden.py --config3     # config 3's board through main.cpp, P = 1 (≈2.5 h, 1 CPU)

The harnesses (oracle/ref_harness_{serial,mpi}.cpp) drive the reference's own
initializeBoard / updateBoard / distr_borders, compiled from /root/reference.
Every fixture is data: packed boards (np.packbits, MSB-first, row-major) and a
manifest of popcounts + sha256 per generation.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
REF = os.path.join(HERE, "_ref")
MPIRUN = "/opt/conda/bin/mpirun"


def _stats(path: str, n: int):
    d = open(path, "rb").read()
    bits = np.unpackbits(np.frombuffer(d, np.uint8))[: n * n]
    return d, int(bits.sum()), hashlib.sha256(d).hexdigest()


def run_case(name, kind, n, procs, gens, every, keep_files, tmp):
    prefix = os.path.join(tmp, name)
    if kind == "serial":
        cmd = [os.path.join(REF, "ref_harness_serial"), str(n), str(gens), str(every), prefix]
    else:
        cmd = [MPIRUN, "-np", str(procs), os.path.join(REF, "ref_harness_mpi"),
               str(n), str(gens), str(every), prefix]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
    m = int(round(procs ** 0.5))
    entry = {
        "name": name, "source": kind, "n": n, "procs": procs,
        "mode": "serial_compat" if kind == "serial" else ("dead" if m == 1 else "mesh_compat"),
        "mesh_m": m, "gens": {}, "files": {},
    }
    dumped = [0] + [g for g in range(1, gens + 1) if g % every == 0]
    blob = []
    for g in dumped:
        d, pop, sha = _stats(f"{prefix}_g{g}.bin", n)
        entry["gens"][str(g)] = {"popcount": pop, "sha256": sha}
        if keep_files == "all":
            blob.append(d)
        elif g in keep_files:
            fn = f"{name}_g{g}.bin"
            open(os.path.join(OUT, fn), "wb").write(d)
            entry["files"][str(g)] = fn
    if keep_files == "all":
        fn = f"{name}_all.bin"
        open(os.path.join(OUT, fn), "wb").write(b"".join(blob))
        entry["files"]["all"] = fn
        entry["all_gens"] = dumped
        entry["bytes_per_board"] = len(blob[0])
    return entry


def full_size(tag, name, n, procs):
    """A BASELINE configuration in full through main.cpp's own functions, 1000
    generations; digests only (the boards are 32-128 MiB packed):
    tests/golden/<tag>.json, generations 0, 500, 1000."""
    tmp = tempfile.mkdtemp(prefix="gol" + tag)
    try:
        entry = run_case(name, "mpi", n, procs, 1000, 500, [], tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    entry["generator"] = (f"oracle/gen_golden.py --{tag} (main.cpp via oracle/ref_harness_mpi.cpp, "
                          f"mpirun -np {procs})")
    with open(os.path.join(OUT, f"{tag}.json"), "w") as f:
        json.dump(entry, f, indent=1)
    print("wrote", os.path.join(OUT, f"{tag}.json"))


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("gen_golden.py runs only where /root/reference exists")
    subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)
    os.makedirs(OUT, exist_ok=True)
    if "--config2" in sys.argv[1:]:   # config 2 exactly: a 4×4 mesh (mesh-compat), 16384²
        return full_size("config2", "mpi_P16_n16384", 16384, 16)
    if "--config3" in sys.argv[1:]:   # config 3's 32768² board on one rank (dead boundary, srand(0))
        return full_size("config3", "mpi_P1_n32768", 32768, 1)
    tmp = tempfile.mkdtemp(prefix="golgold")
    cases = []
    try:
        # config 1: main_serial.cpp 1024², 100 generations (serial-compat)
        cases.append(run_case("serial_n1024", "serial", 1024, 1, 100, 1, [0, 1, 100], tmp))
        cases.append(run_case("serial_n48", "serial", 48, 1, 30, 1, "all", tmp))
        cases.append(run_case("serial_n37", "serial", 37, 1, 30, 1, "all", tmp))
        # main.cpp on P = 1, 4, 9, 16 ranks (dead / mesh-compat m=2,3,4)
        for P in (1, 4, 9, 16):
            cases.append(run_case(f"mpi_P{P}_n48", "mpi", 48, P, 30, 1, "all", tmp))
        for P in (1, 4, 16):
            cases.append(run_case(f"mpi_P{P}_n1024", "mpi", 1024, P, 100, 5, [0, 100], tmp))
        # run.sh:4-5 smoke sizes, 50 generations on 4 ranks
        for n in (8, 10):
            cases.append(run_case(f"mpi_P4_n{n}", "mpi", n, 4, 50, 1, "all", tmp))
        # a 1-rank 96² (dead) run long enough for gliders to hit the edges
        cases.append(run_case("mpi_P1_n96", "mpi", 96, 1, 200, 1, "all", tmp))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    manifest = {
        "format": "np.packbits(board, MSB-first, row-major); *_all.bin = boards of all_gens concatenated",
        "generator": "oracle/gen_golden.py (reference functions via oracle/ref_harness_*.cpp)",
        "cases": cases,
    }
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
