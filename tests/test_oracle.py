"""The CPU oracle (oracle/golcpu.c) pinned against the reference's own outputs.

tests/golden/ was produced by oracle/gen_golden.py, which runs the reference's
initializeBoard / updateBoard / distr_borders (main.cpp, main_serial.cpp,
compiled from /root/reference) through oracle/ref_harness_*.cpp.  The SURVEY
§8c KATs were measured independently with the patched reference binaries.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from oracle import golcpu as g

MODE = {"serial_compat": g.SERIAL_COMPAT, "dead": g.DEAD, "mesh_compat": g.MESH_COMPAT}


def oracle_initial(case):
    n, m = case["n"], case["mesh_m"]
    if case["mode"] == "serial_compat":
        return g.init_serial(n)
    if m == 1:
        return g.init_dead(n, n, seed=0)   # srand(rank=0) ≡ srand(1)
    return g.init_mesh(n, m)


def golden_boards(d, case):
    n = case["n"]
    if "all" in case["files"]:
        blob = open(os.path.join(d, case["files"]["all"]), "rb").read()
        bpb = case["bytes_per_board"]
        return {gen: g.unpack(blob[i * bpb:(i + 1) * bpb], n, n) for i, gen in enumerate(case["all_gens"])}
    return {int(k): g.unpack(open(os.path.join(d, fn), "rb").read(), n, n) for k, fn in case["files"].items()}


# ----------------------------------------------------------------- glibc rand

@pytest.mark.parametrize("seed", [0, 1, 2, 7, 15, 1804289383, 0x7FFFFFFF, 0x80000001, 0xDEADBEEF])
def test_rand_restatement_matches_libc(seed):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    ref = [libc.rand() for _ in range(3000)]
    assert list(g.rand_seq(seed, 3000)) == ref


def test_rand_kats():
    # first rand() with no srand; srand(1804289383) stream; srand(0) ≡ srand(1)
    assert g.rand_seq(1, 1)[0] == 1804289383
    assert list(g.rand_seq(1804289383, 5)) == [1362961854, 8891098, 392263175, 158428306, 2074436122]
    assert (g.rand_seq(0, 500) == g.rand_seq(1, 500)).all()


@pytest.mark.parametrize("offset", [1, 2, 30, 31, 32, 61, 997, 123457])
def test_stream_jump_matches_sequential(offset):
    seq = g.stream_cells(3, 0, offset + 700)
    assert (g.stream_cells(3, offset, 700) == seq[offset:]).all()


def test_stream_density():
    cells = g.stream_cells(1, 0, 300000)
    assert abs(cells.mean() - 1 / 3) < 0.01


# ------------------------------------------------------------ SURVEY KATs

KATS = {  # (mode, n, m): {gen: (popcount, sha256 prefix)}   SURVEY.md §8c
    ("serial", 1024, 1): {0: (348344, "55d025a34cdc034e"), 1: (379967, "09534f3e2c1d9380"),
                          10: (235314, "394bb8fc9db2b662"), 50: (129687, "704fd7cf284fdd56"),
                          100: (99504, "e54b6e7e66b7bb68")},
    ("dead", 1024, 1): {0: (349495, "24a885e604b27592"), 50: (129314, "af2c6fb65e13872b"),
                        100: (100059, "68da06c4255f013e")},
    ("mesh", 1024, 2): {0: (349038, "bb10c0e6078deac7"), 50: (131291, "44582f9b72853f63"),
                        100: (101697, "e60094abd5561959")},
    ("mesh", 1024, 4): {0: (349661, "c7c6b7349b637b5a"), 50: (130275, "57b4a9e14a893cd3"),
                        100: (99370, "5280eb572fdfd0a7")},
}


@pytest.mark.parametrize("key", list(KATS))
def test_survey_kats(key):
    kind, n, m = key
    if kind == "serial":
        b, mode = g.init_serial(n), g.SERIAL_COMPAT
    elif kind == "dead":
        b, mode = g.init_dead(n, n, seed=0), g.DEAD
    else:
        b, mode = g.init_mesh(n, m), g.MESH_COMPAT
    done = 0
    for gen, (pop, sha) in sorted(KATS[key].items()):
        b = g.run(b, gen - done, mode, m)
        done = gen
        assert int(b.sum()) == pop
        assert hashlib.sha256(g.packbits(b)).hexdigest()[:16] == sha


# ------------------------------------------------------------ golden fixtures

def test_manifest_covers_survey_cases(golden):
    _, cases = golden
    for name in ["serial_n1024", "mpi_P1_n48", "mpi_P4_n48", "mpi_P9_n48", "mpi_P16_n48",
                 "mpi_P1_n1024", "mpi_P4_n1024", "mpi_P16_n1024", "mpi_P4_n8", "mpi_P4_n10"]:
        assert name in cases


def _case_names():
    import json
    d = os.path.join(os.path.dirname(__file__), "golden")
    return [c["name"] for c in json.load(open(os.path.join(d, "manifest.json")))["cases"]]


@pytest.mark.parametrize("name", _case_names())
def test_oracle_matches_reference_fixture(golden, name):
    d, cases = golden
    case = cases[name]
    boards = golden_boards(d, case)
    mode, m = MODE[case["mode"]], case["mesh_m"]
    b = oracle_initial(case)
    done = 0
    for gen in sorted(int(x) for x in case["gens"]):
        b = g.run(b, gen - done, mode, m)
        done = gen
        ent = case["gens"][str(gen)]
        assert int(b.sum()) == ent["popcount"], (name, gen)
        assert g.digest(b) == ent["sha256"], (name, gen)
        if gen in boards:
            assert (b == boards[gen]).all()


FULL_SIZE = [t for t in ("config2", "config3")
             if os.path.exists(os.path.join(os.path.dirname(__file__), "golden", f"{t}.json"))]


@pytest.mark.parametrize("tag", FULL_SIZE)
def test_full_size_generation0_matches_reference(tag):
    """tests/golden/config2.json / config3.json hold BASELINE configs 2 and 3 run
    in full through main.cpp's own functions (oracle/gen_golden.py --config2 /
    --config3; the GPU tests compare whole boards against them): the oracle's
    generation-0 board at that size hashes to the reference's."""
    import json
    path = os.path.join(os.path.dirname(__file__), "golden", f"{tag}.json")
    case = json.load(open(path))
    b = oracle_initial(case)
    assert b.shape == (case["n"], case["n"])
    assert int(b.sum()) == case["gens"]["0"]["popcount"]
    assert g.digest(b) == case["gens"]["0"]["sha256"]


def test_ref_shaped_restatement_matches_dead_oracle():
    # the bool**-layout port used as the fallback CPU baseline computes the same board
    L, gens = 64, 12
    live = g.ref_shaped_run(L, gens, 1)
    assert live == int(g.run(g.init_dead(L, L, 1), gens, g.DEAD).sum())


@pytest.mark.parametrize("shape", [(1, 1), (3, 70), (64, 64), (97, 130)])
def test_fast_dead_stepper_matches_oracle(shape):
    """run_dead_fast (the long light-cone windows' stepper) = run(..., DEAD)."""
    rng = np.random.default_rng(shape[0] + 7 * shape[1])
    b = (rng.random(shape) < 0.4).astype(np.uint8)
    for gens in (0, 1, 13):
        assert (g.run_dead_fast(b, gens) == g.run(b, gens, g.DEAD)).all(), (shape, gens)
    # light cone: an interior window from its grown generation-0 region
    rows, cols, gens = 120, 150, 9
    full = g.init_dead(rows, cols, 1)
    want = g.run(full, gens, g.DEAD)
    for r0, c0 in ((0, 0), (40, 50), (100, 120)):
        assert (g.lightcone(rows, cols, gens, r0, c0, 20, 30) == want[r0:r0 + 20, c0:c0 + 30]).all()


@pytest.mark.parametrize("n,m", [(48, 3), (60, 5), (64, 2), (100, 4), (30, 30)])
def test_fast_mesh_stepper_matches_oracle(n, m):
    """run_mesh_fast (per-block ghost columns, main.cpp's swapped halos) =
    run(..., MESH_COMPAT) (the global wiring of SURVEY Appendix A)."""
    rng = np.random.default_rng(n * m)
    b = (rng.random((n, n)) < 0.4).astype(np.uint8)
    for gens in (1, 9):
        assert (g.run_mesh_fast(b, gens, m) == g.run(b, gens, g.MESH_COMPAT, m)).all(), (n, m, gens)


def test_text_body_format():
    assert g.text_body(np.array([[0, 1], [1, 0]], np.uint8)) == b"0\t1\t\n1\t0\t\n"
