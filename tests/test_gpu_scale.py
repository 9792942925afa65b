"""Full-size parity at the BASELINE configurations (GPU).

* config 4 at full length: 131072², one slab, k=8, the default schedule (the
  split interior: two half-launches per k-step, one round of equal chunks each
  = policy -1, plus the seam band), 1000 generations;
* config 5 rehearsed on ONE MI355X: the 8-GPU weak-scaling grid
  (8 × 131072 rows × 131072 = 1,048,576 × 131,072 cells, 32 GiB of ping-pong
  buffers) as 8 row slabs in one process (PEER transport: the slab/halo code
  path of the RCCL transport with hipMemcpyAsync in place of ncclSend/Recv);
  the same grid as 8 rank contexts (the RCCL transport itself) is
  tests/rccl_shim_check.py --config5.

The board is the srand(1) row-major glibc stream generated on the device;
light-cone windows (tests: oracle/golcpu.py lightcone) check corners, slab
seams, XCD row-band seams, strip seams and rows past 2^19 against the oracle.
"""
import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu

WORKERS = min(12, os.cpu_count() or 4)


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def check_windows(e, rows, cols, gens, wins, h=64, w=64):
    got = {rc: e.download_window(rc[0], rc[1], h, w) for rc in wins}
    with ThreadPoolExecutor(WORKERS) as ex:   # the oracle releases the GIL
        want = dict(zip(wins, ex.map(lambda rc: g.lightcone(rows, cols, gens, rc[0], rc[1], h, w), wins)))
    bad = [(rc, int((got[rc] != want[rc]).sum())) for rc in wins if (got[rc] != want[rc]).any()]
    assert not bad, bad
    return sum(int(v.sum()) for v in got.values())


@pytest.mark.timeout(420)
def test_headline_k16_config_full_length(gh):
    """BASELINE config 4 as bench.py runs it since round 6: one slab, k = 16
    (bit_chain_kernel<2>: two pair waves per strip, rows handed through LDS),
    the default schedule (split interior, one round per half), exactly 1000
    generations (62 k-steps of 16 and a last 8-deep one through the pair
    kernel); light-cone windows at the corners, XCD band seams, strip seams and
    the split's seam band."""
    n, gens = 131072, 1000
    with gh.Engine(n, n, layout="bit", tblock_k=16) as e:
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == 2
        e.initialize_board("stream", 1)
        e.step(gens)
        e.sync()
        seam = lambda s: 128 * (62 * s + 1)
        wins = [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64), (16384 - 32, 777), (65536 - 31, 70000),
                (n // 2 - 16 - 40, seam(7) - 20), (40000, seam(1) - 32), (98765, seam(5) - 10), (12345, seam(16) - 40)]
        check_windows(e, n, n, gens, wins)


@pytest.mark.timeout(420)
def test_headline_config_full_length(gh):
    """BASELINE config 4 exactly as bench.py runs it: one slab, k=8, the
    default schedule (split interior, policy -1 per half-launch, the schedule
    trial on), 1000 generations (125 k-steps = 375 dispatches)."""
    n, k, gens = 131072, 8, 1000
    with gh.Engine(n, n, layout="bit", tblock_k=k) as e:
        e.initialize_board("stream", 1)
        e.step(gens)
        e.sync()
        # k=8 runs on 4-word (128-column) lane groups: interior wave strips store
        # 62 lanes, strip s starts at column 128·(62s + 1)
        seam = lambda s: 128 * (62 * s + 1)
        wins = [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64),          # corners (dead edges)
                (16384 - 32, 777), (65536 - 31, 70000), (114688 - 33, n - 69),  # XCD row-band seams
                (40000, seam(1) - 32), (98765, seam(5) - 10),                  # strip seams
                (12345, seam(16) - 40), (77777, seam(9) - 33), (n // 2, n // 2),
                (3 * 16384 + 9000, seam(12) - 31),
                # the folded tail strip (units 931-960, both half-waves) and its seam
                # with the end-aligned last strip (unit 961); XCD band start inside it
                (50000, 128 * 961 - 32), (16384 - 30, 128 * 945), (90001, 128 * 931 + 1000)]
        live = check_windows(e, n, n, gens, wins)
        assert live > 0
        assert 0.02 * n * n < e.popcount() < 0.5 * n * n


@pytest.mark.timeout(420)
def test_config5_rehearsal_peer(gh):
    """The 8-GPU grid (config 5) as 8 slabs on this GPU: uneven k-steps
    (short blocks between full ones), windows at all 7 slab seams, the first
    and last rows and rows past 2^19."""
    H, cols, k = 131072, 131072, 8
    rows = 8 * H
    steps = [8, 3, 8, 8, 5, 8, 8]
    gens = sum(steps)
    with gh.Engine(rows, cols, n_gpus=8, layout="bit", tblock_k=k) as e:
        e.initialize_board("stream", 1)
        # generation 0 deep in the last slab (the jump-ahead of the init past 2^37 draws)
        w0 = e.download_window(rows - 5, 100003, 3, 300)
        assert (w0 == g.init_dead(3, 300, 1, row0=rows - 5, full_cols=cols, col0=100003)).all()
        for st in steps:
            e.step(st)
        e.sync()
        wins = [(s * H - 32, (s * 9973) % (cols - 64)) for s in range(1, 8)]   # every seam
        wins += [(0, 5), (rows - 64, cols - 64), (600000, 4000), (1000000 - 7, 77777)]
        check_windows(e, rows, cols, gens, wins)


@pytest.mark.timeout(420)
@pytest.mark.parametrize("k,gens", [(32, 1024), (28, 1008)])
def test_config3_bench_shape_full_length(gh, k, gens):
    """BASELINE config 3 exactly as bench.py's byte32768 workload runs it:
    32768² byte board, ONE slab, the default chunk policy (one round of equal
    chunks: ≈274-row chunks at 2 waves/SIMD), ≈1000 generations.  k = 32 (the
    default: two window slots per stage, a 6-phase trip) and k = 28 (three
    slots).  Windows straddle chunk seams (multiples of ≈274 rows), strip seams
    (multiples of 1984 columns) and the corners."""
    n = 32768
    with gh.Engine(n, n, layout="byte", tblock_k=k) as e:
        assert e.get_option(gh.OPT_CHUNK_ROWS) == -1
        e.initialize_board("stream", 1)
        e.step(gens)
        e.sync()
        wins = [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64),             # corners (dead edges)
                (274 - 32, 1984 - 32), (274 * 60 - 30, 1984 * 9 - 33),           # chunk x strip seams
                (274 * 119 - 34, 1984 * 16 - 31), (16384 - 32, n - 1984 - 32),   # last strip seam
                (n // 2 + 7, 3 * 1984 + 700),
                (274 * 3 - 31, 1984 * 2 - 32), (5000, 1984 * 7 - 30), (274 * 31 - 33, 1984 * 15 - 32),
                (20000, 1984 * 16 + 500), (274 * 88 + 5, 32 * 946)]
        check_windows(e, n, n, gens, wins)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("policy", [-3, -6])
def test_headline_trial_candidates_full_size(gh, policy):
    """The k=8 schedule trial switches the 131072² headline among -104 (guided:
    the full-length test above), -6 and -3 (equal trip-aligned chunks) after
    step 400; each candidate is forced here at full size and checked at chunk
    seams, XCD band seams, strip seams of the 128-column lane groups and the
    corners."""
    n, k, gens = 131072, 8, 128
    with gh.Engine(n, n, layout="bit", tblock_k=k) as e:
        e.set_option(gh.OPT_CHUNK_ROWS, policy)
        e.initialize_board("stream", 1)
        e.step(gens)
        e.sync()
        # chunks: rows covered in `-policy` rounds of the resident waves over 16.5 strips
        # (the folded strip covers two chunk-rows), trip-aligned
        ch = {-3: 360, -6: 184}[policy]   # 2048 resident waves / 16.5 strips = 124 per round
        seam = lambda s: 128 * (62 * s + 1)
        wins = [(0, 0), (n - 64, n - 64), (ch - 32, seam(1) - 30), (ch * 57 - 30, 20000),
                (ch * 90 - 33, seam(8) - 31), (16384 - 32, 777), (5 * 16384 - 30, n - seam(1) - 40),
                (7 * 16384 + 8191, 65536), (ch * 37 + 5, seam(15) - 29),
                (ch * 64 - 31, 128 * 961 - 33), (ch * 25 - 33, 128 * 950)]   # folded strip
        check_windows(e, n, n, gens, wins)


def config2_golden():
    with open(os.path.join(os.path.dirname(__file__), "golden", "config2.json")) as f:
        return json.load(f)


def config3_golden():
    with open(os.path.join(os.path.dirname(__file__), "golden", "config3.json")) as f:
        return json.load(f)


def text_board(path, n):
    """A `.gol` part file ("first last" rows, a blank line, rows of "v\t") as
    (first row, cells)."""
    with open(path, "rb") as f:
        first, last = map(int, f.readline().split())
        f.readline()
        raw = np.frombuffer(f.read(), np.uint8)
    return first, raw.reshape(last - first + 1, 2 * n + 1)[:, 0:2 * n:2] - ord("0")


@pytest.mark.timeout(420)
@pytest.mark.parametrize("layout,k", [("bit", 16), ("bit", 8), ("bit", 1), ("byte", 48), ("byte", 32), ("byte", 1)])
def test_config2_reference_full_length(gh, layout, k):
    """BASELINE config 2 in full against the reference itself: main.cpp under
    mpirun -np 16 (a 4×4 mesh, the swapped column halos of main.cpp:36-65),
    16384², 1000 generations; sha256 of the whole board at generations 0, 500
    and 1000 (tests/golden/config2.json, made by oracle/gen_golden.py
    --config2 from the reference's own functions).  Every fused depth the
    bench runs, both layouts."""
    case = config2_golden()
    n, m = case["n"], case["mesh_m"]
    with gh.Engine(n, n, layout=layout, boundary="mesh_compat", mesh_m=m, tblock_k=k) as e:
        e.initialize_board("mesh", 0)
        done = 0
        for gen in sorted(int(x) for x in case["gens"]):
            e.step(gen - done)
            done = gen
            assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (layout, k, gen)


@pytest.mark.timeout(420)
def test_config2_driver_full_length(tmp_path):
    """The same run through the reference-CLI driver: bin/gol --procs 16 (the
    emulated 4×4 mesh) on 2 slabs at k = 16, the snapshot at generation 1000
    written as main.cpp's text parts; the parts' board hashes to the
    reference's digest."""
    case = config2_golden()
    n, gens = case["n"], 1000
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi_amd", "bin", "gol")
    subprocess.run([exe, "--procs", "16", "--gpus", "2", "-k", "16", "--save", str(n), str(n), str(gens), str(gens),
                    "t", "1"], cwd=tmp_path, check=True, capture_output=True, timeout=300)
    name = [f for f in os.listdir(tmp_path) if f.endswith(".gol") and "_" not in f][0][:-4]
    got = np.empty((n, n), np.uint8)
    for p in range(2):
        first, cells = text_board(tmp_path / f"{name}_{gens}_{p}.gol", n)
        got[first:first + cells.shape[0]] = cells
    assert g.digest(got) == case["gens"][str(gens)]["sha256"]


@pytest.mark.timeout(420)
@pytest.mark.parametrize("layout,k,core", [("byte", 48, None), ("byte", 32, None), ("byte", 1, None), ("byte", 64, None),
                                           ("byte", 48, 4), ("byte", 56, None), ("bit", 16, None), ("bit", 8, None)])
def test_config3_reference_full_length(gh, layout, k, core):
    """BASELINE config 3's board in full against the reference itself: main.cpp's
    own functions on one rank (dead boundary, srand(0) = srand(1), the 32768²
    board), 1000 generations; sha256 of the whole board at generations 0, 500
    and 1000 (tests/golden/config3.json, made by oracle/gen_golden.py
    --config3).  The byte board at the bench's depths and kernels (k = 48 the
    chain, 32 one wave per strip, 1, 64, the pair chain at 48 and 56), and the
    bit board's k = 16 / 8 kernels on the same cells."""
    case = config3_golden()
    n = case["n"]
    with gh.Engine(n, n, layout=layout, tblock_k=k) as e:
        if core is not None:
            e.set_option(gh.OPT_BYTE_CORE, core)
        e.initialize_board("stream", 1)
        done = 0
        for gen in sorted(int(x) for x in case["gens"]):
            e.step(gen - done)
            done = gen
            assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (layout, k, core, gen)
