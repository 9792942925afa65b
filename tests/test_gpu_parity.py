"""GPU parity: libgolhip.so (hand-written gfx950 kernels) vs the oracle / goldens.

Everything here runs through the C ABI (mpi_amd.golhip -> libgolhip.so) on
cuda:0 and compares bit-exactly with:
  * tests/golden/ (boards produced by the reference's own functions), and
  * oracle/golcpu.c (the CPU restatement pinned by those goldens),
over every boundary convention, both layouts, fused generations k = 1..8,
several row slabs on one GPU (the halo-exchange path), and odd shapes.
At BASELINE size (131072²) parity is checked through light-cone windows.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def engine(gh, rows, cols, **kw):
    return gh.Engine(rows, cols, **kw)


def rand_board(rng, rows, cols, p=0.35):
    return (rng.random((rows, cols)) < p).astype(np.uint8)


# ------------------------------------------------------------------ goldens

def golden_cases(golden, modes):
    d, cases = golden
    return [(d, c) for c in cases.values() if c["mode"] in modes]


def load_boards(d, case):
    from tests.test_oracle import golden_boards
    return golden_boards(d, case)


def check_case(gh, d, case, layout, k, slabs, overlap=1):
    n, m = case["n"], case["mesh_m"]
    mode = case["mode"]
    boundary = mode
    init = {"serial_compat": ("serial", g.SERIAL_SEED), "dead": ("stream", 0), "mesh_compat": ("mesh", 0)}[mode]
    with engine(gh, n, n, n_gpus=slabs, layout=layout, boundary=boundary, mesh_m=m, tblock_k=k) as e:
        e.set_option(gh.OPT_OVERLAP, overlap)
        if layout == "bit" and mode == "mesh_compat" and (n // m) % 32:
            e.upload(g.init_mesh(n, m))   # the bit layout's device init needs 32-column-aligned blocks
        else:
            e.initialize_board(*init)
        boards = load_boards(d, case)
        gens = sorted(int(x) for x in case["gens"])
        done = 0
        for gen in gens:
            e.step(gen - done)
            done = gen
            b = e.download()
            ent = case["gens"][str(gen)]
            assert g.digest(b) == ent["sha256"], (case["name"], layout, k, slabs, gen, int(b.sum()),
                                                   ent["popcount"])
            if gen in boards:
                assert (b == boards[gen]).all()
            assert e.popcount() == ent["popcount"]


@pytest.mark.parametrize("layout", ["bit", "byte"])
@pytest.mark.parametrize("k", [1, 3, 8])
@pytest.mark.parametrize("slabs", [1, 2, 3])
def test_serial_goldens(gh, golden, layout, k, slabs):
    for d, case in golden_cases(golden, {"serial_compat"}):
        if case["n"] < 3 * slabs * k and slabs > 1:
            continue
        check_case(gh, d, case, layout, k, slabs)


@pytest.mark.parametrize("layout", ["bit", "byte"])
@pytest.mark.parametrize("k", [1, 2, 5, 8])
@pytest.mark.parametrize("slabs", [1, 2, 4])
def test_dead_goldens(gh, golden, layout, k, slabs):
    for d, case in golden_cases(golden, {"dead"}):
        if case["n"] // slabs < k:
            continue
        check_case(gh, d, case, layout, k, slabs)


@pytest.mark.parametrize("layout", ["bit", "byte"])
@pytest.mark.parametrize("k", [1, 3, 8])
@pytest.mark.parametrize("slabs", [1, 2, 3])
def test_mesh_goldens(gh, golden, layout, k, slabs):
    """main.cpp on P = 4, 9, 16 ranks (swapped column halos) against the
    reference's own boards: any layout and fused depth (reversed column blocks)."""
    for d, case in golden_cases(golden, {"mesh_compat"}):
        if case["n"] // slabs < k:
            continue
        check_case(gh, d, case, layout, k, slabs)


def test_no_overlap_path(gh, golden):
    for d, case in golden_cases(golden, {"dead"}):
        if case["n"] >= 96:
            check_case(gh, d, case, "bit", 4, 3, overlap=0)


# ---------------------------------------------------------------- oracle, shapes

SHAPES = [(1, 1), (1, 77), (77, 1), (2, 2), (3, 130), (37, 1000), (1000, 37), (257, 4099), (64, 4096),
          (130, 8000), (513, 129)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_dead_random_shapes(gh, shape, layout):
    rows, cols = shape
    rng = np.random.default_rng(rows * 7919 + cols)
    b0 = rand_board(rng, rows, cols)
    for k in (1, 4, 7):
        for slabs in (1, 2):
            if rows // slabs < k:
                continue
            with engine(gh, rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
                e.upload(b0)
                assert (e.download() == b0).all()
                e.step(11)
                got = e.download()
            assert (got == g.run(b0, 11, g.DEAD)).all(), (shape, layout, k, slabs)


@pytest.mark.parametrize("chunk", [8, 37, 256, -1, -3, -104])
def test_bit_chunk_policies(gh, chunk):
    rng = np.random.default_rng(1000 + chunk)
    rows, cols = 300, 9000
    b0 = rand_board(rng, rows, cols)
    ref = g.run(b0, 24, g.DEAD)
    for k in (1, 2, 4, 5, 7, 8):
        with engine(gh, rows, cols, layout="bit", tblock_k=k) as e:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
            e.upload(b0)
            e.step(24)
            assert (e.download() == ref).all(), (chunk, k)


@pytest.mark.parametrize("slabs", [1, 2])
def test_k8_schedule_trial(gh, slabs):
    """The k=8 schedule trial (gol_runtime.cpp tune_slot): after 400 k-steps the
    candidate chunk policies take turns on 18 real steps and the fastest stays;
    results are unchanged throughout, and a caller-set policy is kept.  k = 8
    contexts start on the split interior (default policy -1, candidates
    -1/-2/-3) when its three streams per slab fit the hardware queues
    (3 x slabs per device + 1 <= GPU_MAX_HW_QUEUES, HIP's default 4: one slab);
    with the split off the guided -104 and its candidates return."""
    rng = np.random.default_rng(77 + slabs)
    rows, cols = 256, 4096
    b0 = rand_board(rng, rows, cols)
    gens = 8 * 440
    ref = g.run_dead_fast(b0, gens)
    split = 2 if 3 * slabs + 1 <= hw_queues() else 1
    with engine(gh, rows, cols, n_gpus=slabs, layout="bit", tblock_k=8) as e:
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == split
        assert e.get_option(gh.OPT_CHUNK_ROWS) == (-1 if split == 2 else -104)
        e.upload(b0)
        e.step(gens)
        assert (e.download() == ref).all()
        assert e.get_option(gh.OPT_CHUNK_ROWS) in ((-1, -2, -3) if split == 2 else (-104, -6, -3))
    with engine(gh, rows, cols, n_gpus=slabs, layout="bit", tblock_k=8) as e:
        e.set_option(gh.OPT_INTERIOR_SPLIT, 1)
        assert e.get_option(gh.OPT_CHUNK_ROWS) == -104
        e.upload(b0)
        e.step(gens)
        assert (e.download() == ref).all()
        assert e.get_option(gh.OPT_CHUNK_ROWS) in (-104, -6, -3)
    with engine(gh, rows, cols, layout="bit", tblock_k=8) as e:
        e.set_option(gh.OPT_CHUNK_ROWS, 64)
        e.upload(b0)
        e.step(gens)
        assert e.get_option(gh.OPT_CHUNK_ROWS) == 64
        assert (e.download() == ref).all()


def hw_queues():
    """Hardware queues per device the HIP runtime gives this process (gol_runtime.cpp hw_queue_budget)."""
    try:
        n = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        n = 0
    return n if n > 0 else 4


def fold_gap(cols):
    """Units the k=8 pair kernel's folded strip stores (gol_kernels.hip fold_gap; 0: no fold)."""
    t = (cols + 127) // 128
    ns = 1 if t <= 64 else (2 if t <= 126 else 2 + (t - 126 + 61) // 62)
    gap = t - 64 - 62 * (ns - 2)
    return gap if ns >= 3 and 1 <= gap <= 30 else 0


FOLD_SHAPES = [(600, 16384), (333, 25600), (257, 24525), (410, 19968), (200, 19841)]


@pytest.mark.parametrize("shape", FOLD_SHAPES)
@pytest.mark.parametrize("chunk", [-104, -6, -3, 8, 37, 200])
def test_k8_folded_strip(gh, shape, chunk):
    """The k=8 pair kernel's folded tail strip (strip_geometry_fold): one wave's
    two half-waves cover the last gap of 128-column units for two chunk-rows
    (lanes 32-63 on the second chunk-row's rows).  Widths with gaps of 2-30
    units; guided, round and fixed chunk policies (even and odd numbers of
    chunk-rows, so unpaired folded items too; a band's first and last
    chunk-rows are unpaired, chunks shorter than the cone take the tall-chunk
    fallback); 1 and 2 slabs."""
    rows, cols = shape
    assert fold_gap(cols) > 0
    rng = np.random.default_rng(rows * 31 + cols + chunk)
    b0 = rand_board(rng, rows, cols)
    ref = g.run(b0, 32, g.DEAD)
    for slabs in (1, 2):
        with engine(gh, rows, cols, n_gpus=slabs, layout="bit", tblock_k=8) as e:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
            e.upload(b0)
            e.step(32)
            got = e.download()
        bad = np.argwhere(got != ref)
        assert bad.size == 0, (shape, chunk, slabs, len(bad), bad[:4].tolist())


@pytest.mark.parametrize("shape", [(97, 1000), (300, 9000), (64, 130), (1000, 37), (70, 64), (40, 65), (9, 4000)])
def test_bit_every_k_and_slabs(gh, shape):
    """Every fused depth k = 1..8 (each has its own pipeline variant: load-ring
    depth, stage chains), 1-3 slabs, against the oracle."""
    rows, cols = shape
    rng = np.random.default_rng(rows + 3 * cols)
    b0 = rand_board(rng, rows, cols)
    ref = g.run(b0, 24, g.DEAD)
    for k in range(1, 9):
        for slabs in (1, 2, 3):
            if rows // slabs < k:
                continue
            with engine(gh, rows, cols, n_gpus=slabs, layout="bit", tblock_k=k) as e:
                e.upload(b0)
                e.step(24)
                assert (e.download() == ref).all(), (shape, k, slabs)


# byte board, bit-sliced core (bytebit kernel): strips of 3968 columns, 4 blocks
# of 64 lanes × 16 columns, k up to 16 generations per HBM pass
BB_SHAPES = [(1, 1), (5, 17), (40, 3968), (41, 3969), (70, 3984), (33, 4000), (90, 7936), (64, 7953),
             (130, 8000), (17, 12000), (300, 640), (1000, 37), (50, 1920), (61, 1921), (45, 3840), (30, 5777),
             (44, 1984), (52, 1985), (33, 5952), (29, 1983)]


@pytest.mark.parametrize("shape", BB_SHAPES)
@pytest.mark.parametrize("boundary", ["dead", "serial_compat"])
def test_bytebit_random_shapes(gh, shape, boundary):
    rows, cols = shape
    if boundary == "serial_compat" and (rows < 2 or cols < 2):
        return
    rng = np.random.default_rng(rows * 31 + cols)
    b0 = rand_board(rng, rows, cols)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    mode = g.DEAD if boundary == "dead" else g.SERIAL_COMPAT
    gens = 33
    ref = g.run(b0, gens, mode)
    for k in (4, 8, 12, 16, 20, 24, 28, 32):
        for slabs in (1, 2, 3):
            if rows // slabs < k or (slabs > 1 and rows < 2 * slabs):
                continue
            with engine(gh, rows, cols, n_gpus=slabs, layout="byte", boundary=boundary, tblock_k=k) as e:
                e.upload(b0)
                e.step(gens - gens % k)
                if gens % k:
                    e.step(gens % k)   # partial last block: fewer generations than k
                got = e.download()
            assert (got == ref).all(), (shape, boundary, k, slabs, int((got != ref).sum()))


@pytest.mark.parametrize("chunk", [8, 37, 256, -1, -3, -104])
def test_bytebit_chunks_and_core_switch(gh, chunk):
    rng = np.random.default_rng(1000 + chunk)
    rows, cols = 400, 9000
    b0 = rand_board(rng, rows, cols)
    ref = g.run(b0, 24, g.DEAD)
    for k in (8, 12, 24):
        for core in (1, 0):
            if core == 0 and k > 8:
                continue
            with engine(gh, rows, cols, layout="byte", tblock_k=k) as e:
                e.set_option(gh.OPT_BYTE_CORE, core)
                e.set_option(gh.OPT_CHUNK_ROWS, chunk)
                e.upload(b0)
                e.step(24)
                assert (e.download() == ref).all(), (chunk, k, core)


@pytest.mark.parametrize("shape", [(300, 4096), (333, 6400), (257, 4961), (410, 4992), (200, 12000)])
@pytest.mark.parametrize("chunk", [-1, -3, 8, 37, -104])
def test_bytebit_wide_shapes(gh, shape, chunk):
    """The bytebit kernel (k = 20..32: one 32-column word per lane, strips of
    1984 columns) on boards 4096-12000 columns wide whose last strip is
    partial, even and odd numbers of chunk-rows, 1 and 2 slabs.  (A folded
    tail strip for this kernel, like the k=8 pair kernel's, was built and
    measured a tie: DESIGN.md §3.)"""
    rows, cols = shape
    rng = np.random.default_rng(rows * 17 + cols + chunk)
    b0 = rand_board(rng, rows, cols)
    ref = g.run(b0, 64, g.DEAD)
    for k in (20, 24, 28, 32):
        for slabs in (1, 2):
            with engine(gh, rows, cols, n_gpus=slabs, layout="byte", tblock_k=k) as e:
                e.set_option(gh.OPT_CHUNK_ROWS, chunk)
                e.upload(b0)
                e.step(64 - 64 % k)
                if 64 % k:
                    e.step(64 % k)
                got = e.download()
            bad = np.argwhere(got != ref)
            assert bad.size == 0, (shape, chunk, k, slabs, len(bad), bad[:4].tolist())


@pytest.mark.parametrize("k", [16, 24, 28, 32])
def test_bytebit_32768_lightcone(gh, k):
    """BASELINE config 3 size: byte board 32768², k=16 / 24 / 28 / 32, two slabs
    on one GPU; strip seams (3968 / 1984 columns) and the last, partial strip."""
    n, gens = 32768, 48
    with engine(gh, n, n, layout="byte", tblock_k=k, n_gpus=2) as e:
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(0, 0), (n // 2 - 32, 3968 - 30), (n - 64, n - 64), (n // 2 - 3, n - 64),
                         (12345, 3968 * 5 - 10), (777, 1984 - 30), (20001, 1984 * 15 - 33),
                         (n // 2 + 100, 1984 * 16 - 31), (9000, 32 * 945)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (r0, c0)


@pytest.mark.parametrize("layout,k", [("bit", 8), ("bit", 3), ("byte", 8), ("byte", 28), ("byte", 3)])
@pytest.mark.parametrize("slabs", [2, 3])
def test_uneven_steps_across_slabs(gh, layout, k, slabs):
    """Steps shorter and longer than the previous one (a short last block, then
    full blocks): the halo rows a deeper step sends were partly written by the
    previous step's interior kernel (gol_runtime.cpp exchange(), "grow")."""
    rng = np.random.default_rng(k * 10 + slabs)
    rows, cols = 70 * slabs + 17, 2100
    b0 = rand_board(rng, rows, cols)
    steps = [1, k, 2, k, k, 1, 3, k]
    with engine(gh, rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
        e.upload(b0)
        for st in steps:
            e.step(st)
        got = e.download()
    assert (got == g.run(b0, sum(steps), g.DEAD)).all(), (layout, k, slabs)


@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_serial_random_rect(gh, layout):
    rng = np.random.default_rng(5)
    rows, cols = 71, 190
    b0 = rand_board(rng, rows, cols)
    with engine(gh, rows, cols, layout=layout, boundary="serial_compat", tblock_k=3, n_gpus=2) as e:
        e.upload(b0)
        b0m = b0.copy()
        b0m[-1, :] = 0
        b0m[:, -1] = 0
        assert (e.download() == b0m).all()
        e.step(10)
        got = e.download()
    assert (got == g.run(b0m, 10, g.SERIAL_COMPAT)).all()


def mismatch(got, want):
    """'' when equal, else a summary naming the first bad cell and whether
    every mismatch is a lost live cell (1 -> 0, e.g. a late zero-fill)."""
    bad = np.argwhere(got != want)
    if bad.size == 0:
        return ""
    lost = bool(((want[got != want] == 1) & (got[got != want] == 0)).all())
    r, c = bad[0].tolist()
    return (f"{len(bad)} of {want.size} cells differ; first at ({r},{c}) got {int(got[r, c])} want "
            f"{int(want[r, c])}; rows {int(bad[:, 0].min())}..{int(bad[:, 0].max())}; all 1->0: {lost}")


@pytest.mark.parametrize("n,m", [(48, 3), (60, 5), (1026, 3), (100, 4), (64, 64), (300, 2)])
@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_mesh_random(gh, n, m, layout):
    rng = np.random.default_rng(n + m)
    b0 = rand_board(rng, n, n)
    want = g.run(b0, 9, g.MESH_COMPAT, m)
    for slabs in (1, 4):
        for k in (1, 4, 8):
            with engine(gh, n, n, n_gpus=slabs, layout=layout, boundary="mesh_compat", mesh_m=m, tblock_k=k) as e:
                e.upload(b0)
                d = mismatch(e.download(), b0)
                assert not d, ("round trip", slabs, k, d)
                e.step(9)
                d = mismatch(e.download(), want)
                assert not d, ("9 generations", slabs, k, d)
                # windows across block edges (logical -> storage column runs)
                c0 = max(0, n // m - 2)
                w = e.download_window(n // 3, c0, min(20, n - n // 3), min(n - c0, n // m + 5))
                assert (w == want[n // 3:n // 3 + w.shape[0], c0:c0 + w.shape[1]]).all()


@pytest.mark.parametrize("layout", ["bit", "byte"])
@pytest.mark.parametrize("boundary", ["dead", "mesh_compat"])
def test_fresh_board_roundtrip(gh, layout, boundary):
    """Create → upload → download with no step in between, on freshly
    allocated 4096² boards in 4 slabs, several times in a row (each context may
    reuse the previous one's freed memory).  The zero-fill of new boards must
    be ordered before the first upload on the slabs' non-blocking streams
    (GPUTEST_r04's red test_mesh_random[byte-1026-3] was a late fill)."""
    n = 4096
    rng = np.random.default_rng(4096)
    b0 = rand_board(rng, n, n)
    for i in range(3):
        with engine(gh, n, n, n_gpus=4, layout=layout, boundary=boundary, mesh_m=4, tblock_k=8) as e:
            e.upload(b0)
            d = mismatch(e.download(), b0)
            assert not d, (i, d)
            assert e.popcount() == int(b0.sum())


@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_mesh_text_roundtrip(gh, layout):
    """Snapshot text of a MESH_COMPAT board is in logical column order."""
    rng = np.random.default_rng(17)
    n, m = 96, 3
    b0 = rand_board(rng, n, n)
    with engine(gh, n, n, layout=layout, boundary="mesh_compat", mesh_m=m, tblock_k=2, n_gpus=2) as e:
        e.upload(b0)
        e.step(6)
        want = g.run(b0, 6, g.MESH_COMPAT, m)
        txt = e.format_text(0, 0, n, n)
        assert txt == g.text_body(want)
        e.parse_text(5, 7, 40, 50, g.text_body(b0[5:45, 7:57]))
        want[5:45, 7:57] = b0[5:45, 7:57]
        assert (e.download() == want).all()


def test_extremes(gh):
    for layout in ("bit", "byte"):
        for fill in (0, 1):
            b0 = np.full((50, 70), fill, np.uint8)
            with engine(gh, 50, 70, layout=layout, tblock_k=2) as e:
                e.upload(b0)
                e.step(6)
                assert (e.download() == g.run(b0, 6, g.DEAD)).all()
    # a glider flying into the bottom-right corner
    b0 = np.zeros((40, 40), np.uint8)
    b0[1, 2] = b0[2, 3] = b0[3, 1] = b0[3, 2] = b0[3, 3] = 1
    with engine(gh, 40, 40, layout="bit", tblock_k=8, n_gpus=3) as e:
        e.upload(b0)
        e.step(200)
        assert (e.download() == g.run(b0, 200, g.DEAD)).all()


# ---------------------------------------------------------------- init

@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_init_stream_matches_oracle(gh, layout):
    rows, cols = 700, 5000
    for slabs in (1, 3):
        for seed in (0, 1, 12345):
            with engine(gh, rows, cols, layout=layout, n_gpus=slabs) as e:
                e.initialize_board("stream", seed)
                got = e.download()
            assert (got == g.init_dead(rows, cols, seed)).all(), (slabs, seed)


def test_init_serial_and_mesh(gh):
    with engine(gh, 300, 300, layout="bit", boundary="serial_compat", n_gpus=2) as e:
        e.initialize_board("serial", g.SERIAL_SEED)
        assert (e.download() == g.init_serial(300)).all()
    with engine(gh, 256, 256, layout="byte", boundary="mesh_compat", mesh_m=4, n_gpus=3) as e:
        e.initialize_board("mesh", 0)
        assert (e.download() == g.init_mesh(256, 4)).all()
    with engine(gh, 256, 256, layout="bit", n_gpus=1, mesh_m=2) as e:
        e.initialize_board("mesh", 0)
        assert (e.download() == g.init_mesh(256, 2)).all()


# ---------------------------------------------------------------- windows / io

def test_window_io(gh):
    rng = np.random.default_rng(11)
    rows, cols = 333, 2000
    b0 = rand_board(rng, rows, cols)
    for layout in ("bit", "byte"):
        with engine(gh, rows, cols, layout=layout, n_gpus=2) as e:
            e.upload(b0)
            w = e.download_window(100, 37, 200, 1001)
            assert (w == b0[100:300, 37:1038]).all()
            patch = rand_board(rng, 50, 77)
            e.upload_window(150, 13, patch)
            b1 = b0.copy()
            b1[150:200, 13:90] = patch
            assert (e.download() == b1).all()
            assert e.popcount() == int(b1.sum())


# ---------------------------------------------------------------- full size

def lightcone_check(e, rows, cols, gens, r0, c0, h, w, seed=1):
    """Window [r0,r0+h)×[c0,c0+w) of generation `gens` vs the oracle run on the
    gen-0 window grown by `gens` cells (clipped at the grid edge, which is dead)."""
    R0, C0 = max(0, r0 - gens), max(0, c0 - gens)
    R1, C1 = min(rows, r0 + h + gens), min(cols, c0 + w + gens)
    b0 = g.init_dead(R1 - R0, C1 - C0, seed, row0=R0, full_cols=cols, col0=C0)
    ref = g.run(b0, gens, g.DEAD)[r0 - R0:r0 - R0 + h, c0 - C0:c0 - C0 + w]
    got = e.download_window(r0, c0, h, w)
    return (got == ref).all()


def test_baseline_size_lightcone(gh):
    """131072² bit layout (BASELINE config 4): init on device, 16 generations in
    k=4 blocks, then corner/edge/interior windows vs the oracle light cone."""
    n, gens = 131072, 16
    with engine(gh, n, n, layout="bit", tblock_k=4) as e:
        e.initialize_board("stream", 1)
        # generation-0 spot check deep in the grid (jump-ahead of the init)
        w0 = e.download_window(99999, 70001, 3, 500)
        assert (w0 == g.init_dead(3, 500, 1, row0=99999, full_cols=n, col0=70001)).all()
        e.step(gens)
        e.sync()
        for (r0, c0) in [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64), (65536 - 20, 4096 * 16 - 30),
                         (12345, 777), (n // 2, n // 2)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (r0, c0)
        live = e.popcount()
        assert 0.05 * n * n < live < 0.5 * n * n


def test_baseline_size_two_slabs_lightcone(gh):
    """131072² bit layout as two slabs on one GPU (the halo path of config 5 at
    full width), k=8 with a short block in between, windows at the slab seam."""
    n = 131072
    with engine(gh, n, n, layout="bit", tblock_k=8, n_gpus=2) as e:
        e.initialize_board("stream", 1)
        for st in (8, 3, 8, 5):
            e.step(st)
        gens = 24
        for (r0, c0) in [(n // 2 - 40, 0), (n // 2 - 32, n - 64), (n // 2 + 5, 70000), (0, 1000), (n - 64, 5)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (r0, c0)


def test_byte_32768_lightcone(gh):
    n, gens = 32768, 6
    with engine(gh, n, n, layout="byte", tblock_k=2, n_gpus=2) as e:
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(0, 0), (n // 2 - 32, 1000), (n - 64, n - 64), (n // 2 - 3, n - 64)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (r0, c0)


# ---------------------------------------------------------------- driver

def test_driver_serial_snapshots(gh, tmp_path):
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    subprocess.run([exe, "--mode", "serial", "48", "48", "10", "30"], cwd=tmp_path, check=True,
                   capture_output=True)
    mains = [f for f in os.listdir(tmp_path) if f.endswith(".gol") and "_" not in f]
    assert len(mains) == 1
    name = mains[0][:-4]
    assert open(tmp_path / mains[0]).read().split() == ["48", "48", "10", "30", "1"]
    b = g.init_serial(48)
    for it in (0, 10, 20, 30):
        if it:
            b = g.run(b, 10, g.SERIAL_COMPAT)
        lines = open(tmp_path / f"{name}_{it}_0.gol").read().splitlines()
        assert lines[0] == "0 48" and lines[1] == "0 48"
        cells = np.array([[int(t) for t in ln.split()] for ln in lines[2:]], np.uint8)
        assert (cells == b).all(), it
    # the reference's timing files
    assert (tmp_path / f"{name}_detailed.out").exists() and (tmp_path / f"{name}_compact.csv").exists()


def test_driver_mpi_mesh(gh, tmp_path):
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    subprocess.run([exe, "--procs", "4", "--gpus", "2", "--save", "64", "64", "5", "10", "t", "1"],
                   cwd=tmp_path, check=True, capture_output=True)
    name = [f for f in os.listdir(tmp_path) if f.endswith(".gol") and "_" not in f][0][:-4]
    b = g.run(g.init_mesh(64, 2), 10, g.MESH_COMPAT, 2)
    got = np.zeros((64, 64), np.uint8)
    for p in range(2):
        lines = open(tmp_path / f"{name}_10_{p}.gol").read().splitlines()
        r0, r1 = map(int, lines[0].split())
        c0, c1 = map(int, lines[1].split())
        got[r0:r1 + 1, c0:c1 + 1] = np.array([[int(t) for t in ln.split()] for ln in lines[2:]])
    assert (got == b).all()
    csv = open(tmp_path / "t_compact.csv").read().splitlines()
    assert csv[0].startswith("X,Y,#P") and len(csv[1].split(",")) == 12 and csv[1].split(",")[2] == "4"


@pytest.mark.parametrize("layout,k", [("byte", 28), ("bit", 8)])
def test_driver_dead_mode_uneven_gap(gh, tmp_path, layout, k):
    """bin/gol --mode dead with a snapshot gap that is not a multiple of k (short
    blocks between full ones) on 2 slabs: every part file vs the oracle."""
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    rows, cols, gap, iters = 300, 2100, 10, 40
    r = subprocess.run([exe, "--mode", "dead", "--layout", layout, "-k", str(k), "--gpus", "2", "--save",
                        str(rows), str(cols), str(gap), str(iters)], cwd=tmp_path, check=True, capture_output=True,
                       text=True)
    # the driver steps straight to each snapshot, so the fused kernels run (gol_step's
    # blocks: min(k, left), a byte-board block > 8 without a bytebit kernel runs as 8);
    # one timed interior launch per block and slab
    def blocks(n):
        c = 0
        while n > 0:
            b = min(k, n)
            if layout == "byte" and b > 8 and b % 4:
                b = 8
            n, c = n - b, c + 1
        return c
    assert f"launches={2 * blocks(gap) * iters // gap}" in r.stdout, r.stdout
    name = [f for f in os.listdir(tmp_path) if f.endswith(".gol") and "_" not in f][0][:-4]
    b = g.init_dead(rows, cols, 1)
    for it in range(0, iters + 1, gap):
        if it:
            b = g.run(b, gap, g.DEAD)
        got = np.zeros((rows, cols), np.uint8)
        for p in range(2):
            lines = open(tmp_path / f"{name}_{it}_{p}.gol").read().splitlines()
            r0, r1 = map(int, lines[0].split())
            got[r0:r1 + 1] = np.array([[int(t) for t in ln.split()] for ln in lines[2:]], np.uint8)
        assert (got == b).all(), it


@pytest.mark.parametrize("mode,layout,k,parts", [("dead", "bit", 8, 2), ("dead", "byte", 32, 3), ("mpi", "bit", 3, 2),
                                                  ("serial", "byte", 4, 2)])
def test_driver_rccl_ranks(gh, tmp_path, mode, layout, k, parts):
    """bin/gol --rccl: the slabs as RCCL ranks of one process (one rank context
    and communicator per device, a host thread each, halo rows through
    ncclSend/Recv — main.cpp:36-65's exchange, the ranks of main.cpp:154-164).
    One GPU holds every rank here (--same-device), which real RCCL refuses, so
    the ranks bind the in-process RCCL stand-in (--rccl-lib
    tests/shim/libfake_rccl.so); the kernels, slabs, halo events and snapshot
    writes are the library's own.  Every part file at every gap vs the oracle,
    and the same files as the one-context --gpus N run (peer copies)."""
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    shim = os.path.join(ROOT, "tests", "shim", "libfake_rccl.so")
    n = 192 if mode != "dead" else 0
    rows, cols, gap, iters = (n, n, 7, 21) if n else (300, 2100, 10, 40)
    args = ["--mode", mode, "--layout", layout, "-k", str(k), "--gpus", str(parts), "--save"]
    if mode == "mpi":
        args += ["--procs", "4"]
    outs = {}
    for tag, extra in (("rccl", ["--rccl", "--same-device", "--rccl-lib", shim]), ("peer", [])):
        d = tmp_path / tag
        d.mkdir()
        r = subprocess.run([exe] + args + extra + [str(rows), str(cols), str(gap), str(iters)], cwd=d,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (tag, r.stdout[-2000:], r.stderr[-2000:])
        assert ("(rccl ranks)" in r.stdout) == (tag == "rccl")
        name = [f for f in os.listdir(d) if f.endswith(".gol") and "_" not in f][0][:-4]
        outs[tag] = (d, name)
    if mode == "serial":
        b, m = g.init_serial(rows), g.SERIAL_COMPAT
    elif mode == "mpi":
        b, m = g.init_mesh(rows, 2), g.MESH_COMPAT
    else:
        b, m = g.init_dead(rows, cols, 1), g.DEAD
    for it in range(0, iters + 1, gap):
        if it:
            b = g.run(b, gap, m, mesh_m=2) if mode == "mpi" else g.run(b, gap, m)
        for tag, (d, name) in outs.items():
            got = np.zeros((rows, cols), np.uint8)
            for p in range(parts):
                lines = open(d / f"{name}_{it}_{p}.gol").read().splitlines()
                r0, r1 = map(int, lines[0].split())
                got[r0:r1 + 1] = np.array([[int(t) for t in ln.split()] for ln in lines[2:]], np.uint8)
            assert (got == b).all(), (tag, it, int((got != b).sum()))


def _part_window(path, n, r0, c0, h, w):
    """Cells [r0, r0+h) × [c0, c0+w) from a `.gol` part file (inclusive
    header "first last" rows, then rows of "v\t" tokens), without parsing it all."""
    with open(path, "rb") as f:
        first = int(f.readline().split()[0])
        f.readline()
        base = f.tell()
        out = np.empty((h, w), np.uint8)
        for i in range(h):
            f.seek(base + (r0 + i - first) * (2 * n + 1) + 2 * c0)
            out[i] = np.frombuffer(f.read(2 * w), np.uint8)[0::2] - ord("0")
    return out


@pytest.mark.timeout(420)
def test_driver_mpi_p16_16384(gh, tmp_path):
    """main.cpp's P=16 semantics (BASELINE config 2's rule: a 4×4 mesh with the
    swapped column halos of main.cpp:51-54) at 16384² through bin/gol --procs 16
    --gpus 2 -k 3: windows straddling the 4096-column block edges and the slab
    seam, at generations 0 and 6, vs the oracle's per-block ghost-column run."""
    n, gens, m = 16384, 6, 4
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    subprocess.run([exe, "--procs", "16", "--gpus", "2", "-k", "3", "--save", str(n), str(n), str(gens), str(gens),
                    "t", "1"], cwd=tmp_path, check=True, capture_output=True, timeout=300)
    name = [f for f in os.listdir(tmp_path) if f.endswith(".gol") and "_" not in f][0][:-4]
    want = {0: g.init_mesh(n, m)}
    want[gens] = g.run_mesh_fast(want[0], gens, m)
    L = n // m
    wins = [(0, 0), (n // 2 - 64, L - 32), (n // 2, 3 * L - 40), (100, 2 * L - 32), (n - 64, n - 64),
            (12000, L - 1), (5000, 3 * L - 63), (n // 2 + 3, 2 * L - 2)]
    for it in (0, gens):
        for r0, c0 in wins:
            p = r0 // (n // 2)
            if (r0 + 63) // (n // 2) != p:   # a window inside one part file
                continue
            got = _part_window(tmp_path / f"{name}_{it}_{p}.gol", n, r0, c0, 64, 64)
            assert (got == want[it][r0:r0 + 64, c0:c0 + 64]).all(), (it, r0, c0)
    csv = open(tmp_path / "t_compact.csv").read().splitlines()
    assert csv[0].startswith("X,Y,#P") and csv[1].split(",")[:3] == [str(n), str(n), "16"]   # --procs 16 (main.cpp:341-362)


@pytest.mark.parametrize("layout,k", [("bit", 8), ("bit", 3), ("bit", 1), ("byte", 32), ("byte", 1), ("byte", 8)])
@pytest.mark.parametrize("slabs", [1, 2, 3])
def test_interior_split(gh, layout, k, slabs):
    """GOL_OPT_INTERIOR_SPLIT = 2: each slab's interior as two launches on two
    streams with a seam band between them (the next step's first half overlaps
    this step's second half).  Boards tall enough to split (>= 64k interior rows
    per slab) and a short one that steps whole, uneven step depths, the option
    toggled mid-run; bit-exact against the oracle."""
    rows = max(64 * k * slabs + 4 * k * slabs + 37, 160 * slabs)
    cols = 2100 if layout == "bit" else 4100
    rng = np.random.default_rng(rows * 13 + k * 7 + slabs)
    b0 = rand_board(rng, rows, cols)
    steps = [k, k, 1, k, 2, k, k]
    with engine(gh, rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
        e.upload(b0)
        e.set_option(gh.OPT_INTERIOR_SPLIT, 2)
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == 2
        for st in steps[:4]:
            e.step(st)
        mid = e.download_window(rows // 2 - 20, 0, 40, cols)   # across the seam band
        e.set_option(gh.OPT_INTERIOR_SPLIT, 1)
        e.step(steps[4])
        e.set_option(gh.OPT_INTERIOR_SPLIT, 2)
        for st in steps[5:]:
            e.step(st)
        got = e.download()
    g4 = g.run_dead_fast(b0, sum(steps[:4]))
    d = mismatch(mid, g4[rows // 2 - 20:rows // 2 + 20])
    assert not d, ("mid-run window", d)
    d = mismatch(got, g.run_dead_fast(b0, sum(steps)))
    assert not d, (layout, k, slabs, d)


def test_interior_split_short_slab(gh):
    """A slab too short to split steps whole under GOL_OPT_INTERIOR_SPLIT = 2."""
    rng = np.random.default_rng(5150)
    b0 = rand_board(rng, 300, 3000)
    with engine(gh, 300, 3000, n_gpus=2, layout="bit", tblock_k=8) as e:
        e.upload(b0)
        e.set_option(gh.OPT_INTERIOR_SPLIT, 2)
        e.step(40)
        assert (e.download() == g.run(b0, 40, g.DEAD)).all()
    with engine(gh, 64, 64, layout="bit", tblock_k=2) as e:
        for bad in (0, 5):
            with pytest.raises(gh.GolError):
                e.set_option(gh.OPT_INTERIOR_SPLIT, bad)


@pytest.mark.parametrize("layout,k", [("bit", 8), ("bit", 3), ("byte", 32)])
@pytest.mark.parametrize("slabs", [1, 2])
@pytest.mark.parametrize("parts", [3, 4])
def test_interior_split_parts(gh, layout, k, slabs, parts):
    """GOL_OPT_INTERIOR_SPLIT = 3 / 4: the interior in that many launches on as
    many streams, a seam band at every cut; a board tall enough for all parts,
    uneven step depths, the part count changed mid-run (4 -> 2 -> parts, and a
    slab too short for all parts takes fewer); bit-exact against the oracle."""
    rows = (32 * k * parts + 4 * k + 29) * slabs
    cols = 2100 if layout == "bit" else 4100
    rng = np.random.default_rng(rows * 7 + k * 3 + slabs + parts)
    b0 = rand_board(rng, rows, cols)
    steps = [k, 1, k, k, 2, k, k, 3]
    with engine(gh, rows, cols, n_gpus=slabs, layout=layout, tblock_k=k) as e:
        e.upload(b0)
        e.set_option(gh.OPT_INTERIOR_SPLIT, parts)
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == parts
        for st in steps[:3]:
            e.step(st)
        e.set_option(gh.OPT_INTERIOR_SPLIT, 2)
        for st in steps[3:5]:
            e.step(st)
        e.set_option(gh.OPT_INTERIOR_SPLIT, parts)
        for st in steps[5:]:
            e.step(st)
        got = e.download()
    d = mismatch(got, g.run_dead_fast(b0, sum(steps)))
    assert not d, (layout, k, slabs, parts, d)
    # a short slab: parts fall back to what fits (here one or two)
    rows2 = 32 * k * 2 + 4 * k + 5
    b1 = rand_board(rng, rows2, cols)
    with engine(gh, rows2, cols, layout=layout, tblock_k=k) as e:
        e.upload(b1)
        e.set_option(gh.OPT_INTERIOR_SPLIT, parts)
        e.step(3 * k + 1)
        assert (e.download() == g.run_dead_fast(b1, 3 * k + 1)).all()

@pytest.mark.parametrize("parts", [3, 4])
def test_interior_split_cuts_fixed_across_depths(gh, parts):
    """The fuzz case that found it (tools/fuzz.py seed 521, case 56): 2 slabs of
    1058 rows, bit k = 5, split into 4, steps 14/11/5 (blocks 5,5,4,5,5,1,5),
    guided chunks.  The cuts between parts were taken over [lo+k, hi-k), so a
    block of another depth moved them by a row or two and a part overwrote rows
    the neighbouring part of the previous step (another stream, not waited for)
    still read.  The cuts now come from the context's depth; the same run, many
    shallow/deep alternations, bit-exact."""
    rows, cols, k = 2116, 47, 5
    rng = np.random.default_rng(521056 + parts)
    b0 = rand_board(rng, rows, cols)
    steps = [14, 11, 5, 1, 5, 2, 9, 1, 1, 13]
    with engine(gh, rows, cols, n_gpus=2, layout="bit", tblock_k=k) as e:
        e.set_option(gh.OPT_CHUNK_ROWS, -103)
        e.set_option(gh.OPT_INTERIOR_SPLIT, parts)
        e.upload(b0)
        for st in steps:
            e.step(st)
        got = e.download()
    d = mismatch(got, g.run_dead_fast(b0, sum(steps)))
    assert not d, (parts, d)



@pytest.mark.timeout(300)
@pytest.mark.parametrize("split", [2, 1])
def test_headline_split_full_size(gh, split):
    """The headline shape (131072², bit, k = 8) with the split interior (the
    default) and without it: 96 generations (default schedule, trial off),
    light-cone windows across the seam band, the XCD band seams and the
    corners."""
    n, gens = 131072, 96
    with engine(gh, n, n, layout="bit", tblock_k=8) as e:
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == 2
        e.set_option(gh.OPT_SCHEDULE_TRIAL, 0)
        e.set_option(gh.OPT_INTERIOR_SPLIT, split)
        assert e.get_option(gh.OPT_CHUNK_ROWS) == (-1 if split == 2 else -104)
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(n // 2 - 32, 5000), (n // 2 - 8 - 64, 70001), (n // 2 + 8, n - 64), (0, 0),
                         (n - 64, n - 64), (16384 * 3 - 30, 1000), (16384 * 5 + 7, 99999)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (r0, c0)
