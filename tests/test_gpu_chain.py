"""GPU parity of the byte board's chain kernel (bytebit_coop_kernel,
gol_kernels.hip): a workgroup of 2 or 4 waves per column strip, each wave
running 12 or 16 of the K fused generations, rows handed from wave to wave
through LDS (K = 24, 32: 2 waves; K = 48, 64: 4 waves).  Bit-exact against
the oracle (oracle/golcpu.c, pinned by the reference goldens) on odd shapes
around the strip widths (1984 columns at K <= 32, 1920 at K = 48, 64), every
chunk policy, 1-3 slabs, both boundaries, short last blocks; the reference
goldens; and light-cone windows at BASELINE config 3's 32768².
(main.cpp:79-103 / main_serial.cpp:45-71: updateBoard, K generations per pass.)"""
import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu

CHAIN = 3   # GOL_OPT_BYTE_CORE: the chain kernel
DEPTHS = (24, 32, 48, 64)


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def rand_board(rng, rows, cols, p=0.35):
    return (rng.random((rows, cols)) < p).astype(np.uint8)


def run_chain(gh, b0, gens, k, slabs=1, boundary="dead", chunk=None, mesh_m=1):
    rows, cols = b0.shape
    with gh.Engine(rows, cols, n_gpus=slabs, layout="byte", boundary=boundary, mesh_m=mesh_m, tblock_k=k) as e:
        e.set_option(gh.OPT_BYTE_CORE, CHAIN)
        if chunk is not None:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
        e.upload(b0)
        e.step(gens - gens % k)
        if gens % k:
            e.step(gens % k)   # a short last block (another kernel: the board must carry over)
        return e.download()


def mismatch(got, ref):
    bad = np.argwhere(got != ref)
    return None if bad.size == 0 else (len(bad), bad[:4].tolist())


SHAPES = [(1, 1), (5, 17), (70, 1919), (71, 1920), (66, 1921), (40, 1984), (41, 1985), (90, 3840), (64, 3841),
          (130, 3968), (33, 4000), (300, 640), (400, 37), (170, 5777), (200, 7681)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("boundary", ["dead", "serial_compat"])
def test_chain_random_shapes(gh, shape, boundary):
    rows, cols = shape
    if boundary == "serial_compat" and (rows < 2 or cols < 2):
        return
    rng = np.random.default_rng(rows * 131 + cols)
    b0 = rand_board(rng, rows, cols)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    gens = 70
    ref = g.run(b0, gens, g.DEAD if boundary == "dead" else g.SERIAL_COMPAT)
    for k in DEPTHS:
        for slabs in (1, 2, 3):
            if rows // slabs < k or (slabs > 1 and rows < 2 * slabs):
                continue
            d = mismatch(run_chain(gh, b0, gens, k, slabs, boundary), ref)
            assert d is None, (shape, boundary, k, slabs, d)


@pytest.mark.parametrize("chunk", [-1, -2, -3, 8, 37, 256, -104])
def test_chain_chunk_policies(gh, chunk):
    """Every chunk policy (the chain kernel plans one item per workgroup; a
    guided policy runs as one round), tall and short chunks, partial strips."""
    rng = np.random.default_rng(2000 + chunk)
    rows, cols = 700, 9000
    b0 = rand_board(rng, rows, cols)
    gens = 128
    ref = g.run_dead_fast(b0, gens)
    for k in DEPTHS:
        for slabs in (1, 2):
            d = mismatch(run_chain(gh, b0, gens, k, slabs, chunk=chunk), ref)
            assert d is None, (chunk, k, slabs, d)


def test_chain_matches_wave_kernel_and_swar(gh):
    """K = 24 and 32 through the chain kernel, the one-wave kernel and the
    default; K = 48 and 64 ignore the one-wave choice (chain only); all equal."""
    rng = np.random.default_rng(77)
    rows, cols = 333, 6100
    b0 = rand_board(rng, rows, cols)
    ref = g.run_dead_fast(b0, 192)
    for k in DEPTHS:
        for core in (1, 2, 3):
            with gh.Engine(rows, cols, layout="byte", tblock_k=k) as e:
                e.set_option(gh.OPT_BYTE_CORE, core)
                assert e.get_option(gh.OPT_BYTE_CORE) == core
                e.upload(b0)
                e.step(192)
                d = mismatch(e.download(), ref)
            assert d is None, (k, core, d)


@pytest.mark.parametrize("k", [32, 64])
def test_chain_goldens(gh, golden, k):
    """The reference's own boards: serial 1024² (main_serial.cpp) and
    mpirun -np 1/4/16 (main.cpp) at 1024², through the chain kernel."""
    d, cases = golden
    for name, case in cases.items():
        n = case["n"]
        if n < 1024:
            continue
        mode, m = case["mode"], case["mesh_m"]
        init = {"serial_compat": ("serial", g.SERIAL_SEED), "dead": ("stream", 0), "mesh_compat": ("mesh", 0)}[mode]
        with gh.Engine(n, n, layout="byte", boundary=mode, mesh_m=m, tblock_k=k) as e:
            e.set_option(gh.OPT_BYTE_CORE, CHAIN)
            e.initialize_board(*init)
            done = 0
            for gen in sorted(int(x) for x in case["gens"]):
                e.step(gen - done)
                done = gen
                assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (name, k, gen)


def lightcone_check(e, rows, cols, gens, r0, c0, h, w, seed=1):
    R0, C0 = max(0, r0 - gens), max(0, c0 - gens)
    R1, C1 = min(rows, r0 + h + gens), min(cols, c0 + w + gens)
    b0 = g.init_dead(R1 - R0, C1 - C0, seed, row0=R0, full_cols=cols, col0=C0)
    ref = g.run(b0, gens, g.DEAD)[r0 - R0:r0 - R0 + h, c0 - C0:c0 - C0 + w]
    return (e.download_window(r0, c0, h, w) == ref).all()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [32, 64])
def test_chain_32768_lightcone(gh, k):
    """BASELINE config 3's board (32768², srand(1) stream, dead boundary) through
    the chain kernel, one slab, default one-round chunks: windows at strip seams
    (1984 / 1920 columns), chunk seams, the corners and the last partial strip."""
    n, gens = 32768, 2 * k
    W = 1984 if k <= 32 else 1920
    with gh.Engine(n, n, layout="byte", tblock_k=k) as e:
        e.set_option(gh.OPT_BYTE_CORE, CHAIN)
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64), (n // 2 - 32, W - 30),
                         (12345, 5 * W - 10), (20001, 15 * W - 33), (n // 3, 16 * W - 31), (9000, n - 100)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (k, r0, c0)


# ------------------------------------------------ bit board: chains of pair waves
# bit_chain_kernel<S> (gol_kernels.hip): k = 16 / 32 generations per HBM pass on
# the k = 8 layout (4-word groups), a chain of 2 / 4 waves per strip, each the
# 8-stage row-pair pipeline, rows handed through the next wave's LDS ring.

BIT_SHAPES = [(40, 40), (70, 300), (129, 1000), (300, 2100), (333, 8193), (600, 16384), (257, 24525),
              (410, 19968), (200, 19841), (1000, 129)]


@pytest.mark.parametrize("shape", BIT_SHAPES)
@pytest.mark.parametrize("boundary", ["dead", "serial_compat"])
def test_bit_chain_random_shapes(gh, shape, boundary):
    """Odd shapes (the folded tail strip's widths among them), 1-3 slabs, the
    split interior on (the default) and off, a short last block (a 16-deep
    block and 8-deep ones after k-deep ones), both boundaries; bit-exact."""
    rows, cols = shape
    rng = np.random.default_rng(rows * 7 + cols)
    b0 = rand_board(rng, rows, cols)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    for k in (16, 32):
        gens = 3 * k + 21
        ref = g.run(b0, gens, g.DEAD if boundary == "dead" else g.SERIAL_COMPAT)
        for slabs in (1, 2, 3):
            if rows // slabs < k or (slabs > 1 and rows < 2 * slabs):
                continue
            for split in (None, 1):
                with gh.Engine(rows, cols, n_gpus=slabs, layout="bit", boundary=boundary, tblock_k=k) as e:
                    if split:
                        e.set_option(gh.OPT_INTERIOR_SPLIT, split)
                    e.upload(b0)
                    e.step(gens - gens % k)
                    e.step(gens % k)
                    d = mismatch(e.download(), ref)
                assert d is None, (shape, boundary, k, slabs, split, d)


@pytest.mark.parametrize("chunk", [-1, -2, -3, 8, 37, 256, -104])
def test_bit_chain_chunk_policies(gh, chunk):
    rng = np.random.default_rng(3000 + chunk)
    rows, cols = 900, 20000
    b0 = rand_board(rng, rows, cols)
    gens = 128
    ref = g.run_dead_fast(b0, gens)
    for k in (16, 32):
        for slabs in (1, 2):
            with gh.Engine(rows, cols, n_gpus=slabs, layout="bit", tblock_k=k) as e:
                e.set_option(gh.OPT_CHUNK_ROWS, chunk)
                e.upload(b0)
                e.step(gens)
                d = mismatch(e.download(), ref)
            assert d is None, (chunk, k, slabs, d)


def test_bit_chain_mesh_goldens(gh, golden):
    """main.cpp's mesh semantics (swapped column halos) and the serial and P=1
    references at 1024², through the k = 16 / 32 chains."""
    d, cases = golden
    for name, case in cases.items():
        n = case["n"]
        if n < 1024:
            continue
        mode, m = case["mode"], case["mesh_m"]
        init = {"serial_compat": ("serial", g.SERIAL_SEED), "dead": ("stream", 0), "mesh_compat": ("mesh", 0)}[mode]
        for k in (16, 32):
            with gh.Engine(n, n, layout="bit", boundary=mode, mesh_m=m, tblock_k=k) as e:
                e.initialize_board(*init)
                done = 0
                for gen in sorted(int(x) for x in case["gens"]):
                    e.step(gen - done)
                    done = gen
                    assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (name, k, gen)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", [16, 32])
def test_bit_chain_131072_lightcone(gh, k):
    """BASELINE config 4's board (131072², srand(1), dead boundary) through the
    chain at its default schedule (split interior, one round per half): windows
    at the corners, strip seams (128·(62s + 1) columns), the folded strip, the
    split's seam band and chunk seams."""
    n, gens = 131072, 3 * k
    seam = lambda s: 128 * (62 * s + 1)
    with gh.Engine(n, n, layout="bit", tblock_k=k) as e:
        assert e.get_option(gh.OPT_INTERIOR_SPLIT) == 2 and e.get_option(gh.OPT_CHUNK_ROWS) == -1
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64), (n // 2 - 32, seam(3) - 30),
                         (n // 2 - k - 40, 70001), (12345, seam(15) - 10), (99999, n - 3000), (777, seam(8) - 33)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (k, r0, c0)


# ------------------------------------- byte board through the bit board's pair waves
# bytepair_chain_kernel<S> (GOL_OPT_BYTE_CORE = 4): a pack wave (byte rows from
# HBM into 4-word bit groups), S = k / 8 pair waves, an unpack wave, per strip
# of 62 stored 128-column lane units (7936 columns; 63 at the grid edges) with
# the folded tail strip; k = 16, 32, 48.  k = 24 and 56 run the pack and the
# unpack inside the first and last wave, each with 4 pair stages of its own
# (pair_event IN = 2 / OUT = 2); k = 56 runs it whatever the byte core.

PAIR = 4
PAIR_DEPTHS = (16, 24, 32, 48, 56)
PAIR_SHAPES = [(1, 1), (5, 17), (40, 129), (70, 7935), (71, 7936), (66, 8064), (64, 8065), (90, 15872),
               (130, 16001), (33, 4000), (300, 640), (400, 37), (170, 23000), (200, 24525), (100, 32768)]


def run_pair(gh, b0, gens, k, slabs=1, boundary="dead", chunk=None):
    rows, cols = b0.shape
    with gh.Engine(rows, cols, n_gpus=slabs, layout="byte", boundary=boundary, tblock_k=k) as e:
        e.set_option(gh.OPT_BYTE_CORE, PAIR)
        assert e.get_option(gh.OPT_BYTE_CORE) == PAIR
        if chunk is not None:
            e.set_option(gh.OPT_CHUNK_ROWS, chunk)
        e.upload(b0)
        e.step(gens - gens % k)
        if gens % k:
            e.step(gens % k)
        return e.download()


@pytest.mark.parametrize("shape", PAIR_SHAPES)
@pytest.mark.parametrize("boundary", ["dead", "serial_compat"])
def test_pair_chain_random_shapes(gh, shape, boundary):
    rows, cols = shape
    if boundary == "serial_compat" and (rows < 2 or cols < 2):
        return
    rng = np.random.default_rng(rows * 977 + cols)
    b0 = rand_board(rng, rows, cols)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    gens = 110
    ref = g.run(b0, gens, g.DEAD if boundary == "dead" else g.SERIAL_COMPAT)
    for k in PAIR_DEPTHS:
        for slabs in (1, 2, 3):
            if rows // slabs < k or (slabs > 1 and rows < 2 * slabs):
                continue
            d = mismatch(run_pair(gh, b0, gens, k, slabs, boundary), ref)
            assert d is None, (shape, boundary, k, slabs, d)


@pytest.mark.parametrize("chunk", [-1, -2, -3, 8, 37, 256, -104])
def test_pair_chain_chunk_policies(gh, chunk):
    """Every chunk policy, with the folded strip (23000 columns: 3 strips, a
    fold of 2 × 32 lanes) and without (16001: 2 edge strips, 6 units past)."""
    rng = np.random.default_rng(4000 + chunk)
    for cols in (23000, 16001):
        rows = 700
        b0 = rand_board(rng, rows, cols)
        gens = 144
        ref = g.run_dead_fast(b0, gens)
        for k in PAIR_DEPTHS:
            for slabs in (1, 2):
                d = mismatch(run_pair(gh, b0, gens, k, slabs, chunk=chunk), ref)
                assert d is None, (chunk, cols, k, slabs, d)


def test_pair_chain_goldens(gh, golden):
    """The reference's own 1024² boards (serial, mpirun -np 1/4/16) through
    the pair chain at k = 16, 32 and 48."""
    d, cases = golden
    for name, case in cases.items():
        n = case["n"]
        if n < 1024:
            continue
        mode, m = case["mode"], case["mesh_m"]
        init = {"serial_compat": ("serial", g.SERIAL_SEED), "dead": ("stream", 0), "mesh_compat": ("mesh", 0)}[mode]
        for k in PAIR_DEPTHS:
            with gh.Engine(n, n, layout="byte", boundary=mode, mesh_m=m, tblock_k=k) as e:
                e.set_option(gh.OPT_BYTE_CORE, PAIR)
                e.initialize_board(*init)
                done = 0
                for gen in sorted(int(x) for x in case["gens"]):
                    e.step(gen - done)
                    done = gen
                    assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (name, k, gen)


@pytest.mark.parametrize("k", PAIR_DEPTHS)
def test_pair_chain_config2_reference(gh, k):
    """BASELINE config 2 in full (main.cpp under mpirun -np 16, 16384², 1000
    generations) through the pair chain: the reference's whole-board digests."""
    import json
    import os
    case = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "config2.json")))
    n, m = case["n"], case["mesh_m"]
    with gh.Engine(n, n, layout="byte", boundary="mesh_compat", mesh_m=m, tblock_k=k) as e:
        e.set_option(gh.OPT_BYTE_CORE, PAIR)
        e.initialize_board("mesh", 0)
        done = 0
        for gen in sorted(int(x) for x in case["gens"]):
            e.step(gen - done)
            done = gen
            assert g.digest(e.download()) == case["gens"][str(gen)]["sha256"], (k, gen)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("k", PAIR_DEPTHS)
def test_pair_chain_32768_lightcone(gh, k):
    """BASELINE config 3's board (32768², srand(1), dead boundary) through the
    pair chain, one slab, default one-round chunks: windows at the corners,
    strip seams (128·(62s + 1) columns), the folded strip and chunk seams."""
    n, gens = 32768, 2 * k
    seam = lambda s: 128 * (62 * s + 1)
    with gh.Engine(n, n, layout="byte", tblock_k=k) as e:
        e.set_option(gh.OPT_BYTE_CORE, PAIR)
        e.initialize_board("stream", 1)
        e.step(gens)
        for (r0, c0) in [(0, 0), (0, n - 64), (n - 64, 0), (n - 64, n - 64), (n // 2 - 32, seam(1) - 30),
                         (12345, seam(2) - 10), (20001, seam(3) - 33), (n // 3, n - 900), (9000, 128 * 250 - 40)]:
            assert lightcone_check(e, n, n, gens, r0, c0, 64, 64), (k, r0, c0)


def test_pair_chain_option_range(gh):
    """GOL_OPT_BYTE_CORE takes 0..4; 5 is rejected and leaves the setting."""
    with gh.Engine(64, 64, layout="byte", tblock_k=48) as e:
        e.set_option(gh.OPT_BYTE_CORE, PAIR)
        with pytest.raises(Exception):
            e.set_option(gh.OPT_BYTE_CORE, 5)
        assert e.get_option(gh.OPT_BYTE_CORE) == PAIR
