"""The persistent bit kernel (GOL_OPT_PERSISTENT, the single-slab default).

All full k-steps of one gol_step run in ONE launch: each wave owns a (chunk,
strip) item for every step and starts step t when the 8 neighbouring items
have published step t-1 (write-through stores, per-item flags, agent-scope
acquire).  Checked bit-exactly against the oracle on shapes where neighbour
items sit on different XCDs (many short chunks), with a short last block, and
against the one-launch-per-step path at 16384².
"""
import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


SHAPES = [(2048, 2048), (1000, 4099), (300, 9000), (97, 1000), (64, 130), (3000, 640)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_persistent_matches_oracle(gh, shape, k):
    rows, cols = shape
    rng = np.random.default_rng(rows * 31 + cols + k)
    b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
    gens = 9 * k + k // 2   # nine fused steps in one launch, then a short block
    with gh.Engine(rows, cols, layout="bit", tblock_k=k) as e:
        assert e.get_option(gh.OPT_PERSISTENT) == 1
        e.upload(b0)
        e.step(gens)
        got = e.download()
    assert (got == g.run_dead_fast(b0, gens)).all(), (shape, k)


@pytest.mark.parametrize("boundary", ["serial_compat", "dead"])
def test_persistent_boundaries_and_repeated_calls(gh, boundary):
    rows, cols = 1500, 3100
    rng = np.random.default_rng(7)
    b0 = (rng.random((rows, cols)) < 0.4).astype(np.uint8)
    if boundary == "serial_compat":
        b0[-1, :] = 0
        b0[:, -1] = 0
    mode = g.SERIAL_COMPAT if boundary == "serial_compat" else g.DEAD
    with gh.Engine(rows, cols, layout="bit", boundary=boundary, tblock_k=8) as e:
        e.upload(b0)
        done = 0
        for gens in (16, 40, 7, 64):   # several persistent launches on one context
            e.step(gens)
            done += gens
        got = e.download()
    assert (got == g.run(b0, done, mode)).all()


def test_persistent_vs_stepwise_16384(gh):
    n, k, gens = 16384, 8, 400
    outs = []
    for persist in (1, 0):
        with gh.Engine(n, n, layout="bit", tblock_k=k) as e:
            e.set_option(gh.OPT_PERSISTENT, persist)
            e.initialize_board("stream", 1)
            e.step(gens)
            outs.append((e.popcount(), e.download()))
    assert outs[0][0] == outs[1][0]
    assert (outs[0][1] == outs[1][1]).all()
    win = g.lightcone(n, n, gens, 8190, 8000, 48, 48)
    assert (outs[0][1][8190:8238, 8000:8048] == win).all()
