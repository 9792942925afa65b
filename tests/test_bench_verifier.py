"""bench.py's self-check (life_cpu: a bit-parallel host stepper independent of
the device kernels and of oracle/) against the oracle, and its light-cone
window geometry.  CPU only."""
import numpy as np
import pytest

import bench
from oracle import golcpu as g


@pytest.mark.parametrize("shape", [(1, 1), (5, 63), (7, 64), (9, 65), (40, 130), (77, 200), (64, 1000)])
def test_life_cpu_matches_oracle(shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    b = (rng.random(shape) < 0.4).astype(np.uint8)
    for gens in (0, 1, 7):
        assert (bench.life_cpu(b, gens) == g.run(b, gens, g.DEAD)).all(), (shape, gens)


class _FakeEngine:
    """download_window over a host board (stands in for the GPU in this test)."""

    def __init__(self, board):
        self.b = board

    def download_window(self, r0, c0, h, w):
        return self.b[r0:r0 + h, c0:c0 + w].copy()


@pytest.mark.parametrize("r0,c0", [(0, 0), (50, 60), (170, 230), (95, 0)])
def test_lightcone_window(r0, c0):
    rng = np.random.default_rng(r0 + c0)
    rows, cols, gens = 200, 300, 12
    b0 = (rng.random((rows, cols)) < 0.35).astype(np.uint8)
    v = bench.Verifier(_FakeEngine(b0), rows, cols, r0, c0, gens, h=30, w=40)
    assert v.check(_FakeEngine(g.run(b0, gens, g.DEAD)))["ok"]
    bad = g.run(b0, gens, g.DEAD)
    bad[r0 + 3, c0 + 5] ^= 1
    assert not v.check(_FakeEngine(bad))["ok"]
