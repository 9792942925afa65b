"""mpi_amd — MI355X-native Game-of-Life engine (the hot path of arthurdecloedt/mpi).

The compute lives in ``libgolhip.so`` (hand-written gfx950 HIP kernels behind
the C ABI of ``include/golhip.h``); ``bin/gol`` is the reference-compatible C++
driver.  This package only binds the library (``mpi_amd.golhip``) and builds it.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 4) -> None:
    """Compile libgolhip.so and bin/gol for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", HERE, "all"], check=True)


from .golhip import Engine, GolError, load, slab_plan, unique_id, version  # noqa: E402,F401
