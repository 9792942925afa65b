"""CPU oracle bindings — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product package
``mpi_amd`` never imports it.

Wraps ``oracle/libgolcpu.so`` (``oracle/golcpu.c``, a plain-C restatement of
main.cpp:68-103 / main_serial.cpp:34-71 and glibc's TYPE_3 ``rand``).  Boards are
``numpy.uint8`` arrays of 0/1, row-major, shape (rows, cols).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

DEAD, SERIAL_COMPAT, MESH_COMPAT = 0, 1, 2
SERIAL_SEED = 1804289383  # first glibc rand() with no srand (main_serial.cpp:150)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libgolcpu.so")
_lib = None


def build() -> str:
    """Compile libgolcpu.so (gcc, seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE, "libgolcpu.so"], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(
            os.path.join(_HERE, "golcpu.c")
        ):
            build()
        L = ctypes.CDLL(_LIB)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i64, u32, u64 = ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
        L.gol_oracle_rand_seq.argtypes = [u32, i64, ctypes.POINTER(ctypes.c_int32)]
        L.gol_oracle_stream_cells.argtypes = [u32, u64, i64, u8p]
        L.gol_oracle_init_stream.argtypes = [u8p, i64, i64, u32, u64]
        L.gol_oracle_init_serial.argtypes = [u8p, i64]
        L.gol_oracle_init_mesh.argtypes = [u8p, i64, ctypes.c_int]
        for f in ("gol_oracle_step_dead", "gol_oracle_step_serial"):
            getattr(L, f).argtypes = [u8p, u8p, i64, i64]
        L.gol_oracle_step_mesh.argtypes = [u8p, u8p, i64, i64, ctypes.c_int]
        L.gol_oracle_run.argtypes = [u8p, i64, i64, ctypes.c_int, ctypes.c_int, i64]
        L.gol_oracle_run.restype = ctypes.c_int
        L.gol_oracle_run_dead_fast.argtypes = [u8p, i64, i64, i64]
        L.gol_oracle_run_dead_fast.restype = ctypes.c_int
        L.gol_oracle_run_mesh_fast.argtypes = [u8p, i64, i64, ctypes.c_int, i64]
        L.gol_oracle_run_mesh_fast.restype = ctypes.c_int
        L.gol_oracle_ref_shaped_run.argtypes = [i64, i64, u32]
        L.gol_oracle_ref_shaped_run.restype = i64
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def rand_seq(seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.int32)
    lib().gol_oracle_rand_seq(seed, count, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def stream_cells(seed: int, offset: int, count: int) -> np.ndarray:
    out = np.empty(count, np.uint8)
    lib().gol_oracle_stream_cells(seed, offset, count, _p(out))
    return out


def init_dead(rows: int, cols: int, seed: int = 1, row0: int = 0, full_cols: int | None = None,
              col0: int = 0) -> np.ndarray:
    """Rows [row0,row0+rows) × cols [col0,col0+cols) of the srand(seed) row-major
    grid of width ``full_cols`` (MPI np=1 convention; srand(0) ≡ srand(1))."""
    fc = cols if full_cols is None else full_cols
    out = np.empty((rows, cols), np.uint8)
    if col0 == 0 and fc == cols:
        lib().gol_oracle_init_stream(_p(out), rows, cols, seed, row0 * fc)
    else:
        for i in range(rows):
            out[i] = stream_cells(seed, (row0 + i) * fc + col0, cols)
    return out


def init_serial(n: int) -> np.ndarray:
    out = np.empty((n, n), np.uint8)
    lib().gol_oracle_init_serial(_p(out), n)
    return out


def init_mesh(n: int, m: int) -> np.ndarray:
    out = np.empty((n, n), np.uint8)
    lib().gol_oracle_init_mesh(_p(out), n, m)
    return out


def run(board: np.ndarray, gens: int, mode: int = DEAD, mesh_m: int = 1) -> np.ndarray:
    b = np.ascontiguousarray(board, dtype=np.uint8).copy()
    rc = lib().gol_oracle_run(_p(b), b.shape[0], b.shape[1], mode, mesh_m, gens)
    if rc != 0:
        raise ValueError(f"gol_oracle_run rc={rc}")
    return b


def run_dead_fast(board: np.ndarray, gens: int) -> np.ndarray:
    """DEAD generations on zero-padded buffers (same rule as run(..., DEAD); the
    long light-cone windows of the full-size GPU tests).  Releases the GIL."""
    b = np.ascontiguousarray(board, dtype=np.uint8).copy()
    rc = lib().gol_oracle_run_dead_fast(_p(b), b.shape[0], b.shape[1], gens)
    if rc != 0:
        raise MemoryError("gol_oracle_run_dead_fast")
    return b


def run_mesh_fast(board: np.ndarray, gens: int, m: int) -> np.ndarray:
    """MESH_COMPAT(m) generations with main.cpp's per-block ghost columns
    (same result as run(..., MESH_COMPAT, m), for large boards)."""
    b = np.ascontiguousarray(board, dtype=np.uint8).copy()
    rc = lib().gol_oracle_run_mesh_fast(_p(b), b.shape[0], b.shape[1], m, gens)
    if rc != 0:
        raise ValueError(f"gol_oracle_run_mesh_fast rc={rc}")
    return b


def lightcone(rows: int, cols: int, gens: int, r0: int, c0: int, h: int, w: int, seed: int = 1) -> np.ndarray:
    """Window [r0,r0+h)×[c0,c0+w) of generation `gens` of the srand(seed)
    row-major dead-boundary grid rows×cols: the oracle run on the generation-0
    window grown by `gens` cells (clipped at the grid edge, which is dead; at a
    cut edge the error moves inward one cell per generation and never reaches
    the window)."""
    R0, C0 = max(0, r0 - gens), max(0, c0 - gens)
    R1, C1 = min(rows, r0 + h + gens), min(cols, c0 + w + gens)
    b0 = init_dead(R1 - R0, C1 - C0, seed, row0=R0, full_cols=cols, col0=C0)
    return run_dead_fast(b0, gens)[r0 - R0:r0 - R0 + h, c0 - C0:c0 - C0 + w]


def ref_shaped_run(L: int, gens: int, seed: int = 1) -> int:
    return lib().gol_oracle_ref_shaped_run(L, gens, seed)


def text_body(board: np.ndarray) -> bytes:
    """The `.gol` part-file body writeBoardToFile writes (main.cpp:117-124):
    "v\t" per cell, "\n" per row."""
    n, m = board.shape
    out = np.empty((n, 2 * m + 1), np.uint8)
    out[:, 0:2 * m:2] = (board != 0) + ord("0")
    out[:, 1:2 * m:2] = ord("\t")
    out[:, -1] = ord("\n")
    return out.tobytes()


def packbits(board: np.ndarray) -> bytes:
    """np.packbits(MSB-first, row-major) — the fixture format of tests/golden."""
    return np.packbits(board.astype(np.uint8).ravel()).tobytes()


def unpack(data: bytes, rows: int, cols: int) -> np.ndarray:
    bits = np.unpackbits(np.frombuffer(data, np.uint8))[: rows * cols]
    return bits.reshape(rows, cols).astype(np.uint8)


def digest(board: np.ndarray) -> str:
    return hashlib.sha256(packbits(board)).hexdigest()
