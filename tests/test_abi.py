"""CPU checks of the C ABI boundary: libgolhip.so loads, exports every entry
point include/golhip.h declares, and its host-only logic (slab plan, error
paths) behaves — no GPU needed, no compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "golhip.h")


@pytest.fixture(scope="module")
def lib():
    from mpi_amd import golhip
    if not os.path.exists(golhip.LIB_PATH):
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "mpi_amd"), "libgolhip.so"], check=True)
    return golhip.load()


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gol_\w+)\s*\(", text, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for n in ["gol_create", "gol_create_rank", "gol_init_glibc", "gol_upload", "gol_step", "gol_sync",
              "gol_download", "gol_popcount", "gol_last_error", "gol_destroy"]:
        assert n in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "mpi_amd", "libgolhip.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(gol_\w+)", out))
    assert set(declared()) <= exported


def test_binding_covers_header(lib):
    from mpi_amd import golhip
    assert set(golhip.EXPORTS) == set(declared())


def test_library_is_gfx950_code(lib):
    from mpi_amd import golhip
    assert "gfx950" in golhip.version()
    blob = open(os.path.join(ROOT, "mpi_amd", "libgolhip.so"), "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("rows,world", [(1, 1), (7, 3), (131072, 8), (1048576, 8), (1000, 7), (10, 10)])
def test_slab_plan_partitions_rows(lib, rows, world):
    from mpi_amd import golhip
    nxt = 0
    sizes = []
    for r in range(world):
        r0, n = golhip.slab_plan(rows, world, r)
        assert r0 == nxt and n >= 1
        nxt += n
        sizes.append(n)
    assert nxt == rows and max(sizes) - min(sizes) <= 1


def test_slab_plan_rejects_bad_args(lib):
    r0, n = ctypes.c_int64(), ctypes.c_int64()
    assert lib.gol_slab_plan(10, 0, 0, ctypes.byref(r0), ctypes.byref(n)) == -1
    assert lib.gol_slab_plan(10, 2, 2, ctypes.byref(r0), ctypes.byref(n)) == -1
    assert lib.gol_slab_plan(0, 1, 0, ctypes.byref(r0), ctypes.byref(n)) == -1


def test_create_validates_before_touching_a_device(lib):
    p = ctypes.c_void_p()
    # invalid arguments are rejected with EINVAL / EUNSUPPORTED on any host
    assert lib.gol_create(ctypes.byref(p), 0, 10, 1, 1, 0, 1, 1) == -1
    assert lib.gol_create(ctypes.byref(p), 10, 10, 1, 7, 0, 1, 1) == -1          # bad layout
    assert lib.gol_create(ctypes.byref(p), 10, 10, 1, 1, 0, 1, 9) == -1          # k > 8
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 1, 0, 1, 12) == -1         # bit layout: k <= 8, 16, 32
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 1, 0, 1, 24) == -1
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 1, 0, 1, 64) == -1
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 0, 1, 10) == -1         # byte: k in 1..8, 12, 16
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 0, 1, 17) == -1
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 0, 1, 36) == -1
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 0, 1, 40) == -1         # byte: chains at 48, 56, 64 only
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 0, 1, 72) == -1
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 0, 2, 3, 4) == -1          # mesh: cols % m != 0
    assert lib.gol_create(ctypes.byref(p), 64, 64, 1, 1, 2, 0, 4) == -1          # mesh: m < 1
    assert lib.gol_create(ctypes.byref(p), 12, 64, 4, 1, 0, 1, 8) == -1          # slabs thinner than k
    assert lib.gol_create(ctypes.byref(p), 16, 1 << 25, 1, 0, 0, 1, 1) == -5     # rows too wide (byte)
    assert lib.gol_create(ctypes.byref(p), 16, (1 << 31) - 64, 1, 1, 0, 1, 8) == -5   # rows too wide (bit)
    assert not p.value


def test_no_silent_fallback_without_gpu(lib):
    """Without a visible GPU the engine refuses to run (there is no CPU path)."""
    from mpi_amd import golhip
    try:
        import torch
        has_gpu = torch.cuda.device_count() > 0
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU visible")
    with pytest.raises(golhip.GolError) as e:
        golhip.Engine(64, 64)
    assert e.value.code == -2


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    from mpi_amd import golhip
    monkeypatch.setattr(golhip, "_lib", None)
    monkeypatch.setattr(golhip, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="missing"):
        golhip.load()


def test_driver_usage_message():
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    if not os.path.exists(exe):
        pytest.skip("driver not built")
    r = subprocess.run([exe, "1", "2"], capture_output=True, text=True)
    assert r.returncode == 1 and "four arguments" in r.stdout
    r = subprocess.run([exe, "--procs", "3", "9", "9", "1", "1"], capture_output=True, text=True,
                       cwd="/tmp")
    assert r.returncode == 1 and "Illegal board size" in r.stdout


def test_text_bytes_and_part_geometry(lib, tmp_path):
    from mpi_amd import golhip
    assert lib.gol_text_bytes(3, 5) == 33 and lib.gol_text_bytes(0, 7) == 0
    assert lib.gol_text_bytes(-1, 5) == -1
    p = tmp_path / "x_0_1.gol"
    p.write_bytes(b"12 13\n4 6\n" + b"0\t1\t0\t\n1\t1\t1\t\n")
    assert golhip.part_geometry(str(p)) == (12, 4, 2, 3, 10)
    p.write_bytes(b"0 2\n0 3\n" + b"0\t1\t0\t\n1\t1\t")
    with pytest.raises(golhip.GolError):
        golhip.part_geometry(str(p))


def test_driver_resume_needs_from(tmp_path):
    exe = os.path.join(ROOT, "mpi_amd", "bin", "gol")
    if not os.path.exists(exe):
        pytest.skip("driver not built")
    (tmp_path / "run.gol").write_text("32 32 5 10 1\n")
    r = subprocess.run([exe, "--resume", "run"], capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 1 and "--from" in r.stdout
    r = subprocess.run([exe, "--resume", "nope", "--from", "5"], capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 1 and "main .gol" in r.stdout
