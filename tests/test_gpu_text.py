"""GPU tests of the snapshot text path: the `.gol` part-file body
of main.cpp:106-129 formatted and parsed on the device (gol_text.hip) and
streamed through pinned buffers (gol_runtime.cpp text_io).

The expected text is built here with numpy from the same cells the engine
holds (downloaded through gol_download_window) — the byte format is the one
`std::ostream_iterator<bool>(f, "\\t")` + `std::endl` produces and
gol_visualization.py:29-33 reads back.  Small GOL_TEXT_BLOCK_BYTES values force
many pipelined blocks so the double-buffering is exercised on small grids.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import golcpu as g

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "mpi_amd", "bin", "gol")


@pytest.fixture(scope="module")
def gh():
    from mpi_amd import golhip
    golhip.load()
    return golhip


def body(cells: np.ndarray) -> bytes:
    n, m = cells.shape
    out = np.empty((n, 2 * m + 1), np.uint8)
    out[:, 0:2 * m:2] = cells + ord("0")
    out[:, 1:2 * m:2] = ord("\t")
    out[:, -1] = ord("\n")
    return out.tobytes()


def rand_board(rng, rows, cols, p=0.4):
    return (rng.random((rows, cols)) < p).astype(np.uint8)


LAYOUTS = ["bit", "byte"]


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("slabs", [1, 3])
@pytest.mark.parametrize("block", [None, 1, 1000])
def test_format_matches_reference_text(gh, layout, slabs, block):
    rng = np.random.default_rng(7)
    rows, cols = 67, 389
    b = rand_board(rng, rows, cols)
    with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, tblock_k=2) as e:
        if block is not None:
            e.set_option(gh.OPT_TEXT_BLOCK_BYTES, block)
        e.upload(b)
        e.step(5)
        ref = g.run(b, 5, g.DEAD)
        assert e.format_text(0, 0, rows, cols) == body(ref)
        for (r0, c0, nr, nc) in [(5, 37, 40, 200), (66, 388, 1, 1), (0, 127, 67, 130), (22, 0, 23, 389)]:
            assert e.format_text(r0, c0, nr, nc) == body(ref[r0:r0 + nr, c0:c0 + nc]), (r0, c0, nr, nc)


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("slabs", [1, 2])
def test_parse_roundtrip_and_continue(gh, layout, slabs):
    rng = np.random.default_rng(11)
    rows, cols = 150, 301
    b = rand_board(rng, rows, cols)
    with gh.Engine(rows, cols, n_gpus=slabs, layout=layout, tblock_k=3) as e:
        e.set_option(gh.OPT_TEXT_BLOCK_BYTES, 3000)
        e.parse_text(0, 0, rows, cols, body(b))
        assert (e.download() == b).all()
        # window parse into an existing board, then the generations continue from it
        w = rand_board(rng, 70, 99)
        e.parse_text(40, 130, 70, 99, body(w))
        b2 = b.copy()
        b2[40:110, 130:229] = w
        assert (e.download() == b2).all()
        e.step(7)
        assert (e.download() == g.run(b2, 7, g.DEAD)).all()


def test_parse_serial_compat_keeps_last_row_and_column_dead(gh):
    rng = np.random.default_rng(3)
    n = 64
    b = rand_board(rng, n, n, 0.6)
    with gh.Engine(n, n, boundary="serial_compat", layout="bit") as e:
        e.parse_text(0, 0, n, n, body(b))
        got = e.download()
        want = b.copy()
        want[-1, :] = 0
        want[:, -1] = 0
        assert (got == want).all()
        e.step(9)
        assert (e.download() == g.run(want, 9, g.SERIAL_COMPAT)).all()


@pytest.mark.parametrize("layout", ["bit", "byte"])
def test_parse_rejects_malformed_text(gh, layout):
    rows, cols = 10, 20
    good = bytearray(body(np.zeros((rows, cols), np.uint8)))
    with gh.Engine(rows, cols, layout=layout) as e:
        with pytest.raises(gh.GolError) as ex:
            e.parse_text(0, 0, rows, cols, bytes(good[:-1]))           # length mismatch
        assert ex.value.code == -1
        bad = bytearray(good)
        bad[3 * 41 + 2 * 7 + 1] = ord(" ")                              # row 3, column 7 separator
        bad[5 * 41 + 2 * 2] = ord("2")                                   # row 5, column 2 value
        with pytest.raises(gh.GolError, match=r"byte 138 \(row 3, column 7"):
            e.parse_text(0, 0, rows, cols, bytes(bad))
        bad = bytearray(good)
        bad[9 * 41 + 40] = ord("\t")                                     # last newline
        with pytest.raises(gh.GolError, match="byte 409"):
            e.parse_text(0, 0, rows, cols, bytes(bad))


def test_save_and_load_part_files(gh, tmp_path):
    rng = np.random.default_rng(5)
    rows, cols = 200, 333
    b = rand_board(rng, rows, cols)
    with gh.Engine(rows, cols, n_gpus=2, layout="bit", tblock_k=4) as e:
        e.set_option(gh.OPT_TEXT_BLOCK_BYTES, 5000)
        e.upload(b)
        e.save_part(str(tmp_path / "p0.gol"), 0, 120)                             # main.cpp header
        e.save_part(str(tmp_path / "p1.gol"), 120, 80, header=(120, 200, 0, 333))  # main_serial header
        lines = open(tmp_path / "p0.gol").read().splitlines()
        assert lines[:2] == ["0 119", "0 332"]
        assert (np.array([[int(t) for t in ln.split()] for ln in lines[2:]]) == b[:120]).all()
    with gh.Engine(rows, cols, n_gpus=1, layout="byte") as e2:
        assert e2.load_part(str(tmp_path / "p0.gol")) == (0, 0, 120, 333)
        assert e2.load_part(str(tmp_path / "p1.gol")) == (120, 0, 80, 333)
        assert (e2.download() == b).all()


def test_format_at_baseline_width(gh):
    """Full 131072-column rows across a slab seam (2 slabs) after 8 fused generations."""
    rows, cols = 4096, 131072
    with gh.Engine(rows, cols, n_gpus=2, layout="bit", tblock_k=8) as e:
        e.initialize_board("stream", 1)
        e.step(8)
        r0 = rows // 2 - 3
        got = e.format_text(r0, 0, 6, cols)
        assert got == body(e.download_window(r0, 0, 6, cols))
        # parse it back one row lower on a fresh engine
        with gh.Engine(rows, cols, layout="bit") as f:
            f.parse_text(r0 + 1, 0, 6, cols, got)
            assert f.popcount() == got.count(b"1")
            assert (f.download_window(r0 + 1, 0, 6, cols) == e.download_window(r0, 0, 6, cols)).all()


def _run(args, cwd):
    return subprocess.run([EXE] + args, cwd=cwd, check=True, capture_output=True, text=True)


def _main_name(d):
    return [f for f in os.listdir(d) if f.endswith(".gol") and "_" not in f][0][:-4]


@pytest.mark.parametrize("mode,extra,n", [("dead", ["--gpus", "2", "-k", "3"], 96),
                                          ("serial", [], 64),
                                          ("mpi", ["--procs", "4", "--gpus", "2"], 64)])
def test_driver_resume_reproduces_the_run(gh, tmp_path, mode, extra, n):
    """Run 0..20 saving every 5; resume the same run from iteration 10 and
    check that iterations 15 and 20 are rewritten byte-identically."""
    a = tmp_path / "a"
    a.mkdir()
    _run(["--mode", mode, "--save"] + extra + [str(n), str(n), "5", "20"], a)
    name = _main_name(a)
    b = tmp_path / "b"
    shutil.copytree(a, b)
    for it in (15, 20):
        for p in range(2):
            f = b / f"{name}_{it}_{p}.gol"
            if f.exists():
                f.unlink()
    _run(["--mode", mode, "--save"] + extra + ["--resume", name, "--from", "10"], b)
    for it in (15, 20):
        for p in range(2 if "--gpus" in extra else 1):
            assert open(b / f"{name}_{it}_{p}.gol", "rb").read() == open(a / f"{name}_{it}_{p}.gol", "rb").read()
