"""ctypes binding of ``libgolhip.so`` (the C ABI declared in ``include/golhip.h``).

Host-side mirror of the reference's hot-path interface.  The reference is a
C++ program whose generation loop (main.cpp:291-305) calls

    updateBoard(board, board2, options)      main.cpp:93-103  -> Engine.update_board / step
    swap(board, board2)                      main.cpp:294-296 -> ping-pong inside the context
    distr_borders(board, nbr, comm, options) main.cpp:36-65   -> halo exchange inside step
    initializeBoard(board, options, rank)    main.cpp:68-77   -> Engine.initialize_board

This module never computes a generation itself: every call goes to the HIP
library, and importing it on a machine without ``libgolhip.so`` raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LAYOUT = {"byte": 0, "bit": 1}
BOUNDARY = {"dead": 0, "serial_compat": 1, "mesh_compat": 2}
INIT = {"stream": 0, "serial": 1, "mesh": 2}
SERIAL_SEED = 1804289383

OPT_CHUNK_ROWS = 1
OPT_KERNEL_TIMING = 2
OPT_OVERLAP = 4
OPT_BYTE_CORE = 5
OPT_TEXT_BLOCK_BYTES = 10
OPT_SCHEDULE_TRIAL = 11
OPT_INTERIOR_SPLIT = 12
OPT_SCHED_TRACE = 13
OPT_COMM_TIMING = 14
OPT_HALO_EXCHANGE = 15
# retired in 0.2 (accepted by gol_set_option as no-ops; kept so old callers still run)
OPT_WORDS_PER_LANE = 3
OPT_SPLIT = 6

ERRORS = {0: "OK", -1: "EINVAL", -2: "EHIP", -3: "ERCCL", -4: "ENOMEM", -5: "EUNSUPPORTED", -6: "ESTATE"}

EXPORTS = [
    "gol_create", "gol_create_rank", "gol_get_unique_id", "gol_slab_plan", "gol_set_option", "gol_get_option",
    "gol_init_glibc", "gol_upload", "gol_upload_window", "gol_step", "gol_sync", "gol_download",
    "gol_download_window", "gol_popcount", "gol_generation", "gol_kernel_time", "gol_last_error",
    "gol_destroy", "gol_version", "gol_text_bytes", "gol_format_text", "gol_write_text", "gol_parse_text",
    "gol_read_text", "gol_download_window_async", "gol_clock_start", "gol_clock_stop", "gol_rccl_selftest",
    "gol_sched_trace", "gol_comm_time",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GOL_LIB") or os.path.join(_HERE, "libgolhip.so")
_lib = None


class GolError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def load() -> ctypes.CDLL:
    """Load libgolhip.so; raise if it was not built (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C mpi_amd` or __graft_entry__.build()"
        )
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    i64, i32, u32 = ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i64p = ctypes.POINTER(ctypes.c_int64)
    dp = ctypes.POINTER(ctypes.c_double)
    sig = {
        "gol_create": ([ctypes.POINTER(P), i64, i64, i32, i32, i32, i32, i32], i32),
        "gol_create_rank": ([ctypes.POINTER(P), i64, i64, i32, i32, i32, u8p, i32, i32, i32, i32], i32),
        "gol_get_unique_id": ([u8p], i32),
        "gol_slab_plan": ([i64, i32, i32, i64p, i64p], i32),
        "gol_set_option": ([P, i32, i64], i32),
        "gol_get_option": ([P, i32, i64p], i32),
        "gol_init_glibc": ([P, i32, u32], i32),
        "gol_upload": ([P, u8p, i64], i32),
        "gol_upload_window": ([P, i64, i64, i64, i64, u8p, i64], i32),
        "gol_step": ([P, i64], i32),
        "gol_sync": ([P, dp], i32),
        "gol_download": ([P, u8p, i64], i32),
        "gol_download_window": ([P, i64, i64, i64, i64, u8p, i64], i32),
        "gol_popcount": ([P, i64p], i32),
        "gol_generation": ([P, i64p], i32),
        "gol_kernel_time": ([P, dp, i64p, i32], i32),
        "gol_comm_time": ([P, dp, dp, i64p, i32], i32),
        "gol_sched_trace": ([P, i64p, i64, i64p], i32),
        "gol_last_error": ([P], ctypes.c_char_p),
        "gol_destroy": ([P], None),
        "gol_version": ([], ctypes.c_char_p),
        "gol_text_bytes": ([i64, i64], i64),
        "gol_format_text": ([P, i64, i64, i64, i64, ctypes.c_char_p, i64], i32),
        "gol_write_text": ([P, i64, i64, i64, i64, i32], i32),
        "gol_parse_text": ([P, i64, i64, i64, i64, ctypes.c_char_p, i64], i32),
        "gol_read_text": ([P, i64, i64, i64, i64, i32], i32),
        "gol_download_window_async": ([P, i64, i64, i64, i64, u8p, i64], i32),
        "gol_clock_start": ([P, ctypes.c_double], i32),
        "gol_clock_stop": ([P, dp, dp], i32),
        "gol_rccl_selftest": ([i32, i64, i32, dp, ctypes.c_char_p, i32], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def version() -> str:
    return load().gol_version().decode()


def slab_plan(rows: int, world: int, rank: int) -> tuple[int, int]:
    """Row range (row0, nrows) of slab `rank` of `world` (host-only, no GPU)."""
    r0, n = ctypes.c_int64(), ctypes.c_int64()
    rc = load().gol_slab_plan(rows, world, rank, ctypes.byref(r0), ctypes.byref(n))
    if rc:
        raise GolError(rc, "gol_slab_plan")
    return r0.value, n.value


def unique_id() -> bytes:
    """RCCL bootstrap blob (rank 0 creates it, the caller broadcasts it)."""
    buf = (ctypes.c_uint8 * 128)()
    rc = load().gol_get_unique_id(buf)
    if rc:
        raise GolError(rc, "gol_get_unique_id (RCCL unavailable?)")
    return bytes(buf)


def rccl_selftest(device: int = 0, nbytes: int = 8 * 16896, reps: int = 20) -> tuple[float, str]:
    """Real RCCL through the library's own binding: a 1-rank communicator sends
    two halo-sized messages to itself per group, `reps` groups; raises on any
    error or byte mismatch.  Returns (device µs per group, message)."""
    us = ctypes.c_double()
    msg = ctypes.create_string_buffer(512)
    rc = load().gol_rccl_selftest(device, nbytes, reps, ctypes.byref(us), msg, len(msg))
    if rc:
        raise GolError(rc, msg.value.decode())
    return us.value, msg.value.decode()


def part_geometry(path: str) -> tuple[int, int, int, int, int]:
    """(row0, col0, nrows, ncols, body_offset) of a `.gol` part file: origin from
    the two header lines, shape from the body (main.cpp:106-129 layout)."""
    with open(path, "rb") as f:
        l1, l2 = f.readline(), f.readline()
        off = f.tell()
        first = f.readline()
        size = os.fstat(f.fileno()).st_size
    row0, col0 = int(l1.split()[0]), int(l2.split()[0])
    if not first.endswith(b"\n") or len(first) % 2 == 0:
        raise GolError(-1, f"{path}: malformed first body row")
    rowlen = len(first)
    if (size - off) % rowlen:
        raise GolError(-1, f"{path}: body of {size - off} bytes is not a whole number of {rowlen}-byte rows")
    return row0, col0, (size - off) // rowlen, (rowlen - 1) // 2, off


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class Engine:
    """One Game-of-Life board on the GPU(s).

    Single process: ``Engine(rows, cols, n_gpus=N)`` cuts the grid into N row
    slabs (slab s on device s % visible).  One process per GPU:
    ``Engine(rows, cols, rank=r, world=W, device=d, uid=blob)``.
    """

    def __init__(self, rows: int, cols: int, *, n_gpus: int = 1, layout: str = "bit",
                 boundary: str = "dead", mesh_m: int = 1, tblock_k: int = 1,
                 rank: int | None = None, world: int | None = None, device: int = 0,
                 uid: bytes | None = None):
        self.lib = load()
        self._pending = []   # arrays the library fills at the next synchronising call
        self.rows, self.cols = rows, cols
        self.layout, self.boundary, self.tblock_k = layout, boundary, tblock_k
        self._c = ctypes.c_void_p()
        if rank is None:
            rc = self.lib.gol_create(ctypes.byref(self._c), rows, cols, n_gpus, LAYOUT[layout],
                                     BOUNDARY[boundary], mesh_m, tblock_k)
            self.rank, self.world = 0, 1
        else:
            u = None
            if uid is not None:
                u = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
            rc = self.lib.gol_create_rank(ctypes.byref(self._c), rows, cols, rank, world, device, u,
                                          LAYOUT[layout], BOUNDARY[boundary], mesh_m, tblock_k)
            self.rank, self.world = rank, world
        if rc:
            raise GolError(rc, "gol_create failed (see stderr)")

    # ------------------------------------------------------------ plumbing
    def _chk(self, rc: int, what: str):
        if rc:
            raise GolError(rc, f"{what}: {self.lib.gol_last_error(self._c).decode()}")

    def close(self):
        if self._c:
            self.lib.gol_destroy(self._c)
            self._c = ctypes.c_void_p()
        self._pending = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, opt: int, value: int):
        self._chk(self.lib.gol_set_option(self._c, opt, value), "gol_set_option")

    def get_option(self, opt: int) -> int:
        v = ctypes.c_int64()
        self._chk(self.lib.gol_get_option(self._c, opt, ctypes.byref(v)), "gol_get_option")
        return v.value

    # ------------------------------------------------------------ board state
    def initialize_board(self, mode: str = "stream", seed: int = 1):
        """initializeBoard (main.cpp:68-77 / main_serial.cpp:34-43), on device."""
        self._chk(self.lib.gol_init_glibc(self._c, INIT[mode], seed), "gol_init_glibc")

    def upload(self, board: np.ndarray):
        b = np.ascontiguousarray(board != 0, dtype=np.uint8)   # bool cells (main.cpp:73)
        assert b.shape == (self.rows, self.cols)
        self._chk(self.lib.gol_upload(self._c, _u8(b), b.shape[1]), "gol_upload")

    def upload_window(self, row0: int, col0: int, win: np.ndarray):
        w = np.ascontiguousarray(win != 0, dtype=np.uint8)
        self._chk(self.lib.gol_upload_window(self._c, row0, col0, w.shape[0], w.shape[1], _u8(w),
                                             w.shape[1]), "gol_upload_window")

    def download(self) -> np.ndarray:
        out = np.zeros((self.rows, self.cols), np.uint8)
        self._chk(self.lib.gol_download(self._c, _u8(out), self.cols), "gol_download")
        return out

    def download_window(self, row0: int, col0: int, nrows: int, ncols: int) -> np.ndarray:
        out = np.zeros((nrows, ncols), np.uint8)
        self._chk(self.lib.gol_download_window(self._c, row0, col0, nrows, ncols, _u8(out), ncols),
                  "gol_download_window")
        return out

    def download_window_async(self, row0: int, col0: int, nrows: int, ncols: int) -> np.ndarray:
        """Enqueue a copy of the window behind the steps enqueued so far; the
        returned array is filled by the next synchronising call (sync, popcount,
        download...).  Keep it alive until then."""
        out = np.zeros((nrows, ncols), np.uint8)
        self._chk(self.lib.gol_download_window_async(self._c, row0, col0, nrows, ncols, _u8(out), ncols),
                  "gol_download_window_async")
        self._pending.append(out)   # kept alive here until a synchronising call has filled it
        return out

    def clock_start(self, max_ms: float):
        """Start the clock probe (one wave on its own stream, stops by itself after max_ms)."""
        self._chk(self.lib.gol_clock_start(self._c, max_ms), "gol_clock_start")

    def clock_stop(self) -> tuple[float, float]:
        """(shader clock in MHz, span in ms) over the probe's lifetime."""
        mhz, span = ctypes.c_double(), ctypes.c_double()
        self._chk(self.lib.gol_clock_stop(self._c, ctypes.byref(mhz), ctypes.byref(span)), "gol_clock_stop")
        return mhz.value, span.value

    # ------------------------------------------------------------ snapshot text
    def format_text(self, row0: int, col0: int, nrows: int, ncols: int) -> bytes:
        """`.gol` part-file body of a window (main.cpp:106-129), formatted on the device."""
        n = self.lib.gol_text_bytes(nrows, ncols)
        buf = ctypes.create_string_buffer(max(n, 1))
        self._chk(self.lib.gol_format_text(self._c, row0, col0, nrows, ncols, buf, n), "gol_format_text")
        return buf.raw[:n]

    def parse_text(self, row0: int, col0: int, nrows: int, ncols: int, text: bytes):
        """Inverse of format_text: load a window from `.gol` body text (snapshot resume)."""
        self._chk(self.lib.gol_parse_text(self._c, row0, col0, nrows, ncols, text, len(text)), "gol_parse_text")

    def save_part(self, path: str, row0: int, nrows: int, *, col0: int = 0, ncols: int | None = None,
                  header: tuple[int, int, int, int] | None = None):
        """Write one part file: the two header lines (default: inclusive ranges,
        main.cpp:255-258) and the device-formatted body, streamed to the fd."""
        ncols = self.cols - col0 if ncols is None else ncols
        h = header or (row0, row0 + nrows - 1, col0, col0 + ncols - 1)
        with open(path, "wb") as f:
            f.write(f"{h[0]} {h[1]}\n{h[2]} {h[3]}\n".encode())
            f.flush()
            self._chk(self.lib.gol_write_text(self._c, row0, col0, nrows, ncols, f.fileno()), "gol_write_text")

    def load_part(self, path: str) -> tuple[int, int, int, int]:
        """Read one part file back (either header convention): the window's
        origin is the header's first row / column, its shape comes from the
        body (row length and byte count).  Returns (row0, col0, nrows, ncols)."""
        row0, col0, nrows, ncols, off = part_geometry(path)
        fd = os.open(path, os.O_RDONLY)
        try:
            os.lseek(fd, off, os.SEEK_SET)
            self._chk(self.lib.gol_read_text(self._c, row0, col0, nrows, ncols, fd), "gol_read_text")
        finally:
            os.close(fd)
        return row0, col0, nrows, ncols

    # ------------------------------------------------------------ hot path
    def step(self, generations: int = 1):
        """updateBoard + swap + distr_borders, `generations` times (async)."""
        self._chk(self.lib.gol_step(self._c, generations), "gol_step")

    update_board = step

    def sync(self) -> float:
        ms = ctypes.c_double()
        self._chk(self.lib.gol_sync(self._c, ctypes.byref(ms)), "gol_sync")
        self._pending = []
        return ms.value

    def popcount(self) -> int:
        v = ctypes.c_int64()
        self._chk(self.lib.gol_popcount(self._c, ctypes.byref(v)), "gol_popcount")
        self._pending = []
        return v.value

    @property
    def generation(self) -> int:
        v = ctypes.c_int64()
        self._chk(self.lib.gol_generation(self._c, ctypes.byref(v)), "gol_generation")
        return v.value

    def sched_trace(self):
        """The recorded schedule (GOL_OPT_SCHED_TRACE) as an (n, 7) int64 array
        (kind, stream, event, slab, buffer, row0, row1); clears the record."""
        n = ctypes.c_int64()
        self._chk(self.lib.gol_sched_trace(self._c, None, 0, ctypes.byref(n)), "gol_sched_trace")
        out = np.zeros((n.value, 7), np.int64)
        self._chk(self.lib.gol_sched_trace(self._c, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n.value,
                                           ctypes.byref(n)), "gol_sched_trace")
        return out

    def comm_time(self, reset: bool = False) -> tuple[float, float, int]:
        """(exchange ms, bands ms, k-steps) of the comm stream (GOL_OPT_COMM_TIMING)."""
        ex, bd, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        self._chk(self.lib.gol_comm_time(self._c, ctypes.byref(ex), ctypes.byref(bd), ctypes.byref(n), int(reset)),
                  "gol_comm_time")
        self._pending = []
        return ex.value, bd.value, n.value

    def kernel_time(self, reset: bool = False) -> tuple[float, int]:
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._chk(self.lib.gol_kernel_time(self._c, ctypes.byref(ms), ctypes.byref(n), int(reset)),
                  "gol_kernel_time")
        self._pending = []
        return ms.value, n.value
