// gol_runtime.cpp — the C ABI (include/golhip.h) over the gfx950 kernels.
//
// Replaces the reference's per-rank runtime (main.cpp:149-369): the MPI
// Cartesian mesh becomes row slabs (one per GPU, or several per GPU for
// testing), distr_borders (main.cpp:36-65) becomes a k-row halo exchange
// (RCCL send/recv between processes, or hipMemcpyAsync between slabs of one
// process), the per-generation MPI_Barrier (main.cpp:297) becomes stream/event
// ordering, and updateBoard (main.cpp:93-103) becomes the pipelined kernels of
// gol_kernels.hip fusing k generations per launch.
//
// Per slab and per k-generation step t (cur = buf[t%2], nxt = buf[(t+1)%2]):
//   comm stream : exchange halos of cur  ->  boundary-band kernel (cur -> nxt)
//   comp stream : interior kernel (cur -> nxt), rows whose light cone is local
// so the exchange and the boundary bands hide under the interior kernel.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <errno.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/golhip.h"
#include "glibc_jump.h"
#include "gol_internal.h"

using namespace gol;

// ------------------------------------------------------------------ RCCL (dlopen)
// RCCL is bound at run time so the library loads (and its CPU-side entry
// points work) on hosts without it, and so that a process that already holds
// a librccl.so.1 (e.g. torch's) shares that one copy.
namespace {
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    const char *source = "";   // "global scope" or the path dlopen'ed
};

RcclApi load_rccl();

// Resolved once per process; rank contexts created from several threads at once
// (the one-GPU rank rehearsals) all see the finished table.
RcclApi &rccl() {
    static RcclApi api = load_rccl();
    return api;
}

RcclApi load_rccl() {
    RcclApi api;
    // (RTLD_DEFAULT is a null handle, so "found in the global scope" needs its own flag)
    void *h = RTLD_DEFAULT;
    const bool global = dlsym(RTLD_DEFAULT, "ncclGetUniqueId") != nullptr;
    api.source = "global scope";
    if (!global) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL), api.source = "librccl.so.1";
    if (!global && !h)
        h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL), api.source = "/opt/rocm/lib/librccl.so.1";
    if (!global && !h) {
        api.err = std::string("cannot load librccl.so.1: ") + (dlerror() ? dlerror() : "?");
        return api;
    }
#define GOL_SYM(field, name)                                                 \
    api.field = reinterpret_cast<decltype(api.field)>(dlsym(h, name));       \
    if (!api.field) {                                                        \
        api.err = std::string("librccl lacks ") + name;                      \
        return api;                                                          \
    }
    GOL_SYM(GetUniqueId, "ncclGetUniqueId")
    GOL_SYM(CommInitRank, "ncclCommInitRank")
    GOL_SYM(Send, "ncclSend")
    GOL_SYM(Recv, "ncclRecv")
    GOL_SYM(GroupStart, "ncclGroupStart")
    GOL_SYM(GroupEnd, "ncclGroupEnd")
    GOL_SYM(AllReduce, "ncclAllReduce")
    GOL_SYM(CommDestroy, "ncclCommDestroy")
    GOL_SYM(GetErrorString, "ncclGetErrorString")
#undef GOL_SYM
    api.ok = true;
    return api;
}
} // namespace

// ------------------------------------------------------------------ context

namespace {
constexpr int kMaxParts = 4;   // GOL_OPT_INTERIOR_SPLIT's largest value

struct Slab {
    int index = 0;       // global slab id
    int device = 0;
    int64_t row0 = 0, H = 0; // global rows [row0, row0+H)
    int row_lo = 0, row_hi = 0; // storage rows outside are dead
    void *buf[2] = {nullptr, nullptr};
    unsigned long long *d_count = nullptr;
    hipStream_t comp = nullptr, comm = nullptr;
    // GOL_OPT_INTERIOR_SPLIT = P >= 2: interior parts 1 .. P-1 run on streams of their own
    // (part 0 on comp); nx = how many such streams exist (created on first use)
    hipStream_t part[kMaxParts - 1] = {};
    int nx = 0;
    hipEvent_t ev_bnd[2] = {}, ev_int[2] = {}, ev_exch[2] = {};
    hipEvent_t ev_part[kMaxParts - 1][2] = {};   // ... and their completion per step parity
    hipEvent_t ev_join[kMaxParts - 1] = {};      // ... join them into another stream
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    // GOL_OPT_COMM_TIMING: per k-step, timing events on the comm stream around the
    // halo exchange (0 -> 1) and around the boundary and seam bands (2 -> 3); a
    // ring of kCommRing steps, the oldest harvested (long complete) when reused
    std::vector<std::array<hipEvent_t, 4>> comm_ev;
    size_t comm_head = 0, comm_live = 0, comm_cur = 0;
    double comm_exch_ms = 0.0, comm_band_ms = 0.0;
    int64_t comm_steps = 0;
};

struct TimedLaunch {
    hipEvent_t a, b;
    int device;   // the events' device (several slabs may sit on several devices)
};

// A window copy enqueued by gol_download_window_async: device staging ->
// pinned host staging on the slab's streams; the pinned rows reach the
// caller's buffer at the next synchronising call.
// Staging buffers are pooled per context (device + pinned pairs, reused by
// size): hipMalloc / hipHostMalloc / hipFree can wait for the whole device, so
// after the first copy of a given size none of them runs on the way to a
// timed region.
struct Staging {
    int device = 0;
    size_t bytes = 0;
    uint8_t *dtmp = nullptr;   // device staging (bit layout: unpacked bytes)
    uint8_t *pinned = nullptr;
    bool busy = false;
};
struct PendingWindow {
    size_t stage = 0;          // index into gol_ctx::staging
    uint8_t *host = nullptr;   // caller's rows, leading dimension ld
    int64_t ld = 0, nrows = 0, ncols = 0;
};

// The schedule trial of the k=8 bit kernel (see tune_slot).
// (2-word groups: six rounds are the default; 4-word groups: guided, 4 rounds;
// the first candidate is the default, see common_create)
constexpr int kTuneCandG2[3] = {-6, -3, -103};
constexpr int kTuneCandG4[3] = {-104, -6, -3};
// k = 8 with the split interior (GOL_OPT_INTERIOR_SPLIT = 2, the default for a
// k = 8 context of at most kSplitSlabsPerDevice slabs per device): one round of
// equal chunks per half-launch — 147.1-148.5 k against 138.3 k unsplit at the
// guided default; two rounds tie on one box and lose 1.6 % on another, three lose
// 0.8 % (profiles/r05l_bit_sweep.jsonl, r05t_cut_ab.jsonl; the trial's margin for
// these candidates: kTuneMarginSplit).  Halves of 35/42/58 % lose 1.5-5 % against 50 %.
constexpr int kTuneCandSplit[3] = {-1, -2, -3};
constexpr int kSplitChunk = -1;
constexpr int kSplitParts = 2;   // the default GOL_OPT_INTERIOR_SPLIT of such a context
// a split slab holds three streams (halves + seam/halo); more slabs per device than
// this would share hardware queues (GPU_MAX_HW_QUEUES) and already fill each
// other's launch tails (8 slabs on one GPU: profiles/r05f_slab_probe.jsonl)
constexpr int kSplitSlabsPerDevice = 4;
const int *tune_cand(const gol_ctx *c);
// Starts past the DVFS ramp of a GPU that idled (≈0.25 s of k=8 steps: 1.97 ->
// 2.38 GHz, bench.py clock.settle_blocks_mhz, profiles/r03e_steps.jsonl).
constexpr int kTuneStart = 400, kTuneRounds = 8, kTuneN = 3 * kTuneRounds;
// A candidate replaces the default only when its median step is this much
// shorter (the default won on 7 of 8 boxes in round 2; a noisy pick of the
// guided schedule cost 5 % once in r03e).
constexpr double kTuneMargin = 0.985;
// Under the split interior -1 won or tied on every box measured in round 5
// (tune.py and slab_probe: 0-1.6 % over -2, more over -3), while the trial's
// 24-step medians kept -2 on two of six bench runs, 2-4.5 % slower per clock
// on the headline (profiles/r05u_bench_driver_cmd.json, r05af_driver_2.json):
// its noise exceeds the candidates' spread, so another policy must be clearly faster.
constexpr double kTuneMarginSplit = 0.96;
// RCCL mode: the ranks agree on one policy (ncclAllReduce MAX of the three
// medians) at a fixed k-step after the trial's last one — the same step on
// every rank, so the collective sits at the same place in every rank's
// sequence of communicator operations.  The host blocks there for the trial's
// marks, which completed ~this many steps of queued work earlier.
constexpr int kTuneAgreeAfter = 16;
// Timed launches kept in flight at most (GOL_OPT_KERNEL_TIMING): a ring, the
// oldest pair is harvested (long complete by then) when it is reused.
constexpr size_t kTimedRing = 1024;
// GOL_OPT_COMM_TIMING: k-steps of comm-stream event quads kept in flight per slab.
constexpr size_t kCommRing = 256;
} // namespace

struct gol_ctx {
    int64_t rows = 0, cols = 0;
    int layout = GOL_LAYOUT_BIT, boundary = GOL_DEAD, mesh_m = 1, K = 1;
    int hk = 1;                  // halo rows per side (= K)
    int nslabs = 1;              // total slabs (all processes)
    int transport = GOL_XPORT_NONE;
    int rank = 0, world = 1;     // RCCL mode
    ncclComm_t comm = nullptr;
    int64_t active_rows = 0, active_cols = 0;
    int perm_m = 1;              // MESH_COMPAT: column blocks stored in reverse order (see validate)
    int64_t perm_L = 0;          // columns per block
    int64_t pitch_bytes = 0;     // row pitch
    int64_t row_bytes = 0;       // bytes per row that may hold cells
    int nunits = 0;              // stencil units (bit words / byte dwords) per row
    int gw = 2;                  // bit layout: words per column group (bit_group_words(K))
    uint32_t last_mask = 0;
    int chunk_rows = 256;
    bool overlap = true;
    int split = 1;               // interior launches per slab and step (GOL_OPT_INTERIOR_SPLIT)
    int byte_core = kByteCoreDefault;   // byte layout: bit-sliced core where k allows (GOL_OPT_BYTE_CORE)
    bool timing = false;
    bool comm_timing = false;    // GOL_OPT_COMM_TIMING
    bool halo_exchange = true;   // GOL_OPT_HALO_EXCHANGE (0: diagnostic, the exchange is skipped)
    int64_t text_block_bytes = 64LL << 20;   // snapshot text staging block (GOL_OPT_TEXT_BLOCK_BYTES)
    std::vector<Slab> slabs;     // slabs held by this context
    int cur = 0;                 // parity of the buffer holding the current generation
    int64_t generation = 0;
    int64_t step_index = 0;      // k-steps enqueued (event ring parity)
    int last_k = 0;              // generations of the previous k-step (0: none yet)
    bool batch_open = false;
    std::vector<TimedLaunch> timed;   // ring of kTimedRing event pairs
    size_t timed_head = 0;       // oldest pair not yet harvested
    size_t timed_live = 0;       // pairs recorded and not yet harvested
    int64_t launch_count = 0;    // main-kernel launches (counted on the host, timing or not)
    // schedule trial of the k=8 bit kernel (see tune_slot): candidate chunk
    // policies take turns on real steps, the fastest median stays
    bool chunk_user = false;     // GOL_OPT_CHUNK_ROWS set by the caller: no trial
    int user_chunk = 0;          // ... its value (RCCL mode: applied at the agreement step if set mid-trial)
    bool trial_enabled = true;   // GOL_OPT_SCHEDULE_TRIAL
    bool trial_committed = false; // RCCL mode: this rank started recording; it runs the trial (and its
                                  // restarts) to the agreement whatever its own options say
    int tune_phase = 0;          // 0 not started, 1 recording, 2 waiting for the events, 3 done
    int tune_n = 0;              // trial steps recorded
    int tune_default = -6;       // policy in force until the trial's result is known
    const int *trial_cand = nullptr;   // the candidates the trial's slots time (frozen when recording
    double trial_margin = 1.0;         // starts, with its margin: see tune_before)
    std::vector<hipEvent_t> tune_ev;   // per slab: kTuneN + 1 step-end marks on the compute stream
    int64_t tune_agree_step = -1;      // RCCL mode: k-step at which the ranks agree (phase 2)
    double *agree_dev = nullptr;       // RCCL mode: 3 medians, device (ncclAllReduce MAX) ...
    double *agree_host = nullptr;      // ... and pinned host copy
    std::vector<PendingWindow> pending;
    std::vector<Staging> staging;
    std::vector<size_t> release_at_sync;   // staging of a failed async copy: busy until the next sync
    // clock probe (gol_clock_start / gol_clock_stop)
    hipStream_t clk_stream = nullptr;
    unsigned long long *clk_out = nullptr;   // device: memtime0, realtime0, memtime1, realtime1
    int *clk_stop = nullptr;                  // pinned host flag the probe polls
    int clk_device = 0;
    bool clk_running = false;
    double timed_ms = 0.0;
    int64_t timed_count = 0;
    // GOL_OPT_SCHED_TRACE: the enqueue order of every event record/wait, host sync
    // and board access of the step path (gol_sched_trace; tests/sched_race.py)
    bool tracing = false;
    bool trace_full = false;      // the record hit kTraceMaxOps: later ops were dropped
    std::vector<int64_t> trace;   // kTraceFields per op
    std::string err;
};

namespace {
// Schedule trace: op = {kind, stream, object, slab, buffer, row0, row1}.  A
// record/wait names the event as object; a board access names (slab, buffer)
// and storage rows [row0, row1) (every column).  Untraced calls behave the same.
constexpr int kTraceFields = 7;
constexpr size_t kTraceMaxOps = size_t(1) << 22;   // 224 MiB of record at most
enum { TR_RECORD = 1, TR_WAIT = 2, TR_STREAM_SYNC = 3, TR_EVENT_SYNC = 4, TR_READ = 5, TR_WRITE = 6 };

void tr_op(gol_ctx *c, int kind, const void *st, const void *obj, int64_t slab = -1, int64_t buf = -1,
           int64_t r0 = 0, int64_t r1 = 0) {
    if (!c->tracing || c->trace_full) return;
    if (c->trace.size() >= kTraceMaxOps * kTraceFields) {
        c->trace_full = true;
        return;
    }
    const int64_t v[kTraceFields] = {kind, (int64_t)(intptr_t)st, (int64_t)(intptr_t)obj, slab, buf, r0, r1};
    c->trace.insert(c->trace.end(), v, v + kTraceFields);
}
hipError_t tr_record(gol_ctx *c, hipEvent_t e, hipStream_t st) {
    tr_op(c, TR_RECORD, st, e);
    return hipEventRecord(e, st);
}
hipError_t tr_wait(gol_ctx *c, hipStream_t st, hipEvent_t e) {
    tr_op(c, TR_WAIT, st, e);
    return hipStreamWaitEvent(st, e, 0);
}
hipError_t tr_ssync(gol_ctx *c, hipStream_t st) {
    tr_op(c, TR_STREAM_SYNC, st, nullptr);
    return hipStreamSynchronize(st);
}
hipError_t tr_esync(gol_ctx *c, hipEvent_t e) {
    tr_op(c, TR_EVENT_SYNC, nullptr, e);
    return hipEventSynchronize(e);
}
}  // namespace

namespace {
int fail(gol_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(c, expr)                                                                    \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail((c), GOL_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
    } while (0)

#define NCCLCHK(c, expr)                                                                   \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess)                                                             \
            return fail((c), GOL_ERCCL, "%s failed: %s", #expr, rccl().GetErrorString(r_)); \
    } while (0)

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Storage column of logical column lc (MESH_COMPAT: reversed column blocks).
int64_t phys_col(const gol_ctx *c, int64_t lc) {
    if (c->perm_m <= 1) return lc;
    const int64_t cy = lc / c->perm_L;
    return (c->perm_m - 1 - cy) * c->perm_L + (lc - cy * c->perm_L);
}

// fn(lc, pc, n) for every maximal run of the logical columns [col0, col0+ncols)
// that is contiguous in storage (one run unless MESH_COMPAT); stops at an error.
template <typename F>
int for_col_runs(const gol_ctx *c, int64_t col0, int64_t ncols, F &&fn) {
    for (int64_t lc = col0; lc < col0 + ncols;) {
        int64_t n = col0 + ncols - lc;
        if (c->perm_m > 1) n = std::min(n, (lc / c->perm_L + 1) * c->perm_L - lc);
        const int rc = fn(lc, phys_col(c, lc), n);
        if (rc) return rc;
        lc += n;
    }
    return GOL_OK;
}

void slab_plan(int64_t rows, int world, int rank, int64_t *row0, int64_t *nrows) {
    const int64_t base = rows / world, rem = rows % world;
    *row0 = rank * base + std::min<int64_t>(rank, rem);
    *nrows = base + (rank < rem ? 1 : 0);
}

int64_t storage_rows(const gol_ctx *c, const Slab &s) { return s.H + 2 * c->hk; }

int validate(gol_ctx *c, int64_t rows, int64_t cols, int nslabs, int layout, int boundary, int mesh_m,
             int k) {
    if (rows < 1 || cols < 1) return fail(c, GOL_EINVAL, "rows/cols must be positive");
    if (rows > (1LL << 30) || cols > (1LL << 31) - 64) return fail(c, GOL_EINVAL, "grid too large");
    if (layout != GOL_LAYOUT_BIT && layout != GOL_LAYOUT_BYTE) return fail(c, GOL_EINVAL, "bad layout");
    if (boundary < GOL_DEAD || boundary > GOL_MESH_COMPAT) return fail(c, GOL_EINVAL, "bad boundary");
    if (k < 1 || (k > 8 && !(layout == GOL_LAYOUT_BYTE ? bytebit_supported(k) : bit_depth_supported(k))))
        return fail(c, GOL_EINVAL,
                    "tblock_k must be in [1,8] (bit layout: also 16 or 32; byte layout: also 12, 16, 20, 24, 28, 32, "
                    "48 or 64)");
    if (nslabs < 1) return fail(c, GOL_EINVAL, "need at least one slab");
    // MESH_COMPAT(m) is main.cpp on an m×m mesh: column block cy's left ghost
    // column holds the LAST column of block cy+1 and its right ghost the FIRST
    // column of block cy-1 (the swapped halos of main.cpp:51-54), rows are
    // exchanged normally.  Stored with its column blocks in reverse order
    // (block cy at m-1-cy), those wires are plain adjacency: the board is an
    // ordinary dead-boundary board, so every kernel (bit or byte, any k) runs
    // it unchanged and only the I/O paths map columns (phys_col).
    if (boundary == GOL_MESH_COMPAT && (mesh_m < 1 || cols % mesh_m != 0))
        return fail(c, GOL_EINVAL, "MESH_COMPAT needs cols %% mesh_m == 0");
    if (boundary == GOL_SERIAL_COMPAT && (rows < 2 || cols < 2))
        return fail(c, GOL_EINVAL, "SERIAL_COMPAT needs rows, cols >= 2");
    // every wave's buffer window (>= 2k+8 rows) must stay far below the kernels'
    // out-of-range offset (2^30 B): rows of at most ~2^29/(2k+8) bytes
    const int64_t row_b = layout == GOL_LAYOUT_BIT ? (cols + 31) / 32 * 4 : cols;
    if (row_b * (2 * k + 8) >= (1LL << 28))
        return fail(c, GOL_EUNSUPPORTED, "rows of %lld bytes are too wide for tblock_k=%d", (long long)row_b, k);
    const int64_t hmin = rows / nslabs;
    if (nslabs > 1 && hmin < k)
        return fail(c, GOL_EINVAL, "slabs of %lld rows are thinner than tblock_k=%d", (long long)hmin, k);
    return GOL_OK;
}

// Row pitch = the row rounded up to 256 B plus a pad.  Power-of-two pitches
// (131072 bit columns = 16 KiB, 16384/32768 byte columns) put the same column
// of every row on the same HBM channels; the pad spreads them.  Interleaved
// A/B over pads 0-2048 B (profiles/r02k_pad_sweep*.jsonl, r02l_*pad*.jsonl):
// bit +128 B: +5.5 % at k=1, +6 % at k=2 (the 8-B-per-lane row loads);
// byte +512 B: +2 % at 32768 k=1, equal at 16384 (+128 B loses 13 % there:
// 16-B-per-lane loads prefer a different pad); the VALU-bound k=8 bit and
// k=28 byte kernels are unchanged.  DESIGN.md §3.
constexpr int64_t kPitchPadBit = 128, kPitchPadByte = 512;

void set_geometry(gol_ctx *c) {
    c->active_rows = c->boundary == GOL_SERIAL_COMPAT ? c->rows - 1 : c->rows;
    c->active_cols = c->boundary == GOL_SERIAL_COMPAT ? c->cols - 1 : c->cols;
    if (c->layout == GOL_LAYOUT_BIT) {
        // 64-column groups of 2 words, rows padded to 128-column blocks (gol_internal.h)
        const int64_t words = (c->cols + 127) / 128 * 4;
        c->pitch_bytes = round_up(words, 64) * 4 + kPitchPadBit;
        c->row_bytes = words * 4;
        c->nunits = (int)((c->active_cols + 127) / 128 * 4);
        c->last_mask = 0;
    } else {
        const int64_t dws = (c->cols + 3) / 4;
        c->pitch_bytes = round_up(dws, 64) * 4 + kPitchPadByte;
        c->row_bytes = dws * 4;
        c->nunits = (int)((c->active_cols + 3) / 4);
        const int rem = (int)(c->active_cols % 4);
        static const uint32_t m[4] = {0x01010101u, 0x00000001u, 0x00000101u, 0x00010101u};
        c->last_mask = m[rem];
    }
}

int alloc_slab(gol_ctx *c, Slab &s) {
    HIPCHK(c, hipSetDevice(s.device));
    const size_t bytes = (size_t)storage_rows(c, s) * c->pitch_bytes;
    for (int i = 0; i < 2; ++i) HIPCHK(c, hipMalloc(&s.buf[i], bytes));
    HIPCHK(c, hipMalloc(&s.d_count, sizeof(unsigned long long)));
    HIPCHK(c, hipStreamCreateWithFlags(&s.comp, hipStreamNonBlocking));
    // Zero both boards ON the slab's own stream and wait for it: the slab's
    // streams are non-blocking, so a null-stream hipMemset (asynchronous for
    // device memory) is not ordered before their work — a late fill could land
    // on top of the first upload (GPUTEST_r04: test_mesh_random[byte-1026-3]).
    for (int i = 0; i < 2; ++i) HIPCHK(c, hipMemsetAsync(s.buf[i], 0, bytes, s.comp));
    HIPCHK(c, tr_ssync(c, s.comp));
    if (c->nslabs == 1) {
        // one slab has no halo path: one stream.  (A process gets few hardware
        // queues — GPU_MAX_HW_QUEUES, 4 by default — and streams beyond them
        // share one: work queued behind a long kernel of another stream waits
        // for it, e.g. behind the clock probe.)
        s.comm = s.comp;
    } else {
        // the halo path (exchange + boundary bands) gates the next interior kernel:
        // its stream gets the device's highest priority, so its small kernels take
        // CU slots as the running interior kernel frees them
        int prio_lo = 0, prio_hi = 0;
        HIPCHK(c, hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        HIPCHK(c, hipStreamCreateWithPriority(&s.comm, hipStreamNonBlocking, prio_hi));
    }
    for (int i = 0; i < 2; ++i) {
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_bnd[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_int[i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_exch[i], hipEventDisableTiming));
    }
    HIPCHK(c, hipEventCreate(&s.ev_start));
    HIPCHK(c, hipEventCreate(&s.ev_stop));
    const bool top = s.index == 0, bottom = s.index == c->nslabs - 1;
    s.row_lo = top ? c->hk : 0;
    s.row_hi = (int)(c->hk + s.H + (bottom ? 0 : c->hk));
    if (bottom && c->boundary == GOL_SERIAL_COMPAT) s.row_hi -= 1;   // global row rows-1 is dead
    return GOL_OK;
}

void free_slab(Slab &s) {
    (void)hipSetDevice(s.device);
    for (int i = 0; i < 2; ++i) {
        if (s.buf[i]) (void)hipFree(s.buf[i]);
        if (s.ev_bnd[i]) (void)hipEventDestroy(s.ev_bnd[i]);
        if (s.ev_int[i]) (void)hipEventDestroy(s.ev_int[i]);
        for (int j = 0; j < kMaxParts - 1; ++j)
            if (s.ev_part[j][i]) (void)hipEventDestroy(s.ev_part[j][i]);
        if (s.ev_exch[i]) (void)hipEventDestroy(s.ev_exch[i]);
    }
    if (s.d_count) (void)hipFree(s.d_count);
    if (s.ev_start) (void)hipEventDestroy(s.ev_start);
    if (s.ev_stop) (void)hipEventDestroy(s.ev_stop);
    for (auto &q : s.comm_ev)
        for (hipEvent_t e : q) (void)hipEventDestroy(e);
    for (int j = 0; j < kMaxParts - 1; ++j)
        if (s.ev_join[j]) (void)hipEventDestroy(s.ev_join[j]);
    for (int j = 0; j < s.nx; ++j) (void)hipStreamDestroy(s.part[j]);
    if (s.comm && s.comm != s.comp) (void)hipStreamDestroy(s.comm);
    if (s.comp) (void)hipStreamDestroy(s.comp);
}

Slab *find_slab(gol_ctx *c, int index) {
    for (auto &s : c->slabs)
        if (s.index == index) return &s;
    return nullptr;
}

// Make `st` wait for everything enqueued so far on slab s's interior-part
// streams (GOL_OPT_INTERIOR_SPLIT >= 2; nothing to do without them).
int join_parts(gol_ctx *c, Slab &s, hipStream_t st) {
    for (int j = 0; j < s.nx; ++j) {
        HIPCHK(c, tr_record(c, s.ev_join[j], s.part[j]));
        HIPCHK(c, tr_wait(c, st, s.ev_join[j]));
    }
    return GOL_OK;
}

// `st` waits for slab s's interior work of step parity q (every part when split)
int wait_interior(gol_ctx *c, Slab &s, hipStream_t st, int q) {
    HIPCHK(c, tr_wait(c, st, s.ev_int[q]));
    for (int j = 0; j < s.nx; ++j) HIPCHK(c, tr_wait(c, st, s.ev_part[j][q]));
    return GOL_OK;
}

// Streams and events for an interior split into `parts` (created on first use,
// after a sync; never removed while the slab lives).
int enable_split(gol_ctx *c, Slab &s, int parts) {
    HIPCHK(c, hipSetDevice(s.device));
    int prio_lo = 0, prio_hi = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    if (s.comm == s.comp)   // a single slab's seam bands need a stream of their own
        HIPCHK(c, hipStreamCreateWithPriority(&s.comm, hipStreamNonBlocking, prio_hi));
    for (; s.nx < parts - 1; ++s.nx) {
        const int j = s.nx;
        for (int i = 0; i < 2; ++i)
            HIPCHK(c, hipEventCreateWithFlags(&s.ev_part[j][i], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_join[j], hipEventDisableTiming));
        // (normal priority: the other parts at high priority tie at -1 and lose 6 % at -2,
        // profiles/r05ab_ppri_ab.jsonl)
        HIPCHK(c, hipStreamCreateWithFlags(&s.part[j], hipStreamNonBlocking));
    }
    return GOL_OK;
}

// --------------------------------------------------------------- stencil launch

int launch_stencil(gol_ctx *c, Slab &s, int gens, int r0, int r1, hipStream_t st, bool timed) {
    if (r1 <= r0) return GOL_OK;
    StencilArgs a;
    a.src = s.buf[c->cur];
    a.dst = s.buf[c->cur ^ 1];
    a.pitch = c->pitch_bytes / 4;
    a.nunits = c->nunits;
    a.last_mask = c->last_mask;
    a.active_cols = c->active_cols;
    a.row_lo = s.row_lo;
    a.row_hi = s.row_hi;
    a.out_r0 = r0;
    a.out_r1 = r1;
    a.chunk_rows = c->chunk_rows;
    a.gw = c->gw;
    TimedLaunch *tl = nullptr;
    if (timed) c->launch_count++;
    if (timed && c->timing) {
        if (c->timed_live == kTimedRing) {   // reuse the oldest pair: harvest it first
            TimedLaunch &o = c->timed[c->timed_head];
            HIPCHK(c, tr_esync(c, o.b));
            float ms = 0.f;
            HIPCHK(c, hipEventElapsedTime(&ms, o.a, o.b));
            c->timed_ms += ms;
            c->timed_count++;
            c->timed_head = (c->timed_head + 1) % kTimedRing;
            c->timed_live--;
        }
        const size_t slot = (c->timed_head + c->timed_live) % kTimedRing;
        while (c->timed.size() <= slot) {
            TimedLaunch t;
            HIPCHK(c, hipEventCreate(&t.a));
            HIPCHK(c, hipEventCreate(&t.b));
            t.device = s.device;
            c->timed.push_back(t);
        }
        tl = &c->timed[slot];
        if (tl->device != s.device) {   // the ring wrapped onto a slab of another device: new pair here
            HIPCHK(c, hipSetDevice(tl->device));
            HIPCHK(c, hipEventDestroy(tl->a));
            HIPCHK(c, hipEventDestroy(tl->b));
            HIPCHK(c, hipSetDevice(s.device));
            HIPCHK(c, hipEventCreate(&tl->a));
            HIPCHK(c, hipEventCreate(&tl->b));
            tl->device = s.device;
        }
        c->timed_live++;
        HIPCHK(c, tr_record(c, tl->a, st));
    }
    tr_op(c, TR_READ, st, nullptr, s.index, c->cur, std::max<int64_t>(0, r0 - gens),
          std::min<int64_t>(s.H + 2 * c->hk, (int64_t)r1 + gens));
    tr_op(c, TR_WRITE, st, nullptr, s.index, c->cur ^ 1, r0, r1);
    if (c->layout == GOL_LAYOUT_BIT) {
        HIPCHK(c, launch_bit_pipe(a, gens, st));
    } else {
        if (c->byte_core && bytebit_supported(gens))
            HIPCHK(c, launch_bytebit_pipe(a, gens, st, c->byte_core));
        else
            HIPCHK(c, launch_byte_pipe(a, gens, st));
    }
    if (tl) HIPCHK(c, tr_record(c, tl->b, st));
    return GOL_OK;
}

// GOL_OPT_COMM_TIMING: harvest the oldest event quad of slab s (blocks for it).
int comm_harvest_one(gol_ctx *c, Slab &s) {
    auto &q = s.comm_ev[s.comm_head];
    HIPCHK(c, tr_esync(c, q[3]));
    float a = 0.f, b = 0.f;
    HIPCHK(c, hipEventElapsedTime(&a, q[0], q[1]));
    HIPCHK(c, hipEventElapsedTime(&b, q[2], q[3]));
    s.comm_exch_ms += a;
    s.comm_band_ms += b;
    s.comm_steps++;
    s.comm_head = (s.comm_head + 1) % kCommRing;
    s.comm_live--;
    return GOL_OK;
}
// mark i (0: before the exchange, 1: after it, 2: before the bands, 3: after
// them) of this k-step on slab s's comm stream; mark 0 opens the step's quad
int comm_mark(gol_ctx *c, Slab &s, int i) {
    if (!c->comm_timing) return GOL_OK;
    if (i == 0) {
        if (s.comm_live == kCommRing)
            if (int rc = comm_harvest_one(c, s)) return rc;
        s.comm_cur = (s.comm_head + s.comm_live) % kCommRing;
        while (s.comm_ev.size() <= s.comm_cur) {
            std::array<hipEvent_t, 4> q{};
            for (auto &e : q) HIPCHK(c, hipEventCreate(&e));
            s.comm_ev.push_back(q);
        }
        s.comm_live++;
    }
    HIPCHK(c, tr_record(c, s.comm_ev[s.comm_cur][i], s.comm));
    return GOL_OK;
}

// Halo exchange of `k` rows for every local slab.
//  PEER: each slab pulls its neighbours' edge rows (hipMemcpyAsync on its comm stream).
//  RCCL: ncclSend/ncclRecv pairs with rank±1 inside one group.
// When this step is deeper than the previous one (k > last_k, e.g. a full
// k-step after a short last block), the k edge rows it sends were partly
// written by the previous step's INTERIOR kernel, not only by its boundary
// bands: the sender's interior event joins the dependencies ("grow").
int exchange(gol_ctx *c, Slab &s, int k, int64_t t) {
    const int p = (int)(t & 1), pp = p ^ 1;
    if (!c->halo_exchange) {   // diagnostic (GOL_OPT_HALO_EXCHANGE = 0): no rows move, the halos go stale
        if (c->transport != GOL_XPORT_RCCL) HIPCHK(c, tr_record(c, s.ev_exch[p], s.comm));
        return GOL_OK;
    }
    const bool grow = t > 0 && k > c->last_k;
    uint8_t *cur = static_cast<uint8_t *>(s.buf[c->cur]);
    const size_t rowb = (size_t)c->pitch_bytes;
    const size_t nbytes = (size_t)k * rowb;
    uint8_t *top_halo = cur + (size_t)(c->hk - k) * rowb;           // rows [hk-k, hk)
    uint8_t *bot_halo = cur + (size_t)(c->hk + s.H) * rowb;         // rows [hk+H, hk+H+k)
    uint8_t *top_rows = cur + (size_t)c->hk * rowb;                 // rows [hk, hk+k)
    uint8_t *bot_rows = cur + (size_t)(c->hk + s.H - k) * rowb;     // rows [hk+H-k, hk+H)
    if (c->transport == GOL_XPORT_RCCL) {
        RcclApi &R = rccl();
        if (grow)
            if (int rc = wait_interior(c, s, s.comm, pp)) return rc;
        const int64_t hk = c->hk, H = s.H;
        if (c->rank > 0) {
            tr_op(c, TR_READ, s.comm, nullptr, s.index, c->cur, hk, hk + k);
            tr_op(c, TR_WRITE, s.comm, nullptr, s.index, c->cur, hk - k, hk);
        }
        if (c->rank < c->world - 1) {
            tr_op(c, TR_READ, s.comm, nullptr, s.index, c->cur, hk + H - k, hk + H);
            tr_op(c, TR_WRITE, s.comm, nullptr, s.index, c->cur, hk + H, hk + H + k);
        }
        NCCLCHK(c, R.GroupStart());
        if (c->rank > 0) {
            NCCLCHK(c, R.Send(top_rows, nbytes, ncclUint8, c->rank - 1, c->comm, s.comm));
            NCCLCHK(c, R.Recv(top_halo, nbytes, ncclUint8, c->rank - 1, c->comm, s.comm));
        }
        if (c->rank < c->world - 1) {
            NCCLCHK(c, R.Send(bot_rows, nbytes, ncclUint8, c->rank + 1, c->comm, s.comm));
            NCCLCHK(c, R.Recv(bot_halo, nbytes, ncclUint8, c->rank + 1, c->comm, s.comm));
        }
        NCCLCHK(c, R.GroupEnd());
        return GOL_OK;
    }
    // PEER: pull from neighbours once their previous boundary bands are written
    Slab *up = find_slab(c, s.index - 1), *dn = find_slab(c, s.index + 1);
    if (up) {
        if (t > 0) HIPCHK(c, tr_wait(c, s.comm, up->ev_bnd[pp]));
        if (grow)
            if (int rc = wait_interior(c, *up, s.comm, pp)) return rc;
        const uint8_t *src = static_cast<uint8_t *>(up->buf[c->cur]) + (size_t)(c->hk + up->H - k) * rowb;
        tr_op(c, TR_READ, s.comm, nullptr, up->index, c->cur, c->hk + up->H - k, c->hk + up->H);
        tr_op(c, TR_WRITE, s.comm, nullptr, s.index, c->cur, c->hk - k, c->hk);
        HIPCHK(c, hipMemcpyAsync(top_halo, src, nbytes, hipMemcpyDeviceToDevice, s.comm));
    }
    if (dn) {
        if (t > 0) HIPCHK(c, tr_wait(c, s.comm, dn->ev_bnd[pp]));
        if (grow)
            if (int rc = wait_interior(c, *dn, s.comm, pp)) return rc;
        const uint8_t *src = static_cast<uint8_t *>(dn->buf[c->cur]) + (size_t)c->hk * rowb;
        tr_op(c, TR_READ, s.comm, nullptr, dn->index, c->cur, c->hk, c->hk + k);
        tr_op(c, TR_WRITE, s.comm, nullptr, s.index, c->cur, c->hk + s.H, c->hk + s.H + k);
        HIPCHK(c, hipMemcpyAsync(bot_halo, src, nbytes, hipMemcpyDeviceToDevice, s.comm));
    }
    HIPCHK(c, tr_record(c, s.ev_exch[p], s.comm));
    return GOL_OK;
}

int open_batch(gol_ctx *c) {
    if (c->batch_open) return GOL_OK;
    for (auto &s : c->slabs) {
        HIPCHK(c, hipSetDevice(s.device));
        HIPCHK(c, tr_record(c, s.ev_start, s.comp));
        HIPCHK(c, tr_wait(c, s.comm, s.ev_start));
        for (int j = 0; j < s.nx; ++j) HIPCHK(c, tr_wait(c, s.part[j], s.ev_start));
    }
    c->batch_open = true;
    return GOL_OK;
}

// Schedule trial (bit layout, k = 8, default policy): the best chunk policy
// differs between boxes of the MI355X pool (six equal rounds won on 7 of 8
// boxes by 1-7 %, the guided XCD-banded schedule by 5 % on one:
// DESIGN.md §3), so after kTuneStart k-steps (past the clock ramp of a fresh
// GPU) the candidates take turns on kTuneRounds real steps each — a schedule
// never changes the result — and one beating the default's median by more
// than 1.5 % replaces it.  Every local slab marks the end of each trial step
// on its compute stream (after its interior kernel and its boundary bands);
// a step's time is the largest mark-to-mark interval over the slabs (the step
// period, so concurrent slabs on one device are timed together), and the
// candidate with the fastest median is kept.  The host never waits for it:
// the previous default stays in force until the last marks have completed
// (hipEventQuery at each later step and at every synchronising call).
// RCCL mode: every rank must keep the SAME policy (a rank's own medians include
// waiting for its neighbours' halos, so ranks could otherwise settle on
// different picks): at k-step trial_end + kTuneAgreeAfter each rank blocks for
// its marks, the ranks take the element-wise MAX of their three medians with
// ncclAllReduce on the library's communicator (the slowest rank's step under
// each policy), and all apply the same rule to the same numbers.
// A caller-set GOL_OPT_CHUNK_ROWS, or GOL_OPT_SCHEDULE_TRIAL = 0, turns it off;
// a step that cannot take part (a short k-step) restarts it from the next one.
const int *tune_cand(const gol_ctx *c) {
    return c->split >= 2 ? kTuneCandSplit : (c->gw == 4 ? kTuneCandG4 : kTuneCandG2);
}

bool tune_eligible(const gol_ctx *c, int k) {
    const bool shape = c->layout == GOL_LAYOUT_BIT && c->K == 8 && k == 8;
    // RCCL mode, once recording: only the step shape (collective: every rank steps the
    // same generations) decides, never a rank-local option — every rank must reach
    // the allreduce of tune_agree.  The options apply to what a rank keeps (tune_pick).
    if (c->transport == GOL_XPORT_RCCL && c->trial_committed) return shape;
    return c->trial_enabled && !c->chunk_user && shape;
}

// mark `i` (0 .. kTuneN) on every local slab's compute stream, after step work
// enqueued so far (slab stream `s.comm` carries the boundary bands: joined first)
int tune_mark(gol_ctx *c, int i, int p) {
    const size_t per = kTuneN + 1;
    for (size_t si = 0; si < c->slabs.size(); ++si) {
        Slab &s = c->slabs[si];
        HIPCHK(c, hipSetDevice(s.device));
        if (c->nslabs > 1 || s.nx) HIPCHK(c, tr_wait(c, s.comp, s.ev_bnd[p]));
        if (int rc = join_parts(c, s, s.comp)) return rc;
        HIPCHK(c, tr_record(c, c->tune_ev[si * per + i], s.comp));
    }
    return GOL_OK;
}

// the three candidates' median step times once every mark has completed
// (wait: block for them); *ready = false if they have not (wait == false)
int tune_medians(gol_ctx *c, bool wait, double med[3], bool *ready) {
    *ready = false;
    const size_t per = kTuneN + 1;
    for (size_t si = 0; si < c->slabs.size(); ++si) {
        HIPCHK(c, hipSetDevice(c->slabs[si].device));
        hipEvent_t last = c->tune_ev[si * per + kTuneN];
        if (wait) {
            HIPCHK(c, tr_esync(c, last));
        } else {
            const hipError_t q = hipEventQuery(last);
            if (q == hipErrorNotReady) return GOL_OK;
            HIPCHK(c, q);
        }
    }
    std::vector<double> v[3];
    for (int i = 0; i < kTuneN; ++i) {
        double step = 0.0;
        for (size_t si = 0; si < c->slabs.size(); ++si) {
            float ms = 0.f;
            HIPCHK(c, hipSetDevice(c->slabs[si].device));
            HIPCHK(c, hipEventElapsedTime(&ms, c->tune_ev[si * per + i], c->tune_ev[si * per + i + 1]));
            step = std::max(step, (double)ms);
        }
        v[i % 3].push_back(step);
    }
    for (int j = 0; j < 3; ++j) {
        std::sort(v[j].begin(), v[j].end());
        med[j] = v[j][v[j].size() / 2];
    }
    *ready = true;
    return GOL_OK;
}

// phase 2 -> 3: keep the default unless another candidate's median is shorter by the margin
void tune_pick(gol_ctx *c, const double med[3]) {
    c->tune_phase = 3;
    c->trial_committed = false;
    if (c->chunk_user) {   // the caller set a policy meanwhile: it stays
        c->chunk_rows = c->user_chunk;
        return;
    }
    if (!c->trial_enabled) {   // the caller turned the trial off meanwhile (RCCL mode: after it agreed)
        c->chunk_rows = c->tune_default;
        return;
    }
    const int *cand = c->trial_cand ? c->trial_cand : tune_cand(c);
    if (cand != tune_cand(c)) {   // RCCL mode: this rank changed its split mid-trial; the medians
        c->chunk_rows = c->tune_default;   // time the old candidates: it keeps the new split's default
        return;
    }
    const int best = (int)(std::min_element(med, med + 3) - med);
    int pick = 0;   // cand[0] is the default policy
    for (int j = 0; j < 3; ++j)
        if (cand[j] == c->tune_default) pick = j;
    if (med[best] < c->trial_margin * med[pick]) pick = best;
    c->chunk_rows = cand[pick];
}

// phase 2 -> 3 once every mark has completed (wait: block for them, at a sync).
// RCCL mode decides only at its agreement step (tune_agree), never here.
int tune_poll(gol_ctx *c, bool wait) {
    if (c->tune_phase != 2 || c->transport == GOL_XPORT_RCCL) return GOL_OK;
    double med[3];
    bool ready = false;
    if (int rc = tune_medians(c, wait, med, &ready)) return rc;
    if (ready) tune_pick(c, med);
    return GOL_OK;
}

// RCCL mode, phase 2, at k-step tune_agree_step on every rank: the same pick everywhere
int tune_agree(gol_ctx *c) {
    double med[3];
    bool ready = false;
    if (int rc = tune_medians(c, true, med, &ready)) return rc;
    Slab &s = c->slabs[0];
    HIPCHK(c, hipSetDevice(s.device));
    if (!c->agree_dev) {
        HIPCHK(c, hipMalloc(&c->agree_dev, 3 * sizeof(double)));
        HIPCHK(c, hipHostMalloc(&c->agree_host, 3 * sizeof(double), hipHostMallocDefault));
    }
    memcpy(c->agree_host, med, sizeof med);
    // on the comm stream: behind the previous step's exchange and boundary bands,
    // ahead of this step's exchange — the same place on every rank
    HIPCHK(c, hipMemcpyAsync(c->agree_dev, c->agree_host, sizeof med, hipMemcpyHostToDevice, s.comm));
    NCCLCHK(c, rccl().AllReduce(c->agree_dev, c->agree_dev, 3, ncclFloat64, ncclMax, c->comm, s.comm));
    HIPCHK(c, hipMemcpyAsync(c->agree_host, c->agree_dev, sizeof med, hipMemcpyDeviceToHost, s.comm));
    HIPCHK(c, tr_ssync(c, s.comm));
    memcpy(med, c->agree_host, sizeof med);
    tune_pick(c, med);
    return GOL_OK;
}

// before step t: the trial slot of this step (-1: none); sets its policy
int tune_before(gol_ctx *c, int k, int *slot) {
    *slot = -1;
    if (c->tune_phase == 2) {
        if (c->transport == GOL_XPORT_RCCL)
            return c->step_index == c->tune_agree_step ? tune_agree(c) : GOL_OK;
        return tune_poll(c, false);
    }
    // RCCL mode: once recording, a rank-local option change must not take this rank
    // out of the agreement the other ranks will enter (ncclAllReduce at tune_agree_step
    // would hang): the trial (restarts included) runs on to the agreement, and the
    // option decides only what this rank keeps afterwards (tune_pick, tune_eligible).
    if (c->tune_phase == 1 && !tune_eligible(c, k)) {
        // cut short: by a caller's option (the trial ends; a caller's policy stays) or by
        // a step that cannot take part (a short k-step: start over from the next full one;
        // a short step is collective, so every rank of an RCCL job restarts at it)
        const bool restart = (c->transport == GOL_XPORT_RCCL && c->trial_committed) ||
                             (c->trial_enabled && !c->chunk_user);
        if (!c->chunk_user) c->chunk_rows = c->tune_default;
        c->tune_phase = restart ? 0 : 3;
        if (c->chunk_user && c->tune_phase == 0) c->chunk_rows = c->user_chunk;
        return GOL_OK;
    }
    if (c->tune_phase == 3) return GOL_OK;
    if (c->tune_phase == 0 && (!tune_eligible(c, k) || c->step_index < kTuneStart)) return GOL_OK;
    if (c->tune_phase == 0) {
        if (c->tune_ev.empty()) {
            c->tune_ev.resize(c->slabs.size() * (kTuneN + 1));
            for (size_t si = 0; si < c->slabs.size(); ++si) {
                HIPCHK(c, hipSetDevice(c->slabs[si].device));
                for (int i = 0; i <= kTuneN; ++i) HIPCHK(c, hipEventCreate(&c->tune_ev[si * (kTuneN + 1) + i]));
            }
        }
        if (!c->trial_committed) {   // (a restart keeps the first default and candidates)
            c->tune_default = c->chunk_rows;
            // the slots time this candidate set to the end of the trial: in RCCL mode a
            // rank-local split change mid-trial must not switch the set under the same
            // slot indices (the MAX allreduce would mix its medians into every rank's pick)
            c->trial_cand = tune_cand(c);
            c->trial_margin = c->split >= 2 ? kTuneMarginSplit : kTuneMargin;
        }
        c->tune_n = 0;
        c->tune_phase = 1;
        if (c->transport == GOL_XPORT_RCCL) c->trial_committed = true;
        // mark 0 = the end of the previous step (its parity: the buffers have swapped since)
        if (int rc = tune_mark(c, 0, (int)((c->step_index - 1) & 1))) return rc;
    }
    *slot = c->tune_n;
    c->chunk_rows = c->trial_cand[*slot % 3];
    return GOL_OK;
}

int tune_after(gol_ctx *c, int slot, int p) {
    if (slot < 0) return GOL_OK;
    if (int rc = tune_mark(c, slot + 1, p)) return rc;
    if (++c->tune_n == kTuneN) {
        c->chunk_rows = c->tune_default;
        c->tune_phase = 2;
        c->tune_agree_step = c->step_index + 1 + kTuneAgreeAfter;
    }
    return GOL_OK;
}

int one_step(gol_ctx *c, int k) {
    const int64_t t = c->step_index;
    const int p = (int)(t & 1), pp = p ^ 1;
    const int hk = c->hk;
    int tslot = -1;
    if (int rc = tune_before(c, k, &tslot)) return rc;
    // GOL_OPT_INTERIOR_SPLIT = P >= 2: a slab's interior runs as P launches on P
    // streams (part 0 on comp, part j on s.part[j-1]), cut at rows m_1 < ... <
    // m_{P-1}; the seam band [m_j-k, m_j+k) of each cut runs on the comm stream
    // beside the boundary bands.  A part of step t+1 needs only the seam bands
    // of step t (which need every part of step t-1) and its own part of step t
    // (stream order), so it starts while the other parts of step t drain: the
    // launches fill each other's tails.
    auto nparts = [&](const Slab &s, int lo, int hi) -> int {
        if (c->split < 2 || s.nx < c->split - 1 || !c->overlap) return 1;
        // (the context's depth, not this block's: a short block splits where a full one does)
        int np = c->split;
        while (np > 1 && hi - lo < 32 * c->K * np) --np;
        return np;
    };
    // The interior [lo, hi) in np parts: part j = [cut(j) + k, cut(j+1) - k), the
    // first from lo, the last to hi.  The cuts (and np) come from a range [clo, chi)
    // that does not depend on this block's depth k: a cut that moved between a short
    // block and a full one would let a part read rows the neighbouring part of the
    // previous step writes on another stream, or overwrite rows it still reads.
    auto cut = [](int clo, int chi, int np, int j) { return clo + (int)((int64_t)(chi - clo) * j / np); };
    auto parts = [&](Slab &s, int lo, int hi, int clo, int chi, int np) -> int {
        for (int j = 0; j < np; ++j) {
            hipStream_t st = j == 0 ? s.comp : s.part[j - 1];
            const int a = j == 0 ? lo : cut(clo, chi, np, j) + k;
            const int b = j == np - 1 ? hi : cut(clo, chi, np, j + 1) - k;
            if (t > 0) HIPCHK(c, tr_wait(c, st, s.ev_bnd[pp]));
            if (int rc = launch_stencil(c, s, k, a, b, st, true)) return rc;
            HIPCHK(c, tr_record(c, j == 0 ? s.ev_int[p] : s.ev_part[j - 1][p], st));
        }
        for (int j = np - 1; j < s.nx; ++j)   // streams this slab leaves idle: keep their events current
            HIPCHK(c, tr_record(c, s.ev_part[j][p], s.comp));
        return GOL_OK;
    };
    auto seams = [&](Slab &s, int clo, int chi, int np) -> int {
        for (int j = 1; j < np; ++j) {
            const int m = cut(clo, chi, np, j);
            if (int rc = launch_stencil(c, s, k, m - k, m + k, s.comm, false)) return rc;
        }
        return GOL_OK;
    };
    if (c->nslabs == 1) {
        Slab &s = c->slabs[0];
        HIPCHK(c, hipSetDevice(s.device));
        const int lo = hk, hi = (int)(hk + s.H), np = nparts(s, lo, hi);
        if (np == 1) {
            if (s.nx) {   // a split context stepping whole (a short slab): keep the events current
                if (t > 0) HIPCHK(c, tr_wait(c, s.comp, s.ev_bnd[pp]));
                if (t > 0)
                    if (int rc = wait_interior(c, s, s.comp, pp)) return rc;
            }
            int rc = launch_stencil(c, s, k, lo, hi, s.comp, true);
            if (rc) return rc;
            if (s.nx) {
                HIPCHK(c, tr_record(c, s.ev_int[p], s.comp));
                for (int j = 0; j < s.nx; ++j) HIPCHK(c, tr_record(c, s.ev_part[j][p], s.comp));
                HIPCHK(c, tr_record(c, s.ev_bnd[p], s.comp));
            }
        } else {
            // seam bands on the comm stream: after every part of step t-1
            if (t > 0)
                if (int rc = wait_interior(c, s, s.comm, pp)) return rc;
            if (int rc = seams(s, lo, hi, np)) return rc;
            HIPCHK(c, tr_record(c, s.ev_bnd[p], s.comm));
            // the parts: after the seam bands of step t-1
            if (int rc = parts(s, lo, hi, lo, hi, np)) return rc;
        }
    } else {
        // exchange first for every slab (peer pulls need all neighbours' events of t-1)
        for (auto &s : c->slabs) {
            HIPCHK(c, hipSetDevice(s.device));
            int rc = comm_mark(c, s, 0);
            if (!rc) rc = exchange(c, s, k, t);
            if (!rc) rc = comm_mark(c, s, 1);
            if (rc) return rc;
        }
        for (auto &s : c->slabs) {
            HIPCHK(c, hipSetDevice(s.device));
            const int lo = hk, hi = (int)(hk + s.H);
            const bool thin = s.H <= 2 * k;
            // boundary bands on the comm stream, after the exchange
            if (t > 0)
                if (int rc = wait_interior(c, s, s.comm, pp)) return rc;
            if (c->transport == GOL_XPORT_PEER) {
                // neighbours must have pulled our previous edge rows before we overwrite them
                Slab *up = find_slab(c, s.index - 1), *dn = find_slab(c, s.index + 1);
                if (up) HIPCHK(c, tr_wait(c, s.comm, up->ev_exch[p]));
                if (dn) HIPCHK(c, tr_wait(c, s.comm, dn->ev_exch[p]));
            }
            if (int rc = comm_mark(c, s, 2)) return rc;
            if (!c->overlap || thin) {
                int rc = launch_stencil(c, s, k, lo, hi, s.comm, true);
                if (!rc) rc = comm_mark(c, s, 3);
                if (rc) return rc;
                HIPCHK(c, tr_record(c, s.ev_bnd[p], s.comm));
                HIPCHK(c, tr_record(c, s.ev_int[p], s.comm));
                for (int j = 0; j < s.nx; ++j) HIPCHK(c, tr_record(c, s.ev_part[j][p], s.comm));
                continue;
            }
            // (cuts over [lo + K, hi - K): the same for every block depth k <= K)
            const int clo = lo + c->K, chi = hi - c->K, np = nparts(s, clo, chi);
            int rc = launch_stencil(c, s, k, lo, lo + k, s.comm, false);
            if (!rc) rc = launch_stencil(c, s, k, hi - k, hi, s.comm, false);
            if (!rc) rc = seams(s, clo, chi, np);
            if (!rc) rc = comm_mark(c, s, 3);
            if (rc) return rc;
            HIPCHK(c, tr_record(c, s.ev_bnd[p], s.comm));
            // interior on the compute stream(s): needs the previous boundary (and seam) bands
            if (int rc2 = parts(s, lo + k, hi - k, clo, chi, np)) return rc2;
        }
    }
    if (int rc = tune_after(c, tslot, p)) return rc;
    c->cur ^= 1;
    c->step_index++;
    c->generation += k;
    c->last_k = k;
    return GOL_OK;
}

int sync_all(gol_ctx *c, double *elapsed_ms) {
    double ms_max = 0.0;
    for (auto &s : c->slabs) {
        HIPCHK(c, hipSetDevice(s.device));
        if (c->batch_open) {
            hipEvent_t e;
            HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIPCHK(c, tr_record(c, e, s.comm));
            HIPCHK(c, tr_wait(c, s.comp, e));
            if (int rc = join_parts(c, s, s.comp)) return rc;
            HIPCHK(c, tr_record(c, s.ev_stop, s.comp));
            HIPCHK(c, tr_esync(c, s.ev_stop));
            HIPCHK(c, hipEventDestroy(e));
            float ms = 0.f;
            HIPCHK(c, hipEventElapsedTime(&ms, s.ev_start, s.ev_stop));
            ms_max = std::max(ms_max, (double)ms);
        }
        HIPCHK(c, tr_ssync(c, s.comm));
        HIPCHK(c, tr_ssync(c, s.comp));
        for (int j = 0; j < s.nx; ++j) HIPCHK(c, tr_ssync(c, s.part[j]));
    }
    c->batch_open = false;
    for (; c->timed_live > 0; --c->timed_live) {
        const TimedLaunch &o = c->timed[c->timed_head];
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, o.a, o.b));
        c->timed_ms += ms;
        c->timed_count++;
        c->timed_head = (c->timed_head + 1) % kTimedRing;
    }
    if (int rc = tune_poll(c, true)) return rc;
    for (size_t i : c->release_at_sync) c->staging[i].busy = false;   // a failed async copy's staging
    c->release_at_sync.clear();
    // windows enqueued by gol_download_window_async: their copies are complete
    std::vector<PendingWindow> pend;
    pend.swap(c->pending);
    for (auto &w : pend) {
        Staging &b = c->staging[w.stage];
        for (int64_t r = 0; r < w.nrows; ++r) memcpy(w.host + r * w.ld, b.pinned + r * w.ncols, (size_t)w.ncols);
        b.busy = false;
    }
    if (elapsed_ms) *elapsed_ms = ms_max;
    return GOL_OK;
}

// A pooled staging pair (device + pinned) of at least `bytes` on `device`,
// marked busy; the smallest free one that fits, else a new one.  While the
// clock probe runs nothing is allocated — hipMalloc / hipHostMalloc can wait
// for the whole device, i.e. for the probe (the 10-s stall of DESIGN.md §5):
// GOL_ESTATE if no pooled buffer fits then.
int acquire_staging(gol_ctx *c, int device, size_t bytes, size_t *idx) {
    size_t pick = c->staging.size();
    for (size_t i = 0; i < c->staging.size(); ++i) {
        const Staging &b = c->staging[i];
        if (!b.busy && b.device == device && b.bytes >= bytes &&
            (pick == c->staging.size() || b.bytes < c->staging[pick].bytes))
            pick = i;
    }
    if (pick == c->staging.size()) {
        if (c->clk_running)
            return fail(c, GOL_ESTATE,
                        "no pooled staging of %zu bytes is free while the clock probe runs (an allocation "
                        "would wait for the probe): copy a window of this size once before gol_clock_start",
                        bytes);
        HIPCHK(c, hipSetDevice(device));
        // The pool stays bounded: an idle entry of this device that is too small is
        // freed and its slot reused (slots are never erased: pending copies and
        // release_at_sync hold indices), so a context copying windows of growing
        // sizes keeps one pair per concurrently busy copy, not one per size.
        for (size_t i = 0; i < c->staging.size() && pick == c->staging.size(); ++i) {
            Staging &o = c->staging[i];
            if (o.busy || o.device != device) continue;
            (void)hipFree(o.dtmp);
            (void)hipHostFree(o.pinned);
            o.dtmp = nullptr;
            o.pinned = nullptr;
            o.bytes = 0;
            pick = i;
        }
        Staging b;
        b.device = device;
        b.bytes = bytes;
        HIPCHK(c, hipMalloc(&b.dtmp, bytes));
        if (hipHostMalloc(&b.pinned, bytes, hipHostMallocDefault) != hipSuccess) {
            (void)hipFree(b.dtmp);
            return fail(c, GOL_ENOMEM, "pinned staging of %zu bytes", bytes);
        }
        if (pick == c->staging.size()) c->staging.push_back(b);
        else c->staging[pick] = b;
    }
    c->staging[pick].busy = true;
    *idx = pick;
    return GOL_OK;
}

// Enqueue a copy of a window as it stands after every step enqueued so far:
// unpack (bit) or gather (byte) into device staging on the slab's compute
// stream, then an async D2H copy into pinned staging; sync_all delivers it.
// All staging is acquired before anything is enqueued, and the caller's
// buffer is registered for delivery only once every slab's copy is enqueued:
// a failed call leaves no pending write into the caller's memory (its staging
// stays busy until the next sync, as copies may be in flight).
int window_async(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, uint8_t *host, int64_t ld) {
    if (nrows < 0 || ncols < 0 || row0 < 0 || col0 < 0 || row0 + nrows > c->rows || col0 + ncols > c->cols)
        return fail(c, GOL_EINVAL, "window outside the grid");
    if (ld < ncols) return fail(c, GOL_EINVAL, "ld < ncols");
    if (nrows == 0 || ncols == 0) return GOL_OK;
    int64_t held = 0;
    for (auto &s : c->slabs) held += std::max<int64_t>(0, std::min(row0 + nrows, s.row0 + s.H) - std::max(row0, s.row0));
    if (held != nrows) return fail(c, GOL_EINVAL, "window rows are not all held by this context");
    struct Piece {
        Slab *s;
        int64_t r0, r1;
        size_t stage;
    };
    std::vector<Piece> pieces;
    for (auto &s : c->slabs) {
        const int64_t r0 = std::max(row0, s.row0), r1 = std::min(row0 + nrows, s.row0 + s.H);
        if (r1 <= r0) continue;
        size_t st = 0;
        if (int rc = acquire_staging(c, s.device, (size_t)((r1 - r0) * ncols), &st)) {
            for (auto &p : pieces) c->staging[p.stage].busy = false;   // nothing enqueued yet
            return rc;
        }
        pieces.push_back({&s, r0, r1, st});
    }
    auto enqueue = [&](const Piece &p) -> int {
        Slab &s = *p.s;
        Staging &buf = c->staging[p.stage];
        const int64_t nr = p.r1 - p.r0;
        HIPCHK(c, hipSetDevice(s.device));
        // the last step's boundary bands run on the comm stream: join it
        hipEvent_t e;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const hipError_t e1 = tr_record(c, e, s.comm);
        const hipError_t e2 = e1 == hipSuccess ? tr_wait(c, s.comp, e) : e1;
        (void)hipEventDestroy(e);
        HIPCHK(c, e2);
        if (int rc = join_parts(c, s, s.comp)) return rc;   // (a split interior's other parts)
        const int64_t srow = c->hk + (p.r0 - s.row0);
        tr_op(c, TR_READ, s.comp, nullptr, s.index, c->cur, srow, srow + nr);
        int rc = for_col_runs(c, col0, ncols, [&](int64_t lc, int64_t pc, int64_t n) -> int {
            uint8_t *d = buf.dtmp + (lc - col0);
            if (c->layout == GOL_LAYOUT_BYTE)
                HIPCHK(c, hipMemcpy2DAsync(d, ncols, static_cast<uint8_t *>(s.buf[c->cur]) + srow * c->pitch_bytes + pc,
                                           c->pitch_bytes, n, nr, hipMemcpyDeviceToDevice, s.comp));
            else
                HIPCHK(c, launch_unpack_window(static_cast<uint32_t *>(s.buf[c->cur]), c->pitch_bytes / 4, d, ncols,
                                               srow, pc, nr, n, c->gw, s.comp));
            return GOL_OK;
        });
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(buf.pinned, buf.dtmp, (size_t)(nr * ncols), hipMemcpyDeviceToHost, s.comp));
        // The other streams of the slab wait for later steps' events only, recorded after
        // other work than this copy on the compute stream (a split interior's parts wait for
        // seam bands; without overlap the whole step runs on the comm stream): they must
        // wait for the copy before a later step overwrites these rows (found by the
        // schedule check, tests/test_gpu_sched.py)
        if (s.nx || s.comm != s.comp) {
            hipEvent_t f;
            HIPCHK(c, hipEventCreateWithFlags(&f, hipEventDisableTiming));
            hipError_t f1 = tr_record(c, f, s.comp);
            if (f1 == hipSuccess && s.comm != s.comp) f1 = tr_wait(c, s.comm, f);
            for (int j = 0; j < s.nx && f1 == hipSuccess; ++j) f1 = tr_wait(c, s.part[j], f);
            (void)hipEventDestroy(f);
            HIPCHK(c, f1);
        }
        return GOL_OK;
    };
    for (const auto &p : pieces) {
        if (int rc = enqueue(p)) {
            for (auto &q : pieces) c->release_at_sync.push_back(q.stage);
            return rc;
        }
    }
    for (const auto &p : pieces) {
        PendingWindow w;
        w.stage = p.stage;
        w.host = host + (p.r0 - row0) * ld;
        w.ld = ld;
        w.nrows = p.r1 - p.r0;
        w.ncols = ncols;
        c->pending.push_back(w);
    }
    return GOL_OK;
}

// ------------------------------------------------------------------- init units

struct UnitPlan {
    std::vector<InitUnit> units;
    int maxlen = 0;
};

int run_units(gol_ctx *c, Slab &s, UnitPlan &plan) {
    if (plan.units.empty()) return GOL_OK;
    static const JumpTable jt;
    const int seg = 2048;
    const int T = std::max(1, (plan.maxlen + seg - 1) / seg);
    std::vector<uint32_t> mats((size_t)T * 961);
    const Mat31 step = jt.power(seg);
    Mat31 m = JumpTable::identity();
    for (int t = 0; t < T; ++t) {
        memcpy(&mats[(size_t)t * 961], m.a, sizeof m.a);
        m = JumpTable::mat_mul(m, step);
    }
    InitUnit *d_units = nullptr;
    uint32_t *d_mats = nullptr;
    HIPCHK(c, hipMalloc(&d_units, plan.units.size() * sizeof(InitUnit)));
    HIPCHK(c, hipMalloc(&d_mats, mats.size() * sizeof(uint32_t)));
    // on the slab's stream: ordered before the generator without relying on the
    // null stream (the host vectors outlive the hipStreamSynchronize below)
    HIPCHK(c, hipMemcpyAsync(d_units, plan.units.data(), plan.units.size() * sizeof(InitUnit), hipMemcpyHostToDevice,
                             s.comp));
    HIPCHK(c, hipMemcpyAsync(d_mats, mats.data(), mats.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s.comp));
    // bit layout: the generator writes linear words (bit i = column 32w+i) into the
    // spare buffer, then one pass regroups them into 2-word groups
    const bool bit = c->layout == GOL_LAYOUT_BIT;
    void *target = bit ? s.buf[c->cur ^ 1] : s.buf[c->cur];
    hipError_t e = launch_init_units(d_units, (int)plan.units.size(), d_mats, T, seg, target, c->pitch_bytes, bit,
                                     s.comp);
    if (e == hipSuccess && bit)
        e = launch_interleave_rows(static_cast<const uint32_t *>(target), static_cast<uint32_t *>(s.buf[c->cur]),
                                   c->pitch_bytes / 4, c->hk, s.H, (c->cols + 127) / 128, c->gw, s.comp);
    if (e == hipSuccess && bit)
        e = hipMemsetAsync(target, 0, (size_t)storage_rows(c, s) * c->pitch_bytes, s.comp);
    hipError_t e2 = tr_ssync(c, s.comp);
    (void)hipFree(d_units);
    (void)hipFree(d_mats);
    HIPCHK(c, e);
    HIPCHK(c, e2);
    return GOL_OK;
}

int init_slab(gol_ctx *c, Slab &s, int mode, uint32_t seed) {
    static const JumpTable jt;
    UnitPlan plan;
    const int64_t hk = c->hk;
    auto add_units = [&](uint32_t stream_seed, uint64_t first_offset, uint64_t stride, int64_t g0, int64_t g1,
                         int32_t col0, int32_t len) {
        if (g1 <= g0 || len <= 0) return;
        uint32_t w[31];
        glibc_seed_window(stream_seed, w);
        jt.jump(first_offset, w);
        const Mat31 st = jt.power(stride);
        for (int64_t g = g0; g < g1; ++g) {
            InitUnit u;
            u.row = hk + (g - s.row0);
            u.col0 = col0;
            u.len = len;
            memcpy(u.w, w, sizeof w);
            u.pad = 0;
            plan.units.push_back(u);
            JumpTable::mat_vec(st, w, w);
        }
        plan.maxlen = std::max(plan.maxlen, (int)len);
    };
    // logical columns [lcol0, lcol0+len) of rows [g0, g1), draw `first_offset` at (g0, lcol0):
    // one unit run per storage-contiguous piece
    bool misaligned = false;
    auto add_cols = [&](uint32_t stream_seed, uint64_t first_offset, uint64_t stride, int64_t g0_, int64_t g1_,
                        int64_t lcol0, int64_t len) {
        for_col_runs(c, lcol0, len, [&](int64_t lc, int64_t pc, int64_t n) {
            // the bit-layout writer stores whole 32-column words: runs must start on one
            if (c->layout == GOL_LAYOUT_BIT && pc % 32 != 0) misaligned = true;
            add_units(stream_seed, first_offset + (uint64_t)(lc - lcol0), stride, g0_, g1_, (int32_t)pc, (int32_t)n);
            return GOL_OK;
        });
    };
    const int64_t g0 = s.row0, g1 = s.row0 + s.H;
    if (mode == GOL_INIT_STREAM) {
        add_cols(seed, (uint64_t)g0 * c->cols, c->cols, g0, g1, 0, c->active_cols);
        if (c->boundary == GOL_SERIAL_COMPAT) {   // keep the inactive last row dead
            const int64_t gl = std::min(g1, c->rows - 1);
            plan.units.erase(std::remove_if(plan.units.begin(), plan.units.end(),
                                            [&](const InitUnit &u) { return u.row - hk + s.row0 >= gl; }),
                             plan.units.end());
        }
    } else if (mode == GOL_INIT_SERIAL) {
        if (c->rows != c->cols) return fail(c, GOL_EINVAL, "GOL_INIT_SERIAL needs a square grid");
        const int64_t n = c->cols;
        const int64_t e1 = std::min(g1, n - 1);
        if (e1 > g0) add_cols(seed, (uint64_t)(g0 + 1) * n + 1, n, g0, e1, 0, n - 1);
    } else if (mode == GOL_INIT_MESH) {
        const int m = c->mesh_m;
        if (c->rows != c->cols || m < 1 || c->cols % m != 0)
            return fail(c, GOL_EINVAL, "GOL_INIT_MESH needs a square grid with cols %% mesh_m == 0");
        const int64_t L = c->cols / m;
        for (int64_t cx = g0 / L; cx * L < g1; ++cx) {
            const int64_t b0 = std::max(g0, cx * L), b1 = std::min(g1, (cx + 1) * L);
            for (int cy = 0; cy < m; ++cy)
                add_cols(seed + (uint32_t)(cx * m + cy), (uint64_t)(b0 - cx * L) * L, L, b0, b1, cy * L, L);
        }
    } else {
        return fail(c, GOL_EINVAL, "unknown init mode %d", mode);
    }
    if (misaligned)
        return fail(c, GOL_EUNSUPPORTED,
                    "on-device init of the bit layout needs column blocks on 32-column boundaries "
                    "(upload the board, or use the byte layout)");
    return run_units(c, s, plan);
}

// Zero the cells outside the active region (SERIAL_COMPAT: last row and column),
// enqueued on the slab's compute stream (the caller synchronises it).
int enforce_inactive(gol_ctx *c, Slab &s, int buf) {
    if (c->boundary != GOL_SERIAL_COMPAT) return GOL_OK;
    uint8_t *b = static_cast<uint8_t *>(s.buf[buf]);
    const int64_t gl = c->rows - 1;
    if (gl >= s.row0 && gl < s.row0 + s.H)
        HIPCHK(c, hipMemsetAsync(b + (size_t)(c->hk + gl - s.row0) * c->pitch_bytes, 0, c->pitch_bytes, s.comp));
    if (c->layout == GOL_LAYOUT_BYTE)
        HIPCHK(c, hipMemset2DAsync(b + (size_t)c->hk * c->pitch_bytes + (c->cols - 1), c->pitch_bytes, 0, 1, s.H,
                                   s.comp));
    // bit layout: the pack kernel already clears columns >= active_cols
    return GOL_OK;
}

// ------------------------------------------------------------------ windows
// Host <-> device windows go through the pooled staging (acquire_staging) in
// row blocks of at most kIoBlock bytes, with stream syncs only: no hipMalloc /
// hipFree / hipDeviceSynchronize, so a window copy completes while the clock
// probe runs (it used to wait for the probe).
constexpr int64_t kIoBlock = 64LL << 20;

// host rows [r0, r1) of the window -> slab s: pinned staging, H2D, then a
// strided device copy + normalisation (byte) or the pack kernel (bit)
int upload_piece(gol_ctx *c, Slab &s, int64_t r0, int64_t r1, int64_t col0, int64_t ncols, const uint8_t *hrows,
                 int64_t ld) {
    const int64_t nr = r1 - r0;
    size_t st = 0;
    if (int rc = acquire_staging(c, s.device, (size_t)(nr * ncols), &st)) return rc;
    Staging &b = c->staging[st];
    for (int64_t r = 0; r < nr; ++r) memcpy(b.pinned + r * ncols, hrows + r * ld, (size_t)ncols);
    const int64_t srow = c->hk + (r0 - s.row0);
    uint8_t *board = static_cast<uint8_t *>(s.buf[c->cur]);
    auto enqueue = [&]() -> int {
        HIPCHK(c, hipSetDevice(s.device));
        tr_op(c, TR_WRITE, s.comp, nullptr, s.index, c->cur, srow, srow + nr);
        HIPCHK(c, hipMemcpyAsync(b.dtmp, b.pinned, (size_t)(nr * ncols), hipMemcpyHostToDevice, s.comp));
        return for_col_runs(c, col0, ncols, [&](int64_t lc, int64_t pc, int64_t n) -> int {
            const uint8_t *cells = b.dtmp + (lc - col0);
            if (c->layout == GOL_LAYOUT_BYTE) {
                uint8_t *d = board + srow * c->pitch_bytes + pc;
                HIPCHK(c, hipMemcpy2DAsync(d, c->pitch_bytes, cells, ncols, n, nr, hipMemcpyDeviceToDevice, s.comp));
                // cells are bools (main.cpp:73): any nonzero byte is a live cell
                HIPCHK(c, launch_normalize_bytes(d, c->pitch_bytes, nr, n, s.comp));
            } else {
                HIPCHK(c, launch_pack_window(cells, ncols, reinterpret_cast<uint32_t *>(board), c->pitch_bytes / 4,
                                             srow, pc, nr, n, c->active_cols, c->gw, s.comp));
            }
            return GOL_OK;
        });
    };
    int rc = enqueue();
    if (rc) {
        c->release_at_sync.push_back(st);   // work may be in flight: busy until the next sync
        return rc;
    }
    HIPCHK(c, tr_ssync(c, s.comp));
    b.busy = false;
    return GOL_OK;
}

int window_io(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, uint8_t *host, int64_t ld,
              bool upload) {
    if (nrows < 0 || ncols < 0 || row0 < 0 || col0 < 0 || row0 + nrows > c->rows || col0 + ncols > c->cols)
        return fail(c, GOL_EINVAL, "window outside the grid");
    if (ld < ncols) return fail(c, GOL_EINVAL, "ld < ncols");
    if (nrows == 0 || ncols == 0) return GOL_OK;
    if (int rc = sync_all(c, nullptr)) return rc;
    const int64_t br = std::max<int64_t>(1, kIoBlock / ncols);
    bool any = false;
    // slab by slab (a rank context moves the rows it holds; the others stay untouched)
    for (size_t si = 0; si < c->slabs.size(); ++si) {
        Slab &s = c->slabs[si];
        const int64_t r0 = std::max(row0, s.row0), r1 = std::min(row0 + nrows, s.row0 + s.H);
        if (r1 <= r0) continue;
        any = true;
        for (int64_t a = r0; a < r1; a += br) {
            const int64_t e = std::min(r1, a + br);
            uint8_t *h = host + (a - row0) * ld;
            int rc = upload ? upload_piece(c, s, a, e, col0, ncols, h, ld) : window_async(c, a, col0, e - a, ncols, h, ld);
            if (!rc && !upload) rc = sync_all(c, nullptr);
            if (rc) return rc;
        }
        if (upload) {
            if (int rc = enforce_inactive(c, s, c->cur)) return rc;
            HIPCHK(c, hipSetDevice(s.device));
            HIPCHK(c, tr_ssync(c, s.comp));
        }
    }
    if (!any && c->transport != GOL_XPORT_RCCL) return fail(c, GOL_EINVAL, "window holds no local rows");
    return GOL_OK;
}

// ------------------------------------------------------------------ snapshot text
// The `.gol` part-file body (main.cpp:106-129) is formatted / parsed on the
// device (gol_text.hip); the host only moves finished bytes.  Blocks of rows
// go through two pinned buffers so the host's write()/read() of block i
// overlaps the device work and PCIe copy of block i±1.
struct TextHost {
    char *out = nullptr;        // memory sink
    const char *in = nullptr;   // memory source
    int fd = -1;                // file descriptor sink / source
    int64_t pos = 0;            // bytes moved so far
};

int host_put(gol_ctx *c, TextHost &h, const char *buf, int64_t n) {
    if (h.out) {
        memcpy(h.out + h.pos, buf, (size_t)n);
    } else {
        for (int64_t done = 0; done < n;) {
            const ssize_t w = write(h.fd, buf + done, (size_t)std::min<int64_t>(n - done, 1 << 30));
            if (w < 0 && errno == EINTR) continue;
            if (w <= 0) return fail(c, GOL_EINVAL, "write(fd %d): %s", h.fd, strerror(errno));
            done += w;
        }
    }
    h.pos += n;
    return GOL_OK;
}

int host_get(gol_ctx *c, TextHost &h, char *buf, int64_t n) {
    if (h.in) {
        memcpy(buf, h.in + h.pos, (size_t)n);
    } else {
        for (int64_t done = 0; done < n;) {
            const ssize_t r = read(h.fd, buf + done, (size_t)std::min<int64_t>(n - done, 1 << 30));
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) return fail(c, GOL_EINVAL, "read(fd %d): %s", h.fd, strerror(errno));
            if (r == 0)
                return fail(c, GOL_EINVAL, "snapshot text ends after %lld of %lld bytes", (long long)(h.pos + done),
                            (long long)(h.pos + n));
            done += r;
        }
    }
    h.pos += n;
    return GOL_OK;
}

struct TextBuffers {
    char *pinned[2] = {nullptr, nullptr};
    char *dtext = nullptr;
    uint8_t *dcells = nullptr;
    unsigned long long *derr = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~TextBuffers() {
        for (int i = 0; i < 2; ++i) {
            if (pinned[i]) (void)hipHostFree(pinned[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
        }
        if (dtext) (void)hipFree(dtext);
        if (dcells) (void)hipFree(dcells);
        if (derr) (void)hipFree(derr);
    }
};

int text_io(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, TextHost &h, bool upload) {
    if (nrows < 0 || ncols < 0 || row0 < 0 || col0 < 0 || row0 + nrows > c->rows || col0 + ncols > c->cols)
        return fail(c, GOL_EINVAL, "window outside the grid");
    if (nrows == 0 || ncols == 0) return GOL_OK;
    // every row of the window must be held here (a rank formats / parses its own part)
    int64_t held = 0;
    for (auto &s : c->slabs) held += std::max<int64_t>(0, std::min(row0 + nrows, s.row0 + s.H) - std::max(row0, s.row0));
    if (held != nrows) return fail(c, GOL_EINVAL, "text window rows are not all held by this context");
    // the text path allocates its pinned blocks per call, and an allocation can
    // wait for the whole device (i.e. for a running probe)
    if (c->clk_running) return fail(c, GOL_ESTATE, "snapshot text while the clock probe runs");
    {
        int rc = sync_all(c, nullptr);
        if (rc) return rc;
    }
    const int64_t rowlen = 2 * ncols + 1;
    const int64_t br = std::max<int64_t>(1, c->text_block_bytes / rowlen);
    const bool bit = c->layout == GOL_LAYOUT_BIT;
    for (auto &s : c->slabs) {
        const int64_t r0 = std::max(row0, s.row0), r1 = std::min(row0 + nrows, s.row0 + s.H);
        if (r1 <= r0) continue;
        HIPCHK(c, hipSetDevice(s.device));
        const int64_t nb = (r1 - r0 + br - 1) / br, bmax = std::min(br, r1 - r0);
        TextBuffers t;
        for (int i = 0; i < 2; ++i) {
            HIPCHK(c, hipHostMalloc(&t.pinned[i], (size_t)(bmax * rowlen), hipHostMallocDefault));
            HIPCHK(c, hipEventCreateWithFlags(&t.ev[i], hipEventDisableTiming));
        }
        HIPCHK(c, hipMalloc(&t.dtext, (size_t)round_up(bmax * rowlen, 256)));
        const bool staged = bit || c->perm_m > 1;   // parse into a cell buffer, then place the column runs
        if (upload) {
            if (staged) HIPCHK(c, hipMalloc(&t.dcells, (size_t)(bmax * ncols)));
            HIPCHK(c, hipMalloc(&t.derr, sizeof(unsigned long long)));
            HIPCHK(c, hipMemsetAsync(t.derr, 0xff, sizeof(unsigned long long), s.comm));
        }
        uint8_t *cur = static_cast<uint8_t *>(s.buf[c->cur]);
        auto rows_of = [&](int64_t i) { return std::min(br, r1 - r0 - i * br); };
        // device part of block i, on the (idle) comm stream, ending with event ev[i&1]
        auto enqueue = [&](int64_t i) -> int {
            const int64_t a = r0 + i * br, nr = rows_of(i), bytes = nr * rowlen;
            const int64_t srow = c->hk + (a - s.row0);
            char *pin = t.pinned[i & 1];
            if (!upload) {
                HIPCHK(c, launch_format_text(cur, c->pitch_bytes, bit ? c->gw : 0, srow, col0, nr, ncols, c->perm_m,
                                             c->perm_L, t.dtext, s.comm));
                HIPCHK(c, hipMemcpyAsync(pin, t.dtext, (size_t)bytes, hipMemcpyDeviceToHost, s.comm));
            } else {
                HIPCHK(c, hipMemcpyAsync(t.dtext, pin, (size_t)bytes, hipMemcpyHostToDevice, s.comm));
                const int64_t base = (a - row0) * rowlen;
                if (staged) {
                    HIPCHK(c, launch_parse_text(t.dtext, nr, ncols, t.dcells, ncols, base, t.derr, s.comm));
                    int rc2 = for_col_runs(c, col0, ncols, [&](int64_t lc, int64_t pc, int64_t n) -> int {
                        const uint8_t *cells = t.dcells + (lc - col0);
                        if (bit)
                            HIPCHK(c, launch_pack_window(cells, ncols, reinterpret_cast<uint32_t *>(cur),
                                                         c->pitch_bytes / 4, srow, pc, nr, n, c->active_cols, c->gw,
                                                         s.comm));
                        else
                            HIPCHK(c, hipMemcpy2DAsync(cur + srow * c->pitch_bytes + pc, c->pitch_bytes, cells, ncols,
                                                       n, nr, hipMemcpyDeviceToDevice, s.comm));
                        return GOL_OK;
                    });
                    if (rc2) return rc2;
                } else {
                    HIPCHK(c, launch_parse_text(t.dtext, nr, ncols, cur + srow * c->pitch_bytes + col0,
                                                c->pitch_bytes, base, t.derr, s.comm));
                }
            }
            HIPCHK(c, tr_record(c, t.ev[i & 1], s.comm));
            return GOL_OK;
        };
        int rc = GOL_OK;
        if (!upload) {
            for (int64_t i = 0; i < std::min<int64_t>(nb, 2) && !rc; ++i) rc = enqueue(i);
            for (int64_t i = 0; i < nb && !rc; ++i) {
                HIPCHK(c, tr_esync(c, t.ev[i & 1]));
                rc = host_put(c, h, t.pinned[i & 1], rows_of(i) * rowlen);
                if (!rc && i + 2 < nb) rc = enqueue(i + 2);
            }
        } else {
            for (int64_t i = 0; i < nb && !rc; ++i) {
                if (i >= 2) HIPCHK(c, tr_esync(c, t.ev[i & 1]));   // block i-2's copy has left the buffer
                rc = host_get(c, h, t.pinned[i & 1], rows_of(i) * rowlen);
                if (!rc) rc = enqueue(i);
            }
        }
        HIPCHK(c, tr_ssync(c, s.comm));
        if (rc) return rc;
        if (upload) {
            unsigned long long bad = 0;
            HIPCHK(c, hipMemcpy(&bad, t.derr, sizeof bad, hipMemcpyDeviceToHost));
            if (bad != ~0ull) {
                const int64_t off = (int64_t)bad;
                return fail(c, GOL_EINVAL, "malformed snapshot text at byte %lld (row %lld, column %lld of the window)",
                            (long long)off, (long long)(off / rowlen), (long long)((off % rowlen) / 2));
            }
            rc = enforce_inactive(c, s, c->cur);
            if (rc) return rc;
            HIPCHK(c, tr_ssync(c, s.comp));
        }
    }
    return GOL_OK;
}

// Hardware queues a process gets per device: GPU_MAX_HW_QUEUES, HIP's default 4.
int hw_queue_budget() {
    const char *v = getenv("GPU_MAX_HW_QUEUES");
    const int n = v ? atoi(v) : 0;
    return n > 0 ? n : 4;
}

// The split interior by default for a k = 8 bit context (the pair kernel), unless
// its devices hold more than kSplitSlabsPerDevice slabs, or its
// streams would share hardware queues: a split slab holds three streams, and
// every device also has the process's clock-probe stream, so the split is on only
// when 3 x slabs per device + 1 fits GPU_MAX_HW_QUEUES (the HIP default of 4:
// one slab per device, the headline's shape; bench.py asks for 24).
int default_split(gol_ctx *c) {
    if (c->layout != GOL_LAYOUT_BIT || c->K < 8) return GOL_OK;
    std::vector<int> per;
    const int queues = hw_queue_budget();
    for (auto &s : c->slabs) {
        if ((int)per.size() <= s.device) per.resize(s.device + 1, 0);
        ++per[s.device];
        if (per[s.device] > kSplitSlabsPerDevice || 3 * per[s.device] + 1 > queues) return GOL_OK;
    }
    for (auto &s : c->slabs)
        if (int rc = enable_split(c, s, kSplitParts)) return rc;
    c->split = kSplitParts;
    c->chunk_rows = kSplitChunk;
    return GOL_OK;
}

int common_create(gol_ctx *c, int64_t rows, int64_t cols, int layout, int boundary, int mesh_m, int k) {
    c->rows = rows;
    c->cols = cols;
    c->layout = layout;
    c->boundary = boundary;
    c->mesh_m = mesh_m < 1 ? 1 : mesh_m;
    if (boundary == GOL_MESH_COMPAT && c->mesh_m > 1) {
        c->perm_m = c->mesh_m;
        c->perm_L = cols / c->mesh_m;
    }
    c->K = k;
    c->hk = k;
    c->gw = layout == GOL_LAYOUT_BIT ? bit_group_words(k) : 2;
    // Geometry defaults measured on MI355X at 131072² (tools/tune.py):
    // k <= 4 is HBM-bound and wants many short chunks; k >= 6 is VALU-bound and
    // wants long chunks (less vertical recompute).
    // chunk rows: > 0 fixed; -r = exactly r rounds of resident waves; -(100+r) = guided, r rounds of
    // halving chunks (gol_kernels.hip plan_items)
    // k=8: six rounds of equal trip-aligned chunks (184 rows at 131072²): +2 % over three rounds,
    // +7 % over guided 3 rounds, on 4 boxes (profiles/r02p_k8_fine_*.jsonl, r02o_k8_policy_*.jsonl)
    // k=5/6: six rounds (+4.5 % over four), k=7: four rounds (+3 % over two, +7 % over guided)
    // (profiles/r02p_k5to8.jsonl, r02o_k7_policy_ab.jsonl)
    // k=8 on 4-word groups (the pair kernel at 2 waves/SIMD, 17 strips at 131072 columns):
    // guided 4 rounds, +2.2 % over six rounds (-103..-106 within 0.2 %; profiles/r04d_g4_policy_sweep.jsonl)
    static const int kChunk[9] = {16, 16, 16, 32, 32, -6, -6, -4, -6};
    if (c->layout == GOL_LAYOUT_BIT) {
        // k = 16 / 32 (the chain of pair waves): one round of equal chunks
        c->chunk_rows = k > 8 ? -1 : (k == 8 && c->gw == 4) ? -104 : kChunk[k];
    } else {
        // tools/tune.py at 32768² and 16384² (profiles/r02n_*chunk*.jsonl): SWAR k <= 3
        // 32-row chunks (+3-5 % over 64), bytebit k=4 64 rows, k=16 guided 2 rounds,
        // k >= 20 one round of equal chunks (+1 % at 32768², +5 % at 16384² over guided)
        // byte k=1 (2 dwords per lane, 9 rows of prefetch): 16-row chunks +4-6 % over 32 (r03b_byte1_ab)
        c->chunk_rows = k == 1 ? 16 : k <= 3 ? 32 : (k == 4 ? 64 : (k < 16 ? -2 : (k == 16 ? -102 : -1)));
    }
    set_geometry(c);
    return GOL_OK;
}
} // namespace

// ====================================================================== C ABI

extern "C" {

const char *gol_version(void) { return "golhip 0.3 gfx950 (bit+byte register-pipeline stencils, RCCL halos)"; }

int gol_slab_plan(int64_t rows, int world, int rank, int64_t *row0, int64_t *nrows) {
    if (rows < 1 || world < 1 || rank < 0 || rank >= world || !row0 || !nrows) return GOL_EINVAL;
    slab_plan(rows, world, rank, row0, nrows);
    return GOL_OK;
}

int gol_get_unique_id(uint8_t *unique_id) {
    if (!unique_id) return GOL_EINVAL;
    RcclApi &R = rccl();
    if (!R.ok) return GOL_ERCCL;
    ncclUniqueId id;
    if (R.GetUniqueId(&id) != ncclSuccess) return GOL_ERCCL;
    memcpy(unique_id, id.internal, GOL_UNIQUE_ID_BYTES);
    return GOL_OK;
}

int gol_create(gol_ctx **out, int64_t rows, int64_t cols, int n_gpus, int layout, int boundary, int mesh_m,
               int tblock_k) {
    if (!out) return GOL_EINVAL;
    *out = nullptr;
    gol_ctx *c = new gol_ctx();
    int rc = validate(c, rows, cols, n_gpus, layout, boundary, mesh_m, tblock_k);
    if (rc) {
        fprintf(stderr, "gol_create: %s\n", c->err.c_str());
        delete c;
        return rc;
    }
    common_create(c, rows, cols, layout, boundary, mesh_m, tblock_k);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        fprintf(stderr, "gol_create: no HIP device visible\n");
        delete c;
        return GOL_EHIP;
    }
    c->nslabs = n_gpus;
    c->transport = n_gpus > 1 ? GOL_XPORT_PEER : GOL_XPORT_NONE;
    c->slabs.resize(n_gpus);
    for (int i = 0; i < n_gpus; ++i) {
        Slab &s = c->slabs[i];
        s.index = i;
        s.device = i % ndev;
        slab_plan(rows, n_gpus, i, &s.row0, &s.H);
        rc = alloc_slab(c, s);
        if (rc) {
            fprintf(stderr, "gol_create: %s\n", c->err.c_str());
            gol_destroy(c);
            return rc;
        }
    }
    // peer access between distinct devices (xGMI); same-device copies need none
    for (int i = 0; i + 1 < n_gpus; ++i) {
        const int a = c->slabs[i].device, b = c->slabs[i + 1].device;
        if (a != b) {
            (void)hipSetDevice(a);
            (void)hipDeviceEnablePeerAccess(b, 0);
            (void)hipSetDevice(b);
            (void)hipDeviceEnablePeerAccess(a, 0);
            (void)hipGetLastError();
        }
    }
    if (int rc2 = default_split(c)) {
        fprintf(stderr, "gol_create: %s\n", c->err.c_str());
        gol_destroy(c);
        return rc2;
    }
    *out = c;
    return GOL_OK;
}

int gol_create_rank(gol_ctx **out, int64_t rows, int64_t cols, int rank, int world, int device,
                    const uint8_t *unique_id, int layout, int boundary, int mesh_m, int tblock_k) {
    if (!out || world < 1 || rank < 0 || rank >= world) return GOL_EINVAL;
    *out = nullptr;
    gol_ctx *c = new gol_ctx();
    int rc = validate(c, rows, cols, world, layout, boundary, mesh_m, tblock_k);
    if (rc) {
        fprintf(stderr, "gol_create_rank: %s\n", c->err.c_str());
        delete c;
        return rc;
    }
    common_create(c, rows, cols, layout, boundary, mesh_m, tblock_k);
    c->nslabs = world;
    c->rank = rank;
    c->world = world;
    c->transport = world > 1 ? GOL_XPORT_RCCL : GOL_XPORT_NONE;
    c->slabs.resize(1);
    Slab &s = c->slabs[0];
    s.index = rank;
    s.device = device;
    slab_plan(rows, world, rank, &s.row0, &s.H);
    rc = alloc_slab(c, s);
    if (!rc && world > 1) {
        RcclApi &R = rccl();
        if (!R.ok) rc = fail(c, GOL_ERCCL, "%s", R.err.c_str());
        else if (!unique_id) rc = fail(c, GOL_EINVAL, "unique_id required for world > 1");
        else {
            ncclUniqueId id;
            memcpy(id.internal, unique_id, GOL_UNIQUE_ID_BYTES);
            (void)hipSetDevice(device);
            ncclResult_t r = R.CommInitRank(&c->comm, world, id, rank);
            if (r != ncclSuccess) rc = fail(c, GOL_ERCCL, "ncclCommInitRank: %s", R.GetErrorString(r));
        }
        // the schedule trial's agreement buffers (tune_agree), allocated now: an
        // allocation in the middle of a run can wait for the whole device
        if (!rc && (hipMalloc(&c->agree_dev, 3 * sizeof(double)) != hipSuccess ||
                    hipHostMalloc(&c->agree_host, 3 * sizeof(double), hipHostMallocDefault) != hipSuccess))
            rc = fail(c, GOL_ENOMEM, "schedule-trial agreement buffers");
    }
    if (!rc) rc = default_split(c);
    if (rc) {
        fprintf(stderr, "gol_create_rank: %s\n", c->err.c_str());
        gol_destroy(c);
        return rc;
    }
    *out = c;
    return GOL_OK;
}

int gol_set_option(gol_ctx *c, int option, int64_t value) {
    if (!c) return GOL_EINVAL;
    switch (option) {
    case GOL_OPT_CHUNK_ROWS:
        if (value == 0)
            return fail(c, GOL_EUNSUPPORTED, "chunk rows 0 (the work-queue schedule) was retired in 0.2: "
                                             "use > 0 rows, -r rounds or -(100+r) guided");
        if (value < -108 || value > (1 << 20)) return fail(c, GOL_EINVAL, "chunk rows out of range");
        c->chunk_rows = (int)value;
        c->user_chunk = (int)value;
        c->chunk_user = true;
        return GOL_OK;
    case GOL_OPT_KERNEL_TIMING: c->timing = value != 0; return GOL_OK;
    case GOL_OPT_COMM_TIMING: c->comm_timing = value != 0; return GOL_OK;
    case GOL_OPT_HALO_EXCHANGE: c->halo_exchange = value != 0; return GOL_OK;
    case GOL_OPT_OVERLAP: c->overlap = value != 0; return GOL_OK;
    case GOL_OPT_BYTE_CORE:
        if (value < 0 || value > kByteCorePair) return fail(c, GOL_EINVAL, "byte core must be 0 .. 4");
        if (value == 0 && c->layout == GOL_LAYOUT_BYTE && c->K > 8)
            return fail(c, GOL_EUNSUPPORTED, "the byte-SWAR kernel fuses at most 8 generations");
        c->byte_core = (int)value;
        return GOL_OK;
    case GOL_OPT_TEXT_BLOCK_BYTES:
        if (value < 1) return fail(c, GOL_EINVAL, "text block bytes must be positive");
        c->text_block_bytes = value;
        return GOL_OK;
    case GOL_OPT_SCHEDULE_TRIAL: c->trial_enabled = value != 0; return GOL_OK;
    case GOL_OPT_SCHED_TRACE:
        c->tracing = value != 0;
        c->trace.clear();
        c->trace_full = false;
        return GOL_OK;
    case GOL_OPT_INTERIOR_SPLIT: {
        if (value < 1 || value > kMaxParts) return fail(c, GOL_EINVAL, "interior split must be 1 .. %d", kMaxParts);
        if (value == c->split) return GOL_OK;
        // the new stream/event graph starts from an idle context (no half-recorded step behind it)
        bool grows = false;
        for (auto &s : c->slabs) grows = grows || s.nx < value - 1;
        if (c->clk_running && grows)
            return fail(c, GOL_ESTATE, "interior split while the clock probe runs (it creates streams)");
        if (int rc = sync_all(c, nullptr)) return rc;
        if (value >= 2)
            for (auto &s : c->slabs)
                if (int rc = enable_split(c, s, (int)value)) return rc;
        c->split = (int)value;
        // the k = 8 default policy and trial candidates follow the split; a trial under
        // way starts over — except in RCCL mode once it records: like the trial's own
        // options, a rank-local change must not take this rank out of the agreement
        // the other ranks will enter; the rank runs on to it and keeps its own pick
        if (c->layout == GOL_LAYOUT_BIT && c->K == 8 && !c->chunk_user) {
            c->chunk_rows = c->split >= 2 ? kSplitChunk : -104;
            c->tune_default = c->chunk_rows;
            const bool committed = c->transport == GOL_XPORT_RCCL && c->trial_committed;
            if ((c->tune_phase == 1 || c->tune_phase == 2) && !committed) c->tune_phase = 0;
        }
        return GOL_OK;
    }
    case GOL_OPT_WORDS_PER_LANE:   // retired in 0.2 (the kernels fix their lane width): accepted, ignored
    case GOL_OPT_SPLIT:            // retired in 0.2 (boundary bands always split off): accepted, ignored
        return GOL_OK;
    default: return fail(c, GOL_EINVAL, "unknown option %d", option);
    }
}

int gol_get_option(gol_ctx *c, int option, int64_t *value) {
    if (!c || !value) return GOL_EINVAL;
    switch (option) {
    case GOL_OPT_CHUNK_ROWS: *value = c->chunk_rows; return GOL_OK;
    case GOL_OPT_KERNEL_TIMING: *value = c->timing; return GOL_OK;
    case GOL_OPT_OVERLAP: *value = c->overlap; return GOL_OK;
    case GOL_OPT_BYTE_CORE: *value = c->byte_core; return GOL_OK;
    case GOL_OPT_TEXT_BLOCK_BYTES: *value = c->text_block_bytes; return GOL_OK;
    case GOL_OPT_SCHEDULE_TRIAL: *value = c->trial_enabled ? (c->tune_phase == 3 ? 2 : 1) : 0; return GOL_OK;
    case GOL_OPT_INTERIOR_SPLIT: *value = c->split; return GOL_OK;
    case GOL_OPT_SCHED_TRACE: *value = c->tracing; return GOL_OK;
    case GOL_OPT_COMM_TIMING: *value = c->comm_timing; return GOL_OK;
    case GOL_OPT_HALO_EXCHANGE: *value = c->halo_exchange; return GOL_OK;
    case GOL_OPT_WORDS_PER_LANE: *value = c->layout == GOL_LAYOUT_BIT ? c->gw : 4; return GOL_OK;
    case GOL_OPT_SPLIT: *value = 1; return GOL_OK;
    default: return fail(c, GOL_EINVAL, "unknown option %d", option);
    }
}

int gol_init_glibc(gol_ctx *c, int mode, uint32_t seed) {
    if (!c) return GOL_EINVAL;
    // the generator's tables are allocated per call (an allocation can wait for a running probe)
    if (c->clk_running) return fail(c, GOL_ESTATE, "gol_init_glibc while the clock probe runs");
    int rc = sync_all(c, nullptr);
    if (rc) return rc;
    for (auto &s : c->slabs) {   // on the slab's stream (see alloc_slab), before the generator
        HIPCHK(c, hipSetDevice(s.device));
        const size_t bytes = (size_t)storage_rows(c, s) * c->pitch_bytes;
        HIPCHK(c, hipMemsetAsync(s.buf[0], 0, bytes, s.comp));
        HIPCHK(c, hipMemsetAsync(s.buf[1], 0, bytes, s.comp));
        HIPCHK(c, tr_ssync(c, s.comp));
    }
    c->cur = 0;
    c->generation = 0;
    c->step_index = 0;
    // a trial cut short (recording, or RCCL mode waiting for its agreement step,
    // which counts from the step index reset here): start it over on the new board
    if (c->tune_phase == 1 || (c->tune_phase == 2 && c->transport == GOL_XPORT_RCCL)) {
        if (!c->chunk_user) c->chunk_rows = c->tune_default;
        c->tune_phase = 0;
    }
    for (auto &s : c->slabs) {
        HIPCHK(c, hipSetDevice(s.device));
        rc = init_slab(c, s, mode, seed);
        if (rc) return rc;
    }
    return GOL_OK;
}

int gol_upload(gol_ctx *c, const uint8_t *host, int64_t ld) {
    if (!c || !host) return GOL_EINVAL;
    if (c->transport == GOL_XPORT_RCCL) {
        const Slab &s = c->slabs[0];
        return window_io(c, s.row0, 0, s.H, c->cols, const_cast<uint8_t *>(host) + s.row0 * ld, ld, true);
    }
    return window_io(c, 0, 0, c->rows, c->cols, const_cast<uint8_t *>(host), ld, true);
}

int gol_upload_window(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, const uint8_t *host,
                      int64_t ld) {
    if (!c || !host) return GOL_EINVAL;
    return window_io(c, row0, col0, nrows, ncols, const_cast<uint8_t *>(host), ld, true);
}

int gol_download(gol_ctx *c, uint8_t *host, int64_t ld) {
    if (!c || !host) return GOL_EINVAL;
    if (c->transport == GOL_XPORT_RCCL) {
        const Slab &s = c->slabs[0];
        return window_io(c, s.row0, 0, s.H, c->cols, host + s.row0 * ld, ld, false);
    }
    return window_io(c, 0, 0, c->rows, c->cols, host, ld, false);
}

int gol_download_window(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, uint8_t *host,
                        int64_t ld) {
    if (!c || !host) return GOL_EINVAL;
    return window_io(c, row0, col0, nrows, ncols, host, ld, false);
}

int64_t gol_text_bytes(int64_t nrows, int64_t ncols) {
    if (nrows < 0 || ncols < 0) return GOL_EINVAL;
    return nrows * (2 * ncols + 1);
}

int gol_format_text(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, char *out,
                    int64_t out_len) {
    if (!c || !out || out_len < gol_text_bytes(nrows, ncols)) return GOL_EINVAL;
    TextHost h;
    h.out = out;
    return text_io(c, row0, col0, nrows, ncols, h, false);
}

int gol_write_text(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, int fd) {
    if (!c || fd < 0) return GOL_EINVAL;
    TextHost h;
    h.fd = fd;
    return text_io(c, row0, col0, nrows, ncols, h, false);
}

int gol_parse_text(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, const char *text,
                   int64_t len) {
    if (!c || !text) return GOL_EINVAL;
    if (len != gol_text_bytes(nrows, ncols))
        return fail(c, GOL_EINVAL, "snapshot text is %lld bytes, a %lld x %lld window needs %lld", (long long)len,
                    (long long)nrows, (long long)ncols, (long long)gol_text_bytes(nrows, ncols));
    TextHost h;
    h.in = text;
    return text_io(c, row0, col0, nrows, ncols, h, true);
}

int gol_read_text(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, int fd) {
    if (!c || fd < 0) return GOL_EINVAL;
    TextHost h;
    h.fd = fd;
    return text_io(c, row0, col0, nrows, ncols, h, true);
}

int gol_step(gol_ctx *c, int64_t generations) {
    if (!c || generations < 0) return GOL_EINVAL;
    int rc = open_batch(c);
    if (rc) return rc;
    while (generations > 0) {
        int k = (int)std::min<int64_t>(c->K, generations);
        // a short last block of a k>8 board: the byte board's bit-sliced core
        // exists for some depths only (the SWAR kernel up to 8), the bit board's
        // chain for 16 and 32 (the pair kernel up to 8)
        if (k > 8 && c->layout == GOL_LAYOUT_BYTE && !bytebit_supported(k)) k = 8;
        if (k > 8 && c->layout == GOL_LAYOUT_BIT && !bit_depth_supported(k)) k = k >= 16 ? 16 : 8;
        rc = one_step(c, k);
        if (rc) return rc;
        generations -= k;
    }
    return GOL_OK;
}

int gol_sync(gol_ctx *c, double *elapsed_ms) {
    if (!c) return GOL_EINVAL;
    return sync_all(c, elapsed_ms);
}

int gol_popcount(gol_ctx *c, int64_t *live) {
    if (!c || !live) return GOL_EINVAL;
    int rc = sync_all(c, nullptr);
    if (rc) return rc;
    int64_t total = 0;
    for (auto &s : c->slabs) {
        HIPCHK(c, hipSetDevice(s.device));
        HIPCHK(c, hipMemsetAsync(s.d_count, 0, sizeof(unsigned long long), s.comp));
        HIPCHK(c, launch_popcount(s.buf[c->cur], c->pitch_bytes, c->hk, c->hk + s.H, c->row_bytes, s.d_count,
                                  c->layout == GOL_LAYOUT_BIT, s.comp));
        unsigned long long v = 0;
        HIPCHK(c, hipMemcpyAsync(&v, s.d_count, sizeof v, hipMemcpyDeviceToHost, s.comp));
        HIPCHK(c, tr_ssync(c, s.comp));
        total += (int64_t)v;
    }
    *live = total;
    return GOL_OK;
}

int gol_generation(gol_ctx *c, int64_t *generation) {
    if (!c || !generation) return GOL_EINVAL;
    *generation = c->generation;
    return GOL_OK;
}

int gol_sched_trace(gol_ctx *c, int64_t *ops, int64_t cap, int64_t *n) {
    if (!c || !n) return GOL_EINVAL;
    *n = (int64_t)(c->trace.size() / kTraceFields);
    // a truncated record would hide edges: refuse it rather than check half a schedule
    if (c->trace_full) return fail(c, GOL_ESTATE, "schedule trace overflowed (%zu ops): record fewer steps", kTraceMaxOps);
    if (!ops) return GOL_OK;
    if (cap < *n) return fail(c, GOL_EINVAL, "schedule trace holds %lld ops, buffer %lld", (long long)*n, (long long)cap);
    std::copy(c->trace.begin(), c->trace.end(), ops);
    c->trace.clear();
    return GOL_OK;
}

int gol_comm_time(gol_ctx *c, double *exchange_ms, double *bands_ms, int64_t *steps, int reset) {
    if (!c) return GOL_EINVAL;
    int rc = sync_all(c, nullptr);
    if (rc) return rc;
    double ex = 0.0, bd = 0.0;
    int64_t n = 0;
    for (auto &s : c->slabs) {
        HIPCHK(c, hipSetDevice(s.device));
        while (s.comm_live > 0)
            if (int rc2 = comm_harvest_one(c, s)) return rc2;
        // per slab and k-step: the slowest local slab's comm stream
        if (s.comm_steps > 0 && s.comm_exch_ms + s.comm_band_ms > ex + bd) {
            ex = s.comm_exch_ms;
            bd = s.comm_band_ms;
            n = s.comm_steps;
        }
        if (reset) {
            s.comm_exch_ms = s.comm_band_ms = 0.0;
            s.comm_steps = 0;
        }
    }
    if (exchange_ms) *exchange_ms = ex;
    if (bands_ms) *bands_ms = bd;
    if (steps) *steps = n;
    return GOL_OK;
}

int gol_kernel_time(gol_ctx *c, double *total_ms, int64_t *launches, int reset) {
    if (!c) return GOL_EINVAL;
    int rc = sync_all(c, nullptr);
    if (rc) return rc;
    if (total_ms) *total_ms = c->timed_ms;
    if (launches) *launches = c->timing ? c->timed_count : c->launch_count;
    if (reset) {
        c->timed_ms = 0.0;
        c->timed_count = 0;
        c->launch_count = 0;
    }
    return GOL_OK;
}

int gol_download_window_async(gol_ctx *c, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, uint8_t *host,
                              int64_t ld) {
    if (!c || !host) return GOL_EINVAL;
    return window_async(c, row0, col0, nrows, ncols, host, ld);
}

// The probe's stream: ONE per device for the whole process (never destroyed).
// A process gets few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and
// streams beyond them share one in order, so a stencil launch queued behind
// the probe wave on a shared queue would wait until the probe ends: a stream
// per context (three contexts in bench.py) made exactly that happen once.
static std::mutex probe_mu;
static std::vector<const gol_ctx *> probe_owner;   // per device: the context whose probe runs (or null)

static void probe_release(const gol_ctx *c) {
    std::lock_guard<std::mutex> lk(probe_mu);
    if ((int)probe_owner.size() > c->clk_device && probe_owner[c->clk_device] == c) probe_owner[c->clk_device] = nullptr;
}

static hipError_t probe_stream(int device, hipStream_t *out) {
    static std::vector<hipStream_t> streams;
    std::lock_guard<std::mutex> lk(probe_mu);
    if ((int)streams.size() <= device) streams.resize(device + 1, nullptr);
    if (!streams[device]) {
        int lo = 0, hi = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        // highest priority: the probe wave is dispatched ahead of queued stencil blocks
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&streams[device], hipStreamNonBlocking, hi);
        if (e != hipSuccess) return e;
    }
    *out = streams[device];
    return hipSuccess;
}

int gol_clock_start(gol_ctx *c, double max_ms) {
    if (!c || !(max_ms > 0.0)) return GOL_EINVAL;
    if (c->clk_running) return fail(c, GOL_ESTATE, "clock probe already running");
    c->clk_device = c->slabs[0].device;
    HIPCHK(c, hipSetDevice(c->clk_device));
    if (!c->clk_stream) {
        HIPCHK(c, probe_stream(c->clk_device, &c->clk_stream));
        HIPCHK(c, hipMalloc(&c->clk_out, 4 * sizeof(unsigned long long)));
        HIPCHK(c, hipHostMalloc(&c->clk_stop, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    }
    {   // the probe stream is the device's, shared by every context: one probe at a time,
        // or this one would queue behind another's and its span would include the wait
        std::lock_guard<std::mutex> lk(probe_mu);
        if ((int)probe_owner.size() <= c->clk_device) probe_owner.resize(c->clk_device + 1, nullptr);
        if (probe_owner[c->clk_device])
            return fail(c, GOL_ESTATE, "another context's clock probe runs on device %d", c->clk_device);
        probe_owner[c->clk_device] = c;
    }
    __atomic_store_n(c->clk_stop, 0, __ATOMIC_SEQ_CST);
    int *dflag = nullptr;
    // the real-time counter runs at 100 MHz: max_ms bounds the probe whatever the host does
    const unsigned long long ticks = (unsigned long long)(max_ms * 1e5);
    hipError_t e = hipHostGetDevicePointer((void **)&dflag, c->clk_stop, 0);
    if (e == hipSuccess) e = hipMemsetAsync(c->clk_out, 0, 4 * sizeof(unsigned long long), c->clk_stream);
    if (e == hipSuccess) e = launch_clock_probe(c->clk_out, dflag, ticks, c->clk_stream);
    if (e != hipSuccess) {
        probe_release(c);
        return fail(c, GOL_EHIP, "clock probe launch: %s", hipGetErrorString(e));
    }
    c->clk_running = true;
    return GOL_OK;
}

int gol_clock_stop(gol_ctx *c, double *mhz, double *span_ms) {
    if (!c) return GOL_EINVAL;
    if (!c->clk_running) return fail(c, GOL_ESTATE, "clock probe not running");
    __atomic_store_n(c->clk_stop, 1, __ATOMIC_SEQ_CST);
    c->clk_running = false;
    // the device's probe slot is released on every path below: a failed call must
    // not leave it owned (every later gol_clock_start on the device would refuse)
    hipError_t e = hipSetDevice(c->clk_device);
    if (e == hipSuccess) e = tr_ssync(c, c->clk_stream);
    probe_release(c);   // the probe wave has ended (or the stream failed: nothing of ours is queued)
    HIPCHK(c, e);
    unsigned long long v[4] = {0, 0, 0, 0};
    HIPCHK(c, hipMemcpy(v, c->clk_out, sizeof v, hipMemcpyDeviceToHost));
    const double real = (double)(v[3] - v[1]);
    if (mhz) *mhz = real > 0 ? (double)(v[2] - v[0]) / real * 100.0 : 0.0;
    if (span_ms) *span_ms = real * 1e-5;
    return GOL_OK;
}

int gol_rccl_selftest(int device, int64_t bytes, int reps, double *us_per_round, char *msg, int msg_len) {
    auto say = [&](const char *fmt, auto... xs) {
        if (msg && msg_len > 0) snprintf(msg, (size_t)msg_len, fmt, xs...);
    };
    if (bytes < 1 || reps < 1) return GOL_EINVAL;
    RcclApi &R = rccl();
    if (!R.ok) {
        say("%s", R.err.c_str());
        return GOL_ERCCL;
    }
    if (hipSetDevice(device) != hipSuccess) {
        say("hipSetDevice(%d) failed", device);
        return GOL_EHIP;
    }
    ncclUniqueId id;
    ncclComm_t comm = nullptr;
    ncclResult_t r = R.GetUniqueId(&id);
    if (r == ncclSuccess) r = R.CommInitRank(&comm, 1, id, 0);
    if (r != ncclSuccess) {
        say("ncclCommInitRank(1 rank): %s", R.GetErrorString(r));
        return GOL_ERCCL;
    }
    // two halo messages per round, as a rank with two neighbours sends (top and
    // bottom k rows), here both to itself: rank 0's only peer
    const size_t n = (size_t)bytes;
    std::vector<uint8_t> want(2 * n), got(2 * n);
    for (size_t i = 0; i < 2 * n; ++i) want[i] = (uint8_t)((i * 131u + 7u) ^ (i >> 9));
    uint8_t *src = nullptr, *dst = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = GOL_OK;
    auto hip = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == GOL_OK) {
            say("%s: %s", what, hipGetErrorString(e));
            rc = GOL_EHIP;
        }
        return rc == GOL_OK;
    };
    auto nccl = [&](ncclResult_t e, const char *what) {
        if (e != ncclSuccess && rc == GOL_OK) {
            say("%s: %s", what, R.GetErrorString(e));
            rc = GOL_ERCCL;
        }
        return rc == GOL_OK;
    };
    if (hip(hipMalloc(&src, 2 * n), "hipMalloc") && hip(hipMalloc(&dst, 2 * n), "hipMalloc") &&
        hip(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate") &&
        hip(hipEventCreate(&e0), "hipEventCreate") && hip(hipEventCreate(&e1), "hipEventCreate") &&
        hip(hipMemcpy(src, want.data(), 2 * n, hipMemcpyHostToDevice), "hipMemcpy") &&
        hip(hipMemsetAsync(dst, 0, 2 * n, st), "hipMemsetAsync") &&   // on st: ordered before the receives
        hip(hipEventRecord(e0, st), "hipEventRecord")) {
        for (int i = 0; i < reps && rc == GOL_OK; ++i) {
            nccl(R.GroupStart(), "ncclGroupStart");
            nccl(R.Send(src, n, ncclUint8, 0, comm, st), "ncclSend");
            nccl(R.Recv(dst, n, ncclUint8, 0, comm, st), "ncclRecv");
            nccl(R.Send(src + n, n, ncclUint8, 0, comm, st), "ncclSend");
            nccl(R.Recv(dst + n, n, ncclUint8, 0, comm, st), "ncclRecv");
            nccl(R.GroupEnd(), "ncclGroupEnd");
        }
        if (hip(hipEventRecord(e1, st), "hipEventRecord") && hip(hipStreamSynchronize(st), "hipStreamSynchronize") &&
            hip(hipMemcpy(got.data(), dst, 2 * n, hipMemcpyDeviceToHost), "hipMemcpy")) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (us_per_round) *us_per_round = ms * 1e3 / reps;
            size_t bad = 0;
            for (size_t i = 0; i < 2 * n; ++i) bad += got[i] != want[i];
            if (bad) {
                say("%zu of %zu bytes differ after self send/recv", bad, 2 * n);
                rc = GOL_ERCCL;
            } else {
                say("ok: %d rounds of 2 x %lld B self send/recv (RCCL from %s)", reps, (long long)bytes, R.source);
            }
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (src) (void)hipFree(src);
    if (dst) (void)hipFree(dst);
    R.CommDestroy(comm);
    return rc;
}

const char *gol_last_error(gol_ctx *c) { return c ? c->err.c_str() : "null context"; }

void gol_destroy(gol_ctx *c) {
    if (!c) return;
    for (auto &s : c->slabs) {
        (void)hipSetDevice(s.device);
        if (s.comp) (void)tr_ssync(c, s.comp);
        if (s.comm) (void)tr_ssync(c, s.comm);
        for (int j = 0; j < s.nx; ++j) (void)tr_ssync(c, s.part[j]);
    }
    if (c->comm && rccl().ok) rccl().CommDestroy(c->comm);
    for (auto &t : c->timed) {
        (void)hipSetDevice(t.device);
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (size_t i = 0; i < c->tune_ev.size(); ++i) {
        (void)hipSetDevice(c->slabs[i / (kTuneN + 1)].device);
        (void)hipEventDestroy(c->tune_ev[i]);
    }
    for (auto &b : c->staging) {   // the streams are idle now
        (void)hipSetDevice(b.device);
        (void)hipFree(b.dtmp);
        (void)hipHostFree(b.pinned);
    }
    if (c->agree_dev) {
        (void)hipSetDevice(c->slabs[0].device);
        (void)hipFree(c->agree_dev);
        (void)hipHostFree(c->agree_host);
    }
    if (c->clk_stream) {
        (void)hipSetDevice(c->clk_device);
        if (c->clk_running) {   // only this context's own probe is waited for (the stream is the process's)
            __atomic_store_n(c->clk_stop, 1, __ATOMIC_SEQ_CST);
            (void)tr_ssync(c, c->clk_stream);
            probe_release(c);
        }
        (void)hipFree(c->clk_out);
        (void)hipHostFree(c->clk_stop);
    }
    for (auto &s : c->slabs) free_slab(s);
    delete c;
}

} // extern "C"
