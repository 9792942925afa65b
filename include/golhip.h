/*
 * golhip.h — C ABI of the MI355X-native Game-of-Life engine (libgolhip.so).
 *
 * The reference (arthurdecloedt/mpi) has no plugin or FFI API; its hot path is
 * two C++ free functions called from the generation loop of main():
 *
 *   void updateBoard(bool **board, bool **nboard, distrOpt options);            main.cpp:93-103
 *   void distr_borders(bool **board, neighbours nbr, MPI_Comm, distrOpt &);     main.cpp:36-65
 *   void updateBoard(bool **board, distrOpt options);            main_serial.cpp:45-71
 *   void initializeBoard(bool **board, distrOpt options[, int rank]);
 *                                        main.cpp:68-77, main_serial.cpp:34-43
 *
 * plus the MPI runtime around them (MPI_Init/Cart_create/Bcast/Barrier/Reduce,
 * main.cpp:154-164, 233-254, 280-324).  This header is the seam that replaces
 * all of it: one opaque context owns the device boards (ping-pong buffers per
 * row slab), the HIP streams and, for one-process-per-GPU runs, an RCCL
 * communicator for the halo rows.  Plain C types only; no torch, no C++.
 *
 * Conventions
 *  - Every function returns GOL_OK (0) or a negative GOL_E* code; the message
 *    is in gol_last_error(ctx).  No exception crosses the ABI.  (The reference
 *    has no error path beyond MPI_Abort, main.cpp:176-197.)
 *  - Host buffers are caller-owned 0/1 bytes, row-major, leading dimension
 *    `ld` (bytes).  Device memory is owned by the context.
 *  - Coordinates are GLOBAL (row, col) of the rows×cols grid.
 *  - A context is not thread-safe; one host thread drives it.
 *  - gol_step is asynchronous (enqueues on the context's HIP streams);
 *    gol_sync / gol_download / gol_popcount synchronise.
 */
#ifndef GOLHIP_H
#define GOLHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Cell layouts in HBM */
#define GOL_LAYOUT_BYTE 0 /* 1 byte per cell (0/1); row pitch = 256·n + 512 B (channel spread) */
#define GOL_LAYOUT_BIT 1  /* 1 bit per cell; column groups of G u32 words, column 32G·g+G·j+w in
                             word G·g+w, bit j (interleaved: neighbours share a bit); G = 4 for
                             tblock_k = 8, else 2.  Never visible through this ABI (host I/O is
                             0/1 bytes) */

/* Boundary conventions */
#define GOL_DEAD 0          /* non-periodic B3/S23 (main.cpp, P=1; periods {0,0} main.cpp:243) */
#define GOL_SERIAL_COMPAT 1 /* main_serial.cpp:45-71: DEAD on the top-left (n-1)², last row/col 0 */
#define GOL_MESH_COMPAT 2   /* main.cpp on a √P×√P mesh, P=mesh_m²: swapped column halos
                               (main.cpp:51-54); any layout and tblock_k (stored as a dead-boundary
                               board with its column blocks in reverse order) */

/* Seeded initialisation (glibc rand()%3==0, main.cpp:73 / main_serial.cpp:40) */
#define GOL_INIT_STREAM 0 /* srand(seed), row-major over the global grid (MPI np=1 with seed 0≡1) */
#define GOL_INIT_SERIAL 1 /* main_serial.cpp:34-43 with srand(seed): cell (r,c) ← draw (r+1)·n+c+1 */
#define GOL_INIT_MESH 2   /* main.cpp:68-77: block (cx,cy) ← srand(seed + cx·m + cy) */
#define GOL_SERIAL_SEED 1804289383u /* glibc's first rand() with no srand (main_serial.cpp:150) */

/* Halo transports */
#define GOL_XPORT_NONE 0 /* one slab */
#define GOL_XPORT_PEER 1 /* several slabs in this process: hipMemcpyAsync D2D / peer over xGMI */
#define GOL_XPORT_RCCL 2 /* one slab per process: ncclSend/ncclRecv over xGMI */

/* Error codes */
#define GOL_OK 0
#define GOL_EINVAL (-1)
#define GOL_EHIP (-2)
#define GOL_ERCCL (-3)
#define GOL_ENOMEM (-4)
#define GOL_EUNSUPPORTED (-5)
#define GOL_ESTATE (-6)

#define GOL_UNIQUE_ID_BYTES 128

/* gol_set_option keys */
#define GOL_OPT_CHUNK_ROWS 1    /* rows per wave chunk; -r: exactly r rounds of resident waves;
                                   -(100+r): guided static schedule, r rounds of halving chunks.
                                   0 (0.1's work queue) is GOL_EUNSUPPORTED since 0.2.
                                   Setting it turns off the bit k=8 schedule trial; reading it
                                   returns the policy in force (the trial's pick once known) */
#define GOL_OPT_KERNEL_TIMING 2 /* 1: bracket every main-kernel launch with hipEvents (at most 1024
                                   pairs in flight; older ones are harvested as new ones are needed) */
#define GOL_OPT_WORDS_PER_LANE 3 /* retired in 0.2 (lane widths are fixed per kernel): set is a no-op */
#define GOL_OPT_OVERLAP 4       /* multi-slab: 1 = interior kernel overlapped with halo exchange (default) */
#define GOL_OPT_BYTE_CORE 5     /* byte layout: 1 = bit-sliced core where tblock_k is 4, 8, 12, 16, 20,
                                   24, 28, 32, 48 or 64 (default; the kernel per depth is the library's
                                   pick); 2 = its one-wave-per-strip kernel (k <= 32); 3 = its chain
                                   kernel (a workgroup of 2-4 waves per strip splitting the stages,
                                   k = 24, 32, 48, 64; 48 and 64 always run it); 4 = the byte board
                                   through the bit board's pair waves (a pack wave, k / 8 pair waves,
                                   an unpack wave per strip; k = 16, 32, 48, other depths as 1);
                                   0 = byte-SWAR kernel (tblock_k <= 8) */
#define GOL_OPT_SPLIT 6         /* retired in 0.2 (boundary bands are always split off): set is a no-op */
#define GOL_OPT_TEXT_BLOCK_BYTES 10 /* snapshot text: bytes per pinned staging block (default 64 MiB) */
#define GOL_OPT_SCHEDULE_TRIAL 11 /* bit layout, tblock_k = 8, no caller chunk policy: 1 (default) = after
                                     400 k-steps, time the policies -1/-2/-3 (split interior, the k = 8
                                     default) or -104/-6/-3 (unsplit) on 24 real steps (results are
                                     unaffected) and keep the fastest (the default -1 resp. -104 unless
                                     another is > 4 % resp. 1.5 % faster); never blocks the host (the
                                     pick applies once its events have completed); 0 = off.  Reads 2
                                     once the pick is made.  RCCL mode: 16 k-steps after the trial the
                                     ranks take the MAX of their medians (ncclAllReduce on the context's
                                     communicator, the same k-step on every rank) and all keep the same
                                     policy; a short k-step during the trial restarts it.  RCCL mode:
                                     this option and GOL_OPT_CHUNK_ROWS are COLLECTIVE before the trial
                                     starts (set them alike on every rank before k-step 400, or a rank
                                     without the trial leaves the others in the allreduce); set on one
                                     rank once the trial is recording, they do not take that rank out
                                     of it: it joins the agreement and then keeps its own setting */

#define GOL_OPT_INTERIOR_SPLIT 12 /* P = 1 .. 4: a slab's interior runs as P launches on P streams
                                     with a 2k-row seam band at every cut on the halo stream, so the
                                     next step's parts start while this step's parts drain (a slab
                                     takes the most parts with >= 32·tblock_k interior rows each,
                                     down to one).
                                     Default 2 for bit layout at tblock_k = 8 with at most 4 slabs per
                                     device whose 3 streams each (+ the clock probe's) fit the process's
                                     hardware queues (3 x slabs + 1 <= GPU_MAX_HW_QUEUES, HIP default 4:
                                     one slab per device), 1 otherwise.  Setting it synchronises the context; with no
                                     caller chunk policy the k = 8 default policy follows it (-1 split,
                                     -104 unsplit) and a trial under way starts over.  RCCL mode: like
                                     GOL_OPT_SCHEDULE_TRIAL, collective before the trial starts; set on
                                     one rank while the trial records, the rank's slots keep timing
                                     the trial's candidates, it joins the agreement, and then keeps
                                     the new split's default policy */

#define GOL_OPT_SCHED_TRACE 13  /* diagnostic: 1 = record the enqueue order of the step path (event
                                   records and waits, host syncs, board reads/writes per stream) for
                                   gol_sched_trace; setting it clears the record */

#define GOL_OPT_COMM_TIMING 14  /* multi-slab / RCCL mode: 1 = time each local slab's comm-stream work
                                   per k-step with hipEvents — the halo exchange (ncclSend/Recv group or
                                   peer copies) and the boundary + seam bands — read by gol_comm_time */

#define GOL_OPT_HALO_EXCHANGE 15 /* diagnostic: 0 = skip the halo exchange (no rows move between slabs,
                                    so results at slab seams are WRONG): the same slabs, bands and
                                    interior launches without communication, for an interior-only step
                                    time beside the real one (bench.py's N > 1 line); 1 = default.
                                    RCCL mode: collective (set it alike on every rank) */

typedef struct gol_ctx gol_ctx;

/* Single process.  The grid is cut into n_gpus row slabs; slab s lives on HIP
 * device s % (visible devices), so n_gpus > devices exercises the multi-slab
 * path on one GPU.  tblock_k = generations fused per launch and halo depth.
 * Replaces MPI_Init/Dims_create/Cart_create (main.cpp:154-254). */
int gol_create(gol_ctx **out, int64_t rows, int64_t cols, int n_gpus, int layout, int boundary,
               int mesh_m, int tblock_k);

/* One process per GPU (torchrun-style).  This context owns slab `rank` of
 * `world` on HIP device `device`; halos go over RCCL.  `unique_id` is the
 * GOL_UNIQUE_ID_BYTES blob from gol_get_unique_id() on rank 0, broadcast by
 * the caller.  Replaces MPI_Init/Cart_create/Cart_shift (main.cpp:154-254). */
int gol_create_rank(gol_ctx **out, int64_t rows, int64_t cols, int rank, int world, int device,
                    const uint8_t *unique_id, int layout, int boundary, int mesh_m, int tblock_k);
int gol_get_unique_id(uint8_t *unique_id);

/* Row range of slab `rank` of `world` (host-only arithmetic, no GPU needed). */
int gol_slab_plan(int64_t rows, int world, int rank, int64_t *row0, int64_t *nrows);

int gol_set_option(gol_ctx *ctx, int option, int64_t value);
int gol_get_option(gol_ctx *ctx, int option, int64_t *value);

/* On-device glibc-rand initialisation with jump-ahead, bit-identical to the
 * reference's initializeBoard (main.cpp:68-77, main_serial.cpp:34-43). */
int gol_init_glibc(gol_ctx *ctx, int mode, uint32_t seed);

/* Host 0/1 bytes → device (whole grid / a window).  For a rank context only
 * the rows of its slab are taken.  Cells outside the active region of the
 * boundary convention (SERIAL_COMPAT: last row and column) are stored as 0. */
int gol_upload(gol_ctx *ctx, const uint8_t *host, int64_t ld);
int gol_upload_window(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                      const uint8_t *host, int64_t ld);

/* Advance `generations` generations: updateBoard + pointer swap + distr_borders
 * of main.cpp:291-305, `tblock_k` generations per launch and per halo exchange. */
int gol_step(gol_ctx *ctx, int64_t generations);

/* Wait for all enqueued work.  elapsed_ms (may be NULL) = device time from the
 * first gol_step after the previous sync to completion (hipEvents). */
int gol_sync(gol_ctx *ctx, double *elapsed_ms);

/* Device → host 0/1 bytes (whole grid / a window; rank contexts: own slab rows only). */
int gol_download(gol_ctx *ctx, uint8_t *host, int64_t ld);
int gol_download_window(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                        uint8_t *host, int64_t ld);
/* Asynchronous window copy: enqueued behind every gol_step so far (no host
 * wait, no device idle); `host` (caller-owned, valid until then) is filled by
 * the next synchronising call (gol_sync, gol_popcount, gol_download*, ...).
 * Rows must be held by this context.  Snapshot-at-a-generation without a
 * pipeline drain (bench.py takes its verification cone this way). */
int gol_download_window_async(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                              uint8_t *host, int64_t ld);

/* Snapshot text — the body of a `.gol` part file as writeBoardToFile writes it
 * (main.cpp:106-129, main_serial.cpp:74-95; read back by
 * gol_visualization.py:29-33): for every row of the window one "0\t" or "1\t"
 * per cell, then "\n".  The two header lines ("firstRow lastRow" /
 * "firstCol lastCol") stay with the caller.  Formatting and parsing run on the
 * device; the host moves finished bytes (pipelined through pinned buffers).
 * Every row of the window must be held by this context (a rank writes its own
 * part, as in the reference).
 *   gol_text_bytes   bytes of an nrows×ncols body: nrows·(2·ncols+1)
 *   gol_format_text  body → caller memory (out_len >= gol_text_bytes)
 *   gol_write_text   body → file descriptor (write(2), sequential)
 *   gol_parse_text   caller memory (exactly gol_text_bytes) → cells (snapshot resume)
 *   gol_read_text    file descriptor (read(2), positioned at the body) → cells
 * Malformed text (any byte other than the pattern above) is GOL_EINVAL with
 * the offending offset in gol_last_error; the window may then be partly
 * written.  No reference counterpart reads snapshots back. */
int64_t gol_text_bytes(int64_t nrows, int64_t ncols);
int gol_format_text(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, char *out,
                    int64_t out_len);
int gol_write_text(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, int fd);
int gol_parse_text(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, const char *text,
                   int64_t len);
int gol_read_text(gol_ctx *ctx, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, int fd);

/* Live cells held by this context (all its slabs). */
int gol_popcount(gol_ctx *ctx, int64_t *live);

/* Generations advanced so far. */
int gol_generation(gol_ctx *ctx, int64_t *generation);

/* With GOL_OPT_KERNEL_TIMING: summed device time (ms) and count of main-kernel
 * launches since the last reset (the hot kernel's average = total / count).
 * Without it: total 0 and the launch count (counted on the host). */
int gol_kernel_time(gol_ctx *ctx, double *total_ms, int64_t *launches, int reset);

/* With GOL_OPT_COMM_TIMING: device time (ms) the comm stream spent in the halo
 * exchange (*exchange_ms) and in the boundary and seam bands (*bands_ms), summed
 * over *steps k-steps since the last reset, for the local slab whose sum is
 * largest.  Synchronises.  The halo path of main.cpp:291-305 (distr_borders,
 * main.cpp:36-65, plus the per-generation MPI_Barrier) is what this times. */
int gol_comm_time(gol_ctx *ctx, double *exchange_ms, double *bands_ms, int64_t *steps, int reset);

/* Diagnostic (GOL_OPT_SCHED_TRACE): *n = ops recorded; with ops != NULL and
 * cap >= *n, copies them (7 int64 each: kind 1 record / 2 wait / 3 stream sync
 * / 4 event sync / 5 read / 6 write, stream, event, slab, buffer, row0, row1 —
 * storage rows, all columns) and clears the record.  The record holds at
 * most 2^22 ops; past that GOL_ESTATE (set the option again to restart it).  A happens-before check of
 * the streams' order, the event edges and the host syncs over these ops finds
 * any two accesses of the same rows, one a write, left unordered
 * (tests/sched_race.py).  Reference analogue: none (the MPI code is blocking). */
int gol_sched_trace(gol_ctx *ctx, int64_t *ops, int64_t cap, int64_t *n);

/* Clock probe (measurement): gol_clock_start launches a one-wave kernel on a
 * stream of its own that stamps the shader-clock counter (s_memtime) and the
 * 100-MHz real-time counter, sleeps between polls of a host flag, and stops at
 * gol_clock_stop or after max_ms.  mhz = shader cycles / real time over that
 * span: the clock the chip ran at while the enqueued steps executed (the
 * probe itself holds one wave slot of one CU).  While it runs nothing is
 * allocated on the device: window copies (gol_download_window[_async],
 * gol_upload_window) use the context's pooled staging (GOL_ESTATE if no pooled
 * buffer of the size is free: copy one window of that size beforehand), and
 * the snapshot-text calls and gol_init_glibc return GOL_ESTATE. */
int gol_clock_start(gol_ctx *ctx, double max_ms);
int gol_clock_stop(gol_ctx *ctx, double *mhz, double *span_ms);

/* Transport self-test (no context): a 1-rank RCCL communicator on `device`
 * (the library's own dlopen'ed RCCL binding, as gol_create_rank uses it) runs
 * `reps` groups of two ncclSend/ncclRecv pairs of `bytes` each to itself on a
 * non-blocking stream — the halo exchange of a rank with two neighbours — and
 * checks every byte.  us_per_round (may be NULL): device time per group.
 * msg (may be NULL): outcome text. */
int gol_rccl_selftest(int device, int64_t bytes, int reps, double *us_per_round, char *msg, int msg_len);

const char *gol_last_error(gol_ctx *ctx);
void gol_destroy(gol_ctx *ctx);

/* Library / build identification (e.g. "golhip gfx950"). */
const char *gol_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GOLHIP_H */
