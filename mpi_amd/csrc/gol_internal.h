// Internal interface between the runtime (gol_runtime.cpp) and the gfx950
// kernels (gol_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gol {

// Bit layout = interleaved groups of gw u32 words (gw = 2 or 4): a group holds
// 32·gw consecutive columns, column c lives in word gw·(c / 32gw) + c % gw,
// bit (c % 32gw) / gw.  In a group a cell's left and right neighbours are the
// same bit of the adjacent word (one funnel shift at the group ends only), so
// the wider the group, the fewer lane moves per word.  A context's group width
// is fixed at creation (bit_group_words: 4 for the k = 8 pair kernel, 2
// otherwise); rows are padded to whole 128-column blocks (4 words) either way.
constexpr int kGroupWords = 2;   // the width of every kernel but the k = 8 pair kernel's
__host__ __device__ inline int64_t bit_word(int64_t c, int gw) {
    const int lg = gw == 4 ? 2 : 1;
    return ((c >> (5 + lg)) << lg) + (c & (gw - 1));
}
__host__ __device__ inline int bit_pos(int64_t c, int gw) {
    const int lg = gw == 4 ? 2 : 1;
    return (int)((c & (32 * gw - 1)) >> lg);
}

// Geometry of one pipelined-stencil launch.  Rows are STORAGE rows of a slab
// buffer: [0,hk) top halo, [hk,hk+H) slab rows, [hk+H,hk+H+hk) bottom halo.
struct StencilArgs {
    const void *src;
    void *dst;
    int64_t pitch;      // row pitch in u32 words
    int nunits;         // u32 words per row that carry active cells (bit: whole 4-word groups) / dwords (byte)
    uint32_t last_mask; // byte layout: 0x01 per active cell byte of the last active dword
    int64_t active_cols; // bit layout: columns [0, active_cols) are live (masks per interleaved word)
    int row_lo, row_hi; // storage rows outside [row_lo,row_hi) are dead at every generation
    int out_r0, out_r1; // storage rows produced by this launch
    int chunk_rows;     // output rows per wave chunk (see plan_items in gol_kernels.hip)
    int gw;             // bit layout: words per column group (2 or 4)
};

// Bit layout: the group width of a context fusing K generations per launch.
int bit_group_words(int K);

// Bit layout, `gens` generations fused (1..8, or 16 / 32: the chain of pair
// waves on 4-word groups), a.gw-word groups.
bool bit_depth_supported(int gens);
hipError_t launch_bit_pipe(const StencilArgs &a, int gens, hipStream_t s);
// Byte layout, `gens` generations fused (1 <= gens <= 8), 16 cells per lane.
hipError_t launch_byte_pipe(const StencilArgs &a, int gens, hipStream_t s);
// Byte layout with the bit-sliced core (bytebit_pipe_kernel): byte-per-cell in
// HBM, gens in {4, 8, ..., 32, 48, 64} generations fused per launch.
bool bytebit_supported(int gens);
// core: which bit-sliced kernel (GOL_OPT_BYTE_CORE): the default per depth, one
// wave per strip (bytebit_pipe_kernel, k <= 32) or a chain of waves per strip
// (bytebit_coop_kernel, k in {24, 32, 48, 64}; k = 48, 64 have only the chain).
enum { kByteCoreDefault = 1, kByteCoreWave = 2, kByteCoreChain = 3, kByteCorePair = 4 };
bool bytebit_chain_default(int gens);
hipError_t launch_bytebit_pipe(const StencilArgs &a, int gens, hipStream_t s, int core = kByteCoreDefault);

// glibc-rand initialisation: one "unit" = a run of `len` consecutive draws of
// one stream written to storage row `row` starting at column `col0`.
struct InitUnit {
    int64_t row;
    int32_t col0;
    int32_t len;
    uint32_t w[31]; // raw generator values x_o .. x_{o+30} at the unit's first draw
    uint32_t pad;
};
// mats: T jump matrices (31×31, row-major) A^{t·seg}, t = 0..T-1.
hipError_t launch_init_units(const InitUnit *units, int nunits, const uint32_t *mats, int T, int seg,
                             void *dst, int64_t pitch_bytes, int bit_layout, hipStream_t s);

// Linear init words (bit i = column 32w+i) -> gw-word groups, rows [r0, r0+nrows)
// of `blocks` 128-column blocks.
hipError_t launch_interleave_rows(const uint32_t *lin, uint32_t *out, int64_t pitch_words, int64_t r0,
                                  int64_t nrows, int64_t blocks, int gw, hipStream_t s);
// Layout conversion of a window (dst/src host-staging buffers are device memory).
hipError_t launch_pack_window(const uint8_t *bytes, int64_t ld, uint32_t *words, int64_t pitch_words,
                              int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                              int64_t active_cols, int gw, hipStream_t s);
hipError_t launch_unpack_window(const uint32_t *words, int64_t pitch_words, uint8_t *bytes, int64_t ld,
                                int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, int gw, hipStream_t s);
// Snapshot text (main.cpp:106-129 writeBoardToFile body): per row, "0\t"/"1\t" per
// cell then "\n" — rowlen = 2·ncols + 1 bytes; logical column c is read from
// storage column phys(c) (perm_m > 1: MESH_COMPAT's reversed blocks of perm_L).  format: storage rows
// [srow0, srow0+nrows), columns [col0, col0+ncols) of a slab buffer (bit words
// or bytes, pitch in bytes) -> text.  parse: text -> 0/1 bytes (ld); *err
// (preset to ~0) receives err_base + the lowest offending byte offset (atomicMin).
// bit_gw: 0 = byte layout, else the bit layout's group width.
hipError_t launch_format_text(const void *buf, int64_t pitch_bytes, int bit_gw, int64_t srow0, int64_t col0,
                              int64_t nrows, int64_t ncols, int perm_m, int64_t perm_L, char *text, hipStream_t s);
hipError_t launch_parse_text(const char *text, int64_t nrows, int64_t ncols, uint8_t *cells, int64_t ld,
                             int64_t err_base, unsigned long long *err, hipStream_t s);

// Byte layout upload: every nonzero byte of the window becomes 1 (bool cells).
hipError_t launch_normalize_bytes(uint8_t *base, int64_t pitch_bytes, int64_t nrows, int64_t ncols, hipStream_t s);

// Clock probe: one wave stamps (s_memtime, s_memrealtime) at start and end into
// out[0..3]; it ends when *stop (host-visible) is nonzero or after max_ticks of
// the 100-MHz real-time counter.
hipError_t launch_clock_probe(unsigned long long *out, const int *stop, unsigned long long max_ticks, hipStream_t s);

// Live-cell count of storage rows [r0,r1), accumulated into *acc.
hipError_t launch_popcount(const void *buf, int64_t pitch_bytes, int64_t r0, int64_t r1,
                           int64_t row_bytes, unsigned long long *acc, int bit_layout, hipStream_t s);

} // namespace gol
