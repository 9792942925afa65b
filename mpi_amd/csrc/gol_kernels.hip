// gol_kernels.hip — hand-written gfx950 (CDNA4) kernels for the Game-of-Life
// generation update (the reference's updateBoard/next, main.cpp:79-103 and
// main_serial.cpp:45-71) and its initialisation (initializeBoard,
// main.cpp:68-77 / main_serial.cpp:34-43).
//
// Design: every stencil kernel is a *register pipeline*.  One
// wave owns a column strip (64 lanes × V u32 words, lanes 0 and 63 are halo
// lanes that are computed but not stored) and walks down a chunk of rows.
// Each row is loaded from HBM exactly once per launch (coalesced V·4-byte
// vectors, prefetched 3 rows ahead) and each output row is stored once.  K
// generations are fused: stage g keeps a 3-row window of generation g-1 in
// VGPRs, so K generations cost one HBM read + one HBM write per cell.
// Horizontal neighbours within a lane come from v_alignbit funnel shifts, and
// across lanes from DPP wave_shr:1 / wave_shl:1 row moves (no LDS round trip).
//
//  * bit layout : 32 cells per word; a row's horizontal 3-sums are two bit-
//                 sliced planes (h0,h1); the vertical 9-sum and the B3/S23
//                 rule are 8 v_bitop3 ops per 32 cells.
//  * byte layout: 1 cell per byte in HBM.  Default: the bytebit kernel packs
//                 each loaded row into bit planes in registers, runs the bit
//                 pipeline (k up to 32) and unpacks before the store; the SWAR
//                 kernel (v_add3_u32 sums of 4 cells per dword) serves k <= 8
//                 when asked for and MESH_COMPAT.
#include "gol_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <map>
#include <mutex>

namespace gol {

// ------------------------------------------------------------- wave helpers

// lane i <- lane i-1 (lane 0 <- 0).  DPP wave_shr:1, a GFX9 full-wave row move.
__device__ __forceinline__ uint32_t from_left_lane(uint32_t x) {
    return __builtin_amdgcn_update_dpp(0u, x, 0x138, 0xf, 0xf, false);
}
// lane i <- lane i+1 (lane 63 <- 0).  DPP wave_shl:1.
__device__ __forceinline__ uint32_t from_right_lane(uint32_t x) {
    return __builtin_amdgcn_update_dpp(0u, x, 0x130, 0xf, 0xf, false);
}
// (hi:lo) >> s, low 32 bits — one v_alignbit_b32.
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

// XCD-aware block remap: consecutive logical blocks land on one XCD (blocks are
// dealt round-robin over the 8 XCDs), so neighbouring strips/chunks share an L2.
// Bijective for any nblocks.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7, x = b & 7, i = b >> 3;
    return (x < r) ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 3-input boolean ops as single v_bitop3_b32 (truth tables over a=0xF0, b=0xCC, c=0xAA).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// Cross-lane neighbour words of the bit stencil.  GOL_XLANE 0: DPP wave_shr/shl
// (a half-rate VALU op); 1: ds_bpermute_b32 (the LDS pipe, no VALU slot; lane
// 0 / 63 wrap around, which only touches the halo lanes).
#ifndef GOL_XLANE
#define GOL_XLANE 0
#endif
template <typename ST>
__device__ __forceinline__ uint32_t xlane_from_left(uint32_t x, const ST &st) {
#if GOL_XLANE == 1
    return (uint32_t)__builtin_amdgcn_ds_bpermute(st.perm_l, (int)x);
#else
    (void)st;
    return __builtin_amdgcn_update_dpp(0u, x, 0x138, 0xf, 0xf, true);   // wave_shr:1
#endif
}
template <typename ST>
__device__ __forceinline__ uint32_t xlane_from_right(uint32_t x, const ST &st) {
#if GOL_XLANE == 1
    return (uint32_t)__builtin_amdgcn_ds_bpermute(st.perm_r, (int)x);
#else
    (void)st;
    return __builtin_amdgcn_update_dpp(0u, x, 0x130, 0xf, 0xf, true);   // wave_shl:1
#endif
}

// Raw buffer I/O.  The resource is wave-uniform; an offset >= num_records reads
// 0 / drops the store, so invalid rows and lanes need no branch and no select,
// and every load is issued unconditionally (exact vmcnt accounting: the
// compiler can keep the 3-row prefetch in flight).
constexpr uint32_t kOOB = 0x40000000u;   // > any window's num_records
// cache-policy bits of the stencil's row loads / stores (gfx950 aux: 2 = nt)
#ifndef GOL_LOAD_AUX
#define GOL_LOAD_AUX 0
#endif
#ifndef GOL_STORE_AUX
#define GOL_STORE_AUX 0
#endif

template <int V>
__device__ __forceinline__ void buf_load(uint32_t (&d)[V], __amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (V == 1) {
        d[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, GOL_LOAD_AUX);
    } else if constexpr (V == 2) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, GOL_LOAD_AUX);
        d[0] = t.x; d[1] = t.y;
    } else {
        static_assert(V % 4 == 0, "V must be 1, 2 or a multiple of 4");
#pragma unroll
        for (int q = 0; q < V / 4; ++q) {
            const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * q, 0, GOL_LOAD_AUX);
            d[4 * q] = t.x; d[4 * q + 1] = t.y; d[4 * q + 2] = t.z; d[4 * q + 3] = t.w;
        }
    }
}
template <int V>
__device__ __forceinline__ void buf_store(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint32_t (&s)[V]) {
    if constexpr (V == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(s[0], r, off, 0, GOL_STORE_AUX);
    } else if constexpr (V == 2) {
        u32x2 t; t.x = s[0]; t.y = s[1];
        __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, GOL_STORE_AUX);
    } else {
#pragma unroll
        for (int q = 0; q < V / 4; ++q) {
            u32x4 t; t.x = s[4 * q]; t.y = s[4 * q + 1]; t.z = s[4 * q + 2]; t.w = s[4 * q + 3];
            __builtin_amdgcn_raw_buffer_store_b128(t, r, off + 16 * q, 0, GOL_STORE_AUX);
        }
    }
}

// Per-wave geometry shared by both pipelines.  Everything that is the same for
// the whole wave is made provably uniform (readfirstlane) so it lives in SGPRs.
template <int V>
struct Strip {
    uint32_t ld_off;     // lane byte offset for loads (kOOB if outside the row pitch)
    uint32_t st_off;     // lane byte offset for stores (kOOB for halo lanes / inactive words)
    uint32_t mask[V];    // active-cell mask per word
    int R0, R1;          // output rows of this wave's chunk (uniform)
    int base_row;        // first row of the buffer window = R0 - K (uniform)
    int perm_l, perm_r;  // ds_bpermute byte addresses of lanes i-1 / i+1 (GOL_XLANE 1)
    __amdgpu_buffer_rsrc_t src, dst;

    // One work item: column strip `strip`, output rows [r0, r1).
    // full == 0: bit layout (quad-interleaved groups, masks from active_cols);
    // otherwise the byte layout's per-dword cell mask (0x01010101).
    __device__ __forceinline__ void setup(const StencilArgs &a, int K, int strip, int r0, int r1, uint32_t full) {
        const int lane = threadIdx.x & 63;
        perm_l = ((lane + 63) & 63) * 4;
        perm_r = ((lane + 1) & 63) * 4;
        const int nr = (a.nunits + V - 1) / V * V;   // active words rounded to V (<= pitch)
        int base = strip * 62 * V;
        const int last = nr - 62 * V;
        if (base > last) base = last > 0 ? last : 0;
        const int64_t word0 = (int64_t)base - V + (int64_t)lane * V;
        const bool lane_in = word0 >= 0 && word0 + V <= a.pitch;
        const bool lane_store = lane >= 1 && lane <= 62 && word0 < nr;
        ld_off = lane_in ? (uint32_t)(word0 * 4) : kOOB;
        st_off = lane_store ? (uint32_t)(word0 * 4) : kOOB;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int64_t wi = word0 + j;
            if (full) {
                mask[j] = (wi < 0 || wi >= a.nunits) ? 0u : (wi == a.nunits - 1 ? a.last_mask : full);
            } else {   // word wi holds columns 128·(wi/4) + 4·bit + wi%4
                const int64_t c0 = (wi >> 2) * 128 + (wi & 3);
                const int64_t n = wi < 0 ? 0 : (a.active_cols - c0 + 3) >> 2;
                mask[j] = n <= 0 ? 0u : (n >= 32 ? 0xffffffffu : ((1u << n) - 1u));
            }
        }
        R0 = r0;
        R1 = r1;
        base_row = R0 - K;
        const int64_t pitch_b = a.pitch * 4;
        const int win_rows = R1 - R0 + 2 * K;
        const int nrec = (int)(win_rows * pitch_b);
        src = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(static_cast<const uint8_t *>(a.src)) + (int64_t)base_row * pitch_b, 0, nrec,
            0x00020000);
        dst = __builtin_amdgcn_make_buffer_rsrc(static_cast<uint8_t *>(a.dst) + (int64_t)base_row * pitch_b, 0,
                                                nrec, 0x00020000);
    }
    // as row_off, also kOOB for rr >= lim; computed unconditionally and selected
    // once (a branch here would split the unrolled loop body into basic blocks)
    __device__ __forceinline__ uint32_t row_off_lim(const StencilArgs &a, int rr, int lim) const {
        const uint32_t off = (uint32_t)((rr - base_row) * (int)(a.pitch * 4));
        return ((rr >= a.row_lo) & (rr < a.row_hi) & (rr < lim)) ? off : kOOB;
    }
    // byte offset of window row `rr` if it is a live row, else kOOB (uniform)
    __device__ __forceinline__ uint32_t row_off(const StencilArgs &a, int rr) const {
        return (rr >= a.row_lo && rr < a.row_hi) ? (uint32_t)((rr - base_row) * (int)(a.pitch * 4)) : kOOB;
    }
};

// Work items of a launch: items [0, nA) are `big_rows`-row chunks covering the
// first rows_A output rows, items [nA, nitems) are `small_rows`-row chunks
// covering the rest (band-major, strip-minor: neighbouring strips of one band
// are taken together and share an L2).  ctr == nullptr: static grid, wave w
// takes item w.  Otherwise a work queue: every wave pulls items from one
// 64-bit counter (the item is counter - base) until the items run out, so the
// launch ends within one small chunk of its last wave — no half-empty SIMDs
// in a long tail.  Every pull past the end still increments the counter; the
// host advances base by nitems + waves per launch, so it is never reset.
struct Sched {
    unsigned long long *ctr;
    unsigned long long base;
    int nitems, nA;
    int big_rows, small_rows, rows_A;
    // guided static schedule (guided != 0): XCD x (= physical block % 8) owns the
    // row band [x·rows/8, (x+1)·rows/8); its waves, in dispatch order, take
    // chunk-rows whose height shrinks round by round (cpr chunk-rows per round,
    // heights h[r]), so early waves amortise the 2k-row warm-up over tall chunks
    // and the launch ends on short ones (no long half-occupied tail).
    int guided, cpr, nrounds;
    int h[8];
};

__device__ __forceinline__ void item_rows(const StencilArgs &a, const Sched &q, int nstrips, int item, int &strip,
                                          int &r0, int &r1) {
    if (item < q.nA) {
        const int band = item / nstrips;
        strip = item - band * nstrips;
        r0 = a.out_r0 + band * q.big_rows;
        r1 = min(r0 + q.big_rows, a.out_r0 + q.rows_A);
    } else {
        const int i2 = item - q.nA, band = i2 / nstrips;
        strip = i2 - band * nstrips;
        r0 = a.out_r0 + q.rows_A + band * q.small_rows;
        r1 = min(r0 + q.small_rows, a.out_r1);
    }
}

__device__ __forceinline__ bool guided_rows(const StencilArgs &a, const Sched &q, int nstrips, int x, int j,
                                            int &strip, int &r0, int &r1) {
    const int cr = j / nstrips;
    strip = j - cr * nstrips;
    const int r = cr / q.cpr;
    if (r >= q.nrounds) return false;
    int row = 0;
    for (int i = 0; i < r; ++i) row += q.cpr * q.h[i];
    row += (cr - r * q.cpr) * q.h[r];
    const int rows = a.out_r1 - a.out_r0;
    const int bs = a.out_r0 + (int)((int64_t)x * rows / 8), be = a.out_r0 + (int)((int64_t)(x + 1) * rows / 8);
    r0 = bs + row;
    if (r0 >= be) return false;
    r1 = min(r0 + q.h[r], be);
    return true;
}

// Drives `body(item)` for every item of this wave (wave-uniform control flow).
// QUEUE is a separate kernel instantiation so the static kernels keep their
// register allocation.
template <bool QUEUE, typename F>
__device__ __forceinline__ void for_each_item(const Sched &q, int nblocks, F &&body) {
    if constexpr (!QUEUE) {
        const int w = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, nblocks) * 4 + (threadIdx.x >> 6));
        if (w < q.nitems) body(w);
        return;
    }
    for (;;) {
        unsigned long long t = 0;
        if ((threadIdx.x & 63) == 0) t = atomicAdd(q.ctr, 1ull);
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)t);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(t >> 32));
        const long long item = (long long)(((unsigned long long)hi << 32) | lo) - (long long)q.base;
        if (item < 0 || item >= q.nitems) break;
        body((int)item);
    }
}

// ---------------------------------------------------------------- bit layout

// Row state of a wave.  The loop is unrolled by 6 phases: the h/c windows
// rotate with period 3 and the load ring with period 6, so every loop-carried
// value keeps one register (no copies across the back edge, hence no forced
// wait on a just-issued prefetch).
template <int V, int K>
struct BitState {
    uint32_t h0[K][3][V], h1[K][3][V], c[K][3][V];
    uint32_t ld[6][V];
};

// B3/S23 on bit-sliced horizontal 3-sums of rows above (a), at (b), below (c):
// 9-sum incl. self = o + 2u + 4(q+v); next = (sum==3) | (alive & sum==4).
// 8 v_bitop3_b32.  `mask` = 0 forces the cell dead (columns outside the grid);
// with alive = 0 there, the result is 0.
__device__ __forceinline__ uint32_t life_bits(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                              uint32_t c0, uint32_t c1, uint32_t alive,
                                              uint32_t mask) {
    const uint32_t o = xor3(a0, b0, c0);
    const uint32_t co = maj(a0, b0, c0);
    const uint32_t p = xor3(a1, b1, c1);
    const uint32_t q = maj(a1, b1, c1);
    const uint32_t u = __builtin_amdgcn_bitop3_b32(co, p, mask, 0x28);   // (co ^ p) & mask
    const uint32_t s = __builtin_amdgcn_bitop3_b32(q, co, p, 0x78);      // q ^ (co & p)
    const uint32_t m = __builtin_amdgcn_bitop3_b32(u, o, s, 0x42);       // u ? o & ~s : ~o & s
    return __builtin_amdgcn_bitop3_b32(m, u, alive, 0xE0);              // m & (u | alive)
}

// One iteration of the register pipeline.  The row loaded 3 iterations ago
// (generation 0, row rho) enters stage 1; stage s turns generation s-1 row
// rho-(s-1) into the horizontal sums of its 3-row window and emits generation
// s row rho-s, which stage s+1 consumes in the same iteration.  The stages of
// one iteration form a chain; consecutive iterations overlap (the unrolled
// body lets the scheduler start iteration i+1's early stages under iteration
// i's late ones).  The stored row is generation K, row rho-K.
template <int V, int K, bool EDGE, int P>
__device__ __forceinline__ void bit_phase(BitState<V, K> &S, const Strip<V> &st, const StencilArgs &a,
                                          int it, int N) {
    const int rho = st.R0 - K + it;   // generation-0 row arriving this iteration
    uint32_t nv[V];
#pragma unroll
    for (int j = 0; j < V; ++j) nv[j] = S.ld[P][j];
    // prefetch row rho+3 (unconditional: OOB reads 0)
    buf_load<V>(S.ld[(P + 3) % 6], st.src, st.ld_off + ((it + 3 < N) ? st.row_off(a, rho + 3) : kOOB));
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P % 3;
#pragma unroll
    for (int g = 0; g < K; ++g) {
        // nv = generation g, row rho-g: horizontal 3-sums into slot C.  Quad-
        // interleaved groups: word w's neighbour columns are words w±1 at the
        // same bit, except at the group ends (one funnel shift each), whose
        // carry bit comes from the neighbouring group (in-lane or a lane move).
        const uint32_t lft = xlane_from_left(nv[V - 1], st);
        const uint32_t rgt = xlane_from_right(nv[0], st);
        // generation g+1, row rho-g-1
        const int x = rho - g - 1;
        const bool valid = !EDGE || (x >= a.row_lo && x < a.row_hi);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            uint32_t L, R;
            if ((j & 3) == 0) L = funnel(nv[j + 3], j == 0 ? lft : nv[j - 1], 31);   // columns 4b-1
            else L = nv[j - 1];
            if ((j & 3) == 3) R = funnel(j == V - 1 ? rgt : nv[j + 1], nv[j - 3], 1); // columns 4b+4
            else R = nv[j + 1];
            S.h0[g][C][j] = xor3(L, nv[j], R);
            S.h1[g][C][j] = maj(L, nv[j], R);
            S.c[g][C][j] = nv[j];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const uint32_t o = life_bits(S.h0[g][A][j], S.h1[g][A][j], S.h0[g][B][j], S.h1[g][B][j],
                                         S.h0[g][C][j], S.h1[g][C][j], S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
    // generation K, row rho-K: stored when it lies in [R0, R1)  (it in [2K, N))
    const uint32_t roff = (it >= 2 * K && it < N) ? (uint32_t)((rho - K - st.base_row) * (int)(a.pitch * 4)) : kOOB;
    buf_store<V>(st.dst, st.st_off + roff, nv);
}

template <int V, int K, bool EDGE>
__device__ __forceinline__ void bit_run(const Strip<V> &st, const StencilArgs &a) {
    BitState<V, K> S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < V; ++j) S.h0[g][s][j] = S.h1[g][s][j] = S.c[g][s][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K;
#pragma unroll
    for (int s = 0; s < 3; ++s)
        buf_load<V>(S.ld[s], st.src, st.ld_off + (s < N ? st.row_off(a, st.R0 - K + s) : kOOB));
    for (int it = 0; it < N; it += 6) {   // iterations past N are harmless: no loads, no stores
        bit_phase<V, K, EDGE, 0>(S, st, a, it, N);
        bit_phase<V, K, EDGE, 1>(S, st, a, it + 1, N);
        bit_phase<V, K, EDGE, 2>(S, st, a, it + 2, N);
        bit_phase<V, K, EDGE, 3>(S, st, a, it + 3, N);
        bit_phase<V, K, EDGE, 4>(S, st, a, it + 4, N);
        bit_phase<V, K, EDGE, 5>(S, st, a, it + 5, N);
    }
}

// Chained pipeline (default for K >= 5: GOL_BIT_CHAINS = 2 chains): the K
// stages form K/CL chains of CL stages; a chain consumes the previous chain's output row from
// the PREVIOUS iteration (kept in pend[]), so the chains of one iteration are
// independent dependency chains (more ILP for 2 waves/SIMD).  Costs 4 VGPRs
// per chain boundary and D = (K-1)/CL more warm-up rows.  CL = K is the plain
// pipeline (bit_phase above).
#ifndef GOL_BIT_CHAINS
#define GOL_BIT_CHAINS 2   // chains per pipeline for K >= 5 (1: the plain pipeline)
#endif
template <int K>
constexpr int bit_chain_len() { return (K >= 5 && GOL_BIT_CHAINS > 1) ? (K + GOL_BIT_CHAINS - 1) / GOL_BIT_CHAINS : K; }
template <int V, int K, int CL>
struct BitChainState {
    static constexpr int NC = (K + CL - 1) / CL;   // chains
    uint32_t h0[K][3][V], h1[K][3][V], c[K][3][V];
    uint32_t pend[NC][V];                          // output row of each chain (previous iteration)
    uint32_t ld[6][V];
};

template <int V, int K, int CL, bool EDGE, int P>
__device__ __forceinline__ void bit_phase_chain(BitChainState<V, K, CL> &S, const Strip<V> &st,
                                                const StencilArgs &a, int it, int N) {
    constexpr int NC = BitChainState<V, K, CL>::NC;
    constexpr int D = (K - 1) / CL;
    const int rho = st.R0 - K + it;   // generation-0 row arriving this iteration
    buf_load<V>(S.ld[(P + 3) % 6], st.src, st.ld_off + ((it + 3 < N) ? st.row_off(a, rho + 3) : kOOB));
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P % 3;
#pragma unroll
    for (int ch = NC - 1; ch >= 0; --ch) {   // descending: pend[ch-1] is read before chain ch-1 rewrites it
        uint32_t nv[V];
#pragma unroll
        for (int j = 0; j < V; ++j) nv[j] = ch == 0 ? S.ld[P][j] : S.pend[ch - 1][j];
#pragma unroll
        for (int g = ch * CL; g < (ch + 1) * CL && g < K; ++g) {
            // nv = generation g, row rho - g - ch
            const uint32_t lft = xlane_from_left(nv[V - 1], st);
            const uint32_t rgt = xlane_from_right(nv[0], st);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                uint32_t L, R;
                if ((j & 3) == 0) L = funnel(nv[j + 3], j == 0 ? lft : nv[j - 1], 31);
                else L = nv[j - 1];
                if ((j & 3) == 3) R = funnel(j == V - 1 ? rgt : nv[j + 1], nv[j - 3], 1);
                else R = nv[j + 1];
                S.h0[g][C][j] = xor3(L, nv[j], R);
                S.h1[g][C][j] = maj(L, nv[j], R);
                S.c[g][C][j] = nv[j];
            }
            const int x = rho - g - ch - 1;   // generation g+1 row produced now
            const bool valid = !EDGE || (x >= a.row_lo && x < a.row_hi);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const uint32_t o = life_bits(S.h0[g][A][j], S.h1[g][A][j], S.h0[g][B][j], S.h1[g][B][j],
                                             S.h0[g][C][j], S.h1[g][C][j], S.c[g][B][j], st.mask[j]);
                nv[j] = valid ? o : 0u;
            }
        }
        if (ch < NC - 1) {
#pragma unroll
            for (int j = 0; j < V; ++j) S.pend[ch][j] = nv[j];
        } else {   // generation K, row rho - K - D: stored when it lies in [R0, R1)  (it in [2K+D, N))
            const uint32_t roff = (it >= 2 * K + D && it < N)
                                      ? (uint32_t)((rho - K - D - st.base_row) * (int)(a.pitch * 4)) : kOOB;
            buf_store<V>(st.dst, st.st_off + roff, nv);
        }
    }
}

template <int V, int K, int CL, bool EDGE>
__device__ __forceinline__ void bit_run_chain(const Strip<V> &st, const StencilArgs &a) {
    using State = BitChainState<V, K, CL>;
    State S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < V; ++j) S.h0[g][s][j] = S.h1[g][s][j] = S.c[g][s][j] = 0u;
#pragma unroll
    for (int c = 0; c < State::NC; ++c)
#pragma unroll
        for (int j = 0; j < V; ++j) S.pend[c][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K + (K - 1) / CL;
#pragma unroll
    for (int s = 0; s < 3; ++s)
        buf_load<V>(S.ld[s], st.src, st.ld_off + (s < N ? st.row_off(a, st.R0 - K + s) : kOOB));
    for (int it = 0; it < N; it += 6) {
        bit_phase_chain<V, K, CL, EDGE, 0>(S, st, a, it, N);
        bit_phase_chain<V, K, CL, EDGE, 1>(S, st, a, it + 1, N);
        bit_phase_chain<V, K, CL, EDGE, 2>(S, st, a, it + 2, N);
        bit_phase_chain<V, K, CL, EDGE, 3>(S, st, a, it + 3, N);
        bit_phase_chain<V, K, CL, EDGE, 4>(S, st, a, it + 4, N);
        bit_phase_chain<V, K, CL, EDGE, 5>(S, st, a, it + 5, N);
    }
}

// ------------------------------------------------ bit layout, row-pair pipeline
// The 9-sum of output row x is H(x-1) + H(x) + H(x+1) (H = the horizontal
// 3-sum of a row, two bit planes).  Output rows r-1 and r share the pair sum
// P = H(r-1) + H(r) (0..6, binary p0/e0/e1: 4 v_bitop3), so a stage takes
// its input rows two at a time ("event") and per output row needs only
//   row r-1: P + H(r-2)      row r: P + H(r+1)
// — a 4-gate rule over (p0, e0, e1, a0, a1, alive) (tools/pair_search.c:
// exhaustive; 3 gates do not exist).  Per 2 output words: 2 rows' H (4) +
// P (4) + 2 × rule (8) = 16 v_bitop3 instead of 20, i.e. 8 per 32
// cell-updates.  The rule relies on alive's row being inside the pair
// (alive ⇒ P ≥ 1, dead ⇒ P ≤ 5: don't-cares the 4-gate circuit needs), which
// holds for both outputs.  Masked columns (grid edges) need one more AND per
// word, so strips with partial masks and chunks near the dead row boundary
// take the EDGE instantiation; the interior runs mask- and select-free.
#ifndef GOL_BIT_PAIR
#define GOL_BIT_PAIR 0        // 1: row-pair stages for the V=4 bit kernel (0: one row per stage)
#endif
#ifndef GOL_PAIR_CHAINS
#define GOL_PAIR_CHAINS 1     // stage chains of the pair pipeline for K >= 5 (see bit_run_chain)
#endif
#ifndef GOL_PAIR_PIN
#define GOL_PAIR_PIN 0        // 1: sched_group_barrier pipeline, 2: events as scheduling regions
#endif
#ifndef GOL_PAIR_RING
#define GOL_PAIR_RING 3       // load ring in events (2 rows each); prefetch distance RING-1 events
#endif

// B3/S23 from the pair code (p0 + 2 e0 + 4 e1 = P), the single row's 3-sum
// (a0 + 2 a1) and the alive bit.  Truth tables: tools/pair_search.c.
__device__ __forceinline__ uint32_t life_pair(uint32_t p0, uint32_t e0, uint32_t e1, uint32_t a0, uint32_t a1,
                                              uint32_t alive) {
    const uint32_t g1 = __builtin_amdgcn_bitop3_b32(p0, a0, alive, 0x43);
    const uint32_t g2 = __builtin_amdgcn_bitop3_b32(e0, e1, a1, 0x6d);
    const uint32_t g3 = __builtin_amdgcn_bitop3_b32(e0, a1, alive, 0x7d);
    return __builtin_amdgcn_bitop3_b32(g3, g1, g2, 0x18);
}

// horizontal 3-sum planes of one row (quad-interleaved groups, see bit_phase)
template <int V, typename ST>
__device__ __forceinline__ void bit_hsum(const uint32_t (&nv)[V], uint32_t (&h0)[V], uint32_t (&h1)[V],
                                         const ST &st) {
    const uint32_t lft = xlane_from_left(nv[V - 1], st);
    const uint32_t rgt = xlane_from_right(nv[0], st);
#pragma unroll
    for (int j = 0; j < V; ++j) {
        uint32_t L, R;
        if ((j & 3) == 0) L = funnel(nv[j + 3], j == 0 ? lft : nv[j - 1], 31);
        else L = nv[j - 1];
        if ((j & 3) == 3) R = funnel(j == V - 1 ? rgt : nv[j + 1], nv[j - 3], 1);
        else R = nv[j + 1];
        h0[j] = xor3(L, nv[j], R);
        h1[j] = maj(L, nv[j], R);
    }
}

template <int V, int K, int CL>
struct PairState {
    static constexpr int NC = (K + CL - 1) / CL;   // stage chains (as BitChainState)
    // per stage, two parity sets: H of rows r-2 (a) and r-1 (b), alive of r-1
    uint32_t a0[K][2][V], a1[K][2][V], b0[K][2][V], b1[K][2][V], bc[K][2][V];
    uint32_t pend[NC][2][V];                        // each chain's 2 output rows of the previous event
    uint32_t ld[GOL_PAIR_RING][2][V];
};

// One event: generation-0 rows rho, rho+1 enter chain 0; stage g of chain ch
// takes generation-g rows r, r+1 (r = rho - g - 2ch) and emits generation
// g+1 rows r-1, r.  The last chain's rows are stored.
template <int V, int K, int CL, bool EDGE, int E>
__device__ __forceinline__ void pair_event(PairState<V, K, CL> &S, const Strip<V> &st, const StencilArgs &a,
                                           int ev) {
    constexpr int NR = GOL_PAIR_RING, NC = PairState<V, K, CL>::NC, D = NC - 1;
    constexpr int q = E & 1, slot = E % NR, nslot = (E + NR - 1) % NR;
    const int rho = st.R0 - K + 2 * ev;
    {   // prefetch event ev + NR - 1 (rows past the window read 0)
        const int pr = rho + 2 * (NR - 1);
        buf_load<V>(S.ld[nslot][0], st.src, st.ld_off + st.row_off_lim(a, pr, st.R1 + K));
        buf_load<V>(S.ld[nslot][1], st.src, st.ld_off + st.row_off_lim(a, pr + 1, st.R1 + K));
#if GOL_PAIR_PIN == 1
        // keep the prefetch at the top of its event: left alone, the scheduler sinks
        // it to the event's end and hoists the next iteration's first uses above the
        // back edge, which costs a vmcnt(0) per loop trip.
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);     // the 2 row loads, then
        __builtin_amdgcn_sched_group_barrier(0x002, 400, 0);   // a slice of VALU work
#elif GOL_PAIR_PIN == 2
        __builtin_amdgcn_sched_barrier(0);   // events as scheduling regions
#endif
    }
#pragma unroll
    for (int ch = NC - 1; ch >= 0; --ch) {   // descending: pend[ch-1] is read before chain ch-1 rewrites it
        uint32_t x0[V], x1[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            x0[j] = ch == 0 ? S.ld[slot][0][j] : S.pend[ch - 1][0][j];
            x1[j] = ch == 0 ? S.ld[slot][1][j] : S.pend[ch - 1][1][j];
        }
#pragma unroll
        for (int g = ch * CL; g < (ch + 1) * CL && g < K; ++g) {
            uint32_t X0[V], X1[V], Y0[V], Y1[V];
            bit_hsum<V>(x0, X0, X1, st);
            bit_hsum<V>(x1, Y0, Y1, st);
            const int r = rho - g - 2 * ch;
            const bool v0 = !EDGE || (r - 1 >= a.row_lo && r - 1 < a.row_hi);
            const bool v1 = !EDGE || (r >= a.row_lo && r < a.row_hi);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const uint32_t B0 = S.b0[g][q][j], B1 = S.b1[g][q][j];
                const uint32_t p0 = B0 ^ X0[j], k = B0 & X0[j];
                const uint32_t e0 = xor3(B1, X1[j], k), e1 = maj(B1, X1[j], k);
                uint32_t o0 = life_pair(p0, e0, e1, S.a0[g][q][j], S.a1[g][q][j], S.bc[g][q][j]);
                uint32_t o1 = life_pair(p0, e0, e1, Y0[j], Y1[j], x0[j]);
                if constexpr (EDGE) {
                    o0 = v0 ? (o0 & st.mask[j]) : 0u;
                    o1 = v1 ? (o1 & st.mask[j]) : 0u;
                }
                S.a0[g][q ^ 1][j] = X0[j];
                S.a1[g][q ^ 1][j] = X1[j];
                S.b0[g][q ^ 1][j] = Y0[j];
                S.b1[g][q ^ 1][j] = Y1[j];
                S.bc[g][q ^ 1][j] = x1[j];
                x0[j] = o0;
                x1[j] = o1;
            }
        }
        if (ch < NC - 1) {
#pragma unroll
            for (int j = 0; j < V; ++j) {
                S.pend[ch][0][j] = x0[j];
                S.pend[ch][1][j] = x1[j];
            }
        } else {   // generation K, rows s, s+1 (s = rho - K - 2D): stored when in [R0, R1)
            const int s = rho - K - 2 * D;
            const int pb = (int)(a.pitch * 4);
            const uint32_t f0 = (uint32_t)((s - st.base_row) * pb), f1 = f0 + (uint32_t)pb;
            const uint32_t o0 = ((s >= st.R0) & (s < st.R1)) ? f0 : kOOB;
            const uint32_t o1 = ((s + 1 >= st.R0) & (s + 1 < st.R1)) ? f1 : kOOB;
            buf_store<V>(st.dst, st.st_off + o0, x0);
            buf_store<V>(st.dst, st.st_off + o1, x1);
        }
    }
}

template <int V, int K, int CL, bool EDGE>
__device__ __forceinline__ void bit_run_pair(const Strip<V> &st, const StencilArgs &a) {
    using State = PairState<V, K, CL>;
    constexpr int NR = GOL_PAIR_RING, D = State::NC - 1;
    constexpr int UE = (NR % 2 == 0) ? NR : 2 * NR;   // events per unrolled body: lcm(2, NR)
    State S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int j = 0; j < V; ++j)
                S.a0[g][p][j] = S.a1[g][p][j] = S.b0[g][p][j] = S.b1[g][p][j] = S.bc[g][p][j] = 0u;
#pragma unroll
    for (int c = 0; c < State::NC; ++c)
#pragma unroll
        for (int j = 0; j < V; ++j) S.pend[c][0][j] = S.pend[c][1][j] = 0u;
    // events until generation-K row R1-1 has been stored
    const int NE = (st.R1 - st.R0 + 2 * K + 2 * D + 1) / 2 + 1;
#pragma unroll
    for (int e = 0; e < NR - 1; ++e) {
        const int pr = st.R0 - K + 2 * e;
        buf_load<V>(S.ld[e][0], st.src, st.ld_off + st.row_off(a, pr));
        buf_load<V>(S.ld[e][1], st.src, st.ld_off + st.row_off(a, pr + 1));
    }
    for (int ev = 0; ev < NE; ev += UE) {   // events past NE are harmless: no stores inside [R0, R1)
        pair_event<V, K, CL, EDGE, 0>(S, st, a, ev);
        pair_event<V, K, CL, EDGE, 1>(S, st, a, ev + 1);
        if constexpr (UE > 2) {
            pair_event<V, K, CL, EDGE, 2>(S, st, a, ev + 2);
            pair_event<V, K, CL, EDGE, 3>(S, st, a, ev + 3);
        }
        if constexpr (UE > 4) {
            pair_event<V, K, CL, EDGE, 4>(S, st, a, ev + 4);
            pair_event<V, K, CL, EDGE, 5>(S, st, a, ev + 5);
        }
    }
}

template <int V, int K, bool QUEUE>
__global__ __launch_bounds__(256, (GOL_BIT_PAIR && V == 4) ? 2 : 1) void bit_pipe_kernel(StencilArgs a, Sched q, int nstrips, int nblocks) {
    const unsigned long long t0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    for_each_item<QUEUE>(q, nblocks, [&](int item) {
        int strip, r0, r1;
        if (!QUEUE && q.guided) {
            if (!guided_rows(a, q, nstrips, blockIdx.x & 7,
                             __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) * 4 + (threadIdx.x >> 6)), strip, r0, r1))
                return;
        } else {
            item_rows(a, q, nstrips, item, strip, r0, r1);
        }
        Strip<V> st;
        st.setup(a, K, strip, r0, r1, 0u);
        // chunks whose light cone stays inside the live rows skip the per-row checks
        if constexpr (GOL_BIT_PAIR && V == 4) {
            constexpr int CL = (K >= 5 && GOL_PAIR_CHAINS > 1) ? (K + GOL_PAIR_CHAINS - 1) / GOL_PAIR_CHAINS : K;
            constexpr int M = 2 * K + 2 * ((K - 1) / CL) + 2;
            uint32_t all = 0xffffffffu;
#pragma unroll
            for (int j = 0; j < V; ++j) all &= st.mask[j];
            const bool full = __builtin_amdgcn_ballot_w64(all != 0xffffffffu) == 0ull;
            if (full && st.R0 - M >= a.row_lo && st.R1 + M <= a.row_hi) bit_run_pair<V, K, CL, false>(st, a);
            else bit_run_pair<V, K, CL, true>(st, a);
            return;
        }
        if constexpr (bit_chain_len<K>() < K && V == 4) {
            constexpr int CL = bit_chain_len<K>(), M = 2 * K + (K - 1) / CL;
            if (st.R0 - M >= a.row_lo && st.R1 + M <= a.row_hi) bit_run_chain<V, K, CL, false>(st, a);
            else bit_run_chain<V, K, CL, true>(st, a);
            return;
        }
        if (st.R0 - 2 * K >= a.row_lo && st.R1 + 2 * K <= a.row_hi) bit_run<V, K, false>(st, a);
        else bit_run<V, K, true>(st, a);
    });
    if (a.stamps) {   // diagnostic only: written to a buffer nothing in the kernel reads
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            const int w = xcd_remap(blockIdx.x, nblocks) * 4 + (threadIdx.x >> 6);
            a.stamps[2 * w] = t0;
            a.stamps[2 * w + 1] = t1;
        }
    }
}

// ------------------------------------------------ bit layout, split pipeline
// The same K-stage register pipeline with the stages split over TWO waves per
// item: role 0 loads rows and runs stages [0, K/2); role 1 runs stages
// [K/2, K) and stores.  Role 0 hands each generation-K/2 row to role 1
// through an LDS ring (2 halves × 6 rows × 64 lanes × 16 B = 12 KiB per
// block); one s_barrier per 6 rows separates writing a half from reading it.
// Each wave holds half the window state, so ~3 waves fit per SIMD instead of
// 2 — more waves to pair for dual VALU issue; the price is the barrier and a
// 6-row lag of role 1 (extra warm-up).  Role 1 starts with 6 iterations of
// garbage input, which only lengthens its warm-up: its stage outputs become
// valid at the same pipeline iteration as in the single-wave kernel.
template <int H>
struct SplitState {
    uint32_t h0[H][3][4], h1[H][3][4], c[H][3][4];
    uint32_t ld[6][4];   // role 0: load ring
};

// stages [KS, KS+H) of one iteration on row nv (generation KS, row rho-KS)
template <int H, int KS, bool EDGE, int P>
__device__ __forceinline__ void split_stages(SplitState<H> &S, uint32_t (&nv)[4], const Strip<4> &st,
                                             const StencilArgs &a, int rho) {
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P % 3;
#pragma unroll
    for (int g = 0; g < H; ++g) {
        const uint32_t lft = xlane_from_left(nv[3], st);
        const uint32_t rgt = xlane_from_right(nv[0], st);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t L = j == 0 ? funnel(nv[3], lft, 31) : nv[j - 1];
            const uint32_t R = j == 3 ? funnel(rgt, nv[0], 1) : nv[j + 1];
            S.h0[g][C][j] = xor3(L, nv[j], R);
            S.h1[g][C][j] = maj(L, nv[j], R);
            S.c[g][C][j] = nv[j];
        }
        const int x = rho - (KS + g) - 1;
        const bool valid = !EDGE || (x >= a.row_lo && x < a.row_hi);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t o = life_bits(S.h0[g][A][j], S.h1[g][A][j], S.h0[g][B][j], S.h1[g][B][j],
                                         S.h0[g][C][j], S.h1[g][C][j], S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
}

#ifndef GOL_SPLIT_BLOCK
#define GOL_SPLIT_BLOCK 6   // rows per barrier (6 or 12)
#endif
constexpr int kSB = GOL_SPLIT_BLOCK;

__device__ __forceinline__ void split_barrier() {
    // LDS writes of this block done, then the workgroup barrier; the "memory"
    // clobber keeps the compiler's LDS accesses on their side of it.  No vmcnt
    // wait: role 0's row prefetches stay in flight across the barrier.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int K, bool EDGE, int P>
__device__ __forceinline__ void split_phase0(SplitState<K / 2> &S, const Strip<4> &st, const StencilArgs &a,
                                             u32x4 (*ring)[kSB][64], int it, int N) {
    const int rho = st.R0 - K + it;
    uint32_t nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) nv[j] = S.ld[P % 6][j];
    buf_load<4>(S.ld[(P + 3) % 6], st.src, st.ld_off + ((it + 3 < N) ? st.row_off(a, rho + 3) : kOOB));
    split_stages<K / 2, 0, EDGE, P % 6>(S, nv, st, a, rho);
    u32x4 t;
    t.x = nv[0]; t.y = nv[1]; t.z = nv[2]; t.w = nv[3];
    ring[(it / kSB) & 1][P][threadIdx.x & 63] = t;
}

template <int K, bool EDGE, int P>
__device__ __forceinline__ void split_phase1(SplitState<K / 2> &S, const Strip<4> &st, const StencilArgs &a,
                                             u32x4 (*ring)[kSB][64], int it, int N) {
    const int it1 = it - kSB;   // role 1 runs one block behind role 0
    const int rho = st.R0 - K + it1;
    const u32x4 t = ring[((it / kSB) + 1) & 1][P][threadIdx.x & 63];
    uint32_t nv[4] = {t.x, t.y, t.z, t.w};
    split_stages<K / 2, K / 2, EDGE, P % 6>(S, nv, st, a, rho);
    const uint32_t roff =
        (it1 >= 2 * K && it1 < N) ? (uint32_t)((rho - K - st.base_row) * (int)(a.pitch * 4)) : kOOB;
    buf_store<4>(st.dst, st.st_off + roff, nv);
}

template <int K, bool EDGE>
__device__ __forceinline__ void split_run(const Strip<4> &st, const StencilArgs &a, u32x4 (*ring)[kSB][64]) {
    constexpr int H = K / 2;
    SplitState<H> S;
#pragma unroll
    for (int g = 0; g < H; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) S.h0[g][s][j] = S.h1[g][s][j] = S.c[g][s][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K;
    const int Ntot = N + kSB;   // role 1 finishes one block later; both roles run the same blocks
    if ((threadIdx.x >> 6) == 0) {
#pragma unroll
        for (int s = 0; s < 3; ++s)
            buf_load<4>(S.ld[s], st.src, st.ld_off + (s < N ? st.row_off(a, st.R0 - K + s) : kOOB));
        for (int it = 0; it < Ntot; it += kSB) {
            split_phase0<K, EDGE, 0>(S, st, a, ring, it, N);
            split_phase0<K, EDGE, 1>(S, st, a, ring, it + 1, N);
            split_phase0<K, EDGE, 2>(S, st, a, ring, it + 2, N);
            split_phase0<K, EDGE, 3>(S, st, a, ring, it + 3, N);
            split_phase0<K, EDGE, 4>(S, st, a, ring, it + 4, N);
            split_phase0<K, EDGE, 5>(S, st, a, ring, it + 5, N);
            if constexpr (kSB == 12) {
                split_phase0<K, EDGE, 6>(S, st, a, ring, it + 6, N);
                split_phase0<K, EDGE, 7>(S, st, a, ring, it + 7, N);
                split_phase0<K, EDGE, 8>(S, st, a, ring, it + 8, N);
                split_phase0<K, EDGE, 9>(S, st, a, ring, it + 9, N);
                split_phase0<K, EDGE, 10>(S, st, a, ring, it + 10, N);
                split_phase0<K, EDGE, 11>(S, st, a, ring, it + 11, N);
            }
            split_barrier();
        }
    } else {
        for (int it = 0; it < Ntot; it += kSB) {
            split_phase1<K, EDGE, 0>(S, st, a, ring, it, N);
            split_phase1<K, EDGE, 1>(S, st, a, ring, it + 1, N);
            split_phase1<K, EDGE, 2>(S, st, a, ring, it + 2, N);
            split_phase1<K, EDGE, 3>(S, st, a, ring, it + 3, N);
            split_phase1<K, EDGE, 4>(S, st, a, ring, it + 4, N);
            split_phase1<K, EDGE, 5>(S, st, a, ring, it + 5, N);
            if constexpr (kSB == 12) {
                split_phase1<K, EDGE, 6>(S, st, a, ring, it + 6, N);
                split_phase1<K, EDGE, 7>(S, st, a, ring, it + 7, N);
                split_phase1<K, EDGE, 8>(S, st, a, ring, it + 8, N);
                split_phase1<K, EDGE, 9>(S, st, a, ring, it + 9, N);
                split_phase1<K, EDGE, 10>(S, st, a, ring, it + 10, N);
                split_phase1<K, EDGE, 11>(S, st, a, ring, it + 11, N);
            }
            split_barrier();
        }
    }
}

// One item (strip, chunk) per 128-thread block.  Every branch below is uniform
// over the block, so both waves execute the same number of barriers.
template <int K>
__global__ __launch_bounds__(128) void bit_split_kernel(StencilArgs a, Sched q, int nstrips, int nblocks) {
    __shared__ u32x4 ring[2][kSB][64];
    int strip, r0, r1;
    if (q.guided) {
        if (!guided_rows(a, q, nstrips, blockIdx.x & 7, (int)(blockIdx.x >> 3), strip, r0, r1)) return;
    } else {
        const int item = xcd_remap(blockIdx.x, nblocks);
        if (item >= q.nitems) return;
        item_rows(a, q, nstrips, item, strip, r0, r1);
    }
    Strip<4> st;
    st.setup(a, K, strip, r0, r1, 0u);
    if (st.R0 - 2 * K >= a.row_lo && st.R1 + 2 * K <= a.row_hi) split_run<K, false>(st, a, ring);
    else split_run<K, true>(st, a, ring);
}

// --------------------------------------------------------------- byte layout
// V = 4 dwords = 16 cells per lane.  Vertical sums first (v_add3 of 3 rows),
// then horizontal byte shifts of the vertical sums.

template <int K>
struct ByteState {
    uint32_t c[K][3][4];
    uint32_t ld[6][4];
};

// s8 = 9-sum − self; next = ((s8 | alive) == 3), SWAR over 4 bytes (values < 16).
__device__ __forceinline__ uint32_t life_bytes(uint32_t t9, uint32_t alive, uint32_t mask) {
    const uint32_t s8 = t9 - alive;
    const uint32_t y = (s8 | alive) ^ 0x03030303u;
    const uint32_t z = y + 0x7f7f7f7fu;
    return (~z >> 7) & mask;   // mask ⊆ 0x01010101
}

template <int K, bool EDGE, int P>
__device__ __forceinline__ void byte_phase(ByteState<K> &S, const Strip<4> &st, const StencilArgs &a, int it,
                                           int N) {
    const int rho = st.R0 - K + it;
    uint32_t nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) nv[j] = S.ld[P][j];
    buf_load<4>(S.ld[(P + 3) % 6], st.src, st.ld_off + ((it + 3 < N) ? st.row_off(a, rho + 3) : kOOB));
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P % 3;
#pragma unroll
    for (int g = 0; g < K; ++g) {
        uint32_t vs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            S.c[g][C][j] = nv[j];
            vs[j] = S.c[g][A][j] + S.c[g][B][j] + nv[j];   // v_add3_u32, bytes <= 3
        }
        const uint32_t lft = __builtin_amdgcn_update_dpp(0u, vs[3], 0x138, 0xf, 0xf, true);
        const uint32_t rgt = __builtin_amdgcn_update_dpp(0u, vs[0], 0x130, 0xf, 0xf, true);
        const int x = rho - g - 1;
        const bool valid = !EDGE || (x >= a.row_lo && x < a.row_hi);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t pv = j == 0 ? lft : vs[j - 1];
            const uint32_t nx = j == 3 ? rgt : vs[j + 1];
            const uint32_t t9 = funnel(vs[j], pv, 24) + vs[j] + funnel(nx, vs[j], 8);
            const uint32_t o = life_bytes(t9, S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
    const uint32_t roff = (it >= 2 * K && it < N) ? (uint32_t)((rho - K - st.base_row) * (int)(a.pitch * 4)) : kOOB;
    buf_store<4>(st.dst, st.st_off + roff, nv);
}

template <int K, bool EDGE>
__device__ __forceinline__ void byte_run(const Strip<4> &st, const StencilArgs &a) {
    ByteState<K> S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) S.c[g][s][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K;
#pragma unroll
    for (int s = 0; s < 3; ++s)
        buf_load<4>(S.ld[s], st.src, st.ld_off + (s < N ? st.row_off(a, st.R0 - K + s) : kOOB));
    for (int it = 0; it < N; it += 6) {
        byte_phase<K, EDGE, 0>(S, st, a, it, N);
        byte_phase<K, EDGE, 1>(S, st, a, it + 1, N);
        byte_phase<K, EDGE, 2>(S, st, a, it + 2, N);
        byte_phase<K, EDGE, 3>(S, st, a, it + 3, N);
        byte_phase<K, EDGE, 4>(S, st, a, it + 4, N);
        byte_phase<K, EDGE, 5>(S, st, a, it + 5, N);
    }
}

template <int K, bool QUEUE>
__global__ __launch_bounds__(256) void byte_pipe_kernel(StencilArgs a, Sched q, int nstrips, int nblocks) {
    for_each_item<QUEUE>(q, nblocks, [&](int item) {
        int strip, r0, r1;
        if (!QUEUE && q.guided) {
            if (!guided_rows(a, q, nstrips, blockIdx.x & 7,
                             __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) * 4 + (threadIdx.x >> 6)), strip, r0, r1))
                return;
        } else {
            item_rows(a, q, nstrips, item, strip, r0, r1);
        }
        Strip<4> st;
        st.setup(a, K, strip, r0, r1, 0x01010101u);
        if (st.R0 - 2 * K >= a.row_lo && st.R1 + 2 * K <= a.row_hi) byte_run<K, false>(st, a);
        else byte_run<K, true>(st, a);
    });
}

// ----------------------------------------------- byte layout, bit-sliced core
// The board stays byte-per-cell in HBM (the reference's bool board: 1 B/cell
// read + 1 B/cell written per launch), but a wave packs each row it loads into
// bit planes, runs the K-stage bit pipeline of the bit layout on them and
// unpacks the output row to bytes before storing it.  The bit core costs
// 15-20 issue slots per 32 cell-updates instead of ~3.5 per cell for byte
// SWAR, so the byte board can afford K = 16-24 generations per HBM pass.
//
// Geometry <V, K>: a lane holds 16·NB columns (NB = 2V dwordx4 loads per row).
//   V = 2 (K <= 16): 4 blocks per wave; lane i of block q holds the 16 columns
//     c0 + S·q + 16i + t, so every load instruction is one coalesced 1-KiB row
//     segment.  HL = ceil(K/16) lanes at each block edge are halo (their outer
//     neighbours are the DPP zero fill; K generations of garbage stay inside
//     their 16·HL columns); blocks overlap by 2·HL lanes (stride
//     S = 16·(64 - 2·HL)), so the strip stores 4·S contiguous columns.  In
//     registers: two words, one 8-bit field per block, bit 8q + j of word w =
//     column t = 2j + w; the left neighbour of word 0 is word 1 shifted up a
//     bit, the right neighbour of word 1 is word 0 shifted down a bit, and the
//     field-end bits come from the adjacent lane (DPP) via a v_bitop3 select.
//   V = 1 (K = 20..32): lane i holds the 32 contiguous columns c0 + 32i + t in
//     one word (bit t), loaded as two 16-B halves (32-B lane stride); lanes 0
//     and 63 are halo (32 columns >= K), the strip stores 62·32 = 1984 columns.
//     Neighbours: funnel shifts with the adjacent lane's word (DPP).
//     Half the per-stage state of V = 2, so K = 24 fits 2 waves/SIMD.
template <int V, int K>
struct BBGeom {
    static constexpr int NB = 2 * V;                          // 16-B loads per lane and row
    static constexpr int HL = V == 2 ? (K + 15) / 16 : 1;     // halo lanes per edge
    static constexpr int LS = V == 2 ? 16 : 32;               // lane stride (columns)
    static constexpr int S = V == 2 ? 16 * (64 - 2 * HL) : 16;   // load (block / half) stride (columns)
    static constexpr int W = V == 2 ? NB * S : 32 * (64 - 2 * HL);   // columns stored per strip
    static constexpr int NX = 4 * NB;                         // raw dwords per lane and row
    static_assert(K <= 16 * HL * (V == 2 ? 1 : 2), "halo narrower than the light cone");
};
static_assert(BBGeom<2, 16>::W == 3968 && BBGeom<1, 24>::W == 1984, "bytebit geometry");

template <int V, int K>
struct ByteBitStrip {
    using G = BBGeom<V, K>;
    uint32_t ld_off[G::NB], st_off[G::NB];   // row-relative byte offsets per block (kOOB: outside)
    uint32_t mask[V];                        // live cells per word
    int R0, R1, base_row;
    __amdgpu_buffer_rsrc_t src, dst;

    __device__ __forceinline__ void setup(const StencilArgs &a, int strip, int r0, int r1) {
        const int lane = threadIdx.x & 63;
        const int64_t pitch_b = a.pitch * 4;
        const int64_t c0 = (int64_t)strip * G::W - G::LS * G::HL;
#pragma unroll
        for (int w = 0; w < V; ++w) mask[w] = 0u;
#pragma unroll
        for (int q = 0; q < G::NB; ++q) {
            const int64_t col = c0 + G::S * q + G::LS * lane;
            const bool in = col >= 0 && col + 16 <= pitch_b;
            ld_off[q] = in ? (uint32_t)col : kOOB;
            st_off[q] = (in && lane >= G::HL && lane < 64 - G::HL && col < a.active_cols) ? (uint32_t)col : kOOB;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int64_t cc = col + t;
                if (cc >= 0 && cc < a.active_cols) {
                    if constexpr (V == 2) mask[t & 1] |= 1u << (8 * q + (t >> 1));
                    else mask[0] |= 1u << (16 * q + t);   // q = half of the lane's 32 columns
                }
            }
        }
        R0 = r0;
        R1 = r1;
        base_row = R0 - K;
        const int win_rows = R1 - R0 + 2 * K;
        const int nrec = (int)(win_rows * pitch_b);
        src = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(static_cast<const uint8_t *>(a.src)) + (int64_t)base_row * pitch_b, 0, nrec,
            0x00020000);
        dst = __builtin_amdgcn_make_buffer_rsrc(static_cast<uint8_t *>(a.dst) + (int64_t)base_row * pitch_b, 0,
                                                nrec, 0x00020000);
    }
    __device__ __forceinline__ uint32_t row_off(const StencilArgs &a, int rr) const {
        return (rr >= a.row_lo && rr < a.row_hi) ? (uint32_t)((rr - base_row) * (int)(a.pitch * 4)) : kOOB;
    }
};

template <int V, int K>
struct ByteBitState {
    uint32_t h0[K][3][V], h1[K][3][V], c[K][3][V];
    uint32_t ld[3][BBGeom<V, K>::NX];   // 3-row load ring of raw 0/1 bytes
};

// V = 2: 16 dwords of 0/1 bytes (block q, dword d: columns 16i + 4d + byte) -> 2 words.
__device__ __forceinline__ void bb_pack(const uint32_t (&x)[16], uint32_t (&w)[2]) {
    uint32_t u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        // byte b of z: cells 4d+b at bits 2d; word w's field = byte w | byte w+2 << 1
        const uint32_t z = x[4 * q] | (x[4 * q + 1] << 2) | (x[4 * q + 2] << 4) | (x[4 * q + 3] << 6);
        u[q] = z | (z >> 15);
    }
    const uint32_t A = __builtin_amdgcn_perm(u[1], u[0], 0x05010400u);   // u0.b0 u1.b0 u0.b1 u1.b1
    const uint32_t B = __builtin_amdgcn_perm(u[3], u[2], 0x05010400u);
    w[0] = __builtin_amdgcn_perm(B, A, 0x05040100u);
    w[1] = __builtin_amdgcn_perm(B, A, 0x07060302u);
}

// V = 1: 8 dwords (the lane's two 16-column halves q) -> 1 word, bit 16q + t.
__device__ __forceinline__ void bb_pack(const uint32_t (&x)[8], uint32_t (&w)[1]) {
    uint32_t f[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        // y: byte b holds cells 4·0+b (bit 0) and 4·1+b (bit 4); z: cells 8+b, 12+b.
        // Gathering byte b down by 7b bits puts them at bits b and 4+b.
        const uint32_t y = x[4 * q] | (x[4 * q + 1] << 4);
        const uint32_t z = x[4 * q + 2] | (x[4 * q + 3] << 4);
        const uint32_t gy = y | (y >> 7) | (y >> 14) | (y >> 21);
        const uint32_t gz = z | (z >> 7) | (z >> 14) | (z >> 21);
        f[q] = (gy & 0xffu) | ((gz & 0xffu) << 8);
    }
    w[0] = f[0] | (f[1] << 16);
}

// V = 2: 2 words -> 16 dwords of 0/1 bytes (inverse of bb_pack).
__device__ __forceinline__ void bb_unpack(const uint32_t (&w)[2], uint32_t (&x)[16], uint32_t hi16) {
    const uint32_t P01 = __builtin_amdgcn_perm(w[1], w[0], 0x05010400u);   // (w0.b0 w1.b0) (w0.b1 w1.b1)
    const uint32_t P23 = __builtin_amdgcn_perm(w[1], w[0], 0x07030602u);   // (w0.b2 w1.b2) (w0.b3 w1.b3)
    uint32_t z[4];
    // z: bytes 0/1 = the fields of words 0/1 (even bits: cells 4d+0 / 4d+1),
    // bytes 2/3 = the same fields >> 1 (cells 4d+2 / 4d+3); select by hi16
    z[0] = __builtin_amdgcn_bitop3_b32(P01, P01 << 15, hi16, 0xD8);
    z[1] = __builtin_amdgcn_bitop3_b32(P01 >> 16, P01 >> 1, hi16, 0xD8);
    z[2] = __builtin_amdgcn_bitop3_b32(P23, P23 << 15, hi16, 0xD8);
    z[3] = __builtin_amdgcn_bitop3_b32(P23 >> 16, P23 >> 1, hi16, 0xD8);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int d = 0; d < 4; ++d) x[4 * q + d] = (z[q] >> (2 * d)) & 0x01010101u;
}

// V = 1: 1 word -> 8 dwords.  Nibble n = cells 4d..4d+3 of a block; spreading
// its bit b to bit 8b is n·(1 + 2^7 + 2^14 + 2^21) (no carries: the partial
// products land on distinct bits) masked to 0x01010101 — a 24-bit multiply.
__device__ __forceinline__ void bb_unpack(const uint32_t (&w)[1], uint32_t (&x)[8], uint32_t) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t n = (w[0] >> (16 * q + 4 * d)) & 0xfu;
            x[4 * q + d] = __umul24(n, 0x204081u) & 0x01010101u;
        }
}

// Horizontal 3-sums (h0 = L^C^R, h1 = maj) of one row of generation g.
__device__ __forceinline__ void bb_hsum(const uint32_t (&nv)[2], uint32_t (&n0)[2], uint32_t (&n1)[2], uint32_t lo,
                                        uint32_t hi) {
    const uint32_t xl = __builtin_amdgcn_update_dpp(0u, nv[1], 0x138, 0xf, 0xf, true);   // wave_shr:1
    const uint32_t xr = __builtin_amdgcn_update_dpp(0u, nv[0], 0x130, 0xf, 0xf, true);   // wave_shl:1
    const uint32_t L0 = __builtin_amdgcn_bitop3_b32(nv[1] << 1, xl >> 7, lo, 0xD8);   // lo ? xl>>7 : w1<<1
    const uint32_t R1 = __builtin_amdgcn_bitop3_b32(nv[0] >> 1, xr << 7, hi, 0xD8);   // hi ? xr<<7 : w0>>1
    n0[0] = xor3(L0, nv[0], nv[1]);
    n1[0] = maj(L0, nv[0], nv[1]);
    n0[1] = xor3(nv[0], nv[1], R1);
    n1[1] = maj(nv[0], nv[1], R1);
}
__device__ __forceinline__ void bb_hsum(const uint32_t (&nv)[1], uint32_t (&n0)[1], uint32_t (&n1)[1], uint32_t,
                                        uint32_t) {
    const uint32_t xl = __builtin_amdgcn_update_dpp(0u, nv[0], 0x138, 0xf, 0xf, true);   // wave_shr:1
    const uint32_t xr = __builtin_amdgcn_update_dpp(0u, nv[0], 0x130, 0xf, 0xf, true);   // wave_shl:1
    const uint32_t L = funnel(nv[0], xl, 31);   // column t-1: (w << 1) | bit 31 of the left lane
    const uint32_t R = funnel(xr, nv[0], 1);    // column t+1: (w >> 1) | bit 0 of the right lane << 31
    n0[0] = xor3(L, nv[0], R);
    n1[0] = maj(L, nv[0], R);
}

template <int V, int K, bool EDGE, int P>
__device__ __forceinline__ void bb_phase(ByteBitState<V, K> &S, const ByteBitStrip<V, K> &st, const StencilArgs &a,
                                         int it, int N, uint32_t lo, uint32_t hi, uint32_t hi16) {
    using G = BBGeom<V, K>;
    const int rho = st.R0 - K + it;   // generation-0 row arriving this iteration (loaded 2 iterations ago)
    uint32_t nv[V];
    bb_pack(S.ld[P], nv);
    {   // prefetch row rho+2 (unconditional: OOB reads 0)
        const uint32_t roff = (it + 2 < N) ? st.row_off(a, rho + 2) : kOOB;
#pragma unroll
        for (int q = 0; q < G::NB; ++q) {
            uint32_t t[4];
            buf_load<4>(t, st.src, st.ld_off[q] + roff);
#pragma unroll
            for (int d = 0; d < 4; ++d) S.ld[(P + 2) % 3][4 * q + d] = t[d];
        }
    }
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P % 3;
#pragma unroll
    for (int g = 0; g < K; ++g) {
        // nv = generation g, row rho-g
        bb_hsum(nv, S.h0[g][C], S.h1[g][C], lo, hi);
#pragma unroll
        for (int j = 0; j < V; ++j) S.c[g][C][j] = nv[j];
        const int x = rho - g - 1;   // generation g+1, row rho-g-1
        const bool valid = !EDGE || (x >= a.row_lo && x < a.row_hi);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const uint32_t o = life_bits(S.h0[g][A][j], S.h1[g][A][j], S.h0[g][B][j], S.h1[g][B][j],
                                         S.h0[g][C][j], S.h1[g][C][j], S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
    // generation K, row rho-K: stored when it lies in [R0, R1)  (it in [2K, N))
    const uint32_t roff = (it >= 2 * K && it < N) ? (uint32_t)((rho - K - st.base_row) * (int)(a.pitch * 4)) : kOOB;
    uint32_t out[G::NX];
    bb_unpack(nv, out, hi16);
#pragma unroll
    for (int q = 0; q < G::NB; ++q) {
        const uint32_t t[4] = {out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]};
        buf_store<4>(st.dst, st.st_off[q] + roff, t);
    }
}

template <int V, int K, bool EDGE>
__device__ __forceinline__ void bb_run(const ByteBitStrip<V, K> &st, const StencilArgs &a) {
    using G = BBGeom<V, K>;
    ByteBitState<V, K> S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < V; ++j) S.h0[g][s][j] = S.h1[g][s][j] = S.c[g][s][j] = 0u;
    // full-rate v_bitop3 needs its constants in VGPRs, not SGPRs: the field-start
    // and field-end bit masks, and the unpack's byte-half select
    uint32_t lo = 0x01010101u, hi = 0x80808080u, hi16 = 0xffff0000u;   // (V = 2 only)
    asm volatile("" : "+v"(lo), "+v"(hi), "+v"(hi16));
    const int N = (st.R1 - st.R0) + 2 * K;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const uint32_t roff = s < N ? st.row_off(a, st.R0 - K + s) : kOOB;
#pragma unroll
        for (int q = 0; q < G::NB; ++q) {
            uint32_t t[4];
            buf_load<4>(t, st.src, st.ld_off[q] + roff);
#pragma unroll
            for (int d = 0; d < 4; ++d) S.ld[s][4 * q + d] = t[d];
        }
    }
    for (int it = 0; it < N; it += 3) {   // iterations past N are harmless: no loads, no stores
        bb_phase<V, K, EDGE, 0>(S, st, a, it, N, lo, hi, hi16);
        bb_phase<V, K, EDGE, 1>(S, st, a, it + 1, N, lo, hi, hi16);
        bb_phase<V, K, EDGE, 2>(S, st, a, it + 2, N, lo, hi, hi16);
    }
}

template <int V, int K>
__global__ __launch_bounds__(256) void bytebit_pipe_kernel(StencilArgs a, Sched q, int nstrips, int nblocks) {
    for_each_item<false>(q, nblocks, [&](int item) {
        int strip, r0, r1;
        if (q.guided) {
            if (!guided_rows(a, q, nstrips, blockIdx.x & 7,
                             __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) * 4 + (threadIdx.x >> 6)), strip, r0, r1))
                return;
        } else {
            item_rows(a, q, nstrips, item, strip, r0, r1);
        }
        ByteBitStrip<V, K> st;
        st.setup(a, strip, r0, r1);
        if (st.R0 - 2 * K >= a.row_lo && st.R1 + 2 * K <= a.row_hi) bb_run<V, K, false>(st, a);
        else bb_run<V, K, true>(st, a);
    });
}

// columns stored per strip of the bytebit kernel for `gens` generations (0: not instantiated)
static inline int bytebit_strip_cols(int gens) {
    switch (gens) {
    case 4: return BBGeom<2, 4>::W;
    case 8: return BBGeom<2, 8>::W;
    case 12: return BBGeom<2, 12>::W;
    case 16: return BBGeom<2, 16>::W;
    case 20: return BBGeom<1, 20>::W;
    case 24: return BBGeom<1, 24>::W;
    case 28: return BBGeom<1, 28>::W;
    case 32: return BBGeom<1, 32>::W;
    default: return 0;
    }
}

// ------------------------------------------------------------ launch helpers

static inline int strips_of(const StencilArgs &a, int v) {
    if (v <= 0) {   // byte layout, bit-sliced core: v = -(columns per strip)
        const int w = -v;
        return (int)std::max<int64_t>(1, (a.active_cols + w - 1) / w);
    }
    const int nr = (a.nunits + v - 1) / v * v;
    const int per = 62 * v;
    return nr <= per ? 1 : (nr + per - 1) / per;
}

// Launch shape per kernel: the split kernels run one item per 128-thread block
// (two waves share an item); everything else one item per wave, 4 per block.
static std::mutex g_shape_mu;
static std::map<const void *, int> g_split_fns;
static void register_split(const void *fn) {
    std::lock_guard<std::mutex> lk(g_shape_mu);
    g_split_fns[fn] = 1;
}
static bool is_split(const void *fn) {
    std::lock_guard<std::mutex> lk(g_shape_mu);
    return g_split_fns.count(fn) != 0;
}
static int block_threads_of(const void *fn) { return is_split(fn) ? 128 : 256; }
static int items_per_block_of(const void *fn) { return is_split(fn) ? 1 : 4; }

// Work items that can be in flight at once for this kernel on the current
// device (occupancy query × CUs × items per block), cached.
static int resident_waves(const void *fn) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair(fn, dev);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int blocks = 0, cus = 0;
    const int threads = block_threads_of(fn);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, threads, 0) != hipSuccess || blocks < 1) blocks = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    const int w = blocks * cus * items_per_block_of(fn);
    cache[key] = w;
    return w;
}

// Work plan of one launch.
//  chunk_rows > 0 : static grid of fixed chunks.
//  chunk_rows < 0 : static grid, chunk = rows covered in exactly r = -chunk_rows
//                   rounds of resident waves.
//  chunk_rows == 0: work queue (needs a counter): ~2 big chunks per resident
//                   wave over the first 80 % of the rows, quarter-size chunks
//                   for the rest, pulled dynamically.
// Chunks never exceed 2^28 bytes of buffer window (kOOB margin).
static Sched plan_items(const StencilArgs &a, int gens, int v, const void *fn, unsigned long long *ctr,
                        unsigned long long base, int &waves, int &nstrips) {
    Sched q{};
    const int rows = a.out_r1 - a.out_r0;
    nstrips = strips_of(a, v);
    const int max_rows = (int)std::max<int64_t>(1, (int64_t)(1 << 28) / (a.pitch * 4) - 2 * gens);
    const int resident = resident_waves(fn);
    if (a.chunk_rows == 0 && ctr) {
        const int rows_A = rows * 4 / 5;
        const int per_strip_big = std::max(1, 2 * resident / nstrips);
        int big = std::min(max_rows, std::max(16, (rows_A + per_strip_big - 1) / per_strip_big));
        int small = std::min(max_rows, std::max(8, big / 4));
        q.ctr = ctr;
        q.base = base;
        q.big_rows = big;
        q.small_rows = small;
        q.rows_A = rows_A;
        q.nA = (rows_A + big - 1) / big * nstrips;
        q.nitems = q.nA + (rows - rows_A + small - 1) / small * nstrips;
        waves = std::min(resident, q.nitems);
        return q;
    }
    // guided (chunk_rows <= -100, -(100 + r) = r rounds): see Sched
    if (a.chunk_rows <= -100 && rows >= 8 * 16) {
        const int rounds = std::min(8, std::max(1, -a.chunk_rows - 100));
        const int rows_x = (rows + 7) / 8;
        const int cpr = std::max(1, resident / 8 / nstrips);
        double sum = 0, f = 1;
        // round-to-round chunk ratio (GOL_GUIDED_RATIO overrides, experiments only)
        static const double ratio = getenv("GOL_GUIDED_RATIO") ? atof(getenv("GOL_GUIDED_RATIO")) : 0.5;
        for (int r = 0; r < rounds; ++r, f *= ratio) sum += f;
        q.guided = 1;
        q.cpr = cpr;
        q.nrounds = rounds;
        const int h0 = (int)std::ceil(rows_x / (cpr * sum));
        int covered = 0;
        f = 1;
        for (int r = 0; r < rounds; ++r, f *= ratio) {
            q.h[r] = std::min(max_rows, std::max(8, (int)std::ceil(h0 * f)));
            covered += cpr * q.h[r];
        }
        while (covered < rows_x) {   // top up the first round until the band is covered
            const int add = std::min(max_rows - q.h[0], (rows_x - covered + cpr - 1) / cpr);
            if (add <= 0) break;
            q.h[0] += add;
            covered += cpr * add;
        }
        if (covered >= rows_x) {
            const int per_x = cpr * nstrips * rounds;
            const int ipb = items_per_block_of(fn);
            const int nb = 8 * ((per_x + ipb - 1) / ipb);
            q.nitems = q.nA = nb * ipb;   // every item slot runs its (guided) body once
            q.big_rows = q.small_rows = q.h[0];
            q.rows_A = rows;
            waves = nb * ipb;
            return q;
        }
        q.guided = 0;   // could not cover the band within the window limit: fall back to static
    }
    int chunk = a.chunk_rows;
    if (chunk <= -100) chunk = -4;
    if (chunk <= 0) {
        const int rounds = chunk < 0 ? -chunk : 1;
        const int per_round = std::max(1, resident / nstrips);
        chunk = std::max(1, (rows + per_round * rounds - 1) / (per_round * rounds));
    }
    chunk = std::min(chunk, max_rows);
    q.ctr = nullptr;
    q.big_rows = q.small_rows = chunk;
    q.rows_A = rows;
    q.nA = q.nitems = (rows + chunk - 1) / chunk * nstrips;
    waves = q.nitems;
    return q;
}

static hipError_t launch_pipe(const void *fn, const StencilArgs &a, int gens, int v, unsigned long long *ctr,
                              unsigned long long *base, hipStream_t s) {
    int waves = 0, ns = 0;
    Sched q = plan_items(a, gens, v, fn, ctr, base ? *base : 0ull, waves, ns);
    if (q.nitems <= 0) return hipSuccess;
    const int ipb = items_per_block_of(fn);
    int nb = (waves + ipb - 1) / ipb;
    if (q.ctr && base) *base += (unsigned long long)q.nitems + (unsigned long long)nb * 4;
    StencilArgs aa = a;
    void *args[] = {&aa, &q, &ns, &nb};
    // diagnostic: GOL_LDS_PAD=<bytes> reserves unused LDS per block to cap the
    // number of resident waves (occupancy experiments)
    static const int lds_pad = getenv("GOL_LDS_PAD") ? atoi(getenv("GOL_LDS_PAD")) : 0;
    return hipLaunchKernel(fn, dim3(nb), dim3(block_threads_of(fn)), args, (size_t)lds_pad, s);
}

template <int V, bool Q>
static const void *bit_kernel(int gens) {
    switch (gens) {
    case 1: return (const void *)&bit_pipe_kernel<V, 1, Q>;
    case 2: return (const void *)&bit_pipe_kernel<V, 2, Q>;
    case 3: return (const void *)&bit_pipe_kernel<V, 3, Q>;
    case 4: return (const void *)&bit_pipe_kernel<V, 4, Q>;
    case 5: return (const void *)&bit_pipe_kernel<V, 5, Q>;
    case 6: return (const void *)&bit_pipe_kernel<V, 6, Q>;
    case 7: return (const void *)&bit_pipe_kernel<V, 7, Q>;
    case 8: return (const void *)&bit_pipe_kernel<V, 8, Q>;
    default: return nullptr;
    }
}

template <bool Q>
static const void *byte_kernel(int gens) {
    switch (gens) {
    case 1: return (const void *)&byte_pipe_kernel<1, Q>;
    case 2: return (const void *)&byte_pipe_kernel<2, Q>;
    case 3: return (const void *)&byte_pipe_kernel<3, Q>;
    case 4: return (const void *)&byte_pipe_kernel<4, Q>;
    case 5: return (const void *)&byte_pipe_kernel<5, Q>;
    case 6: return (const void *)&byte_pipe_kernel<6, Q>;
    case 7: return (const void *)&byte_pipe_kernel<7, Q>;
    case 8: return (const void *)&byte_pipe_kernel<8, Q>;
    default: return nullptr;
    }
}

hipError_t launch_bit_pipe(const StencilArgs &a, int gens, int v, unsigned long long *ctr, unsigned long long *base,
                           hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    const bool q = a.chunk_rows == 0 && ctr;
    const void *fn = v == 4 ? (q ? bit_kernel<4, true>(gens) : bit_kernel<4, false>(gens))
                   : v == 8 ? (q ? bit_kernel<8, true>(gens) : bit_kernel<8, false>(gens))
                            : nullptr;
    if (!fn) return hipErrorInvalidValue;
    return launch_pipe(fn, a, gens, v, ctr, base, s);
}

template <int K>
static const void *split_fn() {
    static const void *f = [] {
        const void *p = (const void *)&bit_split_kernel<K>;
        register_split(p);
        return p;
    }();
    return f;
}

hipError_t launch_bit_split(const StencilArgs &a, int gens, hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    const void *fn = gens == 2 ? split_fn<2>() : gens == 4 ? split_fn<4>() : gens == 6 ? split_fn<6>()
                   : gens == 8 ? split_fn<8>() : nullptr;
    if (!fn) return hipErrorInvalidValue;
    StencilArgs aa = a;
    if (aa.chunk_rows == 0) aa.chunk_rows = -4;   // no work-queue variant
    return launch_pipe(fn, aa, gens, 4, nullptr, nullptr, s);
}

bool bytebit_supported(int gens) { return bytebit_strip_cols(gens) > 0; }

hipError_t launch_bytebit_pipe(const StencilArgs &a, int gens, hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    const void *fn = gens == 4    ? (const void *)&bytebit_pipe_kernel<2, 4>
                     : gens == 8  ? (const void *)&bytebit_pipe_kernel<2, 8>
                     : gens == 12 ? (const void *)&bytebit_pipe_kernel<2, 12>
                     : gens == 16 ? (const void *)&bytebit_pipe_kernel<2, 16>
                     : gens == 20 ? (const void *)&bytebit_pipe_kernel<1, 20>
                     : gens == 24 ? (const void *)&bytebit_pipe_kernel<1, 24>
                     : gens == 28 ? (const void *)&bytebit_pipe_kernel<1, 28>
                     : gens == 32 ? (const void *)&bytebit_pipe_kernel<1, 32>
                                  : nullptr;
    if (!fn) return hipErrorInvalidValue;
    StencilArgs aa = a;
    if (aa.chunk_rows == 0) aa.chunk_rows = -4;   // no work-queue variant
    return launch_pipe(fn, aa, gens, -bytebit_strip_cols(gens), nullptr, nullptr, s);
}

hipError_t launch_byte_pipe(const StencilArgs &a, int gens, unsigned long long *ctr, unsigned long long *base,
                            hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    const void *fn = (a.chunk_rows == 0 && ctr) ? byte_kernel<true>(gens) : byte_kernel<false>(gens);
    if (!fn) return hipErrorInvalidValue;
    return launch_pipe(fn, a, gens, 4, ctr, base, s);
}

// ------------------------------------------------------------ MESH_COMPAT fix-up
// Recomputes the 2·m block-edge columns of each row with the swapped column
// halos of distr_borders (main.cpp:51-54): with L = cols/m, j = c mod L, cy = c/L
//   left(c)  = c-1 if j>0; (cy+2)·L-1 if cy+1<m; else dead
//   right(c) = c+1 if j<L-1; (cy-1)·L if cy>=1; else dead
__global__ void mesh_fixup_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                  int64_t pitch, int64_t cols, int m, int row_lo, int row_hi,
                                  int out_r0, int out_r1) {
    const int64_t L = cols / m;
    const int edges = 2 * m;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nrows = out_r1 - out_r0;
    if (t >= nrows * edges) return;
    const int x = out_r0 + (int)(t / edges);
    const int e = (int)(t % edges);
    const int64_t cy = e >> 1;
    const int64_t c = (e & 1) ? cy * L + L - 1 : cy * L;
    const int64_t j = c - cy * L;
    const int64_t cl = j > 0 ? c - 1 : (cy + 1 < m ? (cy + 2) * L - 1 : -1);
    const int64_t cr = j < L - 1 ? c + 1 : (cy >= 1 ? (cy - 1) * L : -1);
    int s = 0;
    for (int dr = -1; dr <= 1; ++dr) {
        const int rr = x + dr;
        if (rr < row_lo || rr >= row_hi) continue;
        const uint8_t *row = src + (int64_t)rr * pitch;
        if (cl >= 0) s += row[cl];
        if (cr >= 0) s += row[cr];
        if (dr != 0) s += row[c];
    }
    const uint8_t alive = src[(int64_t)x * pitch + c];
    const bool valid = x >= row_lo && x < row_hi;
    dst[(int64_t)x * pitch + c] = (valid && (s == 3 || (alive && s == 2))) ? 1 : 0;
}

hipError_t launch_mesh_fixup(const uint8_t *src, uint8_t *dst, int64_t pitch_bytes, int64_t cols, int m,
                             int row_lo, int row_hi, int out_r0, int out_r1, hipStream_t s) {
    const int64_t n = (int64_t)(out_r1 - out_r0) * 2 * m;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mesh_fixup_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst,
                       pitch_bytes, cols, m, row_lo, row_hi, out_r0, out_r1);
    return hipGetLastError();
}

// ------------------------------------------------------------------ init
// glibc TYPE_3 additive generator, x_t = x_{t-3} + x_{t-31} (mod 2^32),
// rand() = x >> 1.  Lanes of a wave take 64 units with the SAME segment index t,
// so the jump matrix M_t = A^{t·seg} is wave-uniform (scalar loads).

template <bool BITS>
__global__ __launch_bounds__(256) void init_units_kernel(const InitUnit *__restrict__ units, int nunits,
                                                         const uint32_t *__restrict__ mats, int seg,
                                                         void *dst, int64_t pitch_bytes) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    const InitUnit &U = units[u < nunits ? u : 0];
    uint32_t w[31], r[31];
#pragma unroll
    for (int i = 0; i < 31; ++i) w[i] = U.w[i];
    if (t == 0) {
#pragma unroll
        for (int i = 0; i < 31; ++i) r[i] = w[i];
    } else {
        const uint32_t *M = mats + (size_t)t * 961;
#pragma unroll
        for (int i = 0; i < 31; ++i) {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 31; ++k) acc += M[i * 31 + k] * w[k];
            r[i] = acc;
        }
    }
    const int start = t * seg;
    int n = U.len - start;
    if (n > seg) n = seg;
    if (u >= nunits) n = 0;
    const int64_t rowoff = U.row * pitch_bytes;
    uint32_t acc = 0;
    for (int base = 0; base < seg; base += 31) {
#pragma unroll
        for (int i = 0; i < 31; ++i) {
            if (base > 0) r[i] += r[(i + 28) % 31];
            const int pos = base + i;
            // (x>>1) % 3 == 0  <=>  (x>>1)·inv(3) mod 2^32 <= 0x55555555
            const uint32_t cell = (pos < n) && ((r[i] >> 1) * 0xAAAAAAABu <= 0x55555555u);
            if (BITS) {
                acc |= cell << (pos & 31);
                if ((pos & 31) == 31) {
                    if (pos - 31 < n) {
                        uint32_t *row = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(dst) + rowoff);
                        row[(U.col0 + start + pos - 31) >> 5] = acc;
                    }
                    acc = 0;
                }
            } else if (pos < n) {
                static_cast<uint8_t *>(dst)[rowoff + U.col0 + start + pos] = (uint8_t)cell;
            }
        }
    }
}

hipError_t launch_init_units(const InitUnit *units, int nunits, const uint32_t *mats, int T, int seg,
                             void *dst, int64_t pitch_bytes, int bit_layout, hipStream_t s) {
    if (nunits <= 0) return hipSuccess;
    dim3 grid((nunits + 255) / 256, T);
    if (bit_layout)
        hipLaunchKernelGGL(init_units_kernel<true>, grid, dim3(256), 0, s, units, nunits, mats, seg, dst,
                           pitch_bytes);
    else
        hipLaunchKernelGGL(init_units_kernel<false>, grid, dim3(256), 0, s, units, nunits, mats, seg, dst,
                           pitch_bytes);
    return hipGetLastError();
}

// ------------------------------------------------------- layout conversion
// Bit layout = quad-interleaved 128-column groups (bit_word / bit_pos, gol_internal.h).

// bytes (window nrows×ncols, leading dim ld) -> bit words of storage rows
// row0.., columns col0..; partially covered words are merged; cells at columns
// >= active_cols are stored as 0.  One thread per word.
__global__ void pack_window_kernel(const uint8_t *__restrict__ bytes, int64_t ld, uint32_t *words,
                                   int64_t pitch, int64_t row0, int64_t col0, int64_t nrows,
                                   int64_t ncols, int64_t active_cols) {
    const int64_t g0 = col0 >> 7, g1 = (col0 + ncols - 1) >> 7;
    const int64_t nw = (g1 - g0 + 1) * 4;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nw * nrows) return;
    const int64_t r = t / nw, wi = g0 * 4 + t % nw;
    uint32_t *pw = words + (row0 + r) * pitch + wi;
    uint32_t v = *pw;
    const uint8_t *src = bytes + r * ld;
    const int64_t cbase = (wi >> 2) * 128 + (wi & 3);
    for (int j = 0; j < 32; ++j) {
        const int64_t c = cbase + 4 * j;
        if (c < col0 || c >= col0 + ncols) continue;
        const uint32_t bit = (c < active_cols && src[c - col0]) ? 1u : 0u;
        v = (v & ~(1u << j)) | (bit << j);
    }
    *pw = v;
}

__global__ void unpack_window_kernel(const uint32_t *__restrict__ words, int64_t pitch, uint8_t *bytes,
                                     int64_t ld, int64_t row0, int64_t col0, int64_t nrows, int64_t ncols) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nrows * ncols) return;
    const int64_t r = t / ncols, c = t % ncols;
    const int64_t gc = col0 + c;
    bytes[r * ld + c] = (words[(row0 + r) * pitch + bit_word(gc)] >> bit_pos(gc)) & 1u;
}

// Linear words (bit i of word w = column 32w+i, as the init kernel writes them)
// -> quad-interleaved groups.  One thread per 128-column group.
__device__ __forceinline__ uint32_t gather_stride4(uint32_t x, int w) {
    x = (x >> w) & 0x11111111u;
    x = (x | (x >> 3)) & 0x03030303u;
    x = (x | (x >> 6)) & 0x000f000fu;
    return (x | (x >> 12)) & 0x000000ffu;
}

__global__ void interleave_rows_kernel(const uint32_t *__restrict__ lin, uint32_t *__restrict__ out,
                                       int64_t pitch, int64_t r0, int64_t nrows, int64_t groups) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nrows * groups) return;
    const int64_t r = r0 + t / groups, gidx = t % groups;
    const uint4 W = *reinterpret_cast<const uint4 *>(lin + r * pitch + gidx * 4);
    uint4 o;
    uint32_t *po = reinterpret_cast<uint32_t *>(&o);
#pragma unroll
    for (int w = 0; w < 4; ++w)
        po[w] = gather_stride4(W.x, w) | (gather_stride4(W.y, w) << 8) | (gather_stride4(W.z, w) << 16) |
                (gather_stride4(W.w, w) << 24);
    *reinterpret_cast<uint4 *>(out + r * pitch + gidx * 4) = o;
}

hipError_t launch_interleave_rows(const uint32_t *lin, uint32_t *out, int64_t pitch_words, int64_t r0,
                                  int64_t nrows, int64_t groups, hipStream_t s) {
    const int64_t n = nrows * groups;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(interleave_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lin, out,
                       pitch_words, r0, nrows, groups);
    return hipGetLastError();
}

hipError_t launch_pack_window(const uint8_t *bytes, int64_t ld, uint32_t *words, int64_t pitch_words,
                              int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                              int64_t active_cols, hipStream_t s) {
    if (nrows <= 0 || ncols <= 0) return hipSuccess;
    const int64_t nw = (((col0 + ncols - 1) >> 7) - (col0 >> 7) + 1) * 4;
    const int64_t n = nw * nrows;
    hipLaunchKernelGGL(pack_window_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bytes, ld,
                       words, pitch_words, row0, col0, nrows, ncols, active_cols);
    return hipGetLastError();
}

hipError_t launch_unpack_window(const uint32_t *words, int64_t pitch_words, uint8_t *bytes, int64_t ld,
                                int64_t row0, int64_t col0, int64_t nrows, int64_t ncols, hipStream_t s) {
    const int64_t n = nrows * ncols;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_window_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, words,
                       pitch_words, bytes, ld, row0, col0, nrows, ncols);
    return hipGetLastError();
}

// ------------------------------------------------------------------ popcount
// Cells are 0/1 bytes or bits, so popc of every dword counts live cells in both layouts.
__global__ void popcount_kernel(const uint32_t *__restrict__ buf, int64_t pitch_words, int64_t r0,
                                int64_t nrows, int64_t row_words, unsigned long long *acc) {
    const int64_t n = nrows * row_words;
    unsigned long long local = 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / row_words, c = t % row_words;
        local += __popc(buf[(r0 + r) * pitch_words + c]);
    }
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, local);
}

hipError_t launch_popcount(const void *buf, int64_t pitch_bytes, int64_t r0, int64_t r1, int64_t row_bytes,
                           unsigned long long *acc, int bit_layout, hipStream_t s) {
    (void)bit_layout;
    const int64_t nrows = r1 - r0, row_words = (row_bytes + 3) / 4;
    if (nrows <= 0) return hipSuccess;
    int64_t blocks = (nrows * row_words + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(popcount_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint32_t *>(buf), pitch_bytes / 4, r0, nrows, row_words, acc);
    return hipGetLastError();
}

} // namespace gol
