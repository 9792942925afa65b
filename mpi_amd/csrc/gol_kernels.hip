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
//  * byte layout: 1 cell per byte; SWAR sums (v_add3_u32) of 4 cells per dword.
#include "gol_internal.h"

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
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    return (a & b) | (a & c) | (b & c);
}

// XCD-aware block remap: consecutive logical blocks land on one XCD (blocks are
// dealt round-robin over the 8 XCDs), so neighbouring strips/chunks share an L2.
// Bijective for any nblocks.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7, x = b & 7, i = b >> 3;
    return (x < r) ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

template <int V> struct Vec;
template <> struct Vec<1> { using T = uint32_t; };
template <> struct Vec<2> { using T = uint2; };
template <> struct Vec<4> { using T = uint4; };

template <int V>
__device__ __forceinline__ void load_vec(uint32_t (&d)[V], const uint32_t *p) {
    typename Vec<V>::T t = *reinterpret_cast<const typename Vec<V>::T *>(p);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(&t);
#pragma unroll
    for (int j = 0; j < V; ++j) d[j] = q[j];
}
template <int V>
__device__ __forceinline__ void store_vec(uint32_t *p, const uint32_t (&s)[V]) {
    typename Vec<V>::T t;
    uint32_t *q = reinterpret_cast<uint32_t *>(&t);
#pragma unroll
    for (int j = 0; j < V; ++j) q[j] = s[j];
    *reinterpret_cast<typename Vec<V>::T *>(p) = t;
}

// Per-wave geometry shared by both pipelines.
template <int V>
struct Strip {
    int64_t word0;     // first word of this lane
    bool lane_in;      // lane's words lie inside the row pitch (loadable)
    bool lane_store;   // lane stores its words (not a halo lane, inside the active row)
    uint32_t mask[V];  // active-cell mask per word
    int R0, R1;        // output rows of this wave's chunk

    __device__ __forceinline__ bool init(const StencilArgs &a, int nstrips, int nchunks, int nblocks,
                                         uint32_t full) {
        const int lane = threadIdx.x & 63;
        const int w = xcd_remap(blockIdx.x, nblocks) * 4 + (threadIdx.x >> 6);
        if (w >= nstrips * nchunks) return false;
        const int chunk = w / nstrips, strip = w - chunk * nstrips;
        const int nr = (a.nunits + V - 1) / V * V;   // active words rounded to V (<= pitch)
        int base = strip * 62 * V;
        const int last = nr - 62 * V;
        if (base > last) base = last > 0 ? last : 0;
        word0 = (int64_t)base - V + (int64_t)lane * V;
        lane_in = word0 >= 0 && word0 + V <= a.pitch;
        lane_store = lane >= 1 && lane <= 62 && word0 < nr;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int64_t wi = word0 + j;
            mask[j] = (wi < 0 || wi >= a.nunits) ? 0u : (wi == a.nunits - 1 ? a.last_mask : full);
        }
        R0 = a.out_r0 + chunk * a.chunk_rows;
        R1 = min(R0 + a.chunk_rows, a.out_r1);
        return true;
    }
};

// ---------------------------------------------------------------- bit layout

template <int V, int K>
struct BitState {
    uint32_t h0[K][3][V], h1[K][3][V], c[K][3][V];
    uint32_t ld[3][V];
};

// B3/S23 on bit-sliced horizontal 3-sums of rows above (a), at (b), below (c):
// 9-sum incl. self = o + 2u + 4(q+v); next = (sum==3) | (alive & sum==4).
__device__ __forceinline__ uint32_t life_bits(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                              uint32_t c0, uint32_t c1, uint32_t alive,
                                              uint32_t mask) {
    const uint32_t o = a0 ^ b0 ^ c0;
    const uint32_t co = maj3(a0, b0, c0);
    const uint32_t p = a1 ^ b1 ^ c1;
    const uint32_t q = maj3(a1, b1, c1);
    const uint32_t u = (co ^ p) & mask;
    const uint32_t s = q ^ (co & p);
    const uint32_t m = (u & o & ~s) | (~u & ~o & s);
    return m & (u | alive);
}

template <int V, int K, int P>
__device__ __forceinline__ void bit_phase(BitState<V, K> &S, const Strip<V> &st, const StencilArgs &a,
                                          const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                          int it, int N) {
    const int rho = st.R0 - K + it;   // generation-0 row arriving this iteration
    uint32_t nv[V];
#pragma unroll
    for (int j = 0; j < V; ++j) nv[j] = S.ld[P][j];
    {   // prefetch row rho+3 into the slot just consumed
        const int rr = rho + 3;
#pragma unroll
        for (int j = 0; j < V; ++j) S.ld[P][j] = 0u;
        if (it + 3 < N && rr >= a.row_lo && rr < a.row_hi && st.lane_in)
            load_vec<V>(S.ld[P], src + (int64_t)rr * a.pitch + st.word0);
    }
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P;
#pragma unroll
    for (int g = 0; g < K; ++g) {
        // nv = generation g, row rho-g: horizontal 3-sums into slot C
        const uint32_t lft = from_left_lane(nv[V - 1]);
        const uint32_t rgt = from_right_lane(nv[0]);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const uint32_t pv = j == 0 ? lft : nv[j - 1];
            const uint32_t nx = j == V - 1 ? rgt : nv[j + 1];
            const uint32_t L = funnel(nv[j], pv, 31);   // column c-1
            const uint32_t R = funnel(nx, nv[j], 1);    // column c+1
            S.h0[g][C][j] = L ^ nv[j] ^ R;
            S.h1[g][C][j] = maj3(L, nv[j], R);
            S.c[g][C][j] = nv[j];
        }
        // generation g+1, row rho-g-1
        const int x = rho - g - 1;
        const bool valid = x >= a.row_lo && x < a.row_hi;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const uint32_t o = life_bits(S.h0[g][A][j], S.h1[g][A][j], S.h0[g][B][j], S.h1[g][B][j],
                                         S.h0[g][C][j], S.h1[g][C][j], S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
    if (it >= 2 * K && st.lane_store)
        store_vec<V>(dst + (int64_t)(rho - K) * a.pitch + st.word0, nv);
}

template <int V, int K>
__global__ __launch_bounds__(256) void bit_pipe_kernel(StencilArgs a, int nstrips, int nchunks,
                                                       int nblocks) {
    Strip<V> st;
    if (!st.init(a, nstrips, nchunks, nblocks, 0xffffffffu)) return;   // wave-uniform
    const uint32_t *__restrict__ src = static_cast<const uint32_t *>(a.src);
    uint32_t *__restrict__ dst = static_cast<uint32_t *>(a.dst);
    BitState<V, K> S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < V; ++j) S.h0[g][s][j] = S.h1[g][s][j] = S.c[g][s][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int rr = st.R0 - K + s;
#pragma unroll
        for (int j = 0; j < V; ++j) S.ld[s][j] = 0u;
        if (s < N && rr >= a.row_lo && rr < a.row_hi && st.lane_in)
            load_vec<V>(S.ld[s], src + (int64_t)rr * a.pitch + st.word0);
    }
    for (int it = 0; it < N; it += 3) {
        bit_phase<V, K, 0>(S, st, a, src, dst, it, N);
        if (it + 1 < N) bit_phase<V, K, 1>(S, st, a, src, dst, it + 1, N);
        if (it + 2 < N) bit_phase<V, K, 2>(S, st, a, src, dst, it + 2, N);
    }
}

// --------------------------------------------------------------- byte layout
// V = 4 dwords = 16 cells per lane.  Vertical sums first (v_add3 of 3 rows),
// then horizontal byte shifts of the vertical sums.

template <int K>
struct ByteState {
    uint32_t c[K][3][4];
    uint32_t ld[3][4];
};

// s8 = 9-sum − self; next = ((s8 | alive) == 3), SWAR over 4 bytes (values < 16).
__device__ __forceinline__ uint32_t life_bytes(uint32_t t9, uint32_t alive, uint32_t mask) {
    const uint32_t s8 = t9 - alive;
    const uint32_t y = (s8 | alive) ^ 0x03030303u;
    const uint32_t z = y + 0x7f7f7f7fu;
    return (~z >> 7) & mask;   // mask ⊆ 0x01010101
}

template <int K, int P>
__device__ __forceinline__ void byte_phase(ByteState<K> &S, const Strip<4> &st, const StencilArgs &a,
                                           const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                           int it, int N) {
    const int rho = st.R0 - K + it;
    uint32_t nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) nv[j] = S.ld[P][j];
    {
        const int rr = rho + 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) S.ld[P][j] = 0u;
        if (it + 3 < N && rr >= a.row_lo && rr < a.row_hi && st.lane_in)
            load_vec<4>(S.ld[P], src + (int64_t)rr * a.pitch + st.word0);
    }
    constexpr int A = (P + 1) % 3, B = (P + 2) % 3, C = P;
#pragma unroll
    for (int g = 0; g < K; ++g) {
        uint32_t vs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            S.c[g][C][j] = nv[j];
            vs[j] = S.c[g][A][j] + S.c[g][B][j] + nv[j];   // v_add3_u32, bytes <= 3
        }
        const uint32_t lft = from_left_lane(vs[3]);
        const uint32_t rgt = from_right_lane(vs[0]);
        const int x = rho - g - 1;
        const bool valid = x >= a.row_lo && x < a.row_hi;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t pv = j == 0 ? lft : vs[j - 1];
            const uint32_t nx = j == 3 ? rgt : vs[j + 1];
            const uint32_t t9 = funnel(vs[j], pv, 24) + vs[j] + funnel(nx, vs[j], 8);
            const uint32_t o = life_bytes(t9, S.c[g][B][j], st.mask[j]);
            nv[j] = valid ? o : 0u;
        }
    }
    if (it >= 2 * K && st.lane_store)
        store_vec<4>(dst + (int64_t)(rho - K) * a.pitch + st.word0, nv);
}

template <int K>
__global__ __launch_bounds__(256) void byte_pipe_kernel(StencilArgs a, int nstrips, int nchunks,
                                                        int nblocks) {
    Strip<4> st;
    if (!st.init(a, nstrips, nchunks, nblocks, 0x01010101u)) return;
    const uint32_t *__restrict__ src = static_cast<const uint32_t *>(a.src);
    uint32_t *__restrict__ dst = static_cast<uint32_t *>(a.dst);
    ByteState<K> S;
#pragma unroll
    for (int g = 0; g < K; ++g)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) S.c[g][s][j] = 0u;
    const int N = (st.R1 - st.R0) + 2 * K;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int rr = st.R0 - K + s;
#pragma unroll
        for (int j = 0; j < 4; ++j) S.ld[s][j] = 0u;
        if (s < N && rr >= a.row_lo && rr < a.row_hi && st.lane_in)
            load_vec<4>(S.ld[s], src + (int64_t)rr * a.pitch + st.word0);
    }
    for (int it = 0; it < N; it += 3) {
        byte_phase<K, 0>(S, st, a, src, dst, it, N);
        if (it + 1 < N) byte_phase<K, 1>(S, st, a, src, dst, it + 1, N);
        if (it + 2 < N) byte_phase<K, 2>(S, st, a, src, dst, it + 2, N);
    }
}

// ------------------------------------------------------------ launch helpers

static inline void strip_grid(const StencilArgs &a, int v, int &nstrips, int &nchunks, int &nblocks) {
    const int nr = (a.nunits + v - 1) / v * v;
    const int per = 62 * v;
    nstrips = nr <= per ? 1 : (nr + per - 1) / per;
    const int rows = a.out_r1 - a.out_r0;
    nchunks = (rows + a.chunk_rows - 1) / a.chunk_rows;
    nblocks = (nstrips * nchunks + 3) / 4;
}

template <int V>
static hipError_t bit_dispatch(const StencilArgs &a, int gens, hipStream_t s) {
    int ns, nc, nb;
    strip_grid(a, V, ns, nc, nb);
    if (nb == 0) return hipSuccess;
    switch (gens) {
#define GOL_CASE(k) \
    case k: hipLaunchKernelGGL((bit_pipe_kernel<V, k>), dim3(nb), dim3(256), 0, s, a, ns, nc, nb); break;
        GOL_CASE(1) GOL_CASE(2) GOL_CASE(3) GOL_CASE(4) GOL_CASE(5) GOL_CASE(6) GOL_CASE(7) GOL_CASE(8)
#undef GOL_CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_bit_pipe(const StencilArgs &a, int gens, int v, hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    switch (v) {
    case 1: return bit_dispatch<1>(a, gens, s);
    case 2: return bit_dispatch<2>(a, gens, s);
    case 4: return bit_dispatch<4>(a, gens, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_byte_pipe(const StencilArgs &a, int gens, hipStream_t s) {
    if (a.out_r1 <= a.out_r0) return hipSuccess;
    int ns, nc, nb;
    strip_grid(a, 4, ns, nc, nb);
    switch (gens) {
#define GOL_CASE(k) \
    case k: hipLaunchKernelGGL((byte_pipe_kernel<k>), dim3(nb), dim3(256), 0, s, a, ns, nc, nb); break;
        GOL_CASE(1) GOL_CASE(2) GOL_CASE(3) GOL_CASE(4) GOL_CASE(5) GOL_CASE(6) GOL_CASE(7) GOL_CASE(8)
#undef GOL_CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
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

// bytes (window nrows×ncols, leading dim ld) -> bit words of storage rows
// row0.., columns col0..; partial edge words are merged; cells at columns >=
// active_cols are stored as 0.
__global__ void pack_window_kernel(const uint8_t *__restrict__ bytes, int64_t ld, uint32_t *words,
                                   int64_t pitch, int64_t row0, int64_t col0, int64_t nrows,
                                   int64_t ncols, int64_t active_cols) {
    const int64_t w0 = col0 >> 5, w1 = (col0 + ncols - 1) >> 5;
    const int64_t nw = w1 - w0 + 1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nw * nrows) return;
    const int64_t r = t / nw, wi = w0 + t % nw;
    uint32_t *pw = words + (row0 + r) * pitch + wi;
    uint32_t v = *pw;
    const uint8_t *src = bytes + r * ld;
    for (int j = 0; j < 32; ++j) {
        const int64_t c = wi * 32 + j;
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
    bytes[r * ld + c] = (words[(row0 + r) * pitch + (gc >> 5)] >> (gc & 31)) & 1u;
}

hipError_t launch_pack_window(const uint8_t *bytes, int64_t ld, uint32_t *words, int64_t pitch_words,
                              int64_t row0, int64_t col0, int64_t nrows, int64_t ncols,
                              int64_t active_cols, hipStream_t s) {
    if (nrows <= 0 || ncols <= 0) return hipSuccess;
    const int64_t nw = ((col0 + ncols - 1) >> 5) - (col0 >> 5) + 1;
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
