// Snapshot text on the device: the `.gol` part-file body of main.cpp:106-129
// (`writeBoardToFile`: per row one "0\t"/"1\t" token per cell, then "\n").
//
// At 131072² a snapshot is 34 GB of text; formatting it on the host from a
// downloaded board is a serial byte loop, so the text is produced (and, for
// resume, parsed back) by HBM-bound kernels and only the finished bytes cross
// PCIe.  The runtime pipelines blocks of rows through pinned buffers
// (gol_runtime.cpp text_out / text_in).
#include "gol_internal.h"

namespace gol {

namespace {

constexpr int kTextBytesPerThread = 16;

// One thread writes 16 consecutive text bytes (one 16-byte store when aligned).
template <bool BIT>
__global__ __launch_bounds__(256) void format_text_kernel(const uint8_t *__restrict__ buf, int64_t pitch_bytes,
                                                          int64_t srow0, int64_t col0, int64_t nrows,
                                                          int64_t ncols, int pm, int64_t pL, int gw,
                                                          char *__restrict__ text) {
    const int64_t rowlen = 2 * ncols + 1, total = nrows * rowlen;
    const int64_t off = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kTextBytesPerThread;
    if (off >= total) return;
    int64_t r = off / rowlen, p = off - r * rowlen;
    union {
        uint4 v;
        char b[kTextBytesPerThread];
    } out;
#pragma unroll
    for (int i = 0; i < kTextBytesPerThread; ++i) {
        char ch = 0;
        if (r < nrows) {
            if (p == rowlen - 1) {
                ch = '\n';
            } else if (p & 1) {
                ch = '\t';
            } else {
                const int64_t lc = col0 + (p >> 1);
                const int64_t c = pm > 1 ? (pm - 1 - lc / pL) * pL + lc % pL : lc;   // storage column
                const uint8_t *row = buf + (srow0 + r) * pitch_bytes;
                unsigned v;
                if (BIT)
                    v = (reinterpret_cast<const uint32_t *>(row)[bit_word(c, gw)] >> bit_pos(c, gw)) & 1u;
                else
                    v = row[c] & 1u;
                ch = (char)('0' + v);
            }
        }
        out.b[i] = ch;
        if (++p == rowlen) {
            p = 0;
            ++r;
        }
    }
    if (off + kTextBytesPerThread <= total) {
        *reinterpret_cast<uint4 *>(text + off) = out.v;   // text buffers are 256-byte aligned
    } else {
        for (int i = 0; off + i < total; ++i) text[off + i] = out.b[i];
    }
}

// One thread parses 16 cells of one row; the thread holding a row's last cell
// also checks the newline.  Anything but "0\t"/"1\t" ... "\n" is reported.
__global__ __launch_bounds__(256) void parse_text_kernel(const char *__restrict__ text, int64_t nrows,
                                                         int64_t ncols, uint8_t *__restrict__ cells, int64_t ld,
                                                         int64_t err_base, unsigned long long *err) {
    const int64_t per_row = (ncols + 15) / 16;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nrows * per_row) return;
    const int64_t r = t / per_row, c0 = (t - r * per_row) * 16;
    const int64_t rowlen = 2 * ncols + 1;
    const char *src = text + r * rowlen;
    uint8_t *dst = cells + r * ld;
    unsigned long long bad = ~0ull;
    const int n = (int)(ncols - c0 < 16 ? ncols - c0 : 16);
    for (int i = 0; i < n; ++i) {
        const int64_t c = c0 + i;
        const char v = src[2 * c], sep = src[2 * c + 1];
        const bool ok = (v == '0' || v == '1') && sep == '\t';
        if (!ok && bad == ~0ull) bad = (unsigned long long)(r * rowlen + 2 * c + ((v == '0' || v == '1') ? 1 : 0));
        dst[c] = (uint8_t)(v == '1');
    }
    if (c0 + n == ncols && src[rowlen - 1] != '\n' && bad == ~0ull)
        bad = (unsigned long long)(r * rowlen + rowlen - 1);
    if (bad != ~0ull) atomicMin(err, (unsigned long long)err_base + bad);
}

} // namespace

hipError_t launch_format_text(const void *buf, int64_t pitch_bytes, int bit_gw, int64_t srow0, int64_t col0,
                              int64_t nrows, int64_t ncols, int perm_m, int64_t perm_L, char *text, hipStream_t s) {
    const int64_t total = nrows * (2 * ncols + 1);
    if (nrows <= 0 || ncols <= 0) return hipSuccess;
    const int64_t threads = (total + kTextBytesPerThread - 1) / kTextBytesPerThread;
    const dim3 grid((unsigned)((threads + 255) / 256));
    const uint8_t *b = static_cast<const uint8_t *>(buf);
    if (bit_gw)
        hipLaunchKernelGGL(format_text_kernel<true>, grid, dim3(256), 0, s, b, pitch_bytes, srow0, col0, nrows,
                           ncols, perm_m, perm_L, bit_gw, text);
    else
        hipLaunchKernelGGL(format_text_kernel<false>, grid, dim3(256), 0, s, b, pitch_bytes, srow0, col0, nrows,
                           ncols, perm_m, perm_L, 0, text);
    return hipGetLastError();
}

hipError_t launch_parse_text(const char *text, int64_t nrows, int64_t ncols, uint8_t *cells, int64_t ld,
                             int64_t err_base, unsigned long long *err, hipStream_t s) {
    if (nrows <= 0 || ncols <= 0) return hipSuccess;
    const int64_t threads = nrows * ((ncols + 15) / 16);
    hipLaunchKernelGGL(parse_text_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, text, nrows,
                       ncols, cells, ld, err_base, err);
    return hipGetLastError();
}

} // namespace gol
