// band_probe — why the fused byte kernel streams slower than the k=1 kernel.
// Tool, not product:  hipcc --offload-arch=gfx950 -O3 -o tools/band_probe tools/band_probe.hip
//
// Models the bytebit kernel's memory pattern on a 32768 x 32768 byte board
// (pitch 32768 + 512 B): one wave per (strip, chunk), a strip = 2048 B of a
// row (64 lanes x 2 x 16 B), a wave walks its chunk's rows top-down reading
// row r + 2 and writing row r, with W dependent VALU ops per row between the
// two (the stages' compute), at 2 waves/SIMD (64 KiB of LDS per block).
//   layout 0: row-major (row r at r * pitch)
//   layout 1: band-interleaved: with B bands of h rows, row r = band b, offset t
//             lives at memory row t * B + b, so the rows that all bands read at
//             the same moment are adjacent in memory.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// row r of band `band` (t = r - r0): byte offset of its first column
__device__ __forceinline__ size_t row_addr(int t, int r0, int band, int layout, int nb, size_t pitch) {
    return layout == 0 ? (size_t)(r0 + t) * pitch : ((size_t)t * nb + band) * pitch;
}

template <int P>
__device__ __forceinline__ void step(u32x4 (&a)[3][2], const unsigned char *src, unsigned char *dst, int t, int n,
                                     int r0, int band, int layout, int nb, size_t pitch, size_t col, int work,
                                     unsigned &acc) {
    constexpr int slot = P % 3, nxt = (P + 2) % 3;
    const int tt = min(t + 2, n - 1);
#pragma unroll
    for (int q = 0; q < 2; ++q)
        a[nxt][q] = *(const u32x4 *)(src + row_addr(tt, r0, band, layout, nb, pitch) + col + 16 * q);
    u32x4 v0 = a[slot][0], v1 = a[slot][1];
    unsigned x = v0.x ^ v1.y;
    for (int i = 0; i < work; ++i) x = __builtin_amdgcn_bitop3_b32(x, acc, v0.z, 0x96);
    acc ^= x;
    v0.x ^= (acc & 0x80000000u);
    if (t < n) {
        *(u32x4 *)(dst + row_addr(t, r0, band, layout, nb, pitch) + col) = v0;
        *(u32x4 *)(dst + row_addr(t, r0, band, layout, nb, pitch) + col + 16) = v1;
    }
}

__global__ __launch_bounds__(256) void walk_kernel(const unsigned char *src, unsigned char *dst, int rows, size_t pitch,
                                                   int strips, int h, int nb, int layout, int work, int nitems) {
    extern __shared__ unsigned pad[];
    if (work < 0) pad[threadIdx.x] = 0;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nitems) return;
    const int band = w / strips, strip = w - band * strips;
    const int r0 = band * h, n = min(h, rows - r0);
    const size_t col = (size_t)strip * 2048 + lane * 32;
    u32x4 a[3][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q)
            a[s][q] = *(const u32x4 *)(src + row_addr(min(s, n - 1), r0, band, layout, nb, pitch) + col + 16 * q);
    unsigned acc = lane;
    for (int t = 0; t < n; t += 3) {
        step<0>(a, src, dst, t, n, r0, band, layout, nb, pitch, col, work, acc);
        step<1>(a, src, dst, t + 1, n, r0, band, layout, nb, pitch, col, work, acc);
        step<2>(a, src, dst, t + 2, n, r0, band, layout, nb, pitch, col, work, acc);
    }
    if (acc == 0x12345u) dst[0] = 1;
}

int main(int argc, char **argv) {
    const int rows = 32768;
    const size_t pitch = 32768 + 512;
    const int strips = 16;   // 16 x 2048 B = the row
    unsigned char *src, *dst;
    CHK(hipMalloc(&src, rows * pitch));
    CHK(hipMalloc(&dst, rows * pitch));
    CHK(hipMemset(src, 1, rows * pitch));
    CHK(hipFuncSetAttribute((const void *)walk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int works[] = {0, 100, 300};
    const int hs[] = {16, 64, 256};
    for (int rep = 0; rep < 2; ++rep)
        for (int work : works)
            for (int h : hs)
                for (int layout = 0; layout < 2; ++layout) {
                    if (layout == 1 && h != 256) continue;
                    const int nb = (rows + h - 1) / h, nitems = nb * strips, blocks = (nitems + 3) / 4;
                    for (int it = 0; it < 3; ++it)
                        hipLaunchKernelGGL(walk_kernel, dim3(blocks), dim3(256), 65536, 0, src, dst, rows, pitch, strips,
                                           h, nb, layout, work, nitems);
                    CHK(hipEventRecord(e0));
                    const int reps = 10;
                    for (int it = 0; it < reps; ++it)
                        hipLaunchKernelGGL(walk_kernel, dim3(blocks), dim3(256), 65536, 0, src, dst, rows, pitch, strips,
                                           h, nb, layout, work, nitems);
                    CHK(hipEventRecord(e1));
                    CHK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    const double bytes = 2.0 * rows * 32768.0 * reps;
                    printf("{\"rep\": %d, \"work\": %d, \"h\": %d, \"layout\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", rep,
                           work, h, layout ? "band-interleaved" : "row-major", ms / reps, bytes / (ms * 1e-3) / 1e9);
                    fflush(stdout);
                }
    return 0;
}
