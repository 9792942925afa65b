// hbm_probe — STREAM-style calibration of the achievable HBM bandwidth on this
// GPU, for the roofline of the stencil kernels.
// Tool, not product:  hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
// Prints one JSON line per probe: copy (1 R + 1 W), read-only, write-only over
// 2 GiB buffers (the size of one 131072² bit board), 16 B per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// grid-stride copy, UNROLL independent 16-B loads in flight per lane
template <int UNROLL, int AUX>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * stride]);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (AUX) __builtin_nontemporal_store(v[u], &dst[i + u * stride]);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// each wave streams a contiguous chunk of rows (the stencil's access shape):
// rows of `row_v` 16-B vectors at a pitch of `pv` vectors, a wave covers
// 64 lanes × 16 B = 1 KiB of a row
__global__ __launch_bounds__(256) void chunk_copy_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                         size_t row_v, size_t pv, size_t rows, int chunk) {
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t strips = row_v / 64;
    const size_t strip = w % strips, band = w / strips;
    const size_t r0 = band * chunk;
    if (r0 >= rows) return;
    const size_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
    size_t r = r0;
    for (; r + 3 < r1; r += 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[(r + u) * pv + strip * 64 + lane];
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[(r + u) * pv + strip * 64 + lane] = v[u];
    }
    for (; r < r1; ++r) dst[r * pv + strip * 64 + lane] = src[r * pv + strip * 64 + lane];
}

// each wave copies one contiguous span of `span` 16-B vectors, UNROLL wave-wide
// (1 KiB) pieces in flight; AUX = cache-policy bits of the raw buffer ops
template <int UNROLL, int AUX>
__global__ __launch_bounds__(256) void span_copy_kernel(const u32x4 *src, u32x4 *dst, size_t n, size_t span) {
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t v0 = w * span;
    if (v0 >= n) return;
    const size_t v1 = v0 + span < n ? v0 + span : n;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(src + v0), 0,
                                                                   (int)((v1 - v0) * 16), 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst + v0, 0, (int)((v1 - v0) * 16), 0x00020000);
    const size_t len = v1 - v0;
    for (size_t i = 0; i < len; i += 64 * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((i + u * 64 + lane) * 16), 0, AUX);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((i + u * 64 + lane) * 16), 0, AUX);
    }
}

// the stencil's shape with the stencil's raw buffer ops and cache policy AUX
template <int AUX>
__global__ __launch_bounds__(256) void chunk_copy_buf_kernel(const u32x4 *src, u32x4 *dst, size_t row_v, size_t pv,
                                                             size_t rows, int chunk) {
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t strips = row_v / 64;
    const size_t strip = w % strips, band = w / strips;
    const size_t r0 = band * chunk;
    if (r0 >= rows) return;
    const size_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
    const size_t base = r0 * pv + strip * 64;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(src + base), 0,
                                                                   (int)((r1 - r0) * pv * 16), 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, (int)((r1 - r0) * pv * 16),
                                                                   0x00020000);
    for (size_t r = 0; r < r1 - r0; r += 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(((r + u) * pv + lane) * 16), 0, AUX);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)(((r + u) * pv + lane) * 16), 0, AUX);
    }
}

template <int UNROLL>
__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ src, unsigned *out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const u32x4 v = src[i + u * stride];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ __launch_bounds__(256) void write_kernel(u32x4 *__restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        u32x4 v;
        v.x = v.y = v.z = v.w = (unsigned)i;
        dst[i] = v;
    }
}

template <typename F>
static void timeit(const char *name, double bytes, F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    const int reps = 10;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double s = ms * 1e-3 / reps;
    printf("{\"probe\": \"%s\", \"GBps\": %.1f, \"frac_of_8TBps\": %.3f, \"ms\": %.4f}\n", name, bytes / s / 1e9,
           bytes / s / 8e12, s * 1e3);
    fflush(stdout);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main() {
    const size_t bytes = 2ull << 30;
    const size_t n = bytes / 16;
    const size_t alloc = bytes + (64ull << 20);   // room for padded row pitches
    u32x4 *s, *d;
    unsigned *o;
    CHK(hipMalloc(&s, alloc));
    CHK(hipMalloc(&d, alloc));
    CHK(hipMalloc(&o, 4));
    CHK(hipMemset(s, 1, alloc));
    CHK(hipMemset(d, 0, alloc));
    const size_t row_v = 16384 / 16, rows = 131072;
    if (getenv("PROBE_PITCH")) {
        // the stencil's shape at row pitches of 16 KiB + pad (power-of-two pitches
        // alias HBM channels: DESIGN.md §3): algorithmic bytes = 2 × 2 GiB of rows
        for (int rep = 0; rep < 2; ++rep)
            for (int pad : {0, 128, 256}) {
                const size_t pv = row_v + pad / 16;
                for (int chunk : {8, 16}) {
                    const size_t waves = (row_v / 64) * ((rows + chunk - 1) / chunk);
                    char nm[96];
                    snprintf(nm, sizeof nm, "row-chunk copy pitch+%d %d rows", pad, chunk);
                    timeit(nm, 2.0 * bytes,
                           [&] { chunk_copy_kernel<<<(waves + 3) / 4, 256>>>(s, d, row_v, pv, rows, chunk); });
                    snprintf(nm, sizeof nm, "row-chunk copy buffer ops nt pitch+%d %d rows", pad, chunk);
                    timeit(nm, 2.0 * bytes,
                           [&] { chunk_copy_buf_kernel<2><<<(waves + 3) / 4, 256>>>(s, d, row_v, pv, rows, chunk); });
                }
            }
        return 0;
    }
    for (int blocks : {2048, 8192, 16384}) {
        char nm[96];
        snprintf(nm, sizeof nm, "copy u4 %d blocks", blocks);
        timeit(nm, 2.0 * bytes, [&] { copy_kernel<4, 0><<<blocks, 256>>>(s, d, n); });
        snprintf(nm, sizeof nm, "copy u4 nt-store %d blocks", blocks);
        timeit(nm, 2.0 * bytes, [&] { copy_kernel<4, 1><<<blocks, 256>>>(s, d, n); });
        snprintf(nm, sizeof nm, "copy u8 nt-store %d blocks", blocks);
        timeit(nm, 2.0 * bytes, [&] { copy_kernel<8, 1><<<blocks, 256>>>(s, d, n); });
        snprintf(nm, sizeof nm, "read u4 %d blocks", blocks);
        timeit(nm, 1.0 * bytes, [&] { read_kernel<4><<<blocks, 256>>>(s, o, n); });
        snprintf(nm, sizeof nm, "write %d blocks", blocks);
        timeit(nm, 1.0 * bytes, [&] { write_kernel<<<blocks, 256>>>(d, n); });
    }
    // contiguous spans per wave (4 KiB .. 256 KiB), 4 or 8 pieces in flight, plain and nt policy
    for (size_t span_kib : {4, 8, 16, 64}) {
        const size_t span = span_kib * 64;   // 16-B vectors
        const size_t waves = (n + span - 1) / span;
        char nm[96];
        snprintf(nm, sizeof nm, "span copy %zu KiB/wave x8", span_kib);
        timeit(nm, 2.0 * bytes, [&] { span_copy_kernel<8, 0><<<(waves + 3) / 4, 256>>>(s, d, n, span); });
        snprintf(nm, sizeof nm, "span copy %zu KiB/wave x4", span_kib);
        timeit(nm, 2.0 * bytes, [&] { span_copy_kernel<4, 0><<<(waves + 3) / 4, 256>>>(s, d, n, span); });
        snprintf(nm, sizeof nm, "span copy %zu KiB/wave x8 nt", span_kib);
        timeit(nm, 2.0 * bytes, [&] { span_copy_kernel<8, 2><<<(waves + 3) / 4, 256>>>(s, d, n, span); });
    }
    // the stencil's shape: 131072 rows of 16 KiB, one wave per (1 KiB strip, chunk of rows)
    for (int chunk : {8, 16, 32, 64}) {
        const size_t waves = (row_v / 64) * ((rows + chunk - 1) / chunk);
        char nm[96];
        snprintf(nm, sizeof nm, "row-chunk copy %d rows", chunk);
        timeit(nm, 2.0 * bytes, [&] { chunk_copy_kernel<<<(waves + 3) / 4, 256>>>(s, d, row_v, row_v, rows, chunk); });
        snprintf(nm, sizeof nm, "row-chunk copy buffer ops %d rows", chunk);
        timeit(nm, 2.0 * bytes, [&] { chunk_copy_buf_kernel<0><<<(waves + 3) / 4, 256>>>(s, d, row_v, row_v, rows, chunk); });
        snprintf(nm, sizeof nm, "row-chunk copy buffer ops nt %d rows", chunk);
        timeit(nm, 2.0 * bytes, [&] { chunk_copy_buf_kernel<2><<<(waves + 3) / 4, 256>>>(s, d, row_v, row_v, rows, chunk); });
    }
    (void)hipMemcpy(d, s, bytes, hipMemcpyDeviceToDevice);
    timeit("hipMemcpy D2D", 2.0 * bytes, [&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
