// A host-only stand-in for the HIP runtime and the gfx950 kernel launchers
// (test infrastructure): libgolhip's runtime (gol_runtime.cpp, compiled with
// g++) linked against it runs its whole host logic on the CPU — streams,
// events, waits and syncs become inert handles, copies and fills act on host
// memory, kernel launches do nothing.  Its results are meaningless; what it
// is for is GOL_OPT_SCHED_TRACE: the step schedule the runtime enqueues is
// recorded exactly as on the GPU and tests/test_sched_cpu.py checks it for
// races with tests/sched_race.py in the CPU suite.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "../../mpi_amd/csrc/gol_internal.h"

namespace {
struct Handle {
    int kind;
};
hipStream_t new_stream() { return reinterpret_cast<hipStream_t>(new Handle{1}); }
hipEvent_t new_event() { return reinterpret_cast<hipEvent_t>(new Handle{2}); }
}  // namespace

extern "C" {
hipError_t hipGetDeviceCount(int *n) { *n = 1; return hipSuccess; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetLastError() { return hipSuccess; }
const char *hipGetErrorString(hipError_t) { return "fake hip"; }
hipError_t hipDeviceEnablePeerAccess(int, unsigned) { return hipSuccess; }
hipError_t hipDeviceGetStreamPriorityRange(int *lo, int *hi) { *lo = 0; *hi = -1; return hipSuccess; }
hipError_t hipDeviceSynchronize() { return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n) { *p = calloc(1, n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void *p) { free(p); return hipSuccess; }
hipError_t hipHostMalloc(void **p, size_t n, unsigned) { return hipMalloc(p, n); }
hipError_t hipHostFree(void *p) { free(p); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned) { *d = h; return hipSuccess; }
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { memmove(d, s, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind, hipStream_t) {
    memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpy2DAsync(void *d, size_t dp, const void *s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                            hipStream_t) {
    for (size_t r = 0; r < h; ++r) memmove((char *)d + r * dp, (const char *)s + r * sp, w);
    return hipSuccess;
}
hipError_t hipMemset(void *d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
hipError_t hipMemset2DAsync(void *d, size_t p, int v, size_t w, size_t h, hipStream_t) {
    for (size_t r = 0; r < h; ++r) memset((char *)d + r * p, v, w);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = new_stream(); return hipSuccess; }
hipError_t hipStreamCreateWithPriority(hipStream_t *s, unsigned, int) { *s = new_stream(); return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t s) { delete reinterpret_cast<Handle *>(s); return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t *e) { *e = new_event(); return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = new_event(); return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t e) { delete reinterpret_cast<Handle *>(e); return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float *ms, hipEvent_t, hipEvent_t) { *ms = 1.0f; return hipSuccess; }
}

namespace gol {
int bit_group_words(int K) { return K >= 8 ? 4 : 2; }   // as gol_kernels.hip
bool bytebit_supported(int gens) { return (gens >= 4 && gens <= 32 && gens % 4 == 0) || gens == 48 || gens == 64; }
bool bytebit_chain_default(int gens) { return gens >= 48; }
bool bit_depth_supported(int gens) { return (gens >= 1 && gens <= 8) || gens == 16 || gens == 32; }
hipError_t launch_bit_pipe(const StencilArgs &, int, hipStream_t) { return hipSuccess; }
hipError_t launch_byte_pipe(const StencilArgs &, int, hipStream_t) { return hipSuccess; }
hipError_t launch_bytebit_pipe(const StencilArgs &, int, hipStream_t, int) { return hipSuccess; }
hipError_t launch_init_units(const InitUnit *, int, const uint32_t *, int, int, void *, int64_t, int, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_interleave_rows(const uint32_t *, uint32_t *, int64_t, int64_t, int64_t, int64_t, int,
                                  hipStream_t) {
    return hipSuccess;
}
hipError_t launch_pack_window(const uint8_t *, int64_t, uint32_t *, int64_t, int64_t, int64_t, int64_t, int64_t,
                              int64_t, int, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_unpack_window(const uint32_t *, int64_t, uint8_t *, int64_t, int64_t, int64_t, int64_t, int64_t,
                                int, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_format_text(const void *, int64_t, int, int64_t, int64_t, int64_t, int64_t, int, int64_t, char *,
                              hipStream_t) {
    return hipSuccess;
}
hipError_t launch_parse_text(const char *, int64_t, int64_t, uint8_t *, int64_t, int64_t, unsigned long long *,
                             hipStream_t) {
    return hipSuccess;
}
hipError_t launch_normalize_bytes(uint8_t *, int64_t, int64_t, int64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_clock_probe(unsigned long long *, const int *, unsigned long long, hipStream_t) {
    return hipErrorNotSupported;
}
hipError_t launch_popcount(const void *, int64_t, int64_t, int64_t, int64_t, unsigned long long *, int, hipStream_t) {
    return hipSuccess;
}
}  // namespace gol
