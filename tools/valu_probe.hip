// valu_probe — measured VALU issue ceilings on this GPU for the instruction mix
// of the bit-packed stencil (v_bitop3_b32, v_alignbit_b32, DPP row moves).
// Tool, not product:  hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// NC independent chains of 3-input ops: ILP = NC per wave.
template <int NC>
__global__ __launch_bounds__(256) void bitop3_kernel(unsigned *out, int iters, unsigned seed) {
    unsigned x[NC], y = threadIdx.x * 2654435761u + seed, z = y ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = y + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = __builtin_amdgcn_bitop3_b32(x[c], y, z, 0x96);
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = __builtin_amdgcn_bitop3_b32(x[c], z, y, 0xE8);
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) r ^= x[c];
    if (r == 0x12345678u) out[0] = r;
}

// the stencil's per-word pattern: 2 DPP + 2 alignbit + 10 bitop3, NC independent words
template <int NC>
__device__ __forceinline__ void mix_kernel_body(unsigned *out, int iters, unsigned seed) {
    unsigned w[NC], a0[NC], a1[NC], b0[NC], b1[NC];
    const unsigned m = 0xffffffffu;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        w[c] = threadIdx.x * 2654435761u + seed + c;
        a0[c] = w[c] * 3; a1[c] = w[c] * 5; b0[c] = w[c] * 7; b1[c] = w[c] * 11;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const unsigned l = __builtin_amdgcn_update_dpp(0u, w[c], 0x138, 0xf, 0xf, true);
            const unsigned r = __builtin_amdgcn_update_dpp(0u, w[c], 0x130, 0xf, 0xf, true);
            const unsigned L = __builtin_amdgcn_alignbit(w[c], l, 31), R = __builtin_amdgcn_alignbit(r, w[c], 1);
            const unsigned h0 = __builtin_amdgcn_bitop3_b32(L, w[c], R, 0x96);
            const unsigned h1 = __builtin_amdgcn_bitop3_b32(L, w[c], R, 0xE8);
            const unsigned o = __builtin_amdgcn_bitop3_b32(a0[c], b0[c], h0, 0x96);
            const unsigned co = __builtin_amdgcn_bitop3_b32(a0[c], b0[c], h0, 0xE8);
            const unsigned p = __builtin_amdgcn_bitop3_b32(a1[c], b1[c], h1, 0x96);
            const unsigned q = __builtin_amdgcn_bitop3_b32(a1[c], b1[c], h1, 0xE8);
            const unsigned u = __builtin_amdgcn_bitop3_b32(co, p, m, 0x28);
            const unsigned s = __builtin_amdgcn_bitop3_b32(q, co, p, 0x78);
            const unsigned M = __builtin_amdgcn_bitop3_b32(u, o, s, 0x42);
            const unsigned nx = __builtin_amdgcn_bitop3_b32(M, u, b0[c], 0xE0);
            a0[c] = b0[c]; a1[c] = b1[c]; b0[c] = h0; b1[c] = h1; w[c] = nx;
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) r ^= w[c];
    if (r == 0x12345678u) out[0] = r;
}
template <int NC>
__global__ __launch_bounds__(256) void mix_kernel(unsigned *out, int iters, unsigned seed) {
    mix_kernel_body<NC>(out, iters, seed);
}


// single-op throughput probes, ILP 4, 4 ops per chain per iteration
#define PROBE(NAME, EXPR)                                                                        \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, int iters, unsigned seed) {       \
        unsigned x0 = threadIdx.x + seed, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7;                  \
        unsigned y = x0 * 2654435761u, z = y ^ 0x9e3779b9u;                                       \
        const unsigned s = __builtin_amdgcn_readfirstlane(seed * 77u);                           \
        float f0 = x0, f1 = x1, f2 = x2, f3 = x3, fy = y, fz = z;                                 \
        (void)s; (void)f0; (void)f1; (void)f2; (void)f3; (void)fy; (void)fz;                      \
        for (int i = 0; i < iters; ++i) {                                                         \
            _Pragma("unroll") for (int r = 0; r < 4; ++r) { EXPR(x0, f0); EXPR(x1, f1); EXPR(x2, f2); EXPR(x3, f3); } \
        }                                                                                         \
        if ((x0 ^ x1 ^ x2 ^ x3 ^ (unsigned)(f0 + f1 + f2 + f3)) == 0x12345678u) out[0] = 1;       \
    }
#define E_XOR2(x, f) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y))
#define E_BITOP3V(x, f) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z))
#define E_BITOP3S(x, f) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "s"(s))
#define E_ADD3(x, f) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define E_ALIGN(x, f) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(x) : "v"(y))
#define E_DPP(x, f) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x))
#define E_FMA(x, f) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "v"(fy), "v"(fz))
#define E_LSHR(x, f) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(x))
#define E_LSHLOR(x, f) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(x) : "v"(y))
#define E_CND(x, f) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y))
#define E_ADDC(x, f) asm volatile("v_addc_co_u32_e64 %0, s[40:41], %0, %0, s[42:43]" : "+v"(x) : : "s40", "s41")
#define E_ADDC32(x, f) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(x) : : "vcc")
#define E_CMP(x, f) asm volatile("v_cmp_gt_i32_e64 s[40:41], 0, %0" : : "v"(x) : "s40", "s41")
#define E_PERM(x, f) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define E_SHR64(x, f) asm volatile("v_lshrrev_b64 v[60:61], 1, v[60:61]" : : : "v60", "v61")
#define E_BFI(x, f) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
// lane-crossing variants (round 2): DPP row vs wave shifts, DPP on VOP2 ALU ops,
// alignbit with a VGPR shift amount, and two whole funnel-shift sequences
// (x = x<<1 | prev lane's x>>31): DPP mov + alignbit vs lshr + lshl + add_dpp
#define E_DPPROW(x, f) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x))
#define E_ORDPP(x, f) asm volatile("v_or_b32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x) : "v"(y))
#define E_ADDDPP(x, f) asm volatile("v_add_u32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x) : "v"(y))
#define E_ADDDPPROW(x, f) asm volatile("v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x) : "v"(y))
#define E_ALIGNV(x, f) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z))
#define E_LSHL(x, f) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x))
#define E_LSHLV(x, f) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(y))
#define E_FUN_OLD(x, f) { unsigned t_; asm volatile("v_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\tv_alignbit_b32 %0, %0, %1, 31" : "+v"(x), "=&v"(t_)); }
#define E_FUN_NEW(x, f) { unsigned u_, t_; asm volatile("v_lshrrev_b32 %1, 31, %0\n\tv_lshlrev_b32 %2, 1, %0\n\ts_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x), "=&v"(u_), "=&v"(t_)); }
PROBE(p_dpprow, E_DPPROW)
PROBE(p_ordpp, E_ORDPP)
PROBE(p_adddpp, E_ADDDPP)
PROBE(p_adddpprow, E_ADDDPPROW)
PROBE(p_alignv, E_ALIGNV)
PROBE(p_lshl, E_LSHL)
PROBE(p_lshlv, E_LSHLV)
PROBE(p_fun_old, E_FUN_OLD)
PROBE(p_fun_new, E_FUN_NEW)
PROBE(p_xor2, E_XOR2)
PROBE(p_lshr, E_LSHR)
PROBE(p_lshlor, E_LSHLOR)
PROBE(p_cnd, E_CND)
PROBE(p_addc, E_ADDC)
PROBE(p_addc32, E_ADDC32)
PROBE(p_cmp, E_CMP)
PROBE(p_perm, E_PERM)
PROBE(p_shr64, E_SHR64)
PROBE(p_bfi, E_BFI)
PROBE(p_bitop3v, E_BITOP3V)
PROBE(p_bitop3s, E_BITOP3S)
PROBE(p_add3, E_ADD3)
PROBE(p_align, E_ALIGN)
PROBE(p_dppxor, E_DPP)
PROBE(p_fma, E_FMA)

// extern LDS only limits how many blocks share a CU (occupancy control)
template <int NC>
__global__ __launch_bounds__(256) void mix_occ_kernel(unsigned *out, int iters, unsigned seed) {
    extern __shared__ unsigned lds_pad[];
    if (seed == 0xdeadbeefu) lds_pad[threadIdx.x] = 0;
    mix_kernel_body<NC>(out, iters, seed);
}

template <typename F>
static double run(F kern, int blocks, int iters, double ops_per_iter, const char *name, size_t lds = 0) {
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    if (lds) (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, d, iters, 1u);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) {
        printf("{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", name);
        return 0;
    }
    (void)hipEventRecord(a, 0);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, d, iters, 1u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double lane_ops = 5.0 * blocks * 256.0 * iters * ops_per_iter;
    const double rate = lane_ops / (ms * 1e-3);
    const double peak = 256.0 * 4 * 32 * 2.4e9;
    printf("{\"probe\": \"%s\", \"blocks\": %d, \"Tlane_ops\": %.2f, \"frac_of_2.4GHz_peak\": %.3f}\n", name, blocks,
           rate / 1e12, rate / peak);
    (void)hipFree(d);
    return rate;
}

int main() {
    const int iters = 4096;
    for (int blocks : {8192}) {
        run(p_xor2, blocks, iters / 4, 16, "v_xor_b32 ilp4");
        run(p_bitop3v, blocks, iters / 4, 16, "v_bitop3 3xVGPR ilp4");
        run(p_bitop3s, blocks, iters / 4, 16, "v_bitop3 2xVGPR+SGPR ilp4");
        run(p_add3, blocks, iters / 4, 16, "v_add3_u32 ilp4");
        run(p_align, blocks, iters / 4, 16, "v_alignbit ilp4");
        run(p_dppxor, blocks, iters / 4, 16, "v_mov_b32_dpp wave_shr ilp4");
        run(p_fma, blocks, iters / 4, 16, "v_fma_f32 ilp4");
        run(p_lshr, blocks, iters / 4, 16, "v_lshrrev_b32 ilp4");
        run(p_lshlor, blocks, iters / 4, 16, "v_lshl_or_b32 ilp4");
        run(p_cnd, blocks, iters / 4, 16, "v_cndmask_b32 vcc ilp4");
        run(p_addc, blocks, iters / 4, 16, "v_addc_co_u32_e64 sgpr carry ilp4");
        run(p_addc32, blocks, iters / 4, 16, "v_addc_co_u32 vcc ilp4");
        run(p_cmp, blocks, iters / 4, 16, "v_cmp_gt_i32_e64 ilp4");
        run(p_perm, blocks, iters / 4, 16, "v_perm_b32 ilp4");
        run(p_shr64, blocks, iters / 4, 16, "v_lshrrev_b64 ilp1");
        run(p_bfi, blocks, iters / 4, 16, "v_bfi_b32 ilp4");
    }
    if (getenv("PROBE_CROSS")) {
        for (int rep = 0; rep < 2; ++rep) {
            run(p_xor2, 8192, iters / 4, 16, "v_xor_b32 ilp4");
            run(p_bitop3v, 8192, iters / 4, 16, "v_bitop3 3xVGPR ilp4");
            run(p_dppxor, 8192, iters / 4, 16, "v_mov_b32_dpp wave_shr ilp4");
            run(p_dpprow, 8192, iters / 4, 16, "v_mov_b32_dpp row_shr ilp4");
            run(p_ordpp, 8192, iters / 4, 16, "v_or_b32_dpp wave_shr ilp4");
            run(p_adddpp, 8192, iters / 4, 16, "v_add_u32_dpp wave_shr ilp4");
            run(p_adddpprow, 8192, iters / 4, 16, "v_add_u32_dpp row_shr ilp4");
            run(p_align, 8192, iters / 4, 16, "v_alignbit const ilp4");
            run(p_alignv, 8192, iters / 4, 16, "v_alignbit 3xVGPR ilp4");
            run(p_lshl, 8192, iters / 4, 16, "v_lshlrev_b32 const ilp4");
            run(p_lshlv, 8192, iters / 4, 16, "v_lshlrev_b32 vgpr ilp4");
            run(p_fun_old, 8192, iters / 4, 16, "funnel dpp_mov+alignbit (funnels/s) ilp4");
            run(p_fun_new, 8192, iters / 4, 16, "funnel lshr+lshl+add_dpp (funnels/s) ilp4");
        }
        return 0;
    }
    if (getenv("PROBE_QUICK")) return 0;
    for (int blocks : {2048, 8192}) {
        run(bitop3_kernel<1>, blocks, iters, 2 * 1, "bitop3 ilp1");
        run(bitop3_kernel<2>, blocks, iters, 2 * 2, "bitop3 ilp2");
        run(bitop3_kernel<4>, blocks, iters, 2 * 4, "bitop3 ilp4");
        run(bitop3_kernel<8>, blocks, iters, 2 * 8, "bitop3 ilp8");
        run(mix_kernel<1>, blocks, iters / 4, 14 * 1, "stencil-mix ilp1");
        run(mix_kernel<2>, blocks, iters / 4, 14 * 2, "stencil-mix ilp2");
        run(mix_kernel<4>, blocks, iters / 4, 14 * 4, "stencil-mix ilp4");
    }
    // the same mix at a fixed number of resident waves per SIMD (LDS-limited blocks per CU)
    {
        char nm[64];
        const size_t lds_for[5] = {0, 100 << 10, 60 << 10, 45 << 10, 36 << 10};
        for (int w = 1; w <= 4; ++w) {
            snprintf(nm, sizeof nm, "stencil-mix ilp4 %d waves/SIMD", w);
            run(mix_occ_kernel<4>, 256 * w * 4, iters / 4, 14 * 4, nm, lds_for[w]);
            snprintf(nm, sizeof nm, "stencil-mix ilp8 %d waves/SIMD", w);
            run(mix_occ_kernel<8>, 256 * w * 4, iters / 4, 14 * 8, nm, lds_for[w]);
        }
    }
    return 0;
}
