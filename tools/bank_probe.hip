// VGPR operand-bank probe for gfx950 (diagnostic, not part of the library):
// does a 3-VGPR v_bitop3_b32 issue slower when its operands share a bank
// (register index mod 4)?  Explicit registers in inline asm, 4 independent
// chains, full occupancy.   hipcc --offload-arch=gfx950 -O3 -o bank_probe bank_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP4(s) s s s s
#define K(NAME, BODY, CLOB)                                                                  \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, int iters) {                  \
        for (int i = 0; i < iters; ++i) asm volatile(REP4(BODY) ::: CLOB);                  \
        if (iters < 0) out[0] = 1;                                                           \
    }
#define CL "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
// all operands in bank 0
K(b3_same, "v_bitop3_b32 v40, v40, v44, v48 bitop3:0x96\n v_bitop3_b32 v52, v52, v44, v48 bitop3:0x96\n"
           "v_bitop3_b32 v56, v56, v44, v48 bitop3:0x96\n v_bitop3_b32 v60, v60, v44, v48 bitop3:0x96\n", CL)
// operands of one instruction in three different banks, same banks in every chain
K(b3_dist, "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v44, v44, v41, v42 bitop3:0x96\n"
           "v_bitop3_b32 v48, v48, v41, v42 bitop3:0x96\n v_bitop3_b32 v52, v52, v41, v42 bitop3:0x96\n", CL)
// different banks within and across consecutive instructions
K(b3_rot, "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v45, v45, v46, v47 bitop3:0x96\n"
          "v_bitop3_b32 v50, v50, v51, v48 bitop3:0x96\n v_bitop3_b32 v55, v55, v52, v53 bitop3:0x96\n", CL)
// two of three operands in one bank
K(b3_two, "v_bitop3_b32 v40, v40, v44, v42 bitop3:0x96\n v_bitop3_b32 v48, v48, v52, v42 bitop3:0x96\n"
          "v_bitop3_b32 v56, v56, v60, v42 bitop3:0x96\n v_bitop3_b32 v41, v41, v45, v43 bitop3:0x96\n", CL)
K(x2_same, "v_xor_b32 v40, v40, v44\n v_xor_b32 v48, v48, v44\n v_xor_b32 v52, v52, v44\n v_xor_b32 v56, v56, v44\n", CL)
K(x2_dist, "v_xor_b32 v40, v40, v41\n v_xor_b32 v44, v44, v41\n v_xor_b32 v48, v48, v41\n v_xor_b32 v52, v52, v41\n", CL)
K(x2_rot, "v_xor_b32 v40, v40, v41\n v_xor_b32 v45, v45, v46\n v_xor_b32 v50, v50, v51\n v_xor_b32 v55, v55, v52\n", CL)
K(lshr1, "v_lshrrev_b32 v40, 1, v40\n v_lshrrev_b32 v44, 1, v44\n v_lshrrev_b32 v48, 1, v48\n v_lshrrev_b32 v52, 1, v52\n", CL)
K(lshr_rot, "v_lshrrev_b32 v40, 1, v40\n v_lshrrev_b32 v45, 1, v45\n v_lshrrev_b32 v50, 1, v50\n v_lshrrev_b32 v55, 1, v55\n", CL)
// 8 independent chains, rotated banks
K(b3_rot8, "v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v45, v45, v46, v47 bitop3:0x96\n"
           "v_bitop3_b32 v50, v50, v51, v48 bitop3:0x96\n v_bitop3_b32 v55, v55, v52, v53 bitop3:0x96\n"
           "v_bitop3_b32 v56, v56, v57, v58 bitop3:0x96\n v_bitop3_b32 v61, v61, v62, v63 bitop3:0x96\n"
           "v_bitop3_b32 v54, v54, v43, v44 bitop3:0x96\n v_bitop3_b32 v59, v59, v60, v49 bitop3:0x96\n", CL)

template <typename F>
static void run(F kern, int blocks, int iters, double ops_per_iter, const char *name) {
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double rate = 5.0 * blocks * 256.0 * iters * ops_per_iter / (ms * 1e-3);
    printf("{\"probe\": \"%s\", \"blocks\": %d, \"Tlane_ops\": %.2f}\n", name, blocks, rate / 1e12);
    (void)hipFree(d);
}

int main() {
    for (int blocks : {8192, 512, 256}) {   // 8 (several rounds), 2, 1 waves per SIMD
        const int it = 20000;
        run(b3_same, blocks, it, 16, "bitop3 all operands bank 0");
        run(b3_dist, blocks, it, 16, "bitop3 operands banks 0,1,2");
        run(b3_rot, blocks, it, 16, "bitop3 banks rotated per instruction");
        run(b3_two, blocks, it, 16, "bitop3 two operands in one bank");
        run(b3_rot8, blocks, it, 32, "bitop3 rotated, 8 chains");
        run(x2_same, blocks, it, 16, "xor2 same bank");
        run(x2_dist, blocks, it, 16, "xor2 banks 0,1");
        run(x2_rot, blocks, it, 16, "xor2 rotated");
        run(lshr1, blocks, it, 16, "lshr bank 0");
        run(lshr_rot, blocks, it, 16, "lshr rotated");
    }
    return 0;
}
