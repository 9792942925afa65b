// Exhaustive search for the per-output rule circuit of a row-PAIR adder
// structure: the 9-sum of output row x is H(x-1) + P, where P = H(x) + H(x+1)
// is computed once per pair of rows and shared by the two output rows whose
// windows contain the pair.  Inputs per output: the pair code (p0, e0, e1)
// = binary P (0..6), the single row's horizontal sum (a0, a1), alive.
// Question: how many 3-input gates (v_bitop3) does the rule need?
//   gcc -O3 -march=native -o /tmp/ps tools/pair_search.c && /tmp/ps
#include <stdio.h>
#include <stdint.h>

#define NV 6
static uint64_t F, CARE;

static inline uint64_t lut(int tt, uint64_t x, uint64_t y, uint64_t z) {
    uint64_t r = 0;
    for (int k = 0; k < 8; k++)
        if ((tt >> k) & 1) r |= ((k & 4) ? x : ~x) & ((k & 2) ? y : ~y) & ((k & 1) ? z : ~z);
    return r;
}

// is F (on CARE) a function of the signals in s[0..n)?  (n <= 5)
static inline int is_func(const uint64_t *s, int n) {
    for (int cell = 0; cell < (1 << n); cell++) {
        uint64_t m = CARE;
        for (int i = 0; i < n; i++) m &= ((cell >> i) & 1) ? s[i] : ~s[i];
        if (m && (m & F) != m && (m & F) != 0) return 0;
    }
    return 1;
}

// does a LUT exist with F == lut(x,y,z) on CARE?
static inline int fits3(uint64_t x, uint64_t y, uint64_t z) {
    uint64_t s[3] = {x, y, z};
    return is_func(s, 3);
}

int main(void) {
    uint64_t in[NV] = {0};
    F = CARE = 0;
    // vars: 0=p0 1=e0 2=e1 3=a0 4=a1 5=alive
    for (int r = 0; r < 64; r++) {
        for (int v = 0; v < NV; v++) if ((r >> v) & 1) in[v] |= 1ull << r;
        int P = (r & 1) + 2 * ((r >> 1) & 3);
        int A = ((r >> 3) & 1) + 2 * ((r >> 4) & 1);
        int al = (r >> 5) & 1;
        if (P > 6) continue;                 // code 7 unused
        if (al && P == 0) continue;          // alive => its row's H >= 1 => P >= 1
        if (!al && P == 6) continue;         // dead  => its row's H <= 2 => P <= 5
        int S = P + A;
        CARE |= 1ull << r;
        if (S == 3 || (al && S == 4)) F |= 1ull << r;
    }
    long n3 = 0, n4 = 0;
    uint64_t sig[NV + 3];
    for (int v = 0; v < NV; v++) sig[v] = in[v];
    // m = 3 and m = 4 in one sweep: g1, g2 enumerated; m=3: final gate over 3 of 8 signals;
    // m=4: F = g4(g3(u,v,w), y, z) -> first F must be a function of {u,v,w,y,z}, then a g3 LUT.
    #pragma omp parallel for collapse(2) schedule(dynamic) reduction(+:n3,n4) firstprivate(sig)
    for (int abc = 0; abc < 216; abc++)
    for (int t1 = 0; t1 < 256; t1++) {
        int a = abc / 36, b = (abc / 6) % 6, c = abc % 6;
        if (!(a < b && b < c)) continue;
        sig[NV] = lut(t1, sig[a], sig[b], sig[c]);
        for (int d = 0; d < NV + 1; d++) for (int e = d + 1; e < NV + 1; e++) for (int g = e + 1; g < NV + 1; g++)
        for (int t2 = 0; t2 < 256; t2++) {
            sig[NV + 1] = lut(t2, sig[d], sig[e], sig[g]);
            const int ns = NV + 2;
            for (int x = 0; x < ns; x++) for (int y = x + 1; y < ns; y++) for (int z = y + 1; z < ns; z++)
                if (fits3(sig[x], sig[y], sig[z])) {
                    if (++n3 <= 5) printf("m3: g1=%02x(%d,%d,%d) g2=%02x(%d,%d,%d) out(%d,%d,%d)\n", t1, a, b, c, t2, d, e, g, x, y, z);
                }
            if (n3) continue;
            // union of 4 signals: g3 over three of them, g4 over (g3, the fourth, one of the three)
            for (int i0 = 0; i0 < ns; i0++) for (int i1 = i0 + 1; i1 < ns; i1++) for (int i2 = i1 + 1; i2 < ns; i2++)
            for (int i3 = i2 + 1; i3 < ns; i3++) {
                uint64_t s4[4] = {sig[i0], sig[i1], sig[i2], sig[i3]};
                if (!is_func(s4, 4)) continue;
                for (int lo = 0; lo < 4; lo++) for (int sh = 0; sh < 4; sh++) if (sh != lo) {
                    uint64_t u[3]; int k = 0;
                    for (int j = 0; j < 4; j++) if (j != lo) u[k++] = s4[j];
                    for (int t3 = 0; t3 < 256; t3++)
                        if (fits3(lut(t3, u[0], u[1], u[2]), s4[lo], s4[sh])) {
                            if (++n4 <= 10) printf("m4(4): g1=%02x(%d,%d,%d) g2=%02x(%d,%d,%d) g3=%02x\n", t1, a, b, c, t2, d, e, g, t3);
                            break;
                        }
                }
            }
            // m = 4: choose 5 signals among 8 that determine F, split into (u,v,w) and (y,z)
            for (int i0 = 0; i0 < ns; i0++) for (int i1 = i0 + 1; i1 < ns; i1++) for (int i2 = i1 + 1; i2 < ns; i2++)
            for (int i3 = i2 + 1; i3 < ns; i3++) for (int i4 = i3 + 1; i4 < ns; i4++) {
                uint64_t s5[5] = {sig[i0], sig[i1], sig[i2], sig[i3], sig[i4]};
                if (!is_func(s5, 5)) continue;
                int id[5] = {i0, i1, i2, i3, i4};
                for (int p = 0; p < 5; p++) for (int q = p + 1; q < 5; q++) {   // (y,z) = (p,q)
                    uint64_t u[3]; int k = 0;
                    for (int j = 0; j < 5; j++) if (j != p && j != q) u[k++] = s5[j];
                    for (int t3 = 0; t3 < 256; t3++) {
                        uint64_t g3 = lut(t3, u[0], u[1], u[2]);
                        if (fits3(g3, s5[p], s5[q])) {
                            if (++n4 <= 10)
                                printf("m4: g1=%02x(%d,%d,%d) g2=%02x(%d,%d,%d) g3=%02x(%d,%d,%d of {%d,%d,%d,%d,%d}) out(g3,%d,%d)\n",
                                       t1, a, b, c, t2, d, e, g, t3, 0, 1, 2, id[0], id[1], id[2], id[3], id[4], id[p], id[q]);
                            goto next_split;
                        }
                    }
                next_split:;
                }
            }
        }
    }
    printf("m3 circuits: %ld, m4 circuits (tree-shaped final pair): %ld\n", n3, n4);
    return 0;
}
