#include "glibc_jump.h"

#include <string.h>

namespace gol {

void glibc_seed_window(uint32_t seed, uint32_t w[31]) {
    // __srandom_r: state[0] = seed (0 -> 1); state[i] = 16807·state[i-1] mod (2^31-1)
    // via Schrage; fptr = &state[3], rptr = &state[0]; then 310 discarded draws.
    int32_t s[31];
    if (seed == 0) seed = 1;
    s[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        s[i] = word;
    }
    int f = 3, r = 0;
    for (int k = 0; k < 310 + 31; ++k) {
        const uint32_t v = (uint32_t)s[f] + (uint32_t)s[r];
        s[f] = (int32_t)v;
        if (k >= 310) w[k - 310] = v;
        f = (f + 1) % 31;
        r = (r + 1) % 31;
    }
}

Mat31 JumpTable::identity() {
    Mat31 m;
    memset(m.a, 0, sizeof m.a);
    for (int i = 0; i < 31; ++i) m.a[i * 31 + i] = 1;
    return m;
}

Mat31 JumpTable::mat_mul(const Mat31 &x, const Mat31 &y) {
    Mat31 z;
    for (int i = 0; i < 31; ++i)
        for (int j = 0; j < 31; ++j) {
            uint32_t acc = 0;
            for (int k = 0; k < 31; ++k) acc += x.a[i * 31 + k] * y.a[k * 31 + j];
            z.a[i * 31 + j] = acc;
        }
    return z;
}

void JumpTable::mat_vec(const Mat31 &m, const uint32_t in[31], uint32_t out[31]) {
    uint32_t t[31];
    for (int i = 0; i < 31; ++i) {
        uint32_t acc = 0;
        for (int k = 0; k < 31; ++k) acc += m.a[i * 31 + k] * in[k];
        t[i] = acc;
    }
    memcpy(out, t, sizeof t);
}

JumpTable::JumpTable() : pow2_(64) {
    // companion matrix: W'[i] = W[i+1] (i < 30), W'[30] = W[28] + W[0]
    Mat31 a;
    memset(a.a, 0, sizeof a.a);
    for (int i = 0; i < 30; ++i) a.a[i * 31 + i + 1] = 1;
    a.a[30 * 31 + 28] = 1;
    a.a[30 * 31 + 0] = 1;
    pow2_[0] = a;
    for (int b = 1; b < 64; ++b) pow2_[b] = mat_mul(pow2_[b - 1], pow2_[b - 1]);
}

void JumpTable::jump(uint64_t n, uint32_t w[31]) const {
    for (int b = 0; n; ++b, n >>= 1)
        if (n & 1) mat_vec(pow2_[b], w, w);
}

Mat31 JumpTable::power(uint64_t n) const {
    Mat31 r = identity();
    for (int b = 0; n; ++b, n >>= 1)
        if (n & 1) r = mat_mul(r, pow2_[b]);
    return r;
}

} // namespace gol
