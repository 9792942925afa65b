// glibc TYPE_3 rand() restated for the device initialiser, with jump-ahead.
//
// glibc 2.35 random_r.c (__srandom_r, __random_r), the third-party algorithm
// behind the reference's initializeBoard (main.cpp:68-77, main_serial.cpp:34-43):
// a lagged additive generator over Z/2^32 whose written values obey
//     x_t = x_{t-3} + x_{t-31}            (mod 2^32),   rand() = x >> 1.
// A 31-value window W_t = (x_t .. x_{t+30}) advances by the companion matrix A
// (W_{t+1} = A W_t), so any draw offset is reached with ⌈log2 n⌉ mat-vecs.
#pragma once
#include <stdint.h>
#include <vector>

namespace gol {

struct Mat31 {
    uint32_t a[31 * 31];
};

// Window of raw values behind rand_0 .. rand_30 after srand(seed).
void glibc_seed_window(uint32_t seed, uint32_t w[31]);

class JumpTable {
  public:
    JumpTable();
    // w <- A^n w
    void jump(uint64_t n, uint32_t w[31]) const;
    // A^n as a matrix
    Mat31 power(uint64_t n) const;
    static void mat_vec(const Mat31 &m, const uint32_t in[31], uint32_t out[31]);
    static Mat31 mat_mul(const Mat31 &x, const Mat31 &y);
    static Mat31 identity();

  private:
    std::vector<Mat31> pow2_;   // A^(2^b), b = 0..63
};

} // namespace gol
