// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Drives the reference's OWN serial functions, compiled from where they lie
// (/root/reference/main_serial.cpp, passed in as REF_SERIAL by oracle/Makefile):
//   initializeBoard main_serial.cpp:34-43  (srand(seed); padded [0,n-1]² ← rand()%3==0)
//   updateBoard     main_serial.cpp:45-71  (scatter-count with %rows wrap, in-place rule)
// The set-up mirrors main_serial.cpp:136-169: one (n+2)² byte block behind row
// pointers and seed = rand() taken before any srand (glibc default ⇒ 1804289383).
// The block is calloc'ed (the reference mallocs it; fresh pages are zero — SURVEY §8c).
// Dumps the n×n board that writeBoardToFile (main_serial.cpp:74-94) would print
// (padded rows/cols 1..n) as np.packbits bytes: <prefix>_g<gen>.bin.
//
// usage: ref_harness_serial n gens dump_every prefix
#define main gol_serial_reference_main
#include REF_SERIAL
#undef main

#include <cstdio>
#include <cstdlib>
#include <cstring>

static void dump(bool **board, int n, int gen, const char *prefix) {
    std::vector<unsigned char> packed(((size_t)n * n + 7) / 8, 0);
    size_t k = 0;
    for (int i = 1; i <= n; i++)
        for (int j = 1; j <= n; j++, k++)
            if (board[i][j]) packed[k >> 3] |= (unsigned char)(0x80u >> (k & 7));
    char path[1024];
    snprintf(path, sizeof path, "%s_g%d.bin", prefix, gen);
    FILE *f = fopen(path, "wb");
    fwrite(packed.data(), 1, packed.size(), f);
    fclose(f);
}

int main(int argc, char *argv[]) {
    if (argc != 5) {
        fprintf(stderr, "usage: ref_harness_serial n gens dump_every prefix\n");
        return 1;
    }
    int n = atoi(argv[1]), gens = atoi(argv[2]), every = atoi(argv[3]);
    const char *prefix = argv[4];
    bool **board = (bool **)malloc((n + 2) * sizeof(bool *));
    board[0] = (bool *)calloc((size_t)(n + 2) * (n + 2), 1);
    for (int i = 1; i < n + 2; i++) board[i] = board[i - 1] + n + 2;
    int seed = rand();                                 // main_serial.cpp:150
    distrOpt options = {n, n, 1, 1, gens, every, seed, 0, n, n};
    initializeBoard(board, options);
    dump(board, n, 0, prefix);
    for (int i = 1; i <= gens; ++i) {                  // main_serial.cpp:172-178
        updateBoard(board, options);
        if (every > 0 && i % every == 0) dump(board, n, i, prefix);
    }
    return 0;
}
