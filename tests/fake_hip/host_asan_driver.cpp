// Host-code sanitizer run (test infrastructure): the runtime's host code over the
// host-only HIP stand-in, built with -fsanitize=address,undefined into this
// executable, driven through the C ABI — contexts of 1-4 slabs, the split interior
// toggled, uneven steps, async and sync windows, snapshot text, options, the
// schedule trace, destroy.  Any heap / UB error aborts with a report.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../include/golhip.h"

static void chk(int rc, gol_ctx *c, const char *what) {
    if (rc) {
        fprintf(stderr, "%s failed: %d %s\n", what, rc, c ? gol_last_error(c) : "");
        exit(1);
    }
}

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 200;
    std::mt19937 rng(12345);
    auto rnd = [&](int lo, int hi) { return lo + (int)(rng() % (unsigned)(hi - lo + 1)); };
    for (int i = 0; i < cases; ++i) {
        const int slabs = rnd(1, 4), layout = rnd(0, 2) ? GOL_LAYOUT_BIT : GOL_LAYOUT_BYTE;
        const int ks_bit[] = {1, 3, 5, 8, 8}, ks_byte[] = {1, 8, 28, 32};
        const int k = layout == GOL_LAYOUT_BIT ? ks_bit[rnd(0, 4)] : ks_byte[rnd(0, 3)];
        const int64_t rows = (int64_t)slabs * rnd(2 * k + 2, 700), cols = rnd(2, 3000);
        gol_ctx *c = nullptr;
        chk(gol_create(&c, rows, cols, slabs, layout, GOL_DEAD, 1, k), nullptr, "gol_create");
        std::vector<uint8_t> board((size_t)(rows * cols));
        for (auto &b : board) b = (uint8_t)(rng() % 3 == 0);
        chk(gol_upload(c, board.data(), cols), c, "upload");
        chk(gol_set_option(c, GOL_OPT_INTERIOR_SPLIT, rnd(1, 4)), c, "split");
        chk(gol_set_option(c, GOL_OPT_SCHED_TRACE, 1), c, "trace");
        if (rnd(0, 3) == 0) chk(gol_set_option(c, GOL_OPT_CHUNK_ROWS, rnd(0, 1) ? 64 : -3), c, "chunk");
        if (rnd(0, 4) == 0) chk(gol_set_option(c, GOL_OPT_OVERLAP, 0), c, "overlap");
        std::vector<std::vector<uint8_t>> wins;
        const int nsteps = rnd(2, 30);
        for (int s = 0; s < nsteps; ++s) {
            chk(gol_step(c, rnd(1, k)), c, "step");
            if (rnd(0, 5) == 0) {
                const int64_t r0 = rnd(0, (int)rows - 1), c0 = rnd(0, (int)cols - 1);
                const int64_t h = rnd(1, (int)(rows - r0)), w = rnd(1, (int)(cols - c0));
                wins.emplace_back((size_t)(h * w));
                chk(gol_download_window_async(c, r0, c0, h, w, wins.back().data(), w), c, "window_async");
            }
            if (rnd(0, 9) == 0) chk(gol_set_option(c, GOL_OPT_INTERIOR_SPLIT, rnd(1, 4)), c, "split toggle");
        }
        double ms = 0;
        chk(gol_sync(c, &ms), c, "sync");
        int64_t n = 0;
        chk(gol_sched_trace(c, nullptr, 0, &n), c, "trace n");
        std::vector<int64_t> ops((size_t)n * 7 + 1);
        chk(gol_sched_trace(c, ops.data(), n, &n), c, "trace copy");
        chk(gol_download(c, board.data(), cols), c, "download");
        const int64_t tr = rnd(1, (int)rows), tc = rnd(1, (int)std::min<int64_t>(cols, 200));
        std::vector<char> text((size_t)gol_text_bytes(tr, tc));
        chk(gol_format_text(c, 0, 0, tr, tc, text.data(), (int64_t)text.size()), c, "format_text");
        int64_t live = 0;
        chk(gol_popcount(c, &live), c, "popcount");
        gol_destroy(c);
    }
    printf("host asan driver: %d contexts ok\n", cases);
    return 0;
}
