// Host-code ThreadSanitizer run (test infrastructure): rank contexts of one RCCL
// world created, stepped (split interior, short blocks) and destroyed from
// threads at once, over the host-only HIP stand-in and the in-process RCCL
// stand-in (tests/shim/fake_rccl.cpp, linked in: -rdynamic puts its nccl*
// symbols in the global scope where the runtime looks first).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <thread>
#include <vector>
#include "../../include/golhip.h"
int main() {
    for (int it = 0; it < 20; ++it) {
        const int world = 2 + it % 3, k = it % 2 ? 8 : 5;
        const int64_t rows = (int64_t)world * 600, cols = 1000;
        uint8_t uid[GOL_UNIQUE_ID_BYTES];
        if (gol_get_unique_id(uid)) { fprintf(stderr, "uid\n"); return 1; }
        std::vector<std::thread> ts;
        std::vector<int> rcs(world, 0);
        for (int r = 0; r < world; ++r)
            ts.emplace_back([&, r] {
                gol_ctx *c = nullptr;
                int rc = gol_create_rank(&c, rows, cols, r, world, 0, uid, GOL_LAYOUT_BIT, GOL_DEAD, 1, k);
                if (!rc) rc = gol_set_option(c, GOL_OPT_INTERIOR_SPLIT, 2);
                for (int s = 0; s < 30 && !rc; ++s) rc = gol_step(c, s % 7 == 3 ? 2 : k);
                if (!rc) rc = gol_sync(c, nullptr);
                if (c) gol_destroy(c);
                rcs[r] = rc;
            });
        for (auto &t : ts) t.join();
        for (int r = 0; r < world; ++r) if (rcs[r]) { fprintf(stderr, "rank %d rc %d\n", r, rcs[r]); return 1; }
    }
    printf("tsan driver ok\n");
    return 0;
}
