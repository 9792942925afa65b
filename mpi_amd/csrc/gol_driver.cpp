// gol — reference-compatible driver for the MI355X engine.
//
//   gol [options] rows cols iteration_gap iterations [time_file] [first]
//
// Keeps the positional CLI of main.cpp:171-220 / main_serial.cpp:115-130, the
// `<timestamp>.gol` main file (main.cpp:131-147), the per-part snapshot files
// `<name>_<iter>_<part>.gol` (main.cpp:106-129) that gol_visualization.py
// stitches, and the `_detailed.out` / `_compact.csv` timing report
// (main.cpp:310-365; values in µs under the reference's "ms" labels).  All
// compute goes through the C ABI of include/golhip.h.
//
// Options
//   --mode mpi|serial|dead  mpi (default): main.cpp semantics on a √P×√P mesh of
//                           --procs P emulated ranks (P=1: dead boundary);
//                           serial: main_serial.cpp semantics (writes gen 0 and
//                           every gap, like the serial program);
//                           dead: textbook non-periodic B3/S23, any rows×cols.
//   --procs P               emulated MPI ranks for --mode mpi (default 1)
//   --gpus N                row slabs / GPUs (default 1)
//   --layout bit|byte       cell layout (default: bit; byte when --procs P has
//                           blocks of cols/√P not a multiple of 32 columns)
//   -k K                    generations fused per launch (default 1)
//   --save / --no-save      write snapshots every gap generations
//                           (default: on for serial, off for mpi/dead as in main.cpp:208)
//   --seed S                override the srand seed
//   --resume NAME --from I  continue the run of NAME.gol from its saved
//                           iteration I (part files NAME_I_<p>.gol, read back
//                           on the device); rows/cols/gap/iters default to the
//                           main file's; new snapshots continue under NAME
//   --rccl                  the N row slabs as N RCCL ranks of ONE process: one
//                           rank context (gol_create_rank) and one communicator
//                           per device, each driven by a host thread, halo rows
//                           through ncclSend/ncclRecv (the transport of the
//                           one-process-per-GPU path; the default --gpus N path
//                           keeps the slabs in one context with peer copies).
//                           Rank r runs on device r; RCCL refuses two ranks on
//                           one device, so on one GPU this needs --same-device
//                           with an in-process RCCL stand-in (--rccl-lib)
//   --rccl-lib PATH         bind this RCCL library instead of the system's
//                           (loaded into the global scope before any rank;
//                           tests: tests/shim/libfake_rccl.so)
//   --same-device           --rccl: every rank on device 0
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/golhip.h"

namespace {

void die(const char *msg) {
    printf("%s\n", msg);
    exit(1);
}

void check(gol_ctx *c, int rc, const char *what) {
    if (rc != GOL_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, c ? gol_last_error(c) : "");
        exit(1);
    }
}

// main.cpp:131-147 / main_serial.cpp:97-113
std::string set_up_program(long rows, long cols, int gap, int iters, int parts) {
    char buf[50];
    time_t raw;
    time(&raw);
    strftime(buf, sizeof buf, "%Y-%m-%d-%H-%M-%S", localtime(&raw));
    std::string name(buf);
    FILE *f = fopen((name + ".gol").c_str(), "w");
    if (!f) die("cannot create main .gol file");
    fprintf(f, "%ld %ld %d %d %d\n", rows, cols, gap, iters, parts);
    fclose(f);
    return name;
}

// main.cpp:106-129: two header lines, then rows of "v\t" tokens.  The body is
// formatted on the device and streamed to the file (gol_write_text).
void write_part(gol_ctx *ctx, const std::string &name, int iter, int part, long first_row, long last_row,
                long first_col, long last_col, int64_t row0, int64_t nrows, int64_t ncols) {
    std::string path = name + "_" + std::to_string(iter) + "_" + std::to_string(part) + ".gol";
    FILE *f = fopen(path.c_str(), "w");
    if (!f) die("cannot create part .gol file");
    fprintf(f, "%ld %ld\n%ld %ld\n", first_row, last_row, first_col, last_col);
    fflush(f);
    check(ctx, gol_write_text(ctx, row0, 0, nrows, ncols, fileno(f)), "gol_write_text");
    fclose(f);
}

// Snapshot resume: load part file `path` (either header convention: the origin
// is the first number of each header line, the shape comes from the body).
void read_part(gol_ctx *ctx, const std::string &path) {
    FILE *f = fopen(path.c_str(), "r");
    if (!f) die(("cannot open " + path).c_str());
    long r0 = 0, r_end = 0, c0 = 0, c_end = 0;
    if (fscanf(f, "%ld %ld\n%ld %ld", &r0, &r_end, &c0, &c_end) != 4 || fgetc(f) != '\n')
        die(("bad header in " + path).c_str());
    const long off = ftell(f);
    long rowlen = 0;
    for (int ch; (ch = fgetc(f)) != EOF;) {
        ++rowlen;
        if (ch == '\n') break;
    }
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fclose(f);
    if (rowlen < 3 || rowlen % 2 == 0 || (size - off) % rowlen != 0) die(("bad body in " + path).c_str());
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0 || lseek(fd, off, SEEK_SET) != off) die(("cannot open " + path).c_str());
    check(ctx, gol_read_text(ctx, r0, c0, (size - off) / rowlen, (rowlen - 1) / 2, fd), path.c_str());
    close(fd);
}

struct Opts {
    std::string mode = "mpi", layout = "";
    int procs = 1, gpus = 1, k = 1, save = -1;
    long long seed = -1;
    std::string resume;   // --resume NAME: continue the run whose main file is NAME.gol
    int from = -1;        // --from ITER: the saved iteration to continue from
    bool rccl = false, same_device = false;
    std::string rccl_lib;
};

// One rank of --rccl: its context and what it reports.
struct RankRun {
    gol_ctx *ctx = nullptr;
    double dev_ms = 0.0;
    int64_t live = 0, launches = 0;
    std::string err;
};

// Runs fn(r) for r = 0..n-1 on n host threads at once (the rank calls are
// collective: every rank must be inside gol_create_rank / gol_step together).
template <typename F>
void on_ranks(int n, F fn) {
    std::vector<std::thread> ts;
    for (int r = 0; r < n; ++r) ts.emplace_back([&, r] { fn(r); });
    for (auto &t : ts) t.join();
}

} // namespace

int main(int argc, char **argv) {
    auto t_begin = std::chrono::steady_clock::now();
    Opts o;
    std::vector<const char *> pos;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) die("missing option value");
            return argv[++i];
        };
        if (a == "--mode") o.mode = next();
        else if (a == "--procs") o.procs = atoi(next());
        else if (a == "--gpus") o.gpus = atoi(next());
        else if (a == "--layout") o.layout = next();
        else if (a == "-k") o.k = atoi(next());
        else if (a == "--save") o.save = 1;
        else if (a == "--no-save") o.save = 0;
        else if (a == "--seed") o.seed = atoll(next());
        else if (a == "--resume") o.resume = next();
        else if (a == "--from") o.from = atoi(next());
        else if (a == "--rccl") o.rccl = true;
        else if (a == "--rccl-lib") o.rccl_lib = next();
        else if (a == "--same-device") o.same_device = true;
        else pos.push_back(argv[i]);
    }
    long m_rows = 0, m_cols = 0;
    int m_gap = 0, m_iters = 0, m_parts = 0;
    if (!o.resume.empty()) {
        FILE *mf = fopen((o.resume + ".gol").c_str(), "r");
        if (!mf || fscanf(mf, "%ld %ld %d %d %d", &m_rows, &m_cols, &m_gap, &m_iters, &m_parts) != 5)
            die("--resume: cannot read the main .gol file");
        fclose(mf);
        if (o.from < 0) die("--resume needs --from ITER");
        if (pos.empty()) {
            static std::string a0, a1, a2, a3;
            a0 = std::to_string(m_rows), a1 = std::to_string(m_cols), a2 = std::to_string(m_gap),
            a3 = std::to_string(m_iters);
            pos = {a0.c_str(), a1.c_str(), a2.c_str(), a3.c_str()};
        }
    }
    if (pos.size() < 4 || pos.size() > 6)
        die("This program should be called with four arguments! \nThese should be, the total number of rows; "
            "the total number of columns; the gap between saved iterations and the total number of "
            "iterations, in that order.");
    const long rows = atol(pos[0]), cols = atol(pos[1]);
    const int gap = atoi(pos[2]), iters = atoi(pos[3]);
    std::string time_file;
    int first = pos.size() > 5 ? atoi(pos[5]) : 0;

    int boundary = GOL_DEAD, init = GOL_INIT_STREAM, m = 1;
    uint32_t seed = 1;
    int layout = o.layout == "byte" ? GOL_LAYOUT_BYTE : GOL_LAYOUT_BIT;
    bool save = false;
    if (o.mode == "mpi") {
        // main.cpp:194-199
        const float z = std::sqrt((float)o.procs);
        if (rows <= 0 || rows != cols || z != std::floor(z) || rows % (int)z != 0 || rows / (int)z < 4)
            die("Illegal board size parameter combination!");
        m = (int)z;
        seed = 0;   // block (cx,cy) <- srand(cx·m + cy); srand(0) ≡ srand(1)
        if (m > 1) {
            boundary = GOL_MESH_COMPAT;
            init = GOL_INIT_MESH;
            // the bit layout's device init needs 32-column-aligned mesh blocks
            if (o.layout.empty() && (cols / m) % 32 != 0) layout = GOL_LAYOUT_BYTE;
        }
        save = o.save == 1;   // main.cpp:208 hard-codes save_file = 0
    } else if (o.mode == "serial") {
        if (rows != cols) die("serial mode needs rows == cols");
        boundary = GOL_SERIAL_COMPAT;
        init = GOL_INIT_SERIAL;
        seed = GOL_SERIAL_SEED;   // main_serial.cpp:150
        save = o.save != 0;
    } else if (o.mode == "dead") {
        save = o.save == 1;
    } else {
        die("--mode must be mpi, serial or dead");
    }
    if (o.seed >= 0) seed = (uint32_t)o.seed;
    if (gap <= 0 && save) die("iteration_gap must be positive when saving");

    const int parts = o.gpus;
    const int from = o.resume.empty() ? 0 : o.from;
    if (from > iters) die("--from is past the last iteration");
    if (!o.resume.empty() && (m_rows != rows || m_cols != cols)) die("--resume: board size differs from the main file");
    // a resumed run keeps the original name so gol_visualization.py sees one sequence of iterations
    std::string name = o.resume.empty() ? set_up_program(rows, cols, gap, iters, parts) : o.resume;
    if (!o.resume.empty() && parts != m_parts) {
        // the part count of the new snapshots must match the main file
        FILE *mf = fopen((name + ".gol").c_str(), "w");
        if (!mf) die("cannot rewrite the main .gol file");
        fprintf(mf, "%ld %ld %d %d %d\n", rows, cols, gap, std::max(iters, m_iters), parts);
        fclose(mf);
    }
    time_file = pos.size() > 4 ? std::string(pos[4]) : name;

    std::vector<int64_t> row0(parts), nrow(parts);
    for (int p = 0; p < parts; ++p) gol_slab_plan(rows, parts, p, &row0[p], &nrow[p]);
    // --rccl: one rank context per slab; otherwise ONE context holding every slab
    const int nctx = o.rccl ? parts : 1;
    std::vector<RankRun> rk(nctx);
    if (o.rccl) {
        if (!o.rccl_lib.empty() && !dlopen(o.rccl_lib.c_str(), RTLD_NOW | RTLD_GLOBAL))
            die(("--rccl-lib: cannot load " + o.rccl_lib).c_str());
        if (!o.resume.empty() && m_parts != parts) die("--rccl --resume needs the saved run's part count");
    }
    uint8_t uid[GOL_UNIQUE_ID_BYTES];
    if (o.rccl) check(nullptr, gol_get_unique_id(uid), "gol_get_unique_id");
    // part p of a snapshot: the rows of slab p, written by the context holding them
    auto write_snap = [&](gol_ctx *ctx, int iter, int p) {
        if (o.mode == "serial" && parts == 1)   // main_serial.cpp:164-167: "0 n" / "0 n"
            write_part(ctx, name, iter, p, 0, rows, 0, cols, 0, rows, cols);
        else   // main.cpp:255-258: inclusive ranges (gol_visualization.py:33 slices [min, max+1])
            write_part(ctx, name, iter, p, row0[p], row0[p] + nrow[p] - 1, 0, cols - 1, row0[p], nrow[p], cols);
    };
    // set-up of context i (rank i under --rccl): create, then the board
    auto set_up = [&](int i) {
        gol_ctx *ctx = nullptr;
        if (o.rccl)
            check(nullptr, gol_create_rank(&ctx, rows, cols, i, parts, o.same_device ? 0 : i, uid, layout, boundary,
                                           m, o.k), "gol_create_rank");
        else
            check(nullptr, gol_create(&ctx, rows, cols, o.gpus, layout, boundary, m, o.k), "gol_create");
        rk[i].ctx = ctx;
        // launches are counted on the host (gol_kernel_time without GOL_OPT_KERNEL_TIMING): no event pair
        // per launch inside the timed region
        if (o.resume.empty()) {
            check(ctx, gol_init_glibc(ctx, init, seed), "gol_init_glibc");
        } else {
            for (int p = 0; p < m_parts; ++p)
                if (!o.rccl || p == i)
                    read_part(ctx, o.resume + "_" + std::to_string(from) + "_" + std::to_string(p) + ".gol");
        }
        // main_serial.cpp:171 writes generation 0; main.cpp:285 has that write commented out, which
        // leaves gol_visualization.py without its iteration-0 files, so every saving mode writes it.
        if (save && o.resume.empty())
            for (int p = 0; p < parts; ++p)
                if (!o.rccl || p == i) write_snap(ctx, 0, p);
        check(ctx, gol_sync(ctx, nullptr), "gol_sync");
    };
    // the generation loop of context i (main.cpp:291-305): every rank steps the same generations
    auto run = [&](int i) {
        gol_ctx *ctx = rk[i].ctx;
        double dev_ms = 0.0;
        if (save) {
            // step straight to the next snapshot (k-generation blocks inside gol_step)
            for (int a = from; a < iters;) {
                const int next = std::min(iters, (a / gap + 1) * gap);
                check(ctx, gol_step(ctx, next - a), "gol_step");
                a = next;
                if (a % gap == 0) {
                    double ms = 0;
                    check(ctx, gol_sync(ctx, &ms), "gol_sync");
                    dev_ms += ms;
                    for (int p = 0; p < parts; ++p)
                        if (!o.rccl || p == i) write_snap(ctx, a, p);
                }
            }
        } else {
            check(ctx, gol_step(ctx, iters - from), "gol_step");
        }
        double ms = 0;
        check(ctx, gol_sync(ctx, &ms), "gol_sync");
        rk[i].dev_ms = dev_ms + ms;
        double kernel_ms = 0;
        check(ctx, gol_popcount(ctx, &rk[i].live), "gol_popcount");
        check(ctx, gol_kernel_time(ctx, &kernel_ms, &rk[i].launches, 0), "gol_kernel_time");
    };
    if (o.rccl) on_ranks(nctx, set_up);
    else set_up(0);
    auto t_check1 = std::chrono::steady_clock::now();
    if (o.rccl) on_ranks(nctx, run);
    else run(0);
    // the ranks' reduction (main.cpp:319-324): the slowest rank's device time, every rank's cells
    double dev_ms = 0.0;
    int64_t live = 0, launches = 0;
    for (auto &r : rk) {
        dev_ms = std::max(dev_ms, r.dev_ms);
        live += r.live;
        launches += r.launches;
    }
    auto t_end = std::chrono::steady_clock::now();
    if (o.rccl) on_ranks(nctx, [&](int i) { gol_destroy(rk[i].ctx); });
    else gol_destroy(rk[0].ctx);

    // main.cpp:312-364 (µs values, "ms" labels; sums over the emulated parts)
    const long local = (long)std::chrono::duration_cast<std::chrono::microseconds>(t_end - t_begin).count();
    const long nosetup = (long)std::chrono::duration_cast<std::chrono::microseconds>(t_end - t_check1).count();
    const long setup = (long)std::chrono::duration_cast<std::chrono::microseconds>(t_check1 - t_begin).count();
    // main.cpp:341-362 reports the MPI processors; here the emulated ranks of --mode mpi (--procs),
    // which the GPU slabs stand in for.  The GPU count goes to _gcups.csv.
    const int P = o.mode == "mpi" ? o.procs : parts;
    FILE *f = fopen((time_file + "_detailed.out").c_str(), "a");
    if (f) {
        fprintf(f, "Timing results: milliseconds \nsize:%ld by %ld\n%d Processors\n", cols, rows, P);
        fprintf(f, "Full (with setup) \nSingle time (rank 0): %ldms\nAvg single time: %ldms\nSummed time: %ldms\n",
                local, local, local * P);
        fprintf(f, "Without setup \nSingle time (rank 0): %ldms\nAvg single time: %ldms\nSummed time: %ldms\n",
                nosetup, nosetup, nosetup * P);
        fprintf(f, "Setup \nSingle time (rank 0): %ldms\nAvg single time: %ldms\nSummed time: %ldms\n", setup,
                setup, setup * P);
        fprintf(f, "___________________________________________________ \n\n");
        fclose(f);
    }
    f = fopen((time_file + "_compact.csv").c_str(), "a");
    if (f) {
        if (first != 0)
            fprintf(f, "X,Y,#P,full single,full avg,full sum,nosetup single,nosetup avg,nosetup sum,"
                       "setup single ,setup avg ,setup sum \n");
        fprintf(f, "%ld,%ld,%d,%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld\n", cols, rows, P, local, local, local * P,
                nosetup, nosetup, nosetup * P, setup, setup, setup * P);
        fclose(f);
    }
    // additions, in a separate file so the reference's formats stay untouched
    const double gcups = (double)rows * cols * (iters - from) / (dev_ms * 1e-3) / 1e9;
    f = fopen((time_file + "_gcups.csv").c_str(), "a");
    if (f) {
        fprintf(f, "%ld,%ld,%d,%d,%s,%d,%.3f,%.3f,%lld,%lld\n", rows, cols, iters, parts,
                layout == GOL_LAYOUT_BIT ? "bit" : "byte", o.k, dev_ms, gcups, (long long)live, (long long)launches);
        fclose(f);
    }
    printf("0: %s  gens=%d  device %.3f ms  %.1f GCUPS  live=%lld  launches=%lld%s\n", name.c_str(), iters - from,
           dev_ms, gcups, (long long)live, (long long)launches, o.rccl ? "  (rccl ranks)" : "");
    printf("0: all succeeded\n");
    return 0;
}
