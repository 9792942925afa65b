// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Drives the reference's OWN hot-path functions, compiled from where they lie
// (/root/reference/main.cpp, passed in as REF_MAIN by oracle/Makefile):
//   initializeBoard  main.cpp:68-77   (srand(rank); rand()%3==0)
//   distr_borders    main.cpp:36-65   (column halos swapped, then rows)
//   updateBoard/next main.cpp:79-103  (B3/S23 over the padded block)
// The topology set-up mirrors main.cpp:240-276 (√P×√P Cartesian mesh,
// periods {0,0}, reorder=1, coords from the world rank).  Unlike main.cpp the
// boards are calloc'ed, so never-written halos read as 0 — the "zero malloc"
// assumption of SURVEY.md §8c made deterministic.  The reference's main()
// never writes boards (save_file=0, main.cpp:208), so this harness gathers the
// interior blocks to rank 0 and dumps the global n×n board as np.packbits
// (MSB-first, row-major) bytes: <prefix>_g<gen>.bin.
//
// usage: mpirun -np P ref_harness_mpi n gens dump_every prefix
#define main gol_reference_main
#include REF_MAIN
#undef main

#include <cstdio>
#include <cstdlib>
#include <cstring>

static void dump_global(bool **board, int L, int m, int rank, int procs, MPI_Comm comm,
                        int n, int gen, const char *prefix) {
    std::vector<unsigned char> mine((size_t)L * L);
    for (int i = 0; i < L; i++)
        for (int j = 0; j < L; j++) mine[(size_t)i * L + j] = board[i + 1][j + 1] ? 1 : 0;
    if (rank != 0) {
        MPI_Send(mine.data(), L * L, MPI_UNSIGNED_CHAR, 0, 7, MPI_COMM_WORLD);
        return;
    }
    std::vector<unsigned char> g((size_t)n * n, 0), buf((size_t)L * L);
    for (int r = 0; r < procs; r++) {
        if (r == 0) buf = mine;
        else MPI_Recv(buf.data(), L * L, MPI_UNSIGNED_CHAR, r, 7, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
        int coor[2];
        MPI_Cart_coords(comm, r, 2, coor);       // same call as main.cpp:250
        int row0 = coor[0] * L, col0 = coor[1] * L; // down_c / left_c, main.cpp:255-257
        for (int i = 0; i < L; i++)
            memcpy(&g[(size_t)(row0 + i) * n + col0], &buf[(size_t)i * L], L);
    }
    std::vector<unsigned char> packed(((size_t)n * n + 7) / 8, 0);
    for (size_t k = 0; k < (size_t)n * n; k++)
        if (g[k]) packed[k >> 3] |= (unsigned char)(0x80u >> (k & 7));
    char path[1024];
    snprintf(path, sizeof path, "%s_g%d.bin", prefix, gen);
    FILE *f = fopen(path, "wb");
    fwrite(packed.data(), 1, packed.size(), f);
    fclose(f);
}

int main(int argc, char *argv[]) {
    MPI_Init(&argc, &argv);
    int rank, procs;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &procs);
    if (argc != 5) {
        if (rank == 0) fprintf(stderr, "usage: ref_harness_mpi n gens dump_every prefix\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    int n = atoi(argv[1]), gens = atoi(argv[2]), every = atoi(argv[3]);
    const char *prefix = argv[4];
    int m = (int)std::lround(std::sqrt((double)procs));
    if (m * m != procs || n % m != 0 || n / m < 4) {   // main.cpp:194-199
        if (rank == 0) fprintf(stderr, "illegal size/procs combination\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    distrOpt options{};
    options = {n, n, m, m, gens, every, 0, 0, n / m, n / m};   // field order of main.cpp:202-210

    int dims[2] = {m, m}, periods[2] = {0, 0};
    MPI_Dims_create(procs, 2, dims);
    MPI_Comm comm;
    MPI_Cart_create(MPI_COMM_WORLD, 2, dims, periods, 1, &comm);
    int p_up, p_down, p_left, p_right;
    MPI_Cart_shift(comm, 0, 1, &p_up, &p_down);
    MPI_Cart_shift(comm, 1, 1, &p_left, &p_right);
    neighbours nbr = {p_left, p_right, p_down, p_up};

    int L = n / m;
    bool **board = (bool **)malloc((L + 2) * sizeof(bool *));
    bool **board2 = (bool **)malloc((L + 2) * sizeof(bool *));
    bool *d1 = (bool *)calloc((size_t)(L + 2) * (L + 2), 1);
    bool *d2 = (bool *)calloc((size_t)(L + 2) * (L + 2), 1);
    for (int i = 0; i < L + 2; i++) { board[i] = d1 + (size_t)i * (L + 2); board2[i] = d2 + (size_t)i * (L + 2); }

    initializeBoard(board, options, rank);
    distr_borders(board, nbr, comm, options);
    dump_global(board, L, m, rank, procs, comm, n, 0, prefix);
    for (int a = 1; a <= gens; ++a) {          // loop of main.cpp:291-305
        updateBoard(board, board2, options);
        bool **tmp = board; board = board2; board2 = tmp;
        MPI_Barrier(MPI_COMM_WORLD);
        distr_borders(board, nbr, comm, options);
        if (every > 0 && a % every == 0) dump_global(board, L, m, rank, procs, comm, n, a, prefix);
    }
    MPI_Finalize();
    return 0;
}
