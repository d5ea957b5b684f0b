/*
 * gol_fast_gen.c -- golden-checkpoint generator for the full-size north-star boards.  TEST INFRASTRUCTURE
 * ONLY: run here (CPU) by tests/golden/make_golden_full.py; nothing on the GPU box executes it.
 *
 *   gol_fast_gen W H boundary seed generations every threads
 *
 * Seeds a W x H board with the build's large-board init (oracle_seed_splitmix in gol_oracle.c:
 * alive(x, y) = bit (x & 31) of low32(splitmix64(seed ^ (y*ceil(W/32) + x/32)))), packed directly into
 * the canonical 64-cell words, then runs gol_fast.c's carry-save stepper (the synchronous B3/S23 step of
 * GameOfLifeLogic.fs:59-63 under the Reset->State phase barrier; torus GameOfLifeDriver.fs:21-25, bounded
 * Script.fsx:6-13) and prints one JSON line per checkpoint:
 *   {"generation": g, "hash": h, "population": p}
 * generation 0 (the seeded board) first.  Each line is flushed, so a long run can be followed.
 */
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

uint64_t fast_hash(const uint64_t* b, int64_t W, int64_t H);
int64_t fast_population(const uint64_t* b, int64_t W, int64_t H);
int fast_run(uint64_t* board, int64_t W, int64_t H, int boundary, int64_t gens, int threads, int64_t every,
             uint64_t* hashes, int64_t* pops);
int fast_seed_splitmix(uint64_t* board, int64_t W, int64_t H, uint64_t seed);

int main(int argc, char** argv) {
    if (argc != 8) {
        fprintf(stderr, "usage: %s W H boundary(0 torus|1 bounded) seed generations every threads\n", argv[0]);
        return 2;
    }
    const int64_t W = atoll(argv[1]), H = atoll(argv[2]);
    const int boundary = atoi(argv[3]);
    const uint64_t seed = strtoull(argv[4], NULL, 0);
    const int64_t gens = atoll(argv[5]), every = atoll(argv[6]);
    const int threads = atoi(argv[7]);
    if (W < 64 || W % 64 || H < 3 || gens < 0 || every <= 0 || gens % every) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    uint64_t* b = (uint64_t*)malloc((size_t)(W / 64 * H) * sizeof(uint64_t));
    if (!b || fast_seed_splitmix(b, W, H, seed)) {
        fprintf(stderr, "out of memory\n");
        return 1;
    }
    printf("{\"generation\": 0, \"hash\": %" PRIu64 ", \"population\": %" PRId64 "}\n", fast_hash(b, W, H),
           fast_population(b, W, H));
    fflush(stdout);
    uint64_t h;
    int64_t p;
    /* one fast_run per checkpoint interval: progress is printed as it goes */
    for (int64_t g = every; g <= gens; g += every) {
        if (fast_run(b, W, H, boundary, every, threads, every, &h, &p)) {
            fprintf(stderr, "fast_run failed\n");
            return 1;
        }
        printf("{\"generation\": %" PRId64 ", \"hash\": %" PRIu64 ", \"population\": %" PRId64 "}\n", g, h, p);
        fflush(stdout);
    }
    free(b);
    return 0;
}
