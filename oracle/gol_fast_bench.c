/*
 * gol_fast_bench.c -- the "fair CPU" baseline timer ("optionally also report a bit-sliced
 * multithreaded CPU stepper").  TEST / BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg runs it on the
 * GPU box's host cores, outside the timed region; nothing in the product links it.
 *
 *   gol_fast_bench W H boundary threads min_seconds
 *
 * Seeds the bench board (splitmix 0x5EED, fast_seed_splitmix) and runs gol_fast.c's carry-save stepper in
 * chunks of 4 generations until at least min_seconds have passed; prints one JSON line.
 */
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int fast_run(uint64_t* board, int64_t W, int64_t H, int boundary, int64_t gens, int threads, int64_t every,
             uint64_t* hashes, int64_t* pops);
int fast_seed_splitmix(uint64_t* board, int64_t W, int64_t H, uint64_t seed);
int64_t fast_population(const uint64_t* b, int64_t W, int64_t H);

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s W H boundary threads min_seconds\n", argv[0]);
        return 2;
    }
    const int64_t W = atoll(argv[1]), H = atoll(argv[2]);
    const int boundary = atoi(argv[3]), threads = atoi(argv[4]);
    const double min_s = atof(argv[5]);
    uint64_t* b = (uint64_t*)malloc((size_t)(W / 64 * H) * sizeof(uint64_t));
    if (!b || fast_seed_splitmix(b, W, H, 0x5EED)) return 1;
    int64_t gens = 0;
    const double t0 = now();
    double dt = 0;
    while (dt < min_s) {
        if (fast_run(b, W, H, boundary, 4, threads, 0, NULL, NULL)) return 1;
        gens += 4;
        dt = now() - t0;
    }
    printf("{\"width\": %" PRId64 ", \"height\": %" PRId64 ", \"generations\": %" PRId64 ", \"threads\": %d, "
           "\"seconds\": %.6f, \"cell_updates_per_s\": %.3f, \"population\": %" PRId64 "}\n",
           W, H, gens, threads, dt, (double)W * (double)H * (double)gens / dt, fast_population(b, W, H));
    free(b);
    return 0;
}
