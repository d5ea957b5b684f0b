// lib_pipe_bench.hip -- times the library's level-pipelined pass (csrc/gol_pipe.hip, gol::launch_pipe_step) with the
// prototype's method (pipe_proto.hip: ~1 s clock warm-up, a fresh splitmix board advanced past generation 300, then
// at least 240 generations timed by HIP events), so the two can be compared on one box.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../gameoflifewithactors_amd/csrc -o lib_pipe_bench \
//        lib_pipe_bench.hip ../../gameoflifewithactors_amd/csrc/gol_pipe.hip
// Usage: lib_pipe_bench W H K rounds [split [split2 [wrap]]]   (wrap 0: a ghost-row strip of H rows and K ghost rows
// per side, output rows [K, H - K): the N > 1 interior launch)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>

#include "gol_internal.h"

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void seed_k(uint32_t* b, int64_t n, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = seed ^ (uint64_t)i;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    b[i] = (uint32_t)z;
}

int main(int argc, char** argv) {
    const int64_t W = argc > 1 ? atoll(argv[1]) : 65536, H = argc > 2 ? atoll(argv[2]) : 65536;
    const int K = argc > 3 ? atoi(argv[3]) : 32, rounds = argc > 4 ? atoi(argv[4]) : 2;
    const int split = argc > 5 ? (int)(atof(argv[5]) * 65536) : 0;  // < 0: equal shares
    const int split2 = argc > 6 ? (int)(atof(argv[6]) * 65536) : 0;
    const bool wrap = argc > 7 ? atoi(argv[7]) != 0 : true;
    const int64_t ghost = wrap ? 0 : (argc > 8 ? atoll(argv[8]) : K);  // wrap 0: ghost rows per side (the kernel's K by default)
    const int64_t words = W / 32, n = words * (H + 2 * ghost);
    uint32_t *a, *b;
    int* err;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    CHECK(hipMalloc(&err, 4));
    CHECK(hipMemset(err, 0, 4));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    gol::PipeArgs pa{};
    pa.words = words;
    pa.pitch = words;
    pa.rows = H;
    pa.ghost = ghost;
    pa.out_begin = wrap ? 0 : K;
    pa.out_end = wrap ? H : H - K;
    pa.split1 = split;
    pa.split2 = split2;
    pa.err = err;
    {
        gol::PipeArgs q = pa;
        gol::plan_pipe(q, K, wrap, 0);
        printf("plan: nstrips %lld rem %d rq %d rp %d P %d ngroups %lld grows %lld pk [%lld, %lld) npk %lld nrem %lld "
               "split %d/%d grid %lld\n", (long long)q.nstrips, q.rem, q.rq, q.rp, q.P, (long long)q.ngroups,
               (long long)q.grows, (long long)q.pk_lo, (long long)q.pk_hi, (long long)q.npk, (long long)q.nrem, q.split1,
               q.split2, (long long)gol::pipe_grid(q));
    }
    auto pass = [&]() {
        CHECK(gol::launch_pipe_step(a, b, pa, K, wrap, st));
        std::swap(a, b);
    };
    seed_k<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, n, 0x5EEDull);
    CHECK(hipEventRecord(e0, st));
    for (int i = 0;; i++) {
        pass();
        if (i % 16 == 15) {
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms > 1000.0f) break;
        }
    }
    for (int round = 0; round < rounds; round++) {
        seed_k<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, n, 0x5EEDull);
        int gen = 0;
        while (gen < 300) {
            pass();
            gen += K;
        }
        const int np = (240 + K - 1) / K < 8 ? 8 : (240 + K - 1) / K;
        CHECK(hipEventRecord(e0, st));
        for (int i = 0; i < np; i++) pass();
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        int e = 0;
        CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        const double us = ms * 1000.0 / np;
        printf("  round %d library gol_pipe_step K=%d: %.1f us/pass, %.1fk GCUPS (generations %d-%d) err %d\n", round, K, us,
               (double)W * H * K / (us * 1e-6) / 1e12, gen, gen + np * K, e);
        fflush(stdout);
    }
    return 0;
}
