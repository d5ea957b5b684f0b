/*
 * gol_fast.c -- bit-packed multithreaded CPU ORACLE for long runs.  TEST INFRASTRUCTURE ONLY.
 *
 * Same semantics as gol_oracle.c (which it is checked against in tests/test_oracle.py): the synchronous
 * B3/S23 step of the reference actors under the Reset->State phase barrier --
 *   rule      GameOfLife/GameOfLife/GameOfLifeLogic.fs:59-63 (== GameOfLifeAkka/GameofLife.fs:108-112)
 *   torus     GameOfLifeDriver.fs:21-25;  bounded  Script.fsx:6-18
 * -- on boards stored 64 cells per uint64 (bit b of word j of row y = cell (64j + b, y)), so the
 * generator scripts can produce golden checkpoints for the long-run configurations (BASELINE.json
 * configs 2 and 5: 4096^2 x 10k generations, Gosper gun / R-pentomino x 100k generations) in seconds
 * rather than hours.  Deliberately a DIFFERENT formulation from the GPU kernel: each cell's 8 neighbour
 * planes are summed by a plain carry-save adder tree into a 4-bit count, then count == 3 | (alive &
 * count == 2) -- no shared row sums, no LUT tree, no interleaving.
 *
 * Requires W % 64 == 0 and W, H >= 3.  Threads split the rows; one barrier per generation.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FAST_TORUS 0
#define FAST_BOUNDED 1

static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

/* canonical hash (== oracle_hash in gol_oracle.c for W % 64 == 0) */
uint64_t fast_hash(const uint64_t* b, int64_t W, int64_t H) {
    const int64_t nw = W / 64;
    uint64_t h = 0;
    for (int64_t y = 0; y < H; y++)
        for (int64_t j = 0; j < nw; j++)
            h += fmix64(b[y * nw + j] ^ fmix64((uint64_t)(y * nw + j) + 0x9E3779B97F4A7C15ULL));
    return fmix64(h ^ fmix64((uint64_t)W * 0x100000001B3ULL + (uint64_t)H));
}

int64_t fast_population(const uint64_t* b, int64_t W, int64_t H) {
    int64_t p = 0;
    for (int64_t i = 0; i < W / 64 * H; i++) p += __builtin_popcountll(b[i]);
    return p;
}

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* oracle_seed_splitmix (gol_oracle.c) written straight into the 64-cell words: cells 64j .. 64j + 31 are
 * the low 32 bits of splitmix64(seed ^ (y*W/32 + 2j)), cells 64j + 32 .. 64j + 63 those of 2j + 1. */
int fast_seed_splitmix(uint64_t* board, int64_t W, int64_t H, uint64_t seed) {
    if (!board || W < 64 || W % 64 || H < 1) return -1;
    const int64_t nw = W / 64, wc = W / 32;
    for (int64_t y = 0; y < H; y++)
        for (int64_t j = 0; j < nw; j++) {
            const uint64_t lo = (uint32_t)splitmix64(seed ^ (uint64_t)(y * wc + 2 * j));
            const uint64_t hi = (uint32_t)splitmix64(seed ^ (uint64_t)(y * wc + 2 * j + 1));
            board[y * nw + j] = lo | (hi << 32);
        }
    return 0;
}

/* full adder on bit planes */
#define FA(a, b, c, s, co)                 \
    do {                                   \
        uint64_t t_ = (a) ^ (b);           \
        (s) = t_ ^ (c);                    \
        (co) = ((a) & (b)) | (t_ & (c));   \
    } while (0)

/* next state of 64 cells from the 3x3 words around them (l = word to the west, r = to the east) */
static inline uint64_t next_word(uint64_t ul, uint64_t uc, uint64_t ur, uint64_t ml, uint64_t mc, uint64_t mr,
                                 uint64_t dl, uint64_t dc, uint64_t dr) {
    /* the 8 neighbour planes: bit b of each = the neighbour of cell 64j + b in that direction */
    const uint64_t n0 = (uc << 1) | (ul >> 63), n1 = uc, n2 = (uc >> 1) | (ur << 63);
    const uint64_t n3 = (mc << 1) | (ml >> 63), n4 = (mc >> 1) | (mr << 63);
    const uint64_t n5 = (dc << 1) | (dl >> 63), n6 = dc, n7 = (dc >> 1) | (dr << 63);
    /* carry-save sum of the 8 planes -> 4-bit count (c0 c1 c2 c3) */
    uint64_t s1, k1, s2, k2, c0, k4, t1, t2;
    FA(n0, n1, n2, s1, k1);
    FA(n3, n4, n5, s2, k2);
    const uint64_t s3 = n6 ^ n7, k3 = n6 & n7;
    FA(s1, s2, s3, c0, k4);    /* weight-1 bit; k4 carries weight 2 */
    FA(k1, k2, k3, t1, t2);    /* weight 2 (t1) and 4 (t2) */
    const uint64_t c1 = t1 ^ k4;         /* weight-2 bit */
    const uint64_t t3 = t1 & k4;         /* carry into weight 4 */
    const uint64_t c2 = t2 ^ t3, c3 = t2 & t3;
    /* rule GameOfLifeLogic.fs:59-63: count == 3 -> alive; count == 2 -> keep; else dead */
    return c1 & ~c2 & ~c3 & (c0 | mc);
}

/* one output row from rows up / mid / dn (a dead row is passed as an all-zero row) */
static void step_row(const uint64_t* up, const uint64_t* mid, const uint64_t* dn, uint64_t* out, int64_t nw,
                     int torus) {
    if (nw == 1) {
        const uint64_t u = up[0], m = mid[0], d = dn[0], z = torus ? 1 : 0;
        out[0] = next_word(z ? u : 0, u, z ? u : 0, z ? m : 0, m, z ? m : 0, z ? d : 0, d, z ? d : 0);
        return;
    }
    const int64_t e = nw - 1;
    out[0] = next_word(torus ? up[e] : 0, up[0], up[1], torus ? mid[e] : 0, mid[0], mid[1], torus ? dn[e] : 0,
                       dn[0], dn[1]);
    for (int64_t j = 1; j < e; j++)
        out[j] = next_word(up[j - 1], up[j], up[j + 1], mid[j - 1], mid[j], mid[j + 1], dn[j - 1], dn[j], dn[j + 1]);
    out[e] = next_word(up[e - 1], up[e], torus ? up[0] : 0, mid[e - 1], mid[e], torus ? mid[0] : 0, dn[e - 1], dn[e],
                       torus ? dn[0] : 0);
}

typedef struct {
    uint64_t *a, *b;
    int64_t W, H, gens, every;
    int boundary, nthreads;
    uint64_t* hashes;
    int64_t* pops;
    pthread_barrier_t bar;
} fast_job;

typedef struct {
    fast_job* job;
    int tid;
} fast_arg;

static void* worker(void* p) {
    fast_arg* fa = (fast_arg*)p;
    fast_job* J = fa->job;
    const int64_t nw = J->W / 64, H = J->H;
    const int torus = J->boundary == FAST_TORUS;
    const int64_t y0 = H * fa->tid / J->nthreads, y1 = H * (fa->tid + 1) / J->nthreads;
    uint64_t *src = J->a, *dst = J->b;
    uint64_t* zero = (uint64_t*)calloc((size_t)nw, sizeof(uint64_t));
    for (int64_t g = 0; g < J->gens; g++) {
        for (int64_t y = y0; y < y1; y++) {
            const uint64_t* up = y > 0 ? src + (y - 1) * nw : (torus ? src + (H - 1) * nw : zero);
            const uint64_t* dn = y < H - 1 ? src + (y + 1) * nw : (torus ? src : zero);
            step_row(up, src + y * nw, dn, dst + y * nw, nw, torus);
        }
        uint64_t* t = src;
        src = dst;
        dst = t;
        pthread_barrier_wait(&J->bar);
        if (J->every > 0 && (g + 1) % J->every == 0 && fa->tid == 0) {
            const int64_t i = (g + 1) / J->every - 1;
            J->hashes[i] = fast_hash(src, J->W, H);
            J->pops[i] = fast_population(src, J->W, H);
        }
        if (J->every > 0 && (g + 1) % J->every == 0) pthread_barrier_wait(&J->bar);
    }
    free(zero);
    return NULL;
}

/* Run `gens` generations in place on `board` (W/64 words per row, H rows).  If every > 0, records the
 * canonical hash and population after every `every` generations into hashes[i], pops[i] (i = 0 ..
 * gens/every - 1).  Returns 0, or -1 on bad arguments. */
int fast_run(uint64_t* board, int64_t W, int64_t H, int boundary, int64_t gens, int threads, int64_t every,
             uint64_t* hashes, int64_t* pops) {
    if (!board || W < 64 || W % 64 || H < 3 || gens < 0) return -1;
    if (boundary != FAST_TORUS && boundary != FAST_BOUNDED) return -1;
    if (every > 0 && (!hashes || !pops)) return -1;
    if (threads < 1) threads = 1;
    if (threads > H) threads = (int)H;
    const size_t n = (size_t)(W / 64 * H);
    uint64_t* tmp = (uint64_t*)malloc(n * sizeof(uint64_t));
    if (!tmp) return -1;
    fast_job J;
    memset(&J, 0, sizeof J);
    J.a = board;
    J.b = tmp;
    J.W = W;
    J.H = H;
    J.gens = gens;
    J.every = every;
    J.boundary = boundary;
    J.nthreads = threads;
    J.hashes = hashes;
    J.pops = pops;
    pthread_barrier_init(&J.bar, NULL, (unsigned)threads);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    fast_arg* args = (fast_arg*)malloc(sizeof(fast_arg) * (size_t)threads);
    for (int t = 0; t < threads; t++) {
        args[t].job = &J;
        args[t].tid = t;
        pthread_create(&th[t], NULL, worker, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&J.bar);
    if (gens % 2) memcpy(board, tmp, n * sizeof(uint64_t)); /* odd count: result landed in tmp */
    free(args);
    free(th);
    free(tmp);
    return 0;
}
