/*
 * gol_oracle.c -- CPU ORACLE for the Game of Life hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
 * and only as the checker.  The product (libgol_hip.so) never links or calls it.
 *
 * It restates, cell by cell and byte per cell, what the reference computes on the path
 * BASELINE.json `north_star` names (the per-cell actor loop applying B3/S23):
 *
 *   rule      GameOfLife/GameOfLife/GameOfLifeLogic.fs:59-63   (== GameOfLifeAkka/GameofLife.fs:108-112)
 *   torus     GameOfLife/GameOfLife/GameOfLifeDriver.fs:21-25  (== GameofLife.fs:154-158)
 *   bounded   GameOfLife/GameOfLife/Script.fsx:6-18             (skip out-of-range, subtract self)
 *   snapshot  GameOfLifeLogic.fs:47-55 (wasAlive <- isAlive on Reset, State replies wasAlive): under the
 *             Reset->State phase barrier this is a double-buffered synchronous step.
 *   init      GameOfLifeDriver.fs:9-11,16-19 (x outer, y inner, Random.Next() % 2 = 0)
 *             Script.fsx:25-27 (Array2D.init n n, index 0 outer, Random.Next 2 = 0)
 *   pixels    GameOfLifeUI.fs:24-28 (pixels[x + y*size] = 128 | 0), Script.fsx:33-35 (255 | 0)
 *
 * Third-party arithmetic restated here (absent from /root/reference, binaries only):
 *   .NET Framework 4.x System.Random (mscorlib; call sites GameOfLifeDriver.fs:10-11, GameofLife.fs:141-142,
 *   Script.fsx:25,27): Knuth subtractive generator, MSEED = 161803398, 56-entry table.
 *   Pinned only by published values (Random(0).Next() = 1559595546, Random(1) -> 534011718,
 *   Random(42) -> 1434747710); no reference test pins it.
 *
 * PARITY PIN STATUS: the reference holds no tests, fixtures or golden vectors for this path
 *  and cannot be built or run here (F#/.NET/WPF, no dotnet).  This oracle is
 * pinned by external known-answer facts (blinker, block, glider period 4W on a torus, R-pentomino
 * population 116 at generation 1103, Gosper gun period 30, full board dies) and the published .NET
 * Random values, all checked in tests/test_oracle.py.  The board-state parity versus the F# actors
 * themselves is therefore "parity unpinned" beyond those facts.
 *
 * Extra definitions owned by this build (not in the reference; used for large boards):
 *   splitmix init, canonical 64-bit board hash -- see DESIGN.md "Canonical hash".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_TORUS 0
#define OR_BOUNDED 1

/* ------------------------------------------------------------------ .NET System.Random */
typedef struct {
    int32_t seed_array[56];
    int inext, inextp;
} dn_random;

#define DN_MBIG 2147483647
#define DN_MSEED 161803398

static int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

void dn_random_init(dn_random* r, int32_t seed) {
    int32_t subtraction = (seed == INT32_MIN) ? DN_MBIG : (seed < 0 ? -seed : seed);
    int32_t mj = DN_MSEED - subtraction;
    int32_t mk = 1;
    memset(r->seed_array, 0, sizeof(r->seed_array));
    r->seed_array[55] = mj;
    for (int i = 1; i < 55; i++) {
        int ii = (21 * i) % 55;
        r->seed_array[ii] = mk;
        mk = wrap32((int64_t)mj - mk);
        if (mk < 0) mk += DN_MBIG;
        mj = r->seed_array[ii];
    }
    for (int k = 1; k < 5; k++) {
        for (int i = 1; i < 56; i++) {
            r->seed_array[i] = wrap32((int64_t)r->seed_array[i] - r->seed_array[1 + (i + 30) % 55]);
            if (r->seed_array[i] < 0) r->seed_array[i] += DN_MBIG;
        }
    }
    r->inext = 0;
    r->inextp = 21;
}

static int32_t dn_internal_sample(dn_random* r) {
    int loc_inext = r->inext, loc_inextp = r->inextp;
    if (++loc_inext >= 56) loc_inext = 1;
    if (++loc_inextp >= 56) loc_inextp = 1;
    int32_t ret = wrap32((int64_t)r->seed_array[loc_inext] - r->seed_array[loc_inextp]);
    if (ret == DN_MBIG) ret--;
    if (ret < 0) ret += DN_MBIG;
    r->seed_array[loc_inext] = ret;
    r->inext = loc_inext;
    r->inextp = loc_inextp;
    return ret;
}

int32_t dn_random_next(dn_random* r) { return dn_internal_sample(r); }

/* Next(maxValue) = (int)(Sample() * maxValue), Sample() = InternalSample() * (1.0 / MBIG) */
int32_t dn_random_next_max(dn_random* r, int32_t max_value) {
    double s = dn_internal_sample(r) * (1.0 / DN_MBIG);
    return (int32_t)(s * max_value);
}

/* ------------------------------------------------------------------ initial boards */
/* mode 0 "dotnet-mod2": GameOfLifeDriver.fs:9-11,16-19 -- RNG call k goes to (x = k / H, y = k % H),
 *   alive = Next() % 2 = 0.
 * mode 1 "dotnet-next2": Script.fsx:27 -- Array2D.init, index 0 (x) outer, alive = Next 2 = 0. */
int oracle_seed_dotnet(uint8_t* cells, int64_t W, int64_t H, int32_t seed, int mode) {
    if (!cells || W <= 0 || H <= 0 || (mode != 0 && mode != 1)) return -1;
    dn_random r;
    dn_random_init(&r, seed);
    for (int64_t x = 0; x < W; x++)
        for (int64_t y = 0; y < H; y++) {
            int alive = (mode == 0) ? (dn_random_next(&r) % 2 == 0) : (dn_random_next_max(&r, 2) == 0);
            cells[x + y * W] = (uint8_t)alive;
        }
    return 0;
}

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* build-owned init for large boards: alive(x,y) = bit (x & 31) of low32(splitmix64(seed ^ (y*ceil(W/32) + x/32))) */
int oracle_seed_splitmix(uint8_t* cells, int64_t W, int64_t H, uint64_t seed) {
    if (!cells || W <= 0 || H <= 0) return -1;
    int64_t wc = (W + 31) / 32;
    for (int64_t y = 0; y < H; y++)
        for (int64_t c = 0; c < wc; c++) {
            uint32_t bits = (uint32_t)splitmix64(seed ^ (uint64_t)(y * wc + c));
            for (int b = 0; b < 32 && c * 32 + b < W; b++) cells[c * 32 + b + y * W] = (bits >> b) & 1u;
        }
    return 0;
}

/* ------------------------------------------------------------------ one synchronous generation */
/* Rule, GameOfLifeLogic.fs:59-63:  match count with a when a > 3 || a < 2 -> false | 3 -> true | _ -> isAlive */
static inline uint8_t life_rule(int a, uint8_t is_alive) {
    if (a > 3 || a < 2) return 0;
    if (a == 3) return 1;
    return is_alive;
}

int oracle_step(const uint8_t* in, uint8_t* out, int64_t W, int64_t H, int boundary) {
    if (!in || !out || in == out || W < 3 || H < 3) return -1;
    if (boundary != OR_TORUS && boundary != OR_BOUNDED) return -1;
    for (int64_t y = 0; y < H; y++) {
        for (int64_t x = 0; x < W; x++) {
            int a = 0;
            /* neighbour enumeration: dx outer, dy inner, skip (0,0) -- GameOfLifeDriver.fs:21-25 */
            for (int64_t nx = x - 1; nx <= x + 1; nx++)
                for (int64_t ny = y - 1; ny <= y + 1; ny++) {
                    if (nx == x && ny == y) continue;
                    if (boundary == OR_TORUS) {
                        a += in[((nx + W) % W) + ((ny + H) % H) * W];
                    } else if (nx >= 0 && nx < W && ny >= 0 && ny < H) { /* Script.fsx:11 */
                        a += in[nx + ny * W];
                    }
                }
            out[x + y * W] = life_rule(a, in[x + y * W]);
        }
    }
    return 0;
}

/* n generations; result in `cells` (scratch is caller-provided, same size) */
int oracle_run(uint8_t* cells, uint8_t* scratch, int64_t W, int64_t H, int boundary, int64_t gens) {
    for (int64_t g = 0; g < gens; g++) {
        int rc = oracle_step(cells, scratch, W, H, boundary);
        if (rc) return rc;
        memcpy(cells, scratch, (size_t)(W * H));
    }
    return 0;
}

/* ------------------------------------------------------------------ observables */
int64_t oracle_population(const uint8_t* cells, int64_t W, int64_t H) {
    int64_t p = 0;
    for (int64_t i = 0; i < W * H; i++) p += cells[i] != 0;
    return p;
}

static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

/* Canonical hash: sum over 64-cell row chunks of fmix64(v ^ fmix64(key + phi)),
 * key = y * ceil(W/64) + j, bit b of v = cell (64j + b, y); finalised with the board dims. */
uint64_t oracle_hash(const uint8_t* cells, int64_t W, int64_t H) {
    int64_t nc = (W + 63) / 64;
    uint64_t h = 0;
    for (int64_t y = 0; y < H; y++)
        for (int64_t j = 0; j < nc; j++) {
            uint64_t v = 0;
            for (int b = 0; b < 64 && j * 64 + b < W; b++)
                if (cells[j * 64 + b + y * W]) v |= 1ULL << b;
            uint64_t key = (uint64_t)(y * nc + j);
            h += fmix64(v ^ fmix64(key + 0x9E3779B97F4A7C15ULL));
        }
    return fmix64(h ^ fmix64((uint64_t)W * 0x100000001B3ULL + (uint64_t)H));
}

/* GameOfLifeUI.fs:24-28: pixels[x + y*stride] = alive ? alive_value : 0 */
int oracle_render_gray8(const uint8_t* cells, int64_t W, int64_t H, uint8_t* pixels, int64_t stride,
                        uint8_t alive_value) {
    if (stride < W) return -1;
    for (int64_t y = 0; y < H; y++)
        for (int64_t x = 0; x < W; x++) pixels[x + y * stride] = cells[x + y * W] ? alive_value : 0;
    return 0;
}

/* ------------------------------------------------------------------ RLE patterns */
/* Standard Life RLE: '#' comment lines, optional "x = .., y = .." header, tokens
 * [count](b|o|$) and '!' terminator; any letter other than 'b' is alive.  Cells are
 * placed at (x0 + dx, y0 + dy), wrapped modulo the board (torus placement). */
int oracle_place_rle(uint8_t* cells, int64_t W, int64_t H, const char* rle, int64_t x0, int64_t y0) {
    const char* p = rle;
    /* skip comment/header lines */
    for (;;) {
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') p++;
        if (*p == '#' || *p == 'x') {
            while (*p && *p != '\n') p++;
            continue;
        }
        break;
    }
    int64_t dx = 0, dy = 0, count = 0;
    for (; *p && *p != '!'; p++) {
        char c = *p;
        if (c >= '0' && c <= '9') {
            count = count * 10 + (c - '0');
            continue;
        }
        if (c == ' ' || c == '\t' || c == '\r' || c == '\n') continue;
        int64_t n = count ? count : 1;
        count = 0;
        if (c == '$') {
            dy += n;
            dx = 0;
        } else if (c == 'b' || c == '.') {
            dx += n;
        } else if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) {
            for (int64_t i = 0; i < n; i++) {
                int64_t x = ((x0 + dx + i) % W + W) % W, y = ((y0 + dy) % H + H) % H;
                cells[x + y * W] = 1;
            }
            dx += n;
        } else {
            return -1;
        }
    }
    return 0;
}
