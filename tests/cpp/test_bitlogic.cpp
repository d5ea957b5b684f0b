// Host check of the product's bit-sliced rule (gameoflifewithactors_amd/csrc/gol_bitlogic.h)
// against the reference rule (GameOfLifeLogic.fs:59-63) over every 3x3 neighbourhood and over
// random 3-row x 3-word windows.  Built and run by tests/test_bitlogic.py (CPU).
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
#include "../../gameoflifewithactors_amd/csrc/gol_bitlogic.h"
#include "../../gameoflifewithactors_amd/csrc/gol_layout.h"

static int rule(int a, int alive) { return (a > 3 || a < 2) ? 0 : (a == 3 ? 1 : alive); }

static int cell(const uint32_t* row, int x) {  // row of 3 words, x in [-32, 64)
    int w = 1 + (x >> 5);
    return (row[w] >> (x & 31)) & 1;
}

template <int M>
static int check_blocks() {
    int bad = 0;
    const int n = 3 * 32 * M;  // cells per row: blocks prev | mid | next
    for (int it = 0; it < 20000; it++) {
        static unsigned char cells[3][3 * 32 * 4];
        for (int r = 0; r < 3; r++)
            for (int x = 0; x < n; x++) cells[r][x] = (rand() >> 7) & 1;
        uint32_t words[3][3][M];  // [row][block][word]
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++)
                for (int j = 0; j < M; j++) {
                    uint32_t v = 0;
                    for (int b = 0; b < 32; b++) v |= (uint32_t)cells[r][gol::word_bit_cell(k * M + j, b, M)] << b;
                    words[r][k][j] = v;
                }
        uint32_t s[3][M], c[3][M];
        for (int r = 0; r < 3; r++) gol::row_sum_block<M>(words[r][1], words[r][0][M - 1], words[r][2][0], s[r], c[r]);
        for (int j = 0; j < M; j++) {
            const uint32_t nx = gol::life_next(s[0][j], c[0][j], s[1][j], c[1][j], s[2][j], c[2][j], words[1][1][j]);
            for (int b = 0; b < 32; b++) {
                const int64_t x = gol::word_bit_cell(M + j, b, M);  // a cell of the middle block
                int a = 0;
                for (int dy = 0; dy < 3; dy++)
                    for (int dx = -1; dx <= 1; dx++)
                        if (dy != 1 || dx != 0) a += cells[dy][x + dx];
                if ((int)((nx >> b) & 1) != rule(a, cells[1][x])) bad++;
            }
        }
    }
    return bad;
}

int main() {
    int bad = 0;
    // exhaustive: neighbourhood n (9 bits) placed around bit position p of the centre word
    for (int p = 0; p < 32; p++)
        for (int n = 0; n < 512; n++) {
            uint32_t rows[3][3] = {{0}};
            for (int k = 0; k < 9; k++)
                if ((n >> k) & 1) {
                    int dy = k / 3, dx = k % 3 - 1, x = p + dx;
                    int w = 1 + (x < 0 ? -1 : (x >= 32 ? 1 : 0));
                    rows[dy][w] |= 1u << ((x + 32) & 31);
                }
            uint32_t s[3], c[3];
            for (int r = 0; r < 3; r++) gol::row_sum(rows[r][0], rows[r][1], rows[r][2], s[r], c[r]);
            uint32_t nx = gol::life_next(s[0], c[0], s[1], c[1], s[2], c[2], rows[1][1]);
            int a = __builtin_popcount(n) - ((n >> 4) & 1);
            int want = rule(a, (n >> 4) & 1);
            if ((int)((nx >> p) & 1) != want) bad++;
        }
    // random windows: all 32 output bits at once
    srand(12345);
    for (int it = 0; it < 200000; it++) {
        uint32_t rows[3][3];
        for (int r = 0; r < 3; r++)
            for (int w = 0; w < 3; w++) rows[r][w] = ((uint32_t)rand() << 16) ^ (uint32_t)rand();
        uint32_t s[3], c[3];
        for (int r = 0; r < 3; r++) gol::row_sum(rows[r][0], rows[r][1], rows[r][2], s[r], c[r]);
        uint32_t nx = gol::life_next(s[0], c[0], s[1], c[1], s[2], c[2], rows[1][1]);
        for (int x = 0; x < 32; x++) {
            int a = 0;
            for (int dy = 0; dy < 3; dy++)
                for (int dx = -1; dx <= 1; dx++)
                    if (dy != 1 || dx != 0) a += cell(rows[dy], x + dx);
            if ((int)((nx >> x) & 1) != rule(a, cell(rows[1], x))) bad++;
        }
    }
    // interleaved blocks (gol_layout.h): three rows of three blocks, cells -> words, row_sum_block on
    // the middle block of each row, life_next, compared cell by cell with the reference rule
    bad += check_blocks<1>() + check_blocks<2>() + check_blocks<4>();
    // layout helpers are inverse bijections
    for (int ilv : {1, 2, 4})
        for (int64_t x = 0; x < 512; x++) {
            int64_t w;
            int b;
            gol::cell_pos(x, ilv, w, b);
            if (gol::word_bit_cell(w, b, ilv) != x || b < 0 || b > 31 || w != (x / (32 * ilv)) * ilv + (x % ilv)) bad++;
        }
    std::printf("{\"mismatches\": %d}\n", bad);
    return bad != 0;
}
