// pair_search.c -- exhaustive search for a cheaper bit-sliced B3/S23 vertical stage that shares work between
// the two output rows a streaming trip produces together (gol_step.hip processes rows in pairs).
//
// Per output row y the current stage (gol_bitlogic.h life_next) takes the three horizontal row sums
// h = s + 2c (rows y-1, y, y+1) and the centre word, 7 LUT3 ops.  Output y+1 uses rows y, y+1, y+2.  An
// ENCODER computes a code of the shared pair sum P = h_y + h_{y+1} once (g_e gates), and each output
// then evaluates F(code, s_o, c_o, centre) (g_f gates), total g_e + 2 g_f per pair against 14.
//
// Domain of F: code value (3 bits) x h_o (2 bits) x centre (1 bit) = 64 points (one u64 truth table);
// the target is (T == 3) | (T == 4 & centre), T = P + h_o, and points no input reaches are don't-cares.
// The centre of output y is a cell of row y, that of output y+1 a cell of row y+1: h of that row is then
// W + centre + E, so centre = 0 excludes h = 3 and centre = 1 excludes h = 0 (separate care sets).
//
// Build: gcc -O3 -march=native -fopenmp pair_search.c -o pair_search
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;

static inline u64 lut_apply(unsigned L, u64 a, u64 b, u64 c) {
    u64 r = 0;
    for (int i = 0; i < 8; i++)
        if ((L >> i) & 1) r |= ((i & 1) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 4) ? c : ~c);
    return r;
}

// F-domain variables, point p = code | h_o << 3 | centre << 5
static u64 var[6];
static void init_vars(void) {
    for (int v = 0; v < 6; v++) {
        var[v] = 0;
        for (int p = 0; p < 64; p++)
            if ((p >> v) & 1) var[v] |= 1ull << p;
    }
}

// can f (on care) be written as a LUT of (x, y, z)?
static inline int consistent(u64 f, u64 care, u64 x, u64 y, u64 z) {
    for (int m = 0; m < 8; m++) {
        const u64 sel = care & ((m & 1) ? x : ~x) & ((m & 2) ? y : ~y) & ((m & 4) ? z : ~z);
        if ((f & sel) && (~f & sel)) return 0;
    }
    return 1;
}

// minimum LUT3 gates (<= 3, else 4 = "more") for f on care over the 6 variables
static int min_gates(u64 f, u64 care, char* how) {
    u64 sig[9];
    for (int v = 0; v < 6; v++) sig[v] = var[v];
    // 1 gate
    for (int a = 0; a < 6; a++)
        for (int b = a + 1; b < 6; b++)
            for (int c = b + 1; c < 6; c++)
                if (consistent(f, care, sig[a], sig[b], sig[c])) {
                    sprintf(how, "1:(%d,%d,%d)", a, b, c);
                    return 1;
                }
    // 2 gates: g1 over 3 vars, final over 3 of (6 vars + g1) including g1
    for (int a = 0; a < 6; a++)
        for (int b = a + 1; b < 6; b++)
            for (int c = b + 1; c < 6; c++)
                for (unsigned L = 0; L < 256; L++) {
                    const u64 g = lut_apply(L, sig[a], sig[b], sig[c]);
                    for (int d = 0; d < 6; d++)
                        for (int e = d + 1; e < 6; e++)
                            if (consistent(f, care, g, sig[d], sig[e])) {
                                sprintf(how, "2:g1=L%02x(%d,%d,%d) out(g1,%d,%d)", L, a, b, c, d, e);
                                return 2;
                            }
                }
    // 3 gates: g1 over 3 vars; g2 over 3 of (vars + g1); final over 3 of (vars, g1, g2) including g2
    for (int a = 0; a < 6; a++)
        for (int b = a + 1; b < 6; b++)
            for (int c = b + 1; c < 6; c++)
                for (unsigned L1 = 0; L1 < 256; L1++) {
                    sig[6] = lut_apply(L1, sig[a], sig[b], sig[c]);
                    for (int d = 0; d < 7; d++)
                        for (int e = d + 1; e < 7; e++)
                            for (int g = e + 1; g < 7; g++)
                                for (unsigned L2 = 0; L2 < 256; L2++) {
                                    sig[7] = lut_apply(L2, sig[d], sig[e], sig[g]);
                                    for (int x = 0; x < 7; x++)
                                        for (int y = x + 1; y < 7; y++) {
                                            // g1 must be used by g2 or the final gate
                                            if (!(d == 6 || e == 6 || g == 6 || x == 6 || y == 6)) continue;
                                            if (consistent(f, care, sig[7], sig[x], sig[y])) {
                                                sprintf(how, "3:g1=L%02x(%d,%d,%d) g2=L%02x(%d,%d,%d) out(g2,%d,%d)", L1, a,
                                                        b, c, L2, d, e, g, x, y);
                                                return 3;
                                            }
                                        }
                                }
                }
    return 4;
}

// ---- encoders over the 16 pair points q = s_y | c_y << 1 | s_n << 2 | c_n << 3 ----
static int hq(int q, int row) { return row == 0 ? ((q & 1) + 2 * ((q >> 1) & 1)) : (((q >> 2) & 1) + 2 * ((q >> 3) & 1)); }

// F target and care for a code map; returns 0 on conflict (code does not determine the class of P)
static int build_f(const uint16_t tt[3], int centre_row, u64* f, u64* care) {
    int cls[8];
    for (int i = 0; i < 8; i++) cls[i] = -1;
    *f = 0;
    *care = 0;
    for (int q = 0; q < 16; q++) {
        int code = 0;
        for (int b = 0; b < 3; b++) code |= ((tt[b] >> q) & 1) << b;
        int P = hq(q, 0) + hq(q, 1);
        int cl = P > 5 ? 5 : P;
        if (cls[code] >= 0 && cls[code] != cl) return 0;
        cls[code] = cl;
        const int hc = hq(q, centre_row);
        for (int ho = 0; ho < 4; ho++)
            for (int cy = 0; cy < 2; cy++) {
                if (cy == 0 && hc == 3) continue;
                if (cy == 1 && hc == 0) continue;
                const int T = P + ho;
                const int alive = T == 3 || (T == 4 && cy);
                const int p = code | ho << 3 | cy << 5;
                *care |= 1ull << p;
                if (alive) *f |= 1ull << p;
            }
    }
    return 1;
}

#define MAXTT 70000
int main(int argc, char** argv) {
    init_vars();
    const int only_natural = argc > 1 && !strcmp(argv[1], "natural");
    // signals over the 16 pair points
    uint16_t x[4];
    for (int v = 0; v < 4; v++) {
        x[v] = 0;
        for (int q = 0; q < 16; q++)
            if ((q >> v) & 1) x[v] |= 1u << q;
    }
    if (only_natural) {
        // the 4-gate binary encoder: p0 = s_y ^ s_n, k = s_y & s_n, q1 = xor3(k, c_y, c_n), q2 = maj(k, c_y, c_n)
        uint16_t k = x[0] & x[2];
        uint16_t tt[3] = {(uint16_t)(x[0] ^ x[2]), (uint16_t)(k ^ x[1] ^ x[3]),
                          (uint16_t)((k & x[1]) | (k & x[3]) | (x[1] & x[3]))};
        for (int row = 0; row < 2; row++) {
            u64 f, care;
            char how[256];
            build_f(tt, row, &f, &care);
            int g = min_gates(f, care, how);
            printf("natural encoder, centre in row %d: F needs %d gates %s\n", row, g, g <= 3 ? how : "");
        }
        return 0;
    }
    // enumerate encoders of 3 gates (each a LUT3 over the 4 inputs and earlier gates); dedupe by the set of
    // truth tables, keep those whose 3 outputs determine the class of P
    static uint16_t single[MAXTT];
    int ns = 0;
    static unsigned char seen[65536];
    memset(seen, 0, sizeof seen);
    for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++)
            for (int c = b + 1; c < 4; c++)
                for (unsigned L = 0; L < 256; L++) {
                    uint16_t t = (uint16_t)lut_apply(L, x[a], x[b], x[c]);
                    if (!seen[t]) {
                        seen[t] = 1;
                        single[ns++] = t;
                    }
                }
    fprintf(stderr, "distinct one-gate functions: %d\n", ns);
    // encoders: g1 in single; g2 over (x, g1); g3 over (x, g1, g2)
    long tried = 0, valid = 0;
    int best_total = 99;
    // cache of F results per normalized f/care
    for (int i1 = 0; i1 < ns; i1++) {
        uint16_t s5[6];
        memcpy(s5, x, sizeof x);
        s5[4] = single[i1];
        for (int a = 0; a < 5; a++)
            for (int b = a + 1; b < 5; b++)
                for (int c = b + 1; c < 5; c++) {
                    if (c != 4) continue;  // g2 uses g1 (else g2 is another single; covered by ordering below)
                    for (unsigned L2 = 0; L2 < 256; L2++) {
                        uint16_t g2 = (uint16_t)lut_apply(L2, s5[a], s5[b], s5[c]);
                        s5[5] = g2;
                        for (int d = 0; d < 6; d++)
                            for (int e = d + 1; e < 6; e++)
                                for (int g = e + 1; g < 6; g++)
                                    for (unsigned L3 = 0; L3 < 256; L3++) {
                                        uint16_t g3 = (uint16_t)lut_apply(L3, s5[d], s5[e], s5[g]);
                                        uint16_t tt[3] = {s5[4], g2, g3};
                                        u64 f0, c0, f1, c1;
                                        tried++;
                                        if (!build_f(tt, 0, &f0, &c0)) continue;
                                        build_f(tt, 1, &f1, &c1);
                                        valid++;
                                        (void)f1;
                                        (void)c1;
                                        if (valid % 100000 == 1) fprintf(stderr, "valid %ld of %ld\n", valid, tried);
                                    }
                    }
                }
    }
    printf("tried %ld encoders (g2 uses g1), %ld determine the class of P; best %d\n", tried, valid, best_total);
    return 0;
}
