// pair_search2.c -- stage 1: enumerate every 3-gate encoder (LUT3 gates over s_y, c_y, s_n, c_n and earlier
// gates) whose three outputs determine the class of P = h_y + h_n (0..4, >= 5); canonicalise the induced
// F problem (code -> class map, per code the centre values reachable with the centre in row y / row n)
// under the 48 permutations / complements of the code bits; print the distinct keys with one encoder each.
// Stage 2 (pair_f.c) searches the per-output function F of each key.
//
// Build: gcc -O3 -march=native -fopenmp pair_search2.c -o pair_search2
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int hq(int q, int row) { return row == 0 ? ((q & 1) + 2 * ((q >> 1) & 1)) : (((q >> 2) & 1) + 2 * ((q >> 3) & 1)); }
static int cls_of(int q) {
    int P = hq(q, 0) + hq(q, 1);
    return P > 5 ? 5 : P;
}

static void lut_table(uint16_t a, uint16_t b, uint16_t c, uint16_t out[256]) {
    uint16_t m[8];
    for (int i = 0; i < 8; i++) m[i] = ((i & 1) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 4) ? c : ~c);
    out[0] = 0;
    for (int L = 1; L < 256; L++) out[L] = out[L & (L - 1)] | m[__builtin_ctz(L)];
}

// key: per code value v (0..7): class (0..5, 7 = unreached) | reach_y << 3 | reach_n << 5  (8 bits)
typedef struct {
    uint8_t k[8];
} Key;

static int key_of(const uint16_t t[3], Key* out) {
    int cls[8], ry[8], rn[8];
    for (int v = 0; v < 8; v++) cls[v] = 7, ry[v] = rn[v] = 0;
    for (int q = 0; q < 16; q++) {
        int v = ((t[0] >> q) & 1) | ((t[1] >> q) & 1) << 1 | ((t[2] >> q) & 1) << 2;
        int c = cls_of(q);
        if (cls[v] != 7 && cls[v] != c) return 0;
        cls[v] = c;
        int hy = hq(q, 0), hn = hq(q, 1);
        if (hy != 3) ry[v] |= 1;  // centre 0 possible
        if (hy != 0) ry[v] |= 2;  // centre 1 possible
        if (hn != 3) rn[v] |= 1;
        if (hn != 0) rn[v] |= 2;
    }
    // canonical: minimum over 48 transforms of the 8-byte key
    Key best;
    memset(&best, 0xff, sizeof best);
    static const int perms[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
    for (int p = 0; p < 6; p++)
        for (int cm = 0; cm < 8; cm++) {
            Key k;
            for (int v = 0; v < 8; v++) {
                // new code w: bit j of w = bit perms[p][j] of v, xor cm
                int w = 0;
                for (int j = 0; j < 3; j++) w |= ((v >> perms[p][j]) & 1) << j;
                w ^= cm;
                k.k[w] = (uint8_t)(cls[v] | ry[v] << 3 | rn[v] << 5);
            }
            if (memcmp(&k, &best, sizeof k) < 0) best = k;
        }
    *out = best;
    return 1;
}

// open-addressing hash set of keys
#define HBITS 24
static uint64_t* hset;
static uint64_t* henc;  // one encoder per key: g1 | g2 << 16 | g3 << 32
static long nkeys = 0;
static int hinsert(uint64_t key, uint64_t enc) {
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    size_t i = h >> (64 - HBITS);
    const size_t mask = ((size_t)1 << HBITS) - 1;
    for (;;) {
        if (hset[i] == 0) {
            hset[i] = key;
            henc[i] = enc;
            nkeys++;
            return 1;
        }
        if (hset[i] == key) return 0;
        i = (i + 1) & mask;
    }
}

static uint64_t sepA[65536], sepB[65536];
static uint64_t allA, allB;
static void init_sep(void) {
    int n = 0;
    int pp[128], qq[128];
    for (int p = 0; p < 16; p++)
        for (int q = p + 1; q < 16; q++)
            if (cls_of(p) != cls_of(q)) pp[n] = p, qq[n] = q, n++;
    allA = allB = 0;
    for (int i = 0; i < n; i++) {
        if (i < 64) allA |= 1ull << i; else allB |= 1ull << (i - 64);
    }
    for (int t = 0; t < 65536; t++) {
        uint64_t a = 0, b = 0;
        for (int i = 0; i < n; i++)
            if (((t >> pp[i]) & 1) != ((t >> qq[i]) & 1)) {
                if (i < 64) a |= 1ull << i; else b |= 1ull << (i - 64);
            }
        sepA[t] = a, sepB[t] = b;
    }
    fprintf(stderr, "different-class pairs: %d\n", n);
}

int main(void) {
    init_sep();
    hset = calloc((size_t)1 << HBITS, 8);
    henc = calloc((size_t)1 << HBITS, 8);
    uint16_t x[4];
    for (int v = 0; v < 4; v++) {
        x[v] = 0;
        for (int q = 0; q < 16; q++)
            if ((q >> v) & 1) x[v] |= 1u << q;
    }
    // distinct one-gate functions
    static uint16_t single[1024];
    int ns = 0;
    static unsigned char seen[65536];
    for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++)
            for (int c = b + 1; c < 4; c++) {
                uint16_t tab[256];
                lut_table(x[a], x[b], x[c], tab);
                for (int L = 0; L < 256; L++)
                    if (!seen[tab[L]]) seen[tab[L]] = 1, single[ns++] = tab[L];
            }
    fprintf(stderr, "one-gate functions: %d\n", ns);
    long valid = 0;
    for (int i1 = 0; i1 < ns; i1++) {
        uint16_t s[6];
        memcpy(s, x, sizeof x);
        s[4] = single[i1];
        // g2: over any 3 of the 5 signals (it need not use g1)
        for (int a = 0; a < 5; a++)
            for (int b = a + 1; b < 5; b++)
                for (int c = b + 1; c < 5; c++) {
                    uint16_t t2[256];
                    lut_table(s[a], s[b], s[c], t2);
                    for (int L2 = 0; L2 < 256; L2++) {
                        s[5] = t2[L2];
                        const uint64_t A12 = sepA[s[4]] | sepA[s[5]], B12 = sepB[s[4]] | sepB[s[5]];
                        for (int d = 0; d < 6; d++)
                            for (int e = d + 1; e < 6; e++)
                                for (int f = e + 1; f < 6; f++) {
                                    uint16_t t3[256];
                                    lut_table(s[d], s[e], s[f], t3);
                                    for (int L3 = 0; L3 < 256; L3++) {
                                        if ((A12 | sepA[t3[L3]]) != allA || (B12 | sepB[t3[L3]]) != allB) continue;
                                        uint16_t t[3] = {s[4], s[5], t3[L3]};
                                        Key k;
                                        if (!key_of(t, &k)) continue;
                                        valid++;
                                        uint64_t kk;
                                        memcpy(&kk, &k, 8);
                                        hinsert(kk, (uint64_t)t[0] | (uint64_t)t[1] << 16 | (uint64_t)t[2] << 32);
                                    }
                                }
                    }
                }
        if (i1 % 50 == 0) fprintf(stderr, "g1 %d/%d valid %ld keys %ld\n", i1, ns, valid, nkeys);
    }
    fprintf(stderr, "valid encoders %ld, distinct keys %ld\n", valid, nkeys);
    for (size_t i = 0; i < ((size_t)1 << HBITS); i++)
        if (hset[i]) printf("%016llx %012llx\n", (unsigned long long)hset[i], (unsigned long long)henc[i]);
    return 0;
}
