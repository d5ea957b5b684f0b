// gol_bitlogic.h -- bit-sliced B3/S23 for 32 cells per 32-bit word (host + gfx950 device).
//
// Replaces, for 32 cells at once, the per-cell neighbour gather and rule of the reference actor:
//   GameOfLife/GameOfLife/GameOfLifeLogic.fs:56-63  (Akka: GameOfLifeAkka/GameofLife.fs:105-112)
//   a = #alive among 8 neighbours;  a > 3 || a < 2 -> dead;  a = 3 -> alive;  otherwise keep isAlive.
//
// Packing: bit b of word w in row y is cell (x = 32*w + b, y); LSB = smallest x (matches the
// reference's pixels[x + y*size] orientation, GameOfLifeUI.fs:27).
//
// Arithmetic (13 VALU ops per word per generation on gfx950, 2 of them DPP moves done by the caller):
//   row sum   W + C + E of one row as a 2-bit number (s, c): 2 x v_alignbit_b32 + 2 x v_bitop3_b32
//             (xor3 = LUT 0x96, majority = LUT 0xE8)
//   vertical  t = sP + sC + sN + 2 (cP + cC + cN) is the 9-cell sum including the centre; the rule is
//             next = (t == 3) | (alive & t == 4).  A = xor3(s), B = maj3(s), X = xor3(c), Y = maj3(c)
//             then a 3-LUT tree found by exhaustive search (tests/cpp/test_bitlogic.cpp re-checks all 2^9
//             neighbourhoods):  o1 = L(A, Y, alive; 0x27), o2 = L(B, X, Y; 0x19), next = L(o1, o2, A; 0x24).
//
// LUT convention used in this file: lut3(a, b, c, L) = bit (a | b<<1 | c<<2) of L.  gfx950's
// v_bitop3_b32 indexes its immediate with (S0<<2 | S1<<1 | S2), so a -> S2 and c -> S0.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GOL_HD __host__ __device__ __forceinline__
#else
#define GOL_HD static inline
#endif

namespace gol {

template <unsigned L>
GOL_HD uint32_t lut3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(c, b, a, L);
#else
    uint32_t r = 0;
    for (unsigned i = 0; i < 8; i++)
        if ((L >> i) & 1u) r |= ((i & 1u) ? a : ~a) & ((i & 2u) ? b : ~b) & ((i & 4u) ? c : ~c);
    return r;
#endif
}
GOL_HD uint32_t align_right(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

// Horizontal 3-sum of one row around each of 32 cells: (prev word, this word, next word) -> (s, c).
GOL_HD void row_sum(uint32_t prev, uint32_t cur, uint32_t next, uint32_t& s, uint32_t& c) {
    const uint32_t w = align_right(cur, prev, 31);  // west neighbour of every cell
    const uint32_t e = align_right(next, cur, 1);   // east neighbour of every cell
    s = lut3<0x96>(w, cur, e);
    c = lut3<0xE8>(w, cur, e);
}

// Horizontal 3-sums of one block of M interleaved words (gol_layout.h: word j bit b = cell j + M*b).
// West of word j is word j-1 at the same bit, except word 0 whose west is word M-1 one bit lower (the
// bit below bit 0 comes from the previous block's word M-1, `prev_last`); symmetrically for east.
// So a block costs 2 funnel shifts whatever M is (M = 1 reduces to row_sum above).
template <int M>
GOL_HD void row_sum_block(const uint32_t (&r)[M], uint32_t prev_last, uint32_t next_first, uint32_t (&s)[M],
                          uint32_t (&c)[M]) {
    const uint32_t w0 = align_right(r[M - 1], prev_last, 31);
    const uint32_t eN = align_right(next_first, r[0], 1);
#pragma unroll
    for (int j = 0; j < M; j++) {
        const uint32_t w = j == 0 ? w0 : r[j - 1];
        const uint32_t e = j == M - 1 ? eN : r[j + 1];
        s[j] = lut3<0x96>(w, r[j], e);
        c[j] = lut3<0xE8>(w, r[j], e);
    }
}

// Next state of 32 cells from the three row sums (previous, centre, next row) and the centre word.
GOL_HD uint32_t life_next(uint32_t sP, uint32_t cP, uint32_t sC, uint32_t cC, uint32_t sN, uint32_t cN,
                          uint32_t alive) {
    const uint32_t A = lut3<0x96>(sP, sC, sN);
    const uint32_t B = lut3<0xE8>(sP, sC, sN);
    const uint32_t X = lut3<0x96>(cP, cC, cN);
    const uint32_t Y = lut3<0xE8>(cP, cC, cN);
    const uint32_t o1 = lut3<0x27>(A, Y, alive);
    const uint32_t o2 = lut3<0x19>(B, X, Y);
    return lut3<0x24>(o1, o2, A);
}

}  // namespace gol
