// gol_layout.h -- bit-packed row layouts shared by the kernels and the host code.
//
// A board row of W cells is stored as W/32 little-endian 32-bit words.  Rows are grouped into blocks of
// M words (M = "ilv", 1, 2 or 4; 32*M cells per block).  Inside block k, word j (0 <= j < M) bit b holds
//
//       cell x = 32*M*k + j + M*b
//
// M = 1 is the plain layout (bit b of word w = cell 32w + b, as in GameOfLifeUI.fs:27's x order).  With
// M > 1 the horizontal neighbours of a cell sit at the SAME bit of the neighbouring word of its block
// (only words 0 and M-1 need a one-bit funnel shift across the block edge), which removes most of the
// half-rate shifts from the step kernel (DESIGN.md "Interleaved blocks").
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GOL_LAYOUT_HD __host__ __device__ __forceinline__
#else
#define GOL_LAYOUT_HD static inline
#endif

namespace gol {

GOL_LAYOUT_HD int ilv_shift(int ilv) { return ilv == 4 ? 2 : (ilv == 2 ? 1 : 0); }

// cell x of a row -> (stored word index within the row, bit)
GOL_LAYOUT_HD void cell_pos(int64_t x, int ilv, int64_t& word, int& bit) {
    const int sh = ilv_shift(ilv);
    const int64_t blk = x >> (5 + sh);
    const int o = (int)(x & ((32 << sh) - 1));
    word = (blk << sh) + (o & (ilv - 1));
    bit = o >> sh;
}

// stored word w (within the row), bit b -> cell x
GOL_LAYOUT_HD int64_t word_bit_cell(int64_t w, int b, int ilv) {
    const int sh = ilv_shift(ilv);
    return ((w >> sh) << (5 + sh)) + (w & (ilv - 1)) + ((int64_t)b << sh);
}

}  // namespace gol
