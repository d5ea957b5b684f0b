// gol_wave.hip -- single-wave, register-resident pass for the reference-size boards (gfx950).
//
// The reference's own board is 100 x 100 (GameOfLifeLogic.fs:5, GameofLife.fs:18): 10^4 cells, a width that is
// not a multiple of 32.  On such a board every other path is latency-bound: the byte step is one launch per
// generation, the LDS-resident pass (gol_resident.hip) pays a workgroup barrier and LDS round trips per
// generation.  Here ONE wavefront holds the whole board in VGPRs, bit-packed with a masked last word:
//
//   lane L holds rows L*RPL .. L*RPL + RPL-1 (RPL = rows per lane, H % RPL == 0, H / RPL <= 64 lanes),
//   each as NW = ceil(W / 32) words, bit b of word j = cell 32 j + b, bits >= W zero.
//
// A generation is the synchronous B3/S23 step (GameOfLifeLogic.fs:59-63 under the Reset->State barrier)
// with no barrier and no memory traffic at all: horizontal neighbours by funnel shifts inside the lane, with
// the x-wrap fix-up at the ragged row end (torus, GameOfLifeDriver.fs:21-25; dead outside when bounded,
// Script.fsx:6-13); the row sums of the rows above a lane's first row and below its last row come from the
// neighbouring lanes by ds_bpermute (wrapping from the last active lane to lane 0 on a torus); the rule is
// the streaming kernel's LUT tree (gol_bitlogic.h).  The board is read once and written once per call, from
// and to the board's own storage: bytes (ragged widths, one byte per cell) or packed ilv-1 words.
#include "gol_internal.h"
#include "gol_bitlogic.h"

namespace gol {
namespace {

__device__ __forceinline__ uint32_t bperm(int byte_addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(byte_addr, (int)v);
}

// Horizontal 3-sums of one ragged row (NW words, last word holding bits [0, lb]).
template <int NW, bool BOUNDED>
__device__ __forceinline__ void ragged_row_sum(const uint32_t (&w)[NW], int lb, uint32_t lbbit, uint32_t (&s)[NW],
                                               uint32_t (&c)[NW]) {
    // west neighbour of cell 0 is cell W-1 (bit lb of the last word), moved to bit 31 of a carry word
    const uint32_t wcarry = BOUNDED ? 0u : w[NW - 1] << (31 - lb);
    uint32_t west[NW], east[NW];
#pragma unroll
    for (int j = 0; j < NW; j++) west[j] = align_right(w[j], j == 0 ? wcarry : w[j - 1], 31);
#pragma unroll
    for (int j = 0; j + 1 < NW; j++) east[j] = align_right(w[j + 1], w[j], 1);
    // east neighbour of cell W-1 is cell 0: bit 0 of word 0 into bit lb of the last word
    if (BOUNDED)
        east[NW - 1] = w[NW - 1] >> 1;
    else
        east[NW - 1] = lut3<0xEA>(w[NW - 1] >> 1, w[0] << lb, lbbit);  // a | (b & c)
#pragma unroll
    for (int j = 0; j < NW; j++) {
        s[j] = lut3<0x96>(west[j], w[j], east[j]);
        c[j] = lut3<0xE8>(west[j], w[j], east[j]);
    }
}

template <int NW, int RPL, bool BOUNDED, bool BYTES>
__global__ __launch_bounds__(64) void gol_wave_resident(const void* __restrict__ src, void* __restrict__ dst, int W,
                                                        int H, int64_t pitch, int gens) {
    const int lane = threadIdx.x;
    const int nl = H / RPL;  // active lanes
    const bool active = lane < nl;
    const int lb = (W - 1) & 31;
    const uint32_t lbbit = 1u << lb;
    const uint32_t lastmask = lb == 31 ? 0xffffffffu : (lbbit << 1) - 1u;
    uint32_t w[RPL][NW];

    // ---- load the board: byte boards row by row, 64 cells per wave-wide coalesced load, packed by ballot (the
    // 64-bit lane mask is the next two words of the row) into the lane that owns the row; packed boards one word
    // load per owned word
#pragma unroll
    for (int i = 0; i < RPL; i++)
#pragma unroll
        for (int j = 0; j < NW; j++) w[i][j] = 0;
    if (BYTES) {
        // kBatch owner lanes' rows per round: all their loads are issued before the first ballot, so a round
        // waits for memory once (one load, one wait, one ballot per 64 cells cost a memory round trip each:
        // ~30 us of a 100-generation call on the reference's 100^2 board)
        constexpr int kBatch = 8;
        constexpr int kChunks = (NW + 1) / 2;
        const uint8_t* cells = static_cast<const uint8_t*>(src);
        for (int L0 = 0; L0 < nl; L0 += kBatch) {
            uint8_t v[kBatch][RPL][kChunks];
#pragma unroll
            for (int b = 0; b < kBatch; b++)
#pragma unroll
                for (int i = 0; i < RPL; i++)
#pragma unroll
                    for (int c = 0; c < kChunks; c++) {
                        // unconditional loads (address clamped into the board, value masked): a branch per load
                        // would make the compiler wait for each
                        // (owner lanes past the last active lane load a clamped row and keep garbage: no active
                        // lane reads them, and they are never stored)
                        const int x = 64 * c + lane;
                        const int L = L0 + b < nl ? L0 + b : nl - 1;
                        const uint8_t t = cells[(int64_t)(L * RPL + i) * W + (x < W ? x : W - 1)];
                        v[b][i][c] = x < W ? t : (uint8_t)0;
                    }
#pragma unroll
            for (int b = 0; b < kBatch; b++)
#pragma unroll
                for (int i = 0; i < RPL; i++)
#pragma unroll
                    for (int c = 0; c < kChunks; c++) {
                        const uint64_t m = __ballot(v[b][i][c] != 0);
                        if (lane == L0 + b) {
                            w[i][2 * c] = (uint32_t)m;
                            if (2 * c + 1 < NW) w[i][2 * c + 1] = (uint32_t)(m >> 32);
                        }
                    }
        }
    } else if (active) {
#pragma unroll
        for (int i = 0; i < RPL; i++)
#pragma unroll
            for (int j = 0; j < NW; j++)
                w[i][j] = static_cast<const uint32_t*>(src)[(int64_t)(lane * RPL + i) * pitch + j];
    }
    // lanes the rows above the first row / below the last row come from (ds_bpermute byte addresses)
    const int up_lane = lane == 0 ? nl - 1 : lane - 1;
    const int dn_lane = lane + 1 >= nl ? 0 : lane + 1;
    const int up_addr = up_lane * 4, dn_addr = dn_lane * 4;
    const uint32_t up_mask = (BOUNDED && lane == 0) ? 0u : 0xffffffffu;  // dead rows outside a bounded board
    const uint32_t dn_mask = (BOUNDED && lane == nl - 1) ? 0u : 0xffffffffu;

    for (int g = 0; g < gens; g++) {
        uint32_t s[RPL][NW], c[RPL][NW];
#pragma unroll
        for (int i = 0; i < RPL; i++) ragged_row_sum<NW, BOUNDED>(w[i], lb, lbbit, s[i], c[i]);
        uint32_t us[NW], uc[NW], ds[NW], dc[NW];
#pragma unroll
        for (int j = 0; j < NW; j++) {
            us[j] = bperm(up_addr, s[RPL - 1][j]) & up_mask;
            uc[j] = bperm(up_addr, c[RPL - 1][j]) & up_mask;
            ds[j] = bperm(dn_addr, s[0][j]) & dn_mask;
            dc[j] = bperm(dn_addr, c[0][j]) & dn_mask;
        }
#pragma unroll
        for (int i = 0; i < RPL; i++)
#pragma unroll
            for (int j = 0; j < NW; j++) {
                const uint32_t sP = i == 0 ? us[j] : s[i - 1][j], cP = i == 0 ? uc[j] : c[i - 1][j];
                const uint32_t sN = i == RPL - 1 ? ds[j] : s[i + 1][j], cN = i == RPL - 1 ? dc[j] : c[i + 1][j];
                uint32_t v = life_next(sP, cP, s[i][j], c[i][j], sN, cN, w[i][j]);
                if (j == NW - 1) v &= lastmask;
                w[i][j] = v;
            }
    }

    // ---- store: byte boards row by row, each lane writing one cell of a 64-cell run (the owner lane's two
    // words read as scalars), packed boards one word store per owned word
    if (BYTES) {
        uint8_t* cells = static_cast<uint8_t*>(dst);
        for (int L = 0; L < nl; L++) {
#pragma unroll
            for (int i = 0; i < RPL; i++) {
                uint8_t* row = cells + (int64_t)(L * RPL + i) * W;
#pragma unroll
                for (int c = 0; c < (NW + 1) / 2; c++) {
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)w[i][2 * c], L);
                    const uint32_t hi =
                        2 * c + 1 < NW ? (uint32_t)__builtin_amdgcn_readlane((int)w[i][2 * c + 1], L) : 0u;
                    const int x = 64 * c + lane;
                    const uint32_t word = lane < 32 ? lo : hi;
                    if (x < W) row[x] = (uint8_t)((word >> (lane & 31)) & 1u);
                }
            }
        }
        return;
    }
    if (!active) return;
#pragma unroll
    for (int i = 0; i < RPL; i++)
#pragma unroll
        for (int j = 0; j < NW; j++) static_cast<uint32_t*>(dst)[(int64_t)(lane * RPL + i) * pitch + j] = w[i][j];
}

template <int NW, int RPL>
hipError_t launch_nr(const void* src, void* dst, int W, int H, int64_t pitch, int gens, bool bounded, bool bytes,
                     hipStream_t s) {
    if (bounded) {
        if (bytes)
            hipLaunchKernelGGL((gol_wave_resident<NW, RPL, true, true>), dim3(1), dim3(64), 0, s, src, dst, W, H, pitch,
                               gens);
        else
            hipLaunchKernelGGL((gol_wave_resident<NW, RPL, true, false>), dim3(1), dim3(64), 0, s, src, dst, W, H,
                               pitch, gens);
    } else {
        if (bytes)
            hipLaunchKernelGGL((gol_wave_resident<NW, RPL, false, true>), dim3(1), dim3(64), 0, s, src, dst, W, H,
                               pitch, gens);
        else
            hipLaunchKernelGGL((gol_wave_resident<NW, RPL, false, false>), dim3(1), dim3(64), 0, s, src, dst, W, H,
                               pitch, gens);
    }
    return hipGetLastError();
}

template <int NW>
hipError_t launch_n(const void* src, void* dst, int W, int H, int64_t pitch, int gens, bool bounded, bool bytes, int rpl,
                    hipStream_t s) {
    switch (rpl) {
        case 1: return launch_nr<NW, 1>(src, dst, W, H, pitch, gens, bounded, bytes, s);
        case 2: return launch_nr<NW, 2>(src, dst, W, H, pitch, gens, bounded, bytes, s);
        case 3: return launch_nr<NW, 3>(src, dst, W, H, pitch, gens, bounded, bytes, s);
        case 4: return launch_nr<NW, 4>(src, dst, W, H, pitch, gens, bounded, bytes, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace

// Rows per lane for an H-row board: the fewest (1..4) that divide H with at most 64 lanes, or 0.
int wave_resident_rpl(int64_t W, int64_t H) {
    if (W < 3 || W > 128 || H < 3) return 0;
    for (int r = 1; r <= 4; r++)
        if (H % r == 0 && H / r <= 64) return r;
    return 0;
}

hipError_t launch_wave_resident(const void* src, void* dst, int64_t W, int64_t H, int64_t pitch, int64_t gens,
                                bool bounded, bool bytes, hipStream_t s) {
    const int rpl = wave_resident_rpl(W, H);
    if (!rpl || gens < 1 || gens > INT32_MAX || (!bytes && (W % 32 || pitch < W / 32))) return hipErrorInvalidValue;
    const int nw = (int)((W + 31) / 32);
    switch (nw) {
        case 1: return launch_n<1>(src, dst, (int)W, (int)H, pitch, (int)gens, bounded, bytes, rpl, s);
        case 2: return launch_n<2>(src, dst, (int)W, (int)H, pitch, (int)gens, bounded, bytes, rpl, s);
        case 3: return launch_n<3>(src, dst, (int)W, (int)H, pitch, (int)gens, bounded, bytes, rpl, s);
        case 4: return launch_n<4>(src, dst, (int)W, (int)H, pitch, (int)gens, bounded, bytes, rpl, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace gol
