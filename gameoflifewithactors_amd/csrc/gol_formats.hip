// gol_formats.hip -- data formats either side of the hot path, and the generic byte-per-cell step.
//
//   bytes <-> bit-packed rows (pack / unpack; unpack with value 128 or 255 is the render agent's Gray8
//   pixel fill, GameOfLifeUI.fs:24-28 / Script.fsx:33-35), windows, device-side splitmix init,
//   population, the canonical board hash, point placement for RLE patterns, and the byte-per-cell step
//   used for widths that are not a multiple of 32.  Packed layouts: gol_layout.h (interleave ilv).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gol_internal.h"
#include "gol_layout.h"

namespace gol {

// ------------------------------------------------------------------------------------------------
// Generic byte-per-cell step (any width >= 3).  Rule GameOfLifeLogic.fs:59-63, torus
// GameOfLifeDriver.fs:21-25, bounded Script.fsx:6-13.
template <bool BOUNDED>
__global__ __launch_bounds__(256) void gol_bytes_step(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int64_t W, int64_t H) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= W * H) return;
    const int64_t x = idx % W, y = idx / W;
    int n = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; dy++)
#pragma unroll
        for (int dx = -1; dx <= 1; dx++) {
            if (!dx && !dy) continue;
            int64_t nx = x + dx, ny = y + dy;
            if (BOUNDED) {
                if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
            } else {
                nx = nx < 0 ? nx + W : (nx >= W ? nx - W : nx);
                ny = ny < 0 ? ny + H : (ny >= H ? ny - H : ny);
            }
            n += src[nx + ny * W] != 0;
        }
    const uint8_t alive = src[idx] != 0;
    dst[idx] = (n == 3) | ((n == 2) & alive);
}

// ------------------------------------------------------------------------------------------------
// Packed formats.  `pitch` = words per buffer row; owned row y lives at buffer row `row0 + y`.

// bytes (cells[x + y*W], nonzero = alive) -> packed words; one thread per stored word
__global__ void gol_pack(const uint8_t* __restrict__ cells, uint32_t* __restrict__ words, int64_t W, int64_t rows,
                         int64_t pitch, int64_t row0, int ilv) {
    const int64_t wpr = W / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    const uint8_t* p = cells + y * W;
    uint32_t v = 0;
    for (int b = 0; b < 32; b++) v |= (uint32_t)(p[word_bit_cell(w, b, ilv)] != 0) << b;
    words[(row0 + y) * pitch + w] = v;
}

// Ragged byte board (any width) <-> whole consecutive words (the scratch rows of the cooperative and streaming passes
// on ragged boards: `pitch` words per row, bit b of word j = cell 32 j + b, cells past W and words past ceil(W / 32)
// zero).  One wavefront per chunk of 64 words of one row (2048 cells): the bytes move as 64 consecutive cells per
// wave instruction (coalesced byte loads / stores), the bits by ballot (pack) and readlane (unpack).  A thread per
// word walking its own 32 bytes (the round-2 kernels) read the 65535^2 board at a small fraction of HBM rate.
constexpr int kChunkWords = 64;

__device__ __forceinline__ bool ragged_chunk(int64_t words_per_row, int64_t H, int64_t& y, int64_t& w0) {
    const int64_t chunks = (words_per_row + kChunkWords - 1) / kChunkWords;
    const int64_t u = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (u >= chunks * H) return false;
    y = u / chunks;
    w0 = (u - y * chunks) * kChunkWords;
    return true;
}

__global__ __launch_bounds__(256) void gol_pack_ragged(const uint8_t* __restrict__ cells, uint32_t* __restrict__ words,
                                                        int64_t W, int64_t H, int64_t pitch) {
    int64_t y, w0;
    if (!ragged_chunk(pitch, H, y, w0)) return;
    const int lane = threadIdx.x & 63;
    // the row as a buffer resource: cells past W read as 0 (range check), so the loads carry no branch and all 32 are
    // in flight at once
    const __amdgpu_buffer_rsrc_t row =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cells + y * W), (short)0, (int)W, 0x00020000);
    uint8_t v[kChunkWords / 2];
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++)
        v[i] = __builtin_amdgcn_raw_buffer_load_b8(row, (int)((w0 + 2 * i) * 32) + lane, 0, 0);
    uint32_t mine = 0;  // word w0 + lane
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++) {
        const uint64_t m = __ballot(v[i] != 0);
        mine = lane == 2 * i ? (uint32_t)m : (lane == 2 * i + 1 ? (uint32_t)(m >> 32) : mine);
    }
    if (w0 + lane < pitch) words[y * pitch + w0 + lane] = mine;
}
// ... and back: the W cells of each row as 0 / 1 bytes (the byte board's own values)
__global__ __launch_bounds__(256) void gol_unpack_ragged(const uint32_t* __restrict__ words, uint8_t* __restrict__ cells,
                                                          int64_t W, int64_t H, int64_t pitch) {
    const int64_t nw = (W + 31) / 32;
    int64_t y, w0;
    if (!ragged_chunk(nw, H, y, w0)) return;
    const int lane = threadIdx.x & 63;
    const uint32_t mine = w0 + lane < nw ? words[y * pitch + w0 + lane] : 0u;
    // stores past the row's W cells are dropped by the buffer range check
    const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(cells + y * W, (short)0, (int)W, 0x00020000);
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)mine, 2 * i);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)mine, 2 * i + 1);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(((lane < 32 ? lo : hi) >> (lane & 31)) & 1u), row,
                                             (int)((w0 + 2 * i) * 32) + lane, 0, 0);
    }
}

// ---- Ring rows of a ragged TORUS board (DESIGN.md 4.1 "Ragged rows: ring rows").  A row of W cells (W not a multiple
// of 32) is a ring (GameOfLifeDriver.fs:21-25).  It is stored as an ALIGNED row of Wp = 64 * ceil((W + 2 * 64) / 64)
// cells in the packed layout `ilv` (1 or 2): ring position u holds cell x = (u - 64) mod W, so u in [64, 64 + W) are
// the board's cells, u in [0, 64) a copy of its last 64 cells and u in [64 + W, Wp) a copy of its first Wp - W - 64
// (>= 64).  The aligned streaming kernel then steps the ring rows as a torus of width Wp: the only wrong neighbours
// are at the two ends of the extended row, and after a pass of k <= 64 generations their errors have spread k cells,
// not into the board's cells; gol_ring_refresh then rewrites both copies from the board's cells.  Blocks of 64
// cells: u-block c holds words 2c, 2c + 1 (ilv 2: even / odd cells; ilv 1: cells 0-31 / 32-63 of the block).
// A ragged BOUNDED board uses the same block rows without the copies (pad 0: position u = cell u, cells past W zero,
// ceil(W / 64) blocks per row); the kernel's column masks keep those cells dead (gol_step.hip NARROW = 2).
constexpr int64_t kRingPad = 64;  // ring positions before the board's first cell (torus)

__device__ __forceinline__ uint32_t even_bits64(uint64_t x) {
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return (uint32_t)x;
}
// word p (0 / 1) of a 64-cell block given as a mask (bit i = cell i of the block)
__device__ __forceinline__ uint32_t ring_word(uint64_t m, int p, int ilv) {
    return ilv == 2 ? even_bits64(m >> p) : (uint32_t)(m >> (32 * p));
}
#ifndef GOL_CHECK_BOUNDS
#define GOL_CHECK_BOUNDS 0  // diagnostic builds: flag an access outside its row (gol_step.hip gol_debug_bounds)
#endif
#if GOL_CHECK_BOUNDS
__device__ unsigned g_bounds_err_formats;
#endif
// bit of ring position u of a row
__device__ __forceinline__ uint32_t ring_bit(const uint32_t* row, int64_t u, int ilv, int64_t pitch = 0) {
    const int64_t c = u >> 6;
    const int i = (int)(u & 63);
    const int64_t w = 2 * c + (ilv == 2 ? (i & 1) : (i >> 5));
#if GOL_CHECK_BOUNDS
    if (w < 0 || w >= pitch) {
        __hip_atomic_fetch_or(&g_bounds_err_formats, 1u << 20, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
#else
    (void)pitch;
#endif
    return (row[w] >> (ilv == 2 ? (i >> 1) : (i & 31))) & 1u;
}

// bytes -> ring rows.  One wavefront per chunk of 32 u-blocks (64 words) of a row: 64 consecutive ring positions per
// wave load (coalesced except at the two wraps), ballot per block, lanes 2i / 2i + 1 keep block i's words.
__global__ __launch_bounds__(256) void gol_pack_ring(const uint8_t* __restrict__ cells, uint32_t* __restrict__ words,
                                                     int64_t W, int64_t H, int64_t pitch, int ilv, int64_t pad) {
    int64_t y, w0;
    if (!ragged_chunk(pitch, H, y, w0)) return;
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t row =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cells + y * W), (short)0, (int)W, 0x00020000);
    const int64_t Wp = pitch * 32;
    uint8_t v[kChunkWords / 2];
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++) {
        const int64_t u = (w0 + 2 * i) * 32 + lane;
        int64_t x = u - pad;
        if (pad) x = x < 0 ? x + W : (x >= W ? x - W : x);  // the ring's copies (pad 0: cells past W read as 0)
        v[i] = __builtin_amdgcn_raw_buffer_load_b8(row, u < Wp && x < W ? (int)x : (int)W, 0, 0);  // past the row: 0
    }
    uint64_t mine = 0;  // the block of word w0 + lane
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++) {
        const uint64_t m = __ballot(v[i] != 0);
        mine = (lane >> 1) == i ? m : mine;
    }
    if (w0 + lane < pitch) words[y * pitch + w0 + lane] = ring_word(mine, lane & 1, ilv);
}

// ring rows -> bytes (the board's W cells as 0 / 1).  One wavefront per chunk of 32 x-blocks: x-block c is u-block
// c + 1 (kRingPad = 64), whose two words lanes 2i / 2i + 1 load; lane l stores cell 64 c + l.
__global__ __launch_bounds__(256) void gol_unpack_ring(const uint32_t* __restrict__ words, uint8_t* __restrict__ cells,
                                                       int64_t W, int64_t H, int64_t pitch, int ilv, int64_t pad) {
    const int64_t nxw = 2 * ((W + 63) / 64);  // words covering the board's cells
    int64_t y, w0;
    if (!ragged_chunk(nxw, H, y, w0)) return;
    const int lane = threadIdx.x & 63;
    const int64_t wi = pad / 32 + w0 + lane;
    const uint32_t mine = w0 + lane < nxw && wi < pitch ? words[y * pitch + wi] : 0u;
    const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(cells + y * W, (short)0, (int)W, 0x00020000);
#pragma unroll
    for (int i = 0; i < kChunkWords / 2; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)mine, 2 * i);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)mine, 2 * i + 1);
        const uint32_t bit = ilv == 2 ? (((lane & 1) ? hi : lo) >> (lane >> 1)) & 1u
                                      : ((lane < 32 ? lo : hi) >> (lane & 31)) & 1u;
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bit, row, (int)((w0 + 2 * i) * 32) + lane, 0, 0);
    }
}

// Rewrite the copies at both ends of every ring row from the board's cells (u-block 0 <- positions u + W; positions
// u >= 64 + W <- u - W; the board's own cells in the first suffix block are kept): at most 4 blocks per row (the
// suffix spans 64 .. 127 positions).  One wavefront per row; every lane issues its (at most 4) loads before the first
// ballot, so a row costs one memory round trip.  Every source position lies in [64, 64 + W), which this kernel never
// writes.  The host runs it only when the errors from the extended row's two ends could reach the board's cells on
// the next pass: they spread one cell per generation, so every 64 / k passes (gol_capi.cpp ring_age).
__global__ __launch_bounds__(256) void gol_ring_refresh(uint32_t* __restrict__ words, int64_t W, int64_t H,
                                                        int64_t pitch, int ilv) {
    const int64_t y = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (y >= H) return;
    const int lane = threadIdx.x & 63;
    uint32_t* row = words + y * pitch;
    const int64_t nblk = pitch / 2, end = kRingPad + W;
    const int64_t first_suffix = end >> 6;
    uint32_t bit[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t cb = i == 0 ? 0 : first_suffix + i - 1;
        if (cb >= nblk) continue;  // wave-uniform
        const int64_t u = cb * 64 + lane;
        const int64_t src = i == 0 ? u + W : (u >= end ? u - W : u);
        bit[i] = ring_bit(row, src, ilv, pitch);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t cb = i == 0 ? 0 : first_suffix + i - 1;
        if (cb >= nblk) continue;
        const uint64_t m = __ballot(bit[i] != 0);
        if (lane < 2) row[2 * cb + lane] = ring_word(m, lane, ilv);
    }
}

// packed -> bytes: out[x + y*stride] = alive ? value : 0; one thread per stored word
__global__ void gol_unpack(const uint32_t* __restrict__ words, uint8_t* __restrict__ out, int64_t W, int64_t rows,
                           int64_t pitch, int64_t row0, int64_t stride, uint8_t value, int ilv) {
    const int64_t wpr = W / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    const uint32_t v = words[(row0 + y) * pitch + w];
    uint8_t* p = out + y * stride;
    for (int b = 0; b < 32; b++) p[word_bit_cell(w, b, ilv)] = ((v >> b) & 1u) ? value : 0;
}

// window (x0, y0, w, h) of a packed (ilv > 0) or byte (ilv == 0) board -> bytes 0/1, out[i + j*w]
__global__ void gol_region(const void* __restrict__ board, int ilv, int64_t W, int64_t pitch, int64_t x0, int64_t y0,
                           int64_t w, int64_t h, uint8_t* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= w * h) return;
    const int64_t x = x0 + idx % w, y = y0 + idx / w;
    if (ilv > 0) {
        int64_t word;
        int bit;
        cell_pos(x, ilv, word, bit);
        out[idx] = (static_cast<const uint32_t*>(board)[y * pitch + word] >> bit) & 1u;
    } else {
        out[idx] = static_cast<const uint8_t*>(board)[y * W + x] != 0;
    }
}

__global__ void gol_bytes_render(const uint8_t* __restrict__ cells, uint8_t* __restrict__ out, int64_t W, int64_t H,
                                 int64_t stride, uint8_t value) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= W * H) return;
    const int64_t x = idx % W, y = idx / W;
    out[x + y * stride] = cells[idx] ? value : 0;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// alive(x, y) = bit (x & 31) of low32(splitmix64(seed ^ (gy * ceil(W/32) + x/32)))  (DESIGN.md).
// One thread per stored word; its 32 cells come from the (<= ilv) plain words of its block.
__global__ void gol_splitmix_packed(uint32_t* __restrict__ words, int64_t wpr, int64_t rows, int64_t pitch,
                                    int64_t row0, int64_t gy0, uint64_t seed, int ilv) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    const int64_t first = (w / ilv) * ilv;  // first plain word of this block
    uint32_t plain[4];
    for (int i = 0; i < ilv; i++) plain[i] = (uint32_t)splitmix64(seed ^ (uint64_t)((gy0 + y) * wpr + first + i));
    uint32_t v = 0;
    for (int b = 0; b < 32; b++) {
        const int64_t x = word_bit_cell(w, b, ilv) - first * 32;  // cell offset inside the block
        v |= ((plain[x >> 5] >> (x & 31)) & 1u) << b;
    }
    words[(row0 + y) * pitch + w] = v;
}

__global__ void gol_splitmix_bytes(uint8_t* __restrict__ cells, int64_t W, int64_t H, uint64_t seed) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= W * H) return;
    const int64_t x = idx % W, y = idx / W, wc = (W + 31) / 32;
    const uint32_t bits = (uint32_t)splitmix64(seed ^ (uint64_t)(y * wc + x / 32));
    cells[idx] = (bits >> (x & 31)) & 1u;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// One atomic per workgroup (256 threads): every atomicAdd on the single accumulator is a serialized device-scope
// round trip (the per-XCD L2s are not coherent), so one per wave made a 4096^2 population take ~100 us
// (profiles/r4/trace_c2_kernel_stats_j.csv) for 2 MiB of reads.
__device__ __forceinline__ void block_add(uint64_t sum, unsigned long long* acc) {
    __shared__ uint64_t part[4];
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(acc, (unsigned long long)t);
    }
}

// population (any packed layout): adds the popcount of rows [row0, row0+rows) into *acc
__global__ void gol_popcount_packed(const uint32_t* __restrict__ words, int64_t wpr, int64_t rows, int64_t pitch,
                                    int64_t row0, unsigned long long* acc) {
    uint64_t sum = 0;
    const int64_t n = wpr * rows;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x)
        sum += __popc(words[(row0 + idx / wpr) * pitch + idx % wpr]);
    block_add(sum, acc);
}

__global__ void gol_popcount_bytes(const uint8_t* __restrict__ cells, int64_t n, unsigned long long* acc) {
    uint64_t sum = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x)
        sum += cells[idx] != 0;
    block_add(sum, acc);
}

// Canonical 64-cell chunk j of a packed row r (layout ilv): bit i = cell 64j + i, zero past the width.
// The layout-independent form behind the hash and the board snapshot (gol_save_packed).
__device__ __forceinline__ uint64_t canonical_chunk(const uint32_t* r, int64_t W, int64_t j, int ilv) {
    if (ilv == 1) {
        const uint64_t lo = r[2 * j];
        const uint64_t hi = (2 * j + 1 < W / 32) ? r[2 * j + 1] : 0u;
        return lo | (hi << 32);
    }
    uint64_t v = 0;
    for (int i = 0; i < 64 && 64 * j + i < W; i++) {
        int64_t word;
        int bit;
        cell_pos(64 * j + i, ilv, word, bit);
        v |= (uint64_t)((r[word] >> bit) & 1u) << i;
    }
    return v;
}

// Canonical hash partial sum: for 64-cell chunk j of global row gy, v bit i = cell 64j + i;
// sum += fmix64(v ^ fmix64(gy * ceil(W/64) + j + phi)).  One thread per chunk.
__global__ void gol_hash_packed(const uint32_t* __restrict__ words, int64_t W, int64_t rows, int64_t pitch,
                                int64_t row0, int64_t gy0, int ilv, unsigned long long* acc) {
    const int64_t nc = (W + 63) / 64;
    const int64_t n = nc * rows;
    uint64_t sum = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx % nc, y = idx / nc;
        const uint64_t v = canonical_chunk(words + (row0 + y) * pitch, W, j, ilv);
        const uint64_t key = (uint64_t)((gy0 + y) * nc + j);
        sum += fmix64(v ^ fmix64(key + 0x9E3779B97F4A7C15ULL));
    }
    block_add(sum, acc);
}

__global__ void gol_hash_bytes(const uint8_t* __restrict__ cells, int64_t W, int64_t H, unsigned long long* acc) {
    const int64_t nc = (W + 63) / 64;
    const int64_t n = nc * H;
    uint64_t sum = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx % nc, y = idx / nc;
        uint64_t v = 0;
        for (int b = 0; b < 64 && j * 64 + b < W; b++) v |= (uint64_t)(cells[y * W + j * 64 + b] != 0) << b;
        sum += fmix64(v ^ fmix64((uint64_t)idx + 0x9E3779B97F4A7C15ULL));
    }
    block_add(sum, acc);
}

// set the cells listed as (x, y) pairs (RLE placement); ilv == 0: byte board
__global__ void gol_set_points(void* board, int ilv, int64_t W, int64_t pitch, const int64_t* xy, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t x = xy[2 * i], y = xy[2 * i + 1];
    if (ilv > 0) {
        int64_t word;
        int bit;
        cell_pos(x, ilv, word, bit);
        atomicOr(&static_cast<uint32_t*>(board)[y * pitch + word], 1u << bit);
    } else {
        static_cast<uint8_t*>(board)[x + y * W] = 1;
    }
}

// Board snapshot (gol_save_packed / gol_load_packed): canonical chunks out[y * ceil(W/64) + j].
// ilv > 0: packed board rows at buffer row row0 + y; ilv = 0: byte board (cells[x + y*W]).
__global__ void gol_export_canonical(const void* __restrict__ board, int64_t W, int64_t rows, int64_t pitch,
                                     int64_t row0, int ilv, uint64_t* __restrict__ out) {
    const int64_t nc = (W + 63) / 64;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nc * rows) return;
    const int64_t j = idx % nc, y = idx / nc;
    uint64_t v = 0;
    if (ilv > 0) {
        v = canonical_chunk(static_cast<const uint32_t*>(board) + (row0 + y) * pitch, W, j, ilv);
    } else {
        const uint8_t* c = static_cast<const uint8_t*>(board) + y * W;
        for (int b = 0; b < 64 && j * 64 + b < W; b++) v |= (uint64_t)(c[j * 64 + b] != 0) << b;
    }
    out[idx] = v;
}

// inverse: one thread per stored word (packed) or per cell (bytes); bits past the width are ignored
__global__ void gol_import_canonical(const uint64_t* __restrict__ in, int64_t W, int64_t rows, int64_t pitch,
                                     int64_t row0, int ilv, void* __restrict__ board) {
    const int64_t nc = (W + 63) / 64;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ilv > 0) {
        const int64_t wpr = W / 32;
        if (idx >= wpr * rows) return;
        const int64_t w = idx % wpr, y = idx / wpr;
        const uint64_t* r = in + y * nc;
        uint32_t v = 0;
        for (int b = 0; b < 32; b++) {
            const int64_t x = word_bit_cell(w, b, ilv);
            v |= (uint32_t)((r[x >> 6] >> (x & 63)) & 1u) << b;
        }
        static_cast<uint32_t*>(board)[(row0 + y) * pitch + w] = v;
    } else {
        if (idx >= W * rows) return;
        const int64_t x = idx % W, y = idx / W;
        static_cast<uint8_t*>(board)[idx] = (uint8_t)((in[y * nc + (x >> 6)] >> (x & 63)) & 1u);
    }
}

// ------------------------------------------------------------------------------------------------
// Launchers (host).  Geometry was validated by the caller (gol_capi.cpp).

static inline unsigned grid1d(int64_t n, int block = 256) {
    int64_t g = (n + block - 1) / block;
    return (unsigned)(g < 1 ? 1 : g);
}
// reductions (one atomic per workgroup): at least 16 elements per thread, at most 1024 workgroups
static inline unsigned grid_reduce(int64_t n, int block = 256) {
    int64_t g = n / ((int64_t)block * 16);
    if (g > 1024) g = 1024;
    return (unsigned)(g < 1 ? 1 : g);
}

hipError_t launch_bytes_step(const uint8_t* src, uint8_t* dst, int64_t W, int64_t H, bool bounded, hipStream_t s) {
    if (bounded)
        hipLaunchKernelGGL((gol_bytes_step<true>), dim3(grid1d(W * H)), dim3(256), 0, s, src, dst, W, H);
    else
        hipLaunchKernelGGL((gol_bytes_step<false>), dim3(grid1d(W * H)), dim3(256), 0, s, src, dst, W, H);
    return hipGetLastError();
}

hipError_t launch_pack(const uint8_t* cells, uint32_t* words, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                       int ilv, hipStream_t s) {
    hipLaunchKernelGGL(gol_pack, dim3(grid1d(W / 32 * rows)), dim3(256), 0, s, cells, words, W, rows, pitch, row0, ilv);
    return hipGetLastError();
}

// one wave (of 4 per 256-thread block) per 64-word chunk of a row
static unsigned ragged_blocks(int64_t words_per_row, int64_t H) {
    return (unsigned)(((words_per_row + kChunkWords - 1) / kChunkWords * H + 3) / 4);
}

hipError_t launch_pack_ragged(const uint8_t* cells, uint32_t* words, int64_t W, int64_t H, int64_t pitch, hipStream_t s) {
    // rows are addressed through 32-bit buffer offsets
    if (pitch < (W + 31) / 32 || (pitch + kChunkWords) * 32 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gol_pack_ragged, dim3(ragged_blocks(pitch, H)), dim3(256), 0, s, cells, words, W, H, pitch);
    return hipGetLastError();
}

hipError_t launch_unpack_ragged(const uint32_t* words, uint8_t* cells, int64_t W, int64_t H, int64_t pitch,
                                hipStream_t s) {
    if (pitch < (W + 31) / 32 || (pitch + kChunkWords) * 32 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gol_unpack_ragged, dim3(ragged_blocks((W + 31) / 32, H)), dim3(256), 0, s, words, cells, W, H,
                       pitch);
    return hipGetLastError();
}

int64_t ring_pitch(int64_t W, bool torus) { return 2 * ((W + (torus ? 2 * kRingPad : 0) + 63) / 64); }

hipError_t launch_pack_ring(const uint8_t* cells, uint32_t* words, int64_t W, int64_t H, int ilv, bool torus,
                            hipStream_t s) {
    const int64_t pitch = ring_pitch(W, torus);
    if ((ilv != 1 && ilv != 2) || W < 3 * kRingPad || (pitch + kChunkWords) * 32 >= ((int64_t)1 << 31))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(gol_pack_ring, dim3(ragged_blocks(pitch, H)), dim3(256), 0, s, cells, words, W, H, pitch, ilv,
                       torus ? kRingPad : (int64_t)0);
    return hipGetLastError();
}

hipError_t launch_unpack_ring(const uint32_t* words, uint8_t* cells, int64_t W, int64_t H, int ilv, bool torus,
                              hipStream_t s) {
    const int64_t pitch = ring_pitch(W, torus);
    if ((ilv != 1 && ilv != 2) || W < 3 * kRingPad || (pitch + kChunkWords) * 32 >= ((int64_t)1 << 31))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(gol_unpack_ring, dim3(ragged_blocks(2 * ((W + 63) / 64), H)), dim3(256), 0, s, words, cells, W,
                       H, pitch, ilv, torus ? kRingPad : (int64_t)0);
    return hipGetLastError();
}

hipError_t launch_ring_refresh(uint32_t* words, int64_t W, int64_t H, int ilv, hipStream_t s) {
    if ((ilv != 1 && ilv != 2) || W < 3 * kRingPad) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gol_ring_refresh, dim3((unsigned)((H + 3) / 4)), dim3(256), 0, s, words, W, H, ring_pitch(W, true),
                       ilv);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t* words, uint8_t* out, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                         int64_t stride, uint8_t value, int ilv, hipStream_t s) {
    hipLaunchKernelGGL(gol_unpack, dim3(grid1d(W / 32 * rows)), dim3(256), 0, s, words, out, W, rows, pitch, row0,
                       stride, value, ilv);
    return hipGetLastError();
}

hipError_t launch_region(const void* board, int ilv, int64_t W, int64_t pitch, int64_t x0, int64_t y0, int64_t w,
                         int64_t h, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(gol_region, dim3(grid1d(w * h)), dim3(256), 0, s, board, ilv, W, pitch, x0, y0, w, h, out);
    return hipGetLastError();
}

hipError_t launch_bytes_render(const uint8_t* cells, uint8_t* out, int64_t W, int64_t H, int64_t stride,
                               uint8_t value, hipStream_t s) {
    hipLaunchKernelGGL(gol_bytes_render, dim3(grid1d(W * H)), dim3(256), 0, s, cells, out, W, H, stride, value);
    return hipGetLastError();
}

hipError_t launch_splitmix_packed(uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  int64_t gy0, uint64_t seed, int ilv, hipStream_t s) {
    hipLaunchKernelGGL(gol_splitmix_packed, dim3(grid1d(wpr * rows)), dim3(256), 0, s, words, wpr, rows, pitch, row0,
                       gy0, seed, ilv);
    return hipGetLastError();
}

hipError_t launch_splitmix_bytes(uint8_t* cells, int64_t W, int64_t H, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(gol_splitmix_bytes, dim3(grid1d(W * H)), dim3(256), 0, s, cells, W, H, seed);
    return hipGetLastError();
}

hipError_t launch_popcount_packed(const uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_popcount_packed, dim3(grid_reduce(wpr * rows)), dim3(256), 0, s, words, wpr, rows, pitch,
                       row0, acc);
    return hipGetLastError();
}

hipError_t launch_popcount_bytes(const uint8_t* cells, int64_t n, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_popcount_bytes, dim3(grid_reduce(n)), dim3(256), 0, s, cells, n, acc);
    return hipGetLastError();
}

hipError_t launch_hash_packed(const uint32_t* words, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                              int64_t gy0, int ilv, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_hash_packed, dim3(grid_reduce((W + 63) / 64 * rows)), dim3(256), 0, s, words, W, rows, pitch,
                       row0, gy0, ilv, acc);
    return hipGetLastError();
}

hipError_t launch_hash_bytes(const uint8_t* cells, int64_t W, int64_t H, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_hash_bytes, dim3(grid_reduce((W + 63) / 64 * H)), dim3(256), 0, s, cells, W, H, acc);
    return hipGetLastError();
}

hipError_t launch_export_canonical(const void* board, int64_t W, int64_t rows, int64_t pitch, int64_t row0, int ilv,
                                   uint64_t* out, hipStream_t s) {
    hipLaunchKernelGGL(gol_export_canonical, dim3(grid1d((W + 63) / 64 * rows)), dim3(256), 0, s, board, W, rows, pitch,
                       row0, ilv, out);
    return hipGetLastError();
}

hipError_t launch_import_canonical(const uint64_t* in, int64_t W, int64_t rows, int64_t pitch, int64_t row0, int ilv,
                                   void* board, hipStream_t s) {
    const int64_t n = ilv > 0 ? W / 32 * rows : W * rows;
    hipLaunchKernelGGL(gol_import_canonical, dim3(grid1d(n)), dim3(256), 0, s, in, W, rows, pitch, row0, ilv, board);
    return hipGetLastError();
}

hipError_t launch_set_points(void* board, int ilv, int64_t W, int64_t pitch, const int64_t* xy, int64_t n,
                             hipStream_t s) {
    hipLaunchKernelGGL(gol_set_points, dim3(grid1d(n)), dim3(256), 0, s, board, ilv, W, pitch, xy, n);
    return hipGetLastError();
}

}  // namespace gol

#if GOL_CHECK_BOUNDS
extern "C" unsigned gol_debug_bounds_formats(void) {
    unsigned v = 0, z = 0;
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(gol::g_bounds_err_formats), sizeof(v), 0, hipMemcpyDeviceToHost);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gol::g_bounds_err_formats), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    return v;
}
#endif
