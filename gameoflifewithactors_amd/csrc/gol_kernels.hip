// gol_kernels.hip -- gfx950 kernels for the Game of Life hot path.
//
// The reference computes one generation as ~18 mailbox messages per cell (GameOfLifeLogic.fs:39-71,
// GameofLife.fs:88-138).  Here a generation (or K of them) is one launch over a bit-packed board:
//
//   gol_stream_step<K>   THE hot kernel.  One wavefront owns a column strip of 64 words (62 interior +
//                        one halo word per side, lane = word column) and streams down a segment of rows.
//                        Each row loaded from HBM is pushed through K generations held in registers
//                        (a 3-row window of row sums per generation level), so one pass reads and writes
//                        the board once for K generations (temporal blocking).  Horizontal neighbours
//                        come from DPP wave_shr:1 / wave_shl:1; bit carries from v_alignbit_b32; counts
//                        from v_bitop3_b32 (gol_bitlogic.h).  No LDS, no barriers, no atomics.
//   gol_bytes_step       generic one-byte-per-cell step for widths that are not a multiple of 32.
//   pack / unpack / render / splitmix init / population / hash -- the data formats either side.
//
// Board geometry (StripGeom) covers both the single-GPU board (wrap_rows = torus rows wrap inside
// the buffer) and a row strip of a multi-GPU board (owned rows plus `ghost` halo rows above and below,
// filled by the RCCL halo exchange).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <cstdlib>

#include "gol_bitlogic.h"
#include "gol_internal.h"

namespace gol {

static constexpr int kWave = 64;
static constexpr int kInterior = kWave - 2;  // words stored per wave column strip
static constexpr int kWavesPerBlock = 4;

// Cross-lane word exchange.  GOL_XLANE selects the mechanism (measured in tools/ubench/valu_rates.hip:
// a DPP move costs a half-rate VALU issue slot pair on gfx950; ds_bpermute_b32 runs on the LDS pipe
// and leaves the VALU free):
//   0 = DPP wave_shr:1 / wave_shl:1 (both directions on the VALU)
//   1 = ds_bpermute_b32 for both directions (LDS crossbar)
//   2 = left via DPP, right via ds_bpermute (split the two pipes)
#ifndef GOL_XLANE
#define GOL_XLANE 2
#endif
struct XLane {
    int left_addr, right_addr;  // byte addresses of lane-1 / lane+1 for ds_bpermute
    __device__ __forceinline__ explicit XLane(int lane)
        : left_addr(((lane - 1) & 63) << 2), right_addr(((lane + 1) & 63) << 2) {}
    __device__ __forceinline__ uint32_t from_left(uint32_t v) const {  // lane i <- lane i-1
#if GOL_XLANE == 1
        return (uint32_t)__builtin_amdgcn_ds_bpermute(left_addr, (int)v);
#else
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);  // wave_shr:1
#endif
    }
    __device__ __forceinline__ uint32_t from_right(uint32_t v) const {  // lane i <- lane i+1
#if GOL_XLANE == 0
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);  // wave_shl:1
#else
        return (uint32_t)__builtin_amdgcn_ds_bpermute(right_addr, (int)v);
#endif
    }
};

__device__ __forceinline__ int64_t floor_mod(int64_t a, int64_t m) {
    int64_t r = a % m;
    return r < 0 ? r + m : r;
}

// ------------------------------------------------------------------------------------------------
// Temporal-blocked streaming step.  Each wave: strip `sx` (words [62*sx, 62*sx + 62)), output rows
// [seg_begin, seg_end).  Input rows [seg_begin - K, seg_end + K) are streamed; generation level g
// lags level g-1 by one row.  Rows outside a level's valid cone only ever hold pipeline garbage and
// are never stored.
//
// Two rows advance through every level per loop trip: the 3-row window of each level lives in two
// register slots (X, Y) whose roles alternate between the two rows, so no register is ever copied, and
// the second row's DPP reads overlap the first row's arithmetic (DPP needs 2 wait states after the
// VALU write of its source on gfx9-family parts).

// One level for one row: window (prev = P, cur = C) + new row v -> next generation of the C row.
// The new row's sums overwrite the P slot (it becomes the C slot of the following row).
template <bool MASK>
__device__ __forceinline__ uint32_t level_row(const XLane& xl, uint32_t v, uint32_t& sP, uint32_t& cP, uint32_t sC,
                                              uint32_t cC, uint32_t alC, uint32_t rowmask) {
    uint32_t sN, cN;
    row_sum(xl.from_left(v), v, xl.from_right(v), sN, cN);
    uint32_t out = life_next(sP, cP, sC, cC, sN, cN, alC);
    sP = sN;
    cP = cN;
    if (MASK) out &= rowmask;
    return out;
}

// Rows per loop trip: enough independent loads in flight per wave for the memory-bound K = 1 pass,
// fewer for the VALU-bound deep passes (registers go to the K level windows instead).
template <int K>
struct TripRows {
    static constexpr int value = K == 1 ? 8 : 4;
};

// One wavefront's pipeline: K generation levels of 3-row windows held in registers.
template <int K, bool BOUNDED, bool WRAP_ROWS>
struct StreamWave {
    static constexpr int R = TripRows<K>::value;
    static_assert(R % 4 == 0, "slot roles must repeat every trip and registers alternate every two rows");

    const uint32_t* __restrict__ src;
    uint32_t* __restrict__ dst;
    const StreamArgs& a;
    XLane xl;
    uint32_t lc;       // loaded word column (per lane)
    uint32_t colmask;  // bounded: ~0 for on-board columns
    bool store_lane;
    int64_t seg_begin, seg_end, nsteps, ly0;
    int64_t load_br;  // buffer row of the next level-0 row to load (uniform)

    // level state: two row slots (X, Y) of row sums (s, c) and the raw centre word of the Y slot
    uint32_t sX[K], cX[K], sY[K], cY[K], aY[K];

    __device__ __forceinline__ StreamWave(const uint32_t* s, uint32_t* d, const StreamArgs& args, int lane,
                                          int64_t sx, int64_t sy)
        : src(s), dst(d), a(args), xl(lane) {
        const int64_t cw = sx * kInterior - 1 + lane;  // this lane's word column (may be off-board)
        if (BOUNDED) {
            const bool in = cw >= 0 && cw < a.words;
            colmask = in ? 0xffffffffu : 0u;
            lc = in ? (uint32_t)cw : 0u;
        } else {
            colmask = 0xffffffffu;
            lc = (uint32_t)floor_mod(cw, a.words);
        }
        store_lane = lane >= 1 && lane <= kInterior && cw < a.words;
        seg_begin = a.out_begin + sy * a.seg;
        seg_end = seg_begin + a.seg < a.out_end ? seg_begin + a.seg : a.out_end;
        nsteps = (seg_end - seg_begin) + 2 * K;  // level-0 rows streamed
        ly0 = seg_begin - K;                     // level-0 row of step 0
        load_br = WRAP_ROWS ? floor_mod(ly0, a.rows) : ly0 + a.ghost;
#pragma unroll
        for (int g = 0; g < K; g++) sX[g] = cX[g] = sY[g] = cY[g] = aY[g] = 0;
    }

    // Load the next R level-0 rows.  Loads are unconditional (addresses clamped; values masked) so the
    // number of memory operations per trip is fixed and the compiler can wait for exactly the loads.
    __device__ __forceinline__ void load(uint32_t (&buf)[R], int64_t first_step) {
        const int64_t buf_rows = a.rows + 2 * a.ghost;
#pragma unroll
        for (int r = 0; r < R; r++) {
            int64_t br = load_br;
            if (WRAP_ROWS) {
                load_br = br + 1 == a.rows ? 0 : br + 1;
            } else {
                load_br = br + 1;
                br = br < buf_rows ? br : buf_rows - 1;  // past the segment's last step: value unused
            }
            uint32_t v = src[br * a.pitch + lc];
            if (BOUNDED) {
                const int64_t gy = a.y0 + ly0 + first_step + r;
                v = (gy >= 0 && gy < a.height) ? (v & colmask) : 0u;
            }
            buf[r] = v;
        }
    }

    // Push R rows (steps t*R .. t*R+R-1) through the K levels; v[r] becomes row (ly0 + t*R + r - K) of
    // generation K.  SKIP: leave out levels whose inputs in this trip are all pipeline fill (garbage).
    template <bool SKIP>
    __device__ __forceinline__ void process(uint32_t (&v)[R], int64_t t) {
        const int64_t lyt = ly0 + t * R;
#pragma unroll
        for (int g = 0; g < K; g++) {
            // level g's input rows in this trip are valid only from step 2g on
            if (SKIP && t * R + R - 1 < 2 * g) continue;
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
                if (BOUNDED) {  // cells outside the board stay dead at every generation (Script.fsx:11)
                    const int64_t gy = a.y0 + lyt + r - g - 1;  // row produced from v[r] at level g + 1
                    m0 = (gy >= 0 && gy < a.height) ? colmask : 0u;
                    m1 = (gy + 1 >= 0 && gy + 1 < a.height) ? colmask : 0u;
                }
                // even row: window (X = row-2, Y = row-1) -> X;  odd row: (Y, X) -> Y
                const uint32_t o0 = level_row<BOUNDED>(xl, v[r], sX[g], cX[g], sY[g], cY[g], aY[g], m0);
                const uint32_t o1 = level_row<BOUNDED>(xl, v[r + 1], sY[g], cY[g], sX[g], cX[g], v[r], m1);
                aY[g] = v[r + 1];
                v[r] = o0;
                v[r + 1] = o1;
            }
        }
    }

    __device__ __forceinline__ void store_all(const uint32_t (&v)[R], int64_t t) {
        const int64_t lo = ly0 + t * R - K;
        if (store_lane) {
#pragma unroll
            for (int r = 0; r < R; r++) dst[((WRAP_ROWS ? 0 : a.ghost) + lo + r) * a.pitch + lc] = v[r];
        }
    }

    __device__ __forceinline__ void store_masked(const uint32_t (&v)[R], int64_t t) {
        const int64_t lo = ly0 + t * R - K;
        if (store_lane) {
#pragma unroll
            for (int r = 0; r < R; r++)
                if (lo + r >= seg_begin && lo + r < seg_end) dst[((WRAP_ROWS ? 0 : a.ghost) + lo + r) * a.pitch + lc] = v[r];
        }
    }
};

// Temporal-blocked streaming step.  Each wave: strip `sx` (words [62*sx, 62*sx + 62)), output rows
// [seg_begin, seg_end).  Trips: [0, t_fill) pipeline fill (no stores, garbage levels skipped),
// [t_fill, t_tail) steady state (every row stored, fixed memory-op count per trip), [t_tail, ntrips)
// masked tail.  Loads for trip t+1 are issued before trip t computes (one trip of prefetch).
template <int K, bool BOUNDED, bool WRAP_ROWS>
__global__ __launch_bounds__(kWave* kWavesPerBlock) void gol_stream_step(const uint32_t* __restrict__ src,
                                                                          uint32_t* __restrict__ dst,
                                                                          StreamArgs a) {
    using W = StreamWave<K, BOUNDED, WRAP_ROWS>;
    constexpr int R = W::R;
    const int lane = threadIdx.x & (kWave - 1);
    // wave index made provably uniform so all row bookkeeping lives in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wave;
    if (gw >= a.nstrips * a.nsegs) return;
    W w(src, dst, a, lane, gw % a.nstrips, gw / a.nstrips);

    const int64_t ntrips = (w.nsteps + R - 1) / R;
    const int64_t t_fill = (2 * K) / R < ntrips ? (2 * K) / R : ntrips;  // trips entirely before step 2K
    const int64_t first_store_trip = (2 * K + R - 1) / R;
    int64_t t_tail = (2 * K + (w.seg_end - w.seg_begin)) / R;  // trips entirely inside the stored range
    if (t_tail < first_store_trip) t_tail = first_store_trip;
    if (t_tail > ntrips) t_tail = ntrips;

    uint32_t nxt[R], v[R];
    w.load(nxt, 0);
    int64_t t = 0;
    for (; t < t_fill; t++) {
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = nxt[r];
        w.load(nxt, (t + 1) * R);
        w.template process<true>(v, t);
    }
    for (; t < first_store_trip && t < ntrips; t++) {  // transition trip (when R does not divide 2K)
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = nxt[r];
        w.load(nxt, (t + 1) * R);
        w.template process<true>(v, t);
        w.store_masked(v, t);
    }
    for (; t < t_tail; t++) {  // steady state
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = nxt[r];
        w.load(nxt, (t + 1) * R);
        w.template process<false>(v, t);
        w.store_all(v, t);
    }
    for (; t < ntrips; t++) {  // masked tail
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = nxt[r];
        w.load(nxt, (t + 1) * R);
        w.template process<false>(v, t);
        w.store_masked(v, t);
    }
}

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
// Formats.  `pitch` = words per buffer row; rows of a strip start at `row0` inside the buffer.
__global__ void gol_pack(const uint8_t* __restrict__ cells, uint32_t* __restrict__ words, int64_t W, int64_t rows,
                         int64_t pitch, int64_t row0) {
    const int64_t wpr = W / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    const uint8_t* p = cells + y * W + w * 32;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 32; b++) v |= (uint32_t)(p[b] != 0) << b;
    words[(row0 + y) * pitch + w] = v;
}

// packed -> bytes: pixels[x + y*stride] = bit ? value : 0   (GameOfLifeUI.fs:24-28 when value = 128)
__global__ void gol_unpack(const uint32_t* __restrict__ words, uint8_t* __restrict__ out, int64_t W, int64_t rows,
                           int64_t pitch, int64_t row0, int64_t stride, uint8_t value) {
    const int64_t wpr = W / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    const uint32_t v = words[(row0 + y) * pitch + w];
    uint8_t* p = out + y * stride + w * 32;
#pragma unroll
    for (int b = 0; b < 32; b++) p[b] = ((v >> b) & 1u) ? value : 0;
}

// window (x0, y0, w, h) of a packed or byte board -> bytes 0/1, out[i + j*w]
__global__ void gol_region(const void* __restrict__ board, bool packed, int64_t W, int64_t pitch, int64_t x0,
                           int64_t y0, int64_t w, int64_t h, uint8_t* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= w * h) return;
    const int64_t x = x0 + idx % w, y = y0 + idx / w;
    if (packed) {
        const uint32_t v = static_cast<const uint32_t*>(board)[y * pitch + x / 32];
        out[idx] = (v >> (x & 31)) & 1u;
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

// alive(x, y) = bit (x & 31) of low32(splitmix64(seed ^ (gy * ceil(W/32) + x/32)))  
__global__ void gol_splitmix_packed(uint32_t* __restrict__ words, int64_t wpr, int64_t rows, int64_t pitch,
                                    int64_t row0, int64_t gy0, uint64_t seed) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= wpr * rows) return;
    const int64_t w = idx % wpr, y = idx / wpr;
    words[(row0 + y) * pitch + w] = (uint32_t)splitmix64(seed ^ (uint64_t)((gy0 + y) * wpr + w));
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

// population (packed): atomically adds popcount of rows [row0, row0+rows) into *acc
__global__ void gol_popcount_packed(const uint32_t* __restrict__ words, int64_t wpr, int64_t rows, int64_t pitch,
                                    int64_t row0, unsigned long long* acc) {
    uint64_t sum = 0;
    const int64_t n = wpr * rows;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x)
        sum += __popc(words[(row0 + idx / wpr) * pitch + idx % wpr]);
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(acc, (unsigned long long)sum);
}

__global__ void gol_popcount_bytes(const uint8_t* __restrict__ cells, int64_t n, unsigned long long* acc) {
    uint64_t sum = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x)
        sum += cells[idx] != 0;
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(acc, (unsigned long long)sum);
}

// Canonical hash partial sum: chunk j of global row gy = words 2j, 2j+1 (hi = 0 past the row)
__global__ void gol_hash_packed(const uint32_t* __restrict__ words, int64_t wpr, int64_t rows, int64_t pitch,
                                int64_t row0, int64_t gy0, unsigned long long* acc) {
    const int64_t nc = (wpr + 1) / 2;
    const int64_t n = nc * rows;
    uint64_t sum = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx % nc, y = idx / nc;
        const uint32_t* r = words + (row0 + y) * pitch;
        const uint64_t lo = r[2 * j];
        const uint64_t hi = (2 * j + 1 < wpr) ? r[2 * j + 1] : 0u;
        const uint64_t key = (uint64_t)((gy0 + y) * nc + j);
        sum += fmix64((lo | (hi << 32)) ^ fmix64(key + 0x9E3779B97F4A7C15ULL));
    }
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, (unsigned long long)sum);
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
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, (unsigned long long)sum);
}

// ------------------------------------------------------------------------------------------------
// Launchers (host).  All return hipError_t; geometry was validated by the caller (gol_capi.cpp).

static inline unsigned grid1d(int64_t n, int block = 256) {
    int64_t g = (n + block - 1) / block;
    return (unsigned)(g < 1 ? 1 : g);
}
static inline unsigned grid_stride(int64_t n, int block = 256) {
    int64_t g = (n + block - 1) / block;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}

template <int K>
static hipError_t launch_stream_k(const uint32_t* src, uint32_t* dst, const StreamArgs& a, bool bounded, bool wrap,
                                  hipStream_t s) {
    const int64_t waves = a.nstrips * a.nsegs;
    const unsigned blocks = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    const dim3 block(kWave * kWavesPerBlock);
    if (bounded) {
        if (wrap)
            hipLaunchKernelGGL((gol_stream_step<K, true, true>), dim3(blocks), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_stream_step<K, true, false>), dim3(blocks), block, 0, s, src, dst, a);
    } else {
        if (wrap)
            hipLaunchKernelGGL((gol_stream_step<K, false, true>), dim3(blocks), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_stream_step<K, false, false>), dim3(blocks), block, 0, s, src, dst, a);
    }
    return hipGetLastError();
}

int64_t stream_strips(int64_t words) { return (words + kInterior - 1) / kInterior; }

template <int K>
static const void* stream_kernel(bool bounded, bool wrap) {
    if (bounded) return wrap ? (const void*)&gol_stream_step<K, true, true> : (const void*)&gol_stream_step<K, true, false>;
    return wrap ? (const void*)&gol_stream_step<K, false, true> : (const void*)&gol_stream_step<K, false, false>;
}

static int k_index(int k) {
    switch (k) {
        case 1: return 0;
        case 2: return 1;
        case 4: return 2;
        case 8: return 3;
        case 16: return 4;
        case 24: return 5;
        case 32: return 6;
        default: return -1;
    }
}

// Waves of gol_stream_step<K> the current device holds at once (occupancy x CUs), cached per variant.
// Falls back to 4096 when no device answers (host-only planning, e.g. CPU tests).
static int64_t resident_waves(int k, bool bounded, bool wrap) {
    static std::atomic<int64_t> cache[7][2][2];
    const int ki = k_index(k);
    if (ki < 0) return 4096;
    int64_t v = cache[ki][bounded][wrap].load(std::memory_order_relaxed);
    if (v > 0) return v;
    const void* fn = nullptr;
    switch (k) {
        case 1: fn = stream_kernel<1>(bounded, wrap); break;
        case 2: fn = stream_kernel<2>(bounded, wrap); break;
        case 4: fn = stream_kernel<4>(bounded, wrap); break;
        case 8: fn = stream_kernel<8>(bounded, wrap); break;
        case 16: fn = stream_kernel<16>(bounded, wrap); break;
        case 24: fn = stream_kernel<24>(bounded, wrap); break;
        case 32: fn = stream_kernel<32>(bounded, wrap); break;
    }
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, kWave * kWavesPerBlock, 0) != hipSuccess ||
        blocks <= 0 || cus <= 0) {
        (void)hipGetLastError();
        return 4096;
    }
    v = (int64_t)blocks * cus * kWavesPerBlock;
    cache[ki][bounded][wrap].store(v, std::memory_order_relaxed);
    return v;
}

// Work decomposition: nstrips column strips x nsegs row segments, one wave each.  The segment count
// is chosen so the grid is ONE balanced round of resident waves (a partial second round would leave a
// tail of lone waves), with segments no shorter than 2K rows (pipeline fill cost).  GOL_SEG_ROWS
// overrides the segment length (experiments).
void plan_stream(StreamArgs& a, int k, bool bounded, bool wrap) {
    static const int64_t env_seg = [] {
        const char* e = std::getenv("GOL_SEG_ROWS");
        return e ? std::atoll(e) : 0LL;
    }();
    a.nstrips = stream_strips(a.words);
    const int64_t rows = a.out_end - a.out_begin;
    if (rows <= 0) {
        a.nsegs = 0;
        a.seg = 1;
        return;
    }
    int64_t seg = env_seg;
    if (seg <= 0) {
        const int64_t slots = resident_waves(k, bounded, wrap);
        int64_t nsegs = slots / a.nstrips;
        if (nsegs < 1) nsegs = 1;
        const int64_t min_seg = 2 * k > 16 ? 2 * k : 16;
        const int64_t max_segs = rows / min_seg > 0 ? rows / min_seg : 1;
        if (nsegs > max_segs) nsegs = max_segs;
        seg = (rows + nsegs - 1) / nsegs;
    }
    a.seg = seg;
    a.nsegs = (rows + seg - 1) / seg;
}

hipError_t launch_stream_step(const uint32_t* src, uint32_t* dst, StreamArgs a, int k, bool bounded, bool wrap,
                              hipStream_t s) {
    plan_stream(a, k, bounded, wrap);
    if (a.nsegs <= 0) return hipSuccess;
    switch (k) {
        case 1: return launch_stream_k<1>(src, dst, a, bounded, wrap, s);
        case 2: return launch_stream_k<2>(src, dst, a, bounded, wrap, s);
        case 4: return launch_stream_k<4>(src, dst, a, bounded, wrap, s);
        case 8: return launch_stream_k<8>(src, dst, a, bounded, wrap, s);
        case 16: return launch_stream_k<16>(src, dst, a, bounded, wrap, s);
        case 24: return launch_stream_k<24>(src, dst, a, bounded, wrap, s);
        case 32: return launch_stream_k<32>(src, dst, a, bounded, wrap, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_bytes_step(const uint8_t* src, uint8_t* dst, int64_t W, int64_t H, bool bounded, hipStream_t s) {
    if (bounded)
        hipLaunchKernelGGL((gol_bytes_step<true>), dim3(grid1d(W * H)), dim3(256), 0, s, src, dst, W, H);
    else
        hipLaunchKernelGGL((gol_bytes_step<false>), dim3(grid1d(W * H)), dim3(256), 0, s, src, dst, W, H);
    return hipGetLastError();
}

hipError_t launch_pack(const uint8_t* cells, uint32_t* words, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                       hipStream_t s) {
    hipLaunchKernelGGL(gol_pack, dim3(grid1d(W / 32 * rows)), dim3(256), 0, s, cells, words, W, rows, pitch, row0);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t* words, uint8_t* out, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                         int64_t stride, uint8_t value, hipStream_t s) {
    hipLaunchKernelGGL(gol_unpack, dim3(grid1d(W / 32 * rows)), dim3(256), 0, s, words, out, W, rows, pitch, row0,
                       stride, value);
    return hipGetLastError();
}

hipError_t launch_region(const void* board, bool packed, int64_t W, int64_t pitch, int64_t x0, int64_t y0, int64_t w,
                          int64_t h, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(gol_region, dim3(grid1d(w * h)), dim3(256), 0, s, board, packed, W, pitch, x0, y0, w, h, out);
    return hipGetLastError();
}

hipError_t launch_bytes_render(const uint8_t* cells, uint8_t* out, int64_t W, int64_t H, int64_t stride,
                               uint8_t value, hipStream_t s) {
    hipLaunchKernelGGL(gol_bytes_render, dim3(grid1d(W * H)), dim3(256), 0, s, cells, out, W, H, stride, value);
    return hipGetLastError();
}

hipError_t launch_splitmix_packed(uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  int64_t gy0, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(gol_splitmix_packed, dim3(grid1d(wpr * rows)), dim3(256), 0, s, words, wpr, rows, pitch, row0,
                       gy0, seed);
    return hipGetLastError();
}

hipError_t launch_splitmix_bytes(uint8_t* cells, int64_t W, int64_t H, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(gol_splitmix_bytes, dim3(grid1d(W * H)), dim3(256), 0, s, cells, W, H, seed);
    return hipGetLastError();
}

hipError_t launch_popcount_packed(const uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_popcount_packed, dim3(grid_stride(wpr * rows)), dim3(256), 0, s, words, wpr, rows, pitch,
                       row0, acc);
    return hipGetLastError();
}

hipError_t launch_popcount_bytes(const uint8_t* cells, int64_t n, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_popcount_bytes, dim3(grid_stride(n)), dim3(256), 0, s, cells, n, acc);
    return hipGetLastError();
}

hipError_t launch_hash_packed(const uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                              int64_t gy0, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_hash_packed, dim3(grid_stride((wpr + 1) / 2 * rows)), dim3(256), 0, s, words, wpr, rows,
                       pitch, row0, gy0, acc);
    return hipGetLastError();
}

hipError_t launch_hash_bytes(const uint8_t* cells, int64_t W, int64_t H, unsigned long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(gol_hash_bytes, dim3(grid_stride((W + 63) / 64 * H)), dim3(256), 0, s, cells, W, H, acc);
    return hipGetLastError();
}

}  // namespace gol
