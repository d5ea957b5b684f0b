// gol_coop.hip -- persistent register-band pass for mid-size boards (BASELINE config 2: 4096^2) on gfx950.
//
// A 4096^2 board is 2 MiB packed: too large for one CU (gol_resident.hip), too small to fill the chip with the
// streaming pass (gol_step.hip), where each wave is one long serial chain per launch.  Here ONE workgroup of 16
// waves per CU stays resident for a whole gol_step call and owns a band of B rows, held in VGPRs:
//
//   local row i = global row y0 - K + i, i in [0, B + 2K): K halo rows above, the band, K halo rows below;
//   wave v holds local rows [v R, v R + R), lane l the words [l M, l M + M) of each (ilv-1 board, W <= 8192).
//
// Per generation (GameOfLifeLogic.fs:59-63, synchronous as under the Reset->State barrier) each wave writes its
// first and last row to LDS, one workgroup barrier, reads the row above its first and below its last, and
// steps its rows in registers: horizontal neighbours in the lane and from the adjacent lanes (DPP; the x-wrap
// of a torus, GameOfLifeDriver.fs:21-25, by DPP rotate or readlane), the rule from gol_bitlogic.h.  Rows
// outside a bounded board stay dead (Script.fsx:6-13).  Per block of k <= K generations the valid rows shrink
// by one per side and generation, so the band stays exact; between blocks only the band's first and last K rows
// leave the CU.
//
// Hand-off between neighbour bands: data-tagged granules (MI355X_MICROARCH.md "handoff-1to1" and "Valid forms", R2).
// Every word of the band's first and last K rows goes to a dedicated exchange buffer as ONE 8-byte write-through
// (sc1) store {word, tag}, tag = launch epoch << 16 | block + 1; the neighbour's lanes poll exactly the granules
// they need with 8-byte sc1 loads until the tag matches -- no drain, no barrier, no flag, and a torn granule is
// never accepted because data and tag arrive together.  The exchange buffer is double-buffered by block parity:
// a band rewrites parity p after both neighbours have published the next block, which they do after reading
// parity p; the epoch keeps a granule of an earlier launch from matching (the host clears the buffer when the
// 16-bit epoch wraps).  The board buffers are only read at the start and written at the end (kernel boundaries
// order those).  Residency: the grid is one workgroup per CU (LDS request above half the CU's), checked against the
// occupancy API before a plain launch (launch_persistent below; round 4: the cooperative launch API's exit-time
// teardown faulted under rocprofv3); every spin is bounded, and a timed-out wait raises an error word the host
// checks on the next synchronisation.
#include "gol_internal.h"
#include "gol_bitlogic.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <vector>

namespace gol {
namespace {

constexpr int kWaves = 16;                 // waves per workgroup: 4 per SIMD
constexpr int kThreads = 64 * kWaves;
constexpr int kMinLds = 96 * 1024;         // > half the CU's 160 KiB: one workgroup per CU
constexpr unsigned kSpinLimit = 1u << 25;  // ~ 2 s: a wait this long means a band is not resident (default)
// The wave-edge exchange per generation carries the edge rows' horizontal sums (sum and carry of the first and last
// row) in planes of one dword per lane, so no reader re-sums a neighbour's row.  Round 5 re-measured the
// alternatives (profiles/r5/coop_xch_ab_k.log, 4096^2 torus, us/generation): the same sums lane-major with
// ds_write/read_b64 0.571 against 0.558, the raw edge rows lane-major (half the LDS bytes, re-summed by the reader)
// 0.638 -- the generation is bound by its VALU chain, not by the LDS (MI355X_MICROARCH.md "LDS").
constexpr int kSlotRows = 4;  // LDS words per lane and word of a row, per wave and parity
// LDS slots per parity: one per wave, plus a zero slot on each side (the neighbours of the first and last
// waves), so every wave reads its neighbours' slots without a branch
constexpr int kSlots = kWaves + 2;

// GOL_COOP_STAMP (diagnostic builds only, never shipped): per band, wave and block, the time (s_memrealtime, 100 MHz)
// right after the wave issued its hand-off stores for the block, and right after its poll for the block's halo rows
// returned; gol_debug_coop_stamps() copies them out (tools/coop_stamps.py splits a block into compute and hand-off)
#ifndef GOL_COOP_STAMP
#define GOL_COOP_STAMP 0
#endif
#if GOL_COOP_STAMP
constexpr int kStampBands = 256, kStampBlocks = 128;
__device__ unsigned long long g_coop_stamps[kStampBands * kWaves * kStampBlocks * 2];
__device__ __forceinline__ void coop_stamp(int band, int wv, int blk, int what) {
    if (band < kStampBands && blk < kStampBlocks && (threadIdx.x & 63) == 0)
        g_coop_stamps[((band * kWaves + wv) * kStampBlocks + blk) * 2 + what] = __builtin_amdgcn_s_memrealtime();
}
#endif


struct CoopArgs {
    const uint32_t* src;  // board at launch
    uint32_t* dst;        // board after `gens` generations
    uint64_t* xch;        // exchange granules: [2 parity][nwg][2 (band top, band bottom)][K][nw] {word, tag}
    int64_t pitch;        // words per board row
    int nw;               // words per row (W / 32)
    int nl;               // lanes holding words (nw / M)
    int H;                // board rows
    int nwg;              // bands (= workgroups)
    int K;                // generations per block (<= every band's height)
    int gens;
    unsigned epoch;       // launch epoch (16 bits) of the granule tags
    int poll_delay;       // s_sleep 1 periods (64 clocks) before the first poll of a hand-off
    unsigned spin_limit;  // polls before a wait gives up (kSpinLimit unless a test lowers it)
    int* err;             // set to 1 by a timed-out wait
    int rag_lb;           // ragged rows (kLayRagged): bit of the last cell in the last word, (W - 1) & 31
    int rag_last;         // ragged rows: index of the last word that holds cells, ceil(W / 32) - 1
    int xch_bytes;        // bytes of the exchange buffer (the granules' buffer descriptor)
};

// A lane's M words of one row as granules {word, tag}, write-through (8-byte sc1 stores)
template <int M>
__device__ __forceinline__ void st_granules(uint64_t* p, const uint32_t (&w)[M], unsigned tag) {
#pragma unroll
    for (int t = 0; t < M; t++)
        __hip_atomic_store(p + t, (uint64_t)tag << 32 | w[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ... and back, false after the spin limit.  The hand-off is latency-bound: at 4096^2 it costs ~2 us per block
// of 8 generations, 0.25 of the 0.72 us per generation (profiles/r2/coop_decomp_y.log: the pass without it).
// The neighbour publishes at about the time this band starts polling, so a poll issued at once often returns
// before the data is visible and costs a second memory round trip.  Rows of up to 128 words (M <= 2): every
// granule the wave needs (R rows x M words per lane) in ONE batch of 8-byte sc1 loads per poll round, after a
// short delay (`delay` s_sleep 1 periods, 8 by default: ~250 ns); 4096^2 0.70 vs 0.72 us/generation, bounded
// 0.68 vs 0.74, 2048^2 0.41 vs 0.44 (profiles/r2/coop_delay_za.log).  Wider rows (M = 4: 8 granules per lane and
// row pair) ran slower batched (8192 x 4096 1.69 vs 1.61) and poll granule by granule, at once.
// Status of a hand-off wait: the granules arrived, the wait timed out, or another wave of the launch had timed out
// (the launch's error word): the board is invalid, stop waiting.
constexpr int kGot = 0, kTimedOut = 1, kLaunchFailed = 2;
// The error word is read by a wave that is still waiting, every 32 polls (round 5: read before every poll round, its
// load was a memory round trip on the hand-off's critical path -- and its s_waitcnt also waited for the wave's own
// write-through granule stores -- at every block: 4096^2 0.554 -> 0.536 us/generation; rows of 256 words keep the
// read in front of the poll, see the poll site).
__device__ __forceinline__ bool launch_failed(const int* err) {
    return __builtin_amdgcn_ballot_w64(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) != 0;
}
template <int M, int R>
__device__ __forceinline__ int ld_granules(const uint64_t* const (&src)[R], uint32_t (&w)[R][M], unsigned tag,
                                           int delay, unsigned spin_limit, const int* err) {
    if constexpr (M >= 4) {
        int st = kGot;
#pragma unroll
        for (int i = 0; i < R; i++) {
            if (!src[i]) continue;
#pragma unroll
            for (int t = 0; t < M; t++) {
                uint64_t g = __hip_atomic_load(src[i] + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (unsigned it = 0; st == kGot && (unsigned)(g >> 32) != tag; it++) {  // after a failure: no more waits
                    if (it == spin_limit) {
                        st = kTimedOut;
                        break;
                    }
                    if ((it & 31) == 31 && launch_failed(err)) {
                        st = kLaunchFailed;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    g = __hip_atomic_load(src[i] + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                w[i][t] = (uint32_t)g;
            }
        }
        return st;
    }
    for (int i = 0; i < delay; i++) __builtin_amdgcn_s_sleep(1);
    uint64_t v[R][M];
    for (unsigned it = 0;; it++) {
#pragma unroll
        for (int i = 0; i < R; i++)
#pragma unroll
            for (int t = 0; t < M; t++)
                v[i][t] = src[i] ? __hip_atomic_load(src[i] + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : (uint64_t)tag << 32;
        bool miss = false;
#pragma unroll
        for (int i = 0; i < R; i++)
#pragma unroll
            for (int t = 0; t < M; t++) miss = miss || (unsigned)(v[i][t] >> 32) != tag;
        if (__builtin_amdgcn_ballot_w64(miss) == 0) break;  // wave-uniform exit
        if (it == spin_limit) return kTimedOut;
        if ((it & 31) == 31 && launch_failed(err)) return kLaunchFailed;
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int i = 0; i < R; i++)
        if (src[i])
#pragma unroll
            for (int t = 0; t < M; t++) w[i][t] = (uint32_t)v[i][t];
    return kGot;
}

// 16-byte hand-off (round 5): a lane's granules in pairs, as 16-byte write-through stores and 16-byte sc1 polls
// (two {word, tag} granules per access, each 8-byte half written by ONE store: MI355X_MICROARCH.md "Valid forms", R2
// halves) -- half the hand-off's memory instructions at M = 2 and whole 1 KB runs per wave instruction.  Rows of an
// even word count per lane (M = 2, 4) use it: 4096^2 0.693 -> 0.582 us/generation (means of 3 interleaved rounds,
// profiles/r5/coop_g16_ab_b.jsonl / .txt), 0.572 with the lean loop below (coop_variants_ab_d, "g1posl"); 8192 x 4096
// 1.573 -> 1.009 with the 8192-wide poll delay (coop_variants_ab_d "base" -> coop_poll_delay_ab_g "coopd24").
// Rejected A/B variants, same files: two poll rounds kept in flight (slower at 4096^2: the compiler serialises the rounds' register copies),
// bands mapped XCD by XCD so neighbours share an L2 (profiles/r5/ab_xcd_h.log: 8192 x 4096 1.27 vs 1.01), 8-byte
// buffer granules for M = 1 (level with the atomic form).
constexpr int kAuxSc1 = 16;  // buffer instruction cache policy: sc1 (gfx950)
typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2c __attribute__((ext_vector_type(2)));
// Granule accesses of a lane's M words: pairs {word, tag, word, tag} as 16-byte accesses (M even), or single 8-byte
// {word, tag} granules (M = 1).  Buffer instructions with the sc1 policy: never flat (MI355X_MICROARCH.md "Valid
// forms": global_/buffer_ sc1 loads to registers).
template <int M>
struct Gran {
    static constexpr int G = M % 2 == 0 ? 2 : 1;  // granules per access
    static constexpr int N = M / G;               // accesses per row
    using V = typename std::conditional<G == 2, u32x4c, u32x2c>::type;
    __device__ __forceinline__ static V load(__amdgpu_buffer_rsrc_t r, int off) {
        if constexpr (G == 2) return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1);
        else return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSc1);
    }
    // The stores are global_store ... sc1 written out: with the buffer form the compiler waited vmcnt(0) before
    // reusing a store's data or offset registers (before the next granule store, and at the top of the first generation
    // of every block), so every write-through store waited for the previous one's completion.  A global store reads its
    // address and data registers at issue.  (Not counted by the compiler's wait-count pass: its waits on later loads
    // only get more conservative.)
    __device__ __forceinline__ static void store(uint64_t* p, const uint32_t* w, unsigned tag) {
        if constexpr (G == 2) {
            const u32x4c v = {w[0], tag, w[1], tag};
            // s_nop: a store of more than 8 bytes reads its data registers one cycle after issue, and the hazard
            // recogniser cannot see into the asm to separate the next write of those registers (found by the 8192-wide
            // parity test: two 16-byte stores per row back to back)
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
        } else {
            const u32x2c v = {w[0], tag};
            asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
        }
    }
    __device__ __forceinline__ static bool miss(const V& v, unsigned tag) {
        if constexpr (G == 2) return v.y != tag || v.w != tag;
        else return v.y != tag;
    }
    __device__ __forceinline__ static void take(const V& v, uint32_t* w) {
        w[0] = v.x;
        if constexpr (G == 2) w[1] = v.z;
    }
};
template <int M>
__device__ __forceinline__ void st_granules16(uint64_t* p, const uint32_t (&w)[M], unsigned tag) {
#pragma unroll
    for (int t = 0; t < Gran<M>::N; t++) Gran<M>::store(p + Gran<M>::G * t, &w[Gran<M>::G * t], tag);
}
// Polls of ld_granules16: rows the lane does not need load from an offset past the descriptor's range (zero, no
// memory access, no branch) and are ignored by the tag check.
constexpr int kNoGranule = 0x7fffffff;
template <int M, int R>
__device__ __forceinline__ void issue16(__amdgpu_buffer_rsrc_t xrs, const int (&off)[R],
                                        typename Gran<M>::V (&v)[R][Gran<M>::N]) {
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int t = 0; t < Gran<M>::N; t++)
            v[i][t] = Gran<M>::load(xrs, off[i] == kNoGranule ? kNoGranule : off[i] + 8 * Gran<M>::G * t);
}
template <int M, int R>
__device__ __forceinline__ bool hit16(const int (&off)[R], const typename Gran<M>::V (&v)[R][Gran<M>::N], unsigned tag) {
    bool miss = false;
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int t = 0; t < Gran<M>::N; t++) miss = miss || (off[i] != kNoGranule && Gran<M>::miss(v[i][t], tag));
    return __builtin_amdgcn_ballot_w64(miss) == 0;  // wave-uniform
}
template <int M, int R>
__device__ __forceinline__ void take16(const int (&off)[R], const typename Gran<M>::V (&v)[R][Gran<M>::N],
                                       uint32_t (&w)[R][M]) {
#pragma unroll
    for (int i = 0; i < R; i++)
        if (off[i] != kNoGranule)
#pragma unroll
            for (int t = 0; t < Gran<M>::N; t++) Gran<M>::take(v[i][t], &w[i][Gran<M>::G * t]);
}
template <int M, int R>
__device__ __forceinline__ int ld_granules16(__amdgpu_buffer_rsrc_t xrs, const int (&off)[R], uint32_t (&w)[R][M],
                                             unsigned tag, int delay, unsigned spin_limit, const int* err) {
    for (int i = 0; i < delay; i++) __builtin_amdgcn_s_sleep(1);
    typename Gran<M>::V v[R][Gran<M>::N];
    issue16<M, R>(xrs, off, v);
    for (unsigned it = 0;; it++) {
        if (hit16<M, R>(off, v, tag)) break;
        if (it == spin_limit) return kTimedOut;
        if ((it & 31) == 31 && launch_failed(err)) return kLaunchFailed;
        __builtin_amdgcn_s_sleep(1);
        issue16<M, R>(xrs, off, v);
    }
    take16<M, R>(off, v, w);
    return kGot;
}

// Word of the lane to the left / right.  FULL (all 64 lanes hold words): DPP rotate on a torus, DPP shift with
// zero fill on a bounded board.  Otherwise DPP shift (idle lanes hold zeros, which is a bounded board's dead
// edge) and on a torus the wrap between lane nl - 1 and lane 0 by readlane.
template <bool BOUNDED, bool FULL>
__device__ __forceinline__ uint32_t from_left(uint32_t v, int lane, int nl) {
    if (FULL && !BOUNDED) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xf, 0xf, false);  // wave_ror:1
    uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);                  // wave_shr:1
    if (!BOUNDED) {
        const uint32_t last = (uint32_t)__builtin_amdgcn_readlane((int)v, nl - 1);
        r = lane == 0 ? last : r;
    }
    return r;
}
template <bool BOUNDED, bool FULL>
__device__ __forceinline__ uint32_t from_right(uint32_t v, int lane, int nl) {
    if (FULL && !BOUNDED) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xf, 0xf, false);  // wave_rol:1
    uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);                  // wave_shl:1
    if (!BOUNDED) {
        const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
        r = lane == nl - 1 ? first : r;
    }
    return r;
}

// Horizontal 3-sums of this lane's M words of one row: M consecutive words of an ilv-1 board (2 funnel shifts
// per word), or one interleaved block of an ilv-M board (gol_layout.h: 2 funnel shifts per block).
template <int M, bool ILV, bool BOUNDED, bool FULL>
__device__ __forceinline__ void lane_row_sum(const uint32_t (&r)[M], int lane, int nl, uint32_t (&s)[M],
                                             uint32_t (&c)[M]) {
    const uint32_t left = from_left<BOUNDED, FULL>(r[M - 1], lane, nl);
    const uint32_t right = from_right<BOUNDED, FULL>(r[0], lane, nl);
    if (ILV) {
        row_sum_block<M>(r, left, right, s, c);
        return;
    }
#pragma unroll
    for (int j = 0; j < M; j++) row_sum(j == 0 ? left : r[j - 1], r[j], j == M - 1 ? right : r[j + 1], s[j], c[j]);
}

// Word layouts of a band row: consecutive words of an ilv-1 board, interleaved blocks of an ilv-M board, or the
// consecutive words of a ragged row (width not a multiple of 32: the byte board packed by the host into a scratch
// buffer of whole words, cells past W zero, the row end fixed up at bit level).
constexpr int kLayWords = 0, kLayInterleaved = 1, kLayRagged = 2;

// Horizontal 3-sums of a lane's M consecutive words of a ragged row (GameOfLifeDriver.fs:21-25 on a torus: the
// west neighbour of cell 0 is cell W - 1, bit `lb` of word `last`, held by lane lane_last at position t_last;
// the east neighbour of cell W - 1 is cell 0; Script.fsx:6-13 when bounded: dead beyond both ends).  The lanes
// exchange edge words with zero fill; the two row-end words are then patched, as in the single-wave pass
// (gol_wave.hip).
template <int M, bool BOUNDED>
__device__ __forceinline__ void ragged_row_sum(const uint32_t (&r)[M], int lane, int lane_last, int t_last, int lb,
                                               uint32_t (&s)[M], uint32_t (&c)[M]) {
    const uint32_t left = (uint32_t)__builtin_amdgcn_mov_dpp((int)r[M - 1], 0x138, 0xf, 0xf, true);  // wave_shr:1
    const uint32_t right = (uint32_t)__builtin_amdgcn_mov_dpp((int)r[0], 0x130, 0xf, 0xf, true);     // wave_shl:1
    uint32_t west[M], east[M];
#pragma unroll
    for (int t = 0; t < M; t++) {
        west[t] = align_right(r[t], t == 0 ? left : r[t - 1], 31);
        east[t] = align_right(t == M - 1 ? right : r[t + 1], r[t], 1);
    }
    if (!BOUNDED) {
        uint32_t lw = r[0];
#pragma unroll
        for (int t = 1; t < M; t++) lw = t == t_last ? r[t] : lw;
        const uint32_t last = (uint32_t)__builtin_amdgcn_readlane((int)lw, lane_last);
        const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)r[0], 0);
        if (lane == 0) west[0] = (r[0] << 1) | ((last >> lb) & 1u);
#pragma unroll
        for (int t = 0; t < M; t++)
            if (lane == lane_last && t == t_last) east[t] = (r[t] >> 1) | ((first & 1u) << lb);
    }
#pragma unroll
    for (int t = 0; t < M; t++) {
        s[t] = lut3<0x96>(west[t], r[t], east[t]);
        c[t] = lut3<0xE8>(west[t], r[t], east[t]);
    }
}

template <int M, int R, int LAY, bool BOUNDED, bool FULL>
__global__ __launch_bounds__(kThreads) void gol_band_pass(CoopArgs a) {
    constexpr bool ILV = LAY == kLayInterleaved;
    constexpr bool RAG = LAY == kLayRagged;
#ifdef GOL_COOP_PAD  // A/B (instruction-alignment study, round 6): GOL_COOP_PAD 4-byte s_nops at the entry
#define GOL_COOP_STR2(x) #x
#define GOL_COOP_STR(x) GOL_COOP_STR2(x)
    asm volatile(".rept " GOL_COOP_STR(GOL_COOP_PAD) "\n\ts_nop 0\n\t.endr");
#endif
    extern __shared__ uint32_t xs[];  // [2 parity][kSlots][kSlotRows][M][64 lanes]; slots 0 and kSlots - 1 stay zero
    const int band = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int y0 = (int)((int64_t)a.H * band / a.nwg);
    const int y1 = (int)((int64_t)a.H * (band + 1) / a.nwg);
    const int B = y1 - y0;
    const int K = a.K;
    const int L = B + 2 * K;  // local rows
    const int r0 = wv * R;    // this wave's first local row
    const int nl = a.nl;
    const bool lane_on = FULL || lane < nl;  // full rows: every lane holds words
    const int col = lane * M;  // this lane's first word
    // ragged rows: the lane holding the last word, its position there, and per word the mask of cells on the row
    // (the other layouts compile none of this: their instruction streams are the measured ones)
    [[maybe_unused]] int lane_last = 0, t_last = 0;
    [[maybe_unused]] uint32_t wmask[M];
    if constexpr (RAG) {
        lane_last = a.rag_last / M;
        t_last = a.rag_last % M;
        const uint32_t lastmask = a.rag_lb == 31 ? 0xffffffffu : (2u << a.rag_lb) - 1u;
#pragma unroll
        for (int t = 0; t < M; t++)
            wmask[t] = col + t < a.rag_last ? 0xffffffffu : (col + t == a.rag_last ? lastmask : 0u);
    }
    const int up = band > 0 ? band - 1 : (BOUNDED ? -1 : a.nwg - 1);
    const int dn = band + 1 < a.nwg ? band + 1 : (BOUNDED ? -1 : 0);
    auto gy_of = [&](int i) { return y0 - K + i; };
    auto on_board = [&](int gy) { return gy >= 0 && gy < a.H; };
    auto wrap = [&](int gy) { return gy < 0 ? gy + a.H : (gy >= a.H ? gy - a.H : gy); };
    auto xrow = [&](int parity, int b, int side, int i) {  // exchange row (band b's top / bottom K rows, row i)
        return a.xch + ((((int64_t)parity * a.nwg + b) * 2 + side) * K + i) * a.nw;
    };
    auto tag_of = [&](int blk) { return a.epoch << 16 | (unsigned)(blk + 1); };  // tag of block blk's granules
    constexpr bool G16 = M % 2 == 0;  // 16-byte granule pairs (M = 1: 8-byte atomic granules)
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(a.xch, (short)0, a.xch_bytes, 0x00020000);

    // ---- the band and its halo from the board (plain loads: the board buffers are not handed off in-kernel)
    uint32_t w[R][M];
#pragma unroll
    for (int i = 0; i < R; i++) {
        const int gy = gy_of(r0 + i);
#pragma unroll
        for (int j = 0; j < M; j++) w[i][j] = 0;
        if (r0 + i < L && lane_on && (!BOUNDED || on_board(gy))) {
            const uint32_t* row = a.src + (int64_t)wrap(gy) * a.pitch + col;
#pragma unroll
            for (int j = 0; j < M; j++) w[i][j] = row[j];
        }
    }

    // The band's initial rows must have arrived before the generation loop: a wait left for the compiler lands
    // INSIDE the loop (first use), and there s_waitcnt vmcnt(0) also waits for the hand-off's write-through
    // stores (vmcnt counts stores): every producer wave then stalled for its stores' completion in the first
    // generation of every block.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (wv == 0 || wv == kWaves - 1) {  // the zero slots beside the first and last waves (both parities)
        const int z = wv == 0 ? 0 : kSlots - 1;
#pragma unroll
        for (int par = 0; par < 2; par++)
#pragma unroll
            for (int t = 0; t < kSlotRows * M; t++) xs[((par * kSlots + z) * kSlotRows * M + t) * 64 + lane] = 0u;
    }  // ordered before their first read by the first generation's barrier

    const int nblk = (a.gens + K - 1) / K;
    bool failed = false;  // wave-uniform: a hand-off wait of this launch timed out
    for (int blk = 0; blk < nblk; blk++) {
        const int k = a.gens - blk * K < K ? a.gens - blk * K : K;
        if (blk > 0) {
            // halo rows: the neighbours' edge rows of block blk - 1 (parity (blk - 1) & 1), polled granule by granule
            const int par = (blk - 1) & 1;
            const uint64_t* src[R];
#pragma unroll
            for (int i = 0; i < R; i++) {
                const int li = r0 + i;
                src[i] = nullptr;
                if (!lane_on) continue;
                if (li < K && up >= 0) src[i] = xrow(par, up, 1, li) + col;                              // up band's bottom rows
                else if (li >= K + B && li < L && dn >= 0) src[i] = xrow(par, dn, 0, li - K - B) + col;  // dn band's top rows
            }
            bool any = false;
#pragma unroll
            for (int i = 0; i < R; i++) any = any || src[i] != nullptr;
            // Once any wave of the launch has timed out (this one, or another band's: the error word, which a waiting
            // wave reads every 32 polls) the board is invalid: stop waiting, so a launch with a non-resident band ends
            // after about one spin limit instead of one per block.  No early exit: every wave still meets the
            // generation barriers.
            int st = kGot;
            // Rows of 256 words (M = 4) keep a read of the error word in front of their poll: there that memory round
            // trip is worth its latency -- 8192 x 2048 0.89 against 0.99 us/generation without it, 8192 x 4096 1.03
            // against 1.08, where no first-poll delay matched it (24 / 40 / 64: 0.98 / 1.00 / 1.06,
            // profiles/r5/coop_poll_throttle_ab_n.log, coop_delay_ab_m.log).  A missed poll round of these rows is 4 KB
            // per wave; polling one granule pair per lane after a miss was slower still (1.02).
            if constexpr (M >= 4)
                if (!failed && __builtin_amdgcn_ballot_w64(any) != 0 && launch_failed(a.err)) failed = true;
            if (!failed && __builtin_amdgcn_ballot_w64(any) != 0) {
                if constexpr (G16) {
                    int off[R];
#pragma unroll
                    for (int i = 0; i < R; i++) off[i] = src[i] ? (int)((src[i] - a.xch) * 8) : kNoGranule;
                    st = ld_granules16<M, R>(xrs, off, w, tag_of(blk - 1), a.poll_delay, a.spin_limit, a.err);
                    // the polled rounds have all returned (the tag checks waited for them); saying so here keeps the
                    // wait-count pass from assuming poll loads in flight at the granule stores and generation loop
                    // below, where a vmcnt(0) would also wait for this wave's write-through stores
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                } else {
                    st = ld_granules<M, R>(src, w, tag_of(blk - 1), a.poll_delay, a.spin_limit, a.err);
                }
            }
            if (st == kTimedOut) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st != kGot) failed = true;
        }
#if GOL_COOP_STAMP
        coop_stamp(band, wv, blk, 1);
#endif
        // k generations: generation j computes local rows [K - k + 1 + j, K + B + k - 1 - j); this wave's rows
        // [r0, r0 + R) meet them while j < j_act.  The wave's interior rows do not depend on the exchange: they are
        // stepped between publishing the edge rows' sums and the barrier, so the barrier wait and the LDS round trip
        // overlap them.
        const int j_act = __builtin_amdgcn_readfirstlane(std::min(K + B + k - 1 - r0, r0 + R - K + k - 1));
        for (int j = 0; j < k; j++) {
            const int gen = blk * K + j;  // generation of this launch
            const int par = gen & 1;      // alternates across blocks too: no barrier separates them
            // the slot of wave wv - 1 (slot index wv): this wave's reads and writes are all at positive constant
            // offsets from it (one address per generation; the ds instructions' immediate offsets do the rest)
            uint32_t* nb = xs + ((par * kSlots + wv) * kSlotRows * M) * 64 + lane;
            auto put = [&](int w_rel, int q, const uint32_t (&v)[M]) {
#pragma unroll
                for (int t = 0; t < M; t++) nb[((w_rel * kSlotRows + q) * M + t) * 64] = v[t];
            };
            auto get = [&](int w_rel, int q, uint32_t (&v)[M]) {
#pragma unroll
                for (int t = 0; t < M; t++) v[t] = nb[((w_rel * kSlotRows + q) * M + t) * 64];
            };
            auto row_sums = [&](const uint32_t (&r)[M], uint32_t (&sv)[M], uint32_t (&cv)[M]) {
                if constexpr (RAG)
                    ragged_row_sum<M, BOUNDED>(r, lane, lane_last, t_last, a.rag_lb, sv, cv);
                else
                    lane_row_sum<M, ILV, BOUNDED, FULL>(r, lane, nl, sv, cv);
            };
            // (dead outside a bounded board at every generation: `dead` below)
            // generation j produces this wave's rows while j < j_act (block constant, one scalar compare per
            // generation), and the wave's edge rows are read by a producing neighbour one generation longer
            const bool active = j < j_act;
            const bool sums = j <= j_act;
            uint32_t so[R][M], co[R][M];
            if (sums) {
                // the row sums of the first and last rows, while a producing neighbour reads them (inactive waves
                // too: their rows border active ones)
#pragma unroll
                for (int i = 0; i < R; i++) row_sums(w[i], so[i], co[i]);
                put(1, 0, so[0]);
                put(1, 1, co[0]);
                put(1, 2, so[R - 1]);
                put(1, 3, co[R - 1]);
            }
            // the wave's interior rows need no neighbour: stepped while the edge rows travel through LDS
            if (active) {
#pragma unroll
                for (int i = 1; i + 1 < R; i++) {
                    const bool dead = BOUNDED && !on_board(gy_of(r0 + i));
#pragma unroll
                    for (int t = 0; t < M; t++) {
                        const uint32_t v = life_next(so[i - 1][t], co[i - 1][t], so[i][t], co[i][t], so[i + 1][t],
                                                     co[i + 1][t], w[i][t]);
                        w[i][t] = dead || !lane_on ? 0u : (RAG ? v & wmask[t] : v);
                    }
                }
            }
            __syncthreads();
            if (!active) continue;
            uint32_t sa[M], ca[M], sb[M], cb[M];
            get(0, 2, sa);
            get(0, 3, ca);
            get(2, 0, sb);
            get(2, 1, cb);
            constexpr int kEdgeRows = R > 1 ? 2 : 1;  // rows 0 and R - 1 (interior rows are done)
#pragma unroll
            for (int e = 0; e < kEdgeRows; e++) {
                const int i = e == 0 ? 0 : R - 1;
                const bool dead = BOUNDED && !on_board(gy_of(r0 + i));
#pragma unroll
                for (int t = 0; t < M; t++) {
                    const uint32_t v = life_next(i == 0 ? sa[t] : so[i - 1][t], i == 0 ? ca[t] : co[i - 1][t], so[i][t],
                                                 co[i][t], i == R - 1 ? sb[t] : so[i + 1][t],
                                                 i == R - 1 ? cb[t] : co[i + 1][t], w[i][t]);
                    w[i][t] = dead || !lane_on ? 0u : (RAG ? v & wmask[t] : v);
                }
            }
        }
        if (blk + 1 == nblk) continue;  // the last block hands nothing off (continue: the measured instruction stream)
        // ---- hand-off: the band's first and last K rows as granules of parity blk & 1
        const int par = blk & 1;
#pragma unroll
        for (int i = 0; i < R; i++) {
            const int li = r0 + i;
            // a band shorter than 2K rows has rows in both ranges: each goes to both sides
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const int e = side == 0 ? li - K : li - B;  // row index within the band's top / bottom K rows
                if (e < 0 || e >= K || !lane_on) continue;
                if constexpr (G16)
                    st_granules16<M>(xrow(par, band, side, e) + col, w[i], tag_of(blk));
                else
                    st_granules<M>(xrow(par, band, side, e) + col, w[i], tag_of(blk));
            }
        }
#if GOL_COOP_STAMP
        coop_stamp(band, wv, blk, 0);
#endif
    }
    // ---- the band to the result buffer
    if (!lane_on) return;
#pragma unroll
    for (int i = 0; i < R; i++) {
        const int li = r0 + i;
        if (li >= K && li < K + B) {
            uint32_t* row = a.dst + (int64_t)gy_of(li) * a.pitch + col;
#pragma unroll
            for (int t = 0; t < M; t++) row[t] = w[i][t];
        }
    }
}

constexpr int kRows[] = {1, 2, 3, 4, 6, 8};  // rows per wave instantiated

template <int M, int R, int LAY>
const void* kernel_mri(bool bounded, bool full) {
    if (LAY == kLayRagged)  // ragged rows never use the full-wave rotate (the row end is patched at bit level)
        return bounded ? (const void*)&gol_band_pass<M, R, LAY, true, false> : (const void*)&gol_band_pass<M, R, LAY, false, false>;
    if (bounded)
        return full ? (const void*)&gol_band_pass<M, R, LAY, true, true> : (const void*)&gol_band_pass<M, R, LAY, true, false>;
    return full ? (const void*)&gol_band_pass<M, R, LAY, false, true> : (const void*)&gol_band_pass<M, R, LAY, false, false>;
}

template <int M, int LAY>
const void* kernel_ml(int r, bool bounded, bool full) {
    switch (r) {
        case 1: return kernel_mri<M, 1, LAY>(bounded, full);
        case 2: return kernel_mri<M, 2, LAY>(bounded, full);
        case 3: return kernel_mri<M, 3, LAY>(bounded, full);
        case 4: return kernel_mri<M, 4, LAY>(bounded, full);
        case 6: return kernel_mri<M, 6, LAY>(bounded, full);
        case 8: return kernel_mri<M, 8, LAY>(bounded, full);
    }
    return nullptr;
}

template <int M>
const void* kernel_m(int r, int lay, bool bounded, bool full) {
    if (lay == kLayInterleaved) {  // interleaved boards (ilv == M)
        if constexpr (M > 1) return kernel_ml<M, kLayInterleaved>(r, bounded, full);
        return nullptr;
    }
    if (lay == kLayRagged) return kernel_ml<M, kLayRagged>(r, bounded, full);
    return kernel_ml<M, kLayWords>(r, bounded, full);
}

}  // namespace

// Words per lane for a row of nw words (0: the width does not fit one wave).
int coop_m(int64_t nw) {
    const int m = nw <= 64 ? 1 : (nw <= 128 ? 2 : 4);
    return nw <= 256 && nw % m == 0 ? m : 0;
}

// min_rows: rows per wave at least (the board's "coop_r" option, A/B: fewer, taller wave slices re-sum fewer
// neighbour rows; 1 by default).
bool coop_plan(int64_t W, int64_t H, int k, int* nwg, int* B, int* R, int min_rows) {
    if (min_rows < 1 || min_rows > 8) min_rows = 1;
    const int cus = device_cus();
    if (cus <= 0 || W < 32 || W % 32 || H < 3 || k < 1 || !coop_m(W / 32)) return false;
    // balanced bands of >= k rows each (a k-row halo then comes from ONE neighbour band), one per CU at most
    int64_t n = H / k < cus ? H / k : cus;
    if (n < 1) return false;
    const int64_t b = (H + n - 1) / n;  // the largest band
    int64_t rows = (b + 2 * k + kWaves - 1) / kWaves;  // rows per wave
    if (rows < min_rows) rows = min_rows;
    int r = 0;
    for (int c : kRows)
        if (c >= rows) {
            r = c;
            break;
        }
    if (!r) return false;
    *nwg = (int)n;
    *B = (int)b;
    if (R) *R = r;
    return true;
}

int64_t coop_xch_words(int64_t W, int nwg, int k) { return (int64_t)2 * 2 * nwg * 2 * k * (W / 32); }

hipError_t launch_coop_pass(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch, int ilv, int k,
                            int64_t gens, bool bounded, unsigned epoch, int* err, uint32_t* xch, int64_t xch_words,
                            hipStream_t s, int64_t ragged_w, const CoopTuning& tune) {
    int nwg = 0, B = 0, R = 0;
    if (!coop_plan(W, H, k, &nwg, &B, &R, tune.min_rows) || gens < 1 || gens > 65535 || pitch < W / 32 ||
        coop_xch_words(W, nwg, k) > xch_words)
        return hipErrorInvalidValue;
    const int nw = (int)(W / 32);
    const int M = coop_m(nw);
    if (ilv != 1 && ilv != M) return hipErrorInvalidValue;
    // ragged rows: W is the padded width of the scratch rows (whole words, a multiple of M), ragged_w the board's
    if (ragged_w && (ilv != 1 || ragged_w > W || ragged_w <= W - 32 * M)) return hipErrorInvalidValue;
    CoopArgs a;
    a.src = src;
    a.dst = dst;
    a.xch = reinterpret_cast<uint64_t*>(xch);
    a.xch_bytes = (int)std::min<int64_t>(xch_words * 4, 0x7fffffff);
    a.pitch = pitch;
    a.nw = nw;
    a.nl = nw / M;
    a.H = (int)H;
    a.nwg = nwg;
    a.K = k;
    a.gens = (int)gens;
    a.epoch = epoch & 0xffffu;
    a.err = err;
    a.rag_lb = ragged_w ? (int)((ragged_w - 1) & 31) : 31;
    a.rag_last = ragged_w ? (int)((ragged_w + 31) / 32 - 1) : nw - 1;
    a.poll_delay = tune.poll_delay >= 0 ? tune.poll_delay : 8;  // s_sleep periods before a first poll (ld_granules)
    a.spin_limit = tune.spin_limit ? tune.spin_limit : kSpinLimit;
    const bool full = a.nl == 64;
    const int lay = ragged_w ? kLayRagged : (ilv == M && M > 1 ? kLayInterleaved : kLayWords);
    const void* fn = M == 1 ? kernel_m<1>(R, lay, bounded, full)
                            : (M == 2 ? kernel_m<2>(R, lay, bounded, full) : kernel_m<4>(R, lay, bounded, full));
    if (!fn) return hipErrorInvalidValue;
    const size_t need = (size_t)2 * kSlots * kSlotRows * M * 64 * 4;
    const size_t lds = need > (size_t)kMinLds ? need : (size_t)kMinLds;
    if (hipError_t e = set_max_dynamic_lds(fn, (int)lds)) return e;
    void* args[] = {&a};
    return launch_persistent(fn, (unsigned)nwg, kThreads, args, lds, s, !tune.plain_launch);
}

// ---- device-keyed host state of the persistent passes (every cache keyed by device, so a process
// driving boards on several GPUs -- or GPUs of different CU counts -- never uses another device's answer)

int device_cus() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    static std::mutex mu;
    static std::vector<std::pair<int, int>> known;  // (device, CUs)
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& k : known)
        if (k.first == dev) return k.second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    known.emplace_back(dev, n);
    return n;
}

hipError_t set_max_dynamic_lds(const void* fn, int bytes) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    static std::mutex mu;
    static std::vector<std::pair<int, const void*>> done;
    std::lock_guard<std::mutex> lock(mu);
    if (std::find(done.begin(), done.end(), std::make_pair(dev, fn)) != done.end()) return hipSuccess;
    if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes)) return e;
    done.emplace_back(dev, fn);
    return hipSuccess;
}

int64_t persistent_capacity(const void* fn, unsigned threads, size_t lds) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    struct Fit {
        int dev;
        const void* fn;
        unsigned threads;
        size_t lds;
        int64_t resident;  // workgroups the device holds at once
    };
    static std::mutex mu;
    static std::vector<Fit> fits;
    std::lock_guard<std::mutex> lock(mu);
    for (const Fit& f : fits)
        if (f.dev == dev && f.fn == fn && f.threads == threads && f.lds == lds) return f.resident;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)threads, lds) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -1;
    const int64_t resident = (int64_t)per_cu * cus;
    fits.push_back({dev, fn, threads, lds, resident});
    return resident;
}

// Persistent passes of every board in the process run one at a time per device.  Each
// launch waits on the device's last persistent launch (hipStreamWaitEvent) and becomes the new last one: two grids
// whose bands spin on each other are then never resident together, so two handles stepping mid-size boards from two
// threads on their own streams cannot split the CUs between them and starve both (gol.h: separate handles are
// independent).  A per-device mutex orders the wait, the launch and the record.  Ordinary launches (the streaming
// pass, I/O kernels) of other streams still share the device; they end on their own, so a persistent grid waits for
// CUs they hold at most for their duration (the spin limit is ~2 s).
namespace {
struct DeviceSerial {
    int dev;
    std::mutex* mu;
    hipEvent_t last;
};
}  // namespace

hipError_t launch_persistent(const void* fn, unsigned grid, unsigned threads, void** args, size_t lds, hipStream_t s,
                             bool cooperative) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    const int64_t resident = persistent_capacity(fn, threads, lds);
    if (resident < 0) return hipErrorInvalidValue;
    if ((int64_t)grid > resident) return hipErrorCooperativeLaunchTooLarge;
    static std::mutex table_mu;
    static std::vector<DeviceSerial> table;  // entries are never removed (one per device)
    std::mutex* mu = nullptr;
    hipEvent_t last = nullptr;  // per device, both fixed once created (the table itself may grow)
    {
        std::lock_guard<std::mutex> lock(table_mu);
        for (const DeviceSerial& d : table)
            if (d.dev == dev) {
                mu = d.mu;
                last = d.last;
            }
        if (!mu) {
            if (hipError_t e = hipEventCreateWithFlags(&last, hipEventDisableTiming)) return e;
            mu = new std::mutex;
            table.push_back({dev, mu, last});
        }
    }
    std::lock_guard<std::mutex> lock(*mu);
    if (hipError_t e = hipStreamWaitEvent(s, last, 0)) return e;  // an unrecorded event: no wait
    const hipError_t e = cooperative ? hipLaunchCooperativeKernel(fn, dim3(grid), dim3(threads), args, (unsigned)lds, s)
                                     : hipLaunchKernel(fn, dim3(grid), dim3(threads), args, lds, s);
    if (e != hipSuccess) return e;
    return hipEventRecord(last, s);
}

}  // namespace gol

#if GOL_COOP_STAMP
extern "C" int gol_debug_coop_stamps(unsigned long long* out, long long n) {
    const long long cap = (long long)gol::kStampBands * gol::kWaves * gol::kStampBlocks * 2;
    if (n > cap) n = cap;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gol::g_coop_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
