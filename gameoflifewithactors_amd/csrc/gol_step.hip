// gol_step.hip -- the hot kernel: temporal-blocked streaming step of a bit-packed board on gfx950.
//
// Replaces one or more `updateView()` ticks of the reference (GameOfLifeDriver.fs:32-34), i.e. the
// per-cell actor protocol of GameOfLifeLogic.fs:39-71 / GameofLife.fs:88-138, for all cells at once.
//
// Decomposition: one wavefront owns a column strip of 64 blocks (62 interior + one halo block per side;
// lane = block of M words, gol_layout.h) and streams down a segment of rows.  Every row loaded from HBM
// (one 4*M-byte vector load per lane) is pushed through K generations held in registers -- per
// generation level a 3-row window of horizontal row sums -- so a pass reads and writes the board once
// per K generations.  Neighbour words come from the lane's own registers (interleaved layout), the
// block-edge words from the neighbouring lanes (DPP wave_shr:1 / wave_shl:1, rotates on seam strips), bit carries
// from v_alignbit_b32, counts from v_bitop3_b32 (gol_bitlogic.h).  No workgroup barriers and no atomics: each wave is
// independent.  The deep passes (K > 1) stage the next trip's rows through the wave's own LDS slice
// (buffer_load_dword ... lds, StreamWave::stage_load), which frees the prefetch registers; the K = 1 pass keeps a
// second register buffer instead.
//
// Variants measured and removed from this file (DESIGN.md 4.1 "Negative results"; the logs stay under
// profiles/r1/): full-row workgroups with an LDS edge exchange (fullrow_sweep.log), ds_bpermute cross-lane
// moves in one or both directions (ab_xlane2.log, variant_job_ab.log), batched / late exchanges
// (ab_early.log), breadth-first levels (ab_breadth.log), per-row-pair fences (ab_fence.log), s_setprio
// fairness (tail_*.log), 8-row trips (ab_r8.log) and the no-memory / no-arithmetic ceiling builds
// (ceiling_ab.log).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "gol_bitlogic.h"
#include "gol_layout.h"
#include "gol_internal.h"

#if GOL_CHECK_BOUNDS
extern "C" unsigned gol_debug_bounds_formats(void);  // gol_formats.hip
#endif
namespace gol {

static constexpr int kWave = 64;
static constexpr int kInterior = kWave - 2;  // blocks stored per wave column strip (deep passes)
static constexpr int kSeamInterior = kWave - 1;  // ... per seam strip (torus: one lane holds both halos)
// 8 waves per workgroup: the deep passes run 2-3 waves per SIMD, so a workgroup spans the CU's SIMDs
// twice (profiles/r1/ab_fence2.log: +3-6 % at K = 16 / 32 over 4-wave workgroups)
#ifndef GOL_WAVES_PER_BLOCK
#define GOL_WAVES_PER_BLOCK 8
#endif
static constexpr int kWavesPerBlock = GOL_WAVES_PER_BLOCK;
// Waves per workgroup of a variant: 4 x the waves each SIMD holds at the kernel's register footprint, so
// ONE workgroup fills a CU and the waves sharing a SIMD (w, w + 4, w + 8) belong to the same workgroup
// (their age order is then known: see the group split in plan_stream).  (K, M) = (12, 2) runs 12-wave
// workgroups at 3 waves/SIMD (168 VGPRs; profiles/r1/w12_sweep*.log) in both torus variants and on bounded
// boards at least a strip wide (edge-fill strips: row masks only, 153 VGPRs; ragged rows, NARROW = 2, the same with
// their column-mask AND).  The NARROW = 1 bounded variant (a board narrower than one strip) also carries per-lane
// column masks in its row-mask op, which spill at that budget (185 VGPRs; round 1 measured 41k GCUPS with 12-wave
// workgroups, 74k with 8, profiles/r1/strip_bounded_sweep.log), so it keeps 8.
template <int K, int M, bool BOUNDED, bool WRAP_ROWS, int NARROW>
struct Wpb {
    static constexpr int value = NARROW != 1 && K == 12 && M == 2 ? 12 : kWavesPerBlock;
};

// Block-edge words of the neighbouring lanes, by DPP (a half-rate VALU move on gfx950,
// profiles/r1/valu_rates_gfx950.jsonl).  ds_bpermute_b32 in either direction measured 2-17 % slower under
// the level-fenced schedule below (its ~60-cycle latency; profiles/r1/ab_xlane2.log).
// ROT (torus): rotates, so lane 0's left neighbour is lane 63 -- the seam lane of a seam strip, a halo lane (whose
// outer edge is garbage anyway) otherwise.  Bounded boards shift with zero fill: the dead cells beyond the
// board's edge in the edge-fill strips.
// GOL_AB_TORUS_SHIFT, GOL_AB_NOSEAMDMA (timing studies only, WRONG boards): the torus deep pass with the bounded
// pass's zero-fill shifts instead of rotates / without its seam DMA and merge, to price each against the bounded pass
#ifndef GOL_AB_TORUS_SHIFT
#define GOL_AB_TORUS_SHIFT 0
#endif
#ifndef GOL_AB_NOSEAMDMA
#define GOL_AB_NOSEAMDMA 0
#endif
// GOL_SEAM_SMEM (round 5, default 2): the seam lane's half-blocks read by the scalar unit -- the R x M seam words of a
// trip are the same for every lane, so each row's M words come as one s_load into SGPRs -- instead of round 4's seam
// LDS-DMA and its broadcast LDS reads at the trip's top.  1: each row's s_load with the row's DMAs; 2: the next trip's
// R s_loads at the end of this trip, after its row DMAs have brought those lines (the seam block sits beside lane 0's)
// into L2.  The (12, 2) torus pass drops from 164 to 156 VGPRs.  4 interleaved rounds at the bench window, us per
// pass: 1 against the LDS seam 431.8 / 434.6 (profiles/r5/torus_seam_smem_y.jsonl), but its fills missed L2 (HBM fetch
// +13 %); 2 against 1: 431.8 / 440.3 with the fetch bytes back at the LDS seam's (torus_seam_late_z.jsonl,
// fetch_seam_smem*_z.json).  (The board buffer a pass reads is never written during it: the scalar cache, refilled
// at every dispatch, holds no stale line.)
#ifndef GOL_SEAM_SMEM
#define GOL_SEAM_SMEM 2
#endif
// GOL_AB_BSPREAD (A/B): the bounded deep passes spread their row DMAs over the levels as the torus ones do
#ifndef GOL_AB_BSPREAD
#define GOL_AB_BSPREAD 0
#endif
// GOL_AB_WRAPPTR (A/B): the single-board torus walks its rows with a running address (reset at the wrap), as the
// bounded pass does, instead of a 64-bit row multiply per row
#ifndef GOL_AB_WRAPPTR
#define GOL_AB_WRAPPTR 0
#endif
template <bool ROT>
__device__ __forceinline__ uint32_t from_left(uint32_t v) {  // lane i <- lane i-1
    if (ROT && !GOL_AB_TORUS_SHIFT) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xf, 0xf, false);  // wave_ror:1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);              // wave_shr:1
}
template <bool ROT>
__device__ __forceinline__ uint32_t from_right(uint32_t v) {  // lane i <- lane i+1
    if (ROT && !GOL_AB_TORUS_SHIFT) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xf, 0xf, false);  // wave_rol:1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);              // wave_shl:1
}

// Prefetch placement of the deep passes on seam strips (torus), GOL_SEAM_SPREAD: 0 = all R rows' DMAs at the trip's
// top (the bounded passes' placement), 1 = one row's DMAs after each of the first R generation levels, 3 = the rows'
// own-word DMAs at the top and one row's seam DMAs after each of the first R levels, 4 = row r's own-word DMAs after
// level 2r and its seam DMAs after level 2r + 1, 5 = the same every 3 levels (3r, 3r + 1); -1 (default) = 4.  Rows a short pass (K below the
// levels a mode needs) has not issued by its last level are issued after it; the pipeline-fill trips (which skip
// levels) keep every DMA at the top.  Round 3, interleaved on one box at generation 300 (profiles/r3/ab_spread_modes_i.log),
// GCUPS for modes 1 / 0 / 3 / 4: (12, 2) 114.3 / 113.4 / 113.6 / 113.8, (16, 2) 115.2 / 113.0 / 115.4 / 116.5.
// On bounded boards (no seam DMAs) spreading lost 5 % (profiles/r3/ab_spread_h.log): they keep mode 0.
// Round 4, one seam DMA per trip (GOL_SEAM1), (12, 2) at generation 300, 3 interleaved rounds (profiles/r4/
// ab_spread_o.log), us per pass for modes 1 / 0 / 3 / 4: 440.8 / 508.1 / 503.7 / 435.9 -- (12, 2) moves to mode 4;
// mode 5 against 4, 4 rounds on another box: 472.5 / 446.7 (ab_spread5_q.log).
#ifndef GOL_SEAM_SPREAD
#define GOL_SEAM_SPREAD -1
#endif
// GOL_STAMP (diagnostic builds only): every wave records its start / end time (s_memrealtime, 100 MHz)
// into g_stamps; gol_debug_stamps() copies them out (tools/tail.py measures the launch tail)
#ifndef GOL_STAMP
#define GOL_STAMP 0
#endif
#if GOL_STAMP
static constexpr int kStamps = 1 << 16;
__device__ unsigned long long g_stamps[2][kStamps];
#endif
// sched_barrier mask: every instruction class may cross except DS (0x80 all DS, 0x100 DS read, 0x200 DS write)
static constexpr int kAllButDs = 0x1 | 0x2 | 0x4 | 0x8 | 0x10 | 0x20 | 0x40 | 0x400;

// A wave-uniform 64-bit value the compiler cannot prove uniform (e.g. derived from float math), moved to SGPRs
__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t floor_mod(int64_t a, int64_t m) {
    int64_t r = a % m;
    return r < 0 ? r + m : r;
}

// Buffer-resource memory access: one uniform descriptor per row (SGPRs) + a 32-bit per-lane byte offset.
// Offsets past num_records are dropped by the hardware range check, so lanes that must not store (halo
// lanes, off-board blocks) store without a branch and every trip issues the same number of memory
// operations -- which lets the compiler wait for exactly the prefetched loads (vmcnt counts stores too).
static constexpr int kNoStore = 0x7ffffff0;  // offset beyond any row: store dropped
static constexpr int kRsrcWord3 = 0x00020000;  // raw buffer, 32-bit data format (gfx9-family)
static constexpr int kWaitVm0 = 0x0F70;        // s_waitcnt vmcnt(0) (expcnt, lgkmcnt left at max)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int M>
struct Vec;
template <>
struct Vec<1> {
    __device__ __forceinline__ static void load(__amdgpu_buffer_rsrc_t r, int off, uint32_t (&w)[1]) {
        w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    }
    __device__ __forceinline__ static void store(__amdgpu_buffer_rsrc_t r, int off, const uint32_t (&w)[1]) {
        __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, 0, 0);
    }
};
template <>
struct Vec<2> {
    __device__ __forceinline__ static void load(__amdgpu_buffer_rsrc_t r, int off, uint32_t (&w)[2]) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        w[0] = t.x;
        w[1] = t.y;
    }
    __device__ __forceinline__ static void store(__amdgpu_buffer_rsrc_t r, int off, const uint32_t (&w)[2]) {
        const u32x2 t = {w[0], w[1]};
        __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, 0);
    }
};
template <>
struct Vec<4> {
    __device__ __forceinline__ static void load(__amdgpu_buffer_rsrc_t r, int off, uint32_t (&w)[4]) {
        const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        w[0] = t.x;
        w[1] = t.y;
        w[2] = t.z;
        w[3] = t.w;
    }
    __device__ __forceinline__ static void store(__amdgpu_buffer_rsrc_t r, int off, const uint32_t (&w)[4]) {
        const u32x4 t = {w[0], w[1], w[2], w[3]};
        __builtin_amdgcn_raw_buffer_store_b128(t, r, off, 0, 0);
    }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const uint32_t* row, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(row), (short)0, (int)bytes, kRsrcWord3);
}
// GOL_CHECK_BOUNDS (diagnostic builds only, never shipped): every descriptor's [base, base + range) is checked
// against the buffer it addresses; a violation sets bit `tag` of g_bounds_err (gol_debug_bounds reads and clears it)
// and the descriptor gets range 0, so the access is dropped instead of faulting.
#ifndef GOL_CHECK_BOUNDS
#define GOL_CHECK_BOUNDS 0
#endif
#if GOL_CHECK_BOUNDS
__device__ unsigned g_bounds_err;
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t checked_rsrc(const void* base, int64_t bytes, const void* buf,
                                                               int64_t buf_bytes, int tag) {
#if GOL_CHECK_BOUNDS
    const int64_t off = (const char*)base - (const char*)buf;
    if (bytes > 0 && (off < 0 || off + bytes > buf_bytes)) {
        if ((threadIdx.x & 63) == 0)  // a vector atomic (lane-dependent branch)
            __hip_atomic_fetch_or(&g_bounds_err, 1u << tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bytes = 0;
    }
#else
    (void)buf;
    (void)buf_bytes;
    (void)tag;
#endif
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, kRsrcWord3);
}

// Rows per loop trip (even, and a multiple of 4 so register roles repeat every trip): enough loads in
// flight for the memory-bound K = 1 pass, fewer for the deep passes whose registers hold the windows.
template <int K, int M>
struct TripRows {
    static constexpr int value = (K == 1 && M == 1) ? 8 : 4;  // 8-row deep trips: -2.5 % (ab_r8.log)
};

// One wavefront's pipeline: K generation levels of 3-row windows of M-word blocks held in registers.
// NARROW = 1 on a bounded board: the board is narrower than one wave strip, so lanes can lie off the board and every
// level masks columns as well as rows.  Bounded boards at least a strip wide use edge-fill strips (no lane off
// the board) and mask rows only: the column mask and its register are compiled out -- unless NARROW = 2: a RAGGED
// bounded row (width not a multiple of the block) on edge-fill strips, whose last block holds cells past the board's
// edge (a.rag_w), so every level also ANDs the per-word column masks (all ones except on the lane holding that
// block).  On a torus NARROW = 1 is the M = 1 ragged-row variant (kRagged).
template <int K, int M, bool BOUNDED, bool WRAP_ROWS, int NARROW>
struct StreamWave {
    static constexpr int R = TripRows<K, M>::value;
    static_assert(R % 4 == 0, "slot roles must repeat every trip and registers alternate every two rows");
    using V = Vec<M>;
    // K = 1 wave strips have no halo lanes: all 64 lanes are stored, and the two words beyond the
    // strip's ends (left of lane 0, right of lane 63) are loaded from memory with the row (one extra
    // dword load per row; lanes 1-62 reload their own word, an L1 hit).  Stores are then whole
    // 64-block runs: 256 / 512 / 1024 B aligned, instead of 62-block runs at 248 B offsets
    // (profiles/r1/k1_nohalo_ab.log: 3.9-4.1 -> 4.7-5.1 TB/s).
    // RAGGED torus rows (NARROW on a torus; M = 1): the width is not a multiple of 32.  Scratch rows of
    // ceil(W / 32) words hold the cells, the last word partial (a.rag_bits cells), and the row is a ring of W cells
    // (GameOfLifeDriver.fs:21-25): the lane holding word 0 takes its west carry from bit rag_bits - 1 of the word
    // before it, the lane holding the last word its east carry at bit rag_bits - 1 from the word after it, and the
    // last word's bits past the row are cleared every generation (DESIGN.md 4.1 "Ragged rows").
    static constexpr bool kRagged = !BOUNDED && NARROW == 1;
    static constexpr bool kRagEdge = BOUNDED && NARROW == 2;  // ragged bounded rows on edge-fill strips
    static_assert(!kRagged || (M == 1 && WRAP_ROWS), "ragged rows: single boards of consecutive words");
    static constexpr bool kNoHalo = K == 1 && !kRagged;
    static constexpr int kStripBlocks = kNoHalo ? kWave : kInterior;
    // per-lane column masks: narrow (or ragged) bounded boards, and the K = 1 halo-free strips (their last strip
    // may end past the board's last block)
    // (NARROW = 2 keeps its column masks too, applied by their own AND: kRagEdge)
    static constexpr bool kColMask = BOUNDED && (NARROW == 1 || kNoHalo);

    // Seam strips (torus deep passes, a.seam): lanes 0..62 hold 63 consecutive blocks and all store; lane 63, the
    // SEAM lane, holds the first half of the block right of lane 62 (bits 0..15 of its words: cells 0..16M-1 of
    // the interleaved block) and the second half of the block left of lane 0 (bits 16..31).  With rotating DPP
    // moves the row is then a ring whose only break is in the middle of the seam lane, and the wrong cells the
    // break produces spread one cell per generation: after K <= 16M generations they have not reached either
    // end of the seam lane, so lanes 0..62 are exact.  One halo lane per wave instead of two: a 65536-cell row
    // at M = 2 is 16 seam strips plus 16 blocks, against 17 strips of 62 (DESIGN.md 4.1 "Seam strips").
#ifndef GOL_AB_NOSEAM
#define GOL_AB_NOSEAM 0
#endif
    static constexpr bool kSeam = !GOL_AB_NOSEAM && !BOUNDED && !(K == 1) && !kRagged;
    // ONE seam DMA per trip (round 4): a global_load_lds_dword with a per-lane address, lane i loading word i % M of
    // the block left of lane 0 in row (i / M) % R of the trip; the R x M words land side by side in a 64-dword LDS
    // slot, which every lane then reads as a broadcast and only the seam lane merges (`hmask`).  Round 3 issued M
    // DMAs per row (every lane reloading its own word, a cache hit, so that one lane in 64 got its half-block): twice
    // the bounded pass's VMEM and LDS instructions (SQ_INSTS_VMEM_RD / SQ_INSTS_LDS 1.93x, profiles/r3/pmc_sq).
#ifndef GOL_SEAM1
#define GOL_SEAM1 1
#endif
    static constexpr bool kSeam1 = kSeam && GOL_SEAM1;
    // Deep passes (K > 1) stage their prefetched rows through LDS (see `stage` below); the K = 1 pass keeps two
    // register buffers (it has registers to spare, and its halo-free strips load a neighbour word per row).
    static constexpr bool kStage = !kNoHalo;

    const uint32_t* __restrict__ src;
    uint32_t* __restrict__ dst;
    const StreamArgs& a;
    int load_off;      // this lane's byte offset in a row (its block column; remainder waves: plus its sub-strip's rows)
    int store_off;     // = load_off for interior on-board lanes, kNoStore otherwise
    uint32_t colmask[M];  // kColMask: per word of the lane's block, its cells on the board (~0 inside, 0 off it)
    int64_t row_bytes;
    int64_t span_bytes;  // bytes a row descriptor covers: the row, or (remainder waves) every sub-strip's row
    // kStage: rows are prefetched straight to LDS (buffer_load_dword ... lds), not to registers: a second prefetch
    // buffer of R x M VGPRs -- with the seam lane's extra half-block -- spilled the (12, 2) pass at its 168-VGPR
    // budget.  The trip reads its rows back at its top, after the wait, so a bounded board's row masks apply there
    // and never make a trip wait for its own prefetch.  kSeam: per row and word a second dword load lands in the
    // stage, the word at seam_off -- for the seam lane the block left of lane 0, for every other lane its own word
    // again (a cache hit) -- and each lane takes the high half of its word from it: a no-op except on the seam lane.
    int seam_off = 0;
    // M dword LDS-DMAs per row and kind.  (One dwordx3 DMA per row at M = 2 -- there is no dwordx2 form -- saves 8
    // instructions per trip but strides the stage 12 bytes per lane: the LDS reads then need more address registers
    // than the (12, 2) pass has, and it spilled.)
    static constexpr int kDmaWords = 1;  // dwords per lane per DMA
    static constexpr int kDmas = M;      // DMAs per row and kind
    using Stage = uint32_t[2][kSeam && !kSeam1 ? 2 : 1][R][kDmas][kWave * kDmaWords];  // [parity][row, seam][row][dma][lane x words]
    Stage* stage = nullptr;
    // kSeam1: the per-trip seam slot [parity][lane], this lane's row (relative to the trip's first) and byte offset in
    // the seam DMA, and the seam lane's merge mask (0xffff0000 on the seam lane of a seam strip, 0 elsewhere: remainder
    // waves and halo-lane strips merge nothing)
    using SeamStage = uint32_t[2][kWave];
    SeamStage* seam1 = nullptr;
    // GOL_SEAM_SMEM: the next trip's seam words (SGPRs), the seam column's byte offset in a row, and whether this wave
    // merges a seam (a seam strip, not a remainder wave)
    static constexpr bool kSmem = kSeam1 && GOL_SEAM_SMEM;
    struct SmemSeam {
        uint32_t s[R][M];
        int64_t col;  // in words
        bool on;
        int64_t row[R];  // GOL_SEAM_SMEM 2: the buffer rows of the next trip, loaded at the trip's end
    };
    struct NoSmem {};
    [[no_unique_address]] typename std::conditional<kSmem, SmemSeam, NoSmem>::type sm;
    int seam1_delta = 0;  // (lane / M) % R rows + the word (lane % M) of the block left of lane 0, in bytes
    uint32_t hmask = 0;
    template <int WORDS>
    __device__ __forceinline__ static void dma(__amdgpu_buffer_rsrc_t rs, uint32_t* lds, int off) {
        auto* p = (__attribute__((address_space(3))) void*)lds;
        if constexpr (WORDS == 3)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, p, 12, off, 0, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, p, 4, off, 0, 0, 0);
    }
    __device__ __forceinline__ uint32_t staged(int par, int kind, int r, int j, int lane) const {
        return kDmas == 1 ? (*stage)[par][kind][r][0][lane * kDmaWords + j] : (*stage)[par][kind][r][j][lane];
    }
    int64_t seg_begin, seg_end, nsteps, ly0;
    __device__ __forceinline__ int64_t buf_bytes() const { return (a.rows + 2 * a.ghost) * a.pitch * 4; }
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t src_rs(const uint32_t* base, int64_t bytes, int tag) const {
        return checked_rsrc(base, bytes, src, buf_bytes(), tag);
    }
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t dst_rs(const void* base, int64_t bytes, int tag) const {
        return checked_rsrc(base, bytes, dst, buf_bytes(), tag);
    }
    // kStage walks, wave-uniform (SGPRs): a bounded board's next row to load (byte address and step index; rows
    // outside [step_lo, step_hi] load nothing), and every variant's next output row to store (byte address and step
    // relative to seg_begin)
    uint64_t lptr = 0, sptr = 0;
    int lrow = 0, sd = 0;
    int64_t load_br;  // wrap: buffer row of the next level-0 row to load; else buffer row of step 0 (uniform)
    int seglen = 0, step_lo = 0, step_hi = 0, mrow_lo = 0, mrow_hi = 0;
    bool edge_fill = false;  // bounded: strips placed so that no lane is off the board (constructor)

    // Bounded boards: trips [t_top, t_bot) produce no row off the board at any level (trip t produces the rows
    // of steps t*R - K .. t*R + R - 2) and run the unmasked arithmetic of the torus strips; the others mask
    // the rows off the board dead at every level.  A board narrower than a strip (no edge-fill strips) masks
    // its columns in every trip: t_top = t_bot = 0.  Wave-uniform (the bounds are loop limits: a lane-varying
    // exit would turn the trip loop into a divergent loop).
    int t_top = 0, t_bot = 0;

    // level state: two row slots (X, Y) of block row sums (s, c) and the raw centre block of slot Y
    uint32_t sX[K][M], cX[K][M], sY[K][M], cY[K][M], aY[K][M];

    // K = 1 halo-free strips: byte offset of this lane's neighbour word, and its bounded-board mask
    int nb_off = 0;
    uint32_t nbmask = 0xffffffffu;
    // kRagged: west carry shift (32 - rag_bits on the lane holding word 0), east carry position (rag_bits - 1 on
    // the lane holding the last word, else 31) and the cells of the lane's word on the row
    uint32_t rag_shw = 0, rag_she = 31, rag_mask = 0xffffffffu;
    // kRagEdge: this wave holds the ragged row's partial block (wave-uniform)
    bool rag_wave = false;

    // First row (relative to the group segment of `len` rows) of the i-th oldest wave's share.  Shares
    // fall geometrically with age, ratio rho = (1 - f) / f (f = a.split / 65536 = the oldest wave's share
    // of a pair), applied to each wave's streamed rows (its share plus the 2K-row pipeline fill).
    __device__ __forceinline__ int64_t group_cut(int64_t len, int i) const {
        constexpr int n = Wpb<K, M, BOUNDED, WRAP_ROWS, NARROW>::value / 4;
        if (i <= 0) return 0;
        if (i >= n) return len;
        const float f = (float)a.split * (1.0f / 65536.0f);
        const float rho = (1.0f - f) / f;
        // a.split2 (three-wave groups): the middle wave's share of the two younger waves' rows, so the ratio between
        // the youngest and the middle wave is set apart from the one between the middle and the oldest
        const float f2 = a.split2 > 0 ? (float)a.split2 * (1.0f / 65536.0f) : f;
        const float rho2 = (1.0f - f2) / f2;
        float pw = 1.0f, sum = 0.0f, head = 0.0f;
        for (int j = 0; j < n; j++) {
            if (j == i) head = sum;
            sum += pw;
            pw *= j == 0 ? rho : rho2;
        }
        const float total = (float)(len + 2 * K * n);
        int64_t cut = (int64_t)(total * head / sum + 0.5f) - 2 * K * i;
        return cut < 0 ? 0 : (cut > len ? len : cut);
    }

    // Bounded boards: the cells of word j of block cb that lie on the board -- all of an inside block, none of an
    // outside one, and of a ragged row's last block (a.rag_w cells per row, Script.fsx:6-13) the cells x < rag_w
    // (word j bit b is cell 32 M cb + j + M b, gol_layout.h)
    __device__ __forceinline__ uint32_t cell_mask(int64_t cb, int j, int64_t nblocks) const {
        if (cb < 0 || cb >= nblocks) return 0u;
        if (!a.rag_w) return 0xffffffffu;
        const int64_t left = a.rag_w - 32 * M * cb - j;  // cells from this word's first cell to the row's end
        const int64_t nbits = left <= 0 ? 0 : (left + M - 1) / M;
        return nbits >= 32 ? 0xffffffffu : (1u << nbits) - 1u;
    }

    // `lane`: lane within the wave's strip.  `role`: -1 = the wave owns segment sy; 0, 1, ... = the
    // oldest, next, ... wave of the SIMD group sharing group segment sy (split by a.split, see plan_stream)
    // `rem_count` > 0: a remainder wave of the seam geometry whose lanes hold rem_count sub-strips of (a.rem + 2)
    // lanes, sub-strip j on segment sy + j (all of length a.seg); 0: a strip sx of segment sy.
    __device__ __forceinline__ StreamWave(const uint32_t* s, uint32_t* d, const StreamArgs& args, int lane,
                                          int64_t sx, int64_t sy, int role = -1, int rem_count = 0)
        : src(s), dst(d), a(args) {
        const int64_t nblocks = a.words / M;
        row_bytes = a.words * 4;
        span_bytes = row_bytes;
        // Bounded boards at least a strip wide (edge-fill strips): the first strip starts at the board's first
        // block and the last ends at its last block, so the dead cells beyond the left / right edge arrive as
        // the zeros the DPP moves write into lanes 0 / 63 (bound_ctrl), and no lane is ever off the board --
        // no column mask at any level.  Interior strips overlap by two blocks as on a torus (halo lanes).
        // this lane's block column (may be off-board)
        int64_t cb = kNoHalo ? sx * kWave + lane : sx * kInterior - 1 + lane;
        if constexpr (BOUNDED && !kNoHalo && NARROW != 1) {  // the host picks NARROW = 1 exactly when nblocks < kWave
            edge_fill = true;
            cb = (sx == a.nstrips - 1 ? nblocks - kWave : sx * kInterior) + lane;
        }
        int64_t lc;
        if (BOUNDED) {
            const bool in = cb >= 0 && cb < nblocks;
#pragma unroll
            for (int j = 0; j < M; j++) colmask[j] = cell_mask(cb, j, nblocks);
            if constexpr (kRagEdge) {
                bool part = false;
#pragma unroll
                for (int j = 0; j < M; j++) part = part || colmask[j] != 0xffffffffu;
                rag_wave = __builtin_amdgcn_ballot_w64(part) != 0;
            }
            lc = in ? cb : 0;
        } else if (kRagged) {
            // strips of 62 stored words over the ring positions -o .. nw - 1 - o (o = a.rag_origin: 1, or 2 when
            // the last strip's right halo lane would be the partial word), so the partial word is never a halo
            // lane next to a stored lane (its few cells could not carry a K-deep halo): strip sx, lane l holds
            // position 62 sx + l - 1 - o
            const int64_t p = sx * kInterior + lane - 1 - a.rag_origin;
            lc = floor_mod(p, nblocks);
#pragma unroll
            for (int j = 0; j < M; j++) colmask[j] = 0xffffffffu;
            cb = p;
            rag_shw = lc == 0 ? 32u - (uint32_t)a.rag_bits : 0u;
            rag_she = lc == nblocks - 1 ? (uint32_t)a.rag_bits - 1u : 31u;
            rag_mask = lc == nblocks - 1 ? (1u << a.rag_bits) - 1u : 0xffffffffu;
        } else {
#pragma unroll
            for (int j = 0; j < M; j++) colmask[j] = 0xffffffffu;
            lc = floor_mod(cb, nblocks);
        }
        load_off = (int)(lc * 4 * M);
        if (kNoHalo) {
            store_off = cb < nblocks ? load_off : kNoStore;
            // lane 0: last word of the block to the left; lane 63: first word of the block to the right
            const int64_t nbc = lane == 0 ? cb - 1 : (lane == kWave - 1 ? cb + 1 : lc);
            const int nbw = lane == 0 ? M - 1 : 0;
            int64_t nl;
            if (BOUNDED) {
                const bool in = nbc >= 0 && nbc < nblocks;
                nbmask = cell_mask(nbc, nbw, nblocks);
                nl = in ? nbc : 0;
            } else {
                nbmask = 0xffffffffu;
                nl = floor_mod(nbc, nblocks);
            }
            nb_off = (int)((nl * M + nbw) * 4);
        } else if (BOUNDED && edge_fill) {  // lane 0 is a halo lane unless it is the board's first block, lane 63 unless the last
            store_off = ((lane >= 1 || sx == 0) && (lane <= kInterior || sx == a.nstrips - 1)) ? load_off : kNoStore;
        } else if (kRagged) {
            store_off = (lane >= 1 && lane <= kInterior && cb <= nblocks - 1 - a.rag_origin) ? load_off : kNoStore;
        } else {
            store_off = (lane >= 1 && lane <= kInterior && cb < nblocks) ? load_off : kNoStore;
        }
        if constexpr (kSeam) {
            if (a.seam && rem_count == 0) {  // seam strip sx: blocks 63 sx .. 63 sx + 62, then the seam lane
                const int64_t b = sx * kSeamInterior + lane;
                if (lane < kSeamInterior) {
                    load_off = store_off = (int)(floor_mod(b, nblocks) * 4 * M);
                } else {
                    load_off = (int)(floor_mod(b, nblocks) * 4 * M);                          // right of lane 62
                    seam_off = (int)(floor_mod(sx * kSeamInterior - 1, nblocks) * 4 * M);     // left of lane 0
                    store_off = kNoStore;
                }
            } else if (a.seam) {  // remainder wave: sub-strip j = lane / (rem + 2) on segment sy + j
                const int q = a.rem + 2;
                const int j = lane / q, i = lane - j * q;
                const int64_t b = a.nstrips * kSeamInterior - 1 + i;  // halo, the rem remainder blocks, halo
                const int64_t delta = (int64_t)j * a.seg * a.pitch * 4;  // this sub-strip's rows (bytes)
                load_off = (int)(floor_mod(b, nblocks) * 4 * M + (j < rem_count ? delta : 0));
                store_off = (j < rem_count && i >= 1 && i <= a.rem) ? load_off : kNoStore;
                span_bytes = (int64_t)(rem_count - 1) * a.seg * a.pitch * 4 + row_bytes;
            }
            if (lane < kSeamInterior || !a.seam || rem_count) seam_off = load_off;
            if constexpr (kSeam1) {
                seam1_delta = (int)(((lane / M) % R) * a.pitch * 4) + 4 * (lane % M) +
                              (a.seam && rem_count == 0 ? (int)(floor_mod(sx * kSeamInterior - 1, nblocks) * 4 * M) : 0);
                hmask = a.seam && rem_count == 0 && lane == kWave - 1 ? 0xffff0000u : 0u;
                if constexpr (kSmem) {
                    sm.on = a.seam && rem_count == 0;
                    sm.col = sm.on ? floor_mod(sx * kSeamInterior - 1, nblocks) * M : 0;
#pragma unroll
                    for (int r = 0; r < R; r++)
#pragma unroll
                        for (int j = 0; j < M; j++) sm.s[r][j] = 0u;
                }
            }
        }
        seg_begin = a.out_begin + sy * a.seg;
        seg_end = seg_begin + a.seg < a.out_end ? seg_begin + a.seg : a.out_end;
        if (role >= 0) {  // group segment: wave `role` (0 = oldest) takes its share, in age order
            const int64_t len = seg_end - seg_begin;
            const int64_t b0 = seg_begin;
            seg_begin = b0 + group_cut(len, role);
            seg_end = b0 + group_cut(len, role + 1);
            if (!WRAP_ROWS || kStage) {
                // the group cut is float VALU math: without this the segment bounds live in 8 VGPRs, and
                // the ghost-row variant spills at the 3-waves/SIMD budget (a scratch reload every loop
                // trip; profiles/r1/ab_uniform.log: strip K = 12 86k -> 97k GCUPS); on a bounded board the
                // per-level row masks then stay scalar (s_cmp / s_cselect) instead of 64-bit VALU compares
                // and v_cndmask.  The single-board torus variant loses 4-8 % with it (its register
                // allocation changes), so it keeps VGPR bounds.
                seg_begin = uniform64(seg_begin);
                seg_end = uniform64(seg_end);
            }
        }
        nsteps = (seg_end - seg_begin) + 2 * K;  // level-0 rows streamed
        if (BOUNDED || kStage) seglen = (int)(seg_end - seg_begin);  // < 2^30 (plan_stream)
        ly0 = seg_begin - K;                     // level-0 row of step 0
        load_br = WRAP_ROWS ? floor_mod(ly0, a.rows) : ly0 + a.ghost;
        if (BOUNDED) {  // steps whose row lies on the board: global row a.y0 + ly0 + st in [0, height)
            const int64_t lo = -(a.y0 + ly0), hi = a.height - (a.y0 + ly0);
            const int64_t cap = (int64_t)1 << 30;
            mrow_lo = (int)(lo < -cap ? -cap : (lo > cap ? cap : lo));
            mrow_hi = (int)(hi < -cap ? -cap : (hi > cap ? cap : hi));
        }
        if (BOUNDED && edge_fill) {
            // first trip whose lowest produced row is on the board: t*R - K >= mrow_lo; first trip whose
            // highest is off it: t*R + R - 2 >= mrow_hi
            const int up = mrow_lo + K, dn = mrow_hi - R + 2;
            t_top = up <= 0 ? 0 : (up + R - 1) / R;
            t_bot = dn <= 0 ? 0 : (dn + R - 1) / R;
        }
        if (BOUNDED) {
            // steps whose level-0 row lies in the buffer, as 32-bit step indices: the per-row clamp below is
            // then 32-bit scalar arithmetic (the scalar unit has no 64-bit ordered compare)
            const int64_t lo = -load_br, hi = a.rows + 2 * a.ghost - 1 - load_br;
            const int64_t cap = (int64_t)1 << 30;
            step_lo = (int)(lo < -cap ? -cap : (lo > cap ? cap : lo));
            step_hi = (int)(hi < -cap ? -cap : (hi > cap ? cap : hi));
        }
        if constexpr (kStage) {
            const uint64_t pitch_bytes = (uint64_t)a.pitch * 4;
            if (BOUNDED || (GOL_AB_WRAPPTR && WRAP_ROWS))
                lptr = (uint64_t)(uintptr_t)src + (uint64_t)load_br * pitch_bytes;  // (bounded: may precede the buffer)
            sd = -R - 2 * K;  // the first store (at trip 0's top) is trip -1's: nothing valid
            sptr = (uint64_t)(uintptr_t)dst + (uint64_t)((WRAP_ROWS ? 0 : a.ghost) + seg_begin + sd) * pitch_bytes;
        }
#pragma unroll
        for (int g = 0; g < K; g++)
#pragma unroll
            for (int j = 0; j < M; j++) sX[g][j] = cX[g][j] = sY[g][j] = cY[g][j] = aY[g][j] = 0;
    }

    // Load the next R level-0 rows into `buf` (bounded boards and the K = 1 pass).  Loads are unconditional
    // (addresses clamped, values masked) so every trip issues a fixed number of memory operations and the compiler
    // waits for exactly the loads.
    __device__ __forceinline__ void load(uint32_t (&buf)[R][M], uint32_t (&nb)[R], int64_t first_step) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            int64_t br = load_br;
            if (WRAP_ROWS) {
                load_br = br + 1 == a.rows ? 0 : br + 1;
            } else if (BOUNDED) {
                // rows outside the buffer (beyond a bounded board's edge, or past the segment's last
                // step) are never used unmasked: clamp the address into the buffer (32-bit step indices,
                // scalar; load_br stays the buffer row of step 0)
                int st = (int)first_step + r;
                st = st < step_lo ? step_lo : (st > step_hi ? step_hi : st);
                br = load_br + st;
            } else {
                // ghost-row strips: the same clamp on 64-bit rows (this variant's measured instruction stream)
                const int64_t buf_rows = a.rows + 2 * a.ghost;
                load_br = br + 1;
                br = br < 0 ? 0 : (br < buf_rows ? br : buf_rows - 1);
            }
            V::load(src_rs(src + br * a.pitch, span_bytes, 1), load_off, buf[r]);
            if (kNoHalo) nb[r] = __builtin_amdgcn_raw_buffer_load_b32(src_rs(src + br * a.pitch, row_bytes, 2), nb_off, 0, 0);
            if (BOUNDED) {
                const uint32_t rm = row_mask((int)first_step + r);
#pragma unroll
                for (int j = 0; j < M; j++) buf[r][j] = kColMask ? lut3<0x80>(buf[r][j], colmask[j], rm) : buf[r][j] & rm;
                if (kNoHalo) nb[r] = lut3<0x80>(nb[r], nbmask, rm);
            }
        }
    }

    // Bounded boards: all-ones if the row of step `st` (level-0 row ly0 + st, or at level g the row it produces)
    // is on the board, else 0.  32-bit step bounds set up once (the scalar unit has no 64-bit ordered compare;
    // a 64-bit one goes to the VALU as v_cmp_*_u64 + v_cndmask per row and level), wave-uniform.
    __device__ __forceinline__ uint32_t row_mask(int st) const {
        return (st >= mrow_lo && st < mrow_hi) ? 0xffffffffu : 0u;
    }

    // kStage: prefetch the next R level-0 rows into stage parity PAR.  A bounded board walks a running address (two
    // scalar adds per row instead of a clamp and a 64-bit multiply); its rows outside the buffer get an empty
    // descriptor, so their loads return zeros that nothing uses unmasked.  The torus and ghost-row strips keep the
    // row-index walk (wrap at the board's last row; clamp to the strip's buffer): the running address there measured
    // 8 % slower on the (12, 2) torus with an instruction stream that differs only in scalar order
    // (profiles/r3/ab_torus_load_addr.log, "new" vs "wl").
    template <int PAR>
    __device__ __forceinline__ void stage_load() {
#pragma unroll
        for (int r = 0; r < R; r++) stage_load_row<PAR, 3>(r);
    }
    // KINDS: 1 = the row's own-word DMAs (advancing the row walk; the descriptor is kept for the seam DMAs), 2 = its
    // seam DMAs (kept descriptor), 3 = both
    __amdgpu_buffer_rsrc_t row_rs[R];
    // kSeam1: the trip's one seam DMA, issued with its first row (buffer row br0, wave-uniform): lane i loads from row
    // br0 + (i / M) % R through a range-checked descriptor based at row br0.  Ghost-row strips: rows past the buffer
    // (only the tail trip's unused rows) read as 0.  Single board: a trip whose rows wrap past the board's last row
    // (first and last segments) splits the lanes -- rows before the wrap from the descriptor at br0, the others from
    // one based at row 0 -- so every lane reads its row.  No per-lane 64-bit address is formed.
    template <int PAR>
    __device__ __forceinline__ void stage_load_seam1(int64_t br0) {
        const int64_t pb = a.pitch * 4;
        uint32_t* lds = &(*seam1)[PAR][0];
        const uint32_t* base = src + br0 * a.pitch;
        if (WRAP_ROWS) {
            if (br0 + R <= a.rows) {
                dma<1>(src_rs(base, R * pb, 3), lds, seam1_delta);
            } else {
                const int n1 = (int)((a.rows - br0) * pb);  // bytes of the rows before the wrap (>= one row)
                if (seam1_delta < n1)
                    dma<1>(src_rs(base, n1, 4), lds, seam1_delta);
                else
                    dma<1>(src_rs(src, R * pb, 5), lds, seam1_delta - n1);
            }
        } else {
            const int64_t left = (a.rows + 2 * a.ghost - br0) * pb;
            dma<1>(src_rs(base, left < R * pb ? left : R * pb, 6), lds, seam1_delta);
        }
    }
    // GOL_SEAM_SMEM: one scalar load of row r's M seam words (wave-uniform address)
    __device__ __forceinline__ void smem_seam_row(int r, int64_t br) {
        if constexpr (kSmem) {
            typedef uint32_t su32xM __attribute__((ext_vector_type(M)));
            const auto* q = (const __attribute__((address_space(4))) su32xM*)(uintptr_t)(src + br * a.pitch + sm.col);
            const su32xM x = *q;
#pragma unroll
            for (int j = 0; j < M; j++) sm.s[r][j] = x[j];
        }
    }
    // GOL_SEAM_SMEM 2: the next trip's seam words at the end of this trip, when its row DMAs have filled the lines
    __device__ __forceinline__ void smem_seam_late() {
        if constexpr (kSmem && GOL_SEAM_SMEM == 2) {
            if (sm.on) {
#pragma unroll
                for (int r = 0; r < R; r++) smem_seam_row(r, sm.row[r]);
            }
        }
    }
    template <int PAR, int KINDS>
    __device__ __forceinline__ void stage_load_row(int r) {
        if constexpr ((KINDS & 1) == 0) {
#pragma unroll
            for (int d = 0; d < kDmas; d++)
                if constexpr (kSeam && !kSeam1) dma<kDmaWords>(row_rs[r], &(*stage)[PAR][kSeam ? 1 : 0][r][d][0], seam_off + 4 * d);
        } else {
            __amdgpu_buffer_rsrc_t rs;
            if constexpr (BOUNDED) {
                const bool inside = lrow >= step_lo && lrow <= step_hi;
                rs = src_rs(reinterpret_cast<const uint32_t*>(lptr), inside ? span_bytes : 0, 7);
                lptr += (uint64_t)a.pitch * 4;
                lrow++;
            } else {
                int64_t br = load_br;
                [[maybe_unused]] const uint64_t p = lptr;
                if (WRAP_ROWS) {
                    load_br = br + 1 == a.rows ? 0 : br + 1;
                    if constexpr (GOL_AB_WRAPPTR) lptr = load_br == 0 ? (uint64_t)(uintptr_t)src : p + (uint64_t)a.pitch * 4;
                } else {
                    const int64_t buf_rows = a.rows + 2 * a.ghost;
                    load_br = br + 1;
                    br = br < 0 ? 0 : (br < buf_rows ? br : buf_rows - 1);
                }
                rs = src_rs(GOL_AB_WRAPPTR && WRAP_ROWS ? reinterpret_cast<const uint32_t*>(p) : src + br * a.pitch, span_bytes, 8);
                if constexpr (kSmem && GOL_SEAM_SMEM == 2) {
                    sm.row[r] = br;
                } else if constexpr (kSmem) {
                    if (sm.on) smem_seam_row(r, br);
                } else if constexpr (kSeam1 && !GOL_AB_NOSEAMDMA) {
                    if (r == 0) stage_load_seam1<PAR>(br);
                }
            }
            if constexpr ((KINDS & 2) == 0 && !kSeam1) row_rs[r] = rs;
#pragma unroll
            for (int d = 0; d < kDmas; d++) {
                dma<kDmaWords>(rs, &(*stage)[PAR][0][r][d][0], load_off + 4 * d);
                if constexpr (kSeam && !kSeam1 && (KINDS & 2))
                    dma<kDmaWords>(rs, &(*stage)[PAR][kSeam ? 1 : 0][r][d][0], seam_off + 4 * d);
            }
        }
    }
    // kStage, after the wait for stage parity PAR and the previous trip's stores: read the trip's words from the stage
    // straight into the row buffer (and the seam words), before the next prefetch is issued, so the LDS latency
    // hides behind it ...
    struct Seam {
        uint32_t s[kSeam ? R : 1][M];
    };
    // kStage: store the previous trip's R output rows (running store address; rows outside the segment -- the
    // pipeline fill and the tail -- get an empty descriptor and are dropped)
    __device__ __forceinline__ void store_staged(const uint32_t (&v)[R][M]) {
        const uint64_t pitch_bytes = (uint64_t)a.pitch * 4;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int d = sd + r;
            const bool valid = d >= 0 && d < seglen;
            V::store(dst_rs(reinterpret_cast<void*>(sptr + r * pitch_bytes), valid ? span_bytes : 0, 9),
                     store_off, v[r]);
        }
        sptr += R * pitch_bytes;
        sd += R;
    }
    template <int PAR>
    __device__ __forceinline__ void stage_read(uint32_t (&v)[R][M], int lane) {
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int j = 0; j < M; j++) v[r][j] = staged(PAR, 0, r, j, lane);
    }
    template <int PAR>
    __device__ __forceinline__ void stage_read_seam(Seam& t, int lane) {
        if constexpr (kSeam1 && GOL_AB_NOSEAMDMA) {
        } else if constexpr (kSmem) {
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int j = 0; j < M; j++) t.s[r][j] = sm.s[r][j];
        } else if constexpr (kSeam1) {  // the same R x M words for every lane (a broadcast read)
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int j = 0; j < M; j++) t.s[r][j] = (*seam1)[PAR][r * M + j];
        } else if constexpr (kSeam) {
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int j = 0; j < M; j++) t.s[r][j] = staged(PAR, kSeam ? 1 : 0, r, j, lane);
        }
    }
    // ... and make them the rows of steps first_step ..: kSeam, each word's high half from the seam word; bounded, rows
    // off the board (and, NARROW, columns off it) dead (Script.fsx:11).
    __device__ __forceinline__ void stage_in(uint32_t (&v)[R][M], const Seam& t, int64_t first_step) {
        (void)first_step;
        (void)t;
#pragma unroll
        for (int r = 0; r < R; r++) {
            [[maybe_unused]] uint32_t rm = 0xffffffffu;
            if constexpr (BOUNDED) rm = row_mask((int)first_step + r);
#pragma unroll
            for (int j = 0; j < M; j++) {
                if constexpr (kSeam1 && GOL_AB_NOSEAMDMA)
                    ;
                else if constexpr (kSeam1)
                    v[r][j] = lut3<0xD8>(hmask, t.s[kSeam ? r : 0][j], v[r][j]);
                else if constexpr (kSeam)
                    v[r][j] = lut3<0xD8>(0xffff0000u, t.s[kSeam ? r : 0][j], v[r][j]);
                else if constexpr (BOUNDED)
                    v[r][j] = kColMask || kRagEdge ? lut3<0x80>(v[r][j], colmask[j], rm) : v[r][j] & rm;
            }
        }
    }

    // One level, one row: window (prev P, centre C) + new row v -> next generation of the C row.
    // The new row's sums overwrite the P slot (it becomes the centre slot of the following row).
    template <bool MASK>
    __device__ __forceinline__ void level_row(uint32_t (&v)[M], uint32_t left, uint32_t right, uint32_t (&sP)[M],
                                              uint32_t (&cP)[M],
                                              const uint32_t (&sC)[M], const uint32_t (&cC)[M],
                                              const uint32_t (&alC)[M], uint32_t rowmask, uint32_t (&out)[M]) {
        uint32_t sN[M], cN[M];
        if constexpr (kRagged) {  // the ring closes at bit level between the last word and word 0
            const uint32_t w = align_right(v[0], left << rag_shw, 31);
            const uint32_t e = (right << rag_she) | (v[0] >> 1);  // v[0]'s bits past the row are clear
            sN[0] = lut3<0x96>(w, v[0], e);
            cN[0] = lut3<0xE8>(w, v[0], e);
        } else {
            row_sum_block<M>(v, left, right, sN, cN);
        }
#pragma unroll
        for (int j = 0; j < M; j++) {
            out[j] = life_next(sP[j], cP[j], sC[j], cC[j], sN[j], cN[j], alC[j]);
            if (kRagged) out[j] &= rag_mask;
            if (BOUNDED && MASK) out[j] = kColMask ? lut3<0x80>(out[j], colmask[j], rowmask) : out[j] & rowmask;  // dead off the board
            sP[j] = sN[j];
            cP[j] = cN[j];
        }
    }

    // Push R rows (steps t*R .. t*R+R-1) through the K levels; v[r] becomes row (ly0 + t*R + r - K) of
    // generation K.  SKIP: leave out levels whose inputs in this trip are all pipeline fill (garbage).
    template <bool SKIP, bool MASK, typename Hook>
    __device__ __forceinline__ void process(uint32_t (&v)[R][M], const uint32_t (&nb)[R], int64_t t, Hook&& hook) {
        [[maybe_unused]] const int64_t lyt = ly0 + t * R;
        if constexpr (kNoHalo) {  // K = 1: lanes 0 / 63 keep the loaded neighbour word (bound_ctrl off)
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
                if (BOUNDED && MASK) {
                    m0 = row_mask((int)t * R + r - 1);
                    m1 = row_mask((int)t * R + r);
                }
                const uint32_t l0 = (uint32_t)__builtin_amdgcn_update_dpp((int)nb[r], (int)v[r][M - 1], 0x138, 0xf, 0xf, false);
                const uint32_t r0 = (uint32_t)__builtin_amdgcn_update_dpp((int)nb[r], (int)v[r][0], 0x130, 0xf, 0xf, false);
                const uint32_t l1 =
                    (uint32_t)__builtin_amdgcn_update_dpp((int)nb[r + 1], (int)v[r + 1][M - 1], 0x138, 0xf, 0xf, false);
                const uint32_t r1 =
                    (uint32_t)__builtin_amdgcn_update_dpp((int)nb[r + 1], (int)v[r + 1][0], 0x130, 0xf, 0xf, false);
                uint32_t o0[M], o1[M];
                level_row<MASK>(v[r], l0, r0, sX[0], cX[0], sY[0], cY[0], aY[0], m0, o0);
                level_row<MASK>(v[r + 1], l1, r1, sY[0], cY[0], sX[0], cX[0], v[r], m1, o1);
#pragma unroll
                for (int j = 0; j < M; j++) {
                    aY[0][j] = v[r + 1][j];
                    v[r][j] = o0[j];
                    v[r + 1][j] = o1[j];
                }
            }
            return;
        }
        // Level g+1's right-hand exchange is issued as soon as level g has produced the row, and a full
        // scheduling barrier separates the levels: without it the scheduler interleaves levels and the
        // live register set grows past the occupancy steps (K = 16, M = 2: 256 VGPRs, 1 wave/SIMD; with
        // it 213, 2 waves/SIMD; profiles/r1/ab_early.log, ab_fence2.log).
        uint32_t right[R];
#pragma unroll
        for (int r = 0; r < R; r++) right[r] = from_right<!BOUNDED>(v[r][0]);
#pragma unroll
        for (int g = 0; g < K; g++) {
            if (SKIP && t * R + R - 1 < 2 * g) continue;  // level g's inputs are valid from step 2g on (SKIP: no hook)
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
                if (BOUNDED && MASK) {  // cells outside the board stay dead at every generation (Script.fsx:11)
                    m0 = row_mask((int)t * R + r - g - 1);  // row produced from v[r] at level g + 1
                    m1 = row_mask((int)t * R + r - g);
                }
                // even row: window (X = row-2, Y = row-1) -> X;  odd row: (Y, X) -> Y
                uint32_t o0[M], o1[M];
                level_row<MASK>(v[r], from_left<!BOUNDED>(v[r][M - 1]), right[r], sX[g], cX[g], sY[g], cY[g], aY[g], m0, o0);
                level_row<MASK>(v[r + 1], from_left<!BOUNDED>(v[r + 1][M - 1]), right[r + 1], sY[g], cY[g], sX[g], cX[g],
                                v[r], m1, o1);
#pragma unroll
                for (int j = 0; j < M; j++) {
                    aY[g][j] = v[r + 1][j];
                    v[r][j] = o0[j];
                    v[r + 1][j] = o1[j];
                }
                if (g + 1 < K) {
                    right[r] = from_right<!BOUNDED>(o0[0]);
                    right[r + 1] = from_right<!BOUNDED>(o1[0]);
                    __builtin_amdgcn_sched_barrier(kAllButDs);
                }
            }
            if constexpr (kRagEdge) {
                // a ragged row's cells past its end, dead at every level: only the wave holding the partial block
                // masks (one uniform branch per level; the other waves run the NARROW = 0 arithmetic).  After the
                // level, before the next one reads its rows: within a level only its inputs are read, and the
                // neighbour words already sent on (`right`) carry the partial block's cell 0, which is on the board.
                // (Round 4 ANDed every word of every wave at every level, in the row mask's 3-input op: the
                // (12, 2) pass needed 172 VGPRs and spilled 4 at its 168-VGPR budget.)
                // (in place, written out: a C++ AND made the compiler move the rows between registers on the
                // other path to join the two)
                if (rag_wave) {
#pragma unroll
                    for (int r = 0; r < R; r++)
#pragma unroll
                        for (int j = 0; j < M; j++) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[r][j]) : "v"(colmask[j]));
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // level g+1 may not be hoisted next to its exchanges
            hook(g);
        }
    }
    template <bool SKIP, bool MASK>
    __device__ __forceinline__ void process(uint32_t (&v)[R][M], const uint32_t (&nb)[R], int64_t t) {
        process<SKIP, MASK>(v, nb, t, [](int) {});
    }

    __device__ __forceinline__ void store_row(const uint32_t (&v)[M], int64_t row, bool valid) {
        V::store(dst_rs(dst + ((WRAP_ROWS ? 0 : a.ghost) + row) * a.pitch, valid ? span_bytes : 0, 10), store_off, v);
    }
    // Store trip t's outputs.  Rows outside the segment (pipeline fill and the tail) get an empty
    // descriptor (num_records 0): the stores are dropped by the range check with no branch, and the row
    // address is clamped so no out-of-buffer pointer is ever formed.
    __device__ __forceinline__ void store_masked(const uint32_t (&v)[R][M], int64_t t) {
        if constexpr (BOUNDED) {  // 32-bit step arithmetic: scalar compares
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int d = (int)t * R + r - 2 * K;  // output row (ly0 + t*R + r - K) - seg_begin
                const bool valid = d >= 0 && d < seglen;
                store_row(v[r], seg_begin + (valid ? d : 0), valid);
            }
        } else {  // the torus variants keep their measured instruction streams (profiles/r2/ab_torus_d.log)
            const int64_t lo = ly0 + t * R - K;
#pragma unroll
            for (int r = 0; r < R; r++) {
                const bool valid = lo + r >= seg_begin && lo + r < seg_end;
                store_row(v[r], valid ? lo + r : seg_begin, valid);
            }
        }
    }
};

// Minimum waves per SIMD the register allocator must fit (1 = compiler's choice), per variant.
template <int K, int M, bool BOUNDED, bool WRAP_ROWS, int NARROW>
struct MinWaves {
    static constexpr int value =
        Wpb<K, M, BOUNDED, WRAP_ROWS, NARROW>::value > 8 ? Wpb<K, M, BOUNDED, WRAP_ROWS, NARROW>::value / 4 : 1;
};

// Wave strips: Wpb waves per workgroup, each its own column strip and segment (or a share of a group
// segment, see plan_stream).
template <int K, int M, bool BOUNDED, bool WRAP_ROWS, int NARROW>
__global__ __launch_bounds__((kWave * Wpb<K, M, BOUNDED, WRAP_ROWS, NARROW>::value))
__attribute__((amdgpu_waves_per_eu(MinWaves<K, M, BOUNDED, WRAP_ROWS, NARROW>::value)))
void gol_stream_step(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, StreamArgs a) {
    using W = StreamWave<K, M, BOUNDED, WRAP_ROWS, NARROW>;
    constexpr int R = W::R;
    const int lane = threadIdx.x & (kWave - 1);
    int64_t sx, sy;
    int role = -1;
    // wave index made provably uniform so all row bookkeeping lives in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int WPB = Wpb<K, M, BOUNDED, WRAP_ROWS, NARROW>::value;
    int64_t unit;  // a strip's segment (or SIMD group segment), then the seam geometry's remainder units
    if (a.split > 0) {  // waves w, w + 4, ... share a SIMD: one group segment between them
        unit = (int64_t)blockIdx.x * 4 + (wave & 3);
        role = wave >> 2;  // 0 = the oldest
    } else {
        unit = (int64_t)blockIdx.x * WPB + wave;
    }
    const int64_t main_units = a.nstrips * a.nsegs;
    if (unit >= main_units + a.rem_units) return;
    int rem_count = 0;
    if (unit < main_units) {
        sx = unit % a.nstrips;
        sy = unit / a.nstrips;
    } else {
        // remainder unit r (seam geometry): segments 1 .. rem_mid, all of length a.seg and with every row they
        // stream inside the board, rem_p at a time (sub-strip j = segment sy + j: a per-lane row offset); the
        // others alone (the first segment's rows wrap or reach the ghost rows, the last is shorter)
        const int64_t r = unit - main_units;
        const int64_t packed = (a.rem_mid + a.rem_p - 1) / a.rem_p;
        sx = a.nstrips;
        if (r >= 1 && r <= packed) {
            sy = 1 + (r - 1) * a.rem_p;
            const int64_t left = 1 + a.rem_mid - sy;
            rem_count = (int)(left < a.rem_p ? left : a.rem_p);
        } else {
            sy = r == 0 ? 0 : r - packed + a.rem_mid;
            rem_count = 1;
        }
    }
    W w(src, dst, a, lane, sx, sy, role, rem_count);
#if GOL_STAMP
    const int64_t stamp_id = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t stamp_t0 = __builtin_amdgcn_s_memrealtime();
#endif

    const int64_t ntrips = (w.nsteps + R - 1) / R;
    const int64_t t_fill = (2 * K) / R < ntrips ? (2 * K) / R : ntrips;  // trips entirely before step 2K

    // Row buffers: B is the staged passes' one buffer; A / B alternate roles in the K = 1 pass.  NA / NB: the K = 1
    // halo-free strips' neighbour words.  Stores are deferred by one trip in both (see the loops below).
    uint32_t A[R][M], B[R][M], NA[R], NB[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        NA[r] = NB[r] = 0;
#pragma unroll
        for (int j = 0; j < M; j++) B[r][j] = 0;
    }
    if constexpr (!W::kStage) w.load(A, NA, 0);
    using Skip = std::true_type;
    using NoSkip = std::false_type;
    using P0 = std::integral_constant<int, 0>;  // staged trips: read stage parity 0, prefetch into parity 1
    using P1 = std::integral_constant<int, 1>;
    const int64_t fill_pairs = (t_fill < ntrips ? t_fill : ntrips) / 2;
    int64_t t = 0;
    if constexpr (W::kStage) {
        // Deep passes: one row buffer in registers, rows staged through LDS (stage_load / stage_in).  Trip t:
        //   [wait for all memory ops of trip t-1] [store trip t-1's outputs] [read trip t's rows from the stage]
        //   [prefetch trip t+1 into the other stage parity] [compute trip t in place]
        // Stores are deferred by one trip so the wait at the top never covers an operation issued less than a whole
        // trip earlier (the wait-count pass treats pending loads and stores as completing out of order).
        __shared__ typename W::Stage stage[WPB];
        w.stage = &stage[wave];
        __shared__ uint32_t seam1_stage[W::kSeam1 ? WPB : 1][2][W::kSeam1 ? kWave : 1];
        if constexpr (W::kSeam1) w.seam1 = &seam1_stage[wave];
        uint32_t NV[R];  // (K = 1 neighbour words: unused here)
#pragma unroll
        for (int r = 0; r < R; r++) NV[r] = 0;
        w.template stage_load<0>();
        w.smem_seam_late();  // (GOL_SEAM_SMEM 2: trip 0's seam words)
        auto trip = [&](int64_t tt, auto skip, auto mask, auto par) {
            constexpr int PAR = decltype(par)::value;
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_staged(B);
            w.template stage_read<PAR>(B, lane);
            // (GOL_SEAM_SMEM: the seam words taken before this trip's prefetch loads the next trip's over them)
            [[maybe_unused]] typename W::Seam st_smem;
            if constexpr (W::kSmem) w.template stage_read_seam<PAR>(st_smem, lane);
            __builtin_amdgcn_sched_barrier(0);  // the row reads before the prefetch: their latency hides behind it
            // prefetch placement (GOL_SEAM_SPREAD above): rows issued at the top, after level g, and after the levels
            // (the pipeline-fill trips, which skip levels, keep every DMA at the top)
            constexpr int kSpread = GOL_SEAM_SPREAD >= 0 ? GOL_SEAM_SPREAD : 4;
            constexpr int kMode = (W::kSeam || (BOUNDED && GOL_AB_BSPREAD)) && !decltype(skip)::value ? kSpread : 0;
            if constexpr (kMode == 0) w.template stage_load<1 - PAR>();
            if constexpr (kMode == 3) {
#pragma unroll
                for (int r = 0; r < R; r++) w.template stage_load_row<1 - PAR, 1>(r);
            }
            typename W::Seam st;
            if constexpr (W::kSmem)
                st = st_smem;
            else
                w.template stage_read_seam<PAR>(st, lane);
            w.stage_in(B, st, tt * R);
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the trip
            auto hook = [&](int g) {
                if constexpr (kMode == 1 || kMode == 3) {
                    if (g < R) {
                        w.template stage_load_row<1 - PAR, kMode == 1 ? 3 : 2>(g);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                } else if constexpr (kMode == 4) {
                    if (g < 2 * R) {
                        if (g % 2 == 0)
                            w.template stage_load_row<1 - PAR, 1>(g / 2);
                        else
                            w.template stage_load_row<1 - PAR, 2>(g / 2);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                } else if constexpr (kMode == 5) {  // A/B: row r's DMAs after levels 3r and 3r + 1
                    if (g < 3 * R && g % 3 < 2) {
                        if (g % 3 == 0)
                            w.template stage_load_row<1 - PAR, 1>(g / 3);
                        else
                            w.template stage_load_row<1 - PAR, 2>(g / 3);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            };
            w.template process<decltype(skip)::value, decltype(mask)::value>(B, NV, tt, hook);
            // a pass shallower than the levels the mode spreads over: the rows not yet issued
            if constexpr (kMode == 1 || kMode == 3) {
#pragma unroll
                for (int r = K; r < R; r++) w.template stage_load_row<1 - PAR, kMode == 1 ? 3 : 2>(r);
            } else if constexpr (kMode == 4) {
#pragma unroll
                for (int g = K; g < 2 * R; g++) {
                    if (g % 2 == 0)
                        w.template stage_load_row<1 - PAR, 1>(g / 2);
                    else
                        w.template stage_load_row<1 - PAR, 2>(g / 2);
                }
            } else if constexpr (kMode == 5) {
#pragma unroll
                for (int g = K; g < 3 * R; g++) {
                    if (g % 3 == 0)
                        w.template stage_load_row<1 - PAR, 1>(g / 3);
                    else if (g % 3 == 1)
                        w.template stage_load_row<1 - PAR, 2>(g / 3);
                }
            }
            w.smem_seam_late();  // (GOL_SEAM_SMEM 2)
        };
        using Mask = std::true_type;
        using NoMask = std::false_type;
        if constexpr (!BOUNDED) {
            for (int64_t p = 0; p < fill_pairs; p++, t += 2) {  // pipeline fill: all-garbage levels skipped
                trip(t, Skip{}, NoMask{}, P0{});
                trip(t + 1, Skip{}, NoMask{}, P1{});
            }
            for (; t + 1 < ntrips; t += 2) {  // steady state (the odd fill / transition trip runs here unskipped)
                trip(t, NoSkip{}, NoMask{}, P0{});
                trip(t + 1, NoSkip{}, NoMask{}, P1{});
            }
            if (t < ntrips) trip(t++, NoSkip{}, NoMask{}, P0{});
        } else {
            // Bounded board: the trips that produce rows off the board (the fill trips and, in the steady state,
            // t < t_top or t >= t_bot: near the board's top and bottom edges) mask them dead at every level; the
            // others run the unmasked arithmetic of the torus strips.
            for (int64_t p = 0; p < fill_pairs; p++, t += 2) {
                trip(t, Skip{}, Mask{}, P0{});
                trip(t + 1, Skip{}, Mask{}, P1{});
            }
            for (; t + 1 < ntrips && t < w.t_top; t += 2) {
                trip(t, NoSkip{}, Mask{}, P0{});
                trip(t + 1, NoSkip{}, Mask{}, P1{});
            }
            const int64_t t_end = w.t_bot < ntrips ? w.t_bot : ntrips;
            for (; t + 1 < t_end; t += 2) {
                trip(t, NoSkip{}, NoMask{}, P0{});
                trip(t + 1, NoSkip{}, NoMask{}, P1{});
            }
            for (; t + 1 < ntrips; t += 2) {
                trip(t, NoSkip{}, Mask{}, P0{});
                trip(t + 1, NoSkip{}, Mask{}, P1{});
            }
            if (t < ntrips) trip(t++, NoSkip{}, Mask{}, P0{});
        }
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        w.store_staged(B);
    } else if constexpr (!BOUNDED) {
        // K = 1 (rows of trip t in `cur`, trip t-1's outputs in `other`):
        //   [wait for all memory ops of trip t-1] [store `other`] [prefetch trip t+1 into `other`]
        //   [compute trip t in place in `cur`]
        // the two row buffers alternate roles (A/B) so no register copy or early wait joins a prefetch.
        auto trip = [&](uint32_t (&cur)[R][M], uint32_t (&other)[R][M], uint32_t (&ncur)[R], uint32_t (&nother)[R],
                        int64_t tt, auto skip) {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(other, tt - 1);
            w.load(other, nother, (tt + 1) * R);
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the trip
            w.template process<decltype(skip)::value, false>(cur, ncur, tt);
        };
        for (int64_t p = 0; p < fill_pairs; p++, t += 2) {
            trip(A, B, NA, NB, t, Skip{});
            trip(B, A, NB, NA, t + 1, Skip{});
        }
        for (; t + 1 < ntrips; t += 2) {
            trip(A, B, NA, NB, t, NoSkip{});
            trip(B, A, NB, NA, t + 1, NoSkip{});
        }
        if (t < ntrips) {  // odd trip count: one more trip, outputs land in A
            trip(A, B, NA, NB, t, NoSkip{});
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(A, t);
        } else {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(B, t - 1);
        }
    } else {
        // K = 1 on a bounded board: every trip masks (halo-free strips carry per-lane column masks)
        auto trip = [&](uint32_t (&cur)[R][M], uint32_t (&other)[R][M], uint32_t (&ncur)[R], uint32_t (&nother)[R],
                        int64_t tt, auto skip) {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(other, tt - 1);
            w.load(other, nother, (tt + 1) * R);
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the trip
            w.template process<decltype(skip)::value, true>(cur, ncur, tt);
        };
        for (int64_t p = 0; p < fill_pairs; p++, t += 2) {
            trip(A, B, NA, NB, t, Skip{});
            trip(B, A, NB, NA, t + 1, Skip{});
        }
        for (; t + 1 < ntrips; t += 2) {
            trip(A, B, NA, NB, t, NoSkip{});
            trip(B, A, NB, NA, t + 1, NoSkip{});
        }
        if (t < ntrips) {
            trip(A, B, NA, NB, t, NoSkip{});
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(A, t);
        } else {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            w.store_masked(B, t - 1);
        }
    }
#if GOL_STAMP
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0 && stamp_id < kStamps) {
        g_stamps[0][stamp_id] = stamp_t0;
        g_stamps[1][stamp_id] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ------------------------------------------------------------------------------------------------
// Supported (K, M) instantiations.  M = 1: any board with W % 32 == 0; M = 2 / 4 need W % 64 / 128.
// Deeper K needs 5*M*K window registers per lane, so the deepest K shrinks as M grows.
// (a register-usage study may compile a subset: -DGOL_KM_SUBSET(X)='X(12, 2)')
#ifdef GOL_KM_SUBSET
#define GOL_FOR_EACH_KM(X) GOL_KM_SUBSET(X)
#else
#define GOL_FOR_EACH_KM(X)                                                                               \
    X(1, 1) X(2, 1) X(4, 1) X(8, 1) X(16, 1) X(24, 1) X(32, 1)                                           \
    X(1, 2) X(2, 2) X(4, 2) X(8, 2) X(12, 2) X(16, 2)                                                    \
    X(1, 4) X(2, 4) X(4, 4) X(6, 4) X(8, 4)
#endif

// (K, ilv 4) with K = 16 / 32 is the level-pipelined pass (gol_pipe.hip, torus boards only)
bool stream_supported(int k, int ilv) {
#define GOL_SUP(K_, M_) \
    if (k == K_ && ilv == M_) return true;
    GOL_FOR_EACH_KM(GOL_SUP)
#undef GOL_SUP
    return ilv == 4 && pipe_supported(k);
}

int stream_max_k(int ilv) { return ilv == 1 ? 32 : (ilv == 2 ? 16 : 32); }

int stream_largest_k(int64_t n, int cap, int ilv, int64_t words, bool bounded) {
    static const int ks[] = {32, 24, 16, 12, 8, 6, 4, 2, 1};
    for (int k : ks) {
        if (k > cap || k > n || !stream_supported(k, ilv)) continue;
        // the level-pipelined depths (16 / 32 at ilv 4) only where that pass runs (torus rows of a full strip)
        if (ilv == 4 && pipe_supported(k) && !pipe_applies(words, ilv, k, bounded, 0)) continue;
        return k;
    }
    return 1;
}

// The NARROW template value of a pass.  Torus: 1 = the M = 1 ragged-row variant (StreamWave kRagged).  Bounded: 1 = a
// board narrower than one wave strip (halo-lane strips, column masks at every level), 2 = a ragged row (rag_bits: the
// board's width is not a multiple of 32; a.rag_w) at least a strip wide (edge-fill strips, column masks at every
// level), 0 = edge-fill strips without column masks.
static int stream_narrow(int64_t words, int ilv, int k, bool bounded, int rag_bits = 0) {
    if (!bounded) return rag_bits != 0 ? 1 : 0;
    if (k <= 1) return 0;  // K = 1: halo-free strips with per-lane column masks anyway
    if (words / ilv < kWave) return 1;
    return rag_bits != 0 ? 2 : 0;
}

// Variants: torus with rows wrapping in the buffer (single board), torus strip with ghost rows, ragged torus rows
// (single board, ilv 1), bounded (never wraps: rows beyond the board are masked dead; narrow and ragged boards
// mask columns too).
template <int K, int M>
static const void* stream_kernel(bool bounded, bool wrap, int narrow) {
    if (bounded)
        return narrow == 1 ? (const void*)&gol_stream_step<K, M, true, false, 1>
                           : (narrow == 2 ? (const void*)&gol_stream_step<K, M, true, false, 2>
                                          : (const void*)&gol_stream_step<K, M, true, false, 0>);
    if (narrow) {
        if constexpr (M == 1) return wrap ? (const void*)&gol_stream_step<K, 1, false, true, 1> : nullptr;
        return nullptr;
    }
    return wrap ? (const void*)&gol_stream_step<K, M, false, true, 0>
                : (const void*)&gol_stream_step<K, M, false, false, 0>;
}

static const void* kernel_for(int k, int ilv, bool bounded, bool wrap, int narrow) {
#define GOL_KPTR(K_, M_) \
    if (k == K_ && ilv == M_) return stream_kernel<K_, M_>(bounded, wrap, narrow);
    GOL_FOR_EACH_KM(GOL_KPTR)
#undef GOL_KPTR
    return nullptr;
}

int64_t stream_strips(int64_t words, int ilv, int k, bool bounded, int rag_bits) {
    const int64_t nblocks = words / ilv;
    if (rag_bits && !bounded) return (nblocks + kInterior - 1) / kInterior;  // ragged torus rows: see plan_stream
    if (k == 1) return (nblocks + kWave - 1) / kWave;  // K = 1: halo-free strips
    // bounded edge-fill strips (StreamWave::edge_fill): strip 0 stores blocks [0, 63), strip s stores
    // [62 s + 1, 62 s + 63), the last ends at the board's last block
    if (bounded && nblocks >= kWave) return (nblocks - 1 + kInterior - 1) / kInterior;
    // halo-lane strips (torus; bounded NARROW = 1: narrow rows): strip s stores blocks [62 s, 62 s + 62)
    return (nblocks + kInterior - 1) / kInterior;
}

// Waves per workgroup of a variant (Wpb)
int stream_wpb(int64_t words, int k, int ilv, bool bounded, bool wrap, int rag_bits) {
    const int narrow = stream_narrow(words, ilv, k, bounded, rag_bits);
#define GOL_WPBQ(K_, M_)                                                                                 \
    if (k == K_ && ilv == M_)                                                                            \
        return bounded ? (narrow == 1 ? Wpb<K_, M_, true, false, 1>::value                               \
                                      : (narrow == 2 ? Wpb<K_, M_, true, false, 2>::value : Wpb<K_, M_, true, false, 0>::value)) \
                       : (narrow ? Wpb<K_, M_, false, true, 1>::value                                     \
                                 : (wrap ? Wpb<K_, M_, false, true, 0>::value : Wpb<K_, M_, false, false, 0>::value));
    GOL_FOR_EACH_KM(GOL_WPBQ)
#undef GOL_WPBQ
    return kWavesPerBlock;
}

// Pair split (1/65536 units): the share of a pair segment given to the older of the two waves that
// share a SIMD.  VALU issue favours the older wave (MI355X_MICROARCH.md "Two waves per SIMD"), so with
// equal segments it finishes early and leaves the younger alone at the single-wave issue rate
// (tools/tail.py: 65536^2, K = 16 -- waves 0-3 of every workgroup busy 489 us, waves 4-7 747 us).
// A board's "split" option (gol_set_option) overrides it for experiments.
int stream_pair_split(int k, int ilv, bool bounded, bool wrap, bool single) {
    if (kWavesPerBlock < 8) return 0;
    // Round 5, with the middle wave's share set apart (stream_split2), at the bench window (generation 300+), 4
    // interleaved rounds (profiles/r5/split2_confirm_g.jsonl, us per pass, mean): single-board torus (12, 2) 0.66 / 0.76
    // 442.5 against 0.70 / geometric 445.8; bounded (12, 2) 0.60 / 0.72 431.0 against 0.64 / geometric 436.0.  The
    // per-role tails of a stamped build (profiles/r5/split2_tails_f.jsonl): torus roles ending at 439 / 378 / 436 us with
    // geometric shares, 440 / 417 / 430 with 0.68 / 0.76.  Both retunes were measured on single boards only, so the
    // ghost-row strips of N > 1 keep round 4's measured split on either boundary (`single`: one strip holding the whole
    // board, ghost 0): torus strips fall through to 0.70 below, bounded strips keep 0.64.
    if (bounded && ilv == 2 && k == 12) return (int)((single ? 0.60 : 0.64) * 65536);
    if (!bounded && wrap && ilv == 2 && k == 12) return (int)(0.66 * 65536);
    // measured at 65536^2 (profiles/r1/split_sweep*.log, two boxes): the deep passes gain 3-9 %; the
    // shallow ones (short, memory-bound trips) are left unpaired
    // (12, 2) runs 12-wave workgroups at 3 waves/SIMD: three-way groups (profiles/r1/w12_sweep*.log)
    // Round 3, staged passes, fresh 65536^2 board, forward + reverse sweep (profiles/r3/split_sweep_f.log): torus
    // (12, 2) 0.64 / 0.68 / 0.72 -> 95.9k / 96.8k / 95.0k; torus (16, 2) 0.60 / 0.64 / 0.68 / 0.72 -> 101.8k / 107.5k /
    // 107.6k / 104.7k; bounded (12, 2) 0.60 / 0.64 / 0.68 -> 96.6k / 99.0k / 95.4k; bounded (16, 2) 0.56 / 0.60 /
    // 0.64 / 0.68 -> 112.5k / 112.0k / 106.2k / 100.7k (a slope now, not round 2's cliff).
    if (bounded && ilv == 2 && k == 16) return (int)(0.60 * 65536);
    // (bounded (12, 2): 0.64 until round 5, above)
    if (ilv == 1 && k >= 24) return (int)(0.60 * 65536);
    if (ilv == 2 && k == 12) return (int)(0.70 * 65536);
    if (ilv == 2 && k >= 16) return (int)(0.66 * 65536);
    if (ilv == 4 && k >= 8) return (int)(0.55 * 65536);
    return 0;
}

// Waves of a stream-kernel variant the current device holds at once (occupancy x CUs), cached.  Falls back
// to 4096 waves when no device answers (host-only planning, e.g. CPU tests).
static int64_t resident_units(int64_t words, int k, int ilv, bool bounded, bool wrap, int rag_bits) {
    static std::atomic<int64_t> cache[33][5][2][2][3];
    const int64_t fallback = 4096;
    if (k < 0 || k > 32 || ilv < 1 || ilv > 4) return fallback;
    if (bounded) wrap = false;
    const int narrow = stream_narrow(words, ilv, k, bounded, rag_bits);
    int64_t v = cache[k][ilv][bounded][wrap][narrow].load(std::memory_order_relaxed);
    if (v > 0) return v;
    const void* fn = kernel_for(k, ilv, bounded, wrap, narrow);
    const int wpb = stream_wpb(words, k, ilv, bounded, wrap, rag_bits);
    const int threads = kWave * wpb;
    int dev = 0, cus = 0, blocks = 0;
    if (!fn || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, threads, 0) != hipSuccess || blocks <= 0 ||
        cus <= 0) {
        (void)hipGetLastError();
        return fallback;
    }
    v = (int64_t)blocks * cus * wpb;
    cache[k][ilv][bounded][wrap][narrow].store(v, std::memory_order_relaxed);
    return v;
}

// Remainder units of the seam geometry for nsegs segments (kernel: the unit mapping in gol_stream_step).
static int64_t seam_rem_units(const StreamArgs& a, int64_t nsegs, int64_t rem_mid) {
    if (!a.seam || a.rem == 0 || nsegs <= 0) return 0;
    return 1 + (rem_mid + a.rem_p - 1) / a.rem_p + (nsegs - 1 - rem_mid);
}

// Does the seam geometry apply?  Torus deep passes (the bounded edge-fill strips keep their zero-fill edges) on rows
// of at least one seam strip, with K <= 16 M (the break in the middle of the seam lane must not reach its ends).
static bool seam_applies(const StreamArgs& a, int k, bool bounded) {
    return !GOL_AB_NOSEAM && a.seam_opt >= 0 && !bounded && !a.rag_bits && k > 1 && k <= 16 * a.ilv && a.words / a.ilv >= kSeamInterior;
}

// Work decomposition: nstrips column strips x nsegs row segments, one wave each (or one SIMD group of
// waves per segment with the pair split), plus the seam geometry's remainder units.  The segment count makes the
// grid ONE balanced round of resident waves (a partial second round would leave a tail of lone waves), with
// segments no shorter than 2K rows (pipeline fill cost).  a.split_opt / a.seg_opt / a.seam_opt (a board's "split" /
// "seg_rows" / "seam" options) override the split, the segment length and the geometry for experiments.
// Three-wave groups: the middle wave's share of the two younger waves' rows (1/65536), 0 = geometric.
int stream_split2(int k, int ilv, bool bounded, bool wrap, bool single) {
    if (kWavesPerBlock < 8 || ilv != 2 || k != 12 || !single) return 0;  // (12, 2) single boards: see stream_pair_split
    if (bounded) return (int)(0.72 * 65536);
    return wrap ? (int)(0.76 * 65536) : 0;
}

void plan_stream(StreamArgs& a, int k, bool bounded, bool wrap) {
    const bool single = a.ghost == 0 && a.rows == a.height;  // the whole board in one buffer (not a ghost-row strip)
    a.split = a.split_opt > 0 ? a.split_opt : (a.split_opt < 0 ? 0 : stream_pair_split(k, a.ilv, bounded, wrap, single));
    a.split2 = a.split2_opt > 0 ? a.split2_opt : stream_split2(k, a.ilv, bounded, wrap, single);
    const int64_t nblocks = a.words / a.ilv;
    a.seam = seam_applies(a, k, bounded) ? 1 : 0;
    a.rem = 0;
    a.rem_p = 1;
    a.rem_units = 0;
    a.rem_mid = 0;
    if (a.seam) {
        a.nstrips = nblocks / kSeamInterior;
        a.rem = (int32_t)(nblocks - a.nstrips * kSeamInterior);
        a.rem_p = a.rem ? (kWave / (a.rem + 2) > 0 ? kWave / (a.rem + 2) : 1) : 1;
    } else {
        a.nstrips = stream_strips(a.words, a.ilv, k, bounded, a.rag_bits);
    }
    // Ragged torus rows (StreamWave kRagged): the strips start at ring position -1 (the partial last word, then word
    // 0, ...), unless the last strip's right halo lane would then be the partial word next to a stored word; then
    // at position -2.
    a.rag_origin = 1;
    if (a.rag_bits && !bounded && (a.nstrips * kInterior - 1 + 1) % nblocks == 0) a.rag_origin = 2;
    const int64_t rows = a.out_end - a.out_begin;
    if (rows <= 0) {
        a.nsegs = 0;
        a.seg = 1;
        return;
    }
    // a launch too short for one full group segment per strip (e.g. a k-row halo band) runs one wave per
    // segment: splitting a handful of rows only multiplies the pipeline fill
    const int wpb = stream_wpb(a.words, k, a.ilv, bounded, wrap, a.rag_bits);
    if (a.split && rows < (int64_t)(wpb / 4) * (2 * k > 16 ? 2 * k : 16)) a.split = 0;
    const int group = a.split ? wpb / 4 : 1;  // waves per segment
    int64_t seg = a.seg_opt;
    int64_t slots = 0;
    if (seg <= 0) {
        int64_t units = resident_units(a.words, k, a.ilv, bounded, wrap, a.rag_bits);
        if (a.spare > 0) units = units > a.spare + 1 ? units - a.spare : 1;
        slots = units / group;
        // waves per segment: the strips, plus (seam geometry) a 1/rem_p share of a remainder wave
        const double per_seg = (double)a.nstrips + (a.seam && a.rem ? 1.0 / a.rem_p : 0.0);
        int64_t nsegs = (int64_t)((double)slots / per_seg);
        if (nsegs < 1) nsegs = 1;
        int64_t min_seg = (2 * k > 16 ? 2 * k : 16) * group;
        // A launch too small to fill a quarter of the device is latency-bound: each wave is one serial
        // chain of (segment + 2k) rows x k levels, so shorter segments (more, shorter chains) finish sooner
        // despite the extra pipeline fill.  1024^2: 549 -> 696 GCUPS, 4096^2: 8.7k -> 10.5k at K = 8, ilv 1
        // (profiles/r1/small_seg.log).  Large boards are bounded by `slots` below and do not change.
        if ((rows / min_seg) * a.nstrips * group < units / 4) min_seg = (k > 8 ? k : 8) * group;
        const int64_t max_segs = rows / min_seg > 0 ? rows / min_seg : 1;
        if (nsegs > max_segs) nsegs = max_segs;
        seg = (rows + nsegs - 1) / nsegs;
    }
    if (seg > ((int64_t)1 << 30)) seg = (int64_t)1 << 30;  // the kernel counts a segment's rows in 32 bits
    a.seg = seg;
    a.nsegs = (rows + seg - 1) / seg;
    if (a.seam && a.rem) {
        // the per-lane row offsets of a packed remainder wave are 32-bit byte offsets into one descriptor
        const int64_t row_bytes = a.words * 4, step = seg * (a.pitch > 0 ? a.pitch : a.words) * 4;
        const int64_t fit = 1 + ((((int64_t)1 << 31) - 1 - row_bytes) / step);
        if (a.rem_p > fit) a.rem_p = (int32_t)(fit > 1 ? fit : 1);
        // segments 1 .. rem_mid share remainder waves: every row they stream must lie in the board / buffer
        // without a wrap.  Sub-strip j reads its rows at a fixed offset from sub-strip 0's walk, which wraps (single
        // board) or clamps (ghost-row strip) only for itself; so the last packed segment's rows -- its k halo rows
        // below and the walk's overshoot -- must end inside the buffer.  The walk prefetches whole trips of R = 4
        // rows, one trip ahead, and the last trip prefetches one more (unused): ceil((seg + 2k) / 4) + 1 trips, up to
        // 7 rows past the seg + 2k the segment streams.  Round 3 let those rows run past the buffer's end: reads
        // beyond the allocation, harmless unless the next page was unmapped -- an illegal-address fault in round 4's
        // suite on an 8209 x 40 ragged board (ring rows of 262 words, 42 KB), found by the GOL_CHECK_BOUNDS build
        // (descriptor tag 8) and reproduced on the CPU by walking the plan.
        const int64_t trip = 4;  // TripRows of every seam pass (K > 1)
        const int64_t over = ((seg + 2 * k + trip - 1) / trip + 1) * trip - (seg + 2 * k);
        const int64_t limit = wrap ? a.rows : a.rows + a.ghost;  // first row index past the buffer (owned-row units)
        int64_t mid = a.nsegs - 2;
        const int64_t fit_mid = (limit - a.out_begin - k - over) / seg - 1;  // (m + 1) seg + k + over <= limit - out_begin
        if (fit_mid < mid) mid = fit_mid;
        // sub-strip j streams rows [(j + 1) seg - k, (j + 2) seg + k) of the buffer at a fixed offset from
        // sub-strip 0's walk: a segment shorter than k (the "seg_rows" option can ask for one) would make segment 1's
        // first rows wrap or leave the buffer, so such segments run as lone remainder units
        if (seg < k) mid = 0;
        a.rem_mid = mid > 0 ? mid : 0;
        a.rem_units = seam_rem_units(a, a.nsegs, a.rem_mid);
    }
}

template <int K, int M>
static hipError_t launch_km(const uint32_t* src, uint32_t* dst, const StreamArgs& a, bool bounded, bool wrap,
                            hipStream_t s) {
    const int WPB = stream_wpb(a.words, K, M, bounded, wrap, a.rag_bits);
    const int64_t waves = (a.nstrips * a.nsegs + a.rem_units) * (a.split ? WPB / 4 : 1);
    const unsigned blocks = (unsigned)((waves + WPB - 1) / WPB);
    const dim3 block(kWave * WPB);
    if (bounded) {
        const int narrow = stream_narrow(a.words, M, K, true, a.rag_bits);
        if (narrow == 1)
            hipLaunchKernelGGL((gol_stream_step<K, M, true, false, 1>), dim3(blocks), block, 0, s, src, dst, a);
        else if (narrow == 2)
            hipLaunchKernelGGL((gol_stream_step<K, M, true, false, 2>), dim3(blocks), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_stream_step<K, M, true, false, 0>), dim3(blocks), block, 0, s, src, dst, a);
    } else if (a.rag_bits) {
        if constexpr (M == 1) {
            if (!wrap) return hipErrorInvalidValue;
            hipLaunchKernelGGL((gol_stream_step<K, 1, false, true, 1>), dim3(blocks), block, 0, s, src, dst, a);
        } else {
            return hipErrorInvalidValue;
        }
    } else {
        if (wrap)
            hipLaunchKernelGGL((gol_stream_step<K, M, false, true, 0>), dim3(blocks), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_stream_step<K, M, false, false, 0>), dim3(blocks), block, 0, s, src, dst, a);
    }
    return hipGetLastError();
}

PipeArgs pipe_args(const StreamArgs& a, bool bounded) {
    PipeArgs p{};
    p.words = a.words;
    p.pitch = a.pitch;
    p.rows = a.rows;
    p.ghost = a.ghost;
    p.out_begin = a.out_begin;
    p.out_end = a.out_end;
    p.split1 = a.pipe_split_opt;
    p.split2 = a.pipe_split2_opt;
    p.spare_waves = a.spare;
    p.err = a.pipe_err ? a.pipe_err : pipe_error_word();
    p.bounded = bounded ? 1 : 0;
    if (bounded) {  // the board's rows in owned-row coordinates, clipped to the buffer (Script.fsx:6-13)
        const int64_t lo = -a.y0 > -a.ghost ? -a.y0 : -a.ghost;
        const int64_t hi = a.height - a.y0 < a.rows + a.ghost ? a.height - a.y0 : a.rows + a.ghost;
        p.live_lo = (int32_t)lo;
        p.live_hi = (int32_t)hi;
    }
    return p;
}

hipError_t launch_stream_step(const uint32_t* src, uint32_t* dst, StreamArgs a, int k, bool bounded, bool wrap,
                              hipStream_t s) {
    if (a.ilv == 4 && pipe_supported(k)) {  // the level-pipelined pass (callers check where it applies; gol_pipe.hip)
        if (!pipe_applies(a.words, a.ilv, k, bounded, a.rag_bits)) return hipErrorInvalidValue;
        return launch_pipe_step(src, dst, pipe_args(a, bounded), k, wrap, s);
    }
    plan_stream(a, k, bounded, wrap);
    if (a.nsegs <= 0) return hipSuccess;
#define GOL_LAUNCH(K_, M_) \
    if (k == K_ && a.ilv == M_) return launch_km<K_, M_>(src, dst, a, bounded, wrap, s);
    GOL_FOR_EACH_KM(GOL_LAUNCH)
#undef GOL_LAUNCH
    return hipErrorInvalidValue;
}

}  // namespace gol

#if GOL_CHECK_BOUNDS
extern "C" unsigned gol_debug_bounds(void) {  // diagnostic builds: violation bits of the step kernels, then cleared
    unsigned v = 0, z = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(gol::g_bounds_err), sizeof(v), 0, hipMemcpyDeviceToHost);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gol::g_bounds_err), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    return v | gol_debug_bounds_formats();
}
#endif
#if GOL_STAMP
extern "C" int gol_debug_stamps(unsigned long long* out, long long n) {
    if (n > 2 * gol::kStamps) n = 2 * gol::kStamps;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gol::g_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
