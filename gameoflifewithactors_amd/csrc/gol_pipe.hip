// gol_pipe.hip -- the level-pipelined deep pass (round 6): K generations per pass with each wave holding D of them.
//
// Replaces, like gol_stream_step (gol_step.hip), K `updateView()` ticks of the reference (GameOfLifeDriver.fs:32-34):
// the per-cell actor protocol of GameOfLifeLogic.fs:39-71 applied to every cell K times, B3/S23 by gol_bitlogic.h.
//
// Why a pipeline.  The streaming pass keeps all K levels of a column strip in ONE wave's registers: its window is 5 K M
// VGPRs, so (K, M) = (12, 2) runs 3 waves per SIMD and M = 4 -- half the cross-lane moves and funnel shifts per word
// (9 + 8 / M issue slots per word and generation: 11 instead of 13) -- fits only at K <= 8.  Here the K levels of a
// strip are split over S waves of D = K / S levels each, a PIPELINE:
//   stage 0     streams the level-0 rows from HBM (one 16-byte buffer_load ... lds per lane and row, a trip ahead),
//   stage s     pushes each row through its D levels (the same level-fenced schedule as the streaming pass) and hands its
//               level-(s + 1) D rows to stage s + 1 through a ring of LDS rows,
//   stage S - 1 stores level K.
// A wave's window is 5 D M = 80 VGPRs at (D, M) = (4, 4): 126 VGPRs in all, 4 waves per SIMD.  A pipeline streams its
// segment once, so the recomputed halo rows are one cone per pipeline (K (K - 1) level-rows), not one per wave.
//
// Ring protocol (per pipeline and stage boundary, no workgroup barrier): the producer writes output row j into slot
// j mod NR and then publishes prod = rows written; the consumer waits for prod, reads the rows, and publishes
// cons = rows read at its next trip's top; the producer waits for cons before overwriting a slot.  LDS operations of
// one wave are performed in order, so a counter written after the data is never seen before the data, and a slot is
// never overwritten before the reads that preceded the consumer's counter; the signal fences only keep the compiler
// from moving LDS accesses across the counter accesses.  Every wait is bounded (spin_limit polls): a wait that gives up
// sets *err and the wave stops (a guard against a bug, not a condition of normal use -- all waves a wait depends on are
// in the same workgroup, so resident together).
//
// Work decomposition (plan_pipe).  Column strips of 62 stored blocks with a halo lane per side (a wave's 64 lanes, a
// block of M = 4 words = 128 cells per lane); the blocks a row has past the last full strip go to remainder
// workgroups whose lanes hold rp sub-strips of (rem + 2) lanes, sub-strip j on row group gy + j (a per-lane row offset,
// as the streaming pass's remainder waves).  A workgroup is P pipelines x S stages = 16 waves (one per CU) and owns
// one group of rows of one strip; its P pipelines share the group's rows by age (VALU issue favours the older wave of
// a SIMD, MI355X_MICROARCH.md "Two waves per SIMD": shares fall geometrically, `split1` / `split2`, as plan_stream's
// group cut), and pipeline p's stage s is wave S p + (s + p) mod S, so every SIMD holds every stage.  The grid is one
// round of resident workgroups.
//
// Variants: WRAP (single torus board: the rows wrap at the board's edge, GameOfLifeDriver.fs:21-25), torus ghost-row
// strips (multi-GPU: rows outside the buffer are clamped, only ever feeding rows nobody stores), and BND (bounded
// boards and strips, Script.fsx:6-13: dead beyond the edges).  A bounded row of nblocks >= 64 blocks is covered by
// strips of 64 lanes whose first stores 63 blocks from the board's left edge on lane 0, whose last stores 63 up to
// the right edge on lane 63, and whose others store 62 between halo lanes, the blocks left between the last of these and
// the right edge strip going to remainder workgroups as on the torus; the lane moves shift in zeros at the wave's
// ends, which is the dead column beyond each edge at no extra instruction.  Rows outside the board load as zeros (a
// descriptor of no bytes) and the trips that reach them zero the rows they compute there, level by level.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <vector>

#include "gol_bitlogic.h"
#include "gol_internal.h"

#define GOL_PIPE_STR2(x) #x
#define GOL_PIPE_STR(x) GOL_PIPE_STR2(x)

namespace gol {

namespace {

constexpr int kWave = 64;
constexpr int kInterior = kWave - 2;  // blocks stored per full strip
constexpr int kM = 4;                 // words per block (ilv 4)
constexpr int kR = 4;                 // rows per trip
constexpr int kNT = 2;                // trips per ring (NR = 8 rows)
constexpr int kNoStore = 0x7ffffff0;  // a lane offset past any row: its store is dropped by the range check
constexpr int kRsrcWord3 = 0x00020000;
constexpr int kWaitVm0 = 0x0F70;  // s_waitcnt vmcnt(0)
constexpr int kAllButDs = 0x1 | 0x2 | 0x4 | 0x8 | 0x10 | 0x20 | 0x40 | 0x400;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Z (bounded boards): shifts with zero fill, so a board edge on a wave's outer lane sees dead cells beyond it
template <bool Z>
__device__ __forceinline__ uint32_t from_left(uint32_t v) {  // lane i <- lane i - 1 (wave_ror:1; Z: wave_shr:1, lane 0 <- 0)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, Z ? 0x138 : 0x13C, 0xf, 0xf, Z);
}
template <bool Z>
__device__ __forceinline__ uint32_t from_right(uint32_t v) {  // lane i <- lane i + 1 (wave_rol:1; Z: wave_shl:1, lane 63 <- 0)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, Z ? 0x130 : 0x134, 0xf, 0xf, Z);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, kRsrcWord3);
}
// The ring's counter and row accesses are written out: the wait-count pass cannot tell them from the first stage's
// LDS-DMA destination, and put an s_waitcnt vmcnt(0) in front of every one -- so the last stage waited for its own row
// stores at every trip's top (and the first for its prefetch at every hand-off).  LDS operations of one wave are
// performed in order; each read waits for its data (lgkmcnt(0)) before the asm ends; the "memory" clobbers keep the
// compiler's own memory accesses on their side.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void lds_publish(int* p, int v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
#ifndef GOL_PIPE_SLEEP  // s_sleep periods (64 clocks) between polls
#define GOL_PIPE_SLEEP 1
#endif
#ifndef GOL_PIPE_POLL_ALIGN
#define GOL_PIPE_POLL_ALIGN 6
#endif
// Wait until the LDS word at `p` is >= need: poll, then s_sleep 1 between polls; returns the polls left (0: gave up).
// One asm loop whose head is aligned (GOL_PIPE_POLL_ALIGN, log2 bytes; the padding is jumped over): the compiler's own
// loop put the head wherever the code before it ended, and the pass's speed followed that address by 25 % with an
// 8-byte period (s_nop padding before the trip loop: 967-972 us per 65536^2 pass at an odd number of 4-byte nops,
// 1196-1210 at an even one, profiles/r6/pipe/r6h)
__device__ __forceinline__ int lds_wait(const int* p, int need, int limit) {
    int left = limit, tmp;
    asm volatile(
        "s_branch 2f\n"
        ".p2align " GOL_PIPE_STR(GOL_PIPE_POLL_ALIGN) "\n"
        "1:\n\t"
        "s_sleep " GOL_PIPE_STR(GOL_PIPE_SLEEP) "\n\t"
        "s_sub_i32 %[left], %[left], 1\n\t"
        "s_cmp_le_i32 %[left], 0\n\t"
        "s_cbranch_scc1 3f\n"
        "2:\n\t"
        "ds_read_b32 %[tmp], %[addr]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_gt_i32 vcc, %[need], %[tmp]\n\t"
        "s_cbranch_vccnz 1b\n"
        "3:"
        : [left] "+s"(left), [tmp] "=&v"(tmp)
        : [addr] "v"(lds_addr(p)), [need] "s"(need)
        : "vcc", "scc", "memory");
    return left;
}
// four consecutive ring rows (one trip: 4 KB from `p`, lane-major 16 bytes per lane)
__device__ __forceinline__ void lds_read_trip(const uint32_t* p, u32x4& r0, u32x4& r1, u32x4& r2, u32x4& r3) {
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\tds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
        : "v"(lds_addr(p))
        : "memory");
}
__device__ __forceinline__ void lds_write_row(uint32_t* p, const u32x4& w) {
    asm volatile("ds_write_b128 %0, %1" : : "v"(lds_addr(p)), "v"(w) : "memory");
}

// A wave-uniform 64-bit value the compiler cannot prove uniform (float math), moved to SGPRs
__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// First row (relative to a group of len rows) of the i-th oldest of n pipelines: shares fall geometrically with age,
// ratio (1 - f1) / f1 after the oldest and (1 - f2) / f2 after that, applied to each pipeline's streamed rows (its
// share plus the 2K-row cone); split1 <= 0: equal shares.
__host__ __device__ __forceinline__ int64_t pipe_cut(int64_t len, int i, int n, int split1, int split2, int K) {
    if (i <= 0) return 0;
    if (i >= n) return len;
    if (split1 <= 0) return len * i / n;
    const float f1 = (float)split1 * (1.0f / 65536.0f), f2 = (float)(split2 > 0 ? split2 : split1) * (1.0f / 65536.0f);
    const float r1 = (1.0f - f1) / f1, r2 = (1.0f - f2) / f2;
    float pw = 1.0f, sum = 0.0f, head = 0.0f;
    for (int j = 0; j < n; j++) {
        if (j == i) head = sum;
        sum += pw;
        pw *= j == 0 ? r1 : r2;
    }
    const float total = (float)(len + 2 * K * n);
    const int64_t c = (int64_t)(total * head / sum + 0.5f) - 2 * K * i;
    return c < 0 ? 0 : (c > len ? len : c);
}

}  // namespace

// Which group (and, in a remainder workgroup, how many packed sub-strips) workgroup `grp` owns; false: none.
__host__ __device__ __forceinline__ bool pipe_unit(const PipeArgs& a, int64_t grp, int64_t* sx, int64_t* gy, int* cnt) {
    *cnt = 0;
    if (grp < a.nstrips * a.ngroups) {
        *sx = grp % a.nstrips;
        *gy = grp / a.nstrips;
        return true;
    }
    const int64_t r = grp - a.nstrips * a.ngroups;
    if (r >= a.nrem) return false;
    *sx = a.nstrips;
    if (r < a.npk) {  // packed: groups pk_lo + r rp .. (rp at a time, all of grows rows inside the buffer)
        *gy = a.pk_lo + r * a.rp;
        const int64_t left = a.pk_hi - *gy;
        *cnt = (int)(left < a.rp ? left : a.rp);
    } else {  // lone: groups [0, pk_lo) and [pk_hi, ngroups)
        const int64_t l = r - a.npk;
        *gy = l < a.pk_lo ? l : a.pk_hi + (l - a.pk_lo);
        *cnt = 1;
    }
    return *gy < a.ngroups;
}

// Pipeline rows of workgroup group gy: [y0, y0 + L) in owned-row units (relative to out_begin added by the caller)
__host__ __device__ __forceinline__ void pipe_rows(const PipeArgs& a, int64_t gy, int p, int K, int64_t* y0, int64_t* L) {
    const int64_t total = a.out_end - a.out_begin;
    const int64_t g0 = gy * a.grows;
    const int64_t glen = a.grows < total - g0 ? a.grows : total - g0;
    const int64_t c0 = pipe_cut(glen, p, a.P, a.split1, a.split2, K), c1 = pipe_cut(glen, p + 1, a.P, a.split1, a.split2, K);
    *y0 = a.out_begin + g0 + c0;
    *L = glen > 0 ? c1 - c0 : 0;
}

template <int D, int S, int P, bool WRAP, bool BND>
__global__ __launch_bounds__(kWave * S * P) __attribute__((amdgpu_waves_per_eu(S * P / 4)))
void gol_pipe_step(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, PipeArgs a) {
    constexpr int K = D * S, NR = kNT * kR;
    __shared__ __attribute__((aligned(16))) uint32_t dstage[P][2][kR][kWave * kM];         // stage 0: [par][row][lane][word]
    __shared__ __attribute__((aligned(16))) uint32_t ring[P][S - 1][NR][kWave * kM];       // [slot][lane][word]
    __shared__ int ctr[P][S][2];                                                            // [0] rows out, [1] rows in
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if defined(GOL_PIPE_MAP) && GOL_PIPE_MAP == 1  // A/B: the stages in reverse dispatch order (the last stage oldest)
    const int p = wave / S, s = S - 1 - (wave % S + p) % S;
#else
    const int p = wave / S, s = (wave % S + p) % S;
#endif
    if (lane == 0) {
        ctr[p][s][0] = 0;
        ctr[p][s][1] = 0;
    }
    __syncthreads();
#if defined(GOL_PIPE_PRIO) && GOL_PIPE_PRIO > 0  // A/B: static wave priority by stage (MI355X_MICROARCH.md "Two waves per SIMD")
    // 1: the later half of the stages at priority 1, 2: the earlier half, 3: the last stage, 4: the later half at
    // priority 0 (the same code size as 1: the alignment control)
    if (GOL_PIPE_PRIO == 1 || GOL_PIPE_PRIO == 4 ? s >= S / 2 : (GOL_PIPE_PRIO == 2 ? s < S / 2 : s == S - 1))
        __builtin_amdgcn_s_setprio(GOL_PIPE_PRIO == 4 ? 0 : 1);
#endif
#ifdef GOL_PIPE_PAD  // A/B: shift the code after the entry by GOL_PIPE_PAD 4-byte s_nops (instruction alignment study)
    asm volatile(".rept " GOL_PIPE_STR(GOL_PIPE_PAD) "\n\ts_nop 0\n\t.endr");
#endif
    int64_t sx, gy;
    int cnt;
    int64_t y0, L;
    if (!pipe_unit(a, blockIdx.x, &sx, &gy, &cnt)) return;
    pipe_rows(a, gy, p, K, &y0, &L);
    // the group cut is float VALU math: without this the rows and the trip count derived from them live in VGPRs, and
    // the trip loop became an exec-masked loop (1200 against 970 us per 65536^2 pass, profiles/r6/pipe/r6g)
    y0 = uniform64(y0);
    L = uniform64(L);
    if (L <= 0) return;
    const int n_in = (int)(L + 2 * K - 2 * s * D);  // level-sD rows this stage reads: y0 - K + sD + i
    const int n_out = n_in - 2 * D;                 // level-(s+1)D rows it writes: y0 - K + (s+1)D + j
    const int T = (n_in + kR - 1) / kR;
    const int64_t pitch_bytes = a.pitch * 4;
    // this lane's block: strip sx holds blocks 62 sx - 1 .. 62 sx + 62 (lanes 1..62 stored); a remainder sub-strip j
    // (lanes rq j .. rq j + rq - 1) the halo block, the rem remainder blocks and the halo block, on group gy + j
    int64_t cb, delta = 0;
    bool stores;
    if (BND && cnt == 0) {  // bounded: strip sx's lanes hold blocks c .. c + 63; the board's edges on lane 0 / lane 63
        const int64_t last = a.nblocks - kWave;
        const int64_t c = sx + 1 < a.nstrips && sx * kInterior < last ? sx * kInterior : last;
        cb = c + lane;
        stores = (c == 0 || lane >= 1) && (c == last || lane <= kInterior);
    } else if (cnt == 0) {
        const int64_t first = sx * kInterior < a.nblocks - kInterior ? sx * kInterior : a.nblocks - kInterior;
        cb = first - 1 + lane;
        stores = lane >= 1 && lane <= kInterior;
    } else {  // remainder blocks: after the full strips (torus); between the last full strip and the edge strip (bounded)
        const int j = lane / a.rq, i = lane - j * a.rq;
        cb = a.nstrips * kInterior - (BND ? kInterior - 1 : 0) - 1 + i;
        stores = j < cnt && i >= 1 && i <= a.rem;
        delta = j < cnt ? (int64_t)j * a.grows * pitch_bytes : 0;
    }
    cb = cb < 0 ? cb + a.nblocks : (cb >= a.nblocks ? cb - a.nblocks : cb);
    const int load_off = (int)(cb * 4 * kM + delta);
    const int store_off = stores ? load_off : kNoStore;
    // bytes a row descriptor covers: the row, or (packed remainder) every sub-strip's row
    const int64_t span = (cnt > 1 ? (int64_t)(cnt - 1) * a.grows * pitch_bytes : 0) + a.words * 4;
    const int64_t buf_rows = WRAP ? a.rows : a.rows + 2 * a.ghost;

    uint32_t sX[D][kM], cX[D][kM], sY[D][kM], cY[D][kM], aY[D][kM];
#pragma unroll
    for (int g = 0; g < D; g++)
#pragma unroll
        for (int j = 0; j < kM; j++) sX[g][j] = cX[g][j] = sY[g][j] = cY[g][j] = aY[g][j] = 0;

    // stage 0: level-0 rows y0 - K + i; single board: buffer row (y0 - K + i) mod rows; ghost-row strip: ghost + y0 - K
    // + i, clamped into the buffer (clamped rows feed only rows nobody stores)
    int64_t lrow;
    if (WRAP) {
        lrow = (y0 - K) % a.rows;
        lrow = lrow < 0 ? lrow + a.rows : lrow;
    } else {
        lrow = a.ghost + y0 - K;
    }
    // bounded: the live rows [live_lo, live_hi) in buffer rows (32-bit scalars, as the clamp below)
    [[maybe_unused]] const int live_blo = (int)a.ghost + a.live_lo, live_bhi = (int)a.ghost + a.live_hi;
    auto dma_trip = [&](int par) {
#pragma unroll
        for (int r = 0; r < kR; r++) {
            int64_t br = lrow;
            bool dead = false;
            if (WRAP) {
                lrow = lrow + 1 == a.rows ? 0 : lrow + 1;
            } else {
                lrow++;
                // 32-bit scalar compares (the buffer holds < 2^31 rows, pipe_check): the 64-bit clamp became VALU compares
                // into VCC on stage 0's DMA issue, the pipeline's pacer
                const int b32 = (int)br, n32 = (int)buf_rows;
                br = b32 < 0 ? 0 : (b32 < n32 ? b32 : n32 - 1);
                dead = BND && (b32 < live_blo || b32 >= live_bhi);  // a dead row: loads zeros
            }
            auto* q = (__attribute__((address_space(3))) void*)&dstage[p][par][r][0];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(src + br * a.pitch, dead ? 0 : span), q, 16, load_off, 0, 0, 0);
        }
    };
    bool failed = false;
    const int spin_limit = (int)a.spin_limit;
    auto wait_ge = [&](const int* c, int need) {
        if (lds_wait(c, need, spin_limit) <= 0) {
            if (lane == 0) __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // vector atomic; bit 1: the pipeline
            failed = true;
        }
    };

    uint32_t v[kR][kM];
    if (s == 0) dma_trip(0);
    for (int t = 0; t < T && !failed; t++) {
        const int par = t & 1;
        // ---- inputs of trip t: rows kR t .. kR t + kR - 1
        if (s == 0) {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
#pragma unroll
            for (int r = 0; r < kR; r++) {
                const u32x4 x = *(const u32x4*)&dstage[p][par][r][lane * kM];
                v[r][0] = x.x;
                v[r][1] = x.y;
                v[r][2] = x.z;
                v[r][3] = x.w;
            }
            __builtin_amdgcn_sched_barrier(0);  // the reads before the next trip's DMAs overwrite the other parity
            if (t + 1 < T) dma_trip(par ^ 1);
        } else {
            lds_publish(&ctr[p][s][1], kR * t);  // trip t - 1's rows were read (and used)
            wait_ge(&ctr[p][s - 1][0], kR * t + kR < n_in ? kR * t + kR : n_in);
            u32x4 x[kR];  // the trip's 4 rows: ring slots 4t .. 4t + 3 (mod NR = 8) are one 4 KB run
            lds_read_trip(&ring[p][s - 1][(kR * t) % NR][lane * kM], x[0], x[1], x[2], x[3]);
#pragma unroll
            for (int r = 0; r < kR; r++) {
                v[r][0] = x[r].x;
                v[r][1] = x[r].y;
                v[r][2] = x[r].z;
                v[r][3] = x[r].w;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- D levels (the streaming pass's level-fenced schedule, gol_step.hip StreamWave::process): even row r takes
        // the window (X = row - 2, Y = row - 1) and leaves its sums in X, odd row r + 1 takes (Y, X)
        // bounded: this trip's rows, level by level: after level g, v[r] is row yt + r - g - 1 (owned-row coordinates),
        // over [yt - D, yt + kR - 2] in all; a trip reaching outside the live rows zeroes the rows it computes there
        [[maybe_unused]] const int yt = (int)(y0 - K + s * D) + kR * t;
        [[maybe_unused]] const bool edge_trip = BND && (yt - D < a.live_lo || yt + kR - 2 >= a.live_hi);
        uint32_t right[kR];
#pragma unroll
        for (int r = 0; r < kR; r++) right[r] = from_right<BND>(v[r][0]);
#pragma unroll
        for (int g = 0; g < D; g++) {
#pragma unroll
            for (int r = 0; r < kR; r += 2) {
                uint32_t o0[kM], o1[kM], sN[kM], cN[kM];
                row_sum_block<kM>(v[r], from_left<BND>(v[r][kM - 1]), right[r], sN, cN);
#pragma unroll
                for (int j = 0; j < kM; j++) {
                    o0[j] = life_next(sX[g][j], cX[g][j], sY[g][j], cY[g][j], sN[j], cN[j], aY[g][j]);
                    sX[g][j] = sN[j];
                    cX[g][j] = cN[j];
                }
                row_sum_block<kM>(v[r + 1], from_left<BND>(v[r + 1][kM - 1]), right[r + 1], sN, cN);
#pragma unroll
                for (int j = 0; j < kM; j++) {
                    o1[j] = life_next(sY[g][j], cY[g][j], sX[g][j], cX[g][j], sN[j], cN[j], v[r][j]);
                    sY[g][j] = sN[j];
                    cY[g][j] = cN[j];
                }
                if constexpr (BND) {
                    if (edge_trip) {  // rows outside the board stay dead (Script.fsx:6-13)
                        const int ya = yt + r - g - 1;
                        const bool da = ya < a.live_lo || ya >= a.live_hi, db = ya + 1 < a.live_lo || ya + 1 >= a.live_hi;
#pragma unroll
                        for (int j = 0; j < kM; j++) {
                            o0[j] = da ? 0u : o0[j];
                            o1[j] = db ? 0u : o1[j];
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < kM; j++) {
                    aY[g][j] = v[r + 1][j];
                    v[r][j] = o0[j];
                    v[r + 1][j] = o1[j];
                }
                if (g + 1 < D) {
                    right[r] = from_right<BND>(o0[0]);
                    right[r + 1] = from_right<BND>(o1[0]);
                    __builtin_amdgcn_sched_barrier(kAllButDs);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // level g + 1 may not be hoisted next to its exchanges
        }
        // ---- outputs: v[r] is this stage's output row j = kR t + r - 2D
        const int j0 = kR * t - 2 * D;
        if (s == S - 1) {
#pragma unroll
            for (int r = 0; r < kR; r++) {
                const int j = j0 + r;
                const bool valid = j >= 0 && j < n_out;
                const int64_t y = y0 + (valid ? j : 0);
                const u32x4 w = {v[r][0], v[r][1], v[r][2], v[r][3]};
                __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(dst + ((WRAP ? 0 : a.ghost) + y) * a.pitch, valid ? span : 0),
                                                       store_off, 0, 0);
            }
        } else if (j0 + kR > 0) {
            const int jmax = j0 + kR - 1 < n_out - 1 ? j0 + kR - 1 : n_out - 1;
            wait_ge(&ctr[p][s + 1][1], jmax + 1 - NR);  // the slots are free
#pragma unroll
            for (int r = 0; r < kR; r++) {
                const int j = j0 + r;
                if (j >= 0 && j < n_out) lds_write_row(&ring[p][s][j % NR][lane * kM], u32x4{v[r][0], v[r][1], v[r][2], v[r][3]});
            }
            lds_publish(&ctr[p][s][0], j0 + kR < n_out ? j0 + kR : n_out);
        }
    }
}

namespace {

// Pipeline shapes: K = D S generations per pass, P pipelines of S stages per 16-wave workgroup
template <int K>
struct PipeShape;
template <>
struct PipeShape<16> {
    static constexpr int D = 4, S = 4, P = 4;
};
template <>
struct PipeShape<32> {
    static constexpr int D = 4, S = 8, P = 2;
};

// Variants: the single torus board (rows wrap), torus ghost-row strips, bounded boards and strips (rows never wrap)
template <int K>
const void* pipe_kernel(bool wrap, bool bounded) {
    using Sh = PipeShape<K>;
    if (wrap) return (const void*)&gol_pipe_step<Sh::D, Sh::S, Sh::P, true, false>;
    return bounded ? (const void*)&gol_pipe_step<Sh::D, Sh::S, Sh::P, false, true>
                   : (const void*)&gol_pipe_step<Sh::D, Sh::S, Sh::P, false, false>;
}
const void* pipe_kernel_for(int k, bool wrap, bool bounded) {
    if (k == 16) return pipe_kernel<16>(wrap, bounded);
    if (k == 32) return pipe_kernel<32>(wrap, bounded);
    return nullptr;
}
int pipe_pipelines(int k) { return k == 32 ? PipeShape<32>::P : PipeShape<16>::P; }

// workgroups the device holds at once (occupancy x CUs; cached per kernel), 256 without a device (host planning)
int64_t pipe_resident_wgs(int k, bool wrap, bool bounded) {
    static std::atomic<int64_t> cache[2][3];
    const int ki = k == 32 ? 1 : 0, vi = wrap ? 0 : (bounded ? 2 : 1);
    int64_t v = cache[ki][vi].load(std::memory_order_relaxed);
    if (v > 0) return v;
    const void* fn = pipe_kernel_for(k, wrap, bounded);
    int dev = 0, cus = 0, blocks = 0;
    if (!fn || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, kWave * 16, 0) != hipSuccess || blocks <= 0 || cus <= 0) {
        (void)hipGetLastError();
        return 256;
    }
    v = (int64_t)blocks * cus;
    cache[ki][vi].store(v, std::memory_order_relaxed);
    return v;
}

}  // namespace

bool pipe_supported(int k) { return k == 16 || k == 32; }

namespace {
__device__ int g_pipe_err;  // strip passes' error word (boards pass their own)
}  // namespace

int* pipe_error_word() {
    static int* p = nullptr;
    if (!p) {
        void* q = nullptr;
        if (hipGetSymbolAddress(&q, HIP_SYMBOL(g_pipe_err)) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        p = static_cast<int*>(q);
    }
    return p;
}

// torus rows of at least one strip of stored blocks (62), bounded rows of at least one wave of blocks (64: the board's
// edges on a strip's outer lanes)
bool pipe_applies(int64_t words, int ilv, int k, bool bounded, int rag_bits) {
    return !rag_bits && ilv == kM && pipe_supported(k) && words / kM >= (bounded ? kWave : kInterior);
}

int pipe_default_split(int k) {
    // measured at 65536^2 (tools/proto): the oldest pipeline's share of a pair
    return k == 32 ? (int)(0.75 * 65536) : (int)(0.60 * 65536);
}

void plan_pipe(PipeArgs& a, int k, bool wrap, int64_t spare_waves) {
    a.P = pipe_pipelines(k);
    a.nblocks = a.words / kM;
    a.nstrips = a.nblocks / kInterior;
    a.rem = (int32_t)(a.nblocks - a.nstrips * kInterior);
    a.rq = a.rem + 2;
    a.rp = a.rem ? kWave / a.rq : 0;
    if (a.bounded) {  // strips of 64 blocks: the first stores 63 from the board's left edge, the last 63 up to its right
        // edge, the ones between 62 (halo lanes on both sides); the rem blocks left between the last of those and the
        // edge strip go to remainder workgroups as on the torus
        const int64_t edge2 = 2 * kWave - 2;  // blocks the two edge strips store
        a.nstrips = a.nblocks <= kWave ? 1 : (a.nblocks < edge2 ? 2 : 2 + (a.nblocks - edge2) / kInterior);
        a.rem = a.nstrips < 2 ? 0 : (int32_t)(a.nblocks - edge2 - (a.nstrips - 2) * kInterior);
        if (a.rem < 0) a.rem = 0;  // two edge strips overlapping
        a.rq = a.rem + 2;
        a.rp = a.rem ? kWave / a.rq : 0;
    }
    if (a.rem && a.rp < 2) {  // a remainder wider than 30 blocks: one more strip, overlapping the last full one
        a.nstrips++;
        a.rem = 0;
        a.rq = 2;
        a.rp = 0;
    }
    if (a.split1 == 0) a.split1 = pipe_default_split(k);
    if (a.split1 < 0) a.split1 = 0;
    const int64_t rows = a.out_end - a.out_begin;
    a.ngroups = a.grows = a.npk = a.nrem = 0;
    a.pk_lo = a.pk_hi = 0;
    if (rows <= 0) return;
    int64_t wgs = a.wgs_opt > 0 ? a.wgs_opt : pipe_resident_wgs(k, wrap, a.bounded != 0);
    const int64_t spare = (spare_waves + 15) / 16;
    wgs = wgs > spare + 1 ? wgs - spare : 1;
    const int64_t pitch_bytes = a.pitch * 4;
    // rows a packed group's sub-strip may stream: [out_begin + g grows - k, out_begin + (g + 1) grows + k + 4) must lie
    // in the buffer without a wrap or clamp (stage 0 reads whole trips of 4 rows, up to 3 past its last)
    const int64_t lo_lim = wrap ? 0 : -a.ghost, hi_lim = wrap ? a.rows : a.rows + a.ghost;
    auto fill = [&](int64_t ng) {
        a.grows = (rows + ng - 1) / ng;
        a.ngroups = (rows + a.grows - 1) / a.grows;
        a.pk_lo = a.pk_hi = a.ngroups;  // nothing packed: every remainder group alone
        a.npk = 0;
        if (a.rem) {
            int rp = a.rp;
            // per-lane row offsets are 32-bit byte offsets into one descriptor
            const int64_t fit = 1 + ((((int64_t)1 << 31) - 1 - a.words * 4) / (a.grows * pitch_bytes));
            if (rp > fit) rp = (int)(fit > 1 ? fit : 1);
            a.rp = rp;
            int64_t hi = a.ngroups - 1;  // the last group may be short: never packed
            const int64_t by_rows = (hi_lim - a.out_begin - k - kR) / a.grows;  // (g + 1) grows + k + 4 <= hi_lim - ob
            if (by_rows < hi) hi = by_rows;
            const bool low_ok = a.out_begin + a.grows - k >= lo_lim;  // group 1's cone inside the buffer
            if (rp >= 2 && low_ok && hi > 1 && a.grows >= k) {
                a.pk_lo = 1;
                a.pk_hi = hi;
                a.npk = (a.pk_hi - a.pk_lo + rp - 1) / rp;
            }
            a.nrem = a.npk + (a.ngroups - (a.pk_hi - a.pk_lo));
        } else {
            a.nrem = 0;
        }
    };
    int64_t ng = wgs / a.nstrips;
    // groups of at least 2K rows: a pipeline streams its rows plus a 2K-row cone, so a short launch (a ghost-row strip's
    // K-row edge band) in many tiny groups would be nearly all cone; it runs in fewer, taller groups on fewer CUs
    // (leaving the rest to the interior launch it overlaps)
    const int64_t max_ng = rows / (2 * k) > 1 ? rows / (2 * k) : 1;
    if (ng > max_ng) ng = max_ng;
    if (ng < 1) ng = 1;
    for (; ng > 1; ng--) {
        fill(ng);
        if (a.nstrips * a.ngroups + a.nrem <= wgs) break;
    }
    if (ng <= 1) fill(1);
}

int64_t pipe_grid(const PipeArgs& a) { return a.nstrips * a.ngroups + a.nrem; }

int64_t pipe_check_plan(const PipeArgs& a, int k, bool wrap) {
    int64_t bad = 0;
    const int64_t rows = a.out_end - a.out_begin;
    if (rows <= 0) return 0;
    const int64_t pitch_bytes = a.pitch * 4;
    const int64_t lo_lim = wrap ? 0 : -a.ghost, hi_lim = wrap ? a.rows : a.rows + a.ghost;
    std::vector<uint8_t> seen((size_t)(rows * a.nblocks), 0);
    for (int64_t grp = 0; grp < pipe_grid(a); grp++) {
        int64_t sx, gy;
        int cnt;
        if (!pipe_unit(a, grp, &sx, &gy, &cnt)) {
            bad++;  // a launched workgroup with nothing to do
            continue;
        }
        for (int p = 0; p < a.P; p++) {
            int64_t y0, L;
            pipe_rows(a, gy, p, k, &y0, &L);
            if (L <= 0) continue;
            // stage 0 streams level-0 rows y0 - k .. y0 + L + k - 1, in whole trips of 4
            const int64_t n_in = L + 2 * k, streamed = (n_in + kR - 1) / kR * kR;
            for (int lane = 0; lane < kWave; lane++) {
                int64_t cb, delta_rows = 0;
                bool stores;
                if (a.bounded && cnt == 0) {  // as the kernel
                    const int64_t last = a.nblocks - kWave;
                    const int64_t c = sx + 1 < a.nstrips && sx * kInterior < last ? sx * kInterior : last;
                    cb = c + lane;
                    stores = (c == 0 || lane >= 1) && (c == last || lane <= kInterior);
                } else if (cnt == 0) {
                    const int64_t first = sx * kInterior < a.nblocks - kInterior ? sx * kInterior : a.nblocks - kInterior;
                    cb = first - 1 + lane;
                    stores = lane >= 1 && lane <= kInterior;
                } else {
                    const int j = lane / a.rq, i = lane - j * a.rq;
                    cb = a.nstrips * kInterior - (a.bounded ? kInterior - 1 : 0) - 1 + i;
                    stores = j < cnt && i >= 1 && i <= a.rem;
                    delta_rows = j < cnt ? (int64_t)j * a.grows : 0;
                    if (j < cnt && (int64_t)j * a.grows * pitch_bytes + a.nblocks * 4 * kM > (((int64_t)1 << 31) - 1)) bad++;
                    if (cnt > 1 && j < cnt) {  // packed: rows relative to sub-strip 0's, no wrap / clamp allowed
                        const int64_t first_row = y0 - k + delta_rows, last_row = y0 - k + streamed - 1 + delta_rows;
                        if (first_row < lo_lim || last_row >= hi_lim) bad++;
                        if ((gy + j + 1) * a.grows > rows) bad++;  // every packed group has grows rows (the same cuts)
                    }
                }
                cb = cb < 0 ? cb + a.nblocks : (cb >= a.nblocks ? cb - a.nblocks : cb);
                if (!stores) continue;
                for (int64_t y = y0 + delta_rows; y < y0 + delta_rows + L; y++) {
                    const int64_t r = y - a.out_begin;
                    if (r < 0 || r >= rows) {
                        bad++;
                        break;
                    }
                    seen[(size_t)(r * a.nblocks + cb)] = 1;
                }
            }
        }
    }
    for (uint8_t s : seen)
        if (!s) bad++;
    return bad;
}

hipError_t launch_pipe_step(const uint32_t* src, uint32_t* dst, PipeArgs a, int k, bool wrap, hipStream_t s) {
    plan_pipe(a, k, wrap, a.spare_waves);
    const int64_t grid = pipe_grid(a);
    if (grid <= 0) return hipSuccess;
    if (!a.err) return hipErrorInvalidValue;
    if (!wrap && a.rows + 2 * a.ghost >= ((int64_t)1 << 31)) return hipErrorInvalidValue;  // 32-bit row clamp (stage 0)
    if (a.bounded && (wrap || a.nblocks < kWave)) return hipErrorInvalidValue;
    if (a.spin_limit <= 0) a.spin_limit = (int64_t)1 << 22;  // polls of >= 64 clocks: about 0.2-0.5 s
    const dim3 block(kWave * 16);
    if (k == 16) {
        using Sh = PipeShape<16>;
        if (wrap)
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, true, false>), dim3((unsigned)grid), block, 0, s, src, dst, a);
        else if (a.bounded)
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, false, true>), dim3((unsigned)grid), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, false, false>), dim3((unsigned)grid), block, 0, s, src, dst, a);
    } else if (k == 32) {
        using Sh = PipeShape<32>;
        if (wrap)
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, true, false>), dim3((unsigned)grid), block, 0, s, src, dst, a);
        else if (a.bounded)
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, false, true>), dim3((unsigned)grid), block, 0, s, src, dst, a);
        else
            hipLaunchKernelGGL((gol_pipe_step<Sh::D, Sh::S, Sh::P, false, false>), dim3((unsigned)grid), block, 0, s, src, dst, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gol
