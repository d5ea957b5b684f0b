// gol_lanes.hip -- rows-on-lanes band pass for mid-size boards (BASELINE config 2: 4096^2) on gfx950.
//
// The cooperative pass (gol_coop.hip) spreads a band's rows over the 16 waves of a CU, so every generation ends in
// an LDS exchange of the waves' edge rows and a workgroup barrier: at 4096^2 the waves wait there ~60 % of their
// cycles.  This pass turns the band on its side.  A wave owns a WINDOW of the band -- all of its
// rows, B + 2K <= 32 of them, and U = 64 (M - 1) useful columns with 32 halo columns each side -- and steps it K
// generations with no other wave involved: no LDS and no barrier inside a block.
//
//   lane l = 32 h + r holds window row r (r < 32) and half h of the row's 64 M window cells as M words in the
//   interleaved order of gol_layout.h: word t bit b = cell M b + t of the half, so a cell's west and east neighbours
//   are the same bit of the adjacent word except at the two ends.  Half 1 is stored MIRRORED (its cell c is window
//   cell 64 M - 1 - c), so both halves' far ends are their cell 32 M - 1 and meet each other: one v_permlane32_swap
//   per row sum closes the seam, and every half-dependent step below is the same code in both halves.
//
// Per generation (GameOfLifeLogic.fs:59-63, synchronous as under the Reset->State barrier): the rows above and
// below come from lanes l - 1 / l + 1 by DPP (wave_shr / wave_shl; the rows where the two halves' lane ranges meet
// are the window's outermost rows, which the temporal block never needs), their vertical 3-sums (2 v_bitop3 per
// word), the horizontal combination from the adjacent words (2 funnel shifts per M words), and the rule of
// gol_bitlogic.h (7 v_bitop3).  Valid cells shrink by one per side and generation; after k <= K generations the
// band's rows are exact over the useful columns.
//
// Between blocks: (1) the waves of a band swap the 16 cells beside each useful edge through LDS (one barrier per
// block), so every band row is exact over the window again; (2) the band's first and last K rows leave the CU as
// data-tagged granules to the same window of the bands above and below (the hand-off of gol_coop.hip:
// MI355X_MICROARCH.md "handoff-1to1", "Valid forms" R2; parity double-buffered, epoch-tagged).  The board buffers
// are read at the start and written at the end of the launch, staged through LDS as plain words (any board
// interleave).  Rows and columns outside a bounded board are forced dead every generation (Script.fsx:6-13); the
// torus wraps rows through the band ring and columns through the wave ring (GameOfLifeDriver.fs:21-25).
#include "gol_internal.h"
#include "gol_bitlogic.h"

#include <algorithm>
#include <mutex>
#include <vector>

namespace gol {
namespace {

constexpr int kWinRows = 32;                // window rows: one per lane of a half
constexpr int kXchCells = 16;               // halo cells refreshed between blocks (K <= kXchCells)
constexpr unsigned kLaneSpinLimit = 1u << 25;  // ~ 2 s: a wait this long means a band is not resident
// Cost decomposition builds (A/B only, wrong results): 1 = no hand-off (no granule stores or polls), 2 = no hand-off
// and no edge swap between the windows (the generation loops alone)
#ifndef GOL_LANES_DECOMP
#define GOL_LANES_DECOMP 0
#endif

struct LaneArgs {
    const uint32_t* src;  // board at launch
    uint32_t* dst;        // board after `gens` generations
    uint64_t* xch;        // granules: [2 parity][nb][2 (top, bottom)][nx][M][2 halves][K rows] {word, tag}
    int64_t pitch;        // words per board row
    int nw;               // words per row (W / 32)
    int ilv;              // the board's interleave (1, 2, 4)
    int H;
    int nb;               // bands (workgroups)
    int nx;               // windows per band (waves per workgroup)
    int K;
    int gens;
    unsigned epoch;
    int poll_delay;
    unsigned spin_limit;
    int* err;
};

// Value of `v` in the lane 32 away (the other half of the same row): v_permlane32_swap trades the halves of two
// copies; x ^ y ^ v is the partner's value in both halves whichever half each copy received.
__device__ __forceinline__ uint32_t partner(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r[0] ^ r[1] ^ v;
}

// A block of MB board words (gol_layout.h: word j bit b = cell MB b + j) to / from MB plain words (bit i = cell 32 s + i)
template <int MB>
__device__ __forceinline__ void block_to_plain(const uint32_t (&wd)[MB], uint32_t (&p)[MB]) {
#pragma unroll
    for (int s = 0; s < MB; s++) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            const int q = 32 * s + i;
            v |= ((wd[q % MB] >> (q / MB)) & 1u) << i;
        }
        p[s] = v;
    }
}
template <int MB>
__device__ __forceinline__ void plain_to_block(const uint32_t (&p)[MB], uint32_t (&wd)[MB]) {
#pragma unroll
    for (int j = 0; j < MB; j++) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 32; b++) {
            const int q = MB * b + j;
            v |= ((p[q >> 5] >> (q & 31)) & 1u) << b;
        }
        wd[j] = v;
    }
}

// Board rows [first, first + n) (wrapped on a torus, dead outside a bounded board) to plain LDS rows of nw words
template <int MB, bool BOUNDED>
__device__ void stage_in(const LaneArgs& a, uint32_t* rows, int first, int n) {
    const int nblk = a.nw / MB;
    for (int idx = threadIdx.x; idx < n * nblk; idx += blockDim.x) {
        const int i = idx / nblk, k = idx - i * nblk;
        int gy = first + i;
        bool on = true;
        if (gy < 0 || gy >= a.H) {
            if (BOUNDED) on = false;
            else gy = gy < 0 ? gy + a.H : gy - a.H;
        }
        uint32_t wd[MB], p[MB];
        const uint32_t* src = a.src + (int64_t)gy * a.pitch + (int64_t)k * MB;
#pragma unroll
        for (int j = 0; j < MB; j++) wd[j] = on ? src[j] : 0u;
        if constexpr (MB == 1) p[0] = wd[0];
        else block_to_plain<MB>(wd, p);
#pragma unroll
        for (int j = 0; j < MB; j++) rows[i * a.nw + k * MB + j] = p[j];
    }
}
template <int MB>
__device__ void stage_out(const LaneArgs& a, const uint32_t* rows, int first, int n) {
    const int nblk = a.nw / MB;
    for (int idx = threadIdx.x; idx < n * nblk; idx += blockDim.x) {
        const int i = idx / nblk, k = idx - i * nblk;
        uint32_t p[MB], wd[MB];
#pragma unroll
        for (int j = 0; j < MB; j++) p[j] = rows[i * a.nw + k * MB + j];
        if constexpr (MB == 1) wd[0] = p[0];
        else plain_to_block<MB>(p, wd);
        uint32_t* dst = a.dst + (int64_t)(first + i) * a.pitch + (int64_t)k * MB;
#pragma unroll
        for (int j = 0; j < MB; j++) dst[j] = wd[j];
    }
}

// A lane's M granules sit `stride` granules apart: word t of every publishing lane of a window side is one contiguous
// run (lanes of consecutive rows at consecutive granules), so each store / poll instruction touches two short runs
// instead of 64 lanes 8 M bytes apart.
template <int M>
__device__ __forceinline__ void st_granules(uint64_t* p, int stride, const uint32_t (&w)[M], unsigned tag) {
#pragma unroll
    for (int t = 0; t < M; t++)
        __hip_atomic_store(p + (int64_t)t * stride, (uint64_t)tag << 32 | w[t], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// The lane's M granules (src == nullptr: the lane needs none), in one batch of 8-byte sc1 loads per poll round after
// `delay` s_sleep periods; false after the spin limit.
// Returns kGot, kTimedOut, or kLaunchFailed: the launch's error word (another wave timed out), read only while this
// wave waits, every 32 polls -- not at every block, where its load (and its s_waitcnt, which also waited for the
// wave's own granule stores) was a memory round trip in front of every hand-off.
constexpr int kGot = 0, kTimedOut = 1, kLaunchFailed = 2;
template <int M>
__device__ __forceinline__ int ld_granules(const uint64_t* src, int stride, uint32_t (&w)[M], unsigned tag, int delay,
                                           unsigned spin_limit, const int* err) {
    for (int i = 0; i < delay; i++) __builtin_amdgcn_s_sleep(1);
    uint64_t v[M];
    for (unsigned it = 0;; it++) {
        bool miss = false;
#pragma unroll
        for (int t = 0; t < M; t++) {
            v[t] = src ? __hip_atomic_load(src + (int64_t)t * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : (uint64_t)tag << 32;
            miss = miss || (unsigned)(v[t] >> 32) != tag;
        }
        if (__builtin_amdgcn_ballot_w64(miss) == 0) break;  // wave-uniform exit
        if (it == spin_limit) return kTimedOut;
        if ((it & 31) == 31 &&
            __builtin_amdgcn_ballot_w64(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) != 0)
            return kLaunchFailed;
        __builtin_amdgcn_s_sleep(1);
    }
    if (src)
#pragma unroll
        for (int t = 0; t < M; t++) w[t] = (uint32_t)v[t];
    return kGot;
}

template <int M, int MB, bool BOUNDED>
__global__ __launch_bounds__(1024) void gol_lane_pass(LaneArgs a) {
    constexpr int U = 64 * (M - 1);  // useful cells per window
    extern __shared__ uint32_t lds[];  // plain board rows [kWinRows][nw], then edge slots [2][nx][2][32]
    uint32_t* slots = lds + kWinRows * a.nw;
    const int band = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int x = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int h = lane >> 5, r = lane & 31;
    const int nx = a.nx;
    const int y0 = (int)((int64_t)a.H * band / a.nb);
    const int B = (int)((int64_t)a.H * (band + 1) / a.nb) - y0;
    const int K = a.K;
    const int L = B + 2 * K;  // window rows in use
    const int nw = a.nw;
    // plain groups of the half: h = 0 reads groups G0 + g, h = 1 groups G1 - g bit-reversed (mirrored half)
    const int G0 = x * (U / 32) - 1, G1 = (x + 1) * (U / 32);

    // ---- the window from the board, through LDS as plain words
    stage_in<MB, BOUNDED>(a, lds, y0 - K, L);
    __syncthreads();
    uint32_t w[M];
    {
        uint32_t p[M];
#pragma unroll
        for (int g = 0; g < M; g++) {
            int G = h == 0 ? G0 + g : G1 - g;
            bool on = r < L;
            if (G < 0 || G >= nw) {
                if (BOUNDED) on = false;
                else G = G < 0 ? G + nw : G - nw;
            }
            const uint32_t v = on ? lds[r * nw + G] : 0u;
            p[g] = h ? __builtin_bitreverse32(v) : v;
        }
#pragma unroll
        for (int t = 0; t < M; t++) w[t] = 0;
#pragma unroll
        for (int c = 0; c < 32 * M; c++) w[c % M] |= ((p[c >> 5] >> (c & 31)) & 1u) << (c / M);
    }

    // bounded: per lane, the bits that stay (rows outside the board: none; a half whose outer 32 cells lie beyond the
    // board's edge: all but those, which are bits 0 .. (31 - t) / M of word t)
    [[maybe_unused]] uint32_t keepA = ~0u, keepB = ~0u;  // words t <= 31 % M, and the rest
    [[maybe_unused]] bool edge = false;                    // wave-uniform: the window touches the board's edge
    if constexpr (BOUNDED) {
        const int gy = y0 - K + r;
        const bool row_out = gy < 0 || gy >= a.H;
        const bool col_out = (h == 0 && x == 0) || (h == 1 && x == nx - 1);
        constexpr int q = 31 / M;
        keepA = row_out ? 0u : (col_out ? ~((2u << q) - 1u) : ~0u);
        keepB = row_out ? 0u : (col_out ? ~((1u << q) - 1u) : ~0u);
        edge = band == 0 || band == a.nb - 1 || x == 0 || x == nx - 1;
    }

    const int up = band > 0 ? band - 1 : (BOUNDED ? -1 : a.nb - 1);
    const int dn = band + 1 < a.nb ? band + 1 : (BOUNDED ? -1 : 0);
    // granule of word 0 of (parity, band b, side, row e) for this lane's window and half; word t is 2K further
    auto xrow = [&](int parity, int b, int side, int e) {
        return a.xch + (((((int64_t)parity * a.nb + b) * 2 + side) * nx + x) * M) * (2 * K) + h * K + e;
    };
    auto tag_of = [&](int blk) { return a.epoch << 16 | (unsigned)(blk + 1); };

    const int nblk = (a.gens + K - 1) / K;
    bool failed = false;
    for (int blk = 0; blk < nblk; blk++) {
        const int k = a.gens - blk * K < K ? a.gens - blk * K : K;
        if (GOL_LANES_DECOMP == 0 && blk > 0) {
            // the halo rows: the same window of the neighbour bands' edge rows, block blk - 1
            const int par = (blk - 1) & 1;
            const uint64_t* src = nullptr;
            if (r < K && up >= 0) src = xrow(par, up, 1, r);
            else if (r >= K + B && r < L && dn >= 0) src = xrow(par, dn, 0, r - K - B);
            // after a failed wait (this wave's, or another's: the error word, read while waiting) no more waits
            if (!failed && __builtin_amdgcn_ballot_w64(src != nullptr) != 0) {
                const int st = ld_granules<M>(src, 2 * K, w, tag_of(blk - 1), a.poll_delay, a.spin_limit, a.err);
                if (st == kTimedOut) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (st != kGot) failed = true;
            }
        }
        for (int j = 0; j < k; j++) {
            uint32_t sv[M], cv[M];
#pragma unroll
            for (int t = 0; t < M; t++) {
                const uint32_t above = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[t], 0x138, 0xf, 0xf, true);  // wave_shr:1
                const uint32_t below = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[t], 0x130, 0xf, 0xf, true);  // wave_shl:1
                sv[t] = lut3<0x96>(above, w[t], below);
                cv[t] = lut3<0xE8>(above, w[t], below);
            }
            // the two ends of the half: west of cell 0 is outside the window (0); east of cell 32 M - 1 is the
            // other half's cell 32 M - 1
            const uint32_t ps = partner(sv[M - 1]), pc = partner(cv[M - 1]);
            const uint32_t sw0 = sv[M - 1] << 1, cw0 = cv[M - 1] << 1;
            const uint32_t sel = (sv[0] >> 1) | (ps & 0x80000000u), cel = (cv[0] >> 1) | (pc & 0x80000000u);
#pragma unroll
            for (int t = 0; t < M; t++)
                w[t] = life_next(t ? sv[t - 1] : sw0, t ? cv[t - 1] : cw0, sv[t], cv[t], t + 1 < M ? sv[t + 1] : sel,
                                 t + 1 < M ? cv[t + 1] : cel, w[t]);
            if constexpr (BOUNDED) {
                if (edge)
#pragma unroll
                    for (int t = 0; t < M; t++) w[t] &= t <= 31 % M ? keepA : keepB;
            }
        }
        if (blk + 1 == nblk) break;
        // ---- the cells beside the useful edges, between the band's windows (LDS, one barrier)
        if (GOL_LANES_DECOMP < 2) {
            const int par = blk & 1;
            uint32_t e = 0;  // cells [32, 48) of the half: the useful edge (h = 0: left, h = 1: right, reversed)
#pragma unroll
            for (int i = 0; i < kXchCells; i++) {
                constexpr int c0 = 32;
                const int c = c0 + i;
                e |= ((w[c % M] >> (c / M)) & 1u) << i;
            }
            slots[((par * nx + x) * 2 + h) * 32 + r] = e;
            __syncthreads();
            // h = 0: cells [16, 32) are the left neighbour window's right edge; h = 1: the right neighbour's left edge.
            // The neighbour's edge bit i is this half's cell 31 - i (both halves count outward from their edge).
            int xn = h == 0 ? x - 1 : x + 1;
            bool on = true;
            if (xn < 0 || xn >= nx) {
                if (BOUNDED) on = false;
                else xn = xn < 0 ? xn + nx : xn - nx;
            }
            const uint32_t v = on ? slots[((par * nx + xn) * 2 + (h ^ 1)) * 32 + r] : 0u;
#pragma unroll
            for (int j = 32 - kXchCells; j < 32; j++) {
                const int t = j % M, b = j / M, s = 31 - j;  // the bit of v for cell j
                const uint32_t bit = s >= b ? v >> (s - b) : v << (b - s);
                w[t] = (w[t] & ~(1u << b)) | (bit & (1u << b));
            }
        }
        // ---- hand-off: the band's first and last K rows (a band shorter than 2K rows sends some to both sides)
        if (GOL_LANES_DECOMP == 0) {
            const int par = blk & 1;
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const int e = side == 0 ? r - K : r - B;
                if (e >= 0 && e < K && r < L) st_granules<M>(xrow(par, band, side, e), 2 * K, w, tag_of(blk));
            }
        }
    }

    // ---- the band's rows to the board, through LDS as plain words
    __syncthreads();
    if (r >= K && r < K + B) {
#pragma unroll
        for (int g = 1; g < M; g++) {
            uint32_t p = 0;
#pragma unroll
            for (int i = 0; i < 32; i++) {
                const int c = 32 * g + i;
                p |= ((w[c % M] >> (c / M)) & 1u) << i;
            }
            const int G = h == 0 ? G0 + g : G1 - g;
            lds[(r - K) * nw + G] = h ? __builtin_bitreverse32(p) : p;
        }
    }
    __syncthreads();
    stage_out<MB>(a, lds, y0, B);
}

constexpr int kLaneM[] = {3, 5, 9, 17};

template <int M, int MB>
const void* lane_kernel_mb(bool bounded) {
    return bounded ? (const void*)&gol_lane_pass<M, MB, true> : (const void*)&gol_lane_pass<M, MB, false>;
}
template <int M>
const void* lane_kernel_m(int ilv, bool bounded) {
    switch (ilv) {
        case 1: return lane_kernel_mb<M, 1>(bounded);
        case 2: return lane_kernel_mb<M, 2>(bounded);
        case 4: return lane_kernel_mb<M, 4>(bounded);
    }
    return nullptr;
}
const void* lane_kernel(int m, int ilv, bool bounded) {
    switch (m) {
        case 3: return lane_kernel_m<3>(ilv, bounded);
        case 5: return lane_kernel_m<5>(ilv, bounded);
        case 9: return lane_kernel_m<9>(ilv, bounded);
        case 17: return lane_kernel_m<17>(ilv, bounded);
    }
    return nullptr;
}

}  // namespace

bool lanes_plan(int64_t W, int64_t H, int k, int m_opt, LanesPlan* out) {
    if (W < 256 || W % 32 || W > 16384 || H < 3 || k < 1 || k > kXchCells) return false;
    int m = 0;
    if (m_opt) {
        for (int c : kLaneM)
            if (c == m_opt) m = c;
    } else {
        // narrow rows: 128-column windows (more, shorter waves on a small board: 256^2 bounded 0.28 vs 0.32 us per
        // generation at 256 columns, 512^2 0.28 vs 0.33, 512 x 4096 0.33 vs 0.39, profiles/r4/lanes_m3_r.log); wide
        // rows: 512 (fewer halo columns)
        m = W <= 1024 ? (W % 128 == 0 ? 3 : 0) : (W % 512 == 0 ? 9 : (W % 256 == 0 ? 5 : 0));
    }
    if (!m) return false;
    const int64_t u = 64 * (m - 1);
    if (W % u || W / u > 16) return false;
    const int nx = (int)(W / u);
    const int64_t bmax = kWinRows - 2 * k;  // rows a window holds beside its 2k halo rows
    if (bmax < k) return false;
    // the tallest bands that fit a window (the fewest halo rows), more of them while the chip has idle SIMDs,
    // never shorter than k (a k-row halo then comes from ONE neighbour band)
    int64_t nb = (H + bmax - 1) / bmax;
    const int64_t most = H / k;
    const int64_t fill = (1024 + nx - 1) / nx;
    if (nb < fill) nb = std::min(fill, most);
    if (nb > most || nb < 1 || (H + nb - 1) / nb > bmax) return false;
    out->m = m;
    out->nx = nx;
    out->nb = (int)nb;
    out->bmax = (int)((H + nb - 1) / nb);
    return true;
}

int64_t lanes_xch_words(const LanesPlan& p, int k) { return (int64_t)2 * p.nb * 2 * k * p.nx * 2 * p.m * 2; }

namespace {
// LDS of one band: its plain board rows and the edge slots, raised so that at most ceil(nb / CUs) workgroups share a CU
// (the dispatcher would otherwise stack two bands on one CU while another idles, and every band waits on the slowest)
size_t lanes_lds(const LanesPlan& p, int64_t W) {
    size_t lds = ((size_t)kWinRows * (size_t)(W / 32) + (size_t)2 * p.nx * 64) * sizeof(uint32_t);
    const int cus = device_cus();
    if (cus > 0) {
        const size_t per_cu = ((size_t)p.nb + cus - 1) / cus;
        const size_t floor = (size_t)160 * 1024 / (per_cu + 1) + 1024;
        if (floor * per_cu <= (size_t)160 * 1024 && floor > lds) lds = floor;
    }
    return lds;
}
}  // namespace

bool lanes_fits(int64_t W, int64_t H, int k, int m_opt, int ilv, bool bounded) {
    LanesPlan p;
    if (!lanes_plan(W, H, k, m_opt, &p) || (W / 32) % ilv) return false;
    const void* fn = lane_kernel(p.m, ilv, bounded);
    if (!fn || set_max_dynamic_lds(fn, 96 * 1024) != hipSuccess) return false;
    const int64_t resident = persistent_capacity(fn, (unsigned)(64 * p.nx), lanes_lds(p, W));
    return resident >= p.nb;
}

hipError_t launch_lanes_pass(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch, int ilv, int k,
                             int64_t gens, bool bounded, unsigned epoch, int* err, uint32_t* xch, int64_t xch_words,
                             hipStream_t s, int m_opt, const CoopTuning& tune) {
    LanesPlan p;
    if (!lanes_plan(W, H, k, m_opt, &p) || gens < 1 || gens > 65535 || pitch < W / 32 || (W / 32) % ilv ||
        lanes_xch_words(p, k) > xch_words)
        return hipErrorInvalidValue;
    const void* fn = lane_kernel(p.m, ilv, bounded);
    if (!fn) return hipErrorInvalidValue;
    LaneArgs a;
    a.src = src;
    a.dst = dst;
    a.xch = reinterpret_cast<uint64_t*>(xch);
    a.pitch = pitch;
    a.nw = (int)(W / 32);
    a.ilv = ilv;
    a.H = (int)H;
    a.nb = p.nb;
    a.nx = p.nx;
    a.K = k;
    a.gens = (int)gens;
    a.epoch = epoch & 0xffffu;
    a.poll_delay = tune.poll_delay >= 0 ? tune.poll_delay : 8;
    a.spin_limit = tune.spin_limit ? tune.spin_limit : kLaneSpinLimit;
    a.err = err;
    const size_t lds = lanes_lds(p, W);
    if (hipError_t e = set_max_dynamic_lds(fn, 96 * 1024)) return e;
    void* args[] = {&a};
    return launch_persistent(fn, (unsigned)p.nb, (unsigned)(64 * p.nx), args, lds, s, !tune.plain_launch);
}

}  // namespace gol
