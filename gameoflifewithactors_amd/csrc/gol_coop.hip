// gol_coop.hip -- persistent, LDS-banded pass for mid-size boards (BASELINE config 2: 4096^2) on gfx950.
//
// A 4096^2 board is 2 MiB packed: too large for one CU's LDS (gol_resident.hip), too small to fill the chip
// with the streaming pass (gol_step.hip), where each wave is one long serial chain per launch.  Here ONE
// workgroup per CU stays resident for a whole gol_step call and owns a band of B rows.  Per block of k
// generations (k <= K, B >= k) it
//   1. loads its band plus k halo rows on each side (rows wrap on a torus, GameOfLifeDriver.fs:21-25; rows
//      beyond a bounded board are dead, Script.fsx:6-13) from the board buffer into LDS,
//   2. runs k synchronous B3/S23 generations (GameOfLifeLogic.fs:59-63) between two LDS buffers with one
//      workgroup barrier per generation (the halo shrinks by a row per generation; the band stays exact),
//   3. stores its band to the other board buffer and publishes "block done" to its two neighbours,
// and before the next block waits only for its two neighbour bands (their halo rows, and that they have
// finished reading the rows it is about to overwrite).  No grid barrier, one launch per call.
//
// The band stays in LDS for the whole call; only its first and last k rows are handed to the neighbours per
// block.  Hand-off protocol (MI355X_MICROARCH.md "Valid forms", first row of the sc1 table: hipMalloc, one
// workgroup per CU): the edge rows are stored write-through (sc1), every storing wave drains them
// (s_waitcnt vmcnt(0)), a workgroup barrier, then one lane stores the band's flag (sc1); the consumer's one
// lane polls the flags with sc1 loads, a workgroup barrier, and every wave loads the rows with sc1 loads --
// no release / acquire fences (they write back / invalidate whole caches: MI355X_MICROARCH.md
// "publish-large").  Residency: the grid is one workgroup per CU, each asking for more than
// half of the CU's LDS, launched cooperatively (the runtime rejects a grid that cannot be co-resident); every
// spin is bounded and a timed-out wait raises an error word the host checks on the next synchronisation.
#include "gol_internal.h"
#include "gol_bitlogic.h"

#include <cstdlib>

namespace gol {
namespace {

constexpr int kThreads = 1024;
constexpr int kMinLds = 96 * 1024;  // > half the CU's 160 KiB: one workgroup per CU
constexpr unsigned kSpinLimit = 1u << 22;  // ~ seconds: a wait this long means a band is not resident

struct CoopArgs {
    uint32_t* buf[2];
    int64_t pitch;   // words per buffer row
    int wpr;         // words per board row (W / 32)
    int H;           // board rows
    int B;           // rows of the largest band (LDS sizing)
    int nwg;         // bands (= workgroups)
    int K;           // generations per block (<= B)
    int gens;
    int cur;         // buffer holding the board at launch
    unsigned* flags; // per band: blocks completed (zeroed before the launch)
    int* err;        // set to 1 by a timed-out wait
};

// Horizontal 3-sums of word c of an LDS row (ilv-1 layout).
template <bool BOUNDED>
__device__ __forceinline__ uint32_t lds_row(const uint32_t* row, int wpr, int c, uint32_t& s, uint32_t& cy) {
    const uint32_t m = row[c];
    const uint32_t l = (BOUNDED && c == 0) ? 0u : row[c == 0 ? wpr - 1 : c - 1];
    const uint32_t r = (BOUNDED && c == wpr - 1) ? 0u : row[c == wpr - 1 ? 0 : c + 1];
    row_sum(l, m, r, s, cy);
    return m;
}

__device__ __forceinline__ bool wait_flag(const unsigned* f, unsigned target) {
    for (unsigned i = 0; i < kSpinLimit; i++) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
        __builtin_amdgcn_s_sleep(2);
    }
    return false;
}

// sc1 (write-through / L2-coherent) word store and load for the handed-off edge rows
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool BOUNDED>
__global__ __launch_bounds__(kThreads) void gol_coop_pass(CoopArgs a) {
    extern __shared__ uint32_t lds[];
    const int band = blockIdx.x;
    const int tid = threadIdx.x;
    // balanced bands: every band has at least K rows, so a k-row halo comes from ONE neighbour band
    const int y0 = (int)((int64_t)a.H * band / a.nwg);
    const int y1 = (int)((int64_t)a.H * (band + 1) / a.nwg);
    const int own = y1 - y0;
    const int wpr = a.wpr;
    const int K = a.K;
    const int stride = (a.B + 2 * K) * wpr;  // words per LDS buffer; local row K + i = global row y0 + i
    // neighbour bands (a bounded board's end bands have one; a one-band torus is its own neighbour)
    const int up = band > 0 ? band - 1 : (BOUNDED ? -1 : a.nwg - 1);
    const int dn = band + 1 < a.nwg ? band + 1 : (BOUNDED ? -1 : 0);
    const int segs = wpr >= kThreads ? 1 : kThreads / wpr;  // row segments per column
    const int items = wpr * segs;
    const int my_sg = tid / wpr, my_c = tid - my_sg * wpr;  // this thread's first item
    const int nblk = (a.gens + K - 1) / K;
    auto wrap = [&](int gy) { return gy < 0 ? gy + a.H : (gy >= a.H ? gy - a.H : gy); };
    auto on_board = [&](int gy) { return gy >= 0 && gy < a.H; };
    uint32_t* A = lds;  // the band (+ halo) at the start of a block
    uint32_t* Bf = lds + stride;
    // the band and K halo rows per side, once, from the board
    {
        const uint32_t* src = a.buf[a.cur];
        const int n = own + 2 * K;
        for (int i = tid; i < n * wpr; i += kThreads) {
            const int r = i / wpr, c = i - r * wpr;
            const int gy = y0 - K + r;
            uint32_t v = 0;
            if (on_board(gy) || !BOUNDED) v = src[(int64_t)wrap(gy) * a.pitch + c];
            A[r * wpr + c] = v;
        }
        __syncthreads();
    }
    int x = a.cur;  // board buffer the latest hand-off went to
    for (int blk = 0; blk < nblk; blk++) {
        const int k = a.gens - blk * K < K ? a.gens - blk * K : K;
        if (blk > 0) {
            // the neighbours finished block blk - 1: their edge rows are in buf[x] (write-through), and
            // they have read ours from the buffer we are about to write (blk + 1 alternates)
            if (tid == 0) {
                bool ok = true;
                if (up >= 0) ok = wait_flag(a.flags + up, (unsigned)blk) && ok;
                if (dn >= 0) ok = wait_flag(a.flags + dn, (unsigned)blk) && ok;
                if (!ok) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            // halo rows: k above (the up band's last rows), k below (the down band's first rows)
            const uint32_t* src = a.buf[x];
            for (int i = tid; i < 2 * k * wpr; i += kThreads) {
                const int r = i / wpr, c = i - r * wpr;
                const int lr = r < k ? K - k + r : K + own + (r - k);  // local row
                const int gy = y0 - K + lr;
                uint32_t v = 0;
                if (on_board(gy) || !BOUNDED) v = ld_sc1(src + (int64_t)wrap(gy) * a.pitch + c);
                A[lr * wpr + c] = v;
            }
            __syncthreads();
        }
        // k generations in LDS: generation j writes local rows [K - k + 1 + j, K + own + k - 1 - j).  Each
        // item's row segment is fixed for the block (split of generation 0's rows) and clipped per generation:
        // no division in the generation loop.
        const int g0 = K - k + 1, g1 = K + own + k - 1;
        const int my_ra = g0 + my_sg * (g1 - g0) / segs, my_rb = g0 + (my_sg + 1) * (g1 - g0) / segs;
        for (int j = 0; j < k; j++) {
            const int r0 = g0 + j, r1 = g1 - j;
            for (int it = tid; it < items; it += kThreads) {
                int sg = my_sg, c = my_c, ra = my_ra, rb = my_rb;
                if (it != tid) {  // widths beyond 1024 words: more than one item per thread
                    sg = it / wpr;
                    c = it - sg * wpr;
                    ra = g0 + sg * (g1 - g0) / segs;
                    rb = g0 + (sg + 1) * (g1 - g0) / segs;
                }
                ra = ra < r0 ? r0 : ra;
                rb = rb > r1 ? r1 : rb;
                if (ra >= rb) continue;
                uint32_t sP, cP, sC, cC, sN, cN;
                lds_row<BOUNDED>(A + (ra - 1) * wpr, wpr, c, sP, cP);
                uint32_t mC = lds_row<BOUNDED>(A + ra * wpr, wpr, c, sC, cC);
                for (int r = ra; r < rb; r++) {
                    const uint32_t mN = lds_row<BOUNDED>(A + (r + 1) * wpr, wpr, c, sN, cN);
                    uint32_t v = life_next(sP, cP, sC, cC, sN, cN, mC);
                    if (BOUNDED && !on_board(y0 - K + r)) v = 0u;  // dead outside the board at every generation
                    Bf[r * wpr + c] = v;
                    sP = sC, cP = cC, sC = sN, cC = cN, mC = mN;
                }
            }
            __syncthreads();
            uint32_t* t = A;
            A = Bf;
            Bf = t;
        }
        if (blk + 1 == nblk) break;
        // hand-off: the band's first and last k rows, write-through, to the other board buffer
        x ^= 1;
        uint32_t* dst = a.buf[x];
        for (int i = tid; i < 2 * k * wpr; i += kThreads) {
            const int r = i / wpr, c = i - r * wpr;
            const int lr = r < k ? K + r : K + own - k + (r - k);
            st_sc1(dst + (int64_t)(y0 - K + lr) * a.pitch + c, A[lr * wpr + c]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores complete ...
        __syncthreads();                                   // ... before one lane publishes for all
        if (tid == 0) __hip_atomic_store(a.flags + band, (unsigned)(blk + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the whole band to the result buffer (the host flips the board buffer once per block)
    uint32_t* dst = a.buf[a.cur ^ (nblk & 1)];
    for (int i = tid; i < own * wpr; i += kThreads) {
        const int r = i / wpr, c = i - r * wpr;
        dst[(int64_t)(y0 + r) * a.pitch + c] = A[(K + r) * wpr + c];
    }
}

int coop_cus() {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 0;
        return n;
    }();
    return cus;
}

}  // namespace

// Generations per block: GOL_COOP_K overrides (A/B), default 8.
int coop_k() {
    const char* e = std::getenv("GOL_COOP_K");
    const int k = e ? std::atoi(e) : 8;
    return k >= 1 && k <= 64 ? k : 8;
}

bool coop_plan(int64_t W, int64_t H, int k, int* nwg, int* B) {
    const int cus = coop_cus();
    if (cus <= 0 || W < 32 || W % 32 || H < 3 || k < 1) return false;
    const int64_t wpr = W / 32;
    // balanced bands of >= k rows each (a k-row halo then comes from one neighbour band), one per CU at most
    int64_t n = H / k < cus ? H / k : cus;
    if (n < 1) return false;
    const int64_t b = (H + n - 1) / n;  // the largest band
    if (2 * (b + 2 * k) * wpr * 4 > 160 * 1024) return false;
    *nwg = (int)n;
    *B = (int)b;
    return true;
}

hipError_t launch_coop_pass(uint32_t* buf0, uint32_t* buf1, int cur, int64_t W, int64_t H, int64_t pitch,
                            int64_t gens, bool bounded, unsigned* flags, int* err, hipStream_t s) {
    const int k = coop_k();
    int nwg = 0, B = 0;
    if (!coop_plan(W, H, k, &nwg, &B) || gens < 1 || gens > INT32_MAX || pitch < W / 32) return hipErrorInvalidValue;
    CoopArgs a;
    a.buf[0] = buf0;
    a.buf[1] = buf1;
    a.pitch = pitch;
    a.wpr = (int)(W / 32);
    a.H = (int)H;
    a.B = B;
    a.nwg = nwg;
    a.K = k;
    a.gens = (int)gens;
    a.cur = cur;
    a.flags = flags;
    a.err = err;
    const size_t need = (size_t)2 * (B + 2 * k) * a.wpr * 4;
    const size_t lds = need > (size_t)kMinLds ? need : (size_t)kMinLds;
    hipError_t e = hipMemsetAsync(flags, 0, (size_t)nwg * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    const void* fn = bounded ? (const void*)&gol_coop_pass<true> : (const void*)&gol_coop_pass<false>;
    static bool attr_set[2] = {false, false};
    if (!attr_set[bounded]) {
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set[bounded] = true;
    }
    void* args[] = {&a};
    return hipLaunchCooperativeKernel(fn, dim3(nwg), dim3(kThreads), args, (unsigned)lds, s);
}

}  // namespace gol
