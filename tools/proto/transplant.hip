// transplant.hip -- round-6 A/B: the prototype's kernel (pipe_proto.hip, in namespace proto) and the library's
// gol::launch_pipe_step timed alternately in ONE process on one board, with pipe_proto's method.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <utility>
#include <vector>

#include "gol_bitlogic.h"
#include "gol_internal.h"
#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

namespace proto {
using namespace gol;
static constexpr int kWave = 64;
static constexpr int kInterior = 62;
static constexpr int kNoStore = 0x7ffffff0;
static constexpr int kRsrcWord3 = 0x00020000;
static constexpr int kWaitVm0 = 0x0F70;
static constexpr int kAllButDs = 0x1 | 0x2 | 0x4 | 0x8 | 0x10 | 0x20 | 0x40 | 0x400;
static constexpr long kSpinLimit = 1l << 24;  // ~ 0.5-1 s of s_sleep 1

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct PipeArgs {
    int64_t rows;     // H
    int64_t words;    // W / 32
    int64_t nblocks;  // words / M
    int64_t nstrips, ngroups, grows;  // full column strips (62 blocks); group segments per strip, of grows rows
    int rem, rq, rp;                  // remainder blocks past the full strips, lanes per sub-strip (rem + 2), sub-strips per wave
    int64_t nrem;                     // remainder workgroups (after nstrips x ngroups)
    int split1, split2;               // pipeline shares by age (1/65536; 0 = equal shares)
    int rot;                          // 1: pipeline p's stage s is wave S p + (s + p) % S (every SIMD holds every stage)
    unsigned* err;
};

// First row (relative to the group segment of len rows) of the i-th oldest of n pipelines: shares fall geometrically
// with age (the oldest wave of a SIMD issues first), ratio (1 - f1) / f1 after the oldest, (1 - f2) / f2 after that.
__device__ __forceinline__ int64_t pipe_cut(int64_t len, int i, int n, int split1, int split2, int K) {
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
    int64_t c = (int64_t)(total * head / sum + 0.5f) - 2 * K * i;
    return c < 0 ? 0 : (c > len ? len : c);
}

__device__ __forceinline__ uint32_t from_left(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xf, 0xf, false);  // wave_ror:1
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xf, 0xf, false);  // wave_rol:1
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, kRsrcWord3);
}
template <int M>
__device__ __forceinline__ void gstore(__amdgpu_buffer_rsrc_t r, int off, const uint32_t (&w)[M]) {
    if constexpr (M == 4) {
        const u32x4 t = {w[0], w[1], w[2], w[3]};
        __builtin_amdgcn_raw_buffer_store_b128(t, r, off, 0, 0);
    } else if constexpr (M == 2) {
        const u32x2 t = {w[0], w[1]};
        __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(w[0], r, off, 0, 0);
    }
}
__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int M, int D, int S, int P, int NT>
struct PipeCfg {
    static constexpr int R = 4;
    static constexpr int K = D * S;
    static constexpr int NR = NT * R;  // ring rows
    static constexpr int kThreads = kWave * P * S;
};

template <int M, int D, int S, int P, int NT, int MINW, bool X16>
__global__ __launch_bounds__((PipeCfg<M, D, S, P, NT>::kThreads)) __attribute__((amdgpu_waves_per_eu(MINW)))
void pipe_step(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, PipeArgs a) {
    using C = PipeCfg<M, D, S, P, NT>;
    constexpr int R = C::R, K = C::K, NR = C::NR;
    // stage 0's LDS-DMA rows: [par][row][word][lane] (dword DMAs) or [par][row][lane][word] (X16: one 16-byte DMA per row)
    __shared__ __attribute__((aligned(16))) uint32_t dstage[P][2][R][M * kWave];
    __shared__ __attribute__((aligned(16))) uint32_t ring[P][S > 1 ? S - 1 : 1][NR][kWave * M];  // [slot][lane * M + word]
    __shared__ int ctr[P][S][2];                                    // [0] rows published (out), [1] rows read (in)
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p = wave / S, s = a.rot ? (wave % S + p) % S : wave % S;
    if (lane == 0) {
        ctr[p][s][0] = 0;
        ctr[p][s][1] = 0;
    }
    __syncthreads();
    // workgroup = one group: strip sx, group segment gy; pipeline p (p = 0 the oldest) takes its share of its rows.
    // Remainder workgroups hold rp sub-strips of (rem + 2) lanes (a halo lane, the rem remainder blocks, a halo lane),
    // sub-strip j on group segment gy + j (a per-lane row offset): the lone groups 0 and ngroups - 1 (their rows wrap),
    // then the others rp at a time.
    const int64_t grp = blockIdx.x;
    int64_t sx, gy;
    int cnt = 0;  // sub-strips (remainder workgroups)
    if (grp < a.nstrips * a.ngroups) {
        sx = grp % a.nstrips;
        gy = grp / a.nstrips;
    } else {
        const int64_t r = grp - a.nstrips * a.ngroups;
        if (r >= a.nrem) return;
        sx = a.nstrips;
        if (r == 0 || (r == 1 && a.ngroups > 1)) {
            gy = r == 0 ? 0 : a.ngroups - 1;
            cnt = 1;
        } else {
            gy = 1 + (r - 2) * a.rp;
            const int64_t left = a.ngroups - 1 - gy;
            cnt = (int)(left < a.rp ? left : a.rp);
        }
    }
    const int64_t g0 = gy * a.grows;
    if (g0 >= a.rows) return;
    const int64_t glen = a.grows < a.rows - g0 ? a.grows : a.rows - g0;
    const int64_t y0 = g0 + pipe_cut(glen, p, P, a.split1, a.split2, K);
    const int64_t L = g0 + pipe_cut(glen, p + 1, P, a.split1, a.split2, K) - y0;
    if (L <= 0) return;
    const int n_in = (int)(L + 2 * K - 2 * s * D);
    const int n_out = n_in - 2 * D;
    const int T = (n_in + R - 1) / R;
    // column strip sx: lanes 1..62 store blocks 62 sx .. 62 sx + 61; remainder sub-strip j = lane / rq, lane i in it
    int64_t cb;
    bool stores;
    int64_t delta = 0;  // bytes: this lane's sub-strip's rows
    if (cnt == 0) {
        cb = sx * kInterior - 1 + lane;
        stores = lane >= 1 && lane <= kInterior;
    } else {
        const int j = lane / a.rq, i = lane - j * a.rq;
        cb = a.nstrips * kInterior - 1 + i;
        stores = j < cnt && i >= 1 && i <= a.rem;
        delta = j < cnt ? (int64_t)j * a.grows * a.words * 4 : 0;
    }
    cb = cb < 0 ? cb + a.nblocks : (cb >= a.nblocks ? cb - a.nblocks : cb);
    const int load_off = (int)(cb * 4 * M + delta);
    const int store_off = stores ? load_off : kNoStore;
    // bytes a row descriptor covers: the row, or every sub-strip's row
    const int64_t row_bytes = (cnt > 1 ? (int64_t)(cnt - 1) * a.grows * a.words * 4 : 0) + a.words * 4;

    uint32_t sX[D][M], cX[D][M], sY[D][M], cY[D][M], aY[D][M];
#pragma unroll
    for (int g = 0; g < D; g++)
#pragma unroll
        for (int j = 0; j < M; j++) sX[g][j] = cX[g][j] = sY[g][j] = cY[g][j] = aY[g][j] = 0;

    // stage 0: level-0 rows y0 - K + i (mod H)
    int64_t lrow = y0 - K;
    lrow = lrow < 0 ? lrow + a.rows : lrow;
    auto dma_trip = [&](int par) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const __amdgpu_buffer_rsrc_t rs = rsrc(src + lrow * a.words, row_bytes);
            lrow = lrow + 1 == a.rows ? 0 : lrow + 1;
            if constexpr (X16) {
                auto* q = (__attribute__((address_space(3))) void*)&dstage[p][par][r][0];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, q, 16, load_off, 0, 0, 0);
            } else {
#pragma unroll
                for (int j = 0; j < M; j++) {
                    auto* q = (__attribute__((address_space(3))) void*)&dstage[p][par][r][j * kWave];
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, q, 4, load_off + 4 * j, 0, 0, 0);
                }
            }
        }
    };
    bool failed = false;
    auto wait_ge = [&](const int* c, int need) {
        long spins = 0;
        while (lds_ld(c) < need) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(a.err, 1u);
                failed = true;
                break;
            }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };

    uint32_t v[R][M];
    if (s == 0) dma_trip(0);
    for (int t = 0; t < T && !failed; t++) {
        const int par = t & 1;
        // ---- inputs of trip t: rows R t .. R t + R - 1
        if (s == 0) {
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
#pragma unroll
            for (int r = 0; r < R; r++) {
                if constexpr (X16) {
                    const u32x4 x = *(const u32x4*)&dstage[p][par][r][lane * 4];
                    v[r][0] = x.x;
                    v[r][1] = x.y;
                    v[r][2] = x.z;
                    v[r][3] = x.w;
                } else {
#pragma unroll
                    for (int j = 0; j < M; j++) v[r][j] = dstage[p][par][r][j * kWave + lane];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 < T) dma_trip(par ^ 1);
        } else {
            lds_st(&ctr[p][s][1], R * t);  // trip t-1's rows were read (and used)
            const int need = R * t + R < n_in ? R * t + R : n_in;
            wait_ge(&ctr[p][s - 1][0], need);
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t* q = &ring[p][s - 1][(R * t + r) % NR][lane * M];
                if constexpr (M == 4) {
                    const u32x4 x = *(const u32x4*)q;
                    v[r][0] = x.x;
                    v[r][1] = x.y;
                    v[r][2] = x.z;
                    v[r][3] = x.w;
                } else if constexpr (M == 2) {
                    const u32x2 x = *(const u32x2*)q;
                    v[r][0] = x.x;
                    v[r][1] = x.y;
                } else {
                    v[r][0] = q[0];
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- D levels
        uint32_t right[R];
#pragma unroll
        for (int r = 0; r < R; r++) right[r] = from_right(v[r][0]);
#pragma unroll
        for (int g = 0; g < D; g++) {
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                uint32_t o0[M], o1[M], sN[M], cN[M];
                row_sum_block<M>(v[r], from_left(v[r][M - 1]), right[r], sN, cN);
#pragma unroll
                for (int j = 0; j < M; j++) {
                    o0[j] = life_next(sX[g][j], cX[g][j], sY[g][j], cY[g][j], sN[j], cN[j], aY[g][j]);
                    sX[g][j] = sN[j];
                    cX[g][j] = cN[j];
                }
                row_sum_block<M>(v[r + 1], from_left(v[r + 1][M - 1]), right[r + 1], sN, cN);
#pragma unroll
                for (int j = 0; j < M; j++) {
                    o1[j] = life_next(sY[g][j], cY[g][j], sX[g][j], cX[g][j], sN[j], cN[j], v[r][j]);
                    sY[g][j] = sN[j];
                    cY[g][j] = cN[j];
                }
#pragma unroll
                for (int j = 0; j < M; j++) {
                    aY[g][j] = v[r + 1][j];
                    v[r][j] = o0[j];
                    v[r + 1][j] = o1[j];
                }
                if (g + 1 < D) {
                    right[r] = from_right(o0[0]);
                    right[r + 1] = from_right(o1[0]);
                    __builtin_amdgcn_sched_barrier(kAllButDs);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- outputs: v[r] is output row j = R t + r - 2D
        const int j0 = R * t - 2 * D;
        if (s == S - 1) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int j = j0 + r;
                const bool valid = j >= 0 && j < n_out;
                const int64_t y = y0 + (valid ? j : 0);
                gstore<M>(rsrc(dst + y * a.words, valid ? row_bytes : 0), store_off, v[r]);
            }
        } else if (j0 + R > 0) {
            const int jmax = j0 + R - 1 < n_out - 1 ? j0 + R - 1 : n_out - 1;
            wait_ge(&ctr[p][s + 1][1], jmax + 1 - NR);
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int j = j0 + r;
                if (j >= 0 && j < n_out) {
                    uint32_t* q = &ring[p][s][j % NR][lane * M];
                    if constexpr (M == 4) {
                        *(u32x4*)q = u32x4{v[r][0], v[r][1], v[r][2], v[r][3]};
                    } else if constexpr (M == 2) {
                        *(u32x2*)q = u32x2{v[r][0], v[r][1]};
                    } else {
                        q[0] = v[r][0];
                    }
                }
            }
            lds_st(&ctr[p][s][0], j0 + R < n_out ? j0 + R : n_out);
        }
    }
}

// naive reference: one thread per (row, block), one generation, same layout
template <int M>
__global__ void ref_step(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int64_t rows, int64_t words) {
    const int64_t nblocks = words / M;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * nblocks) return;
    const int64_t y = idx / nblocks, b = idx % nblocks;
    uint32_t s[3][M], c[3][M], ctr[M];
    for (int d = 0; d < 3; d++) {
        int64_t yy = y + d - 1;
        yy = yy < 0 ? yy + rows : (yy >= rows ? yy - rows : yy);
        const uint32_t* row = src + yy * words;
        uint32_t w[M];
        for (int j = 0; j < M; j++) w[j] = row[b * M + j];
        const int64_t bp = b == 0 ? nblocks - 1 : b - 1, bn = b == nblocks - 1 ? 0 : b + 1;
        row_sum_block<M>(w, row[bp * M + M - 1], row[bn * M], s[d], c[d]);
        if (d == 1)
            for (int j = 0; j < M; j++) ctr[j] = w[j];
    }
    for (int j = 0; j < M; j++) dst[y * words + b * M + j] = life_next(s[0][j], c[0][j], s[1][j], c[1][j], s[2][j], c[2][j], ctr[j]);
}

__global__ void seed_k(uint32_t* b, int64_t n, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = seed ^ (uint64_t)i;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    b[i] = (uint32_t)z;
}
__global__ void diff_k(const uint32_t* x, const uint32_t* y, int64_t n, unsigned long long* cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && x[i] != y[i]) atomicAdd(cnt, 1ull);
}

struct Runner {
    virtual ~Runner() {}
    virtual const char* name() = 0;
    virtual int K() = 0;
    virtual int M() = 0;
    virtual bool run(const uint32_t* s, uint32_t* d, int64_t H, int64_t words, unsigned* err, int cus, hipStream_t st) = 0;
    virtual void info() = 0;
    virtual bool occ_ok() = 0;
};
static int g_split1 = 0, g_split2 = 0, g_rot = 0;
template <int M_, int D, int S, int P, int NT, int MINW, bool X16 = false>
struct PipeRunner : Runner {
    static_assert(!X16 || M_ == 4, "16-byte DMAs: M = 4");
    using C = PipeCfg<M_, D, S, P, NT>;
    char nm[96];
    PipeRunner() { snprintf(nm, sizeof nm, "pipe<M%d,D%d,S%d,P%d,NT%d,W%d%s>", M_, D, S, P, NT, MINW, X16 ? ",X16" : ""); }
    const char* name() override { return nm; }
    int K() override { return C::K; }
    int M() override { return M_; }
    int occ = 0;
    int wgs_per_cu() {
        if (occ) return occ;
        int n = 0;
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pipe_step<M_, D, S, P, NT, MINW, X16>, C::kThreads, 0));
        return occ = n;
    }
    bool occ_ok() override { return wgs_per_cu() > 0; }
    void info() override {
        hipFuncAttributes at;
        CHECK(hipFuncGetAttributes(&at, (const void*)pipe_step<M_, D, S, P, NT, MINW, X16>));
        printf("  %s: vgprs %d sgprs? scratch %zu B lds %zu B, workgroups/CU %d\n", nm, at.numRegs, at.localSizeBytes,
               at.sharedSizeBytes, wgs_per_cu());
    }
    bool run(const uint32_t* s, uint32_t* d, int64_t H, int64_t words, unsigned* err, int cus, hipStream_t st) override {
        PipeArgs a;
        a.rows = H;
        a.words = words;
        a.nblocks = words / M_;
        const int64_t wgs = (int64_t)cus * wgs_per_cu();
        a.nstrips = a.nblocks / kInterior;
        a.rem = (int)(a.nblocks - a.nstrips * kInterior);
        a.rq = a.rem + 2;
        a.rp = a.rem ? kWave / a.rq : 0;
        if (a.rem && a.rp < 2) {  // a wide remainder: one more (overlapping) strip instead
            a.nstrips++;
            a.rem = 0;
            a.rp = 0;
        }
        // group segments per strip: the most that fit one round of resident workgroups, remainder workgroups included
        int64_t ng = wgs / a.nstrips;
        for (; ng > 1; ng--) {
            const int64_t nrem = a.rem ? (ng <= 2 ? ng : 2 + (ng - 2 + a.rp - 1) / a.rp) : 0;
            if (a.nstrips * ng + nrem <= wgs) break;
        }
        if (ng < 1) ng = 1;
        a.grows = (H + ng - 1) / ng;
        ng = (H + a.grows - 1) / a.grows;
        // packed sub-strips: a group's rows plus the K-row cones stay inside the board (the lone groups 0 and ng - 1 wrap)
        if (a.rem && H - (ng - 1) * a.grows < C::K + 4) {
            printf("  short last group: skipped (prototype)\n");
            return false;
        }
        a.ngroups = ng;
        a.nrem = a.rem ? (ng <= 2 ? ng : 2 + (ng - 2 + a.rp - 1) / a.rp) : 0;
        if (a.rem && ng <= 2) a.nrem = ng;
        a.split1 = g_split1;
        a.split2 = g_split2;
        a.rot = g_rot;
        a.err = err;
        const int64_t grid = a.nstrips * a.ngroups + a.nrem;
        static bool said = false;
        if (!said) {
            said = true;
            printf("  plan: %lld strips + rem %d (%d x %d lanes) x %lld groups of %lld rows, %lld remainder WGs, grid %lld\n",
                   (long long)a.nstrips, a.rem, a.rp, a.rq, (long long)a.ngroups, (long long)a.grows, (long long)a.nrem,
                   (long long)grid);
        }
        hipLaunchKernelGGL((pipe_step<M_, D, S, P, NT, MINW, X16>), dim3((unsigned)grid), dim3(C::kThreads), 0, st, s, d, a);
        return true;
    }
};

}  // namespace proto

int main(int argc, char** argv) {
    const int64_t W = 65536, H = 65536, words = W / 32, n = words * H;
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    proto::g_split1 = proto::g_split2 = (int)(0.65 * 65536);
    proto::g_rot = 1;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *a, *b;
    unsigned* err;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    CHECK(hipMalloc(&err, 4));
    CHECK(hipMemset(err, 0, 4));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    proto::PipeRunner<4, 4, 8, 2, 2, 4, true> pr;
    gol::PipeArgs la{};
    la.words = words;
    la.pitch = words;
    la.rows = H;
    la.out_end = H;
    la.err = (int*)err;
    std::function<void()> lib_pass = [&]() { CHECK(gol::launch_pipe_step(a, b, la, 32, true, st)); std::swap(a, b); };
    std::function<void()> proto_pass = [&]() { pr.run(a, b, H, words, err, cus, st); std::swap(a, b); };
    proto::seed_k<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, n, 0x5EEDull);
    for (int i = 0; i < 1200; i++) (i & 1 ? lib_pass : proto_pass)();  // ~1 s of clock warm-up
    for (int round = 0; round < rounds; round++) {
        for (int which = 0; which < 2; which++) {
            auto& pass = which ? lib_pass : proto_pass;
            proto::seed_k<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(a, n, 0x5EEDull);
            for (int i = 0; i < 10; i++) pass();
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < 8; i++) pass();
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("round %d %s: %.1f us/pass\n", round, which ? "library" : "proto  ", ms * 1000.0 / 8);
            fflush(stdout);
        }
    }
    unsigned e = 0;
    CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("err %u\n", e);
    return 0;
}
