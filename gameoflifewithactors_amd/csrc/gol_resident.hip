// gol_resident.hip -- LDS-resident multi-generation pass for small boards (gfx950).
//
// The streaming pass (gol_step.hip) is built for boards that fill the chip; on the reference-size
// boards (BASELINE configs 1 and 5: the F# default board, glider gun / R-pentomino runs; small bounded
// boards) each pass is a handful of waves and the run is bound by launch + pipeline latency, one launch
// per K generations (one per generation on byte boards).  Here ONE workgroup loads the whole board into
// LDS once, runs all requested generations between two LDS buffers with a workgroup barrier per
// generation, and writes the result back: one launch per gol_step call, HBM touched twice.
//
// Rule and neighbourhood are the same as the streaming kernel and the byte kernel
// (GameOfLifeLogic.fs:56-63; torus GameOfLifeDriver.fs:21-25; bounded Script.fsx:6-13), so the result is
// bit-identical to them (tests/test_gpu_resident.py checks against the oracle and the streaming path).
//
// Capacity: 128 KiB of the CU's 160 KiB LDS hold the two buffers.
//   packed (ilv 1):  2 * H * W/32 words * 4 B  <= 128 KiB  ->  W*H <= 2^19 cells
//   bytes:           2 * W * H bytes           <= 128 KiB  ->  W*H <= 2^16 cells
#include "gol_internal.h"
#include "gol_bitlogic.h"

#include <cstdlib>

namespace gol {
namespace {

constexpr int kLdsBytes = 128 * 1024;

// Work split shared by both kernels: `cols` columns (words or cells) x `nseg` row segments, one
// (column, segment) item per thread while there are more threads than columns.  A thread slides down its
// segment keeping the horizontal 3-sums of the previous, current and next rows in registers, so each
// row is read from LDS once per item (3 reads per word or cell) and there is no divide per cell.
__device__ __forceinline__ void item_rows(int item, int cols, int nseg, int H, int& c, int& y0, int& y1) {
    const int s = item / cols;
    c = item - s * cols;
    y0 = s * H / nseg;  // s * H < 2^29 (nseg <= 1024, cells <= 2^19)
    y1 = (s + 1) * H / nseg;
}

// Packed board, ilv = 1 (bit b of word w = cell 32w + b).
template <bool BOUNDED>
__device__ __forceinline__ uint32_t packed_row(const uint32_t* a, int wpr, int H, int c, int y, uint32_t& s,
                                               uint32_t& cy) {
    if (y < 0 || y >= H) {
        if (BOUNDED) {
            s = cy = 0u;
            return 0u;
        }
        y = y < 0 ? y + H : y - H;
    }
    const uint32_t* row = a + y * wpr;
    const uint32_t m = row[c];
    const uint32_t l = (BOUNDED && c == 0) ? 0u : row[c == 0 ? wpr - 1 : c - 1];
    const uint32_t r = (BOUNDED && c == wpr - 1) ? 0u : row[c == wpr - 1 ? 0 : c + 1];
    row_sum(l, m, r, s, cy);
    return m;
}

template <bool BOUNDED, int NT>
__global__ __launch_bounds__(NT) void gol_resident_packed(const uint32_t* __restrict__ src,
                                                                  uint32_t* __restrict__ dst, int wpr, int H,
                                                                  int64_t pitch, int gens, int nseg) {
    __shared__ uint32_t lds[kLdsBytes / 4];
    const int n = wpr * H, items = wpr * nseg;
    uint32_t* a = lds;
    uint32_t* b = lds + n;
    for (int i = threadIdx.x; i < n; i += NT) a[i] = src[(int64_t)(i / wpr) * pitch + i % wpr];
    __syncthreads();
    int c0 = 0, y00 = 0, y10 = 0;  // this thread's first item, fixed over the generations
    if ((int)threadIdx.x < items) item_rows(threadIdx.x, wpr, nseg, H, c0, y00, y10);
    for (int g = 0; g < gens; g++) {
        for (int it = threadIdx.x; it < items; it += NT) {
            int c = c0, y0 = y00, y1 = y10;
            if (it != (int)threadIdx.x) item_rows(it, wpr, nseg, H, c, y0, y1);
            uint32_t sP, cP, sC, cC, sN, cN;
            packed_row<BOUNDED>(a, wpr, H, c, y0 - 1, sP, cP);
            uint32_t mC = packed_row<BOUNDED>(a, wpr, H, c, y0, sC, cC);
#pragma unroll 4
            for (int y = y0; y < y1; y++) {
                const uint32_t mN = packed_row<BOUNDED>(a, wpr, H, c, y + 1, sN, cN);
                b[y * wpr + c] = life_next(sP, cP, sC, cC, sN, cN, mC);
                sP = sC, cP = cC, sC = sN, cC = cN, mC = mN;
            }
        }
        __syncthreads();
        uint32_t* t = a;
        a = b;
        b = t;
    }
    for (int i = threadIdx.x; i < n; i += NT) dst[(int64_t)(i / wpr) * pitch + i % wpr] = a[i];
}

// Byte board (nonzero = alive on input, 0/1 on output like gol_bytes_step).
template <bool BOUNDED>
__device__ __forceinline__ int bytes_row(const uint8_t* a, int W, int H, int x, int y, int& m) {
    if (y < 0 || y >= H) {
        if (BOUNDED) {
            m = 0;
            return 0;
        }
        y = y < 0 ? y + H : y - H;
    }
    const uint8_t* row = a + y * W;
    m = row[x];
    const int l = (BOUNDED && x == 0) ? 0 : row[x == 0 ? W - 1 : x - 1];
    const int r = (BOUNDED && x == W - 1) ? 0 : row[x == W - 1 ? 0 : x + 1];
    return l + m + r;
}

template <bool BOUNDED, int NT>
__global__ __launch_bounds__(NT) void gol_resident_bytes(const uint8_t* __restrict__ src,
                                                                 uint8_t* __restrict__ dst, int W, int H, int gens,
                                                                 int nseg) {
    __shared__ uint8_t lds[kLdsBytes];
    const int n = W * H, items = W * nseg;
    uint8_t* a = lds;
    uint8_t* b = lds + n;
    for (int i = threadIdx.x; i < n; i += NT) a[i] = src[i] != 0;
    __syncthreads();
    int x0 = 0, y00 = 0, y10 = 0;  // this thread's first item, fixed over the generations
    if ((int)threadIdx.x < items) item_rows(threadIdx.x, W, nseg, H, x0, y00, y10);
    for (int g = 0; g < gens; g++) {
        for (int it = threadIdx.x; it < items; it += NT) {
            int x = x0, y0 = y00, y1 = y10, mP, mC, mN;
            if (it != (int)threadIdx.x) item_rows(it, W, nseg, H, x, y0, y1);
            int hP = bytes_row<BOUNDED>(a, W, H, x, y0 - 1, mP);
            int hC = bytes_row<BOUNDED>(a, W, H, x, y0, mC);
#pragma unroll 4
            for (int y = y0; y < y1; y++) {
                const int hN = bytes_row<BOUNDED>(a, W, H, x, y + 1, mN);
                const int cnt = hP + hC + hN - mC;  // 8 neighbours
                b[y * W + x] = (cnt == 3) | ((cnt == 2) & mC);
                hP = hC, hC = hN, mC = mN;
            }
        }
        __syncthreads();
        uint8_t* t = a;
        a = b;
        b = t;
    }
    for (int i = threadIdx.x; i < n; i += NT) dst[i] = a[i];
}

// Row segments per column: enough items to give every thread one (at least one row each).
int segments(int64_t cols, int64_t H, int nt) {
    const int64_t s = cols >= nt ? 1 : nt / cols;
    return (int)(s < H ? s : H);
}

// Workgroup size: 1024 threads unless the board's "resident_threads" option is 256 (A/B of the barrier cost on
// tiny boards: 256 was slower everywhere, profiles/r1/resident_threads_ab.log).
template <bool BOUNDED>
void launch_packed(const uint32_t* src, uint32_t* dst, int wpr, int H, int64_t pitch, int gens, hipStream_t s,
                   int threads) {
    if (threads == 256)
        hipLaunchKernelGGL((gol_resident_packed<BOUNDED, 256>), dim3(1), dim3(256), 0, s, src, dst, wpr, H, pitch,
                           gens, segments(wpr, H, 256));
    else
        hipLaunchKernelGGL((gol_resident_packed<BOUNDED, 1024>), dim3(1), dim3(1024), 0, s, src, dst, wpr, H, pitch,
                           gens, segments(wpr, H, 1024));
}

template <bool BOUNDED>
void launch_bytes(const uint8_t* src, uint8_t* dst, int W, int H, int gens, hipStream_t s, int threads) {
    if (threads == 256)
        hipLaunchKernelGGL((gol_resident_bytes<BOUNDED, 256>), dim3(1), dim3(256), 0, s, src, dst, W, H, gens,
                           segments(W, H, 256));
    else
        hipLaunchKernelGGL((gol_resident_bytes<BOUNDED, 1024>), dim3(1), dim3(1024), 0, s, src, dst, W, H, gens,
                           segments(W, H, 1024));
}

}  // namespace

bool resident_packed_fits(int64_t W, int64_t H) {
    return W >= 32 && W % 32 == 0 && H >= 1 && 2 * (W / 32) * H * 4 <= kLdsBytes;
}

bool resident_bytes_fits(int64_t W, int64_t H) { return W >= 1 && H >= 1 && 2 * W * H <= kLdsBytes; }

hipError_t launch_resident_packed(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch,
                                  int64_t gens, bool bounded, hipStream_t s, int threads) {
    if (!resident_packed_fits(W, H) || pitch < W / 32 || gens < 1 || gens > INT32_MAX) return hipErrorInvalidValue;
    if (bounded)
        launch_packed<true>(src, dst, (int)(W / 32), (int)H, pitch, (int)gens, s, threads);
    else
        launch_packed<false>(src, dst, (int)(W / 32), (int)H, pitch, (int)gens, s, threads);
    return hipGetLastError();
}

hipError_t launch_resident_bytes(const uint8_t* src, uint8_t* dst, int64_t W, int64_t H, int64_t gens, bool bounded,
                                 hipStream_t s, int threads) {
    if (!resident_bytes_fits(W, H) || gens < 1 || gens > INT32_MAX) return hipErrorInvalidValue;
    if (bounded)
        launch_bytes<true>(src, dst, (int)W, (int)H, (int)gens, s, threads);
    else
        launch_bytes<false>(src, dst, (int)W, (int)H, (int)gens, s, threads);
    return hipGetLastError();
}

}  // namespace gol
