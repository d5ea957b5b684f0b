// Calibration of rocprofv3's HBM byte counters (FETCH_SIZE / WRITE_SIZE) on gfx950 for the access widths
// the step kernel uses (4, 8, 16 bytes per lane, buffer loads/stores).  MI355X_MICROARCH.md "HBM": on
// gfx950 FETCH_SIZE reads 1/2 of a 16-B/lane coalesced stream; other widths are uncalibrated.  Each
// kernel copies exactly BYTES (1 GiB) from src to dst, once per launch, 3 launches per width:
//     true read bytes = true write bytes = 1 GiB per launch.
// tools/pmc_traffic.py divides these by the counters to get per-width correction factors.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

static constexpr size_t BYTES = size_t(1) << 30;

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int W>
struct V;
template <>
struct V<4> {
    using T = uint32_t;
};
template <>
struct V<8> {
    using T = u32x2;
};
template <>
struct V<16> {
    using T = u32x4;
};

template <int W>
__global__ __launch_bounds__(256) void copy_w(const typename V<W>::T* __restrict__ src, typename V<W>::T* __restrict__ dst,
                                              size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    void *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, BYTES) != hipSuccess || hipMalloc(&dst, BYTES) != hipSuccess) return 1;
    (void)hipMemset(src, 0x5a, BYTES);
    (void)hipMemset(dst, 0, BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 256 * 16;
    for (int rep = 0; rep < 3; rep++) {
        float ms[3];
        (void)hipEventRecord(e0);
        copy_w<4><<<blocks, 256>>>((const uint32_t*)src, (uint32_t*)dst, BYTES / 4);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[0], e0, e1);
        (void)hipEventRecord(e0);
        copy_w<8><<<blocks, 256>>>((const u32x2*)src, (u32x2*)dst, BYTES / 8);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[1], e0, e1);
        (void)hipEventRecord(e0);
        copy_w<16><<<blocks, 256>>>((const u32x4*)src, (u32x4*)dst, BYTES / 16);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[2], e0, e1);
        printf("{\"rep\": %d, \"copy_GBps_w4\": %.1f, \"copy_GBps_w8\": %.1f, \"copy_GBps_w16\": %.1f}\n", rep,
               2.0 * BYTES / ms[0] / 1e6, 2.0 * BYTES / ms[1] / 1e6, 2.0 * BYTES / ms[2] / 1e6);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
