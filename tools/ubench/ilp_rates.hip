// Microbenchmark: v_bitop3_b32 issue rate vs independent chains per wave (ILP) and waves per SIMD
// (occupancy) on gfx950.  Each iteration issues 16 bitop3; instruction i extends chain i % CHAINS.
// Prints cycles (at 2.4 GHz) per wave-instruction per SIMD: ~2.5 = the SIMD's full rate.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 2048
#define OP(r) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(r) : "v"(b), "v"(c));

template <int CHAINS>
__global__ __launch_bounds__(256) void k_ilp(uint32_t* out, uint32_t seed) {
    uint32_t a[16];
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = seed * (2 * i + 1) ^ threadIdx.x;
    const uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5555u;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) OP(a[i % CHAINS]);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        int chains;
        kfn f;
    } ks[] = {{1, k_ilp<1>}, {2, k_ilp<2>}, {3, k_ilp<3>}, {4, k_ilp<4>}, {8, k_ilp<8>}, {16, k_ilp<16>}};
    uint32_t* out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        const int blocks = cus * wps;  // 256-thread blocks = one wave per SIMD each
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r + 2);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr = (double)wps * ITERS * 16 * 5;  // wave-instructions per SIMD
            const double ns = ms * 1e6 / instr;
            printf("{\"waves_per_simd\": %d, \"chains\": %d, \"cycles_at_2.4GHz\": %.3f}\n", wps, k.chains, ns * 2.4);
        }
    }
    hipFree(out);
    return 0;
}
