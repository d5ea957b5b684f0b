// Microbenchmark: does v_bitop3_b32 slow down when its three source VGPRs share a register bank
// (VGPR index mod 4)?  8 independent chains, operands pinned to physical VGPRs; waves per SIMD 3 and 8.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 2048

// chains in v32, v36, ... (bank 0); B and C name the two loop-invariant sources' registers
#define CHAIN_KERNEL(NAME, B, C)                                                                          \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                          \
        register uint32_t a0 asm("v32") = seed ^ threadIdx.x;                                           \
        register uint32_t a1 asm("v36") = a0 * 3;                                                       \
        register uint32_t a2 asm("v40") = a0 * 5;                                                       \
        register uint32_t a3 asm("v44") = a0 * 7;                                                       \
        register uint32_t a4 asm("v48") = a0 * 11;                                                      \
        register uint32_t a5 asm("v52") = a0 * 13;                                                      \
        register uint32_t a6 asm("v56") = a0 * 17;                                                      \
        register uint32_t a7 asm("v60") = a0 * 19;                                                      \
        register uint32_t b asm(B) = seed * 0x9E3779B9u + threadIdx.x;                                  \
        register uint32_t c asm(C) = b ^ 0x5555u;                                                       \
        for (int i = 0; i < ITERS; i++) {                                                               \
            asm volatile(                                                                               \
                "v_bitop3_b32 %0, %8, %9, %0 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %1, %8, %9, %1 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %2, %8, %9, %2 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %3, %8, %9, %3 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %4, %8, %9, %4 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %5, %8, %9, %5 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %6, %8, %9, %6 bitop3:0x96\n"                                             \
                "v_bitop3_b32 %7, %8, %9, %7 bitop3:0x96\n"                                             \
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
                : "v"(b), "v"(c));                                                                      \
        }                                                                                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
    }

CHAIN_KERNEL(k_same, "v0", "v4")   // all three sources in bank 0
CHAIN_KERNEL(k_two, "v0", "v5")    // chain + B in bank 0, C in bank 1
CHAIN_KERNEL(k_diff, "v1", "v6")   // banks 0, 1, 2

// sources are the results of the two previous instructions (the shape of the real kernel's trees)
__global__ __launch_bounds__(256) void k_fresh(uint32_t* out, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (2 * i + 1) ^ threadIdx.x;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++)
            asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96"
                         : "+v"(a[i])
                         : "v"(a[(i + 7) & 7]), "v"(a[(i + 6) & 7]));
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        const char* name;
        kfn f;
    } ks[] = {{"same_bank", k_same}, {"two_banks", k_two}, {"three_banks", k_diff}, {"fresh_operands", k_fresh}};
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    for (int wps : {1, 3, 8}) {
        const int blocks = cus * wps;
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
            (void)hipDeviceSynchronize();
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r + 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr = (double)wps * ITERS * 8 * 5;
            printf("{\"waves_per_simd\": %d, \"variant\": \"%s\", \"cycles_at_2.4GHz\": %.3f}\n", wps, k.name,
                   ms * 1e6 / instr * 2.4);
        }
    }
    (void)hipFree(out);
    return 0;
}
