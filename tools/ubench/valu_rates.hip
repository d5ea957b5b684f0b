// Microbenchmark: issue throughput of the VALU instructions the step kernel uses, on gfx950.
// Each lane runs ITERS x (8 independent chains x 1 instruction); grid fills every SIMD with WAVES waves.
// Prints cycles per wave-instruction per SIMD (2.0 = full rate for wave64 on a SIMD32).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define BODY8(INS) INS(a0) INS(a1) INS(a2) INS(a3) INS(a4) INS(a5) INS(a6) INS(a7)

#define DEF_KERNEL64(NAME, ASMSTR)                                                            \
__global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                  \
    uint64_t a0x = seed ^ threadIdx.x, a1x = a0x * 3, a2x = a0x * 5, a3x = a0x * 7, a4x = a0x * 11, \
             a5x = a0x * 13, a6x = a0x * 17, a7x = a0x * 19;                                  \
    uint64_t bb = seed * 0x9E3779B9ull + threadIdx.x;                                         \
    for (int i = 0; i < ITERS; i++) {                                                         \
        BODY8(ASMSTR)                                                                          \
    }                                                                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0x ^ a1x ^ a2x ^ a3x ^ a4x ^ a5x ^ a6x ^ a7x); \
}
#define DEF_KERNEL(NAME, ASMSTR)                                                              \
__global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                  \
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,    \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                        \
    uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5555u;                           \
    int addr = ((threadIdx.x + 1) & 63) << 2; (void)addr;                                     \
    for (int i = 0; i < ITERS; i++) {                                                         \
        BODY8(ASMSTR)                                                                          \
    }                                                                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
}

#define I_XOR(r) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r) : "v"(b));
#define I_XOR3(r) asm volatile("v_xor3_b32 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_BITOP3(r) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(r) : "v"(b), "v"(c));
#define I_ALIGN(r) asm volatile("v_alignbit_b32 %0, %1, %0, 31" : "+v"(r) : "v"(b));
#define I_BFI(r) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_DPP(r) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(r));
#define I_DPPROR(r) asm volatile("v_mov_b32_dpp %0, %0 wave_ror:1 row_mask:0xf bank_mask:0xf" : "+v"(r));
#define I_DPPROL(r) asm volatile("v_mov_b32_dpp %0, %0 wave_rol:1 row_mask:0xf bank_mask:0xf" : "+v"(r));
#define I_DPPSHL(r) asm volatile("v_mov_b32_dpp %0, %0 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(r));
#define I_DPPROW(r) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(r));
#define I_XORDPP(r) asm volatile("v_xor_b32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(r) : "v"(b));
#define I_LSHL(r) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(r));
#define I_ANDOR(r) asm volatile("v_and_or_b32 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(c));
#define I_PKXOR(r) asm volatile("v_lshl_or_b32 %0, %1, 1, %0" : "+v"(r) : "v"(b));

#define I_LSHL64(r) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(r##x));
#define I_LSHR64(r) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(r##x));
#define I_LSHLADD64(r) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(r##x) : "v"(bb));
#define I_ADD(r) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r) : "v"(b));
#define I_ADDC(r) asm volatile("v_addc_co_u32 %0, vcc, %1, %0, vcc" : "+v"(r) : "v"(b) : "vcc");
#define I_OR(r) asm volatile("v_or_b32 %0, %1, %0" : "+v"(r) : "v"(b));
#define I_PERM(r) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(r) : "v"(b), "v"(c));
#define I_ALIGNBYTE(r) asm volatile("v_alignbyte_b32 %0, %1, %0, 1" : "+v"(r) : "v"(b));
#define I_CNDMASK(r) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(r) : "v"(b) : "vcc");
#define I_MOV(r) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(r));
#define I_PKADD16(r) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(r) : "v"(b));
#define I_PKLSHL16(r) asm volatile("v_pk_lshlrev_b16 %0, 1, %0" : "+v"(r));
#define I_BFE(r) asm volatile("v_bfe_u32 %0, %0, 1, 31" : "+v"(r));
#define I_MAD24(r) asm volatile("v_mad_u32_u24 %0, %1, 2, %0" : "+v"(r) : "v"(b));
#define I_PL32(r) asm volatile("v_permlane32_swap %0, %1" : "+v"(r), "+v"(c));
#define I_PL16(r) asm volatile("v_permlane16_swap %0, %1" : "+v"(r), "+v"(c));
#define I_BPERM(r) asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(r) : "v"(addr));
#define I_BPERM_NW(r) asm volatile("ds_bpermute_b32 %0, %1, %0" : "+v"(r) : "v"(addr));
#define I_SWIZ(r) asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(SWAP,1)\n s_waitcnt lgkmcnt(0)" : "+v"(r));
DEF_KERNEL(k_xor, I_XOR)
DEF_KERNEL(k_bitop3, I_BITOP3)
DEF_KERNEL(k_align, I_ALIGN)
DEF_KERNEL(k_bfi, I_BFI)
DEF_KERNEL(k_dpp, I_DPP)
DEF_KERNEL(k_dpprow, I_DPPROW)
DEF_KERNEL(k_dppror, I_DPPROR)
DEF_KERNEL(k_dpprol, I_DPPROL)
DEF_KERNEL(k_dppshl, I_DPPSHL)
DEF_KERNEL(k_xordpp, I_XORDPP)
DEF_KERNEL(k_lshl, I_LSHL)
DEF_KERNEL(k_andor, I_ANDOR)
DEF_KERNEL(k_lshlor, I_PKXOR)
DEF_KERNEL64(k_lshl64, I_LSHL64)
DEF_KERNEL64(k_lshr64, I_LSHR64)
DEF_KERNEL64(k_lshladd64, I_LSHLADD64)
DEF_KERNEL(k_add, I_ADD)
DEF_KERNEL(k_addc, I_ADDC)
DEF_KERNEL(k_or, I_OR)
DEF_KERNEL(k_perm, I_PERM)
DEF_KERNEL(k_alignbyte, I_ALIGNBYTE)
DEF_KERNEL(k_cndmask, I_CNDMASK)
DEF_KERNEL(k_pkadd16, I_PKADD16)
DEF_KERNEL(k_pklshl16, I_PKLSHL16)
DEF_KERNEL(k_bfe, I_BFE)
DEF_KERNEL(k_mad24, I_MAD24)
DEF_KERNEL(k_bperm, I_BPERM)
DEF_KERNEL(k_bperm_nw, I_BPERM_NW)
DEF_KERNEL(k_swiz, I_SWIZ)

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    struct { const char* name; kfn f; } ks[] = {
        {"v_xor_b32", k_xor}, {"v_bitop3_b32", k_bitop3}, {"v_alignbit_b32", k_align},
        {"v_bfi_b32", k_bfi}, {"v_mov_b32_dpp wave_shr", k_dpp}, {"v_mov_b32_dpp row_shr", k_dpprow},
        {"v_mov_b32_dpp wave_ror", k_dppror}, {"v_mov_b32_dpp wave_rol", k_dpprol}, {"v_mov_b32_dpp wave_shl", k_dppshl},
        {"v_xor_b32_dpp row_shr", k_xordpp}, {"v_lshlrev_b32", k_lshl}, {"v_and_or_b32", k_andor},
        {"v_lshl_or_b32", k_lshlor}, {"v_lshlrev_b64", k_lshl64}, {"v_lshrrev_b64", k_lshr64},
        {"v_lshl_add_u64", k_lshladd64}, {"v_add_u32", k_add}, {"v_addc_co_u32", k_addc}, {"v_or_b32", k_or},
        {"v_perm_b32", k_perm}, {"v_alignbyte_b32", k_alignbyte}, {"v_cndmask_b32", k_cndmask},
        {"v_pk_add_u16", k_pkadd16}, {"v_pk_lshlrev_b16", k_pklshl16}, {"v_bfe_u32", k_bfe},
        {"v_mad_u32_u24", k_mad24},
        {"ds_bpermute+wait (latency)", k_bperm}, {"ds_bpermute (throughput)", k_bperm_nw},
        {"ds_swizzle+wait", k_swiz}};
    uint32_t* out;
    for (int wps : {1, 4, 8}) {  // waves per SIMD
        const int blocks = cus * wps;  // 256-thread blocks = 4 waves = one per SIMD
        hipMalloc(&out, (size_t)blocks * 256 * 4);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per SIMD = wps waves x ITERS x 8
            double instr = (double)wps * ITERS * 8 * 5;
            double ns_per = ms * 1e6 / instr;
            printf("{\"waves_per_simd\": %d, \"instr\": \"%s\", \"ns_per_wave_instr_per_simd\": %.4f, \"cycles_at_2.4GHz\": %.3f}\n",
                   wps, k.name, ns_per, ns_per * 2.4);
        }
        hipFree(out);
    }
    return 0;
}
