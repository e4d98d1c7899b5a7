// Issue-rate microbenchmark for the instructions K1's inner loop uses (gfx950).
// Each thread runs 8 independent chains of one instruction; the grid fills every SIMD with
// 8 waves.  Prints SIMD cycles per wave-instruction, relative to the measured clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 512
#define CH(op) op(a0) op(a1) op(a2) op(a3) op(a4) op(a5) op(a6) op(a7)

#define K_BODY(NAME, OP)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {               \
        uint32_t a0 = seed ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                      \
        const uint32_t c = seed | 1u;                                                        \
        for (int i = 0; i < ITERS; ++i) { CH(OP) }                                           \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;         \
    }

#define OP_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MAD64(x) { uint64_t t; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(x), "v"(c) : "vcc"); x = (uint32_t)(t >> 32); }
#define OP_PERM(x) asm volatile("v_perm_b32 %0, %1, %0, %0" : "+v"(x) : "v"(c));
#define OP_SDWA(x) asm volatile("v_lshlrev_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(x) : "v"(c));
#define OP_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x1e" : "+v"(x) : "v"(c));
#define OP_DPP(x) asm volatile("v_mov_b32_dpp %0, %0 wave_shl:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
#define OP_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(x) : "v"(c));
#define OP_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 4" : "+v"(x));

K_BODY(k_add, OP_ADD)
K_BODY(k_mullo, OP_MULLO)
K_BODY(k_mulhi, OP_MULHI)
K_BODY(k_mul24, OP_MUL24)
K_BODY(k_mad64, OP_MAD64)
K_BODY(k_perm, OP_PERM)
K_BODY(k_sdwa, OP_SDWA)
K_BODY(k_bitop3, OP_BITOP3)
K_BODY(k_dpp, OP_DPP)
K_BODY(k_lshlor, OP_LSHLOR)
K_BODY(k_align, OP_ALIGN)

// random LDS reads of a 128 KiB table: 8 independent reads per iteration
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint32_t seed, int width) {
    extern __shared__ uint32_t tab[];
    for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = (seed + threadIdx.x * 8 + j) * 2654435761u;
    for (int i = 0; i < ITERS / 4; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t idx = width == 8 ? ((a[j] >> 17) << 3) & 0x1FFF8 : ((a[j] >> 17) << 2) & 0x1FFFC;
            uint32_t v = width == 8 ? *(const uint32_t *)((const char *)tab + idx) ^ *(const uint32_t *)((const char *)tab + idx + 4)
                                    : *(const uint32_t *)((const char *)tab + idx);
            a[j] = a[j] * 1664525u + v;
        }
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

__global__ void k_clock(unsigned long long *t) {
    unsigned long long a = wall_clock64(), b = clock64();
    __builtin_amdgcn_s_sleep(127);
    for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(127);
    t[0] = wall_clock64() - a; t[1] = clock64() - b;
}

typedef void (*kfn)(uint32_t *, uint32_t);

int main() {
    int dev = 0, ncu = 0, wclk = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, dev);  // kHz
    unsigned long long *dt; hipMalloc(&dt, 16);
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(1), 0, 0, dt);
    unsigned long long ht[2]; hipMemcpy(ht, dt, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)ht[1] / ((double)ht[0] / (wclk * 1e3)) / 1e9;
    printf("CUs %d, shader clock (single wave, s_sleep) %.3f GHz\n", ncu, ghz);
    const int blocks = ncu * 8;  // 8 x 256 threads per CU = 32 waves/CU = 8 per SIMD
    uint32_t *out; hipMalloc(&out, (size_t)blocks * 1024 * 4);
    struct { const char *n; kfn f; } ks[] = {{"v_add_u32", k_add}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
        {"v_mul_u32_u24", k_mul24}, {"v_mad_u64_u32", k_mad64}, {"v_perm_b32", k_perm}, {"v_lshlrev_sdwa", k_sdwa},
        {"v_bitop3_b32", k_bitop3}, {"v_mov_dpp", k_dpp}, {"v_lshl_or_b32", k_lshlor}, {"v_alignbit_b32", k_align}};
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 12345u);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 12345u + r);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double winstr = 5.0 * blocks * 4 * ITERS * 8;   // wave-instructions
        const double per_simd = winstr / (ncu * 4);
        printf("%-16s %.2f cycles/wave-instr/SIMD (at %.2f GHz)\n", k.n, ms * 1e-3 * ghz * 1e9 / per_simd, ghz);
    }
    hipFuncSetAttribute((const void *)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    for (int w : {4, 8}) {
        hipLaunchKernelGGL(k_lds, dim3(ncu), dim3(1024), 131072, 0, out, 1u, w);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_lds, dim3(ncu), dim3(1024), 131072, 0, out, 7u + r, w);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double winstr = 5.0 * ncu * 16 * (ITERS / 4) * 8;  // LDS wave-instructions (b32 or 2x b32)
        printf("lds random %dB: %.2f CU cycles per wave-instruction\n", w, ms * 1e-3 * ghz * 1e9 / (winstr / ncu));
    }
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
