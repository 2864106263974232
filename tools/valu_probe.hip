// valu_probe.hip -- measured int32 VALU throughput on gfx950 for the ops the
// SHA-256 and GF(2^8) kernels are made of (roofline peak calibration).
// Each op is emitted with inline asm on 8 independent register chains so the
// compiler cannot fold it; the in-kernel clock is read with s_memtime /
// s_memrealtime (100 MHz) to separate issue rate from DVFS.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_probe valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP8(INSN)                                                                                  \
    asm volatile(INSN " %0, %0, %8, %9\n\t" INSN " %1, %1, %8, %9\n\t" INSN " %2, %2, %8, %9\n\t" \
                 INSN " %3, %3, %8, %9\n\t" INSN " %4, %4, %8, %9\n\t" INSN " %5, %5, %8, %9\n\t" \
                 INSN " %6, %6, %8, %9\n\t" INSN " %7, %7, %8, %9"                                \
                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                 : "v"(y), "v"(z))
#define OP8_2(INSN)                                                                            \
    asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t" INSN " %3, %3, %8\n\t" \
                 INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t" INSN " %6, %6, %8\n\t" INSN " %7, %7, %8" \
                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                 : "v"(y))

#define OP8_64(INSN)                                                                              \
    asm volatile(INSN " %0, %8, %0\n\t" INSN " %1, %8, %1\n\t" INSN " %2, %8, %2\n\t" INSN " %3, %8, %3\n\t" \
                 INSN " %4, %8, %4\n\t" INSN " %5, %8, %5\n\t" INSN " %6, %8, %6\n\t" INSN " %7, %8, %7" \
                 : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7)         \
                 : "v"(y))
// alternating half-rate / full-rate op (does a half-rate op block the SIMD for 2 issue slots?)
#define MIX8(INSN_A, INSN_B)                                                                        \
    asm volatile(INSN_A " %0, %0, %8, %9\n\t" INSN_B " %1, %1, %8\n\t" INSN_A " %2, %2, %8, %9\n\t" \
                 INSN_B " %3, %3, %8\n\t" INSN_A " %4, %4, %8, %9\n\t" INSN_B " %5, %5, %8\n\t"         \
                 INSN_A " %6, %6, %8, %9\n\t" INSN_B " %7, %7, %8"                                      \
                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                 : "v"(y), "v"(z))

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t y = seed * 0x9E3779B9u + threadIdx.x, z = y ^ 0x5bd1e995u;
    uint32_t v0 = y, v1 = y + 1, v2 = y + 2, v3 = y + 3, v4 = y + 4, v5 = y + 5, v6 = y + 6, v7 = y + 7;
    uint64_t q0 = v0 | (uint64_t)z << 32, q1 = v1 | (uint64_t)z << 32, q2 = v2 | (uint64_t)z << 32,
             q3 = v3 | (uint64_t)z << 32, q4 = v4 | (uint64_t)z << 32, q5 = v5 | (uint64_t)z << 32,
             q6 = v6 | (uint64_t)z << 32, q7 = v7 | (uint64_t)z << 32;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
            if constexpr (OP == 0) OP8("v_alignbit_b32");
            if constexpr (OP == 1) OP8("v_bitop3_b32");
            if constexpr (OP == 2) OP8("v_add3_u32");
            if constexpr (OP == 3) OP8("v_perm_b32");
            if constexpr (OP == 4) OP8_2("v_xor_b32");
            if constexpr (OP == 5) OP8_2("v_add_u32");
            if constexpr (OP == 6) OP8("v_xad_u32");
            if constexpr (OP == 7) OP8("v_lshl_or_b32");
            if constexpr (OP == 8) OP8("v_or3_b32");
            if constexpr (OP == 9) OP8("v_lshl_add_u32");
            if constexpr (OP == 10) OP8("v_alignbyte_b32");
            if constexpr (OP == 11) OP8_2("v_lshrrev_b32");
            if constexpr (OP == 12) OP8_64("v_lshrrev_b64");
            if constexpr (OP == 13) OP8("v_bfi_b32");
            if constexpr (OP == 14) OP8("v_and_or_b32");
            if constexpr (OP == 15) MIX8("v_alignbit_b32", "v_xor_b32");
            if constexpr (OP == 16) OP8("v_add_lshl_u32");
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7 ^ (uint32_t)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);
    if (s == 0x12345678u) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
void run(const char* name, uint32_t* d, uint64_t* dclk, int cus) {
    const int iters = 2048;
    dim3 grid(cus * 8), block(256);   // 8 blocks of 256 per CU = 8 waves per SIMD
    hipLaunchKernelGGL(probe<OP>, grid, block, 0, 0, d, dclk, 1u, 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(probe<OP>, grid, block, 0, 0, d, dclk, 1u, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t clk[2];
    (void)hipMemcpy(clk, dclk, 16, hipMemcpyDeviceToHost);
    double ghz = (double)clk[0] / (clk[1] * 10.0);   // memrealtime = 100 MHz
    double ops = (double)grid.x * block.x * iters * 8 * 8;
    printf("%-14s %7.2f T lane-ops/s  %6.1f lane-ops/clk/CU @2.4GHz  in-kernel clock %.2f GHz -> %6.1f /clk/CU\n",
           name, ops / ms / 1e9, ops / (ms * 1e-3) / (cus * 2.4e9), ghz, ops / (ms * 1e-3) / (cus * ghz * 1e9));
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    int cus = p.multiProcessorCount;
    run<0>("v_alignbit_b32", d, c, cus);
    run<1>("v_bitop3_b32", d, c, cus);
    run<2>("v_add3_u32", d, c, cus);
    run<3>("v_perm_b32", d, c, cus);
    run<4>("v_xor_b32", d, c, cus);
    run<5>("v_add_u32", d, c, cus);
    run<6>("v_xad_u32", d, c, cus);
    run<7>("v_lshl_or_b32", d, c, cus);
    run<8>("v_or3_b32", d, c, cus);
    run<9>("v_lshl_add_u32", d, c, cus);
    run<10>("v_alignbyte_b32", d, c, cus);
    run<11>("v_lshrrev_b32", d, c, cus);
    run<12>("v_lshrrev_b64", d, c, cus);
    run<13>("v_bfi_b32", d, c, cus);
    run<14>("v_and_or_b32", d, c, cus);
    run<15>("alignbit+xor", d, c, cus);
    run<16>("v_add_lshl_u32", d, c, cus);
    return 0;
}
