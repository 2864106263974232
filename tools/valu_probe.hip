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

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t y = seed * 0x9E3779B9u + threadIdx.x, z = y ^ 0x5bd1e995u;
    uint32_t v0 = y, v1 = y + 1, v2 = y + 2, v3 = y + 3, v4 = y + 4, v5 = y + 5, v6 = y + 6, v7 = y + 7;
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
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
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
    return 0;
}
