// operand_probe.hip -- does the issue rate of gfx950's "half-rate" VALU ops
// (v_alignbit, v_add3, v_perm) depend on the operand form (repeated register,
// inline constant, SGPR) rather than on the opcode?  8 independent chains per
// wave, 8 waves per SIMD; lane-ops per clock per CU at the in-kernel clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o operand_probe operand_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH8(FMT)                                                                                        \
    asm volatile(FMT(0) FMT(1) FMT(2) FMT(3) FMT(4) FMT(5) FMT(6) FMT(7)                                \
                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                 : "v"(y), "v"(z), "s"(sc))
// %8 = y (VGPR), %9 = z (VGPR), %10 = sc (SGPR)
#define F_ROT_SAME_IMM(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t"
#define F_ROT_DIFF_IMM(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 7\n\t"
#define F_ROT_3V(i) "v_alignbit_b32 %" #i ", %" #i ", %8, %9\n\t"
#define F_ROT_SAME_V(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", %9\n\t"
#define F_ADD3_3V(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"
#define F_ADD3_IMM(i) "v_add3_u32 %" #i ", %" #i ", %8, 5\n\t"
#define F_ADD3_S(i) "v_add3_u32 %" #i ", %" #i ", %8, %10\n\t"
#define F_BOP3_3V(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t"
#define F_BOP3_SAME(i) "v_bitop3_b32 %" #i ", %" #i ", %" #i ", %8 bitop3:0x96\n\t"
#define F_PERM_3V(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"
#define F_PERM_S(i) "v_perm_b32 %" #i ", %10, %" #i ", %9\n\t"
#define F_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n\t"
#define F_LSHR(i) "v_lshrrev_b32 %" #i ", 7, %" #i "\n\t"
#define F_LSHL_OR(i) "v_lshl_or_b32 %" #i ", %" #i ", 7, %8\n\t"

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t y = seed * 0x9E3779B9u + threadIdx.x, z = (y ^ 0x5bd1e995u) & 31u;
    const uint32_t sc = __builtin_amdgcn_readfirstlane(seed * 3u + 0x01020304u);
    uint32_t v0 = y, v1 = y + 1, v2 = y + 2, v3 = y + 3, v4 = y + 4, v5 = y + 5, v6 = y + 6, v7 = y + 7;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
            if constexpr (OP == 0) CH8(F_ROT_SAME_IMM);
            if constexpr (OP == 1) CH8(F_ROT_DIFF_IMM);
            if constexpr (OP == 2) CH8(F_ROT_3V);
            if constexpr (OP == 3) CH8(F_ROT_SAME_V);
            if constexpr (OP == 4) CH8(F_ADD3_3V);
            if constexpr (OP == 5) CH8(F_ADD3_IMM);
            if constexpr (OP == 6) CH8(F_ADD3_S);
            if constexpr (OP == 7) CH8(F_BOP3_3V);
            if constexpr (OP == 8) CH8(F_BOP3_SAME);
            if constexpr (OP == 9) CH8(F_PERM_3V);
            if constexpr (OP == 10) CH8(F_PERM_S);
            if constexpr (OP == 11) CH8(F_XOR);
            if constexpr (OP == 12) CH8(F_LSHR);
            if constexpr (OP == 13) CH8(F_LSHL_OR);
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
    printf("%-34s %6.1f lane-ops/clk/CU at %.2f GHz (cycles per wave64 instr per SIMD: %.2f)\n", name,
           ops / (ms * 1e-3) / (cus * ghz * 1e9), ghz, 4 * 64 / (ops / (ms * 1e-3) / (cus * ghz * 1e9)));
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    int cus = p.multiProcessorCount;
    run<0>("alignbit v,v(same),v(same),imm", d, c, cus);
    run<1>("alignbit v,v,y,imm", d, c, cus);
    run<2>("alignbit v,v,y,z", d, c, cus);
    run<3>("alignbit v,v(same),v(same),z", d, c, cus);
    run<4>("add3 v,v,y,z", d, c, cus);
    run<5>("add3 v,v,y,imm", d, c, cus);
    run<6>("add3 v,v,y,sgpr", d, c, cus);
    run<7>("bitop3 v,v,y,z", d, c, cus);
    run<8>("bitop3 v,v(same),v(same),y", d, c, cus);
    run<9>("perm v,v,y,z", d, c, cus);
    run<10>("perm v,sgpr,v,z", d, c, cus);
    run<11>("xor v,v,y", d, c, cus);
    run<12>("lshrrev v,imm,v", d, c, cus);
    run<13>("lshl_or v,v,imm,y", d, c, cus);
    return 0;
}
