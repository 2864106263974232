// lookup_probe.hip -- issue rate on gfx950 of a register lookup by a
// wave-uniform index (VGPR index mode: s_set_gpr_idx_on / _idx / _off; gfx950 has no
// v_movrels), the building block of a
// four-Russians bit-sliced GF(2^16) multiply: per output bit
// plane, 4 table planes picked by the twiddle's uniform nibbles, folded with
// two XOR3.  Each variant runs 8 such planes per body; 4 waves per SIMD.
// Reported: SIMD cycles per VALU instruction (2.2 = full rate, 4.1 = the
// half-rate / mixed-stream rate of DESIGN 3.1).
// Build: hipcc --offload-arch=gfx950 -O3 -o lookup_probe lookup_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define TAB_INIT                                                                                          \
    "v_mov_b32 v100, %[y]\n v_add_u32 v101, 1, %[y]\n v_add_u32 v102, 2, %[y]\n v_add_u32 v103, 3, %[y]\n" \
    "v_add_u32 v104, 4, %[y]\n v_add_u32 v105, 5, %[y]\n v_add_u32 v106, 6, %[y]\n v_add_u32 v107, 7, %[y]\n" \
    "v_add_u32 v108, 8, %[y]\n v_add_u32 v109, 9, %[y]\n v_add_u32 v110, 10, %[y]\n v_add_u32 v111, 11, %[y]\n" \
    "v_add_u32 v112, 12, %[y]\n v_add_u32 v113, 13, %[y]\n v_add_u32 v114, 14, %[y]\n v_add_u32 v115, 15, %[y]\n" \
    "v_mov_b32 v120, 0\n v_mov_b32 v121, 0\n v_mov_b32 v122, 0\n v_mov_b32 v123, 0\n"

// one output plane: 4 uniform-index lookups (VGPR index mode: while on,
// SRC0 of every VALU instruction is v[n + index]) + 2 XOR3 into A, B
#define PLANE_NOP(a, b, c, d, A, B)                                                  \
    "s_set_gpr_idx_on " #a ", gpr_idx(SRC0)\n s_nop 0\n v_mov_b32 v116, v100\n"     \
    "s_set_gpr_idx_idx " #b "\n s_nop 0\n v_mov_b32 v117, v100\n"                    \
    "s_set_gpr_idx_idx " #c "\n s_nop 0\n v_mov_b32 v118, v100\n"                    \
    "s_set_gpr_idx_idx " #d "\n s_nop 0\n v_mov_b32 v119, v100\n"                    \
    "s_set_gpr_idx_off\n"                                                          \
    "v_bitop3_b32 " #A ", " #A ", v116, v117 bitop3:0x96\n"                         \
    "v_bitop3_b32 " #B ", " #B ", v118, v119 bitop3:0x96\n"
// the same without wait states after the index writes (timing only: may
// read a stale index)
#define PLANE_NONOP(a, b, c, d, A, B)                                                \
    "s_set_gpr_idx_on " #a ", gpr_idx(SRC0)\n v_mov_b32 v116, v100\n"               \
    "s_set_gpr_idx_idx " #b "\n v_mov_b32 v117, v100\n"                              \
    "s_set_gpr_idx_idx " #c "\n v_mov_b32 v118, v100\n"                              \
    "s_set_gpr_idx_idx " #d "\n v_mov_b32 v119, v100\n"                              \
    "s_set_gpr_idx_off\n"                                                          \
    "v_bitop3_b32 " #A ", " #A ", v116, v117 bitop3:0x96\n"                         \
    "v_bitop3_b32 " #B ", " #B ", v118, v119 bitop3:0x96\n"
// reference: the same shape with plain v_mov from fixed registers (no M0)
#define PLANE_MOV(a, b, c, d, A, B)                                                  \
    "v_mov_b32 v116, v10" #a "\n v_mov_b32 v117, v10" #b "\n"                      \
    "v_mov_b32 v118, v10" #c "\n v_mov_b32 v119, v10" #d "\n"                      \
    "v_bitop3_b32 " #A ", " #A ", v116, v117 bitop3:0x96\n"                         \
    "v_bitop3_b32 " #B ", " #B ", v118, v119 bitop3:0x96\n"
// reference: XOR3 only (6 per plane, independent accumulators)
#define PLANE_XOR(a, b, c, d, A, B)                                                  \
    "v_bitop3_b32 v116, v116, v10" #a ", v10" #b " bitop3:0x96\n"                  \
    "v_bitop3_b32 v117, v117, v10" #c ", v10" #d " bitop3:0x96\n"                  \
    "v_bitop3_b32 v118, v118, v10" #a ", v10" #c " bitop3:0x96\n"                  \
    "v_bitop3_b32 v119, v119, v10" #b ", v10" #d " bitop3:0x96\n"                  \
    "v_bitop3_b32 " #A ", " #A ", v116, v117 bitop3:0x96\n"                         \
    "v_bitop3_b32 " #B ", " #B ", v118, v119 bitop3:0x96\n"

#define BODY(P)                                                                       \
    P(3, 9, 2, 6, v120, v121) P(1, 7, 4, 8, v122, v123) P(5, 0, 9, 2, v120, v121)     \
    P(8, 4, 6, 1, v122, v123) P(2, 5, 7, 3, v120, v121) P(9, 3, 0, 5, v122, v123)     \
    P(6, 8, 1, 7, v120, v121) P(0, 2, 8, 4, v122, v123)

#define KERNEL(NAME, P)                                                                                 \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) { \
        const uint32_t y = seed * 0x9E3779B9u + threadIdx.x;                                            \
        uint32_t acc;                                                                                   \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();              \
        asm volatile(TAB_INIT "s_mov_b32 s60, %[it]\n"                                                  \
                     "1:\n" BODY(P) BODY(P) BODY(P) BODY(P)                                             \
                     "s_sub_u32 s60, s60, 1\n s_cmp_lg_u32 s60, 0\n s_cbranch_scc1 1b\n"                \
                     "v_xor_b32 %[acc], v120, v121\n v_xor_b32 %[acc], %[acc], v122\n"                  \
                     "v_xor_b32 %[acc], %[acc], v123\n"                                                 \
                     : [acc] "=v"(acc)                                                                  \
                     : [y] "v"(y), [it] "s"(iters)                                                      \
                     : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", \
                       "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", \
                       "v120", "v121", "v122", "v123", "s60", "scc");                             \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();              \
        if (acc == 0x12345678u) out[0] = acc;                                                           \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                                                      \
            clk[0] = t1 - t0;                                                                           \
            clk[1] = r1 - r0;                                                                           \
        }                                                                                               \
    }

KERNEL(k_nop, PLANE_NOP)
KERNEL(k_nonop, PLANE_NONOP)
KERNEL(k_mov, PLANE_MOV)
KERNEL(k_xor, PLANE_XOR)

typedef void (*Kern)(uint32_t*, uint64_t*, uint32_t, int);

void run(const char* name, Kern k, uint32_t* d, uint64_t* dclk, int cus, int wps) {
    const int iters = 4096;
    dim3 grid(cus * wps), block(256);   // wps blocks of 4 waves per CU = wps waves per SIMD
    hipLaunchKernelGGL(k, grid, block, 0, 0, d, dclk, 1u, 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, grid, block, 0, 0, d, dclk, 1u, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t clk[2];
    (void)hipMemcpy(clk, dclk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)clk[0] / (clk[1] * 10.0);   // memrealtime = 100 MHz
    // VALU instructions per wave: 4 BODY x 8 planes x 6
    const double valu = (double)grid.x * 4 * iters * 4 * 8 * 6;
    const double simd_cycles = ms * 1e-3 * ghz * 1e9 * cus * 4;
    printf("%-40s waves/SIMD %d  SIMD cycles per VALU instr %.2f  (clock %.2f GHz)\n", name, wps,
           simd_cycles / valu, ghz);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    const int cus = p.multiProcessorCount;
    for (int wps : {2, 4}) {
        run("xor3 only (6 per plane)", k_xor, d, c, cus, wps);
        run("4 v_mov + 2 xor3 per plane", k_mov, d, c, cus, wps);
        run("4 idx lookups (s_nop after idx) + 2 xor3", k_nop, d, c, cus, wps);
        run("4 idx lookups [no wait] + 2 xor3", k_nonop, d, c, cus, wps);
    }
    return 0;
}
