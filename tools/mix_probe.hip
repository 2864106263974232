// mix_probe.hip -- how gfx950 issues a MIX of half-rate (v_alignbit_b32) and
// full-rate (v_xor_b32 / v_bitop3_b32) VALU ops: interleaved one by one, in
// pairs, in blocks, and split across the waves of a SIMD.  Decides whether
// reordering SHA-256's instruction stream can reach the full-rate slots
// (a mixed stream issues at about the half rate).
// Build: hipcc --offload-arch=gfx950 -O3 -o mix_probe mix_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define A(r) "v_alignbit_b32 " r ", " r ", %16, %17\n\t"
#define X(r) "v_xor_b32 " r ", " r ", %16\n\t"
#define B3(r) "v_bitop3_b32 " r ", " r ", %16, %17 bitop3:0x96\n\t"
#define REGS                                                                                             \
    : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),   \
      "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]),           \
      "+v"(v[15])                                                                                        \
    : "v"(y), "v"(z)

// pattern -> (n_half, n_full) per asm block
template <int P>
struct Pat;
// 8 A then 8 X
template <> struct Pat<0> { static constexpr int h = 8, f = 8; };
// (A A X X) x 4
template <> struct Pat<1> { static constexpr int h = 8, f = 8; };
// (A X) x 8
template <> struct Pat<2> { static constexpr int h = 8, f = 8; };
// (A X X) x 5 + A  (1:2-ish)  -> 6 A, 10 X
template <> struct Pat<3> { static constexpr int h = 6, f = 10; };
// 16 A
template <> struct Pat<4> { static constexpr int h = 16, f = 0; };
// 16 X
template <> struct Pat<5> { static constexpr int h = 0, f = 16; };
// split waves: even waves 16 A, odd waves 16 X (counted as 8 + 8 average)
template <> struct Pat<6> { static constexpr int h = 8, f = 8; };
// (A B3) x 8 (bitop3 as the full-rate partner)
template <> struct Pat<7> { static constexpr int h = 8, f = 8; };
// 4 A then 4 X, twice
template <> struct Pat<8> { static constexpr int h = 8, f = 8; };

template <int P>
__global__ __launch_bounds__(512) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t y = seed * 0x9E3779B9u + threadIdx.x, z = y ^ 0x5bd1e995u;
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = y + i;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if constexpr (P == 0)
                asm volatile(A("%0") A("%1") A("%2") A("%3") A("%4") A("%5") A("%6") A("%7") X("%8") X("%9") X("%10")
                                 X("%11") X("%12") X("%13") X("%14") X("%15") REGS);
            if constexpr (P == 1)
                asm volatile(A("%0") A("%1") X("%8") X("%9") A("%2") A("%3") X("%10") X("%11") A("%4") A("%5") X("%12")
                                 X("%13") A("%6") A("%7") X("%14") X("%15") REGS);
            if constexpr (P == 2)
                asm volatile(A("%0") X("%8") A("%1") X("%9") A("%2") X("%10") A("%3") X("%11") A("%4") X("%12") A("%5")
                                 X("%13") A("%6") X("%14") A("%7") X("%15") REGS);
            if constexpr (P == 3)
                asm volatile(A("%0") X("%8") X("%9") A("%1") X("%10") X("%11") A("%2") X("%12") X("%13") A("%3")
                                 X("%14") X("%15") A("%4") X("%6") X("%7") A("%5") REGS);
            if constexpr (P == 4)
                asm volatile(A("%0") A("%1") A("%2") A("%3") A("%4") A("%5") A("%6") A("%7") A("%8") A("%9") A("%10")
                                 A("%11") A("%12") A("%13") A("%14") A("%15") REGS);
            if constexpr (P == 5)
                asm volatile(X("%0") X("%1") X("%2") X("%3") X("%4") X("%5") X("%6") X("%7") X("%8") X("%9") X("%10")
                                 X("%11") X("%12") X("%13") X("%14") X("%15") REGS);
            if constexpr (P == 6) {
                if ((wave >> 2) & 1)   // 512-thread blocks: waves 0-3 and 4-7 share the 4 SIMDs
                    asm volatile(X("%0") X("%1") X("%2") X("%3") X("%4") X("%5") X("%6") X("%7") X("%8") X("%9")
                                     X("%10") X("%11") X("%12") X("%13") X("%14") X("%15") REGS);
                else
                    asm volatile(A("%0") A("%1") A("%2") A("%3") A("%4") A("%5") A("%6") A("%7") A("%8") A("%9")
                                     A("%10") A("%11") A("%12") A("%13") A("%14") A("%15") REGS);
            }
            if constexpr (P == 7)
                asm volatile(A("%0") B3("%8") A("%1") B3("%9") A("%2") B3("%10") A("%3") B3("%11") A("%4") B3("%12")
                                 A("%5") B3("%13") A("%6") B3("%14") A("%7") B3("%15") REGS);
            if constexpr (P == 8)
                asm volatile(A("%0") A("%1") A("%2") A("%3") X("%8") X("%9") X("%10") X("%11") A("%4") A("%5") A("%6")
                                 A("%7") X("%12") X("%13") X("%14") X("%15") REGS);
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) s ^= v[i];
    if (s == 0x12345678u) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int P>
void run(const char* name, uint32_t* d, uint64_t* dclk, int cus, int blocks_per_cu) {
    const int iters = 1024;
    // pattern 6 splits the waves of a 512-thread block (one A wave and one X
    // wave per SIMD); the others use 256-thread blocks
    dim3 grid(P == 6 ? cus * blocks_per_cu / 2 : cus * blocks_per_cu), block(P == 6 ? 512 : 256);
    hipLaunchKernelGGL(probe<P>, grid, block, 0, 0, d, dclk, 1u, 32);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(probe<P>, grid, block, 0, 0, d, dclk, 1u, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t clk[2];
    (void)hipMemcpy(clk, dclk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)clk[0] / (clk[1] * 10.0);   // memrealtime = 100 MHz
    const double insts = (double)grid.x * (block.x / 64) * iters * 4 * 16;   // wave-instructions
    const double cyc = ms * 1e-3 * ghz * 1e9;
    const double per_simd = insts / (cus * 4);                                // wave-instr per SIMD
    const double cpi = cyc / per_simd;                                          // SIMD cycles per wave-instr
    // cost model: half-rate op = 4 cycles, full-rate op = 2 cycles -> ideal CPI
    const double ideal = (Pat<P>::h * 4.0 + Pat<P>::f * 2.0) / 16.0;
    printf("%-22s waves/SIMD %2d  %6.1f lane-ops/clk/CU  SIMD cycles per wave-instr %.2f (4/2 model %.2f)  clock %.2f GHz\n",
           name, blocks_per_cu, insts * 64 / cyc / cus, cpi, ideal, ghz);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    printf("device %s CUs %d\n", p.gcnArchName, p.multiProcessorCount);
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    const int cus = p.multiProcessorCount;
    for (int bpc : {4, 8}) {   // 256-thread blocks per CU = waves per SIMD
        run<4>("16 A (alignbit)", d, c, cus, bpc);
        run<5>("16 X (xor)", d, c, cus, bpc);
        run<0>("8 A then 8 X", d, c, cus, bpc);
        run<8>("(4 A, 4 X) x2", d, c, cus, bpc);
        run<1>("(A A X X) x4", d, c, cus, bpc);
        run<2>("(A X) x8", d, c, cus, bpc);
        run<7>("(A bitop3) x8", d, c, cus, bpc);
        run<3>("(A X X) 1:2", d, c, cus, bpc);
        run<6>("waves: A-only/X-only", d, c, cus, bpc);
    }
    return 0;
}
