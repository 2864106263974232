// bs16_probe.hip -- issue-rate probes for the bitsliced GF(2^16) encoder
// (celestia-app_amd/csrc/bitslice16.h):
//   * v_xor / v_bitop3 streams at 1..4 waves per SIMD (is a full-rate stream
//     full rate at the 2 waves per SIMD of a 256-VGPR kernel?);
//   * DPP-modified v_xor (quad_perm, row_ror:8, row_half_mirror) and
//     v_permlane32_swap / v_permlane16_swap (cross-lane butterflies);
//   * the k = 512 middle phases as the encoder would run them on 8 units per
//     lane: M2 (shard bits 6-8 in registers, one code path) and M1 (bits 3-5,
//     constants depend on the wave: one of 8 code paths per wave, I-cache).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I celestia-app_amd/csrc -o tools/bs16_probe tools/bs16_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "bitslice16.h"

using namespace cda;

#define REGS                                                                                             \
    : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),   \
      "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]),           \
      "+v"(v[15])                                                                                        \
    : "v"(y), "v"(z)
#define X(r) "v_xor_b32 " r ", " r ", %16\n\t"
#define B3(r) "v_bitop3_b32 " r ", " r ", %16, %17 bitop3:0x96\n\t"
#define DQ(r) "v_xor_b32_dpp " r ", %16, " r " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define DR(r) "v_xor_b32_dpp " r ", %17, " r " row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
#define DM(r) "v_xor_b32_dpp " r ", %16, " r " row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
#define X16(M) M("%0") M("%1") M("%2") M("%3") M("%4") M("%5") M("%6") M("%7") M("%8") M("%9") M("%10") M("%11") \
    M("%12") M("%13") M("%14") M("%15")
#define PL32(a, b) "v_permlane32_swap_b32 " a ", " b "\n\t"
#define PL16(a, b) "v_permlane16_swap_b32 " a ", " b "\n\t"

template <int P>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t y = seed * 0x9E3779B9u + threadIdx.x, z = y ^ 0x5bd1e995u;
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = y + i;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if constexpr (P == 0) asm volatile(X16(X) REGS);
            if constexpr (P == 1) asm volatile(X16(B3) REGS);
            if constexpr (P == 2) asm volatile("s_nop 1\n\t" X16(DQ) REGS);
            if constexpr (P == 3) asm volatile("s_nop 1\n\t" X16(DR) REGS);
            if constexpr (P == 4) asm volatile("s_nop 1\n\t" X16(DM) REGS);
            if constexpr (P == 5)   // 8 swaps (each moves 2 registers) + 8 xors
                asm volatile("s_nop 4\n\t" PL32("%0", "%1") PL32("%2", "%3") PL32("%4", "%5") PL32("%6", "%7")
                                 PL32("%8", "%9") PL32("%10", "%11") PL32("%12", "%13") PL32("%14", "%15")
                                     X("%0") X("%2") X("%4") X("%6") X("%8") X("%10") X("%12") X("%14") REGS);
            if constexpr (P == 6)
                asm volatile("s_nop 4\n\t" PL16("%0", "%1") PL16("%2", "%3") PL16("%4", "%5") PL16("%6", "%7")
                                 PL16("%8", "%9") PL16("%10", "%11") PL16("%12", "%13") PL16("%14", "%15")
                                     X("%0") X("%2") X("%4") X("%6") X("%8") X("%10") X("%12") X("%14") REGS);
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

// ---- encoder phases on 8 units (128 planes) per lane ------------------------
constexpr int K = 512;
// M2: shard = base + 64 r (r = register unit 0..7): IFFT d = 64, 128, 256 then FFT back
__device__ __forceinline__ void phase_m2(uint32_t* R) {
    bs16::sfor<0, 3, 1>([&](auto ld) {
        constexpr int dr = 1 << decltype(ld)::value;
        bs16::sfor<0, 8, 2 * dr>([&](auto gg) {
            constexpr int gr = decltype(gg)::value;
            constexpr uint32_t C = bs16::skew_value(K - 1 + 64 * gr + 64 * dr);
            bs16::sfor<gr, gr + dr, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                bs16::ifft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
            });
        });
    });
    bs16::sfor<0, 3, 1>([&](auto ld) {
        constexpr int dr = 4 >> decltype(ld)::value;
        bs16::sfor<0, 8, 2 * dr>([&](auto gg) {
            constexpr int gr = decltype(gg)::value;
            constexpr uint32_t C = bs16::skew_value(64 * gr + 64 * dr - 1);
            bs16::sfor<gr, gr + dr, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                bs16::fft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
            });
        });
    });
}
// M1: shard = 64 U + 8 r + low: IFFT d = 8, 16, 32 then FFT back (constants depend on U)
template <int U>
__device__ __forceinline__ void phase_m1(uint32_t* R) {
    bs16::sfor<0, 3, 1>([&](auto ld) {
        constexpr int dr = 1 << decltype(ld)::value;
        bs16::sfor<0, 8, 2 * dr>([&](auto gg) {
            constexpr int gr = decltype(gg)::value;
            constexpr uint32_t C = bs16::skew_value(K - 1 + 64 * U + 8 * gr + 8 * dr);
            bs16::sfor<gr, gr + dr, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                bs16::ifft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
            });
        });
    });
    bs16::sfor<0, 3, 1>([&](auto ld) {
        constexpr int dr = 4 >> decltype(ld)::value;
        bs16::sfor<0, 8, 2 * dr>([&](auto gg) {
            constexpr int gr = decltype(gg)::value;
            constexpr uint32_t C = bs16::skew_value(64 * U + 8 * gr + 8 * dr - 1);
            bs16::sfor<gr, gr + dr, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                bs16::fft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
            });
        });
    });
}

template <int P>
__global__ __launch_bounds__(256) void enc_probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t R[128];
#pragma unroll
    for (int i = 0; i < 128; i++) R[i] = seed * 0x9E3779B9u + threadIdx.x * 131u + i;
    const uint32_t u = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) + 4 * (blockIdx.x & 1)) & 7;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        if constexpr (P == 0) {
            phase_m2(R);
        } else if constexpr (P == 1) {
            switch (u) {
                case 0: phase_m1<0>(R); break;
                case 1: phase_m1<1>(R); break;
                case 2: phase_m1<2>(R); break;
                case 3: phase_m1<3>(R); break;
                case 4: phase_m1<4>(R); break;
                case 5: phase_m1<5>(R); break;
                case 6: phase_m1<6>(R); break;
                default: phase_m1<7>(R); break;
            }
        } else {
            phase_m1<3>(R);   // one M1 code path for every wave (I-cache reference)
        }
        bs16::fence<128>(R);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 128; i++) s ^= R[i];
    if (s == 0x12345678u) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}


// ---- decomposed layers: constant = compile-time part ^ lane terms ^ wave terms
// x-updates of a layer commute, so each term runs over all the layer's butterflies
// LOW: unit r = shard bits 0..2; lane masks m[0..2] for bits 3..5; u = bits 6..8
template <bool INV, int b>
__device__ __forceinline__ void low_layer(uint32_t* R, const uint32_t* m, uint32_t u) {
    constexpr int d = 1 << b;
    if constexpr (INV)
        bs16::sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & d) == 0)
#pragma unroll
                for (int p = 0; p < 16; p++) R[16 * (i + d) + p] ^= R[16 * i + p];
        });
    bs16::sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr ((i & d) == 0) {
            constexpr uint32_t C0 = bs16::skew_part<INV, 9>(b, (uint32_t)(i & ~(2 * d - 1)));
            bs16::mul_add<C0>(R + 16 * i, R + 16 * (i + d));
            bs16::mul_add_masked<bs16::tbasis(b, 3)>(R + 16 * i, R + 16 * (i + d), m[0]);
            bs16::mul_add_masked<bs16::tbasis(b, 4)>(R + 16 * i, R + 16 * (i + d), m[1]);
            bs16::mul_add_masked<bs16::tbasis(b, 5)>(R + 16 * i, R + 16 * (i + d), m[2]);
        }
    });
    bs16::sfor<0, 3, 1>([&](auto ww) {
        constexpr int w = decltype(ww)::value;
        if (u & (1u << w)) {
            bs16::sfor<0, 8, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                if constexpr ((i & d) == 0) bs16::mul_add<bs16::tbasis(b, 6 + w)>(R + 16 * i, R + 16 * (i + d));
            });
        }
    });
    if constexpr (!INV)
        bs16::sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & d) == 0)
#pragma unroll
                for (int p = 0; p < 16; p++) R[16 * (i + d) + p] ^= R[16 * i + p];
        });
    bs16::fence<128>(R);
}
__device__ __forceinline__ void phase_low(uint32_t* R, const uint32_t* m, uint32_t u) {
    low_layer<true, 0>(R, m, u);
    low_layer<true, 1>(R, m, u);
    low_layer<true, 2>(R, m, u);
    low_layer<false, 2>(R, m, u);
    low_layer<false, 1>(R, m, u);
    low_layer<false, 0>(R, m, u);
}
// M1 decomposed: unit r = shard bits 3..5, u = bits 6..8
template <bool INV, int b>
__device__ __forceinline__ void m1_layer(uint32_t* R, uint32_t u) {
    constexpr int d = 1 << (b - 3);
    if constexpr (INV)
        bs16::sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & d) == 0)
#pragma unroll
                for (int p = 0; p < 16; p++) R[16 * (i + d) + p] ^= R[16 * i + p];
        });
    bs16::sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr ((i & d) == 0) {
            constexpr uint32_t C0 = bs16::skew_part<INV, 9>(b, (uint32_t)(8 * (i & ~(2 * d - 1))));
            bs16::mul_add<C0>(R + 16 * i, R + 16 * (i + d));
        }
    });
    bs16::sfor<0, 3, 1>([&](auto ww) {
        constexpr int w = decltype(ww)::value;
        if (u & (1u << w)) {
            bs16::sfor<0, 8, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                if constexpr ((i & d) == 0) bs16::mul_add<bs16::tbasis(b, 6 + w)>(R + 16 * i, R + 16 * (i + d));
            });
        }
    });
    if constexpr (!INV)
        bs16::sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & d) == 0)
#pragma unroll
                for (int p = 0; p < 16; p++) R[16 * (i + d) + p] ^= R[16 * i + p];
        });
    bs16::fence<128>(R);
}
__device__ __forceinline__ void phase_m1_dec(uint32_t* R, uint32_t u) {
    m1_layer<true, 3>(R, u);
    m1_layer<true, 4>(R, u);
    m1_layer<true, 5>(R, u);
    m1_layer<false, 5>(R, u);
    m1_layer<false, 4>(R, u);
    m1_layer<false, 3>(R, u);
}
// M1 as compile-time regions: IFFT half, FFT half
template <int U, bool INV>
__device__ __forceinline__ void m1_half(uint32_t* R) {
    bs16::sfor<0, 3, 1>([&](auto ld) {
        constexpr int dr = INV ? (1 << decltype(ld)::value) : (4 >> decltype(ld)::value);
        bs16::sfor<0, 8, 2 * dr>([&](auto gg) {
            constexpr int gr = decltype(gg)::value;
            constexpr uint32_t C = INV ? bs16::skew_value(K - 1 + 64 * U + 8 * gr + 8 * dr)
                                       : bs16::skew_value(64 * U + 8 * gr + 8 * dr - 1);
            bs16::sfor<gr, gr + dr, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                if constexpr (INV)
                    bs16::ifft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
                else
                    bs16::fft_bfly<C>(R + 16 * i, R + 16 * (i + dr));
            });
        });
    });
}
template <bool INV>
__device__ __forceinline__ void m1_switch(uint32_t* R, uint32_t u) {
    switch (u) {
        case 0: m1_half<0, INV>(R); break;
        case 1: m1_half<1, INV>(R); break;
        case 2: m1_half<2, INV>(R); break;
        case 3: m1_half<3, INV>(R); break;
        case 4: m1_half<4, INV>(R); break;
        case 5: m1_half<5, INV>(R); break;
        case 6: m1_half<6, INV>(R); break;
        default: m1_half<7, INV>(R); break;
    }
}
template <bool INV>
__device__ __forceinline__ void m1_chain(uint32_t* R, uint32_t u) {
    bs16::sfor<0, 8, 1>([&](auto uu) {
        if (u == (uint32_t)decltype(uu)::value) m1_half<decltype(uu)::value, INV>(R);
    });
}

template <int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void enc_probe2(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    uint32_t R[128];
#pragma unroll
    for (int i = 0; i < 128; i++) R[i] = seed * 0x9E3779B9u + threadIdx.x * 131u + i;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t m[3];
#pragma unroll
    for (int i = 0; i < 3; i++) m[i] = 0u - ((lane >> (3 + i)) & 1);
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        // the wave's U changes every iteration (no loop unswitching; every case runs)
        const uint32_t u = __builtin_amdgcn_readfirstlane((wv + 4 * (blockIdx.x & 1) + (uint32_t)it) & 7);
        if constexpr (P == 0) phase_low(R, m, u);
        if constexpr (P == 1) phase_m1_dec(R, u);
        if constexpr (P == 2) {
            m1_switch<true>(R, u);
            bs16::fence<128>(R);
            m1_switch<false>(R, u);
        }
        if constexpr (P == 3) {
            m1_chain<true>(R, u);
            bs16::fence<128>(R);
            m1_chain<false>(R, u);
        }
        bs16::fence<128>(R);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 128; i++) s ^= R[i];
    if (s == 0x12345678u) out[0] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

static double run_timed(void (*launch)(int, uint32_t*, uint64_t*, int), int iters, uint32_t* d, uint64_t* dc,
                        int grid, double* ghz) {
    launch(grid, d, dc, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    launch(grid, d, dc, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t clk[2];
    (void)hipMemcpy(clk, dc, 16, hipMemcpyDeviceToHost);
    *ghz = (double)clk[0] / (clk[1] * 10.0);   // memrealtime = 100 MHz
    return ms;
}

template <int P>
void run_alu(const char* name, uint32_t* d, uint64_t* dc, int cus, int wps, double per_iter_insts) {
    const int iters = 2048;
    auto L = [](int g, uint32_t* d, uint64_t* c, int it) { hipLaunchKernelGGL(probe<P>, dim3(g), dim3(256), 0, 0, d, c, 1u, it); };
    double ghz;
    const double ms = run_timed(L, iters, d, dc, cus * wps, &ghz);
    const double insts = (double)cus * wps * 4 * iters * per_iter_insts;   // wave-instructions
    const double cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-28s waves/SIMD %d  SIMD cycles per wave-instr %.2f  clock %.2f GHz\n", name, wps,
           cyc / (insts / (cus * 4)), ghz);
}

template <int P, bool V2 = false>
void run_enc(const char* name, uint32_t* d, uint64_t* dc, int cus, int wps) {
    const int iters = 256;
    auto L = [](int g, uint32_t* d, uint64_t* c, int it) {
        if constexpr (V2)
            hipLaunchKernelGGL(enc_probe2<P>, dim3(g), dim3(256), 0, 0, d, c, 1u, it);
        else
            hipLaunchKernelGGL(enc_probe<P>, dim3(g), dim3(256), 0, 0, d, c, 1u, it);
    };
    double ghz;
    const double ms = run_timed(L, iters, d, dc, cus * wps, &ghz);
    const double cyc = ms * 1e-3 * ghz * 1e9;
    // per SIMD: wps waves x iters phases; 8 units x 32 symbols x 6 layers per phase per lane
    const double phases_per_simd = (double)wps * iters;
    printf("%-28s waves/SIMD %d  SIMD cycles per wave-phase %.0f  (per unit-layer %.1f)  clock %.2f GHz\n", name,
           wps, cyc / phases_per_simd, cyc / phases_per_simd / (8 * 6), ghz);
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
    for (int wps : {2}) {
        run_enc<0, true>("LOW decomposed (3 lane+3 wave)", d, c, cus, wps);
        run_enc<1, true>("M1 decomposed (3 wave)", d, c, cus, wps);
        run_enc<2, true>("M1 switch per half", d, c, cus, wps);
        run_enc<3, true>("M1 if-chain per half", d, c, cus, wps);
        run_enc<0>("M2 (one code path)", d, c, cus, wps);
    }
    if (getenv("ALL") == nullptr) return 0;
    for (int wps : {1, 2, 3, 4}) {
        run_alu<0>("xor", d, c, cus, wps, 64);
        run_alu<1>("bitop3", d, c, cus, wps, 64);
        run_alu<2>("xor dpp quad_perm", d, c, cus, wps, 64);
        run_alu<3>("xor dpp row_ror:8", d, c, cus, wps, 64);
        run_alu<4>("xor dpp row_half_mirror", d, c, cus, wps, 64);
        run_alu<5>("permlane32_swap + xor (8+8)", d, c, cus, wps, 64);
        run_alu<6>("permlane16_swap + xor (8+8)", d, c, cus, wps, 64);
    }
    for (int wps : {1, 2}) {
        run_enc<0>("M2 (one code path)", d, c, cus, wps);
        run_enc<2>("M1 U=3 on every wave", d, c, cus, wps);
        run_enc<1>("M1 switch(wave)", d, c, cus, wps);
    }
    return 0;
}
