// sha_probe.hip -- achievable SHA-256 compression rate on gfx950 for the exact
// instruction stream the NMT kernels use (sha256_dev.h sha_compress), with no
// memory traffic: every lane chains compressions on register data.  This is
// the issue ceiling of the mixed alignbit / add3 / bitop3 / add / shift stream
// (tools/valu_probe.hip shows a half-rate op interleaved with a full-rate one
// runs at about the half rate), i.e. the realistic roofline of the hash stages.
// Build: hipcc --offload-arch=gfx950 -O3 -o sha_probe sha_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../celestia-app_amd/csrc/sha256_dev.h"

template <int WAVES_PER_EU>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int iters) {
    cda::ShaState s;
    cda::sha_init(s);
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = seed * 0x9E3779B9u + threadIdx.x * 16 + i + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = w[i] ^ s.h[i & 7];
        cda::sha_compress(s, m);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= s.h[i];
    if (x == 0x12345678u) out[0] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    const int iters = 512;
    for (int bpc : {4, 8, 16}) {   // 256-thread blocks per CU: 1, 2, 4 waves per SIMD
        dim3 grid(cus * bpc), block(256);
        hipLaunchKernelGGL(probe<1>, grid, block, 0, 0, d, c, 1u, 8);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(probe<1>, grid, block, 0, 0, d, c, 1u, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        uint64_t clk[2];
        (void)hipMemcpy(clk, c, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)clk[0] / (clk[1] * 10.0);   // memrealtime = 100 MHz
        const double comp = (double)grid.x * block.x * iters;
        printf("waves/SIMD %d: %.3f G compressions/s  (%.1f T issue-slots/s at 2182 slots)  in-kernel clock %.2f GHz"
               " -> %.1f instr/clk/CU at 1384 instr\n",
               bpc / 4, comp / (ms * 1e-3) / 1e9, comp * 2182 / (ms * 1e-3) / 1e12, ghz,
               comp * 1384 * 64 / (ms * 1e-3) / (cus * ghz * 1e9) / 64);
    }
    return 0;
}
