// sha_latency_probe.hip -- latency of one dependent SHA-256 compression chain
// on gfx950 (the single-square tail: NMT top levels and the data-root tree),
// and what splitting each compression between two waves would buy.
//   lone   : one wave per SIMD, each lane runs a chain of dependent
//            compressions (next message = previous digest) -- today's kernels.
//   split  : two waves per chain: wave 1 expands the message schedule of the
//            next 16-word chunk into LDS while wave 0 runs the rounds of the
//            current chunk (s_barrier between chunks).
// Prints cycles per compression for each (s_memtime).  Planning evidence for
// DESIGN.md §7 item 3; not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -o sha_latency_probe sha_latency_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../celestia-app_amd/csrc/sha256_dev.h"

using namespace cda;

// Round with the shortest dependency chain written out: X = h + K + W + d off
// the chain (h, d are 3 rounds old), e' = X + S1(e) + Ch(e,f,g), a' = e' +
// S0(a) + (Maj(a,b,c) - d).  Measured: no faster than sha_compress for a lone
// wave (the compiler already reassociates those adds) -- the lone wave is
// bound by its own issue rate, ~4.25 cycles per instruction.
__device__ __forceinline__ void sha_compress_lat(ShaState& s, uint32_t w[16]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = add3(w[i & 15], s0, w[(i - 7) & 15]) + s1;
            w[i & 15] = wi;
        }
        const uint32_t X = add3(h, wi, d) + K[i];
        const uint32_t en = add3(X, xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)), ch(e, f, g));
        const uint32_t Z = maj(a, b, c) - d;
        const uint32_t an = add3(en, xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)), Z);
        h = g; g = f; f = e; e = en;
        d = c; c = b; b = a; a = an;
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}


__global__ __launch_bounds__(64) void lone(uint32_t* out, uint64_t* clk, int chain) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * 16 + i + blockIdx.x;
    ShaState s;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chain; c++) {
        sha_init(s);
        sha_compress(s, w);
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = s.h[i & 7] ^ (uint32_t)i;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= w[i];
    out[blockIdx.x * 64 + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

// lone, with the short-dependency round (sha_compress_lat above)
__global__ __launch_bounds__(64) void lone_lat(uint32_t* out, uint64_t* clk, int chain) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = threadIdx.x * 16 + i + blockIdx.x;
    ShaState s;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chain; c++) {
        sha_init(s);
        sha_compress_lat(s, w);
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = s.h[i & 7] ^ (uint32_t)i;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= w[i];
    out[blockIdx.x * 64 + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

// rounds t0..t0+15 of one compression reading W[t] from LDS (t >= 16) or the message
__device__ __forceinline__ void rounds16(uint32_t (&v)[8], const uint32_t* W, int t0) {
    constexpr uint32_t K[64] = CDA_SHA_K;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = t0 + j;
        const uint32_t wi = W[i * 64];
        uint32_t a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], f = v[5], g = v[6], h = v[7];
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t t1 = add3(add3(h, S1, ch(e, f, g)), K[i], wi);
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj(a, b, c);
        v[7] = g; v[6] = f; v[5] = e; v[4] = d + t1;
        v[3] = c; v[2] = b; v[1] = a; v[0] = add3(t1, S0, mj);
    }
}

__global__ __launch_bounds__(128) void split(uint32_t* out, uint64_t* clk, int chain) {
    __shared__ uint32_t W[64 * 64];   // [t][lane]
    const uint32_t lane = threadIdx.x & 63;
    const bool sched = threadIdx.x >= 64;
    uint32_t v[8];
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = lane * 16 + i + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chain; c++) {
        // message words 0..15 (both waves know them: the previous digest was
        // published through LDS at the end of the last compression)
        if (!sched) {
#pragma unroll
            for (int i = 0; i < 16; i++) W[i * 64 + lane] = m[i];
        }
        __syncthreads();
        uint32_t x[16];
#pragma unroll
        for (int i = 0; i < 16; i++) x[i] = W[i * 64 + lane];
        ShaState s;
        sha_init(s);
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = s.h[i];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (sched) {
                if (q < 3) {   // words 16(q+1) .. 16(q+1)+15
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const int i = 16 * (q + 1) + j;
                        const uint32_t w15 = x[(i - 15) & 15], w2 = x[(i - 2) & 15];
                        const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                        const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                        x[i & 15] = add3(x[i & 15], s0, x[(i - 7) & 15]) + s1;
                        W[i * 64 + lane] = x[i & 15];
                    }
                }
            } else {
                rounds16(v, W + lane, 16 * q);
            }
            __syncthreads();
        }
        if (!sched) {
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] += s.h[i];
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = v[i & 7] ^ (uint32_t)i;
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (!sched) {
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) r ^= v[i];
        out[blockIdx.x * 64 + lane] = r;
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 1 << 20);
    (void)hipMalloc(&c, 64);
    const int chain = 64;
    uint64_t h = 0;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(lone, dim3(256), dim3(64), 0, 0, d, c, chain);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (rep) printf("lone  wave : %.0f cycles per compression (s_memtime)\n", (double)h / chain);
        hipLaunchKernelGGL(lone_lat, dim3(256), dim3(64), 0, 0, d, c, chain);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (rep) printf("lone  wave, short-dependency round: %.0f cycles per compression (s_memtime)\n", (double)h / chain);
        hipLaunchKernelGGL(split, dim3(256), dim3(128), 0, 0, d, c, chain);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (rep) printf("split waves: %.0f cycles per compression (s_memtime)\n", (double)h / chain);
    }
    return 0;
}
