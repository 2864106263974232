// sched_probe.hip -- latency of one SHA-256 compression on a lone wave
// (DESIGN.md 7.4): the lane-pair compression as used in the tree tops, the
// same rounds with the message schedule already computed (what a second
// "schedule wave" would hand over through LDS), and the one-lane
// compression.  One 64-thread workgroup per CU (one wave on one SIMD), a
// chain of dependent compressions per lane; reports cycles per compression.
// Build: hipcc --offload-arch=gfx950 -O3 -I../celestia-app_amd/csrc -o sched_probe sched_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#include "sha256_dev.h"

using namespace cda;

// lane-pair rounds over a precomputed schedule W[0..63] (K folded in by the
// caller: KW[i] = K[i] + W[i]), the body of sha_pair_compress without the
// schedule words
__device__ __forceinline__ void pair_rounds(ShaPair& s, const uint32_t (&KW)[64], bool A) {
    const uint32_t r1 = A ? 2u : 6u, r2 = A ? 13u : 11u, r3 = A ? 22u : 25u;
    uint32_t v0 = s.h[0], v1 = s.h[1], v2 = s.h[2], v3 = s.h[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t S = xor3(__builtin_amdgcn_alignbit(v0, v0, r1), __builtin_amdgcn_alignbit(v0, v0, r2),
                                __builtin_amdgcn_alignbit(v0, v0, r3));
        const uint32_t F = pair_sel(ch(v0, v1, v2), maj(v0, v1, v2));
        const uint32_t Y = pair_sel(v3 + KW[i], 0u);
        const uint32_t T = add3(S, F, Y);
        const uint32_t nv = pair_add(T, pair_sel(T, v3));
        v3 = v2; v2 = v1; v1 = v0; v0 = nv;
    }
    s.h[0] += v0; s.h[1] += v1; s.h[2] += v2; s.h[3] += v3;
}

// one-lane rounds over a precomputed K+W schedule
__device__ __forceinline__ void lane_rounds(ShaState& s, const uint32_t (&KW)[64]) {
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t t1 = add3(h, S1, ch(e, f, g)) + KW[i];
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = add3(t1, S0, mj);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

__constant__ const uint32_t kK[64] = CDA_SHA_K;

#define SB __builtin_amdgcn_sched_barrier(0);
// one lane, the schedule word t+16 interleaved op by op into round t, the
// order pinned with sched_barrier (the scheduler may not move anything
// across): the schedule's independent ops fill the round chain's stalls
__device__ __forceinline__ void lane_interleaved(ShaState& s, uint32_t (&w)[16]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
    uint32_t kw[64];
#pragma unroll
    for (int t = 0; t < 16; t++) kw[t] = w[t] + K[t];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const bool sc = i + 16 < 64;
        const int t = i + 16;
        uint32_t w15 = 0, w2 = 0, r7 = 0, r18 = 0, r17 = 0, r19 = 0, x0 = 0, x1 = 0;
        uint32_t e6 = rotr(e, 6); SB
        if (sc) { w15 = w[(t - 15) & 15]; w2 = w[(t - 2) & 15]; r7 = rotr(w15, 7); } SB
        uint32_t e11 = rotr(e, 11); SB
        if (sc) r18 = rotr(w15, 18); SB
        uint32_t e25 = rotr(e, 25); SB
        if (sc) r17 = rotr(w2, 17); SB
        const uint32_t S1 = xor3(e6, e11, e25); SB
        if (sc) r19 = rotr(w2, 19); SB
        const uint32_t chv = ch(e, f, g); SB
        if (sc) x0 = xor3(r7, r18, w15 >> 3); SB
        const uint32_t t1 = add3(h, S1, chv) + kw[i]; SB
        if (sc) x1 = xor3(r17, r19, w2 >> 10); SB
        const uint32_t a2 = rotr(a, 2), a13 = rotr(a, 13), a22 = rotr(a, 22); SB
        if (sc) { w[t & 15] = add3(w[t & 15], x0, w[(t - 7) & 15]) + x1; kw[t] = w[t & 15] + K[t]; } SB
        const uint32_t S0 = xor3(a2, a13, a22), mj = maj(a, b, c); SB
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = add3(t1, S0, mj);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

template <int V>
__global__ __launch_bounds__(64) void probe(uint32_t* out, uint64_t* clk, uint32_t seed, int n) {
    const bool A = threadIdx.x & 1;
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = seed * (j + 1) + threadIdx.x;
    uint32_t KW[64];
    if constexpr (V == 1 || V == 3) {   // a fixed schedule (laundered so it is not folded)
#pragma unroll
        for (int j = 0; j < 64; j++) {
            KW[j] = seed * 0x9E3779B9u + j * 0x85EBCA6Bu + threadIdx.x;
            asm volatile("" : "+v"(KW[j]));
        }
    }
    ShaPair ps;
    ShaState ss;
    sha_pair_init(ps, A);
    sha_init(ss);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; it++) {
        if constexpr (V == 0) {   // lane pair, schedule on the same wave (the tree tops today)
            sha_pair_compress(ps, w, A);
#pragma unroll
            for (int j = 0; j < 4; j++) w[j] ^= ps.h[j];   // next message depends on this digest
        } else if constexpr (V == 1) {   // lane pair, schedule precomputed
            pair_rounds(ps, KW, A);
            KW[0] ^= ps.h[0];   // keep the chain dependent
        } else if constexpr (V == 4) {   // one lane, the schedule as its own phase on the same wave
            uint32_t kw[64];
#pragma unroll
            for (int t = 0; t < 16; t++) kw[t] = w[t] + kK[t];
#pragma unroll
            for (int t = 16; t < 64; t++) {
                const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                w[t & 15] = add3(w[t & 15], xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3), w[(t - 7) & 15]) +
                            xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                kw[t] = w[t & 15] + kK[t];
            }
            asm volatile("" ::: "memory");
            lane_rounds(ss, kw);
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] ^= ss.h[j];
        } else if constexpr (V == 5) {   // one lane, hand-interleaved schedule
            lane_interleaved(ss, w);
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] ^= ss.h[j];
        } else if constexpr (V == 3) {   // one lane, schedule precomputed
            lane_rounds(ss, KW);
            KW[0] ^= ss.h[0];
        } else {   // one lane per compression
            sha_compress(ss, w);
#pragma unroll
            for (int j = 0; j < 8; j++) w[j] ^= ss.h[j];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = ps.h[0] ^ ps.h[3] ^ ss.h[0] ^ ss.h[7] ^ w[5];
    if (acc == 0x12345678u) out[0] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int V>
void run(const char* name, uint32_t* d, uint64_t* c, int cus) {
    const int n = 200;
    hipLaunchKernelGGL(probe<V>, dim3(cus), dim3(64), 0, 0, d, c, 1u, 4);
    hipLaunchKernelGGL(probe<V>, dim3(cus), dim3(64), 0, 0, d, c, 1u, n);
    (void)hipDeviceSynchronize();
    uint64_t clk;
    (void)hipMemcpy(&clk, c, 8, hipMemcpyDeviceToHost);
    printf("%-44s %8.0f cycles per compression (lone wave)\n", name, (double)clk / n);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    uint64_t* c;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&c, 64);
    for (int r = 0; r < 2; r++) {
        run<0>("lane pair, schedule on the same wave", d, c, p.multiProcessorCount);
        run<1>("lane pair, schedule precomputed (K+W)", d, c, p.multiProcessorCount);
        run<2>("one lane per compression", d, c, p.multiProcessorCount);
        run<3>("one lane, schedule precomputed (K+W)", d, c, p.multiProcessorCount);
        run<4>("one lane, schedule as a separate phase", d, c, p.multiProcessorCount);
        run<5>("one lane, schedule hand-interleaved", d, c, p.multiProcessorCount);
    }
    return 0;
}
