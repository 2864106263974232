// Narrow-slice ownership probe: can one workgroup own
// EVERY row and column codeword of a narrow byte slice of a whole k = 128
// square (so Q0 is read once and Q2 never read back)?  Such a workgroup reads
// w bytes of each of the 16 384 Q0 cells (stride 512 B) and writes w bytes of
// each of the 3 x 16 384 parity cells; the 128 / w workgroups that share a
// 128-B line run on one XCD (blockIdx % 8 equal: speed only), so the line
// crosses the fabric once if the L2 keeps it while they read.
//
// Kernels (memory pattern only, no encode), over N squares in the EDS layout
// [N][256][256][512] (Q0 = rows < 128, cols < 128):
//   slice_rw<W> : one 512-thread workgroup per (square, W-byte slice): loads
//                 W bytes of every Q0 cell (32 per thread, all in flight),
//                 stores W bytes to the same offset of Q1, Q2 and Q3
//   line_rw     : the same bytes moved by 128-B-slice workgroups (the current
//                 MODE-2 access shape: 4 lanes x 32 B per line) -- the baseline
//   line_rw16   : the same, 8 lanes x 16 B per line (a whole line per load)
// Prints per kernel: ms per N squares, algorithmic TB/s (32 MiB per square).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr uint32_t K = 128, Wd = 256, SH = 512;
constexpr size_t SQ = (size_t)Wd * Wd * SH;

template <int W>
struct Vec;
template <>
struct Vec<4> { using T = uint32_t; };
template <>
struct Vec<8> { using T = uint2; };
template <>
struct Vec<16> { using T = uint4; };

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }
__device__ __forceinline__ uint32_t mix(uint32_t v, uint32_t s) { return v ^ s; }
__device__ __forceinline__ uint2 mix(uint2 v, uint32_t s) { return make_uint2(v.x ^ s, v.y); }
__device__ __forceinline__ uint4 mix(uint4 v, uint32_t s) { return make_uint4(v.x ^ s, v.y, v.z, v.w); }

// block b: xcd residue x = b % 8, j = b / 8; slices per square S = 512 / W;
// square = 8 * (j / S) + x, slice = j % S -- every slice of a square on one
// residue (one XCD under round-robin dispatch)
template <int W>
__global__ __launch_bounds__(512) void slice_rw(uint8_t* __restrict__ eds, uint32_t nsq) {
    using T = typename Vec<W>::T;
    constexpr uint32_t S = SH / W;
    const uint32_t b = blockIdx.x, x = b % 8, j = b / 8;
    const uint32_t sq = 8 * (j / S) + x, s = j % S;
    if (sq >= nsq) return;
    uint8_t* base = eds + (size_t)sq * SQ + (size_t)s * W;
    T v[32];
    // thread t, item i: Q0 cell i * 512 + t (row-major), 32 cells per thread
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const uint32_t cell = i * 512 + threadIdx.x;    // 0 .. 16383
        const uint32_t r = cell / K, c = cell % K;
        v[i] = *reinterpret_cast<const T*>(base + ((size_t)r * Wd + c) * SH);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) acc ^= fold(v[i]);
#pragma unroll
    for (int q = 1; q < 4; q++) {
        const uint32_t r0 = q & 2 ? K : 0, c0 = q & 1 ? K : 0;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            const uint32_t cell = i * 512 + threadIdx.x;
            const uint32_t r = cell / K + r0, c = cell % K + c0;
            *reinterpret_cast<T*>(base + ((size_t)r * Wd + c) * SH) = mix(v[i], acc + q);
        }
    }
}

// baseline: 128-B slices, lane = 32 B of a line (4 lanes per line), 128 cells
// of a row per wave-instruction group; one workgroup per (square, 128-B
// slice, block of 1024 cells) -- 16 workgroups per (square, slice)
__global__ __launch_bounds__(512) void line_rw(uint8_t* __restrict__ eds, uint32_t nsq) {
    const uint32_t b = blockIdx.x, x = b % 8, j = b / 8;
    const uint32_t per = 4 * 16;                      // (slice, block) pairs per square
    const uint32_t sq = 8 * (j / per) + x, rem = j % per, s = rem / 16, blk = rem % 16;
    if (sq >= nsq) return;
    uint8_t* base = eds + (size_t)sq * SQ + (size_t)s * 128 + 32 * (threadIdx.x & 3);
    uint4 v[16];   // 8 cells per thread x 32 B
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t cell = blk * 1024 + i * 128 + (threadIdx.x >> 2);   // 1024 cells per workgroup
        const uint32_t r = cell / K, c = cell % K;
        const uint8_t* p = base + ((size_t)r * Wd + c) * SH;
        v[2 * i] = *reinterpret_cast<const uint4*>(p);
        v[2 * i + 1] = *reinterpret_cast<const uint4*>(p + 16);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= fold(v[i]);
#pragma unroll
    for (int q = 1; q < 4; q++) {
        const uint32_t r0 = q & 2 ? K : 0, c0 = q & 1 ? K : 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t cell = blk * 1024 + i * 128 + (threadIdx.x >> 2);
            const uint32_t r = cell / K + r0, c = cell % K + c0;
            uint8_t* p = base + ((size_t)r * Wd + c) * SH;
            *reinterpret_cast<uint4*>(p) = mix(v[2 * i], acc + q);
            *reinterpret_cast<uint4*>(p + 16) = v[2 * i + 1];
        }
    }
}

// the same bytes with 8 lanes x 16 B per 128-B line per instruction (a whole
// line per 8 lanes, 2 lines per lane pair of instructions): lane l covers
// 16 B at 16 (l % 8) of the slice's line for 2 cells per load pair
__global__ __launch_bounds__(512) void line_rw16(uint8_t* __restrict__ eds, uint32_t nsq) {
    const uint32_t b = blockIdx.x, x = b % 8, j = b / 8;
    const uint32_t per = 4 * 16;
    const uint32_t sq = 8 * (j / per) + x, rem = j % per, s = rem / 16, blk = rem % 16;
    if (sq >= nsq) return;
    uint8_t* base = eds + (size_t)sq * SQ + (size_t)s * 128 + 16 * (threadIdx.x & 7);
    uint4 v[16];   // 16 cells per thread x 16 B
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t cell = blk * 1024 + i * 64 + (threadIdx.x >> 3);   // 1024 cells per workgroup
        const uint32_t r = cell / K, c = cell % K;
        v[i] = *reinterpret_cast<const uint4*>(base + ((size_t)r * Wd + c) * SH);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= fold(v[i]);
#pragma unroll
    for (int q = 1; q < 4; q++) {
        const uint32_t r0 = q & 2 ? K : 0, c0 = q & 1 ? K : 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t cell = blk * 1024 + i * 64 + (threadIdx.x >> 3);
            const uint32_t r = cell / K + r0, c = cell % K + c0;
            *reinterpret_cast<uint4*>(base + ((size_t)r * Wd + c) * SH) = mix(v[i], acc + q);
        }
    }
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> t;
    launch();
    (void)hipDeviceSynchronize();
    for (int i = 0; i < reps; i++) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 256;   // squares (multiple of 8)
    uint8_t* eds = nullptr;
    CK(hipMalloc(&eds, SQ * n));
    CK(hipMemset(eds, 1, SQ * n));
    const double alg = 4.0 * K * K * SH * n;   // Q0 read + 3 quadrants written
    auto report = [&](const char* name, float ms) {
        printf("%-12s n=%u  %8.3f ms  %.3f ms/128sq  alg %.2f TB/s\n", name, n, ms, ms * 128.0 / n,
               alg / (ms * 1e-3) / 1e12);
    };
    const uint32_t g = (n + 7) / 8 * 8;
    report("line_rw", time_ms([&] { hipLaunchKernelGGL(line_rw, dim3(g * 64), dim3(512), 0, 0, eds, n); }, 10));
    report("line_rw16", time_ms([&] { hipLaunchKernelGGL(line_rw16, dim3(g * 64), dim3(512), 0, 0, eds, n); }, 10));
    report("line_rw_b", time_ms([&] { hipLaunchKernelGGL(line_rw, dim3(g * 64), dim3(512), 0, 0, eds, n); }, 10));
    report("slice_rw16", time_ms([&] { hipLaunchKernelGGL(slice_rw<16>, dim3(g * 32), dim3(512), 0, 0, eds, n); }, 10));
    report("slice_rw8", time_ms([&] { hipLaunchKernelGGL(slice_rw<8>, dim3(g * 64), dim3(512), 0, 0, eds, n); }, 10));
    report("slice_rw4", time_ms([&] { hipLaunchKernelGGL(slice_rw<4>, dim3(g * 128), dim3(512), 0, 0, eds, n); }, 10));
    CK(hipGetLastError());
    CK(hipFree(eds));
    return 0;
}
