// Memory-only replicas of the k = 128 Q0 RS launch (rs8_bs_half_kernel<2>,
// "slices"): the same workgroups, the same loads of Q0 (row and column
// codewords over one 128-B slice of every cell) and the same stores to Q1 /
// Q2, with the XOR networks left out -- the data is copied, so the pattern's
// fabric rate can be compared with the flat copies of tools/bw_probe.hip.
//   lines64 : the kernel's lane mapping -- 4 lanes cover 64 B of a cell per
//             instruction, the second instruction the other 64 B
//   lines128: 8 lanes cover the whole 128-B slice of one cell per instruction
//             (the two shards of a lane pair alternate by instruction)
//   sleepN  : lines64 with N x s_sleep 127 (~8 k cycles each) between the
//             loads and the stores, standing in for the compute phase
//   l128slN : lines128 with the sleeps
//   rows / cols: lines64 with only the row (column) workgroups doing work
//             (the TB/s column still counts the whole launch's bytes)
// In-place EDS of n squares (2k x 2k cells of 512 B), Q0 = rows/cols < 128.
// Prints ms per launch and TB/s at the fabric (Q0 read once + Q1, Q2 written).
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

constexpr uint32_t kK = 128, kW = 256, kCell = 512;
constexpr size_t kRow = (size_t)kW * kCell, kSq = (size_t)kW * kRow;

// ONLY: 0 = rows and columns (the launch), 1 = rows only, 2 = columns only
template <int MAP, int SLEEP = 0, int ONLY = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void q0_pattern(uint8_t* __restrict__ eds, uint32_t nsq) {
    constexpr uint32_t P = 32;   // 256 codewords / 8 per workgroup
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t b = blockIdx.x, grp = b / (8 * P), r = b % (8 * P);
    const uint32_t unit = grp * 8 + (r & 7), j = r >> 3;
    const uint32_t sq = unit >> 2;
    if (sq >= nsq) return;
    if ((ONLY == 1 && j >= 16) || (ONLY == 2 && j < 16)) return;
    const bool col = j >= 16;   // codewords 0..127 rows, 128..255 columns
    const uint32_t cw = 8 * (j & 15) + (l >> 3);
    // per codeword: shard stride, source / destination base
    const size_t sh = col ? kRow : kCell;
    const size_t cwo = col ? (size_t)cw * kCell : (size_t)cw * kRow;
    const size_t dsto = col ? (size_t)kK * kRow : (size_t)kK * kCell;
    uint8_t* base = eds + (size_t)sq * kSq + cwo;
    const uint32_t slice = 128 * (unit & 3);
    // (plain dwords: an array of uint4 stayed in scratch)
    uint32_t R[64];
    auto ld = [&](int i, const uint8_t* a) {
        const uint4 v = *reinterpret_cast<const uint4*>(a);
        R[4 * i] = v.x; R[4 * i + 1] = v.y; R[4 * i + 2] = v.z; R[4 * i + 3] = v.w;
    };
    auto st = [&](int i, uint8_t* a) {
        *reinterpret_cast<uint4*>(a) = make_uint4(R[4 * i], R[4 * i + 1], R[4 * i + 2], R[4 * i + 3]);
    };
    if constexpr (MAP == 0) {
        const uint32_t h = (l >> 2) & 1, c16 = 16 * (l & 3);
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const size_t o = (16 * w + 2 * jj + h) * sh + slice + c16;
            ld(2 * jj, base + o);
            ld(2 * jj + 1, base + o + 64);
        }
        if constexpr (SLEEP > 0) {   // stand-in for the XOR networks between loads and stores
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int z = 0; z < SLEEP; z++) __builtin_amdgcn_s_sleep(127);
        }
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const size_t o = dsto + (16 * w + 2 * jj + h) * sh + slice + c16;
            st(2 * jj, base + o);
            st(2 * jj + 1, base + o + 64);
        }
    } else {
        const uint32_t c16 = 16 * (l & 7);
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const size_t o = (16 * w + 2 * jj + h) * sh + slice + c16;
                ld(2 * jj + h, base + o);
            }
        }
        if constexpr (SLEEP > 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int z = 0; z < SLEEP; z++) __builtin_amdgcn_s_sleep(127);
        }
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const size_t o = dsto + (16 * w + 2 * jj + h) * sh + slice + c16;
                st(2 * jj + h, base + o);
            }
        }
    }
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 256;   // 256: 8 GiB of EDS
    uint8_t* eds;
    CK(hipMalloc(&eds, (size_t)n * kSq));
    CK(hipMemset(eds, 0x3c, (size_t)n * kSq));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t grid = (4 * n + 7) / 8 * 256;
    const double moved = (double)n * 3 * kK * kK * kCell;   // Q0 once + Q1 + Q2
    for (int rep = 0; rep < 2; rep++) {
        for (int m = 0; m < 8; m++) {
            std::vector<float> t;
            for (int r = 0; r < 11; r++) {
                CK(hipEventRecord(e0));
                if (m == 0) hipLaunchKernelGGL(q0_pattern<0>, dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 1) hipLaunchKernelGGL(q0_pattern<1>, dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 2) hipLaunchKernelGGL((q0_pattern<0, 1>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 3) hipLaunchKernelGGL((q0_pattern<0, 2>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 4) hipLaunchKernelGGL((q0_pattern<0, 0, 1>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 5) hipLaunchKernelGGL((q0_pattern<0, 0, 2>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 6) hipLaunchKernelGGL((q0_pattern<1, 1>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                if (m == 7) hipLaunchKernelGGL((q0_pattern<1, 2>), dim3(grid), dim3(512), 64 * 1024, 0, eds, n);
                CK(hipGetLastError());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double ms = t[t.size() / 2];
            printf("%-8s %u squares: %7.3f ms (%.3f ms per 1024)  %.2f TB/s at the fabric if Q0 is read once\n",
                   m == 0 ? "lines64" : m == 1 ? "lines128" : m == 2 ? "sleep1" : m == 3 ? "sleep2" : m == 4 ? "rows" : m == 5 ? "cols" : m == 6 ? "l128sl1" : "l128sl2", n, ms, ms * 1024 / n, moved / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
