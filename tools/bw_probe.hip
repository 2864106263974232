// HBM bandwidth by read : write mix (GPU box; tools/run_r03x.sh builds and
// runs it): the achievable rate for the RS launches' access patterns.
//   copy11  : read N, write N            (the Q3 launch: Q2 -> Q3)
//   copy12  : read N, write 2N           (the Q0 launch: Q0 -> Q1 and Q2)
//   write   : write N
//   read    : read N (summed into one word per thread so the loads stay live)
// plus copy11 / copy12 with one element per thread and no loop.
// 16-B accesses, 512-thread workgroups, grid-stride over 4 GiB (beyond the
// 256 MB MALL), 8 lines in flight per thread.  Prints TB/s at the fabric
// (bytes read + written) per kernel, median of 10 launches.
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

constexpr int kU = 8;   // 16-B elements per thread per iteration

__global__ __launch_bounds__(512) void copy11(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 512 * kU;
    for (size_t base = (size_t)blockIdx.x * 512 * kU + threadIdx.x; base < n; base += stride) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = a[base + u * 512];
#pragma unroll
        for (int u = 0; u < kU; u++) b[base + u * 512] = v[u];
    }
}

__global__ __launch_bounds__(512) void copy12(const uint4* __restrict__ a, uint4* __restrict__ b,
                                               uint4* __restrict__ c, size_t n) {
    const size_t stride = (size_t)gridDim.x * 512 * kU;
    for (size_t base = (size_t)blockIdx.x * 512 * kU + threadIdx.x; base < n; base += stride) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = a[base + u * 512];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            b[base + u * 512] = v[u];
            c[base + u * 512] = make_uint4(v[u].y, v[u].x, v[u].w, v[u].z);
        }
    }
}

__global__ __launch_bounds__(512) void write_only(uint4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 512 * kU;
    for (size_t base = (size_t)blockIdx.x * 512 * kU + threadIdx.x; base < n; base += stride) {
#pragma unroll
        for (int u = 0; u < kU; u++) b[base + u * 512] = make_uint4((uint32_t)base, u, 0, 1);
    }
}

__global__ __launch_bounds__(512) void read_only(const uint4* __restrict__ a, uint32_t* __restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * 512 * kU;
    uint32_t acc = 0;
    for (size_t base = (size_t)blockIdx.x * 512 * kU + threadIdx.x; base < n; base += stride) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = a[base + u * 512];
#pragma unroll
        for (int u = 0; u < kU; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    out[(size_t)blockIdx.x * 512 + threadIdx.x] = acc;
}

// one 16-B element per thread, no loop (grid = n / 256)
__global__ __launch_bounds__(256) void copy11_flat(const uint4* __restrict__ a, uint4* __restrict__ b) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    b[i] = a[i];
}
__global__ __launch_bounds__(256) void copy12_flat(const uint4* __restrict__ a, uint4* __restrict__ b,
                                                    uint4* __restrict__ c) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const uint4 v = a[i];
    b[i] = v;
    c[i] = make_uint4(v.y, v.x, v.w, v.z);
}

int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint4 *a, *b, *c;
    uint32_t* o;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&c, bytes));
    CK(hipMemset(a, 0x5a, bytes));
    CK(hipMemset(b, 0, bytes));
    CK(hipMemset(c, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int k = 0; k < 2; k++) {
        std::vector<float> t;
        for (int r = 0; r < 11; r++) {
            CK(hipEventRecord(e0));
            if (k == 0) hipLaunchKernelGGL(copy11_flat, dim3(n / 256), dim3(256), 0, 0, a, b);
            if (k == 1) hipLaunchKernelGGL(copy12_flat, dim3(n / 256), dim3(256), 0, 0, a, b, c);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[t.size() / 2];
        printf("%s flat (one element per thread): %7.3f ms  %.2f TB/s\n", k ? "copy12" : "copy11", ms,
               (k ? 3.0 : 2.0) * bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    }
    for (int wpc : {2, 4, 8}) {
        const int grid = cus * wpc;
        CK(hipMalloc(&o, (size_t)grid * 512 * 4));
        struct K {
            const char* name;
            double moved;
        } ks[4] = {{"copy11", 2.0 * bytes}, {"copy12", 3.0 * bytes}, {"write", 1.0 * bytes}, {"read", 1.0 * bytes}};
        for (int k = 0; k < 4; k++) {
            std::vector<float> t;
            for (int r = 0; r < 11; r++) {
                CK(hipEventRecord(e0));
                if (k == 0) hipLaunchKernelGGL(copy11, dim3(grid), dim3(512), 0, 0, a, b, n);
                if (k == 1) hipLaunchKernelGGL(copy12, dim3(grid), dim3(512), 0, 0, a, b, c, n);
                if (k == 2) hipLaunchKernelGGL(write_only, dim3(grid), dim3(512), 0, 0, b, n);
                if (k == 3) hipLaunchKernelGGL(read_only, dim3(grid), dim3(512), 0, 0, a, o, n);
                CK(hipGetLastError());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double ms = t[t.size() / 2];
            printf("%-7s workgroups/CU %d: %7.3f ms  %.2f TB/s (read+write at the fabric)\n", ks[k].name, wpc, ms,
                   ks[k].moved / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
        CK(hipFree(o));
    }
    return 0;
}
