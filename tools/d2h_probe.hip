// d2h_probe.hip -- device-to-host copy shapes of the host-buffer pipeline
// (engine.hip host_pipeline / enqueue_parity_d2h): the three parity quadrants
// of k = 128 squares into page-locked host EDS buffers, as (a) one linear copy
// of the same byte count, (b) per square a 2-D copy of Q1 + a linear copy of
// Q2|Q3 (the library's form), (c) (b) with Q1 and Q2|Q3 on two streams, (d)
// (b) beside an H2D stream of the ODS, (e) (b) beside host threads copying Q0.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/d2h_probe tools/d2h_probe.hip -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t k = 128, W = 2 * k, SH = 512, n = 128;
    const size_t sq = W * W * SH, half = k * W * SH, ods = k * k * SH;
    uint8_t *d, *dods, *h, *hods;
    if (hipMalloc(&d, n * sq) != hipSuccess || hipMalloc(&dods, n * ods) != hipSuccess) return 1;
    if (hipHostMalloc((void**)&h, n * sq, 0) != hipSuccess || hipHostMalloc((void**)&hods, n * ods, 0) != hipSuccess) return 1;
    memset(h, 1, n * sq);
    memset(hods, 2, n * ods);
    (void)hipMemset(d, 3, n * sq);
    hipStream_t a, b, c;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&c, hipStreamNonBlocking);
    const double par = (double)n * 3 * ods;
    auto parity = [&](hipStream_t s1, hipStream_t s2) {
        for (size_t i = 0; i < n; i++) {
            (void)hipMemcpy2DAsync(h + i * sq + k * SH, W * SH, d + i * sq + k * SH, W * SH, k * SH, k,
                                   hipMemcpyDeviceToHost, s1);
            (void)hipMemcpyAsync(h + i * sq + half, d + i * sq + half, half, hipMemcpyDeviceToHost, s2);
        }
    };
    auto run = [&](const char* name, auto f) {
        f();
        (void)hipDeviceSynchronize();
        double best = 1e9;
        for (int r = 0; r < 3; r++) {
            const double t0 = now();
            f();
            (void)hipDeviceSynchronize();
            best = std::min(best, now() - t0);
        }
        printf("%-48s %7.1f ms  %6.1f GB/s (parity bytes)\n", name, best * 1e3, par / best / 1e9);
    };
    run("(a) one linear copy of the parity byte count", [&] {
        (void)hipMemcpyAsync(h, d, (size_t)par, hipMemcpyDeviceToHost, a);
    });
    run("(a2) 128 linear copies of 24 MiB", [&] {
        for (size_t i = 0; i < n; i++) (void)hipMemcpyAsync(h + i * sq, d + i * sq, 3 * ods, hipMemcpyDeviceToHost, a);
    });
    run("(b) per square 2-D Q1 + linear Q2|Q3, one stream", [&] { parity(a, a); });
    run("(b2) only the 2-D Q1 copies", [&] {
        for (size_t i = 0; i < n; i++)
            (void)hipMemcpy2DAsync(h + i * sq + k * SH, W * SH, d + i * sq + k * SH, W * SH, k * SH, k,
                                   hipMemcpyDeviceToHost, a);
    });
    run("(c) Q1 and Q2|Q3 on two streams", [&] { parity(a, b); });
    run("(d) (b) beside the ODS H2D on a second stream", [&] {
        (void)hipMemcpyAsync(dods, hods, n * ods, hipMemcpyHostToDevice, c);
        parity(a, a);
    });
    run("(e) (b) beside 8 host threads copying Q0", [&] {
        parity(a, a);
        std::vector<std::thread> th;
        for (int t = 0; t < 8; t++)
            th.emplace_back([&, t] {
                for (size_t i = t; i < n * k; i += 8) {
                    const size_t s = i / k, r = i % k;
                    memcpy(h + s * sq + r * W * SH, hods + i * k * SH, k * SH);
                }
            });
        for (auto& x : th) x.join();
    });
    return 0;
}
