// pcie_probe.hip -- host<->device copy paths for the host-buffer C ABI
// (cda_extend_dah / _batch): pageable hipMemcpy, hipHostRegister of the
// caller's buffer (+ the registration cost), and a pinned staging buffer fed by
// host memcpy.  Decides how cda_extend_dah stages host buffers.
// Build: hipcc --offload-arch=gfx950 -O3 -o pcie_probe pcie_probe.hip -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t MB = 1 << 20;
    for (size_t sz : {32 * MB, 256 * MB}) {
        uint8_t* h = (uint8_t*)aligned_alloc(4096, sz);
        memset(h, 1, sz);
        void* d;
        (void)hipMalloc(&d, sz);
        uint8_t* pin;
        (void)hipHostMalloc((void**)&pin, sz, 0);
        memset(pin, 2, sz);
        auto best = [&](auto f) {
            double b = 1e9;
            for (int r = 0; r < 5; r++) {
                double t = now();
                f();
                (void)hipDeviceSynchronize();
                b = std::min(b, now() - t);
            }
            return b;
        };
        double t_pg_h2d = best([&] { (void)hipMemcpy(d, h, sz, hipMemcpyHostToDevice); });
        double t_pg_d2h = best([&] { (void)hipMemcpy(h, d, sz, hipMemcpyDeviceToHost); });
        double t_pin_h2d = best([&] { (void)hipMemcpy(d, pin, sz, hipMemcpyHostToDevice); });
        double t_pin_d2h = best([&] { (void)hipMemcpy(pin, d, sz, hipMemcpyDeviceToHost); });
        double t_reg = best([&] {
            (void)hipHostRegister(h, sz, hipHostRegisterDefault);
            (void)hipHostUnregister(h);
        });
        double t_reg_h2d = best([&] {
            (void)hipHostRegister(h, sz, hipHostRegisterDefault);
            (void)hipMemcpy(d, h, sz, hipMemcpyHostToDevice);
            (void)hipHostUnregister(h);
        });
        double t_reg_d2h = best([&] {
            (void)hipHostRegister(h, sz, hipHostRegisterDefault);
            (void)hipMemcpy(h, d, sz, hipMemcpyDeviceToHost);
            (void)hipHostUnregister(h);
        });
        auto par_memcpy = [&](uint8_t* dst, const uint8_t* src, int nt) {
            std::vector<std::thread> th;
            const size_t per = sz / nt;
            for (int i = 0; i < nt; i++) th.emplace_back([=] { memcpy(dst + i * per, src + i * per, per); });
            for (auto& t : th) t.join();
        };
        double t_memcpy1 = best([&] { memcpy(pin, h, sz); });
        double t_memcpy8 = best([&] { par_memcpy(pin, h, 8); });
        double t_memcpy16 = best([&] { par_memcpy(pin, h, 16); });
        auto gbs = [&](double t) { return sz / t / 1e9; };
        printf("size %zu MiB: pageable H2D %.1f D2H %.1f | pinned H2D %.1f D2H %.1f | register+unregister %.2f ms | "
               "register+H2D %.1f register+D2H %.1f | host memcpy 1T %.1f 8T %.1f 16T %.1f GB/s\n",
               sz / MB, gbs(t_pg_h2d), gbs(t_pg_d2h), gbs(t_pin_h2d), gbs(t_pin_d2h), t_reg * 1e3, gbs(t_reg_h2d),
               gbs(t_reg_d2h), gbs(t_memcpy1), gbs(t_memcpy8), gbs(t_memcpy16));
        (void)hipFree(d);
        (void)hipHostFree(pin);
        free(h);
    }
    return 0;
}
