"""Generates tools/bs16_phase_probe.hip from celestia-app_amd/csrc/rs_gf16_bs.hip:
a copy of rs16_bs_kernel with s_memtime stamps at every phase boundary (after a
volatile fence of all 128 data registers, so no phase's work moves across a
stamp), plus a driver that runs the Q0 job of n k = 512 squares and prints the
mean phase durations (shader clocks) per workgroup round, for the first and the
last wave of each workgroup.  The outputs are unchanged (probe only).
Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I celestia-app_amd/csrc \\
       -o tools/bs16_phase_probe tools/bs16_phase_probe.hip -Lcelestia-app_amd -lcda"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "celestia-app_amd", "csrc", "rs_gf16_bs.hip")).read()
head = src[src.index("// Three workgroups per CU"):src.index("template <int LOGK>\n__global__")]
k0 = src.index("template <int LOGK>\n__global__")
k1 = src.index("template <int LOGK>\nhipError_t launch_bs")
kern = src[k0:k1]
NS = 12
kern = kern.replace("void rs16_bs_kernel(\n    const RsJob job) {",
                    "void rs16_bs_kernel(\n    const RsJob job, unsigned long long* stamps) {\n"
                    f"    unsigned long long ts[{NS}];\n    int ti = 0;\n"
                    "    auto vfence = [&](uint32_t* r) {\n#pragma unroll\n"
                    "        for (int i = 0; i < 128; i++) asm volatile(\"\" : \"+v\"(r[i]));\n    };\n"
                    "    auto stamp = [&]() { unsigned long long t; asm volatile(\"s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)\" : \"=s\"(t) :: \"memory\"); ts[ti++] = t; };\n"
                    "    stamp();")
kern = kern.replace("    bs16::sfor<0, 8, 1>([&](auto uu) { bs16::block_planes(R + 16 * decltype(uu)::value); });",
                    "    bs16::sfor<0, 8, 1>([&](auto uu) { bs16::block_planes(R + 16 * decltype(uu)::value); });\n"
                    "    vfence(R);\n    stamp();", 1)
marks = ["    bs16::phase_low_ifft<LOGK>(R, m, w);\n"]
kern = kern.replace(marks[0], marks[0] + "    vfence(R);\n    stamp();\n", 1)
body = re.search(r"\n    x12\(false\);.*?bs16::phase_low_fft<LOGK>\(R, m, w\);", kern, re.S).group(0)
new = ""
for line in body.strip("\n").split("\n"):
    new += "\n" + line + "\n    vfence(R);\n    stamp();"
kern = kern.replace(body, new)
# -DNOMEM: no global loads / stores (synthetic registers), to separate compute + exchanges from memory
kern = kern.replace("        const u32x4* p = reinterpret_cast<const u32x4*>(src + o + ls);\n#pragma unroll\n        for (int q = 0; q < 4; q++) {\n            const u32x4 v = p[q];",
                    "        const u32x4* p = reinterpret_cast<const u32x4*>(src + o + ls);\n#pragma unroll\n        for (int q = 0; q < 4; q++) {\n#ifdef NOMEM\n            const u32x4 v = u32x4{o + q, ls ^ q, tid * 7u + u, o * 3u};\n#else\n            const u32x4 v = p[q];\n#endif")
kern = kern.replace("        u32x4* p = reinterpret_cast<u32x4*>(E + o + ld);\n#pragma unroll\n        for (int q = 0; q < 4; q++)\n            p[q] =",
                    "        u32x4* p = reinterpret_cast<u32x4*>(E + o + ld);\n#pragma unroll\n        for (int q = 0; q < 4; q++)\n#ifdef NOMEM\n            if (R[16 * u + 4 * q] == 0x12345678u && R[16 * u + 4 * q + 1] == 0x9abcdef0u) p[q] =\n#else\n            p[q] =\n#endif\n               ")
assert "NOMEM" in kern and kern.count("#ifdef NOMEM") == 2, kern.count("#ifdef NOMEM")
kern = kern.rstrip()
assert kern.endswith("}")
kern = kern[:-1] + (f"    stamp();\n    if ((threadIdx.x & 63) == 0 && (threadIdx.x == 0 || threadIdx.x + 64 == blockDim.x))\n"
                    f"        for (int i = 0; i < {NS}; i++) stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * {2 * NS} + (threadIdx.x ? {NS} : 0) + i] = ts[i];\n}}\n")
drv = r'''
}  // namespace
}  // namespace cda
using namespace cda;
constexpr int NS = NSVAL;
int main(int argc, char** argv) {
    const uint32_t k = 512, n = argc > 1 ? atoi(argv[1]) : 4;
    const size_t W = 2 * k, sq = W * W * 512;
    uint8_t* eds;
    if (hipMalloc(&eds, n * sq) != hipSuccess) return 1;
    (void)hipMemset(eds, 0x5A, n * sq);
    RsJob j = square_job_q0_inplace(eds, k);
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0), nwg = 2 * ncw * n;
    unsigned long long* st;
    (void)hipMalloc(&st, (size_t)nwg * NSx2 * 8);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_bs_kernel<9>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs16_lds_bytes<9>());
    for (int rep = 0; rep < 3; rep++) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(rs16_bs_kernel<9>, dim3(2 * ncw, n), dim3(256), bs16_lds_bytes<9>(), 0, j, st);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("rep %d: %u codewords in %.3f ms\n", rep, ncw * n, ms);
    }
    std::vector<unsigned long long> h((size_t)nwg * NSx2);
    (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    const char* names[NS - 1] = {"load+planes", "LOW ifft", "X12", "M1 ifft", "X23", "M2", "X32", "M1 fft", "X21", "LOW fft", "planes+store"};
    const size_t per_round = 512, rounds = (nwg + per_round - 1) / per_round;
    for (size_t r = 0; r < rounds && r < 8; r++) {
        double sum[2][NS - 1] = {}, tot = 0; int cnt = 0;
        for (size_t i = r * per_round; i < std::min((size_t)nwg, (r + 1) * per_round); i++) {
            for (int wv = 0; wv < 2; wv++)
                for (int p = 0; p < NS - 1; p++) sum[wv][p] += (double)(h[i * NSx2 + wv * NS + p + 1] - h[i * NSx2 + wv * NS + p]);
            tot += (double)(h[i * NSx2 + NS - 1] - h[i * NSx2]); cnt++;
        }
        printf("round %zu: %d WGs, mean total %.0f clocks\n", r, cnt, tot / cnt);
        for (int wv = 0; wv < 2; wv++) {
            printf("  wave %s:", wv ? "last" : "0");
            for (int p = 0; p < NS - 1; p++) printf(" %s %.0f |", names[p], sum[wv][p] / cnt);
            printf("\n");
        }
    }
    return 0;
}
'''.replace("NSx2", str(2 * NS)).replace("NSVAL", str(NS)).replace("NS - 1", str(NS - 1)).replace("[NS - 1]", f"[{NS - 1}]")
out = ("// bs16_phase_probe.hip -- GENERATED by tools/gen_bs16_phase_probe.py from rs_gf16_bs.hip (see there).\n"
       "#include <hip/hip_runtime.h>\n#include <algorithm>\n#include <cstdio>\n#include <cstdlib>\n#include <vector>\n"
       "#include \"bitslice16.h\"\n#include \"cda_kernels.h\"\nnamespace cda {\nnamespace {\n" + head + kern + drv)
out = out.replace("NS]", f"{NS}]").replace("NS;", f"{NS};")
open(os.path.join(ROOT, "tools", "bs16_phase_probe.hip"), "w").write(out)
