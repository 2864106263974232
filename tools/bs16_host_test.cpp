// Host check of the constexpr GF(2^16) Leopard arithmetic (celestia-app_amd/csrc/bitslice16.h)
// against the table build leo_build<16> (leopard_tables.h): field products, the
// whole skew vector, the networks, the signal plans (make_plan) and the block <-> planes transpose.
// Build: g++ -O2 -std=c++20 -I celestia-app_amd/csrc tools/bs16_host_test.cpp -o /tmp/bs16_host_test
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "bitslice16.h"

using namespace cda;

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)rng;
}

// scalar leopard encode of one codeword (K shards x 512 B, lo/hi symbol layout)
template <int K>
static void scalar_encode(const LeoField<16>& F, const uint8_t* data, uint8_t* parity) {
    std::vector<uint32_t> w(K);
    for (int blk = 0; blk < 8; blk++)
        for (int sy = 0; sy < 32; sy++) {
            for (int i = 0; i < K; i++) w[i] = data[i * 512 + 64 * blk + sy] | (uint32_t)data[i * 512 + 64 * blk + 32 + sy] << 8;
            for (int d = 1; d < K; d <<= 1)
                for (int g = 0; g < K; g += 2 * d) {
                    const uint32_t L = F.skew[K - 1 + g + d];
                    for (int i = g; i < g + d; i++) {
                        w[i + d] ^= w[i];
                        if (L != LeoField<16>::MOD) w[i] ^= F.mul_log(w[i + d], L);
                    }
                }
            for (int d = K / 2; d >= 1; d >>= 1)
                for (int g = 0; g < K; g += 2 * d) {
                    const uint32_t L = F.skew[g + d - 1];
                    for (int i = g; i < g + d; i++) {
                        if (L != LeoField<16>::MOD) w[i] ^= F.mul_log(w[i + d], L);
                        w[i + d] ^= w[i];
                    }
                }
            for (int i = 0; i < K; i++) {
                parity[i * 512 + 64 * blk + sy] = (uint8_t)w[i];
                parity[i * 512 + 64 * blk + 32 + sy] = (uint8_t)(w[i] >> 8);
            }
        }
}

// the kernel's schedule (rs_gf16_bs.hip) with every (half, wave, lane) emulated
template <int LOGK>
static void bs_encode(const uint8_t* data, uint8_t* parity) {
    constexpr int NW = 1 << (LOGK - 7);
    constexpr int NL = 2 * NW * 64;   // (half, wave, lane) slots
    std::vector<uint32_t> R((size_t)NL * 128), T(R.size());
    auto at = [&](std::vector<uint32_t>& v, int h, int w, int lane) {
        return v.data() + (((size_t)h * NW + w) * 64 + lane) * 128;
    };
    auto masks = [](int lane, uint32_t* m) {
        for (int i = 0; i < 4; i++) m[i] = 0u - (((lane >> 2) >> i) & 1);
    };
    auto low_s = [](int w, int lane, int u) { return w << 7 | (lane >> 2) << 3 | u; };
    auto m1_s = [](int w, int lane, int u) { const int jl = lane >> 2; return w << 7 | (jl >> 3) << 6 | u << 3 | (jl & 7); };
    auto m2_s = [](int w, int lane, int u) { return u << (LOGK - 3) | w << 4 | (lane >> 2); };
    // move every unit from layout A to layout B (through "LDS": keyed by shard and block)
    auto relayout = [&](auto from, auto to) {
        std::vector<int> where((size_t)2 * (1 << LOGK) * 4 * 0 + 1);
        for (int h = 0; h < 2; h++)
            for (int w = 0; w < NW; w++)
                for (int lane = 0; lane < 64; lane++)
                    for (int u = 0; u < 8; u++) {
                        const int s = from(w, lane, u);
                        // find the destination (w2, lane2, u2) with to(...) == s and the same block
                        for (int w2 = 0; w2 < NW; w2++)
                            for (int l2 = (lane & 3); l2 < 64; l2 += 4)
                                for (int u2 = 0; u2 < 8; u2++)
                                    if (to(w2, l2, u2) == s) memcpy(at(T, h, w2, l2) + 16 * u2, at(R, h, w, lane) + 16 * u, 64);
                    }
        R.swap(T);
    };
    for (int h = 0; h < 2; h++)
        for (int w = 0; w < NW; w++)
            for (int lane = 0; lane < 64; lane++) {
                const int blk = 4 * h + (lane & 3);
                for (int u = 0; u < 8; u++) {
                    memcpy(at(R, h, w, lane) + 16 * u, data + (size_t)low_s(w, lane, u) * 512 + 64 * blk, 64);
                    bs16::block_planes(at(R, h, w, lane) + 16 * u);
                }
                uint32_t m[4];
                masks(lane, m);
                bs16::phase_low_ifft<LOGK>(at(R, h, w, lane), m, w);
            }
    relayout(low_s, m1_s);
    for (int h = 0; h < 2; h++)
        for (int w = 0; w < NW; w++)
            for (int lane = 0; lane < 64; lane++) {
                uint32_t m[4];
                masks(lane, m);
                bs16::phase_m1_ifft<LOGK>(at(R, h, w, lane), m, w);
            }
    relayout(m1_s, m2_s);
    for (int h = 0; h < 2; h++)
        for (int w = 0; w < NW; w++)
            for (int lane = 0; lane < 64; lane++) bs16::phase_m2<LOGK>(at(R, h, w, lane));
    relayout(m2_s, m1_s);
    for (int h = 0; h < 2; h++)
        for (int w = 0; w < NW; w++)
            for (int lane = 0; lane < 64; lane++) {
                uint32_t m[4];
                masks(lane, m);
                bs16::phase_m1_fft<LOGK>(at(R, h, w, lane), m, w);
            }
    relayout(m1_s, low_s);
    for (int h = 0; h < 2; h++)
        for (int w = 0; w < NW; w++)
            for (int lane = 0; lane < 64; lane++) {
                uint32_t m[4];
                masks(lane, m);
                bs16::phase_low_fft<LOGK>(at(R, h, w, lane), m, w);
                const int blk = 4 * h + (lane & 3);
                for (int u = 0; u < 8; u++) {
                    bs16::block_planes(at(R, h, w, lane) + 16 * u);
                    memcpy(parity + (size_t)low_s(w, lane, u) * 512 + 64 * blk, at(R, h, w, lane) + 16 * u, 64);
                }
            }
}

template <int LOGK>
static int check_encode(const LeoField<16>& F) {
    constexpr int K = 1 << LOGK;
    std::vector<uint8_t> data((size_t)K * 512), want(data.size()), got(data.size());
    for (auto& b : data) b = (uint8_t)rnd();
    scalar_encode<K>(F, data.data(), want.data());
    bs_encode<LOGK>(data.data(), got.data());
    size_t diff = 0;
    for (size_t i = 0; i < got.size(); i++) diff += got[i] != want[i];
    printf("bitsliced schedule k=%d: %zu differing parity bytes\n", K, diff);
    return diff ? 1 : 0;
}

int main() {
    auto F = std::make_unique<LeoField<16>>();
    leo_build<16>(*F, 0x1002D, kCantor16);
    int bad = 0;
    // products
    for (int t = 0; t < 200000; t++) {
        const uint32_t a = rnd() & 0xFFFF, b = rnd() & 0xFFFF;
        const uint32_t want = b == 0 ? 0 : F->mul_log(a, F->log[b]);
        if (bs16::fmul(a, b) != want) {
            if (bad++ < 5) printf("fmul(%04x,%04x) = %04x want %04x\n", a, b, bs16::fmul(a, b), want);
        }
    }
    // skew vector (logs in the table; modulus = multiply by zero)
    for (uint32_t j = 0; j < 65535; j++) {
        const uint32_t L = F->skew[j];
        const uint32_t want = L == LeoField<16>::MOD ? 0 : F->exp[L];
        if (bs16::skew_value(j) != want) {
            if (bad++ < 10) printf("skew[%u] = %04x want %04x (log %u)\n", j, bs16::skew_value(j), want, L);
        }
    }
    // networks: c*y through the planes of 32 random symbols
    for (int t = 0; t < 64; t++) {
        const uint32_t j = rnd() % 1023;
        const uint32_t c = bs16::skew_value(j);
        const bs16::Net n = bs16::make_net(c);
        for (int s = 0; s < 64; s++) {
            const uint32_t y = rnd() & 0xFFFF;
            uint32_t got = 0;
            for (int i = 0; i < 16; i++) got |= (uint32_t)(__builtin_popcount(n.row[i] & y) & 1) << i;
            const uint32_t want = c == 0 ? 0 : F->mul_log(y, F->log[c]);
            if (got != want && bad++ < 15) printf("net c=%04x y=%04x: %04x want %04x\n", c, y, got, want);
        }
    }
    // block <-> planes: plane p bit (8q + w) == bit p of symbol 4w + q (lo) / bit p-8 of its hi byte
    {
        uint8_t blk[64];
        for (int i = 0; i < 64; i++) blk[i] = (uint8_t)rnd();
        uint32_t r[16];
        memcpy(r, blk, 64);
        bs16::block_planes(r);
        for (int p = 0; p < 16; p++)
            for (int w = 0; w < 8; w++)
                for (int q = 0; q < 4; q++) {
                    const int sym = 4 * w + q;
                    const uint32_t v = blk[sym] | (uint32_t)blk[sym + 32] << 8;
                    if (((r[p] >> (8 * q + w)) & 1) != ((v >> p) & 1) && bad++ < 20)
                        printf("planes: p %d sym %d\n", p, sym);
                }
        bs16::block_planes(r);
        if (memcmp(r, blk, 64) != 0 && bad++ < 20) printf("block_planes is not self-inverse\n");
    }
    // linearity of the skew in the group position (bitslice16.h skew_part / tbasis)
    for (int b = 0; b < 9; b++)
        for (uint32_t g = 0; g < 512; g += 2u << b) {
            const uint32_t d = 1u << b;
            if (bs16::skew_part<true, 9>(b, g) != bs16::skew_value(511 + g + d) && bad++ < 30)
                printf("ifft skew_part b %d g %u\n", b, g);
            if (bs16::skew_part<false, 9>(b, g) != bs16::skew_value(g + d - 1) && bad++ < 30)
                printf("fft skew_part b %d g %u\n", b, g);
        }
    for (int b = 0; b < 8; b++)
        for (uint32_t g = 0; g < 256; g += 2u << b) {
            const uint32_t d = 1u << b;
            if (bs16::skew_part<true, 8>(b, g) != bs16::skew_value(255 + g + d) && bad++ < 30)
                printf("ifft k256 skew_part b %d g %u\n", b, g);
        }
    // signal plans (make_plan): every derived signal reads only earlier
    // signals, and each planned row, expanded back over the 16 planes, is the
    // network row it replaces (base, masked lane and wave matrices)
    int plan_sigs = 0;
    for (int t = 0; t < 256; t++) {
        uint32_t tl[4], tw[2];
        for (auto& v : tl) v = bs16::skew_value(rnd() % 1023);
        for (auto& v : tw) v = bs16::skew_value(rnd() % 1023);
        const uint32_t c0 = bs16::skew_value(rnd() % 1023);
        const int nl = t % 5, nw = (t / 5) % 3;
        const bs16::SigPlan P = bs16::make_plan(c0, tl, nl, tw, nw);
        plan_sigs += P.n;
        uint32_t sig[48];   // signal -> mask over the 16 planes
        for (int i = 0; i < 16; i++) sig[i] = 1u << i;
        for (int s = 0; s < P.n; s++) {
            const int id = 16 + s;
            if (P.a[s] >= id || P.b[s] >= id || (P.c[s] != 0xFF && P.c[s] >= id)) {
                if (bad++ < 40) printf("plan signal %d reads a later signal\n", id);
                sig[id] = 0;
                continue;
            }
            sig[id] = sig[P.a[s]] ^ sig[P.b[s]] ^ (P.c[s] != 0xFF ? sig[P.c[s]] : 0u);
        }
        auto expand = [&](uint32_t row) {
            uint32_t m = 0;
            for (; row; row &= row - 1) m ^= sig[__builtin_ctz(row)];
            return m;
        };
        auto check = [&](const char* what, uint32_t c, const uint32_t* rows) {
            const bs16::Net n = bs16::make_net(c);
            for (int i = 0; i < 16; i++)
                if (expand(rows[i]) != n.row[i] && bad++ < 40)
                    printf("plan %s row %d c=%04x: %04x want %04x\n", what, i, c, expand(rows[i]), n.row[i]);
        };
        check("base", c0, P.base);
        for (int l = 0; l < nl; l++) check("lane", tl[l], P.lane[l]);
        for (int w = 0; w < nw; w++) check("wave", tw[w], P.wave[w]);
    }
    printf("signal plans: 256 checked, %.1f derived signals each\n", plan_sigs / 256.0);
    bad += check_encode<9>(*F);
    bad += check_encode<8>(*F);
    printf("%s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
    return bad ? 1 : 0;
}
