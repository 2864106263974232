// Host check of the bitsliced GF(2^8) encode core (celestia-app_amd/csrc/bitslice8.h):
// runs passes A/B/C with the kernel's register layouts and exchanges emulated on
// the CPU and compares with a scalar Leopard encoder (same tables).
// Build: g++ -O2 -std=c++20 -I celestia-app_amd/csrc tools/bs8_host_test.cpp -o /tmp/bs8_host_test
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bitslice8.h"

using namespace cda;
using namespace cda::bs8;

static void scalar_encode(std::vector<uint8_t>& w) {   // w[K] symbols -> parity in place
    const int m = K;
    for (int d = 1; d < m; d <<= 1)
        for (int g = 0; g < m; g += 2 * d) {
            const uint32_t L = kField.skew[m - 1 + g + d];
            for (int i = g; i < g + d; i++) {
                w[i + d] ^= w[i];
                if (L != kMod) w[i] ^= kField.mul_log(w[i + d], L);
            }
        }
    for (int d = m / 2; d >= 1; d >>= 1)
        for (int g = 0; g < m; g += 2 * d) {
            const uint32_t L = kField.skew[g + d - 1];
            for (int i = g; i < g + d; i++) {
                if (L != kMod) w[i] ^= kField.mul_log(w[i + d], L);
                w[i + d] ^= w[i];
            }
        }
}

int main() {
    // transpose8 is an involution and maps bit j of byte q of r[i] to bit i of byte q of r[j]
    uint32_t r[8], o[8];
    for (int i = 0; i < 8; i++) r[i] = o[i] = 0x9E3779B9u * (i + 1) ^ 0x7F4A7C15u;
    transpose8(r);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            for (int q = 0; q < 4; q++)
                if (((r[i] >> (8 * q + j)) & 1) != ((o[j] >> (8 * q + i)) & 1)) { printf("transpose FAIL\n"); return 1; }
    transpose8(r);
    if (memcmp(r, o, sizeof r)) { printf("involution FAIL\n"); return 1; }

    // one column group: 32 columns x 128 shards
    std::vector<uint8_t> data(K * 32);
    srand(1);
    for (auto& b : data) b = rand() & 0xFF;
    std::vector<uint8_t> expect(K * 32);
    for (int c = 0; c < 32; c++) {
        std::vector<uint8_t> w(K);
        for (int s = 0; s < K; s++) w[s] = data[s * 32 + c];
        scalar_encode(w);
        for (int s = 0; s < K; s++) expect[s * 32 + c] = w[s];
    }
    // pass A: 8 "waves" u, each R[8t+p] for shard 16u+t
    uint32_t A[8][128];
    for (int u = 0; u < 8; u++) {
        for (int t = 0; t < 16; t++) {
            memcpy(&A[u][8 * t], &data[(16 * u + t) * 32], 32);
            transpose8(&A[u][8 * t]);
        }
        with_u(u, [&](auto U) { pass_a<decltype(U)::value>(A[u]); });
    }
    // exchange A -> B: wave w unit r holds t = 8r + w, R[64r + 8u + p]
    uint32_t B[8][128];
    for (int w = 0; w < 8; w++)
        for (int rr = 0; rr < 2; rr++)
            for (int u = 0; u < 8; u++)
                for (int p = 0; p < 8; p++) B[w][64 * rr + 8 * u + p] = A[u][8 * (8 * rr + w) + p];
    for (int w = 0; w < 8; w++) { pass_b(B[w]); pass_b(B[w] + 64); }
    for (int w = 0; w < 8; w++)
        for (int rr = 0; rr < 2; rr++)
            for (int u = 0; u < 8; u++)
                for (int p = 0; p < 8; p++) A[u][8 * (8 * rr + w) + p] = B[w][64 * rr + 8 * u + p];
    std::vector<uint8_t> got(K * 32);
    for (int u = 0; u < 8; u++) {
        with_u(u, [&](auto U) { pass_c<decltype(U)::value>(A[u]); });
        for (int t = 0; t < 16; t++) {
            transpose8(&A[u][8 * t]);
            memcpy(&got[(16 * u + t) * 32], &A[u][8 * t], 32);
        }
    }
    if (got != expect) { printf("encode FAIL\n"); return 1; }

    // half layout (rs8_bs_half_kernel): lane (u, h) holds shards 16u + 2j + h in
    // H[u][h][8j + p]; the d = 1 steps see the partner lane's planes as P
    uint32_t H[8][2][64];
    const uint32_t hm[2] = {0xFFFFFFFFu, 0u};
    auto cross = [&](int u, int j, auto step) {   // both lanes read the other's pre-step planes
        uint32_t P0[8], P1[8];
        memcpy(P0, &H[u][1][8 * j], 32);
        memcpy(P1, &H[u][0][8 * j], 32);
        step(&H[u][0][8 * j], P0, hm[0]);
        step(&H[u][1][8 * j], P1, hm[1]);
    };
    for (int u = 0; u < 8; u++) {
        for (int h = 0; h < 2; h++)
            for (int j = 0; j < 8; j++) {
                memcpy(&H[u][h][8 * j], &data[(16 * u + 2 * j + h) * 32], 32);
                transpose8(&H[u][h][8 * j]);
            }
        with_u(u, [&](auto U) {
            constexpr int UU = decltype(U)::value;
            sfor<0, 8, 1>([&](auto jj) {
                constexpr int j = decltype(jj)::value;
                cross(u, j, [](uint32_t* x, const uint32_t* P, uint32_t h0) { ifft_d1<ifft_d1_log<UU>(j)>(x, P, h0); });
            });
            for (int h = 0; h < 2; h++) pass_a_hi<UU>(H[u][h]);
        });
    }
    // A -> B: lane (w, h) gets shards 16u + 2w + h of every u in R[8u + p]
    uint32_t HB[8][2][64];
    for (int w = 0; w < 8; w++)
        for (int h = 0; h < 2; h++) {
            for (int u = 0; u < 8; u++) memcpy(&HB[w][h][8 * u], &H[u][h][8 * w], 32);
            pass_b(HB[w][h]);
        }
    for (int w = 0; w < 8; w++)
        for (int h = 0; h < 2; h++)
            for (int u = 0; u < 8; u++) memcpy(&H[u][h][8 * w], &HB[w][h][8 * u], 32);
    std::vector<uint8_t> got2(K * 32);
    for (int u = 0; u < 8; u++) {
        with_u(u, [&](auto U) {
            constexpr int UU = decltype(U)::value;
            for (int h = 0; h < 2; h++) pass_c_hi<UU>(H[u][h]);
            sfor<0, 8, 1>([&](auto jj) {
                constexpr int j = decltype(jj)::value;
                cross(u, j, [](uint32_t* x, const uint32_t* P, uint32_t h0) { fft_d1<fft_d1_log<UU>(j)>(x, P, h0); });
            });
        });
        for (int h = 0; h < 2; h++)
            for (int j = 0; j < 8; j++) {
                transpose8(&H[u][h][8 * j]);
                memcpy(&got2[(16 * u + 2 * j + h) * 32], &H[u][h][8 * j], 32);
            }
    }
    if (got2 != expect) { printf("half-layout encode FAIL\n"); return 1; }
    printf("bs8 host test OK\n");
    return 0;
}
