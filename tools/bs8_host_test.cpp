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
    printf("bs8 host test OK\n");
    return 0;
}
