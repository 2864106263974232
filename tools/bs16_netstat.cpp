// bs16_netstat.cpp -- the GF(2) matrices of every butterfly network of the
// bitsliced k = 512 encoder (bitslice16.h layer8), one line per butterfly:
//   <phase> <layer> <butterfly> <kind>:<16 row masks in hex> ...
// kind: B = base constant (compile-time part), L = masked lane term, W =
// uniform wave term.  Input for tools/bs16_cse.py (network op counts under
// different signal-sharing schemes).
// Build: g++ -O2 -std=c++20 -I celestia-app_amd/csrc tools/bs16_netstat.cpp -o /tmp/bs16_netstat
#include <cstdio>

#include "bitslice16.h"

using namespace cda::bs16;

static void dump(const char* kind, uint32_t c) {
    const Net n = make_net(c);
    printf(" %s:", kind);
    for (int i = 0; i < 16; i++) printf("%04x%s", n.row[i], i < 15 ? "," : "");
}

template <int LOGK, bool INV>
static void layer(const char* ph, int b, int D, int SH, int NL, int LB, int NWB, int WB) {
    for (int i = 0; i < 8; i++) {
        if (i & D) continue;
        printf("%s %d %d", ph, b, i);
        dump("B", skew_part<INV, LOGK>(b, (uint32_t)(i & ~(2 * D - 1)) << SH));
        for (int l = 0; l < NL; l++) dump("L", tbasis(b, LB + l));
        for (int w = 0; w < NWB; w++) dump("W", tbasis(b, WB + w));
        printf("\n");
    }
}

int main() {
    constexpr int K = 9;
    for (int b = 0; b < 3; b++) layer<K, true>("low_ifft", b, 1 << b, 0, 4, 3, K - 7, 7);
    for (int b = 3; b < 6; b++) layer<K, true>("m1_ifft", b, 1 << (b - 3), 3, 1, 6, K - 7, 7);
    for (int b = 6; b < K; b++) layer<K, true>("m2_ifft", b, 1 << (b - (K - 3)), K - 3, 0, 0, 0, 0);
    for (int b = K - 1; b >= K - 3; b--) layer<K, false>("m2_fft", b, 1 << (b - (K - 3)), K - 3, 0, 0, 0, 0);
    for (int b = K - 4; b >= 3; b--) layer<K, false>("m1_fft", b, 1 << (b - 3), 3, 1, 6, K - 7, 7);
    for (int b = 2; b >= 0; b--) layer<K, false>("low_fft", b, 1 << b, 0, 4, 3, K - 7, 7);
    return 0;
}
