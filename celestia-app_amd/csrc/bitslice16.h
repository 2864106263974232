// bitslice16.h -- bitsliced GF(2^16) Leopard arithmetic (host + device).
//
// Restates the field and FFT skew of klauspost/reedsolomon v1.12.1 leopard.go
// (initLUTs: LFSR over 0x1002D + Cantor-basis conversion; initFFT: the skew
// vector) -- EXT module pinned at /root/reference/go.mod:152, reached through
// pkg/appconsts/global_consts.go:92 -> rsmt2d LeoRSCodec.Encode for squares
// wider than 128 -- as constexpr functions, so every butterfly constant of the
// k = 256 / 512 schedules is a compile-time XOR network:
//   * a 32-bit register holds bit p ("plane p") of 32 symbols; a unit is the
//     16 planes of the 32 symbols of one 64-byte block of one shard (symbol s
//     = b[s] | b[s + 32] << 8, leopard.go's lo/hi split layout);
//   * GF addition is one XOR per plane, and multiplication by a constant c is
//     the 16x16 GF(2) matrix of y -> c*y: plane i of c*y is the XOR of the
//     planes j of y with bit i of c*(1<<j) set.
// No tables: Leopard's element a is the polynomial-basis element C(a) = XOR of
// kCantor16[i] over the set bits i of a (initLUTs builds log[a] as the LFSR
// exponent of C(a)), so a*b = C^-1(C(a) (x) C(b)) with (x) the carry-less
// product mod 0x1002D.  The skew vector's field values are XOR sums of the
// initFFT "temp" elements (see skew_value); leopard_tables.h leo_build<16>
// builds the same vector as logs, and tests/test_bitslice16 checks the two
// agree entry by entry.
#pragma once
#include <stdint.h>

#include <type_traits>

#include "leopard_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define B16_HD __host__ __device__ __forceinline__
#else
#define B16_HD inline
#endif

namespace cda {
namespace bs16 {

constexpr uint32_t kPoly = 0x1002D;
constexpr uint32_t kMod = 65535;

// carry-less a*b mod 0x1002D (polynomial basis)
constexpr uint32_t pmul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 16; i++)
        if ((b >> i) & 1) r ^= a << i;
    for (int i = 31; i >= 16; i--)
        if ((r >> i) & 1) r ^= kPoly << (i - 16);
    return r;
}
constexpr uint32_t to_poly(uint32_t a) {
    uint32_t r = 0;
    for (int i = 0; i < 16; i++)
        if ((a >> i) & 1) r ^= kCantor16[i];
    return r;
}
// C^-1 as 16 basis images, by Gauss-Jordan elimination over GF(2)
struct InvBasis {
    uint32_t col[16];   // from_poly(1 << j)
};
constexpr InvBasis make_inv_basis() {
    uint32_t row[16] = {}, aug[16] = {};   // row i: kCantor16[i] (as a poly), aug: 1 << i
    for (int i = 0; i < 16; i++) {
        row[i] = kCantor16[i];
        aug[i] = 1u << i;
    }
    // reduce so that row[j] == 1 << j
    for (int b = 0; b < 16; b++) {
        int piv = -1;
        for (int i = b; i < 16; i++)
            if ((row[i] >> b) & 1) {
                piv = i;
                break;
            }
        if (piv < 0) return InvBasis{};   // singular (never for a Cantor basis)
        uint32_t t = row[b];
        row[b] = row[piv];
        row[piv] = t;
        t = aug[b];
        aug[b] = aug[piv];
        aug[piv] = t;
        for (int i = 0; i < 16; i++)
            if (i != b && ((row[i] >> b) & 1)) {
                row[i] ^= row[b];
                aug[i] ^= aug[b];
            }
    }
    InvBasis r{};
    for (int j = 0; j < 16; j++) r.col[j] = aug[j];   // to_poly(aug[j]) == 1 << j
    return r;
}
inline constexpr InvBasis kInvBasis = make_inv_basis();
constexpr uint32_t from_poly(uint32_t p) {
    uint32_t r = 0;
    for (int j = 0; j < 16; j++)
        if ((p >> j) & 1) r ^= kInvBasis.col[j];
    return r;
}
// Leopard field product of two elements (leopard.go mulLog on values)
constexpr uint32_t fmul(uint32_t a, uint32_t b) { return from_poly(pmul(to_poly(a), to_poly(b))); }
constexpr uint32_t finv(uint32_t a) {   // a^(2^16 - 2)
    uint32_t p = to_poly(a), r = 1, e = 65534;
    while (e) {
        if (e & 1) r = pmul(r, p);
        p = pmul(p, p);
        e >>= 1;
    }
    return from_poly(r);
}

// initFFT's temp vector, level by level: kTemp.t[m][i] (i >= m) is temp[i]
// as a field element during level m's skew fill.  Level m then turns temp[m]
// into log(1 / (T (T ^ 1))) (T = temp[m]) and multiplies every later temp[i]
// by (temp[i] ^ 1) and by that inverse.  (leopard.go uses log[0] = modulus,
// which acts as a factor of 1; no temp value is 0 or 1 for this basis, which
// kTempOk checks, so the plain field form is exact.)
struct Temps {
    uint32_t t[15][15];
    bool ok;
};
constexpr Temps make_temps() {
    Temps T{};
    T.ok = true;
    uint32_t cur[15] = {};
    for (int i = 1; i < 16; i++) cur[i - 1] = 1u << i;
    for (int m = 0; m < 15; m++) {
        for (int i = 0; i < 15; i++) T.t[m][i] = cur[i];
        const uint32_t Tm = cur[m];
        if (Tm == 0 || Tm == 1) T.ok = false;
        const uint32_t inv = finv(fmul(Tm, Tm ^ 1));
        for (int i = m + 1; i < 15; i++) {
            if (cur[i] == 0 || cur[i] == 1) T.ok = false;
            cur[i] = fmul(fmul(cur[i], cur[i] ^ 1), inv);
        }
    }
    return T;
}
inline constexpr Temps kTemps = make_temps();
static_assert(kTemps.ok, "initFFT temp vector hit 0 or 1: the plain field form would differ from leopard.go");

// Field value of the skew vector entry j (0 == "multiply by zero", i.e. the
// log table's modulus).  Entry j belongs to level m = number of trailing ones
// of j, and equals the XOR of temp[i] (level m) over the set bits i + 1 of j
// above bit m.
constexpr uint32_t skew_value(uint32_t j) {
    int m = 0;
    while ((j >> m) & 1) m++;
    if (m >= 15) return 0;
    uint32_t v = 0;
    for (int i = m; i < 15; i++)
        if ((j >> (i + 1)) & 1) v ^= kTemps.t[m][i];
    return v;
}

// The skew constants are linear in the group position (initFFT fills level
// m's entries as XOR sums of temp[i]): the butterfly of layer b (shard
// distance 2^b) over the group starting at shard g uses
//   IFFT (index K - 1 + g + 2^b):  XOR of tbasis(b, k) over the set bits k of g, ^ tbasis(b, log2 K)
//   FFT  (index g + 2^b - 1):      XOR of tbasis(b, k) over the set bits k of g
// (every bit k of g is above b).  So a constant that depends on shard bits held
// by lanes or waves splits into a compile-time part and one term per such bit.
constexpr uint32_t tbasis(int b, int k) { return kTemps.t[b][k - 1]; }
// compile-time part of layer b's constant for the group bits `gbits` (bits > b)
template <bool INV, int LOGK>
constexpr uint32_t skew_part(int b, uint32_t gbits) {
    uint32_t v = INV ? tbasis(b, LOGK) : 0;
    for (int k = b + 1; k < LOGK; k++)
        if ((gbits >> k) & 1) v ^= tbasis(b, k);
    return v;
}

// Rows of the 16x16 GF(2) matrix of y -> c*y: row i = mask over input planes j.
struct Net {
    uint16_t row[16];
};
constexpr Net make_net(uint32_t c) {
    Net n{};
    for (int j = 0; j < 16; j++) {
        const uint32_t col = fmul(c, 1u << j);
        for (int i = 0; i < 16; i++)
            if ((col >> i) & 1) n.row[i] |= (uint16_t)(1u << j);
    }
    return n;
}

template <int B, int E, int STEP, class F>
B16_HD void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + STEP, E, STEP>(f);
    }
}

B16_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // full-rate 3-input XOR
#else
    return a ^ b ^ c;
#endif
}
// (a & m) | (b & ~m), bitwise
B16_HD uint32_t bitsel(uint32_t a, uint32_t b, uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4);
#else
    return (a & m) | (b & ~m);
#endif
}

// acc XOR the signals y[j] for the set bits j of MSK, as 3-input XORs.
template <uint32_t MSK, int J = 0>
B16_HD uint32_t xor_fold(uint32_t acc, const uint32_t* y) {
    if constexpr (J >= 32) {
        return acc;
    } else if constexpr ((MSK >> J) == 0) {
        return acc;
    } else if constexpr (((MSK >> J) & 1) == 0) {
        return xor_fold<MSK, J + 1>(acc, y);
    } else {
        constexpr uint32_t rest = MSK & ~((2u << J) - 1);   // bits above J
        if constexpr (rest == 0) {
            return acc ^ y[J];
        } else {
            constexpr int J2 = __builtin_ctz(rest);
            return xor_fold<MSK & ~((2u << J2) - 1), J2 + 1>(xor3(acc, y[J], y[J2]), y);
        }
    }
}

// x ^= c*y for the constant with field value C (planes x[0..16), y[0..16)).
template <uint32_t C>
B16_HD void mul_add(uint32_t* x, const uint32_t* y) {
    if constexpr (C != 0) {
        constexpr Net n = make_net(C);
        sfor<0, 16, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            x[i] = xor_fold<n.row[i]>(x[i], y);
        });
    }
}

// XOR of the planes y[j] for the set bits j of MSK (MSK != 0).
template <uint32_t MSK>
B16_HD uint32_t xor_sel(const uint32_t* y) {
    constexpr int J = __builtin_ctz(MSK);
    return xor_fold<MSK & ~((2u << J) - 1), J + 1>(y[J], y);
}
// x ^ (p & m)
B16_HD uint32_t xor_and(uint32_t x, uint32_t p, uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(x, p, m, 0x78);
#else
    return x ^ (p & m);
#endif
}

// Pair signals: a butterfly's networks all read the same 16 planes y, so the
// 8 pair sums y[2i] ^ y[2i+1] are formed once (S[16 + i]) and a row picks, per
// pair, y[2i], y[2i+1] or their sum: about 3/4 of the terms of the plain row
// (the LOW phase's networks: -20 % instructions for 8 registers).
struct Sig24 {
    uint32_t s[24];
};
B16_HD void make_sig(Sig24& S, const uint32_t* y) {
#pragma unroll
    for (int j = 0; j < 16; j++) S.s[j] = y[j];
#pragma unroll
    for (int i = 0; i < 8; i++) S.s[16 + i] = y[2 * i] ^ y[2 * i + 1];
}
// a row over 16 planes -> the same sum over the 24 signals
constexpr uint32_t pair_terms(uint32_t row) {
    uint32_t t = 0;
    for (int i = 0; i < 8; i++) {
        const uint32_t c = (row >> (2 * i)) & 3;
        if (c == 1) t |= 1u << (2 * i);
        if (c == 2) t |= 1u << (2 * i + 1);
        if (c == 3) t |= 1u << (16 + i);
    }
    return t;
}
// x ^= c*y from the signals of y
template <uint32_t C>
B16_HD void mul_add_s(uint32_t* x, const Sig24& S) {
    if constexpr (C != 0) {
        constexpr Net n = make_net(C);
        sfor<0, 16, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            x[i] = xor_fold<pair_terms(n.row[i])>(x[i], S.s);
        });
    }
}
// x ^= (c*y) & m for a per-lane all-ones / all-zero mask m: the product by one
// basis term of a lane-dependent constant.
template <uint32_t C>
B16_HD void mul_add_masked_s(uint32_t* x, const Sig24& S, uint32_t m) {
    if constexpr (C != 0) {
        constexpr Net n = make_net(C);
        sfor<0, 16, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr (n.row[i] != 0) x[i] = xor_and(x[i], xor_sel<pair_terms(n.row[i])>(S.s), m);
        });
    }
}

// Optimisation fence for n planes (see bitslice8.h: keeps each layer a
// separate network instead of one reassociated XOR DAG); emits nothing.
template <int N>
B16_HD void fence(uint32_t* r) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < N; i++) asm("" : "+v"(r[i]));
#endif
}

// Butterflies (leopard.go IFFT_DIT2 / FFT_DIT2 on planes): C = field value of
// the skew constant, 0 = multiply by zero.
template <uint32_t C>
B16_HD void ifft_bfly(uint32_t* x, uint32_t* y) {
#pragma unroll
    for (int p = 0; p < 16; p++) y[p] ^= x[p];
    mul_add<C>(x, y);
    fence<16>(x);
    fence<16>(y);
}
template <uint32_t C>
B16_HD void fft_bfly(uint32_t* x, uint32_t* y) {
    mul_add<C>(x, y);
#pragma unroll
    for (int p = 0; p < 16; p++) y[p] ^= x[p];
    fence<16>(x);
    fence<16>(y);
}

// In-place 8x8 bit transpose of every byte lane of r[0..8): afterwards r[i]
// byte q bit j == before r[j] byte q bit i.  Self-inverse.  On the 8 lo (or
// hi) dwords of a 64-byte block (dword w byte q = symbol 4w + q) it leaves in
// r[p] bit 8q + w bit p of symbol 4w + q: plane p, symbols in a fixed order.
B16_HD void transpose8(uint32_t* r) {
    sfor<0, 3, 1>([&](auto ss) {
        constexpr int sh = 4 >> decltype(ss)::value;   // 4, 2, 1
        constexpr uint32_t lo = sh == 4 ? 0x0F0F0F0Fu : sh == 2 ? 0x33333333u : 0x55555555u;
        sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & sh) == 0) {
                const uint32_t a = r[i], b = r[i + sh];
                r[i] = bitsel(a, b << sh, lo);
                r[i + sh] = bitsel(a >> sh, b, lo);
            }
        });
    });
}
// A 64-byte block (dwords 0..7 = lo bytes, 8..15 = hi bytes) <-> its 16 planes
// (plane p < 8 from the lo bytes, p >= 8 from the hi bytes).  Self-inverse.
B16_HD void block_planes(uint32_t* r) {
    transpose8(r);
    transpose8(r + 8);
}

// ---------------------------------------------------------------------------
// The k = 2^LOGK encoder's phases (rs_gf16_bs.hip), on the 8 units R[16 u + p]
// of one lane.  A workgroup holds HALF a codeword (4 of the 8 64-byte blocks
// of every shard; two workgroups per CU), a lane one block (lane & 3) of 8
// shards.  Shard s sits in three layouts (wave w, lane index jl = lane >> 2,
// 4 bits; unit u, 3 bits):
//   LOW: s = w << 7 | jl << 3 | u                       IFFT / FFT b = 0, 1, 2
//   M1 : s = w << 7 | (jl >> 3) << 6 | u << 3 | jl & 7  layers 3, 4, 5
//   M2 : s = u << (LOGK - 3) | w << 4 | jl              layers LOGK-3 .. LOGK-1
// A layer's constant depends on the shard bits above it (tbasis): bits held
// by the unit index are compile-time, bits held by the lane index (LOW: bits
// 3..6; M1: bit 6) enter as masked terms (m[i] = all-ones when the lane holds
// a 1), bits held by the wave index (LOW, M1: bits 7..) as uniform-branch
// terms.  M2's constants depend on unit bits only.  x-updates of one layer
// commute, so each term runs over all the layer's butterflies.
// ---------------------------------------------------------------------------
template <int D>
B16_HD void xor_pairs(uint32_t* R) {   // y ^= x for the pairs (i, i + D) of 8 units
    sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr ((i & D) == 0) {
#pragma unroll
            for (int p = 0; p < 16; p++) R[16 * (i + D) + p] ^= R[16 * i + p];
        }
    });
}
// Greedy shared signals (Paar-style common-subexpression extraction, at
// compile time): all networks of one butterfly read the same 16 planes y, so
// up to kPlanSignals derived signals s[16 + i] = s[a_i] ^ s[b_i] are chosen,
// each time the pair whose replacement saves the most 3-input-XOR ops over
// all the butterfly's rows (base, masked lane and wave rows), and every row
// becomes a mask over the 16 + kPlanSignals signals.  Against the fixed pair
// sums y[2i] ^ y[2i+1] (make_sig): 6 % fewer network ops for the same 8
// registers, 11 % with 12 (tools/bs16_cse.py, profiles/r04/bs16_network_ops.txt);
// with triples 16 measured best (profiles/r04/r04z_signal_budget_ab.txt,
// r04zb_triple_budget_ab.txt).
#ifndef CDA_BS16_PLAN_SIGNALS
#define CDA_BS16_PLAN_SIGNALS 16
#endif
constexpr int kPlanSignals = CDA_BS16_PLAN_SIGNALS;
static_assert(kPlanSignals >= 0 && kPlanSignals <= 16, "rows are 32-bit masks over 16 planes + the derived signals");
#ifndef CDA_BS16_PLAN_TRIPLES
#define CDA_BS16_PLAN_TRIPLES 1
#endif
struct SigPlan {
    uint8_t a[kPlanSignals], b[kPlanSignals], c[kPlanSignals];   // c = 0xFF: a pair
    int n;                 // derived signals in use
    uint32_t base[16];     // row masks over 16 + kPlanSignals signals
    uint32_t lane[6][16];   // up to 6 masked lane terms (tools/probes/rs16_per_wave.patch)
    uint32_t wave[2][16];
};
// ops of a row of t signals: x ^= sum (base / wave) or x ^= sum & m (lane)
constexpr int plan_row_ops(uint32_t msk, bool masked) {
    const int t = __builtin_popcount(msk);
    if (t == 0) return 0;
    return masked ? (t - 1 + 1) / 2 + 1 : (t + 1) / 2;
}
constexpr SigPlan make_plan(uint32_t c0, const uint32_t* tl, int nl, const uint32_t* tw, int nw) {
    SigPlan P{};
    uint32_t rows[16 * 9] = {};
    bool msk[16 * 9] = {};
    int nr = 0;
    auto add = [&](uint32_t c, bool masked) {
        const Net n = make_net(c);
        for (int i = 0; i < 16; i++) {
            rows[nr] = n.row[i];
            msk[nr++] = masked;
        }
    };
    add(c0, false);
    for (int l = 0; l < nl; l++) add(tl[l], true);
    for (int w = 0; w < nw; w++) add(tw[w], false);
    int ns = 16;
    constexpr int N = 16 + kPlanSignals;
    int gain3[CDA_BS16_PLAN_TRIPLES ? N * N * N : 1] = {};
    for (int it = 0; it < kPlanSignals; it++) {
        // a row holding every signal of a pair (triple) drops one (two)
        // terms: it saves ops(t) - ops(t - 1) (ops(t) - ops(t - 2)),
        // whichever set it is; the best set must save more than its own op
        int gain2[N][N] = {};
        int best = 1, ba = -1, bb = -1, bc = -1;
        for (int r = 0; r < nr; r++) {
            const uint32_t row = rows[r];
            const int t = __builtin_popcount(row);
            if (t < 2) continue;
            const uint32_t r1 = row & (row - 1), r2 = r1 & (r1 - 1);   // one / two terms fewer
            const int d2 = plan_row_ops(row, msk[r]) - plan_row_ops(r1, msk[r]);
            const int d3 = t >= 3 ? plan_row_ops(row, msk[r]) - plan_row_ops(r2, msk[r]) : 0;
            for (uint32_t ra = row; ra; ra &= ra - 1) {
                const int a = __builtin_ctz(ra);
                for (uint32_t rb = ra & (ra - 1); rb; rb &= rb - 1) {
                    const int b = __builtin_ctz(rb);
                    if (d2 > 0 && (gain2[a][b] += d2) > best) {
                        best = gain2[a][b];
                        ba = a, bb = b, bc = -1;
                    }
                    if (CDA_BS16_PLAN_TRIPLES && d3 > 0)
                        for (uint32_t rc = rb & (rb - 1); rc; rc &= rc - 1) {
                            const int c = __builtin_ctz(rc);
                            int& g = gain3[(a * N + b) * N + c];
                            if ((g += d3) > best) {
                                best = g;
                                ba = a, bb = b, bc = c;
                            }
                        }
                }
            }
        }
        if (CDA_BS16_PLAN_TRIPLES)
            for (int r = 0; r < nr; r++)   // reset the entries this round touched
                for (uint32_t ra = rows[r]; ra; ra &= ra - 1)
                    for (uint32_t rb = ra & (ra - 1); rb; rb &= rb - 1)
                        for (uint32_t rc = rb & (rb - 1); rc; rc &= rc - 1)
                            gain3[(__builtin_ctz(ra) * N + __builtin_ctz(rb)) * N + __builtin_ctz(rc)] = 0;
        if (ba < 0) break;
        const uint32_t pm = (1u << ba) | (1u << bb) | (bc >= 0 ? 1u << bc : 0u);
        for (int r = 0; r < nr; r++)
            if ((rows[r] & pm) == pm) rows[r] = (rows[r] & ~pm) | (1u << ns);
        P.a[it] = (uint8_t)ba;
        P.b[it] = (uint8_t)bb;
        P.c[it] = bc >= 0 ? (uint8_t)bc : (uint8_t)0xFF;
        ns++;
    }
    P.n = ns - 16;
    int r = 0;
    for (int i = 0; i < 16; i++) P.base[i] = rows[r++];
    for (int l = 0; l < nl; l++)
        for (int i = 0; i < 16; i++) P.lane[l][i] = rows[r++];
    for (int w = 0; w < nw; w++)
        for (int i = 0; i < 16; i++) P.wave[w][i] = rows[r++];
    return P;
}
template <int LOGK, bool INV, int b, int NL, int LB, int NWB, int WB>
constexpr SigPlan layer_plan(uint32_t c0) {
    uint32_t tl[6] = {}, tw[2] = {};
    static_assert(NL <= 6 && NWB <= 2, "SigPlan holds 6 lane and 2 wave terms");
    for (int l = 0; l < NL; l++) tl[l] = tbasis(b, LB + l);
    for (int w = 0; w < NWB; w++) tw[w] = tbasis(b, WB + w);
    return make_plan(c0, tl, NL, tw, NWB);
}
// x ^= rows of plan P over the signals S (xor_fold / xor_sel take 32-bit masks)
template <uint32_t MSK>
B16_HD void plan_row(uint32_t& x, const uint32_t* S) {
    if constexpr (MSK != 0) x = xor_fold<MSK>(x, S);
}
template <uint32_t MSK>
B16_HD void plan_row_masked(uint32_t& x, const uint32_t* S, uint32_t m) {
    if constexpr (MSK != 0) x = xor_and(x, xor_sel<MSK>(S), m);
}

// A layer's lane masks: an array (m[l]) or a functor that derives mask L
// where it is needed (LaneMask: no long-lived mask registers).
template <int L, class M>
B16_HD uint32_t mask_at(const M& m) {
    if constexpr (std::is_pointer_v<M> || std::is_array_v<M>)
        return m[L];
    else
        return m.template get<L>();
}
// All-ones when bit BASE + L of the lane index is set: one v_bfe_i32 (opaque
// asm, so it is neither hoisted nor kept alive across the networks).
template <int BASE>
struct LaneMask {
    uint32_t lane;
    template <int L>
    B16_HD uint32_t get() const {
#if defined(__HIP_DEVICE_COMPILE__)
        uint32_t v;
        asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(v) : "v"(lane), "n"(BASE + L));
        return v;
#else
        return 0u - ((lane >> (BASE + L)) & 1);
#endif
    }
};

// the masks of lane bits from BY up: m + BY for an array, BASE + BY for LaneMask
template <int BY>
B16_HD const uint32_t* shifted(const uint32_t* m) { return m + BY; }
template <int BY, int BASE>
B16_HD LaneMask<BASE + BY> shifted(const LaneMask<BASE>& m) { return LaneMask<BASE + BY>{m.lane}; }

// One layer over the 8 units: unit distance D, shard bit b, the unit index
// holding shard bits from SH up (group bits of unit i: (i & ~(2D-1)) << SH),
// NL masked lane terms (shard bits LB..), NWB uniform wave terms (bits WB..).
// Only butterflies whose two units lie in [ULO, UHI) (the kernel can run a
// layer over units 0..3 while units 4..7 are still loading).
// Per butterfly the shared signals of y are formed once and every term reads
// them; the wave terms are uniform branches.
#ifndef CDA_BS16_PAIR_SIGNALS
template <int LOGK, bool INV, int b, int D, int SH, int NL, int LB, int NWB, int WB, int ULO = 0, int UHI = 8,
          class M>
B16_HD void layer8(uint32_t* R, const M& m, uint32_t u) {
    sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr ((i & D) == 0 && i >= ULO && i + D < UHI) {
            uint32_t* x = R + 16 * i;
            uint32_t* y = R + 16 * (i + D);
            if constexpr (INV) {
#pragma unroll
                for (int p = 0; p < 16; p++) y[p] ^= x[p];
            }
            constexpr uint32_t C0 = skew_part<INV, LOGK>(b, (uint32_t)(i & ~(2 * D - 1)) << SH);
            constexpr SigPlan P = layer_plan<LOGK, INV, b, NL, LB, NWB, WB>(C0);
            uint32_t S[16 + kPlanSignals];
#pragma unroll
            for (int p = 0; p < 16; p++) S[p] = y[p];
            sfor<0, P.n, 1>([&](auto ss) {
                constexpr int s = decltype(ss)::value;
                if constexpr (P.c[s] == 0xFF)
                    S[16 + s] = S[P.a[s]] ^ S[P.b[s]];
                else
                    S[16 + s] = xor3(S[P.a[s]], S[P.b[s]], S[P.c[s]]);
            });
            sfor<0, 16, 1>([&](auto rr) {
                constexpr int r = decltype(rr)::value;
                plan_row<P.base[r]>(x[r], S);
            });
            sfor<0, NL, 1>([&](auto ll) {
                constexpr int l = decltype(ll)::value;
                const uint32_t mk = mask_at<l>(m);
                sfor<0, 16, 1>([&](auto rr) {
                    constexpr int r = decltype(rr)::value;
                    plan_row_masked<P.lane[l][r]>(x[r], S, mk);
                });
            });
            sfor<0, NWB, 1>([&](auto ww) {
                constexpr int w = decltype(ww)::value;
                if (u & (1u << w)) {
                    sfor<0, 16, 1>([&](auto rr) {
                        constexpr int r = decltype(rr)::value;
                        plan_row<P.wave[w][r]>(x[r], S);
                    });
                }
            });
            if constexpr (!INV) {
#pragma unroll
                for (int p = 0; p < 16; p++) y[p] ^= x[p];
            }
            fence<16>(x);
            fence<16>(y);
        }
    });
}
#else
template <int LOGK, bool INV, int b, int D, int SH, int NL, int LB, int NWB, int WB, int ULO = 0, int UHI = 8,
          class M>
B16_HD void layer8(uint32_t* R, const M& m, uint32_t u) {
    sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        if constexpr ((i & D) == 0 && i >= ULO && i + D < UHI) {
            uint32_t* x = R + 16 * i;
            uint32_t* y = R + 16 * (i + D);
            if constexpr (INV) {
#pragma unroll
                for (int p = 0; p < 16; p++) y[p] ^= x[p];
            }
            Sig24 S;
            make_sig(S, y);
            constexpr uint32_t C0 = skew_part<INV, LOGK>(b, (uint32_t)(i & ~(2 * D - 1)) << SH);
            mul_add_s<C0>(x, S);
            sfor<0, NL, 1>([&](auto ll) {
                constexpr int l = decltype(ll)::value;
                mul_add_masked_s<tbasis(b, LB + l)>(x, S, mask_at<l>(m));
            });
            sfor<0, NWB, 1>([&](auto ww) {
                constexpr int w = decltype(ww)::value;
                if (u & (1u << w)) mul_add_s<tbasis(b, WB + w)>(x, S);
            });
            if constexpr (!INV) {
#pragma unroll
                for (int p = 0; p < 16; p++) y[p] ^= x[p];
            }
            fence<16>(x);
            fence<16>(y);
        }
    });
}
#endif
// LOW layer b (0..2): unit = shard bits 0..2, lane bits 3..6 (m[0..3]), wave bits 7..
template <int LOGK, bool INV, int b, int ULO = 0, int UHI = 8, class M>
B16_HD void low_layer(uint32_t* R, const M& m, uint32_t u) {
    layer8<LOGK, INV, b, 1 << b, 0, 4, 3, LOGK - 7, 7, ULO, UHI>(R, m, u);
}
// M1 layer b (3..5): unit = shard bits 3..5, lane bit 6 (m[3]), wave bits 7..
template <int LOGK, bool INV, int b, class M>
B16_HD void m1_layer(uint32_t* R, const M& m, uint32_t u) {
    layer8<LOGK, INV, b, 1 << (b - 3), 3, 1, 6, LOGK - 7, 7>(R, shifted<3>(m), u);
}
// M2 layer b (LOGK-3..LOGK-1): unit = shard bits LOGK-3.., no lane / wave terms
template <int LOGK, bool INV, int b>
B16_HD void m2_layer(uint32_t* R) {
    layer8<LOGK, INV, b, 1 << (b - (LOGK - 3)), LOGK - 3, 0, 0, 0, 0>(R, (const uint32_t*)nullptr, 0);
}
// The phases in encode order (leopard.go encode: IFFT over the k data shards
// at coset k, then FFT to the k parity shards):
template <int LOGK, class M>
B16_HD void phase_low_ifft(uint32_t* R, const M& m, uint32_t u) {
    low_layer<LOGK, true, 0>(R, m, u);
    low_layer<LOGK, true, 1>(R, m, u);
    low_layer<LOGK, true, 2>(R, m, u);
}
template <int LOGK, class M>
B16_HD void phase_m1_ifft(uint32_t* R, const M& m, uint32_t u) {   // layers 3..5
    m1_layer<LOGK, true, 3>(R, m, u);
    m1_layer<LOGK, true, 4>(R, m, u);
    m1_layer<LOGK, true, 5>(R, m, u);
}
template <int LOGK>
B16_HD void phase_m2(uint32_t* R) {   // IFFT 6..LOGK-1, FFT LOGK-1..LOGK-3
    sfor<6, LOGK, 1>([&](auto bb) { m2_layer<LOGK, true, decltype(bb)::value>(R); });
    sfor<0, 3, 1>([&](auto bb) { m2_layer<LOGK, false, LOGK - 1 - decltype(bb)::value>(R); });
}
template <int LOGK, class M>
B16_HD void phase_m1_fft(uint32_t* R, const M& m, uint32_t u) {   // layers LOGK-4..3
    sfor<0, LOGK - 6, 1>([&](auto bb) { m1_layer<LOGK, false, LOGK - 4 - decltype(bb)::value>(R, m, u); });
}
template <int LOGK, class M>
B16_HD void phase_low_fft(uint32_t* R, const M& m, uint32_t u) {
    low_layer<LOGK, false, 2>(R, m, u);
    low_layer<LOGK, false, 1>(R, m, u);
    low_layer<LOGK, false, 0>(R, m, u);
}

}  // namespace bs16
}  // namespace cda
