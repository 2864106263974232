// leopard_tables.h -- Leopard GF(2^8) / GF(2^16) tables for the RS kernels.
//
// Restates klauspost/reedsolomon v1.12.1 (EXT module pinned at
// /root/reference/go.mod:152; not vendored) leopard8.go initLUTs8/initFFT8 and
// leopard.go initLUTs/initFFT: LFSR exp/log over poly 0x11D / 0x1002D, Cantor
// basis conversion, FFT skew vector (stored as logs; value == modulus means
// "multiply by zero").  GF(2^8) tables are built at compile time so the
// register-resident encoder (rs_gf8.hip) sees every butterfly constant as an
// immediate; GF(2^16) tables are built on the host (engine) and uploaded.
#pragma once
#include <stdint.h>

namespace cda {

template <int BITS>
struct LeoField {
    static constexpr uint32_t ORDER = 1u << BITS;
    static constexpr uint32_t MOD = ORDER - 1;
    uint16_t log[ORDER];
    uint16_t exp[ORDER];
    uint16_t skew[MOD];

    constexpr uint32_t add_mod(uint32_t a, uint32_t b) const {
        uint32_t s = a + b;
        return (s + (s >> BITS)) & MOD;
    }
    constexpr uint32_t mul_log(uint32_t a, uint32_t log_b) const {
        return a == 0 ? 0 : exp[add_mod(log[a], log_b)];
    }
};

template <int BITS>
constexpr void leo_build(LeoField<BITS>& F, uint32_t poly, const uint16_t* cantor) {
    constexpr uint32_t ORDER = LeoField<BITS>::ORDER, MOD = LeoField<BITS>::MOD;
    uint32_t state = 1;
    for (uint32_t i = 0; i < MOD; i++) {
        F.exp[state] = (uint16_t)i;
        state <<= 1;
        if (state >= ORDER) state ^= poly;
    }
    F.exp[0] = (uint16_t)MOD;
    F.log[0] = 0;
    for (int i = 0; i < BITS; i++) {
        uint32_t width = 1u << i;
        for (uint32_t j = 0; j < width; j++) F.log[j + width] = F.log[j] ^ cantor[i];
    }
    for (uint32_t i = 0; i < ORDER; i++) F.log[i] = F.exp[F.log[i]];
    for (uint32_t i = 0; i < ORDER; i++) F.exp[F.log[i]] = (uint16_t)i;
    F.exp[MOD] = F.exp[0];

    uint32_t temp[BITS > 1 ? BITS - 1 : 1] = {};
    for (int i = 1; i < BITS; i++) temp[i - 1] = 1u << i;
    for (uint32_t i = 0; i < MOD; i++) F.skew[i] = 0;
    for (int m = 0; m < BITS - 1; m++) {
        uint32_t step = 1u << (m + 1);
        F.skew[(1u << m) - 1] = 0;
        for (int i = m; i < BITS - 1; i++) {
            uint32_t s = 1u << (i + 1);
            for (uint32_t j = (1u << m) - 1; j < s; j += step) F.skew[j + s] = F.skew[j] ^ temp[i];
        }
        temp[m] = MOD - F.log[F.mul_log(temp[m], F.log[temp[m] ^ 1])];
        for (int i = m + 1; i < BITS - 1; i++)
            temp[i] = F.mul_log(temp[i], F.add_mod(F.log[temp[i] ^ 1], temp[m]));
    }
    for (uint32_t i = 0; i < MOD; i++) F.skew[i] = F.log[F.skew[i]];
}

constexpr uint16_t kCantor8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
constexpr uint16_t kCantor16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

constexpr LeoField<8> make_gf8() {
    LeoField<8> F{};
    leo_build<8>(F, 0x11D, kCantor8);
    return F;
}

// 2-bit-chunk multiply tables for GF(2^8): for the constant with log L,
// c[q] byte e = mul_log(e << 2q, L), so v_perm_b32(c[q], c[q], (y >> 2q) &
// 0x03030303) multiplies chunk q of four packed symbols; the four partial
// products XOR to L * y.  L = 255 (the modulus) is the identity.
struct Mul8Chunks {
    uint32_t c[4];
};
struct Mul8All {
    Mul8Chunks t[256];
};
constexpr Mul8All make_all_mul8(const LeoField<8>& F) {
    Mul8All a{};
    for (uint32_t l = 0; l < 256; l++)
        for (uint32_t q = 0; q < 4; q++)
            for (uint32_t e = 0; e < 4; e++) a.t[l].c[q] |= (uint32_t)F.mul_log(e << (2 * q), l) << (8 * e);
    return a;
}

// ---------------------------------------------------------------------------
// v_perm_b32 nibble lookup.  For a 16-entry byte table T and nibble vector n
// (four byte lanes, each 0..15):
//   T[n] = perm(A1, A0, n) ^ perm(B1, B0, n ^ 0x08)
// where perm's selector values 8..15 yield the "junk" bytes of the ISA
// (sign-broadcast of bytes 1/3/5/7, 0x00, 0xFF).  A and B are solved so the
// junk cancels ("GF(2^8) multiply").  Byte layout of an 8-byte
// table pair (hi dword, lo dword): entry e lives in byte e.
// ---------------------------------------------------------------------------
struct NibblePerm {
    uint32_t a_lo, a_hi, b_lo, b_hi;
};

constexpr uint8_t sgn(uint8_t x) { return (x & 0x80) ? 0xFF : 0x00; }

constexpr NibblePerm solve_nibble_perm(const uint8_t T[16]) {
    uint8_t A[8] = {}, B[8] = {};
    A[4] = T[4]; A[5] = T[5] ^ 0xFF; A[6] = T[6] ^ 0xFF; A[7] = T[7] ^ 0xFF;
    B[4] = T[12]; B[5] = T[13] ^ 0xFF; B[6] = T[14] ^ 0xFF; B[7] = T[15] ^ 0xFF;
    B[2] = T[10] ^ sgn(A[5]);
    B[3] = T[11] ^ sgn(A[7]);
    A[1] = T[1] ^ sgn(B[3]);
    A[3] = T[3] ^ sgn(B[7]);
    A[2] = T[2] ^ sgn(B[5]);
    B[1] = T[9] ^ sgn(A[3]);
    B[0] = T[8] ^ sgn(A[1]);
    A[0] = T[0] ^ sgn(B[1]);
    NibblePerm p{};
    p.a_lo = A[0] | (uint32_t)A[1] << 8 | (uint32_t)A[2] << 16 | (uint32_t)A[3] << 24;
    p.a_hi = A[4] | (uint32_t)A[5] << 8 | (uint32_t)A[6] << 16 | (uint32_t)A[7] << 24;
    p.b_lo = B[0] | (uint32_t)B[1] << 8 | (uint32_t)B[2] << 16 | (uint32_t)B[3] << 24;
    p.b_hi = B[4] | (uint32_t)B[5] << 8 | (uint32_t)B[6] << 16 | (uint32_t)B[7] << 24;
    return p;
}

// Host/constexpr model of v_perm_b32 (used by tests of the table solver).
constexpr uint8_t perm_byte(uint32_t s0, uint32_t s1, uint8_t sel) {
    uint8_t in[8] = {(uint8_t)s1, (uint8_t)(s1 >> 8), (uint8_t)(s1 >> 16), (uint8_t)(s1 >> 24),
                     (uint8_t)s0, (uint8_t)(s0 >> 8), (uint8_t)(s0 >> 16), (uint8_t)(s0 >> 24)};
    if (sel >= 13) return 0xFF;
    if (sel == 12) return 0x00;
    if (sel == 11) return sgn(in[7]);
    if (sel == 10) return sgn(in[5]);
    if (sel == 9) return sgn(in[3]);
    if (sel == 8) return sgn(in[1]);
    return in[sel];
}

// Multiply-by-constant tables for GF(2^8): low-nibble and high-nibble lookups.
struct Mul8Perm {
    NibblePerm lo, hi;
};

template <int BITS>
constexpr Mul8Perm make_mul8_perm(const LeoField<BITS>& F, uint32_t log_m) {
    uint8_t tl[16] = {}, th[16] = {};
    for (uint32_t n = 0; n < 16; n++) {
        tl[n] = (uint8_t)F.mul_log(n, log_m);
        th[n] = (uint8_t)F.mul_log(n << 4, log_m);
    }
    Mul8Perm m{};
    m.lo = solve_nibble_perm(tl);
    m.hi = solve_nibble_perm(th);
    return m;
}

}  // namespace cda
