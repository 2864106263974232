// bitslice8.h -- bitsliced GF(2^8) Leopard encode core for k = 128 (host + device).
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF8 IFFT(coset k)/FFT(coset 0)
// (EXT, pinned at /root/reference/go.mod:152; reached through
// pkg/appconsts/global_consts.go:92 -> rsmt2d LeoRSCodec.Encode) in
// bitsliced form: a 32-bit register holds bit p ("plane p") of 32 symbols, so
//   * GF addition is one XOR per plane (8 per 32 symbols), and
//   * multiplication by a skew constant c is an 8x8 GF(2) matrix: plane i of
//     c*y is the XOR of the planes j of y with bit i of c*(1<<j) set -- a
//     compile-time XOR network of ~16 three-input XORs (v_bitop3) per 32
//     symbols, versus 4 v_perm lookups (half rate) + 7 selector ops per 4
//     symbols in the byte-form encoder (rs_gf8.hip).
// Bytes <-> planes: an in-register 8x8 bit transpose (3 swap stages, 48 ops
// per 32 symbols).
//
// A butterfly constant depends on the shard-index bits ABOVE the layer, so the
// constants are wave-uniform (and compile-time) when lanes differ only in
// columns.  Shard index s = 16u + t (u = bits 4..6, t = bits 0..3):
//   pass A (wave u):  16 shards t in registers, IFFT d = 1, 2, 4, 8;
//   pass B (any wave): 8 shards u for a fixed t, IFFT d = 16, 32, 64 then
//                     FFT d = 64, 32, 16 (constants depend on u only);
//   pass C (wave u):  FFT d = 8, 4, 2, 1.
// Passes A/C are specialised per u (switch), pass B is one code path.  The
// kernel (rs_gf8_bs.hip) moves registers between the layouts through LDS.
#pragma once
#include <stdint.h>

#include <type_traits>

#include "leopard_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BS_HD __host__ __device__ __forceinline__
#else
#define BS_HD inline
#endif

namespace cda {
namespace bs8 {

constexpr int K = 128;               // shards per codeword (ODS width)
constexpr uint32_t kMod = 255;
inline constexpr LeoField<8> kField = make_gf8();

// kNet[L][i] = bitmask over input planes j that feed output plane i of
// (multiply by the constant with log L).
struct Nets {
    uint8_t m[256][8];
};
constexpr Nets make_nets() {
    Nets n{};
    for (uint32_t L = 0; L < 256; L++)
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t col = L == kMod ? 0 : kField.mul_log(1u << j, L);
            for (uint32_t i = 0; i < 8; i++)
                if ((col >> i) & 1) n.m[L][i] |= (uint8_t)(1u << j);
        }
    return n;
}
inline constexpr Nets kNets = make_nets();

template <int B, int E, int STEP, class F>
BS_HD void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + STEP, E, STEP>(f);
    }
}

BS_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // full-rate 3-input XOR
#else
    return a ^ b ^ c;
#endif
}

// XOR of x and the planes y[j] for the set bits j of MSK, as 3-input XORs.
template <uint32_t MSK, int J = 0>
BS_HD uint32_t xor_fold(uint32_t acc, const uint32_t* y) {
    if constexpr (J >= 8 || (MSK >> J) == 0) {
        return acc;
    } else if constexpr (((MSK >> J) & 1) == 0) {
        return xor_fold<MSK, J + 1>(acc, y);
    } else {
        constexpr uint32_t rest = MSK & ~((2u << J) - 1);     // bits above J
        if constexpr (rest == 0) {
            return acc ^ y[J];
        } else {
            constexpr int J2 = __builtin_ctz(rest);
            return xor_fold<MSK & ~((2u << J2) - 1), J2 + 1>(xor3(acc, y[J], y[J2]), y);
        }
    }
}

// x ^= c*y, c = constant with log L (planes x[0..8), y[0..8)).
template <uint32_t L>
BS_HD void mul_add(uint32_t* x, const uint32_t* y) {
    sfor<0, 8, 1>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        x[i] = xor_fold<kNets.m[L][i]>(x[i], y);
    });
}

// Optimisation fence for n planes: the butterfly algebra is all XOR, and LLVM
// reassociates/distributes XOR trees across layers into huge shared DAGs
// (256 VGPRs + spills for 4 layers).  An empty asm per plane after each layer
// keeps every layer a separate network; it emits no instruction.
template <int N>
BS_HD void fence(uint32_t* r) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < N; i++) asm("" : "+v"(r[i]));
#endif
}

template <uint32_t L>
BS_HD void ifft_bfly(uint32_t* x, uint32_t* y) {
#pragma unroll
    for (int p = 0; p < 8; p++) y[p] ^= x[p];
    if constexpr (L != kMod) mul_add<L>(x, y);
    fence<8>(x);
    fence<8>(y);
}
template <uint32_t L>
BS_HD void fft_bfly(uint32_t* x, uint32_t* y) {
    if constexpr (L != kMod) mul_add<L>(x, y);
#pragma unroll
    for (int p = 0; p < 8; p++) y[p] ^= x[p];
    fence<8>(x);
    fence<8>(y);
}

// (a & m) | (b & ~m)
BS_HD uint32_t bitsel(uint32_t a, uint32_t b, uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4);   // m ? a : b, bitwise
#else
    return (a & m) | (b & ~m);
#endif
}

// In-place 8x8 bit transpose of every byte lane: afterwards r[i] byte q bit
// j == before r[j] byte q bit i.  Self-inverse.
BS_HD void transpose8(uint32_t* r) {
    sfor<0, 3, 1>([&](auto ss) {
        constexpr int sh = 4 >> decltype(ss)::value;                 // 4, 2, 1
        constexpr uint32_t lo = sh == 4 ? 0x0F0F0F0Fu : sh == 2 ? 0x33333333u : 0x55555555u;
        sfor<0, 8, 1>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            if constexpr ((i & sh) == 0) {
                const uint32_t a = r[i], b = r[i + sh];
                r[i] = bitsel(a, b << sh, lo);          // low parts of a, low parts of b moved up
                r[i + sh] = bitsel(a >> sh, b, lo);     // high parts of a moved down, high parts of b
            }
        });
    });
}

// ---- pass A: IFFT d = 1..8 over shards 16U + t (R[8t + p]) ----------------
template <int U>
BS_HD void pass_a(uint32_t* R) {
    sfor<0, 4, 1>([&](auto ld) {
        constexpr int d = 1 << decltype(ld)::value;
        sfor<0, 16, 2 * d>([&](auto gg) {
            constexpr int g = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[K - 1 + 16 * U + g + d];
            sfor<g, g + d, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                ifft_bfly<L>(R + 8 * i, R + 8 * (i + d));
            });
        });
    });
}
// ---- pass C: FFT d = 8..1 over shards 16U + t ------------------------------
template <int U>
BS_HD void pass_c(uint32_t* R) {
    sfor<0, 4, 1>([&](auto ld) {
        constexpr int d = 8 >> decltype(ld)::value;
        sfor<0, 16, 2 * d>([&](auto gg) {
            constexpr int g = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[16 * U + g + d - 1];
            sfor<g, g + d, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                fft_bfly<L>(R + 8 * i, R + 8 * (i + d));
            });
        });
    });
}
// ---- pass B: shards 16u + t for u = 0..7 (R[8u + p]), any fixed t ----------
BS_HD void pass_b(uint32_t* R) {
    sfor<0, 3, 1>([&](auto ld) {                      // IFFT d = 16, 32, 64
        constexpr int du = 1 << decltype(ld)::value;
        sfor<0, 8, 2 * du>([&](auto gg) {
            constexpr int g = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[K - 1 + 16 * g + 16 * du];
            sfor<g, g + du, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                ifft_bfly<L>(R + 8 * i, R + 8 * (i + du));
            });
        });
    });
    sfor<0, 3, 1>([&](auto ld) {                      // FFT d = 64, 32, 16
        constexpr int du = 4 >> decltype(ld)::value;
        sfor<0, 8, 2 * du>([&](auto gg) {
            constexpr int g = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[16 * g + 16 * du - 1];
            sfor<g, g + du, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                fft_bfly<L>(R + 8 * i, R + 8 * (i + du));
            });
        });
    });
}

// ---- half layout (rs8_bs_half_kernel): a lane holds 8 of the 16 shards of
// block U, the ones of its parity h (shard 16U + 2j + h in R[8j + p],
// j = 0..7), and its partner lane the other 8.  The IFFT / FFT layers of shard
// distance 2, 4, 8 pair registers of one lane (distance 1, 2, 4) and use the
// same constant in both lanes, so they stay wave-uniform and compile-time;
// only shard distance 1 pairs the two lanes (the *_d1 steps below, given the
// partner's planes P).
template <int U>
BS_HD void pass_a_hi(uint32_t* R) {   // IFFT shard distance 2, 4, 8
    sfor<0, 3, 1>([&](auto ld) {
        constexpr int dj = 1 << decltype(ld)::value;
        sfor<0, 8, 2 * dj>([&](auto gg) {
            constexpr int gj = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[K - 1 + 16 * U + 2 * gj + 2 * dj];
            sfor<gj, gj + dj, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                ifft_bfly<L>(R + 8 * i, R + 8 * (i + dj));
            });
        });
    });
}
template <int U>
BS_HD void pass_c_hi(uint32_t* R) {   // FFT shard distance 8, 4, 2
    sfor<0, 3, 1>([&](auto ld) {
        constexpr int dj = 4 >> decltype(ld)::value;
        sfor<0, 8, 2 * dj>([&](auto gg) {
            constexpr int gj = decltype(gg)::value;
            constexpr uint32_t L = kField.skew[16 * U + 2 * gj + 2 * dj - 1];
            sfor<gj, gj + dj, 1>([&](auto ii) {
                constexpr int i = decltype(ii)::value;
                fft_bfly<L>(R + 8 * i, R + 8 * (i + dj));
            });
        });
    });
}
// x ^ (p & m)
BS_HD uint32_t xor_and(uint32_t x, uint32_t p, uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(x, p, m, 0x78);
#else
    return x ^ (p & m);
#endif
}
// IFFT butterfly of shards (2j, 2j+1) across the lane pair: x = own planes,
// P = the partner's, h0 = all-ones in the lane holding the even shard.  Both
// lanes form y' = x ^ y; the even lane keeps x ^ c*y', the odd lane y'.
template <uint32_t L>
BS_HD void ifft_d1(uint32_t* x, const uint32_t* P, uint32_t h0) {
    uint32_t T[8];
#pragma unroll
    for (int p = 0; p < 8; p++) T[p] = x[p] ^ P[p];
    if constexpr (L != kMod) mul_add<L>(x, T);
#pragma unroll
    for (int p = 0; p < 8; p++) x[p] = bitsel(x[p], T[p], h0);
    fence<8>(x);
}
// FFT butterfly across the lane pair: even lane x' = x ^ c*y (y = P), odd
// lane y' = y ^ x' = y ^ x ^ c*y (y = own): acc = own ^ (P & h1), acc ^= c*Y.
template <uint32_t L>
BS_HD void fft_d1(uint32_t* x, const uint32_t* P, uint32_t h0) {
    uint32_t Y[8];
#pragma unroll
    for (int p = 0; p < 8; p++) {
        Y[p] = bitsel(P[p], x[p], h0);
        x[p] = xor_and(x[p], P[p], ~h0);
    }
    if constexpr (L != kMod) mul_add<L>(x, Y);
    fence<8>(x);
}
template <int U>
constexpr uint32_t ifft_d1_log(int j) { return kField.skew[K - 1 + 16 * U + 2 * j + 1]; }
template <int U>
constexpr uint32_t fft_d1_log(int j) { return kField.skew[16 * U + 2 * j]; }

// Runs f(integral_constant<U>) for U == u as a chain of uniform if-blocks.
template <class F>
BS_HD void with_u_chain(uint32_t u, F&& f) {
    sfor<0, 8, 1>([&](auto uu) {
        if (u == (uint32_t)decltype(uu)::value) f(uu);
    });
}

template <class F>
BS_HD void with_u(uint32_t u, F&& f) {
    switch (u) {
        case 0: f(std::integral_constant<int, 0>{}); break;
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: f(std::integral_constant<int, 3>{}); break;
        case 4: f(std::integral_constant<int, 4>{}); break;
        case 5: f(std::integral_constant<int, 5>{}); break;
        case 6: f(std::integral_constant<int, 6>{}); break;
        default: f(std::integral_constant<int, 7>{}); break;
    }
}

}  // namespace bs8
}  // namespace cda
