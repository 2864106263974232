// sha256_dev.h -- SHA-256 compression and NMT message/node builders.
//
// Device code on 32-bit words.  The compression uses gfx950's three-input
// integer ops explicitly: v_bitop3_b32 for XOR3 / Ch / Maj, v_add3_u32, and
// v_alignbit_b32 rotates -- 14 VALU ops per round and 10 per schedule word,
// 1384 per compression (DESIGN.md "SHA-256 op count").
//
// Byte layouts follow the nmt hasher (in-tree copy
// /root/reference/test/util/malicious/hasher.go:186-310) and the erasured
// wrapper (/root/reference/pkg/wrapper/nmt_wrapper.go:93-140):
//   leaf message  = 0x00 || ns(29) || share(512)              (542 B, 9 blocks)
//   leaf node     = ns || ns || sha256(leaf message)          (90 B)
//   inner message = 0x01 || left(90) || right(90)             (181 B, 3 blocks)
//   inner node    = l.min || (r.min == 0xFF*29 ? l.max : r.max) || sha256(...)
// Nodes are kept on device in 96-byte slots (90 B + 6 zero bytes) so every
// node load/store is 16-byte aligned.
#pragma once
#include <stdint.h>

#ifndef CDA_HD
#define CDA_HD __device__ __forceinline__
#endif

namespace cda {

constexpr int kShare = 512;
constexpr int kNs = 29;
constexpr int kNode = 90;
constexpr int kSlot = 96;       // device node slot (bytes)
constexpr int kSlotWords = 24;

CDA_HD uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__host__ __device__ constexpr uint32_t crotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// v_bitop3_b32: result bit = imm[(a << 2) | (b << 1) | c]
CDA_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
CDA_HD uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }
CDA_HD uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }
CDA_HD uint32_t add3(uint32_t a, uint32_t b, uint32_t c) { return a + b + c; }
// ({hi, lo} >> 8*s)[31:0]  -> v_alignbyte_b32
CDA_HD uint32_t funnel8(uint32_t hi, uint32_t lo, int s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * s));
}
CDA_HD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0x0000FF00u) | ((x << 8) & 0x00FF0000u) | (x << 24);
}

struct ShaState {
    uint32_t h[8];
};

CDA_HD void sha_init(ShaState& s) {
    s.h[0] = 0x6a09e667u; s.h[1] = 0xbb67ae85u; s.h[2] = 0x3c6ef372u; s.h[3] = 0xa54ff53au;
    s.h[4] = 0x510e527fu; s.h[5] = 0x9b05688cu; s.h[6] = 0x1f83d9abu; s.h[7] = 0x5be0cd19u;
}

#define CDA_SHA_K                                                                                        \
    {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u, \
     0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, \
     0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, \
     0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, \
     0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, \
     0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, \
     0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u, \
     0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u}

// One compression; w[] holds the 16 big-endian message words and is consumed.
CDA_HD void sha_compress(ShaState& s, uint32_t w[16]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = add3(w[i & 15], s0, w[(i - 7) & 15]) + s1;
            w[i & 15] = wi;
        }
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t t1 = add3(add3(h, S1, ch(e, f, g)), K[i], wi);
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = add3(t1, S0, mj);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// ---------------------------------------------------------------------------
// Lane-pair compression, for the latency-bound tails (tree tops, data root).
// A wave issues one VALU instruction per ~4 cycles however few lanes are
// active, so a chain of dependent compressions costs its instruction count.
// Lanes 2j (e-side: holds e f g h) and 2j+1 (a-side: a b c d) of a pair run
// ONE instruction stream: per-lane rotate amounts make Sigma1 / Sigma0 (and
// the schedule's sigma1 / sigma0) one alignbit triple; Ch / Maj one Ch over
// a per-lane input (pair_chmaj);
// the pair exchanges T1 and d with a DPP quad_perm swap:
//   e-side:  T = Sigma1 + Ch + (h + K + W) = T1,  e' = T + d(partner)
//   a-side:  T = Sigma0 + Maj             = T2,  a' = T + T1(partner)
// Schedule: x = w[t-2] (e-side) / w[t-15] (a-side); u = sigma + w[t-7] +
// w[t-16]; w[t] = u + sigma(partner).  11 ops per round and 7 per schedule
// word: 1 040 instructions per compression instead of 1 384.  Both lanes of
// a pair must be active and hold the same message words.
// ---------------------------------------------------------------------------
struct ShaPair {
    uint32_t h[4];   // a-side lane: H0..H3; e-side lane: H4..H7
};
CDA_HD bool pair_aside() { return (__lane_id() & 1) != 0; }
// the partner lane's x (quad_perm [1,0,3,2])
CDA_HD uint32_t pair_swap(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false); }
// e-side lane: e_val, a-side lane: a_val.  One v_cndmask on the constant
// odd-lane mask, in asm: written as `A ? w[i] : w[j]` the compiler turns the
// schedule's selects into a per-lane register index (compare/select chains).
// u + (the partner lane's x) as one v_add_u32_dpp: u passes through an
// empty asm so the compiler cannot fold the sum into a v_add3 (which takes no
// DPP operand and would cost a v_mov + v_mov_dpp).  (An explicit asm DPP add
// needs its own s_nop for the VALU-write -> DPP-read hazard and measured
// slower, profiles/r02d_tail.)
CDA_HD uint32_t pair_add(uint32_t u, uint32_t x) {
    asm("" : "+v"(u));
    return u + pair_swap(x);
}
CDA_HD uint32_t pair_sel(uint32_t e_val, uint32_t a_val) {
    if (__builtin_constant_p(e_val == a_val) && e_val == a_val) return e_val;
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(e_val), "v"(a_val), "s"(0xAAAAAAAAAAAAAAAAull));
    return r;
}

// Ch on the e-side lane, Maj on the a-side lane, in two ops instead of
// three (two bitop3 + select): Maj(a, b, c) = Ch(a ^ c, b, c), so both lanes
// run Ch(v0 ^ (v2 & mA), v1, v2) with mA = the a-side lane mask (0 on the
// e-side lane, all ones on the a-side lane; pair_mask()).
CDA_HD uint32_t pair_mask() { return pair_sel(0u, 0xFFFFFFFFu); }
CDA_HD uint32_t pair_chmaj(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t mA) {
    return ch(__builtin_amdgcn_bitop3_b32(v0, v2, mA, 0x78), v1, v2);   // 0x78: a ^ (b & c)
}

CDA_HD void sha_pair_init(ShaPair& s, bool A) {
    s.h[0] = A ? 0x6a09e667u : 0x510e527fu;
    s.h[1] = A ? 0xbb67ae85u : 0x9b05688cu;
    s.h[2] = A ? 0x3c6ef372u : 0x1f83d9abu;
    s.h[3] = A ? 0xa54ff53au : 0x5be0cd19u;
}

CDA_HD void sha_pair_compress(ShaPair& s, uint32_t w[16], bool A) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    const uint32_t r1 = A ? 2u : 6u, r2 = A ? 13u : 11u, r3 = A ? 22u : 25u;   // Sigma0 / Sigma1
    const uint32_t q1 = A ? 7u : 17u, q2 = A ? 18u : 19u, q3 = A ? 3u : 10u;   // sigma0 / sigma1
    const uint32_t mA = pair_mask();
    uint32_t v0 = s.h[0], v1 = s.h[1], v2 = s.h[2], v3 = s.h[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t e2 = w[(i - 2) & 15], a15 = w[(i - 15) & 15], w7 = w[(i - 7) & 15], w16 = w[i & 15];
            // words of constant messages (padding blocks) fold as in sha_compress
            const uint32_t s1c = crotr(e2, 17) ^ crotr(e2, 19) ^ (e2 >> 10);
            const uint32_t s0c = crotr(a15, 7) ^ crotr(a15, 18) ^ (a15 >> 3);
            if (__builtin_constant_p(s1c + s0c)) {
                wi = s1c + s0c + w7 + w16;
            } else {
                const uint32_t x = pair_sel(e2, a15);
                const uint32_t sg =
                    xor3(__builtin_amdgcn_alignbit(x, x, q1), __builtin_amdgcn_alignbit(x, x, q2), x >> q3);
                wi = pair_add(add3(sg, w7, w16), sg);
            }
            w[i & 15] = wi;
        }
        const uint32_t S = xor3(__builtin_amdgcn_alignbit(v0, v0, r1), __builtin_amdgcn_alignbit(v0, v0, r2),
                                __builtin_amdgcn_alignbit(v0, v0, r3));
        const uint32_t F = pair_chmaj(v0, v1, v2, mA);
        const uint32_t Y = pair_sel(v3 + K[i] + wi, 0u);
        const uint32_t T = add3(S, F, Y);
        const uint32_t nv = pair_add(T, pair_sel(T, v3));
        v3 = v2; v2 = v1; v1 = v0; v0 = nv;
    }
    s.h[0] += v0; s.h[1] += v1; s.h[2] += v2; s.h[3] += v3;
}

// The whole digest (H0..H7) in both lanes of the pair.
CDA_HD void sha_pair_digest(const ShaPair& s, bool A, uint32_t (&d)[8]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t o = pair_swap(s.h[j]);
        d[j] = pair_sel(o, s.h[j]);
        d[4 + j] = pair_sel(s.h[j], o);
    }
}


// ---------------------------------------------------------------------------
// Constant message prefixes.  Two hot messages start with constant words:
//   parity leaf, block 0:   0x00 || 0xFF*29 || share...   -> words 0..6
//   inner node whose left child is a parity subtree (min = max = 0xFF*29),
//   block 0:                0x01 || 0xFF*58 || hash...     -> words 0..13
// (3/4 of all leaves and of all inner nodes of an EDS).  The working state
// after those rounds is a compile-time constant (sha_mid), so the
// compression restarts at round R0 (sha_compress_from); schedule words that
// only involve the constant words fold at compile time.
// ---------------------------------------------------------------------------
struct ShaMid {
    uint32_t v[8];   // a..h after R0 rounds from the initial hash value
};
template <int R0>
constexpr ShaMid sha_mid(const uint32_t (&w)[16]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint32_t a = 0x6a09e667u, b = 0xbb67ae85u, c = 0x3c6ef372u, d = 0xa54ff53au;
    uint32_t e = 0x510e527fu, f = 0x9b05688cu, g = 0x1f83d9abu, h = 0x5be0cd19u;
    for (int i = 0; i < R0; i++) {
        const uint32_t S1 = crotr(e, 6) ^ crotr(e, 11) ^ crotr(e, 25);
        const uint32_t t1 = h + S1 + ((e & f) ^ (~e & g)) + K[i] + w[i];
        const uint32_t S0 = crotr(a, 2) ^ crotr(a, 13) ^ crotr(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    return ShaMid{{a, b, c, d, e, f, g, h}};
}
constexpr uint32_t kLeafParityHead[16] = {0x00FFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
constexpr uint32_t kNodeParityHead[16] = {0x01FFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
constexpr int kLeafParityRounds = 7;
constexpr int kNodeParityRounds = 14;
inline constexpr ShaMid kLeafParityMid = sha_mid<kLeafParityRounds>(kLeafParityHead);
inline constexpr ShaMid kNodeParityMid = sha_mid<kNodeParityRounds>(kNodeParityHead);

// First compression of a message whose words 0..R0-1 are HEAD (s holds the
// initial hash value); w[R0..15] are the variable words.  Schedule terms of
// constant words are computed with plain operators so they fold.
template <int R0>
CDA_HD void sha_compress_from(ShaState& s, const ShaMid& m, const uint32_t (&head)[16], uint32_t w[16]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
#pragma unroll
    for (int i = 0; i < R0; i++) w[i] = head[i];
    uint32_t a = m.v[0], b = m.v[1], c = m.v[2], d = m.v[3];
    uint32_t e = m.v[4], f = m.v[5], g = m.v[6], h = m.v[7];
    bool kc[16];   // w[j] known at compile time
#pragma unroll
    for (int j = 0; j < 16; j++) kc[j] = j < R0;
#pragma unroll
    for (int i = R0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const int j15 = (i - 15) & 15, j2 = (i - 2) & 15, j16 = i & 15, j7 = (i - 7) & 15;
            const uint32_t w15 = w[j15], w2 = w[j2];
            const uint32_t s0 = kc[j15] ? (crotr(w15, 7) ^ crotr(w15, 18) ^ (w15 >> 3))
                                        : xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = kc[j2] ? (crotr(w2, 17) ^ crotr(w2, 19) ^ (w2 >> 10))
                                       : xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[j16] + s0 + w[j7] + s1;
            kc[j16] = kc[j16] && kc[j15] && kc[j7] && kc[j2];
            w[j16] = wi;
        }
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t t1 = add3(add3(h, S1, ch(e, f, g)), K[i], wi);
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = add3(t1, S0, mj);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// ---------------------------------------------------------------------------
// Leaf: message word i (big-endian) of 0x00 || ns || share, given the share as
// big-endian words S[0..127] and `parity` (ns = 0xFF*29 instead of share[0:29]).
// Block b needs S[16b-8 .. 16b+8].
// ---------------------------------------------------------------------------
CDA_HD uint32_t leaf_msg_head(const uint32_t* S, bool parity, int i) {   // i in 0..7
    if (parity) {
        if (i == 0) return 0x00FFFFFFu;
        if (i < 7) return 0xFFFFFFFFu;
        return 0xFFFF0000u | (S[0] >> 16);
    }
    if (i == 0) return S[0] >> 8;
    if (i < 7) return funnel8(S[i - 1], S[i], 1);
    return (S[6] << 24) | ((S[7] >> 24) << 16) | (S[0] >> 16);
}
// i in 8..134: bytes 4i.. = share[4i-30 ..]
CDA_HD uint32_t leaf_msg_body(uint32_t s_im8, uint32_t s_im7) { return funnel8(s_im8, s_im7, 2); }
constexpr uint32_t kLeafMsgBits = 542 * 8;

// Leaf node slot words (little-endian u32 as stored in memory), from the ns
// big-endian words NSW[0..7] (byte 28 = NSW[7] >> 24) and digest D[0..7].
CDA_HD void leaf_node_words(const uint32_t NSW[8], const uint32_t D[8], uint32_t out[kSlotWords]) {
    uint32_t be[kSlotWords];
#pragma unroll
    for (int t = 0; t < 7; t++) be[t] = NSW[t];
    be[7] = (NSW[7] & 0xFF000000u) | (NSW[0] >> 8);
#pragma unroll
    for (int t = 8; t < 14; t++) be[t] = funnel8(NSW[t - 8], NSW[t - 7], 1);
    be[14] = (NSW[6] << 24) | ((NSW[7] >> 24) << 16) | (D[0] >> 16);
#pragma unroll
    for (int t = 15; t < 22; t++) be[t] = funnel8(D[t - 15], D[t - 14], 2);
    be[22] = D[7] << 16;
    be[23] = 0;
#pragma unroll
    for (int t = 0; t < kSlotWords; t++) out[t] = bswap32(be[t]);
}

// ---------------------------------------------------------------------------
// Inner node: L, R = big-endian words of the two child slots.  Message word i
// of 0x01 || l(90) || r(90) (181 B, 3 blocks = 48 words).
// ---------------------------------------------------------------------------
CDA_HD uint32_t node_msg(const uint32_t* L, const uint32_t* R, int i) {
    if (i == 0) return 0x01000000u | (L[0] >> 8);
    if (i < 22) return funnel8(L[i - 1], L[i], 1);
    if (i == 22) return (funnel8(L[21], L[22], 1) & 0xFFFFFF00u) | (R[0] >> 24);
    if (i < 45) return funnel8(R[i - 23], R[i - 22], 3);
    if (i == 45) return (R[22] << 8) | 0x00800000u;
    if (i == 47) return 181u * 8u;
    return 0;
}

CDA_HD bool is_parity_min(const uint32_t* R) {
    bool all = true;
#pragma unroll
    for (int t = 0; t < 7; t++) all = all && (R[t] == 0xFFFFFFFFu);
    return all && ((R[7] >> 24) == 0xFFu);
}

// Parent slot (little-endian words) from child big-endian words and digest.
CDA_HD void inner_node_words(const uint32_t* L, const uint32_t* R, const uint32_t D[8], uint32_t out[kSlotWords]) {
    const bool ign = is_parity_min(R);     // IgnoreMaxNamespace(true)
    uint32_t be[kSlotWords];
#pragma unroll
    for (int t = 0; t < 7; t++) be[t] = L[t];
    uint32_t x7 = ign ? L[7] : R[7];
    be[7] = (L[7] & 0xFF000000u) | (x7 & 0x00FFFFFFu);
#pragma unroll
    for (int t = 8; t < 14; t++) be[t] = ign ? L[t] : R[t];
    uint32_t x14 = ign ? L[14] : R[14];
    be[14] = (x14 & 0xFFFF0000u) | (D[0] >> 16);
#pragma unroll
    for (int t = 15; t < 22; t++) be[t] = funnel8(D[t - 15], D[t - 14], 2);
    be[22] = D[7] << 16;
    be[23] = 0;
#pragma unroll
    for (int t = 0; t < kSlotWords; t++) out[t] = bswap32(be[t]);
}

// 96-B node slots: big-endian word view on load, little-endian words on store.
CDA_HD void load_slot_be(const uint8_t* slot, uint32_t (&w)[kSlotWords]) {
    const uint4* p = reinterpret_cast<const uint4*>(slot);
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const uint4 v = p[q];
        w[4 * q + 0] = bswap32(v.x); w[4 * q + 1] = bswap32(v.y);
        w[4 * q + 2] = bswap32(v.z); w[4 * q + 3] = bswap32(v.w);
    }
}
CDA_HD void store_slot(uint8_t* slot, const uint32_t (&w)[kSlotWords]) {
    uint4* p = reinterpret_cast<uint4*>(slot);
#pragma unroll
    for (int q = 0; q < 6; q++) p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// ---------------------------------------------------------------------------
// RFC-6962 (go-square/merkle): leaf = sha256(0x00 || item90), inner =
// sha256(0x01 || a32 || b32).  I = big-endian words of a 96-B slot.
// ---------------------------------------------------------------------------
CDA_HD uint32_t rfc_leaf_msg(const uint32_t* I, int i) {   // 91 B, 2 blocks
    if (i == 0) return I[0] >> 8;
    if (i < 22) return funnel8(I[i - 1], I[i], 1);
    if (i == 22) return (funnel8(I[21], I[22], 1) & 0xFFFFFF00u) | 0x80u;
    if (i == 31) return 91u * 8u;
    return 0;
}
CDA_HD uint32_t rfc_inner_msg(const uint32_t* A, const uint32_t* B, int i) {   // 65 B, 2 blocks
    if (i == 0) return 0x01000000u | (A[0] >> 8);
    if (i < 8) return funnel8(A[i - 1], A[i], 1);
    if (i == 8) return (A[7] << 24) | (B[0] >> 8);
    if (i < 16) return funnel8(B[i - 9], B[i - 8], 1);
    if (i == 16) return (B[7] << 24) | 0x00800000u;
    if (i == 31) return 65u * 8u;
    return 0;
}

// ---------------------------------------------------------------------------
// SHA-256 of one unit: a thread (PAIR = false) or a lane pair (PAIR = true,
// sha_pair_compress: the latency-bound tails, where a wave per SIMD or fewer
// is all the work there is).  Every message word is computed by both lanes.
// ---------------------------------------------------------------------------
template <bool PAIR>
struct Sha;
template <>
struct Sha<false> {
    ShaState st;
    CDA_HD void init(bool) { sha_init(st); }
    CDA_HD void compress(uint32_t (&w)[16], bool) { sha_compress(st, w); }
    CDA_HD void digest(bool, uint32_t (&d)[8]) const {
#pragma unroll
        for (int j = 0; j < 8; j++) d[j] = st.h[j];
    }
};
template <>
struct Sha<true> {
    ShaPair st;
    CDA_HD void init(bool A) { sha_pair_init(st, A); }
    CDA_HD void compress(uint32_t (&w)[16], bool A) { sha_pair_compress(st, w, A); }
    CDA_HD void digest(bool A, uint32_t (&d)[8]) const { sha_pair_digest(st, A, d); }
};

// RFC-6962 leaf digest sha256(0x00 || slot[0:90]); I = big-endian slot words.
template <bool PAIR>
CDA_HD void rfc_leaf_u(const uint32_t (&I)[kSlotWords], uint32_t (&D)[8], bool A) {
    Sha<PAIR> h;
    h.init(A);
    uint32_t w[16];
#pragma unroll
    for (int b = 0; b < 2; b++) {
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rfc_leaf_msg(I, 16 * b + j);
        h.compress(w, A);
    }
    h.digest(A, D);
}
// ---------------------------------------------------------------------------
// RFC-6962 inner node, second block.  The 65-B message 0x01 || a || b leaves
// one data byte in block 1: b[31] || 0x80 || 0 ... || 520 (bits).  Its whole
// message schedule is a function of that byte, so K[t] + W[t] for all 64
// rounds is a 64 KiB compile-time table kRfcPadKW[byte][t] and the block runs
// its rounds with no schedule: 14 instead of ~21.5 VALU ops per round (the
// chains of the latency-bound data-root levels).
// ---------------------------------------------------------------------------
struct RfcPadTable {
    uint32_t kw[256][64];
};
constexpr RfcPadTable make_rfc_pad_table() {
    constexpr uint32_t K[64] = CDA_SHA_K;
    RfcPadTable t{};
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t w[64] = {};
        w[0] = (v << 24) | 0x00800000u;
        w[15] = 65u * 8u;
        for (int i = 16; i < 64; i++) {
            const uint32_t s0 = crotr(w[i - 15], 7) ^ crotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = crotr(w[i - 2], 17) ^ crotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        for (int i = 0; i < 64; i++) t.kw[v][i] = K[i] + w[i];
    }
    return t;
}
#if defined(__HIPCC__)
__device__ constexpr RfcPadTable kRfcPad = make_rfc_pad_table();
#endif

// 64 rounds over precomputed K + W words (kw: 16 x uint4 in registers).
CDA_HD void sha_compress_kw(ShaState& s, const uint4 (&kw)[16]) {
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint4 q = kw[i / 4];
        const uint32_t x = (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w;
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t t1 = add3(h, S1, ch(e, f, g)) + x;
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj(a, b, c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = add3(t1, S0, mj);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}
CDA_HD void sha_pair_compress_kw(ShaPair& s, const uint4 (&kw)[16], bool A) {
    const uint32_t r1 = A ? 2u : 6u, r2 = A ? 13u : 11u, r3 = A ? 22u : 25u;
    const uint32_t mA = pair_mask();
    uint32_t v0 = s.h[0], v1 = s.h[1], v2 = s.h[2], v3 = s.h[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint4 q = kw[i / 4];
        const uint32_t x = (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w;
        const uint32_t S = xor3(__builtin_amdgcn_alignbit(v0, v0, r1), __builtin_amdgcn_alignbit(v0, v0, r2),
                                __builtin_amdgcn_alignbit(v0, v0, r3));
        const uint32_t F = pair_chmaj(v0, v1, v2, mA);
        const uint32_t Y = pair_sel(v3 + x, 0u);
        const uint32_t T = add3(S, F, Y);
        const uint32_t nv = pair_add(T, pair_sel(T, v3));
        v3 = v2; v2 = v1; v1 = v0; v0 = nv;
    }
    s.h[0] += v0; s.h[1] += v1; s.h[2] += v2; s.h[3] += v3;
}

// K[t] + W[t] of all 64 rounds of one block (w: its 16 message words,
// consumed) into kw (64 words, 16-B aligned; e.g. LDS): the message schedule
// computed by a helper lane for sha_*_compress_kw on another wave.
CDA_HD void sha_schedule_kw(uint32_t (&w)[16], uint32_t* kw) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint4* q = reinterpret_cast<uint4*>(kw);
#pragma unroll
    for (int i = 0; i < 64; i += 4) {
        uint32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int t = i + r;
            uint32_t wi;
            if (t < 16) {
                wi = w[t];
            } else {
                const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wi = add3(w[t & 15], s0, w[(t - 7) & 15]) + s1;
                w[t & 15] = wi;
            }
            v[r] = K[t] + wi;
        }
        q[i / 4] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

#if defined(__HIPCC__)
// RFC-6962 inner digest sha256(0x01 || a || b) of two digests; block 1 from
// kRfcPad (its 256 B row: the first 64 B are loaded before block 0 runs, the
// rest 16 rounds ahead of use, so at most 32 table words are live).
template <bool PAIR>
CDA_HD void rfc_inner_u(const uint32_t (&a)[8], const uint32_t (&b)[8], uint32_t (&D)[8], bool A) {
    Sha<PAIR> h;
    h.init(A);
    const uint4* row = reinterpret_cast<const uint4*>(kRfcPad.kw[b[7] & 0xFFu]);
    uint4 kw[16];
#pragma unroll
    for (int q = 0; q < 4; q++) kw[q] = row[q];
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(a, b, j);
    h.compress(w, A);
#pragma unroll
    for (int q = 4; q < 16; q++) kw[q] = row[q];
    if constexpr (PAIR)
        sha_pair_compress_kw(h.st, kw, A);
    else
        sha_compress_kw(h.st, kw);
    h.digest(A, D);
}
#endif

// NMT HashNode of two child slots (big-endian words) into a parent slot
// (little-endian words), per thread or per lane pair; no mid-state branch
// (the tails mix data- and parity-left parents).
template <bool PAIR>
CDA_HD void hash_node_u(const uint32_t (&L)[kSlotWords], const uint32_t (&R)[kSlotWords],
                                            uint32_t (&o)[kSlotWords], bool A) {
    Sha<PAIR> h;
    h.init(A);
    uint32_t w[16], D[8];
#pragma unroll
    for (int b = 0; b < 3; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 16 * b + i);
        h.compress(w, A);
    }
    h.digest(A, D);
    inner_node_words(L, R, D, o);
}

}  // namespace cda
