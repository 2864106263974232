// rs_gf16.hip -- Leopard Reed-Solomon encode over GF(2^16) (k > 128).
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF16.encode (EXT, pinned at
// /root/reference/go.mod:152; selected by reedsolomon.New when data+parity
// shards > 256): the same IFFT(coset k)/FFT(coset 0) schedule as GF(2^8); symbol
// i of every 64-byte block is b[i] | b[i+32] << 8 (lo/hi split layout,
// leopard.go refMulAdd).
//
// MI355X mapping (k = 256, 512: rs16_cw_kernel).  One 1024-thread workgroup
// per codeword (k shards x 512 B).  A lane owns 4 symbols of every shard it
// holds: the lo dword at byte 64b+4q and the hi dword at 64b+32+4q of the
// shard (lane = 8b + q), so a wave spans the full 512-B shard width and all
// its lanes share every butterfly constant (wave-uniform tables in SGPRs).
//   pass A : wave w holds shards [S*w, S*w+S), S = k/16, and runs the IFFT
//            layers d < S in registers;
//   pass B : wave w holds the shards of R = S/16 residues r (r + S*t,
//            t = 0..15) and runs IFFT d = S..k/2 then FFT d = k/2..S;
//   pass A': FFT layers d < S, write parity.
// Passes A / A' run their groups depth-first (CDA_RS16_DFS, see grp_at): A
// consumes the shards as their loads return, A' stores each parity pair right
// after its last butterfly.
// The whole codeword stays in the workgroup's registers; the two layout
// changes are register all-to-alls between the 16 waves through 128 KiB of
// LDS (R rounds each way), so HBM sees only the data read, the optional Q0
// copy and the parity write.
//
// Multiply by a constant c: y is split into 3-bit chunks (bits 0-2, 3-5 and
// the 2-bit 6-7 of each byte); a 3-bit chunk selects one of 8 table bytes
// with v_perm_b32(src0 = SGPR dword, src1 = VGPR dword, sel), a 2-bit chunk
// one of 4 with v_perm_b32(T, T, sel): 12 perms + 10 selector ops + 6 XOR3
// per 4 symbols (mul_add16_c3; the 2-bit layout, -DCDA_RS16_CHUNK2, takes
// 16 + 14 + 8).
//
// k > 512 (and arbitrary shard lengths in rsmt2d Codec.Encode) use the
// LDS-staged log/exp kernel rs16_lds_kernel.
#include <type_traits>

#include "cda_kernels.h"

namespace cda {

namespace {

constexpr uint32_t kMod16 = 65535;

// ---------------------------------------------------------------------------
// register-resident codeword kernel
// ---------------------------------------------------------------------------
struct Chunk16 {   // tables of one constant: t[q][h], q = 2-bit chunk 0..7 of the symbol, h = output byte
    uint32_t t[16];
};

__device__ __forceinline__ uint32_t perm1(uint32_t t, uint32_t sel) { return __builtin_amdgcn_perm(t, t, sel); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// (xl, xh) ^= c * (yl, yh) for 4 symbols; tab = 16 dwords of the constant
// (uniform address -> scalar loads).
__device__ __forceinline__ void mul_add16(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh,
                                          const uint32_t* __restrict__ tab) {
    const uint32_t m = 0x03030303u;
    const uint32_t l0 = yl & m, l1 = (yl >> 2) & m, l2 = (yl >> 4) & m, l3 = (yl >> 6) & m;
    const uint32_t h0 = yh & m, h1 = (yh >> 2) & m, h2 = (yh >> 4) & m, h3 = (yh >> 6) & m;
    // t[2*q + 0] -> lo output byte, t[2*q + 1] -> hi output byte, q: chunks l0..l3 then h0..h3
    uint32_t a = xor3(perm1(tab[0], l0), perm1(tab[2], l1), perm1(tab[4], l2));
    uint32_t b = xor3(perm1(tab[6], l3), perm1(tab[8], h0), perm1(tab[10], h1));
    xl = xor3(xl, a, b);
    xl = xor3(xl, perm1(tab[12], h2), perm1(tab[14], h3));
    a = xor3(perm1(tab[1], l0), perm1(tab[3], l1), perm1(tab[5], l2));
    b = xor3(perm1(tab[7], l3), perm1(tab[9], h0), perm1(tab[11], h1));
    xh = xor3(xh, a, b);
    xh = xor3(xh, perm1(tab[13], h2), perm1(tab[15], h3));
}

__device__ __forceinline__ void mul_add16(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh,
                                          const uint32_t (&tab)[16]) {
    mul_add16(xl, xh, yl, yh, static_cast<const uint32_t*>(tab));
}

// 3-bit chunks (default layout, kGf16TabWords = 24): a 16-bit symbol splits
// into chunks at bits 0-2, 3-5, 6-7 of each byte; a 3-bit chunk indexes 8
// table bytes as v_perm(src0 = entries 4..7 in an SGPR, src1 = entries 0..3 in
// a VGPR, sel) -- gfx9 VOP3 reads one SGPR, so the four src1 dword pairs are
// read from LDS (staged per workgroup) once per butterfly group.  Per 4 symbols: 12 perms + 10
// selector ops + 6 XOR3 (2-bit layout: 16 + 14 + 8).
__device__ __forceinline__ uint32_t perm2(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ void mul_add16_c3(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh,
                                             const uint32_t (&t)[12], const uint32_t (&b)[8]) {
    const uint32_t m7 = 0x07070707u, m3 = 0x03030303u;
#ifndef CDA_RS16_NO_SHIFT64
    // one 64-bit shift serves both halves: the low dword's top bits take junk
    // from yh, which the byte masks drop
    const uint64_t y = (uint64_t)yl | ((uint64_t)yh << 32);
    uint64_t y3, y6;
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(y3) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(y6) : "v"(y));
    const uint32_t c0 = yl & m7, c1 = (uint32_t)y3 & m7, c2 = (uint32_t)y6 & m3;
    const uint32_t c3 = yh & m7, c4 = (uint32_t)(y3 >> 32) & m7, c5 = (uint32_t)(y6 >> 32) & m3;
#else
    const uint32_t c0 = yl & m7, c1 = (yl >> 3) & m7, c2 = (yl >> 6) & m3;
    const uint32_t c3 = yh & m7, c4 = (yh >> 3) & m7, c5 = (yh >> 6) & m3;
#endif
    xl = xor3(xl, perm2(t[0], b[0], c0), perm2(t[2], b[2], c1));
    xl = xor3(xl, perm1(t[8], c2), perm2(t[4], b[4], c3));
    xl = xor3(xl, perm2(t[6], b[6], c4), perm1(t[10], c5));
    xh = xor3(xh, perm2(t[1], b[1], c0), perm2(t[3], b[3], c1));
    xh = xor3(xh, perm1(t[9], c2), perm2(t[5], b[5], c3));
    xh = xor3(xh, perm2(t[7], b[7], c4), perm1(t[11], c5));
}

// tab layout: [skew index][kGf16TabWords dwords].  A skew equal to the modulus means
// "multiply by zero" (leopard skips the multiply); its tables are all zero, so
// the butterfly stays branch-free and bit-identical.
struct Tab16 {
    const uint32_t* __restrict__ t;      // [2k-1][16]
};

// Compile-time loops (full unroll with constant register indices: no
// s_set_gpr_idx register indexing, no scratch).
template <int B, int E, int STEP, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + STEP, E, STEP>(f);
    }
}

// In-register IFFT / FFT layers over N consecutive registers holding shards
// base + i*stride_abs; constant index of group g (register space) is
// IDX(g, d) (uniform).
//
// The N-1 butterfly groups of the layers run as one flat sequence whose
// table loads are software-pipelined: group I first waits for its own table
// dwords (loaded while group I-1 computed; the inline-asm wait), then issues
// the scalar loads of the next multiplying group's tables, then runs its
// butterflies.  Scalar loads return out of order, so waiting for one means
// waiting for all: issuing the next load only after the wait keeps it in
// flight across a whole group.
//
// Group order.  Breadth-first (layer by layer) or depth-first: the IFFT
// (d rising) in post-order -- both halves of a block before the block's own
// layer -- and the FFT (d falling) in pre-order.  Depth-first, pass A's
// butterflies consume the shards in the order their loads return (the first
// groups need registers 0-1 only, instead of layer 2 needing all 2S), and pass
// A' finishes registers in order, so each pair's parity store issues right
// after its last butterfly.
template <int N, bool INV, bool DFS = false>
constexpr int grp_at(int I, bool want_d) {
    if constexpr (!DFS) {
        for (int l = 0; l < 16; l++) {
            const int d = INV ? (1 << l) : ((N / 2) >> l);
            if (d < 1 || d >= N) break;
            const int ng = N / (2 * d);
            if (I < ng) return want_d ? d : 2 * d * I;
            I -= ng;
        }
        return -1;
    } else {
        struct Frame {
            int b, n, st;
        };
        Frame stk[20] = {};
        int sp = 0, cnt = 0;
        stk[sp++] = Frame{0, N, 0};
        while (sp) {
            Frame& f = stk[sp - 1];
            if (f.n < 2) {
                sp--;
            } else if (f.st == 0) {
                f.st = 1;
                if (!INV && cnt++ == I) return want_d ? f.n / 2 : f.b;
                stk[sp++] = Frame{f.b, f.n / 2, 0};
            } else if (f.st == 1) {
                f.st = 2;
                stk[sp++] = Frame{f.b + f.n / 2, f.n / 2, 0};
            } else {
                if (INV && cnt++ == I) return want_d ? f.n / 2 : f.b;
                sp--;
            }
        }
        return -1;
    }
}

template <int B, int E, int N>
__device__ __forceinline__ void launder(uint32_t (&lo)[N], uint32_t (&hi)[N]) {
    if constexpr (B < E) {
        asm volatile("" : "+v"(lo[B]), "+v"(hi[B]));
        launder<B + 1, E>(lo, hi);
    }
}

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
// 16 table dwords into SGPRs (a scalar-cache read; the caller waits).
__device__ __forceinline__ u32x16 sload16(const uint32_t* p) {
    u32x16 v;
    asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
// (with 3-bit chunks only dwords 0..11 are used from SGPRs; the src1 halves,
// dwords 12..19, are staged in LDS per workgroup and read as VGPRs)
struct TabRegs {
    u32x16 a;
};
__device__ __forceinline__ TabRegs load_tabs(const uint32_t* p) {
    TabRegs r;
    r.a = sload16(p);
    return r;
}
// Passes A / A' read both table halves of every constant from LDS (20-dword
// records: src0 dwords 0..11, src1 12..19) instead of a scalar load per
// group, and the exchanges move lo and hi registers in separate 64 KiB rounds
// to make room (128 + 80 KiB would not fit).  The per-wave constants of those
// passes (16 waves x 31 groups x 96 B) do not fit the scalar cache, so every
// scalar load was an L2 round trip, and scalar loads return out of order, so
// they could not be prefetched deeper than one group: all waves of a SIMD
// waited together (round 2).  LDS reads are in order, never
// miss, and the compiler schedules them ahead.  Measured -54 us per k = 512
// square (1.218 -> 1.162 ms, profiles/r03c/ldsa_ab.txt).  CDA_RS16_LDS_A=0
// builds the round-2 scalar-load form (A/B).
#ifndef CDA_RS16_LDS_A
#define CDA_RS16_LDS_A 1
#endif
// CDA_RS16_LDS_B=1 (experiment, needs LDS_A): pass B's tables from LDS as well
#ifndef CDA_RS16_LDS_B
#define CDA_RS16_LDS_B 0
#endif
constexpr uint32_t kTbStride = CDA_RS16_LDS_A ? 20 : 8;   // dwords per constant in the LDS table
constexpr uint32_t kTbSrc1 = CDA_RS16_LDS_A ? 12 : 0;     // offset of the src1 halves in a record
struct TabB {   // src1 halves of one constant, [a][lo/hi] as 8 dwords
    uint4 b0, b1;
};
// plane != 0: plane-major records (chunk q of record idx at TB + 4 idx +
// q plane dwords; rs16_half_kernel), else record-major (kTbStride apart)
__device__ __forceinline__ TabB load_tab_b(const uint32_t* TB, uint32_t idx, uint32_t plane = 0) {
    if (plane) {
        const uint32_t* p = TB + 4 * idx;
        return TabB{*reinterpret_cast<const uint4*>(p + 3 * plane), *reinterpret_cast<const uint4*>(p + 4 * plane)};
    }
    const uint4* p = reinterpret_cast<const uint4*>(TB + idx * kTbStride + kTbSrc1);
    return TabB{p[0], p[1]};
}

// Leopard skips the multiply when the skew is the modulus (log 0).  The FFT
// skew of index 2^j - 1 is always the modulus (initFFT sets skew[(1<<m)-1] = 0
// before taking logs), and in pass B every FFT group with gt = 0 has index
// S*dt - 1: ZERO_G0 drops those multiplies at compile time (480 of the 4 608
// butterfly multiplies of a k = 512 codeword); their tables are all zero, so
// the result is bit-identical either way.
template <int N, bool INV, bool ZERO_G0, bool DFS = false>
constexpr bool grp_mul(int I) {
    return I < N - 1 && !(ZERO_G0 && grp_at<N, INV, DFS>(I, false) == 0);
}
template <int N, bool INV, bool ZERO_G0, bool DFS = false>
constexpr int next_mul(int I) {
    int J = I + 1;
    while (J < N - 1 && !grp_mul<N, INV, ZERO_G0, DFS>(J)) J++;
    return J;
}

struct NoFin {   // layers_regs hook: register i holds its final value
    template <class I>
    __device__ __forceinline__ void operator()(I) const {}
};

// M independent register sets of N shards (pass B's residues) share every
// butterfly constant: one table load and one VGPR copy per group serve all M.
// lidxf (optional): index of a group's constant relative to TB, when TB
// already includes a runtime (per-wave) base -- then the LDS reads are one
// VGPR base + immediate offsets instead of an SGPR address copied to a VGPR
// per group.
template <int N, bool INV, bool ZERO_G0 = false, int M = 1, bool DFS = false, class IdxF, class Fin = NoFin,
          class LIdxF = std::nullptr_t>
__device__ __forceinline__ void layers_regs(uint32_t (&lo)[M * N], uint32_t (&hi)[M * N], const Tab16& T,
                                            const uint32_t* TB, IdxF idxf, Fin fin = Fin{}, LIdxF lidxf = nullptr,
                                            uint32_t plane = 0) {
    static_assert(!(INV && ZERO_G0), "only FFT groups have structural zero skews");
    constexpr int NG = N - 1;
    // The scalar loads are issued from inline asm: the compiler treats loads
    // of the (invariant) tables as freely movable and would sink a plain load
    // back next to its first use.  The wait is explicit for the same reason.
    // group positions are constant-evaluated here (the depth-first search does
    // not fold as a runtime call), so the table addresses stay scalar
    auto tab_ptr = [&](auto II) {
        constexpr int g = grp_at<N, INV, DFS>(decltype(II)::value, false);
        constexpr int d = grp_at<N, INV, DFS>(decltype(II)::value, true);
        return T.t + (size_t)idxf(g, d) * kGf16TabWords;
    };
    auto tab_idx = [&](auto II) {
        constexpr int g = grp_at<N, INV, DFS>(decltype(II)::value, false);
        constexpr int d = grp_at<N, INV, DFS>(decltype(II)::value, true);
        if constexpr (std::is_same_v<LIdxF, std::nullptr_t>)
            return idxf(g, d);
        else
            return lidxf(g, d);
    };
    constexpr int F0 = next_mul<N, INV, ZERO_G0, DFS>(-1);
    using F0c = std::integral_constant<int, (F0 < NG ? F0 : 0)>;
    TabRegs tc{};
    if constexpr (F0 < NG) tc = load_tabs(tab_ptr(F0c{}));
#ifndef CDA_RS16_CHUNK2
    TabB bc{};
    if constexpr (F0 < NG) bc = load_tab_b(TB, tab_idx(F0c{}), plane);
#endif
    sfor<0, NG, 1>([&](auto II) {
        constexpr int I = decltype(II)::value;
        constexpr int g = grp_at<N, INV, DFS>(I, false), d = grp_at<N, INV, DFS>(I, true);
        if constexpr (!grp_mul<N, INV, ZERO_G0, DFS>(I)) {
            sfor<0, M, 1>([&](auto mm) {
                sfor<g, g + d, 1>([&](auto ii) {      // multiply by zero: XOR only
                    constexpr int i = N * decltype(mm)::value + decltype(ii)::value;
                    lo[i + d] ^= lo[i];
                    hi[i + d] ^= hi[i];
                });
            });
            if constexpr (!INV && d == 1 && M == 1) {
                fin(std::integral_constant<int, g>{});
                fin(std::integral_constant<int, g + 1>{});
            }
        } else {
            constexpr int J = next_mul<N, INV, ZERO_G0, DFS>(I);
            using Jc = std::integral_constant<int, (J < NG ? J : 0)>;
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(tc.a)::"memory");   // this group's tables are here
            TabRegs tn;
            if constexpr (J < NG) tn = load_tabs(tab_ptr(Jc{}));
#ifndef CDA_RS16_CHUNK2
            TabB bn;
            if constexpr (J < NG) bn = load_tab_b(TB, tab_idx(Jc{}), plane);
#endif
            // the group's operands pass through volatile asm after the load, so
            // the scheduler cannot hoist the butterflies above it
#ifndef CDA_RS16_NOLAUNDER
            sfor<0, M, 1>([&](auto mm) {
                launder<N * decltype(mm)::value + g, N * decltype(mm)::value + g + 2 * d>(lo, hi);
            });
#endif
#ifdef CDA_RS16_CHUNK2
            uint32_t t[16];
#pragma unroll
            for (int j = 0; j < 16; j++) t[j] = tc.a[j];
#else
            uint32_t t[12];
#pragma unroll
            for (int j = 0; j < 12; j++) t[j] = tc.a[j];
            const uint32_t bv[8] = {bc.b0.x, bc.b0.y, bc.b0.z, bc.b0.w, bc.b1.x, bc.b1.y, bc.b1.z, bc.b1.w};
#endif
            auto mul = [&](uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh) {
#ifdef CDA_RS16_CHUNK2
                mul_add16(xl, xh, yl, yh, t);
#else
                mul_add16_c3(xl, xh, yl, yh, t, bv);
#endif
            };
            sfor<0, M, 1>([&](auto mm) {
                sfor<g, g + d, 1>([&](auto ii) {
                    constexpr int i = N * decltype(mm)::value + decltype(ii)::value;
                    if constexpr (INV) {
                        hi[i + d] ^= hi[i];
                        lo[i + d] ^= lo[i];
                        mul(lo[i], hi[i], lo[i + d], hi[i + d]);
                    } else {
                        mul(lo[i], hi[i], lo[i + d], hi[i + d]);
                        lo[i + d] ^= lo[i];
                        hi[i + d] ^= hi[i];
                    }
                });
            });
            if constexpr (!INV && d == 1 && M == 1) {
                fin(std::integral_constant<int, g>{});
                fin(std::integral_constant<int, g + 1>{});
            }
            if constexpr (J < NG) {
                tc = tn;
#ifndef CDA_RS16_CHUNK2
                bc = bn;
#endif
            }
        }
    });
}
// Passes A / A' with every table dword from LDS (CDA_RS16_LDS_A): per group
// five 16-B reads of the constant's record at TB (+ lidxf(g, d) records), no
// scalar loads; the compiler schedules the reads (in order, LDS-latency).
template <int N, bool INV, bool DFS, class LIdxF, class Fin = NoFin, int M = 1, bool ZERO_G0 = false>
__device__ __forceinline__ void layers_regs_lds(uint32_t (&lo)[M * N], uint32_t (&hi)[M * N], const uint32_t* TB,
                                                LIdxF lidxf, Fin fin = Fin{}, uint32_t plane = 0) {
    constexpr int NG = N - 1;
    sfor<0, NG, 1>([&](auto II) {
        constexpr int I = decltype(II)::value;
        constexpr int g = grp_at<N, INV, DFS>(I, false), d = grp_at<N, INV, DFS>(I, true);
        if constexpr (!grp_mul<N, INV, ZERO_G0, DFS>(I)) {   // multiply by zero: XOR only
            sfor<0, M, 1>([&](auto mm) {
                sfor<g, g + d, 1>([&](auto ii) {
                    constexpr int i = N * decltype(mm)::value + decltype(ii)::value;
                    lo[i + d] ^= lo[i];
                    hi[i + d] ^= hi[i];
                });
            });
        } else {
            uint4 q0, q1, q2, q3, q4;
            if (plane) {   // one VGPR base, the planes as immediate offsets
                const uint32_t* p = TB + 4 * lidxf(g, d);
                q0 = *reinterpret_cast<const uint4*>(p);
                q1 = *reinterpret_cast<const uint4*>(p + plane);
                q2 = *reinterpret_cast<const uint4*>(p + 2 * plane);
                q3 = *reinterpret_cast<const uint4*>(p + 3 * plane);
                q4 = *reinterpret_cast<const uint4*>(p + 4 * plane);
            } else {
                const uint4* p = reinterpret_cast<const uint4*>(TB + lidxf(g, d) * kTbStride);
                q0 = p[0]; q1 = p[1]; q2 = p[2]; q3 = p[3]; q4 = p[4];
            }
            const uint32_t t[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            const uint32_t bv[8] = {q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, q4.z, q4.w};
            sfor<0, M, 1>([&](auto mm) {
                sfor<g, g + d, 1>([&](auto ii) {
                    constexpr int i = N * decltype(mm)::value + decltype(ii)::value;
                    if constexpr (INV) {
                        hi[i + d] ^= hi[i];
                        lo[i + d] ^= lo[i];
                        mul_add16_c3(lo[i], hi[i], lo[i + d], hi[i + d], t, bv);
                    } else {
                        mul_add16_c3(lo[i], hi[i], lo[i + d], hi[i + d], t, bv);
                        lo[i + d] ^= lo[i];
                        hi[i + d] ^= hi[i];
                    }
                });
            });
        }
        if constexpr (!INV && d == 1 && M == 1) {
            fin(std::integral_constant<int, g>{});
            fin(std::integral_constant<int, g + 1>{});
        }
    });
}

#ifndef CDA_RS16_DFS
#define CDA_RS16_DFS 1
#endif
constexpr bool kRs16Dfs = CDA_RS16_DFS != 0;
template <int N, class IdxF, class LIdxF>
__device__ __forceinline__ void ifft_regs(uint32_t (&lo)[N], uint32_t (&hi)[N], const Tab16& T, const uint32_t* TB,
                                          IdxF idxf, LIdxF lidxf) {
    if constexpr (CDA_RS16_LDS_A)
        layers_regs_lds<N, true, kRs16Dfs>(lo, hi, TB, lidxf);
    else
        layers_regs<N, true, false, 1, kRs16Dfs>(lo, hi, T, TB, idxf, NoFin{}, lidxf);
}
template <int N, class IdxF, class Fin, class LIdxF>
__device__ __forceinline__ void fft_regs(uint32_t (&lo)[N], uint32_t (&hi)[N], const Tab16& T, const uint32_t* TB,
                                         IdxF idxf, Fin fin, LIdxF lidxf) {
    if constexpr (CDA_RS16_LDS_A)
        layers_regs_lds<N, false, kRs16Dfs>(lo, hi, TB, lidxf, fin);
    else
        layers_regs<N, false, false, 1, kRs16Dfs>(lo, hi, T, TB, idxf, fin, lidxf);
}

// exchange buffer: [src wave][dst wave][lo/hi][lane] dwords (LDS_A: lo and
// hi in separate rounds, [src][dst][lane])
constexpr uint32_t kXchgBytes = 16 * 16 * (CDA_RS16_LDS_A ? 1 : 2) * 64 * 4;
// + the src1 table halves of the 2K-1 constants, 32 B each (K = 512: 160 KiB total)
template <int K>
constexpr uint32_t cw_lds_bytes() {
#ifdef CDA_RS16_CHUNK2
    return kXchgBytes;
#else
    return kXchgBytes + (2 * K - 1) * kTbStride * 4;
#endif
}


}  // namespace

namespace {

template <int K>
__global__ __launch_bounds__(1024) void rs16_cw_kernel(const uint32_t* __restrict__ tab, const RsJob job) {
    rs_err_init(job);
    extern __shared__ uint32_t X[];
    constexpr int S = K / 16;      // shards per lane in pass A
    constexpr int R = S / 16;      // residues per wave in pass B
    const Tab16 T{tab};
    // the table region's LDS address as a VGPR (not a folded constant), so
    // every table read below is this base (+ a per-wave offset, one v_add
    // per pass) with the constant's index in the instruction's offset field
    uint32_t tb_addr = kXchgBytes;
    asm volatile("" : "+v"(tb_addr));
    const uint32_t* TB = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(X) + tb_addr);
#ifndef CDA_RS16_CHUNK2
    {   // stage dwords 12..19 of every constant's record (its src1 halves)
        uint32_t* tb = X + kXchgBytes / 4;
        for (uint32_t i = threadIdx.x; i < 2 * K - 1; i += 1024) {
            if constexpr (CDA_RS16_LDS_A) {   // the whole record: dwords 0..19
                const uint4* src = reinterpret_cast<const uint4*>(tab + (size_t)i * kGf16TabWords);
                uint4* dst = reinterpret_cast<uint4*>(tb + i * kTbStride);
#pragma unroll
                for (int q = 0; q < 5; q++) dst[q] = src[q];
            } else {
                const uint4* src = reinterpret_cast<const uint4*>(tab + (size_t)i * kGf16TabWords + 12);
                uint4* dst = reinterpret_cast<uint4*>(tb + i * 8);
                dst[0] = src[0];
                dst[1] = src[1];
            }
        }
        __syncthreads();
    }
#endif
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t off = 64 * (lane >> 3) + 4 * (lane & 7);    // lo dword; hi at +32
    // All addressing is a uniform base pointer + a 32-bit byte offset (one
    // VGPR per access, saddr form), so no 64-bit address pairs stay live.
    const bool s1 = job.n_seg > 1 && blockIdx.x >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = s1 ? blockIdx.x - job.seg[0].n_cw : blockIdx.x;
    const uint8_t* src_base = job.src + blockIdx.y * job.src_sq;
    uint8_t* E = job.dst + blockIdx.y * job.dst_sq;
    const uint32_t s0 = g.src_off + c * g.src_cw, ss = g.src_sh;      // data shard i
    const uint32_t d0 = g.dst_off + c * g.dst_cw, ds = g.dst_sh;      // parity / scratch shard i
    const uint32_t c0 = g.cpy_off == kNoCopy ? kNoCopy : g.cpy_off + c * g.cpy_cw;
    // A shard's uniform byte offset is added to the base pointer in SGPRs
    // (SALU) at the use site -- laundered there, so the compiler neither keeps
    // dozens of per-shard pointers live nor moves the add into VALU -- and
    // every access is that pointer + the lane's fixed VGPR offset (saddr).
    auto ld = [&](const uint8_t* base, uint32_t o, uint32_t& l, uint32_t& h) {
        asm volatile("" : "+s"(o));
        const uint8_t* p = base + o;
        l = *reinterpret_cast<const uint32_t*>(p + off);
        h = *reinterpret_cast<const uint32_t*>(p + off + 32);
    };
    auto st = [&](uint8_t* base, uint32_t o, uint32_t l, uint32_t h) {
        asm volatile("" : "+s"(o));
        uint8_t* p = base + o;
        *reinterpret_cast<uint32_t*>(p + off) = l;
        *reinterpret_cast<uint32_t*>(p + off + 32) = h;
    };

    // The whole codeword (K shards x 512 B = 256 KiB at K = 512) stays in the
    // workgroup's registers: 2S dwords per lane.  The layout changes between
    // the passes go through 128 KiB of LDS in R rounds; round q moves the
    // registers j = R*jj + q (jj = 0..15) of every wave t to wave jj, where
    // they become residue R*jj + q's shard t -- in place, so pass B's
    // residue q lives in registers {R*t + q}.
    uint32_t lo[S], hi[S];
    auto xbar = [] { __syncthreads(); };
    // CDA_RS16_LDS_A: the lo and hi registers of a round move in two
    // sub-rounds through a 64 KiB buffer ([src][dst][lane])
    constexpr int NH = CDA_RS16_LDS_A ? 2 : 1;   // sub-rounds per round
    auto xw = [&](uint32_t src_w, uint32_t dst_w, int h) -> uint32_t& {
        if constexpr (CDA_RS16_LDS_A)
            return X[(src_w * 16 + dst_w) * 64 + lane];
        else
            return X[((src_w * 16 + dst_w) * 2 + h) * 64 + lane];
    };
    auto xchg_a_to_b = [&]() {
        sfor<0, R * NH, 1>([&](auto qh) {
            constexpr int q = decltype(qh)::value / NH, hh = decltype(qh)::value % NH;
            if (decltype(qh)::value) xbar();
            sfor<0, 16, 1>([&](auto jj) {
                constexpr int j = R * decltype(jj)::value + q;
                if (NH == 1 || hh == 0) xw(wave, jj.value, 0) = lo[j];
                if (NH == 1 || hh == 1) xw(wave, jj.value, 1) = hi[j];
            });
            xbar();
            sfor<0, 16, 1>([&](auto tt) {
                constexpr int j = R * decltype(tt)::value + q;
                if (NH == 1 || hh == 0) lo[j] = xw(tt.value, wave, 0);
                if (NH == 1 || hh == 1) hi[j] = xw(tt.value, wave, 1);
            });
        });
    };
    auto xchg_b_to_a = [&]() {
        sfor<0, R * NH, 1>([&](auto qh) {
            constexpr int q = decltype(qh)::value / NH, hh = decltype(qh)::value % NH;
            xbar();
            sfor<0, 16, 1>([&](auto tt) {
                constexpr int j = R * decltype(tt)::value + q;
                if (NH == 1 || hh == 0) xw(tt.value, wave, 0) = lo[j];
                if (NH == 1 || hh == 1) xw(tt.value, wave, 1) = hi[j];
            });
            xbar();
            sfor<0, 16, 1>([&](auto jj) {
                constexpr int j = R * decltype(jj)::value + q;
                if (NH == 1 || hh == 0) lo[j] = xw(wave, jj.value, 0);
                if (NH == 1 || hh == 1) hi[j] = xw(wave, jj.value, 1);
            });
        });
    };

    // ---------------- pass A: IFFT d = 1 .. S/2 -------------------------
    const uint32_t base = S * wave;
    sfor<0, S, 1>([&](auto jj) { ld(src_base, s0 + (base + jj.value) * ss, lo[jj.value], hi[jj.value]); });
    if (c0 != kNoCopy) {
        sfor<0, S, 1>([&](auto jj) { st(E, c0 + (base + jj.value) * g.cpy_sh, lo[jj.value], hi[jj.value]); });
    }
    // `base` is re-laundered per table index (like lane_off) so the compiler
    // does not precompute all S-1 group addresses up front and spill them
    auto wave_base = [&]() {
        uint32_t b = base;
        asm volatile("" : "+s"(b));
        return b;
    };
    ifft_regs<S>(lo, hi, T, TB + kTbStride * S * wave, [&](int g, int d) { return (uint32_t)(K - 1 + g + d) + wave_base(); },
                     [](int g, int d) { return (uint32_t)(K - 1 + g + d); });
    xchg_a_to_b();
    // ---------------- pass B: IFFT d = S .. K/2, FFT d = K/2 .. S --------
    // residue R*wave + q: shards R*wave + q + S*t in registers R*t + q
    // all R residues go through each butterfly group together (same constants)
    {
        uint32_t lr[R * 16], hr[R * 16];
        sfor<0, R, 1>([&](auto qq) {
            constexpr int q = decltype(qq)::value;
            sfor<0, 16, 1>([&](auto tt) {
                lr[16 * q + tt.value] = lo[R * tt.value + q];
                hr[16 * q + tt.value] = hi[R * tt.value + q];
            });
        });
        auto fi = [](int gt, int dt) { return (uint32_t)(K - 1 + S * gt + S * dt); };
        auto ff = [](int gt, int dt) { return (uint32_t)(S * gt + S * dt - 1); };
        if constexpr (CDA_RS16_LDS_B) {   // the (uniform) pass-B tables from LDS too
            layers_regs_lds<16, true, false, decltype(fi), NoFin, R, false>(lr, hr, TB, fi);
            layers_regs_lds<16, false, false, decltype(ff), NoFin, R, true>(lr, hr, TB, ff);
        } else {
            layers_regs<16, true, false, R>(lr, hr, T, TB, fi);
            layers_regs<16, false, true, R>(lr, hr, T, TB, ff);
        }
        sfor<0, R, 1>([&](auto qq) {
            constexpr int q = decltype(qq)::value;
            sfor<0, 16, 1>([&](auto tt) {
                lo[R * tt.value + q] = lr[16 * q + tt.value];
                hi[R * tt.value + q] = hr[16 * q + tt.value];
            });
        });
    }
    xchg_b_to_a();
    // ---------------- pass A': FFT d = S/2 .. 1, write parity -------------
    // parity shard j is stored as soon as its last butterfly is done
    auto store_j = [&](auto jj) { st(E, d0 + (base + jj.value) * ds, lo[jj.value], hi[jj.value]); };
    fft_regs<S>(lo, hi, T, TB + kTbStride * S * wave, [&](int g, int d) { return (uint32_t)(g + d - 1) + wave_base(); },
                store_j, [](int g, int d) { return (uint32_t)(g + d - 1); });
}

// ---------------------------------------------------------------------------
// Half-width codeword kernel (default for k = 256 / 512): TWO 512-thread
// workgroups per codeword, workgroup H taking bytes [256H, 256H + 256) of
// every shard (Leopard is independent per symbol position).  Each half is the
// 16-wave schedule above with a "virtual wave" v = 2w + (lane >> 5) of 32
// lanes in place of a hardware wave: v holds shards [S*v, S*v + S) in pass A /
// A' and R residues in pass B, exactly as before, so the passes, constants and
// exchanges are unchanged -- only which lanes hold what.  What changes is the
// occupancy: at <= 128 VGPRs two independent workgroups share a CU, so one's
// exchanges, barrier skew and codeword load / store phases are filled by the
// other's butterflies (the full-width kernel fills a CU with one workgroup, and
// all four waves of a SIMD stalled together at its barriers).
// LDS per workgroup (k = 512: 74.5 KiB, two per CU): one 32 KiB exchange
// sub-round, the records of ONE transform's K constants at a time (the IFFT's
// for pass A, restaged with the FFT's during pass B for pass A') and the 30
// constants of pass B.
// ---------------------------------------------------------------------------
constexpr uint32_t kHalfXchgBytes = 16 * 16 * 32 * 4;
// pass A' records restaged by LDS-DMA (global_load_lds_dwordx4) instead of
// through registers (A/B: -DCDA_RS16_GLDS=0)
#ifndef CDA_RS16_GLDS
#define CDA_RS16_GLDS 1
#endif
constexpr uint32_t kHalfPbRecords = CDA_RS16_GLDS ? 64 : 32;   // pass-B record slots (30 used)
template <int K>
constexpr uint32_t half_lds_bytes() {
    return kHalfXchgBytes + (K + kHalfPbRecords) * kTbStride * 4;
}
// 16 B from global to LDS by LDS-DMA: lane l's bytes land at lds + 16 l
// (lds wave-uniform).  Inline asm, not the builtin: the compiler drains every
// outstanding vector-memory op (vmcnt(0)) before the next LDS read after a
// builtin LDS-DMA -- here the next table or exchange read, long before these
// bytes are needed.  The caller waits for them itself (an explicit vmcnt
// before the barrier that publishes them); the compiler's own vmcnt counts
// stay safe, since these ops are older or extra, never fewer.  M0 is
// compiler-reserved, so it is saved and restored in the same statement.
// Source: a uniform base (SGPRs) + a per-lane 32-bit byte offset (one VGPR).
__device__ __forceinline__ void glds16(const uint32_t* base, uint32_t lane_off, const uint32_t* lds) {
    const uint32_t dst = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)lds;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(lane_off), "s"(base), "s"(__builtin_amdgcn_readfirstlane(dst))
        : "memory");
}
// one 80-B constant record (dwords 0..19 of the global 24-dword record) into LDS
__device__ __forceinline__ void stage_record(uint32_t* dst, const uint32_t* __restrict__ tab, uint32_t idx) {
    const uint4* s = reinterpret_cast<const uint4*>(tab + (size_t)idx * kGf16TabWords);
    uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (int q = 0; q < 5; q++) d[q] = s[q];
}

template <int K>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void rs16_half_kernel(
    const uint32_t* __restrict__ tab, const RsJob job) {
    static_assert(CDA_RS16_LDS_A, "the half-width kernel reads passes A / A' tables from LDS");
    rs_err_init(job);
    extern __shared__ uint32_t X[];
    constexpr int S = K / 16;      // shards per virtual wave in pass A
    constexpr int R = S / 16;      // residues per virtual wave in pass B
    constexpr uint32_t kTA = kHalfXchgBytes / 4;                  // dword offset: this transform's K records
    constexpr uint32_t kTPB = kTA + K * kTbStride;                // the pass-B records
    const Tab16 T{tab};
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63, hv = lane >> 5, sl = lane & 31;
    const uint32_t v = 2 * wave + hv;   // virtual wave (per lane)
    const bool s1 = job.n_seg > 1 && (blockIdx.x >> 1) >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = s1 ? (blockIdx.x >> 1) - job.seg[0].n_cw : (blockIdx.x >> 1);
    const uint8_t* src_base = job.src + (size_t)blockIdx.y * job.src_sq;
    uint8_t* E = job.dst + (size_t)blockIdx.y * job.dst_sq;
    // lane's lo dword in its shard (hi at +32), plus its virtual wave's shard
    // offset: the uniform part of every address is base + (2S*wave + j)*stride
    const uint32_t off = 256 * (blockIdx.x & 1) + 64 * (sl >> 3) + 4 * (sl & 7);
    const uint32_t ss = g.src_sh, ds = g.dst_sh;
    const uint32_t lsrc = off + S * hv * ss, ldst = off + S * hv * ds, lcpy = off + S * hv * g.cpy_sh;
    const uint32_t s0 = g.src_off + c * g.src_cw, d0 = g.dst_off + c * g.dst_cw;
    const uint32_t c0 = g.cpy_off == kNoCopy ? kNoCopy : g.cpy_off + c * g.cpy_cw;
    auto ld = [&](const uint8_t* base, uint32_t o, uint32_t& l, uint32_t& h) {
        asm volatile("" : "+s"(o));
        const uint8_t* p = base + o;
        l = *reinterpret_cast<const uint32_t*>(p + lsrc);
        h = *reinterpret_cast<const uint32_t*>(p + lsrc + 32);
    };
    auto st = [&](uint8_t* base, uint32_t o, uint32_t lo_off, uint32_t l, uint32_t h) {
        asm volatile("" : "+s"(o));
        uint8_t* p = base + o;
        *reinterpret_cast<uint32_t*>(p + lo_off) = l;
        *reinterpret_cast<uint32_t*>(p + lo_off + 32) = h;
    };

    uint32_t lo[S], hi[S];
    auto xbar = [] { __syncthreads(); };
    // exchange sub-round buffer [src v][dst v][32 lanes]; lo and hi registers
    // of a round move in two sub-rounds.  Round q moves registers R*jj + q of
    // virtual wave t to virtual wave jj (in place: pass B's residue q lives in
    // registers {R*t + q}).
    auto xw = [&](uint32_t src_v, uint32_t dst_v) -> uint32_t& { return X[(src_v * 16 + dst_v) * 32 + sl]; };
    // after_first: runs once every wave is past pass A (the first barrier)
    auto xchg_a_to_b = [&](auto after_first) {
        sfor<0, R * 2, 1>([&](auto qh) {
            constexpr int q = decltype(qh)::value / 2, hh = decltype(qh)::value % 2;
            if (decltype(qh)::value) xbar();
            sfor<0, 16, 1>([&](auto jj) {
                constexpr int j = R * decltype(jj)::value + q;
                xw(v, jj.value) = hh ? hi[j] : lo[j];
            });
            xbar();
            if constexpr (decltype(qh)::value == 0) after_first();
            sfor<0, 16, 1>([&](auto tt) {
                constexpr int j = R * decltype(tt)::value + q;
                (hh ? hi[j] : lo[j]) = xw(tt.value, v);
            });
        });
    };
    auto xchg_b_to_a = [&]() {
#if CDA_RS16_GLDS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's restage DMA (glds16)
#endif
        sfor<0, R * 2, 1>([&](auto qh) {
            constexpr int q = decltype(qh)::value / 2, hh = decltype(qh)::value % 2;
            xbar();
            sfor<0, 16, 1>([&](auto tt) {
                constexpr int j = R * decltype(tt)::value + q;
                xw(tt.value, v) = hh ? hi[j] : lo[j];
            });
            xbar();
            sfor<0, 16, 1>([&](auto jj) {
                constexpr int j = R * decltype(jj)::value + q;
                (hh ? hi[j] : lo[j]) = xw(v, jj.value);
            });
        });
    };

    // per-lane LDS base of the virtual wave's records (a VGPR: v is per lane)
    const uint32_t* TBv = X + kTA + (CDA_RS16_GLDS ? 4u : kTbStride) * S * v;
    // Records in LDS: a transform's K records at kTA (position i = the IFFT's
    // constant K-1+i for pass A, the FFT's constant i for pass A'); pass B's
    // at kTPB (position p = gt + dt in 1..15: IFFT constant K-1+S*p; 16 + p:
    // FFT constant S*p-1).  An 80-B record is five 16-B chunks; with
    // CDA_RS16_GLDS they are stored plane-major (chunk q of record i at
    // 16 i + q * plane bytes), so one LDS-DMA wave-instruction moves chunk q
    // of 64 consecutive records (lane = record: a per-lane source offset of
    // 96 * lane), and a record read is still one VGPR base + immediates.
#if CDA_RS16_GLDS
    constexpr uint32_t kPlaneA = 4 * K, kPlaneB = 4 * kHalfPbRecords;   // dwords
    auto dma_records = [&](uint32_t first) {
        constexpr uint32_t kPerPlane = K / 64, kInsts = 5 * kPerPlane;
        const uint32_t lane96 = 96 * lane;
        for (uint32_t m = wave; m < kInsts; m += 8) {
            const uint32_t q = m / kPerPlane, i0 = (m % kPerPlane) * 64;
            glds16(tab + (size_t)(first + i0) * kGf16TabWords + 4 * q, lane96, X + kTA + q * kPlaneA + 4 * i0);
        }
    };
#else
    constexpr uint32_t kPlaneA = 0, kPlaneB = 0;
#endif
    // ---------------- pass A: IFFT d = 1 .. S/2 -------------------------
    const uint32_t wb = 2 * S * wave;
#if CDA_RS16_GLDS
    // The tables' DMA goes out first, then the codeword's loads; the wave
    // waits only for its DMA (vector-memory counts retire in order: all but
    // the last min(2S, 63) loads), and pass A consumes the codeword's loads
    // as they arrive (depth-first) instead of after all of them.
    dma_records(K - 1);
    if (wave < 5) {   // pass B's 64 slots (30 used; the rest get record 0): plane q = wave
        const uint32_t pos = lane, p = pos & 15;
        const uint32_t idx = pos >= 32 || p == 0 ? 0u : pos < 16 ? K - 1 + S * p : S * p - 1;
        glds16(tab + 4 * wave, idx * (kGf16TabWords * 4), X + kTPB + wave * kPlaneB);
    }
    sfor<0, S, 1>([&](auto jj) { ld(src_base, s0 + (wb + jj.value) * ss, lo[jj.value], hi[jj.value]); });
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * S < 63 ? 2 * S : 63) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    sfor<0, S, 1>([&](auto jj) { ld(src_base, s0 + (wb + jj.value) * ss, lo[jj.value], hi[jj.value]); });
    for (uint32_t i = tid; i < K; i += 512) stage_record(X + kTA + i * kTbStride, tab, K - 1 + i);
    if (tid < 32 && (tid & 15))
        stage_record(X + kTPB + tid * kTbStride, tab, tid < 16 ? K - 1 + S * tid : S * (tid - 16) - 1);
    __syncthreads();
#endif
    if (c0 != kNoCopy) {
        sfor<0, S, 1>([&](auto jj) { st(E, c0 + (wb + jj.value) * g.cpy_sh, lcpy, lo[jj.value], hi[jj.value]); });
    }
    layers_regs_lds<S, true, kRs16Dfs>(lo, hi, TBv, [](int gg, int d) { return (uint32_t)(gg + d); }, NoFin{},
                                       kPlaneA);
    // once every wave is past pass A (the exchange's first barrier), the
    // transform records are restaged with the FFT's constants 0..K-1 for pass
    // A'; the B -> A exchange's first barrier publishes them
#if CDA_RS16_GLDS
    // (issued after the exchange: inside it, next to 64 live data registers,
    // the DMA's address arithmetic spilled 34 VGPRs)
    xchg_a_to_b([] {});
    dma_records(0);
#else
    xchg_a_to_b([] {});
    for (uint32_t i = tid; i < K; i += 512) stage_record(X + kTA + i * kTbStride, tab, i);
#endif
    // ---------------- pass B: IFFT d = S .. K/2, FFT d = K/2 .. S --------
    {
        uint32_t lr[R * 16], hr[R * 16];
        sfor<0, R, 1>([&](auto qq) {
            constexpr int q = decltype(qq)::value;
            sfor<0, 16, 1>([&](auto tt) {
                lr[16 * q + tt.value] = lo[R * tt.value + q];
                hr[16 * q + tt.value] = hi[R * tt.value + q];
            });
        });
        const uint32_t* TBB = X + kTPB;
        auto fi = [](int gt, int dt) { return (uint32_t)(K - 1 + S * gt + S * dt); };
        auto ff = [](int gt, int dt) { return (uint32_t)(S * gt + S * dt - 1); };
        auto lfi = [](int gt, int dt) { return (uint32_t)(gt + dt); };
        auto lff = [](int gt, int dt) { return (uint32_t)(16 + gt + dt); };
        if constexpr (CDA_RS16_LDS_B) {
            layers_regs_lds<16, true, false, decltype(lfi), NoFin, R, false>(lr, hr, TBB, lfi, NoFin{}, kPlaneB);
            layers_regs_lds<16, false, false, decltype(lff), NoFin, R, true>(lr, hr, TBB, lff, NoFin{}, kPlaneB);
        } else {
            layers_regs<16, true, false, R>(lr, hr, T, TBB, fi, NoFin{}, lfi, kPlaneB);
            layers_regs<16, false, true, R>(lr, hr, T, TBB, ff, NoFin{}, lff, kPlaneB);
        }
        sfor<0, R, 1>([&](auto qq) {
            constexpr int q = decltype(qq)::value;
            sfor<0, 16, 1>([&](auto tt) {
                lo[R * tt.value + q] = lr[16 * q + tt.value];
                hi[R * tt.value + q] = hr[16 * q + tt.value];
            });
        });
    }
    xchg_b_to_a();
    // ---------------- pass A': FFT d = S/2 .. 1, write parity -------------
    auto store_j = [&](auto jj) { st(E, d0 + (wb + jj.value) * ds, ldst, lo[jj.value], hi[jj.value]); };
    layers_regs_lds<S, false, kRs16Dfs>(lo, hi, TBv, [](int gg, int d) { return (uint32_t)(gg + d - 1); }, store_j,
                                        kPlaneA);
}

// ---------------------------------------------------------------------------
// LDS-staged log/exp kernel (any k with k*64 B of LDS, any shard length)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mul16(const uint16_t* __restrict__ lg, const uint16_t* __restrict__ ex, uint32_t y,
                                          uint32_t L) {
    if (y == 0) return 0;
    uint32_t s = (uint32_t)lg[y] + L;
    s = (s + (s >> 16)) & kMod16;
    return ex[s];
}

// One 64-byte block column of one codeword.  src/dst: shard i at base + i*stride.
__device__ void encode_block_column(const Gf16Dev& t, uint16_t* sym, uint32_t k, const uint8_t* src, size_t src_stride,
                                    uint8_t* dst, size_t dst_stride, uint8_t* copy, size_t copy_stride) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    for (uint32_t w = tid; w < k * 16; w += nt) {
        const uint32_t i = w >> 4, q = w & 15;
        const uint32_t v = reinterpret_cast<const uint32_t*>(src + i * src_stride)[q];
        if (copy) reinterpret_cast<uint32_t*>(copy + i * copy_stride)[q] = v;
        uint8_t* s8 = reinterpret_cast<uint8_t*>(sym + i * 32);
        const uint32_t base = (q & 7) * 4;
        const uint32_t hi = q >> 3;
#pragma unroll
        for (int b = 0; b < 4; b++) s8[2 * (base + b) + hi] = (uint8_t)(v >> (8 * b));
    }
    __syncthreads();
    const uint32_t m = k;
    const uint32_t items = (m / 2) * 32;
    for (uint32_t d = 1; d < m; d <<= 1) {
        for (uint32_t w = tid; w < items; w += nt) {
            const uint32_t p = w >> 5, s = w & 31;
            const uint32_t g = (p / d) * 2 * d, i = g + (p % d);
            const uint32_t L = t.skew[m - 1 + g + d];
            uint32_t x = sym[i * 32 + s], y = sym[(i + d) * 32 + s];
            y ^= x;
            if (L != kMod16) x ^= mul16(t.log, t.exp, y, L);
            sym[i * 32 + s] = (uint16_t)x;
            sym[(i + d) * 32 + s] = (uint16_t)y;
        }
        __syncthreads();
    }
    for (uint32_t d = m >> 1; d >= 1; d >>= 1) {
        for (uint32_t w = tid; w < items; w += nt) {
            const uint32_t p = w >> 5, s = w & 31;
            const uint32_t g = (p / d) * 2 * d, i = g + (p % d);
            const uint32_t L = t.skew[g + d - 1];
            uint32_t x = sym[i * 32 + s], y = sym[(i + d) * 32 + s];
            if (L != kMod16) x ^= mul16(t.log, t.exp, y, L);
            y ^= x;
            sym[i * 32 + s] = (uint16_t)x;
            sym[(i + d) * 32 + s] = (uint16_t)y;
        }
        __syncthreads();
    }
    for (uint32_t w = tid; w < k * 16; w += nt) {
        const uint32_t i = w >> 4, q = w & 15;
        const uint8_t* s8 = reinterpret_cast<const uint8_t*>(sym + i * 32);
        const uint32_t base = (q & 7) * 4, hi = q >> 3;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) v |= (uint32_t)s8[2 * (base + b) + hi] << (8 * b);
        reinterpret_cast<uint32_t*>(dst + i * dst_stride)[q] = v;
    }
}

__global__ __launch_bounds__(256) void rs16_lds_kernel(Gf16Dev t, const RsJob job, uint32_t k) {
    rs_err_init(job);
    extern __shared__ __attribute__((aligned(16))) uint16_t sym[];
    const uint32_t cw = blockIdx.x >> 3;
    const uint32_t blk = blockIdx.x & 7;
    const bool s1 = job.n_seg > 1 && cw >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = s1 ? cw - job.seg[0].n_cw : cw;
    const uint8_t* src = job.src + blockIdx.y * job.src_sq;
    uint8_t* dst = job.dst + blockIdx.y * job.dst_sq;
    const size_t off = (size_t)blk * 64;
    encode_block_column(t, sym, k, src + (size_t)g.src_off + (size_t)c * g.src_cw + off, g.src_sh,
                        dst + (size_t)g.dst_off + (size_t)c * g.dst_cw + off, g.dst_sh,
                        g.cpy_off == kNoCopy ? nullptr : dst + (size_t)g.cpy_off + (size_t)c * g.cpy_cw + off,
                        g.cpy_sh);
}

__global__ __launch_bounds__(256) void rs16_flat_kernel(Gf16Dev t, const uint8_t* __restrict__ data,
                                                       uint8_t* __restrict__ parity, uint32_t k, uint32_t len) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sym[];
    const size_t c = blockIdx.y;
    const size_t off = (size_t)blockIdx.x * 64;
    encode_block_column(t, sym, k, data + c * (size_t)k * len + off, len, parity + c * (size_t)k * len + off, len,
                        nullptr, 0);
}

template <int K>
hipError_t launch_cw(const Gf16Dev& t, const RsJob& j, uint32_t n, hipStream_t s) {
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    static bool attr = false;   // set once per instantiation (function attribute, all devices)
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_cw_kernel<K>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)cw_lds_bytes<K>());
        if (e != hipSuccess) return e;
        attr = true;
    }
    // CDA_RS16_HALF=0: the full-width one-workgroup-per-codeword kernel (A/B)
    static const bool half = [] {
        const char* e = getenv("CDA_RS16_HALF");
        return e ? atoi(e) != 0 : true;
    }();
    if (half) {
        static bool hattr = false;
        if (!hattr) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_half_kernel<K>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)half_lds_bytes<K>());
            if (e != hipSuccess) return e;
            hattr = true;
        }
        hipLaunchKernelGGL(rs16_half_kernel<K>, dim3(2 * ncw, n), dim3(512), half_lds_bytes<K>(), s, t.chunk, j);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(rs16_cw_kernel<K>, dim3(ncw, n), dim3(1024), cw_lds_bytes<K>(), s, t.chunk, j);
    return hipGetLastError();
}

}  // namespace


hipError_t launch_rs8_job(const RsJob& j, uint32_t k, uint32_t n, hipStream_t s);

hipError_t launch_rs(const RsJob& j, uint32_t k, uint32_t n, const Gf16Dev& t, hipStream_t s) {
    if (k == 0 || (k & (k - 1))) return hipErrorInvalidValue;
    if (k <= 128) return launch_rs8_job(j, k, n, s);
    // bitsliced encoder (rs_gf16_bs.hip); CDA_RS16_BS=0 runs the v_perm form (A/B)
    static const bool bs = [] {
        const char* e = getenv("CDA_RS16_BS");
        return e ? atoi(e) != 0 : true;
    }();
    if (bs && (k == 256 || k == 512)) return launch_rs16_bs(j, k, n, s);
    if (t.chunk && t.chunk_k == k) {
        if (k == 256) return launch_cw<256>(t, j, n, s);
        if (k == 512) return launch_cw<512>(t, j, n, s);
    }
    const size_t lds = (size_t)k * 64;
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    hipLaunchKernelGGL(rs16_lds_kernel, dim3(ncw * 8, n), dim3(256), lds, s, t, j, k);
    return hipGetLastError();
}

hipError_t launch_rs16_flat(const Gf16Dev& t, const uint8_t* d, uint8_t* p, uint32_t k, uint32_t len, uint32_t n,
                            hipStream_t s) {
    if (k < 2 || (k & (k - 1)) || len % 64) return hipErrorInvalidValue;
    const size_t lds = (size_t)k * 64;
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    dim3 grid(len / 64, n);
    hipLaunchKernelGGL(rs16_flat_kernel, grid, dim3(256), lds, s, t, d, p, k, len);
    return hipGetLastError();
}

}  // namespace cda
