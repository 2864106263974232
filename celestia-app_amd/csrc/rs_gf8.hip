// rs_gf8.hip -- Leopard Reed-Solomon encode over GF(2^8), k <= 128.
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF8.encode (EXT, pinned at
// /root/reference/go.mod:152) as reached from rsmt2d LeoRSCodec.Encode via
// pkg/appconsts/global_consts.go:92 and pkg/da/data_availability_header.go:74:
// IFFT over coset {k..2k-1} (ifftDITEncoder8, skew offset k-1) then FFT over
// coset 0 (fftDIT8); data shards == parity shards == k (a power of two).
//
// MI355X mapping.  Every byte position of a 512-B shard is an independent
// codeword symbol, so a lane owns one 4-byte column of a codeword across all k
// shards, held in k VGPRs.  All 2*k*log2(k)/2 butterflies of the IFFT+FFT are
// then lane-local register operations with wave-uniform, compile-time
// constants: no LDS, no shuffles.  A wave covers 256 B of every shard, two
// waves a whole codeword.  Loads/stores are 256-B contiguous per
// wave-instruction (share-major streaming).  Column codewords use the same
// code with a k*512-B shard stride (a strided gather, no physical transpose).
//
// GF(2^8) multiply by a constant c: the byte is cut into four 2-bit chunks,
// each looked up in a 4-entry table dword with v_perm_b32(T, T, sel) -- 4 perms
// (half rate), 7 selector ops, 2 XOR3 per 4 bytes; tables are immediates.
#include "cda_kernels.h"
#include "leopard_tables.h"

namespace cda {

namespace {

constexpr LeoField<8> kF8 = make_gf8();

// 2-bit-chunk tables: c[q] byte e = mul_log(e << 2q, L).  v_perm_b32(T, T, sel)
// with sel bytes in 0..3 reads byte sel of T and needs one SGPR operand, so the
// four table dwords are scalar immediates (s_mov) -- no VGPR materialisation.
struct Mul8Chunks {
    uint32_t c[4];
};
struct Mul8All {
    Mul8Chunks t[256];
};
constexpr Mul8All make_all_mul8() {
    Mul8All a{};
    for (uint32_t l = 0; l < 256; l++)
        for (uint32_t q = 0; q < 4; q++)
            for (uint32_t e = 0; e < 4; e++) a.t[l].c[q] |= (uint32_t)kF8.mul_log(e << (2 * q), l) << (8 * e);
    return a;
}
constexpr Mul8All kMul8 = make_all_mul8();
constexpr uint16_t kMod8 = 255;

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x ^ c*y for the compile-time constant with log L (4 perms, 7 selector ops,
// 2 XOR3).
template <uint32_t L>
__device__ __forceinline__ uint32_t mul_add(uint32_t x, uint32_t y) {
    constexpr Mul8Chunks T = kMul8.t[L];
    constexpr uint32_t m = 0x03030303u;
    const uint32_t p0 = perm(T.c[0], T.c[0], y & m);
    const uint32_t p1 = perm(T.c[1], T.c[1], (y >> 2) & m);
    const uint32_t p2 = perm(T.c[2], T.c[2], (y >> 4) & m);
    const uint32_t p3 = perm(T.c[3], T.c[3], (y >> 6) & m);
    return xor3(x, xor3(p0, p1, p2), p3);
}

template <int M, int D, int G>
__device__ __forceinline__ void ifft_group(uint32_t (&v)[M]) {
    constexpr uint32_t L = kF8.skew[M - 1 + G + D];
#pragma unroll
    for (int i = G; i < G + D; i++) {
        v[i + D] ^= v[i];
        if constexpr (L != kMod8) v[i] = mul_add<L>(v[i], v[i + D]);
    }
}
template <int M, int D, int G>
__device__ __forceinline__ void fft_group(uint32_t (&v)[M]) {
    constexpr uint32_t L = kF8.skew[G + D - 1];
#pragma unroll
    for (int i = G; i < G + D; i++) {
        if constexpr (L != kMod8) v[i] = mul_add<L>(v[i], v[i + D]);
        v[i + D] ^= v[i];
    }
}

template <int M, int D, int G = 0>
__device__ __forceinline__ void ifft_layer(uint32_t (&v)[M]) {
    if constexpr (G < M) {
        ifft_group<M, D, G>(v);
        ifft_layer<M, D, G + 2 * D>(v);
    }
}
template <int M, int D, int G = 0>
__device__ __forceinline__ void fft_layer(uint32_t (&v)[M]) {
    if constexpr (G < M) {
        fft_group<M, D, G>(v);
        fft_layer<M, D, G + 2 * D>(v);
    }
}
template <int M, int D = 1>
__device__ __forceinline__ void ifft_all(uint32_t (&v)[M]) {
    if constexpr (D < M) {
        ifft_layer<M, D>(v);
        ifft_all<M, 2 * D>(v);
    }
}
template <int M, int D = M / 2>
__device__ __forceinline__ void fft_all(uint32_t (&v)[M]) {
    if constexpr (D >= 1) {
        fft_layer<M, D>(v);
        fft_all<M, D / 2>(v);
    }
}

template <int M>
__device__ __forceinline__ void encode_regs(uint32_t (&v)[M]) {
    if constexpr (M > 1) {
        ifft_all<M>(v);
        fft_all<M>(v);
    }
}

// One codeword per 128-thread block (two waves x 64 lanes x 4 B = 512 B).
// Register budget: K data VGPRs + temporaries; ask for >= 2 waves per SIMD so
// the VALU issue of one wave hides behind its partner's.
template <int K>
constexpr int waves_per_simd() { return K >= 128 ? 2 : 4; }

template <int K>
__global__ __launch_bounds__(128, waves_per_simd<K>()) void rs8_square_kernel(const uint8_t* __restrict__ ods, uint8_t* __restrict__ eds,
                                                        int phase) {
    constexpr uint32_t W = 2 * K;
    constexpr size_t SH = 512;
    const uint32_t cw = blockIdx.x;
    const size_t sq = blockIdx.y;
    // Uniform base pointer + 32-bit byte offsets (saddr addressing).
    const uint32_t lane4 = threadIdx.x * 4;   // byte offset inside the 512-B shard
    auto lane_off = [&]() { return lane4; };
    const uint8_t* O = ods + sq * (size_t)K * K * SH;
    uint8_t* E = eds + sq * (size_t)W * W * SH;
    const uint8_t* src_base;
    uint32_t s0, ss, d0, ds;
    uint32_t c0 = 0xFFFFFFFFu;
    if (phase == kPhaseQ0) {
        src_base = O;
        if (cw < K) {  // row cw: Q0 -> Q1 (and copy Q0 into the EDS)
            s0 = cw * K * (uint32_t)SH; ss = SH;
            d0 = (cw * W + K) * (uint32_t)SH; ds = SH;
            c0 = cw * W * (uint32_t)SH;
        } else {  // column j: Q0 -> Q2
            const uint32_t j = cw - K;
            s0 = j * (uint32_t)SH; ss = K * (uint32_t)SH;
            d0 = (K * W + j) * (uint32_t)SH; ds = W * (uint32_t)SH;
        }
    } else {  // row K+cw: Q2 -> Q3
        src_base = E;
        s0 = (K + cw) * W * (uint32_t)SH; ss = SH;
        d0 = ((K + cw) * W + K) * (uint32_t)SH; ds = SH;
    }
    uint32_t v[K];
#pragma unroll
    for (int i = 0; i < K; i++)
        v[i] = *reinterpret_cast<const uint32_t*>(src_base + (s0 + i * ss + lane_off()));
    if (c0 != 0xFFFFFFFFu) {
#pragma unroll
        for (int i = 0; i < K; i++) *reinterpret_cast<uint32_t*>(E + (c0 + i * (uint32_t)SH + lane_off())) = v[i];
    }
    encode_regs<K>(v);
#pragma unroll
    for (int i = 0; i < K; i++) *reinterpret_cast<uint32_t*>(E + (d0 + i * ds + lane_off())) = v[i];
}

// Flat codewords: codeword c = data[c*K*len ...], shards of len bytes.
// Grid: (len/512 rounded up, n_code); 128 lanes x 4 B per block.
template <int K>
__global__ __launch_bounds__(128, waves_per_simd<K>()) void rs8_flat_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                      uint32_t len) {
    const size_t c = blockIdx.y;
    const uint32_t off = (blockIdx.x * 128 + threadIdx.x) * 4;
    if (off >= len) return;
    const uint8_t* src = data + c * (size_t)K * len + off;
    uint8_t* dst = parity + c * (size_t)K * len + off;
    uint32_t v[K];
#pragma unroll
    for (int i = 0; i < K; i++) v[i] = *reinterpret_cast<const uint32_t*>(src + (size_t)i * len);
    encode_regs<K>(v);
#pragma unroll
    for (int i = 0; i < K; i++) *reinterpret_cast<uint32_t*>(dst + (size_t)i * len) = v[i];
}

template <int K>
hipError_t launch_sq(const uint8_t* ods, uint8_t* eds, uint32_t n, int phase, hipStream_t s) {
    dim3 grid(phase == kPhaseQ0 ? 2 * K : K, n);
    hipLaunchKernelGGL(rs8_square_kernel<K>, grid, dim3(128), 0, s, ods, eds, phase);
    return hipGetLastError();
}
template <int K>
hipError_t launch_fl(const uint8_t* d, uint8_t* p, uint32_t len, uint32_t n, hipStream_t s) {
    dim3 grid((len / 4 + 127) / 128, n);
    hipLaunchKernelGGL(rs8_flat_kernel<K>, grid, dim3(128), 0, s, d, p, len);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_rs8(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t n, int phase, hipStream_t s) {
    switch (k) {
        case 1: return launch_sq<1>(ods, eds, n, phase, s);
        case 2: return launch_sq<2>(ods, eds, n, phase, s);
        case 4: return launch_sq<4>(ods, eds, n, phase, s);
        case 8: return launch_sq<8>(ods, eds, n, phase, s);
        case 16: return launch_sq<16>(ods, eds, n, phase, s);
        case 32: return launch_sq<32>(ods, eds, n, phase, s);
        case 64: return launch_sq<64>(ods, eds, n, phase, s);
        case 128: return launch_sq<128>(ods, eds, n, phase, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rs8_flat(const uint8_t* d, uint8_t* p, uint32_t k, uint32_t len, uint32_t n, hipStream_t s) {
    switch (k) {
        case 1: return launch_fl<1>(d, p, len, n, s);
        case 2: return launch_fl<2>(d, p, len, n, s);
        case 4: return launch_fl<4>(d, p, len, n, s);
        case 8: return launch_fl<8>(d, p, len, n, s);
        case 16: return launch_fl<16>(d, p, len, n, s);
        case 32: return launch_fl<32>(d, p, len, n, s);
        case 64: return launch_fl<64>(d, p, len, n, s);
        case 128: return launch_fl<128>(d, p, len, n, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace cda
