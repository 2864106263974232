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
#include "knobs.h"
#include <cstdlib>

#include "cda_kernels.h"
#include "leopard_tables.h"

namespace cda {

namespace {

constexpr LeoField<8> kF8 = make_gf8();

// 2-bit-chunk tables (leopard_tables.h make_all_mul8).  v_perm_b32(T, T, sel)
// with sel bytes in 0..3 reads byte sel of T and needs one SGPR operand, so the
// four table dwords are scalar immediates (s_mov) -- no VGPR materialisation.
constexpr Mul8All kMul8 = make_all_mul8(kF8);
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

// Segment of codeword blockIdx.x (uniform) -> byte offsets.
struct SegSel {
    uint32_t s0, ss, d0, ds, c0, cs;
};
__device__ __forceinline__ SegSel select_seg(const RsJob& j, uint32_t cw) {
    const RsSeg& g = (j.n_seg > 1 && cw >= j.seg[0].n_cw) ? j.seg[1] : j.seg[0];
    const uint32_t c = (j.n_seg > 1 && cw >= j.seg[0].n_cw) ? cw - j.seg[0].n_cw : cw;
    SegSel r;
    r.s0 = g.src_off + c * g.src_cw;
    r.ss = g.src_sh;
    r.d0 = g.dst_off + c * g.dst_cw;
    r.ds = g.dst_sh;
    r.c0 = g.cpy_off == kNoCopy ? kNoCopy : g.cpy_off + c * g.cpy_cw;
    r.cs = g.cpy_sh;
    return r;
}

template <int K>
__global__ __launch_bounds__(128, waves_per_simd<K>()) void rs8_job_kernel(const RsJob job) {
    rs_err_init(job);
    const SegSel q = select_seg(job, blockIdx.x);
    // Uniform base pointers + 32-bit byte offsets (saddr addressing).
    const uint8_t* src = job.src + blockIdx.y * job.src_sq;
    uint8_t* dst = job.dst + blockIdx.y * job.dst_sq;
    const uint32_t lane4 = threadIdx.x * 4;   // byte offset inside the 512-B shard
    uint32_t v[K];
#pragma unroll
    for (int i = 0; i < K; i++) v[i] = *reinterpret_cast<const uint32_t*>(src + (q.s0 + i * q.ss + lane4));
    if (q.c0 != kNoCopy) {
#pragma unroll
        for (int i = 0; i < K; i++) *reinterpret_cast<uint32_t*>(dst + (q.c0 + i * q.cs + lane4)) = v[i];
    }
    encode_regs<K>(v);
#pragma unroll
    for (int i = 0; i < K; i++) *reinterpret_cast<uint32_t*>(dst + (q.d0 + i * q.ds + lane4)) = v[i];
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
hipError_t launch_job(const RsJob& j, uint32_t n, hipStream_t s) {
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    hipLaunchKernelGGL(rs8_job_kernel<K>, dim3(ncw, n), dim3(128), 0, s, j);
    return hipGetLastError();
}
template <int K>
hipError_t launch_fl(const uint8_t* d, uint8_t* p, uint32_t len, uint32_t n, hipStream_t s) {
    dim3 grid((len / 4 + 127) / 128, n);
    hipLaunchKernelGGL(rs8_flat_kernel<K>, grid, dim3(128), 0, s, d, p, len);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_rs8_bs(const RsJob& j, uint32_t n, hipStream_t s);

hipError_t launch_rs8_job(const RsJob& j, uint32_t k, uint32_t n, hipStream_t s) {
    // k = 128: bitsliced encoder (rs_gf8_bs.hip) unless a segment is not a
    // multiple of its 4-codeword workgroup (or CDA_RS8_BYTEFORM=1 forces this
    // byte-form encoder, for A/B measurement).
    static const bool byteform = test_knob("CDA_RS8_BYTEFORM") && atoi(test_knob("CDA_RS8_BYTEFORM"));
    if (k == 128 && !byteform && j.seg[0].n_cw % 4 == 0 && (j.n_seg < 2 || j.seg[1].n_cw % 4 == 0))
        return launch_rs8_bs(j, n, s);
    switch (k) {
        case 1: return launch_job<1>(j, n, s);
        case 2: return launch_job<2>(j, n, s);
        case 4: return launch_job<4>(j, n, s);
        case 8: return launch_job<8>(j, n, s);
        case 16: return launch_job<16>(j, n, s);
        case 32: return launch_job<32>(j, n, s);
        case 64: return launch_job<64>(j, n, s);
        case 128: return launch_job<128>(j, n, s);
        default: return hipErrorInvalidValue;
    }
}

RsJob square_job_q0(const uint8_t* ods, uint8_t* eds, uint32_t k) {
    const uint32_t W = 2 * k, SH = 512;
    RsJob j{};
    j.src = ods;
    j.dst = eds;
    j.src_sq = (uint64_t)k * k * SH;
    j.dst_sq = (uint64_t)W * W * SH;
    j.n_seg = 2;
    // rows: ODS row c -> EDS row c (Q0 copy) and Q1
    j.seg[0] = RsSeg{k, 0, k * SH, SH, k * SH, W * SH, SH, 0, W * SH, SH};
    // columns: ODS column c -> Q2 column c
    j.seg[1] = RsSeg{k, 0, SH, k * SH, k * W * SH, SH, W * SH};
    return j;
}

// In place: the ODS already sits in Q0 of the EDS (cda_extend_dah_inplace_*),
// so both segments read Q0 at the EDS row stride and nothing is copied.
RsJob square_job_q0_inplace(uint8_t* eds, uint32_t k) {
    const uint32_t W = 2 * k, SH = 512;
    RsJob j{};
    j.src = eds;
    j.dst = eds;
    j.src_sq = j.dst_sq = (uint64_t)W * W * SH;
    j.n_seg = 2;
    // rows: Q0 row c -> Q1 row c
    j.seg[0] = RsSeg{k, 0, W * SH, SH, k * SH, W * SH, SH};
    // columns: Q0 column c -> Q2 column c
    j.seg[1] = RsSeg{k, 0, SH, W * SH, k * W * SH, SH, W * SH};
    return j;
}

RsJob square_job_q3(uint8_t* eds, uint32_t k) {
    const uint32_t W = 2 * k, SH = 512;
    RsJob j{};
    j.src = eds;
    j.dst = eds;
    j.src_sq = j.dst_sq = (uint64_t)W * W * SH;
    j.n_seg = 1;
    // rows k..2k-1: Q2 -> Q3
    j.seg[0] = RsSeg{k, k * W * SH, W * SH, SH, k * W * SH + k * SH, W * SH, SH};
    return j;
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
