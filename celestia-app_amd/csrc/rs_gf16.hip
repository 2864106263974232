// rs_gf16.hip -- Leopard Reed-Solomon encode over GF(2^16) (k > 128).
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF16.encode (EXT, pinned at
// /root/reference/go.mod:152; selected by reedsolomon.New when data+parity
// shards > 256): same IFFT(coset k)/FFT(coset 0) schedule as GF(2^8); symbol i
// of every 64-byte block is b[i] | b[i+32] << 8 (lo/hi split layout,
// leopard.go refMulAdd).
//
// Round-1 kernel: one workgroup per (codeword, 64-byte block column).  The
// k x 32 symbols of that column are staged in LDS (k = 512 -> 32 KiB) and the
// 2*log2(k) butterfly layers run in place with a barrier per layer.  Multiply
// is exp[log[y] + L] with the two 128 KiB tables read through L1/L2 (they stay
// cache resident).  Correct but gather-bound; the register-resident two-pass
// encoder is the planned replacement ("next").
#include "cda_kernels.h"

namespace cda {

namespace {

constexpr uint32_t kMod16 = 65535;

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
    // load: thread handles (shard i, word q) -- 16 words of 4 bytes per shard block
    for (uint32_t w = tid; w < k * 16; w += nt) {
        const uint32_t i = w >> 4, q = w & 15;
        const uint32_t v = reinterpret_cast<const uint32_t*>(src + i * src_stride)[q];
        if (copy) reinterpret_cast<uint32_t*>(copy + i * copy_stride)[q] = v;
        // bytes 4q..4q+3 of the block: lo bytes for q < 8, hi bytes for q >= 8
        uint8_t* s8 = reinterpret_cast<uint8_t*>(sym + i * 32);
        const uint32_t base = (q & 7) * 4;
        const uint32_t hi = q >> 3;
#pragma unroll
        for (int b = 0; b < 4; b++) s8[2 * (base + b) + hi] = (uint8_t)(v >> (8 * b));
    }
    __syncthreads();
    const uint32_t m = k;
    const uint32_t items = (m / 2) * 32;
    for (uint32_t d = 1; d < m; d <<= 1) {       // IFFT (ifftDITEncoder)
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
    for (uint32_t d = m >> 1; d >= 1; d >>= 1) {  // FFT (fftDIT)
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

__global__ __launch_bounds__(256) void rs16_square_kernel(Gf16Dev t, const uint8_t* __restrict__ ods,
                                                         uint8_t* __restrict__ eds, uint32_t k, int phase) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sym[];
    constexpr size_t SH = 512;
    const uint32_t W = 2 * k;
    const uint32_t cw = blockIdx.x >> 3;       // 8 blocks of 64 B per share
    const uint32_t blk = blockIdx.x & 7;
    const size_t sq = blockIdx.y;
    const uint8_t* O = ods + sq * (size_t)k * k * SH;
    uint8_t* E = eds + sq * (size_t)W * W * SH;
    const size_t off = (size_t)blk * 64;
    if (phase == kPhaseQ0) {
        if (cw < k) {
            encode_block_column(t, sym, k, O + (size_t)cw * k * SH + off, SH, E + ((size_t)cw * W + k) * SH + off, SH,
                                E + (size_t)cw * W * SH + off, SH);
        } else {
            const uint32_t j = cw - k;
            encode_block_column(t, sym, k, O + (size_t)j * SH + off, (size_t)k * SH,
                                E + ((size_t)k * W + j) * SH + off, (size_t)W * SH, nullptr, 0);
        }
    } else {
        const uint8_t* src = E + (size_t)(k + cw) * W * SH + off;
        encode_block_column(t, sym, k, src, SH, E + ((size_t)(k + cw) * W + k) * SH + off, SH, nullptr, 0);
    }
}

__global__ __launch_bounds__(256) void rs16_flat_kernel(Gf16Dev t, const uint8_t* __restrict__ data,
                                                       uint8_t* __restrict__ parity, uint32_t k, uint32_t len) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sym[];
    const size_t c = blockIdx.y;
    const size_t off = (size_t)blockIdx.x * 64;
    encode_block_column(t, sym, k, data + c * (size_t)k * len + off, len, parity + c * (size_t)k * len + off, len,
                        nullptr, 0);
}

}  // namespace

hipError_t launch_rs16(const Gf16Dev& t, const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t n, int phase,
                       hipStream_t s) {
    if (k < 2 || (k & (k - 1)) || k > 32768) return hipErrorInvalidValue;
    const size_t lds = (size_t)k * 64;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid((phase == kPhaseQ0 ? 2 * k : k) * 8, n);
    hipLaunchKernelGGL(rs16_square_kernel, grid, dim3(256), lds, s, t, ods, eds, k, phase);
    return hipGetLastError();
}

hipError_t launch_rs16_flat(const Gf16Dev& t, const uint8_t* d, uint8_t* p, uint32_t k, uint32_t len, uint32_t n,
                            hipStream_t s) {
    if (k < 2 || (k & (k - 1)) || len % 64) return hipErrorInvalidValue;
    const size_t lds = (size_t)k * 64;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid(len / 64, n);
    hipLaunchKernelGGL(rs16_flat_kernel, grid, dim3(256), lds, s, t, d, p, k, len);
    return hipGetLastError();
}

}  // namespace cda
