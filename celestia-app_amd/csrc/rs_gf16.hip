// rs_gf16.hip -- Leopard Reed-Solomon encode over GF(2^16) (k > 128): dispatch
// and the generic LDS-staged kernels.
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF16.encode (EXT, pinned at
// /root/reference/go.mod:152; selected by reedsolomon.New when data + parity
// shards > 256): the IFFT(coset k) / FFT(coset 0) schedule; symbol i of every
// 64-byte block is b[i] | b[i+32] << 8 (lo/hi split layout, leopard.go
// refMulAdd).
//
// k = 256 / 512 squares run the bitsliced encoder (rs_gf16_bs.hip: compile-time
// XOR networks, two half-codeword workgroups per codeword); other k and
// arbitrary shard lengths (rsmt2d Codec.Encode) use the LDS-staged log/exp
// kernel below.  Rounds 1-3's byte-form v_perm encoders (rs16_cw_kernel,
// rs16_half_kernel) were replaced in round 4.
#include "cda_kernels.h"

namespace cda {

namespace {

constexpr uint32_t kMod16 = 65535;

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

}  // namespace

hipError_t launch_rs8_job(const RsJob& j, uint32_t k, uint32_t n, hipStream_t s);

hipError_t launch_rs(const RsJob& j, uint32_t k, uint32_t n, const Gf16Dev& t, hipStream_t s) {
    if (k == 0 || (k & (k - 1))) return hipErrorInvalidValue;
    if (k <= 128) return launch_rs8_job(j, k, n, s);
    if (k == 256 || k == 512) return launch_rs16_bs(j, k, n, s);
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
