// rs_gf8_bs.hip -- bitsliced Leopard GF(2^8) encode for k = 128 (the
// appconsts max square, configs 2 and 4).
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF8.encode (EXT, pinned at
// /root/reference/go.mod:152) as reached from rsmt2d LeoRSCodec.Encode
// (pkg/appconsts/global_consts.go:92, pkg/da/data_availability_header.go:74);
// the algorithm core (planes, XOR networks, pass split) is bitslice8.h.
//
// MI355X mapping.  One 512-thread workgroup (8 waves) encodes 4 codewords x
// 512 columns; lane l of every wave owns codeword l/16 and the 32 columns
// {16c..16c+15} u {256+16c..256+16c+15} of every shard (c = l%16), so each
// 16-B load/store instruction moves 256 contiguous bytes per codeword.
//   pass A  wave u: loads its 16 shards 16u..16u+15 (32 x dwordx4 per lane),
//           optionally stores them unchanged (ODS -> EDS Q0 copy), transposes
//           bytes to planes, IFFT d = 1..8 (code specialised per u);
//   A->B    2 rounds through 128 KiB of LDS: wave w receives, for t = w and
//           t = w + 8, the 8 shards 16u + t of every u (a register all-to-all
//           between the 8 waves of one lane index);
//   pass B  IFFT d = 16, 32, 64 and FFT d = 64, 32, 16 (one code path);
//   B->C    the inverse exchange;
//   pass C  wave u: FFT d = 8..1, planes -> bytes, stores 16 parity shards.
// 128 data VGPRs per lane, 2 waves per SIMD, 1 workgroup per CU.
#include "bitslice8.h"
#include "cda_kernels.h"

namespace cda {

namespace {

using namespace bs8;

// Tuning knob: CDA_RS8_NUM_VGPR caps the kernel's VGPRs (the attribute counts
// half of gfx950's unified file) so that a leaf-kernel wave fits beside the
// two RS waves of a SIMD when the two-stream pipeline co-runs them.
#ifdef CDA_RS8_NUM_VGPR
#define CDA_RS8_ATTR __attribute__((amdgpu_num_vgpr(CDA_RS8_NUM_VGPR)))
#else
#define CDA_RS8_ATTR
#endif

constexpr uint32_t kLdsBytes = 8 * 8 * 8 * 64 * 4;   // E[u][tt][p][lane] dwords

__global__ __launch_bounds__(512) CDA_RS8_ATTR void rs8_bs_kernel(const RsJob job) {
    extern __shared__ uint32_t E[];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = threadIdx.x & 63;
    const uint32_t cwg = 4 * blockIdx.x;
    const bool s1 = job.n_seg > 1 && cwg >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = (s1 ? cwg - job.seg[0].n_cw : cwg) + (l >> 4);
    const uint32_t col = 16 * (l & 15);
    const uint8_t* src = job.src + blockIdx.y * job.src_sq;
    uint8_t* dst = job.dst + blockIdx.y * job.dst_sq;
    const uint32_t s0 = g.src_off + c * g.src_cw + col;
    const uint32_t d0 = g.dst_off + c * g.dst_cw + col;
    const uint32_t u = w;
    // The per-u specialised passes run under an if-chain on a copy of the wave
    // index the compiler must treat as divergent: EXEC-masked blocks keep all
    // 128 planes in the same VGPRs across the 8 variants (a uniform switch
    // makes the register allocator shuffle and spill them at the merge).  The
    // value is wave-uniform at run time, so s_cbranch_execz skips 7 of the 8.
    uint32_t ud = threadIdx.x >> 6;
    asm volatile("" : "+v"(ud));

    uint32_t R[128];
    // ---- pass A --------------------------------------------------------
#pragma unroll
    for (int t = 0; t < 16; t++) {
        const uint32_t o = s0 + (16 * u + t) * g.src_sh;
        const uint4 a = *reinterpret_cast<const uint4*>(src + o);
        const uint4 b = *reinterpret_cast<const uint4*>(src + o + 256);
        R[8 * t + 0] = a.x; R[8 * t + 1] = a.y; R[8 * t + 2] = a.z; R[8 * t + 3] = a.w;
        R[8 * t + 4] = b.x; R[8 * t + 5] = b.y; R[8 * t + 6] = b.z; R[8 * t + 7] = b.w;
    }
    if (g.cpy_off != kNoCopy) {
        const uint32_t c0 = g.cpy_off + c * g.cpy_cw + col;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint32_t o = c0 + (16 * u + t) * g.cpy_sh;
            *reinterpret_cast<uint4*>(dst + o) = make_uint4(R[8 * t], R[8 * t + 1], R[8 * t + 2], R[8 * t + 3]);
            *reinterpret_cast<uint4*>(dst + o + 256) =
                make_uint4(R[8 * t + 4], R[8 * t + 5], R[8 * t + 6], R[8 * t + 7]);
        }
    }
#pragma unroll
    for (int t = 0; t < 16; t++) transpose8(R + 8 * t);
    with_u_chain(ud, [&](auto U) { pass_a<decltype(U)::value>(R); });

    // ---- A -> B: round r moves t = 8r + tt (tt = 0..7) ---------------------
#pragma unroll
    for (int r = 0; r < 2; r++) {
        if (r) __syncthreads();
#pragma unroll
        for (int tt = 0; tt < 8; tt++)
#pragma unroll
            for (int p = 0; p < 8; p++) E[((u * 8 + tt) * 8 + p) * 64 + l] = R[8 * (8 * r + tt) + p];
        __syncthreads();
#pragma unroll
        for (int uu = 0; uu < 8; uu++)
#pragma unroll
            for (int p = 0; p < 8; p++) R[64 * r + 8 * uu + p] = E[((uu * 8 + w) * 8 + p) * 64 + l];
    }
    // ---- pass B: units t = w (R[0..64)) and t = w + 8 (R[64..128)) ---------
    pass_b(R);
    pass_b(R + 64);
    // ---- B -> C ------------------------------------------------------------
#pragma unroll
    for (int r = 0; r < 2; r++) {
        __syncthreads();
#pragma unroll
        for (int uu = 0; uu < 8; uu++)
#pragma unroll
            for (int p = 0; p < 8; p++) E[((uu * 8 + w) * 8 + p) * 64 + l] = R[64 * r + 8 * uu + p];
        __syncthreads();
#pragma unroll
        for (int tt = 0; tt < 8; tt++)
#pragma unroll
            for (int p = 0; p < 8; p++) R[8 * (8 * r + tt) + p] = E[((u * 8 + tt) * 8 + p) * 64 + l];
    }
    // ---- pass C --------------------------------------------------------
    with_u_chain(ud, [&](auto U) { pass_c<decltype(U)::value>(R); });
#pragma unroll
    for (int t = 0; t < 16; t++) {
        transpose8(R + 8 * t);
        const uint32_t o = d0 + (16 * u + t) * g.dst_sh;
        *reinterpret_cast<uint4*>(dst + o) = make_uint4(R[8 * t], R[8 * t + 1], R[8 * t + 2], R[8 * t + 3]);
        *reinterpret_cast<uint4*>(dst + o + 256) = make_uint4(R[8 * t + 4], R[8 * t + 5], R[8 * t + 6], R[8 * t + 7]);
    }
}

}  // namespace

// Bitsliced path for k = 128 codewords of 512-B shards (segments of the job
// must hold a multiple of 4 codewords).
hipError_t launch_rs8_bs(const RsJob& j, uint32_t n, hipStream_t s) {
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    if (j.seg[0].n_cw % 4 || (j.n_seg > 1 && j.seg[1].n_cw % 4)) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rs8_bs_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(rs8_bs_kernel, dim3(ncw / 4, n), dim3(512), kLdsBytes, s, j);
    return hipGetLastError();
}

}  // namespace cda
