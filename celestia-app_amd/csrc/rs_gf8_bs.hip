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
#include "knobs.h"
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
    rs_err_init(job);
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

// ---------------------------------------------------------------------------
// Half-footprint variant: one 512-thread workgroup encodes 2 codewords x 512
// columns.  Lane l of wave u owns codeword l/32, shard parity h = (l/16)&1 and
// the same 32 columns as above (16*(l%16) ..), i.e. shards 16u + 2j + h,
// j = 0..7: 64 data VGPRs instead of 128, so a CU holds two workgroups at four
// waves per SIMD and one workgroup's loads and stores overlap the other's XOR
// networks (rs8_bs_kernel alternates load -> compute -> store per CU:
// profiles/r02_rs8_phases.txt).  Shard distance 1 pairs lane l with l ^ 16
// (ds_swizzle); every other layer stays in-lane (bitslice8.h pass_*_hi).  The
// exchanges move half the planes per round through 64 KiB of LDS.
// ---------------------------------------------------------------------------
constexpr uint32_t kHalfLdsBytes = 8 * 8 * 4 * 64 * 4;   // E[a][b][4 planes][lane] dwords

template <int MODE>
__device__ __forceinline__ uint32_t swap_h(uint32_t v) {   // lane l <- its shard-parity partner
    if constexpr (MODE == 2)
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);   // bit mode: and 0x1F, xor 0x04
    else
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);   // bit mode: and 0x1F, xor 0x10
}

// Workgroup -> work mapping, three modes:
//   MODE 0: two codewords per workgroup, every lane 32 columns as above.
//   MODE 1 (small jobs, e.g. one square: config 2): one codeword per
//     workgroup, lanes 32..63 idle (their loads and stores masked off), so a
//     job of n codewords fills n workgroups instead of n / 2 -- for a single
//     k = 128 square the first launch then covers all 256 CUs instead of 128.
//   MODE 2 (batches; "slices"): Leopard is independent per byte position,
//     so a workgroup takes EIGHT codewords restricted to one 128-byte slice
//     [128g, 128g + 128) of every shard (lane l: codeword l/8, shard parity
//     (l/4)&1, the 32 contiguous bytes 128g + 32(l%4)), and the workgroups of
//     one (square, slice) unit -- every row AND every column codeword of the
//     launch over that slice -- are numbered so that they share a block
//     index residue mod 8, i.e. one XCD under the round-robin dispatch: the
//     Q0 launch's row and column passes then read each 128-B line of Q0 from
//     the fabric once (the second read hits the XCD's L2) instead of twice.
//     Speed only; correctness does not depend on the placement.
// The codewords of one workgroup (every MODE): lane codeword cwb + lcw of
// square sq, lane columns col..col+15 and col+kHi..col+kHi+15 (cwb uniform:
// segments hold whole workgroups).  E: the exchange buffer (64 KiB of LDS).
template <int MODE>
__device__ __forceinline__ void rs8_half_body(const RsJob& job, uint32_t* E, uint32_t sq, uint32_t cwb, uint32_t lcw,
                                              uint32_t col) {
    constexpr bool ONE = MODE == 1;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t l = threadIdx.x & 63;
    const uint32_t h = MODE == 2 ? (l >> 2) & 1 : (l >> 4) & 1;
    const uint32_t h0 = h ? 0u : 0xFFFFFFFFu;
    const bool s1 = job.n_seg > 1 && cwb >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const bool live = !ONE || l < 32;
    const uint32_t c = (s1 ? cwb - job.seg[0].n_cw : cwb) + lcw;
    // the second 16 B of a lane's 32 columns: 256 bytes on (modes 0, 1: 16
    // lanes x 16 B = 256 contiguous bytes per load), or 64 (mode 2: 4 lanes
    // read one 64-B half of the slice's 128-B line per load)
    constexpr uint32_t kHi = MODE == 2 ? 64 : 256;
    const uint8_t* src = job.src + (size_t)sq * job.src_sq;
    uint8_t* dst = job.dst + (size_t)sq * job.dst_sq;
    const uint32_t u = w;
    const uint32_t s0 = g.src_off + c * g.src_cw + col + (16 * u + h) * g.src_sh;   // shard 16u + h
    const uint32_t d0 = g.dst_off + c * g.dst_cw + col + (16 * u + h) * g.dst_sh;
    uint32_t ud = threadIdx.x >> 6;   // divergent copy of u for the per-U chains (see rs8_bs_kernel)
    asm volatile("" : "+v"(ud));
    // Wave priority 2 while loading, 0 in the passes, 1 from pass C (the
    // stores) on, as in rs_gf16_bs.hip: the two co-resident workgroups' loads
    // and stores issue ahead of the other's XOR networks.  Config 4's RS
    // 8.73-8.78 -> 8.62-8.65 ms per 1 024 squares, 128 squares -3 % on one
    // box (profiles/r05/rs8_prio_ab.txt), equal on another
    // (final_vs_r05z_ab.txt); CDA_RS8_PRIO=0 turns it off.
    if (job.prio) __builtin_amdgcn_s_setprio(2);

    uint32_t R[64];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t o = s0 + 2 * j * g.src_sh;
        uint4 a = make_uint4(0, 0, 0, 0), b = a;
        if (live) {
            a = *reinterpret_cast<const uint4*>(src + o);
            b = *reinterpret_cast<const uint4*>(src + o + kHi);
        }
        R[8 * j + 0] = a.x; R[8 * j + 1] = a.y; R[8 * j + 2] = a.z; R[8 * j + 3] = a.w;
        R[8 * j + 4] = b.x; R[8 * j + 5] = b.y; R[8 * j + 6] = b.z; R[8 * j + 7] = b.w;
    }
    if (live && g.cpy_off != kNoCopy) {
        const uint32_t c0 = g.cpy_off + c * g.cpy_cw + col + (16 * u + h) * g.cpy_sh;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t o = c0 + 2 * j * g.cpy_sh;
            *reinterpret_cast<uint4*>(dst + o) = make_uint4(R[8 * j], R[8 * j + 1], R[8 * j + 2], R[8 * j + 3]);
            *reinterpret_cast<uint4*>(dst + o + kHi) =
                make_uint4(R[8 * j + 4], R[8 * j + 5], R[8 * j + 6], R[8 * j + 7]);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) transpose8(R + 8 * j);
    if (job.prio) __builtin_amdgcn_s_setprio(0);
    // ---- pass A: IFFT shard distance 1 (across the lane pair), then 2, 4, 8
    with_u_chain(ud, [&](auto U) {
        constexpr int UU = decltype(U)::value;
        sfor<0, 8, 1>([&](auto jj) {
            constexpr int j = decltype(jj)::value;
            uint32_t P[8];
#pragma unroll
            for (int p = 0; p < 8; p++) P[p] = swap_h<MODE>(R[8 * j + p]);
            ifft_d1<ifft_d1_log<UU>(j)>(R + 8 * j, P, h0);
        });
        pass_a_hi<UU>(R);
    });
    // ---- A -> B: register j of wave u -> register u of wave j; round r moves
    // planes 4r..4r+3 (slot [a][b] = pass-A wave b's register a)
#pragma unroll
    for (int r = 0; r < 2; r++) {
        if (r) __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int pp = 0; pp < 4; pp++) E[((j * 8 + u) * 4 + pp) * 64 + l] = R[8 * j + 4 * r + pp];
        __syncthreads();
#pragma unroll
        for (int uu = 0; uu < 8; uu++)
#pragma unroll
            for (int pp = 0; pp < 4; pp++) R[8 * uu + 4 * r + pp] = E[((w * 8 + uu) * 4 + pp) * 64 + l];
    }
    // ---- pass B: shards 16u + 2w + h of every u (R[8u + p])
    pass_b(R);
    // ---- B -> A
#pragma unroll
    for (int r = 0; r < 2; r++) {
        __syncthreads();
#pragma unroll
        for (int uu = 0; uu < 8; uu++)
#pragma unroll
            for (int pp = 0; pp < 4; pp++) E[((w * 8 + uu) * 4 + pp) * 64 + l] = R[8 * uu + 4 * r + pp];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int pp = 0; pp < 4; pp++) R[8 * j + 4 * r + pp] = E[((j * 8 + u) * 4 + pp) * 64 + l];
    }
    if (job.prio) __builtin_amdgcn_s_setprio(1);
    // ---- pass C: FFT shard distance 8, 4, 2, then 1 across the lane pair
    with_u_chain(ud, [&](auto U) {
        constexpr int UU = decltype(U)::value;
        pass_c_hi<UU>(R);
        sfor<0, 8, 1>([&](auto jj) {
            constexpr int j = decltype(jj)::value;
            uint32_t P[8];
#pragma unroll
            for (int p = 0; p < 8; p++) P[p] = swap_h<MODE>(R[8 * j + p]);
            fft_d1<fft_d1_log<UU>(j)>(R + 8 * j, P, h0);
        });
    });
#pragma unroll
    for (int j = 0; j < 8; j++) {
        transpose8(R + 8 * j);
        const uint32_t o = d0 + 2 * j * g.dst_sh;
        if (live) {
            *reinterpret_cast<uint4*>(dst + o) = make_uint4(R[8 * j], R[8 * j + 1], R[8 * j + 2], R[8 * j + 3]);
            *reinterpret_cast<uint4*>(dst + o + kHi) =
                make_uint4(R[8 * j + 4], R[8 * j + 5], R[8 * j + 6], R[8 * j + 7]);
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void rs8_bs_half_kernel(const RsJob job,
                                                                                                   uint32_t nsq) {
    constexpr bool ONE = MODE == 1;
    extern __shared__ uint32_t E[];
    const uint32_t l = threadIdx.x & 63;
    // cwb: the workgroup's first codeword, lane codeword cwb + lcw, lane
    // columns col..col+15 and col+kHi..col+kHi+15
    uint32_t sq, cwb, lcw, col;
    if constexpr (MODE == 2) {
        // grid: groups of 8 units x P workgroups, unit u's j-th workgroup at
        // block 8P*(u/8) + 8j + u%8
        const uint32_t ncw = job.seg[0].n_cw + (job.n_seg > 1 ? job.seg[1].n_cw : 0);
        const uint32_t P = ncw / 8;
        const uint32_t b = blockIdx.x, grp = b / (8 * P), r = b % (8 * P);
        const uint32_t unit = grp * 8 + (r & 7), j = r >> 3;
        sq = unit >> 2;
        if (sq >= nsq) return;   // the last group's missing units
        cwb = 8 * j;
        lcw = l >> 3;
        col = 128 * (unit & 3) + 16 * (l & 3);
        if (job.err_init && (unit & 3) == 0 && j == 0 && threadIdx.x == 0) job.err_init[sq] = 0xFFFFFFFFu;
    } else {
        rs_err_init(job);
        sq = blockIdx.y;
        cwb = ONE ? blockIdx.x : 2 * blockIdx.x;
        lcw = ONE ? 0u : l >> 5;
        col = 16 * (l & 15);
    }
    rs8_half_body<MODE>(job, E, sq, cwb, lcw, col);
}

}  // namespace

// Which k = 128 bitsliced kernel (CDA_RS8_BS = 1: 4 codewords per workgroup,
// 2: the half-footprint variant; A/B knob).
static int rs8_variant() {
    static const int v = [] {
        const char* e = test_knob("CDA_RS8_BS");
        return e ? atoi(e) : 2;
    }();
    return v;
}

// Bitsliced path for k = 128 codewords of 512-B shards (segments of the job
// must hold a multiple of 4 codewords).
hipError_t launch_rs8_bs(const RsJob& j, uint32_t n, hipStream_t s) {
    if (rs8_variant() == 2) {
        if (j.seg[0].n_cw % 2 || (j.n_seg > 1 && j.seg[1].n_cw % 2)) return hipErrorInvalidValue;
        const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
        // CDA_RS8_LDS (tuning): LDS reserved per workgroup, >= 64 KiB; above
        // 80 KiB one workgroup per CU, leaving VGPRs for co-running hash waves
        static const uint32_t lds = [] {
            const char* e = test_knob("CDA_RS8_LDS");
            const uint32_t v = e ? (uint32_t)atoi(e) : 0;
            return v > kHalfLdsBytes && v <= 160 * 1024 ? v : kHalfLdsBytes;
        }();
        static bool attr = false;
        if (lds > 64 * 1024 && !attr) {
            for (const void* f : {reinterpret_cast<const void*>(rs8_bs_half_kernel<0>),
                                  reinterpret_cast<const void*>(rs8_bs_half_kernel<1>),
                                  reinterpret_cast<const void*>(rs8_bs_half_kernel<2>)}) {
                hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            attr = true;
        }
        // a job that cannot fill the chip with two codewords per workgroup
        // (fewer than 2 per CU: one k = 128 square has 256 + 128) takes one
        // per workgroup (CDA_RS8_ONE=0/1 forces either, A/B knob)
        static const int one_env = [] {
            const char* e = test_knob("CDA_RS8_ONE");
            return e ? atoi(e) : -1;
        }();
        const bool one = one_env >= 0 ? one_env != 0 : (uint64_t)ncw * n < 2u * 256u;
        // batches: XCD-aware 128-B slices (CDA_RS8_SLICE=0 turns them off, A/B knob)
        static const int slice_env = [] {
            const char* e = test_knob("CDA_RS8_SLICE");
            return e ? atoi(e) : 1;
        }();
        // only where two segments read the same bytes (the Q0 launch: rows
        // and columns of Q0); the Q3 launch (rows of Q2, no re-read) runs
        // faster in mode 0 (3.17 vs 3.43 ms per 1024 squares, while the Q0
        // launch gains 6.06 -> 5.49; profiles/r03g/slice_ab.txt)
        const bool slice = !one && slice_env != 0 && j.n_seg == 2 && j.seg[0].n_cw % 8 == 0 &&
                           j.seg[1].n_cw % 8 == 0;
        if (one)
            hipLaunchKernelGGL(rs8_bs_half_kernel<1>, dim3(ncw, n), dim3(512), lds, s, j, n);
        else if (slice)
            hipLaunchKernelGGL(rs8_bs_half_kernel<2>, dim3((4 * n + 7) / 8 * ncw), dim3(512), lds, s, j, n);
        else
            hipLaunchKernelGGL(rs8_bs_half_kernel<0>, dim3(ncw / 2, n), dim3(512), lds, s, j, n);
        return hipGetLastError();
    }
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
