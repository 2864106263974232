// rs_gf16_bs.hip -- bitsliced Leopard GF(2^16) encode for k = 256 / 512.
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF16.encode (EXT, pinned at
// /root/reference/go.mod:152; selected by reedsolomon.New when data + parity
// shards > 256, i.e. squares wider than 128): IFFT of the k data shards at
// coset k (skew[k - 1 + g + d]), then FFT to the k parity shards (skew[g + d
// - 1]), on symbols b[i] | b[i + 32] << 8 of every 64-byte block.
//
// MI355X mapping.  TWO workgroups per codeword, each over 4 of the 8 64-byte
// blocks of every shard (Leopard is independent per symbol position), and
// three workgroups per CU (k = 512: 4 waves, 256 threads, 168 VGPRs and
// 32 KiB of LDS each), so one's loads, stores, exchanges and barrier waits
// run under the others' XOR networks.  A lane holds 8 "units" -- the 16
// bit-planes of the 32 symbols of one block of one shard (128 VGPRs,
// bitslice16.h) -- so GF addition is one XOR per plane and multiplying by a butterfly constant is a compile-time XOR
// network of full-rate v_bitop3 / v_xor (about 2 SIMD cycles per
// wave-instruction; the byte-form v_perm multiply it replaces issues at the
// half rate and needs 3.6x the instructions: tools/bs16_probe.hip,
// profiles/r04_bs16_probe*.txt).  A butterfly constant depends on the shard
// bits above its layer; the three layouts of bitslice16.h keep those bits in
// the unit index where they can:
//   load, planes, LOW IFFT (b = 0..2)       [LOW: unit = shard bits 0..2]
//   X12: unit <-> lane bits 3..5 within each wave, through LDS
//   M1 IFFT (b = 3..5)                      [M1: unit = bits 3..5]
//   X23: all-to-all between the waves through LDS
//   M2 IFFT / FFT (the top three bits)      [M2: unit = bits k-3..]
//   X32, M1 FFT, X21, LOW FFT, planes -> bytes, store.
// LOW's constants also depend on the lane (bits 3..6) and the wave (bits 7..),
// M1's on the lane (bit 6) and the wave: the skew is linear in the group
// position, so those enter as masked and uniform-branch terms (layer8).
#include <mutex>

#include "bitslice16.h"
#include "cda_kernels.h"

namespace cda {

namespace {

// Three workgroups per CU (168 VGPRs, 32 KiB of LDS each): a CU always has
// a third wave on each SIMD to issue while one waits at a barrier or on
// memory; at two per CU (208 VGPRs, no spills) the encoder was 15-20 % slower
// (profiles/r04d/, r04f/).  Prefetching the next round's codewords into L2 /
// MALL with LDS-DMA during the compute phases was slower still (r04d).
constexpr int kWavesPerSimd = 3;
// Exchange buffer: kChunksPerRound 16-byte chunks (4 planes) of every unit of
// the workgroup per round (four rounds per exchange); 8 consecutive lanes
// always address 8 distinct 16-byte bank groups (see the slot functions).
constexpr int kChunksPerRound = 1;
template <int LOGK>
constexpr uint32_t bs16_lds_bytes() {
    return (uint32_t)kChunksPerRound * (1u << LOGK) * 4 * 16;   // shards x 4 blocks x 16 B per chunk
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_st(u32x4* X, uint32_t idx, const uint32_t* r) {
    X[idx] = u32x4{r[0], r[1], r[2], r[3]};
}
__device__ __forceinline__ void lds_ld(const u32x4* X, uint32_t idx, uint32_t* r) {
    const u32x4 v = X[idx];
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = v.w;
}

template <int LOGK>
__global__ __launch_bounds__(64 << (LOGK - 7)) __attribute__((amdgpu_waves_per_eu(kWavesPerSimd))) void rs16_bs_kernel(
    const RsJob job) {
    constexpr int NW = 1 << (LOGK - 7);    // waves per workgroup
    constexpr int K = 1 << LOGK;
    rs_err_init(job);
    // Wave priority 2 while this workgroup loads, 0 in the butterflies and
    // exchanges, 1 from the LOW FFT / store phase on: with three workgroups
    // per CU in different phases, the loads and stores issue ahead of the
    // co-resident workgroups' XOR networks.  One k = 512 square: RS 0.288 ->
    // 0.276 ms; at 16 squares per launch (every slot busy) +3 %, so the engine
    // sets job.prio for small batches only (profiles/r05/rs16_prio_ab.txt).
    if (job.prio) __builtin_amdgcn_s_setprio(2);
    extern __shared__ u32x4 X[];
    const uint32_t tid = threadIdx.x;
    // Lane-derived values are recomputed from tid once per exchange call and
    // per butterfly phase (the empty asm keeps the compiler from carrying them
    // across the phases, where it spilled them): k = 512 13 -> 0 spilled
    // values, 889 -> 814 MB per square at the fabric, RS equal at batch 1 and
    // -5 % at batch 16 (profiles/r05/rs16_spill_ab.txt; recomputing at every
    // use cost +14 % VALU instructions).
    struct LaneIds {
        uint32_t lane, b4, jl;
    };
    auto ids = [&]() {
        uint32_t t = tid;
        asm volatile("" : "+v"(t));
        const uint32_t l = t & 63;
        return LaneIds{l, l & 3, l >> 2};
    };
    auto lane_masks = [&](uint32_t (&m)[4]) {
        const uint32_t jl = ids().jl;
#pragma unroll
        for (int i = 0; i < 4; i++) m[i] = 0u - ((jl >> i) & 1);
    };
    // The wave -> shard-bit mapping is rotated per workgroup: the wave with
    // wave bits 11 runs both uniform-branch terms of every LOW / M1 butterfly,
    // the one with 00 none, and the waves of a workgroup go to the SIMDs of a
    // CU in index order, so without the rotation one SIMD of every CU runs the
    // heaviest wave of each co-resident workgroup.  Round 5, interleaved A/B
    // (profiles/r05/rs16_ab.txt): RS per k = 512 square 0.320 -> 0.312 ms
    // (batch 1), 0.271 -> 0.257 (4), 0.257 -> 0.250 (16).
    const uint32_t w = __builtin_amdgcn_readfirstlane(((tid >> 6) + (blockIdx.x >> 1) + blockIdx.y) & (NW - 1));
    const uint32_t cw = blockIdx.x >> 1, half = blockIdx.x & 1;
    const bool s1 = job.n_seg > 1 && cw >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = s1 ? cw - job.seg[0].n_cw : cw;
    const uint8_t* src = job.src + (size_t)blockIdx.y * job.src_sq;
    uint8_t* E = job.dst + (size_t)blockIdx.y * job.dst_sq;
    // LOW layout: unit u of lane (b4, jl) of wave w is shard w << 7 | jl << 3 | u,
    // block 4 half + b4: uniform part (w, u) in SGPRs + a per-lane offset
    const uint32_t s0 = g.src_off + c * g.src_cw + (w << 7) * g.src_sh;
    const uint32_t d0 = g.dst_off + c * g.dst_cw + (w << 7) * g.dst_sh;
    const uint32_t ls = 64 * (4 * half + ids().b4) + 8 * ids().jl * g.src_sh;
    uint32_t R[128];
    // ---- load + planes + LOW IFFT --------------------------------------------
    bs16::sfor<0, 8, 1>([&](auto uu) {
        constexpr int u = decltype(uu)::value;
        uint32_t o = s0 + u * g.src_sh;
        asm volatile("" : "+s"(o));
        const u32x4* p = reinterpret_cast<const u32x4*>(src + o + ls);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 v = p[q];
            R[16 * u + 4 * q + 0] = v.x;
            R[16 * u + 4 * q + 1] = v.y;
            R[16 * u + 4 * q + 2] = v.z;
            R[16 * u + 4 * q + 3] = v.w;
        }
    });
    if (g.cpy_off != kNoCopy) {   // the ODS copy into Q0 (packed entry)
        const uint32_t c0 = g.cpy_off + c * g.cpy_cw + (w << 7) * g.cpy_sh;
        const uint32_t lc = 64 * (4 * half + ids().b4) + 8 * ids().jl * g.cpy_sh;
        bs16::sfor<0, 8, 1>([&](auto uu) {
            constexpr int u = decltype(uu)::value;
            uint32_t o = c0 + u * g.cpy_sh;
            asm volatile("" : "+s"(o));
            u32x4* p = reinterpret_cast<u32x4*>(E + o + lc);
#pragma unroll
            for (int q = 0; q < 4; q++)
                p[q] = u32x4{R[16 * u + 4 * q], R[16 * u + 4 * q + 1], R[16 * u + 4 * q + 2], R[16 * u + 4 * q + 3]};
        });
    }
    // (Masks derived at each use, bs16::LaneMask<0>{jl}: 16 instead of 20
    // spills, but RS +6-8 % at batch 4; profiles/r05/leaf_overlap_lanemask_ab.txt.)
    uint32_t m[4];
    lane_masks(m);
    // LOW IFFT layer 0 pairs units (0,1), (2,3), ..., layer 1 pairs within
    // 0..3 and within 4..7: each pair / quad of units goes through the layers
    // it can as soon as its loads land (the wait for a unit's data sits
    // before its planes transform), while the later units still load.
    auto planes2 = [&](auto uu) {
        constexpr int u = decltype(uu)::value;
        bs16::block_planes(R + 16 * u);
        bs16::block_planes(R + 16 * (u + 1));
        bs16::low_layer<LOGK, true, 0, u, u + 2>(R, m, w);
    };
    planes2(std::integral_constant<int, 0>{});
    planes2(std::integral_constant<int, 2>{});
    bs16::low_layer<LOGK, true, 1, 0, 4>(R, m, w);
    planes2(std::integral_constant<int, 4>{});
    planes2(std::integral_constant<int, 6>{});
    bs16::low_layer<LOGK, true, 1, 4, 8>(R, m, w);
    bs16::low_layer<LOGK, true, 2>(R, m, w);

    if (job.prio) __builtin_amdgcn_s_setprio(0);
    // ---- exchanges ------------------------------------------------------------
    // X12 / X21 (LOW <-> M1, within each wave): unit u of lane (b4, jl) <->
    // unit jl & 7 of lane (b4, (jl & 8) | u).  Slot ((chunk * NW + w) * 8 +
    // dst unit) * 64 + (dst lane ^ (dst unit & 1) << 2): the XOR keeps the two
    // jl of an 8-lane group on distinct bank groups for writer and reader.
    auto x12 = [&](bool barrier) {
        const LaneIds I = ids();
        if (barrier) __syncthreads();   // the buffer's previous readers (other waves) are done
        bs16::sfor<0, 4 / kChunksPerRound, 1>([&](auto rr) {
            constexpr int rnd = decltype(rr)::value;
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t du = I.jl & 7, dl = (I.b4 | ((I.jl & 8) | u) << 2) ^ ((du & 1) << 2);
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value, q = rnd * kChunksPerRound + cq;
                    lds_st(X, ((cq * NW + w) * 8 + du) * 64 + dl, R + 16 * u + 4 * q);
                });
            });
            // same wave: its LDS ops complete in order, the compiler waits for the data
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value, q = rnd * kChunksPerRound + cq;
                    lds_ld(X, ((cq * NW + w) * 8 + u) * 64 + (I.lane ^ ((u & 1) << 2)), R + 16 * u + 4 * q);
                });
            });
        });
    };
    // X23 / X32 (M1 <-> M2, all waves): slot (chunk * K + shard) * 4 + b4.
    //   M1 (w, jl, u): shard w << 7 | (jl >> 3) << 6 | u << 3 | jl & 7
    //   M2 (w, jl, u): shard u << (LOGK - 3) | w << 4 | jl
    auto m1_shard = [&](uint32_t u, uint32_t jl) { return w << 7 | (jl >> 3) << 6 | u << 3 | (jl & 7); };
    auto m2_shard = [&](uint32_t u, uint32_t jl) { return u << (LOGK - 3) | w << 4 | jl; };
    auto x23 = [&](bool to_m2) {
        const LaneIds I = ids();
        bs16::sfor<0, 4 / kChunksPerRound, 1>([&](auto rr) {
            constexpr int rnd = decltype(rr)::value;
            __syncthreads();
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t sh = to_m2 ? m1_shard(u, I.jl) : m2_shard(u, I.jl);
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value;
                    lds_st(X, (cq * K + sh) * 4 + I.b4, R + 16 * u + 4 * (rnd * kChunksPerRound + cq));
                });
            });
            __syncthreads();
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t sh = to_m2 ? m2_shard(u, I.jl) : m1_shard(u, I.jl);
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value;
                    lds_ld(X, (cq * K + sh) * 4 + I.b4, R + 16 * u + 4 * (rnd * kChunksPerRound + cq));
                });
            });
        });
    };

    x12(false);   // the first exchange: the workgroup's LDS is untouched so far
    lane_masks(m);
    bs16::phase_m1_ifft<LOGK>(R, m, w);
    x23(true);
    bs16::phase_m2<LOGK>(R);
    x23(false);
    lane_masks(m);
    bs16::phase_m1_fft<LOGK>(R, m, w);
    x12(true);
    lane_masks(m);
    if (job.prio) __builtin_amdgcn_s_setprio(1);
    // ---- LOW FFT, planes -> bytes, store parity --------------------------------
    auto store = [&](auto uu) {
        constexpr int u = decltype(uu)::value;
        bs16::block_planes(R + 16 * u);
        uint32_t o = d0 + u * g.dst_sh;
        asm volatile("" : "+s"(o));
        const LaneIds I = ids();
        u32x4* p = reinterpret_cast<u32x4*>(E + o + 64 * (4 * half + I.b4) + 8 * I.jl * g.dst_sh);
#pragma unroll
        for (int q = 0; q < 4; q++)
            p[q] = u32x4{R[16 * u + 4 * q], R[16 * u + 4 * q + 1], R[16 * u + 4 * q + 2], R[16 * u + 4 * q + 3]};
    };
    // mirror of the entry: each pair of units stores as soon as it is done
    auto store2 = [&](auto uu) {
        constexpr int u = decltype(uu)::value;
        bs16::low_layer<LOGK, false, 0, u, u + 2>(R, m, w);
        store(std::integral_constant<int, u>{});
        store(std::integral_constant<int, u + 1>{});
    };
    bs16::low_layer<LOGK, false, 2>(R, m, w);
    bs16::low_layer<LOGK, false, 1, 0, 4>(R, m, w);
    store2(std::integral_constant<int, 0>{});
    store2(std::integral_constant<int, 2>{});
    bs16::low_layer<LOGK, false, 1, 4, 8>(R, m, w);
    store2(std::integral_constant<int, 4>{});
    store2(std::integral_constant<int, 6>{});
}

template <int LOGK>
hipError_t launch_bs(const RsJob& j, uint32_t n, hipStream_t s) {
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    // function attribute, set once per instantiation (contexts on several host
    // threads may launch at once)
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
        attr = hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_bs_kernel<LOGK>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs16_lds_bytes<LOGK>());
    });
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(rs16_bs_kernel<LOGK>, dim3(2 * ncw, n), dim3(64 << (LOGK - 7)), bs16_lds_bytes<LOGK>(), s, j);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_rs16_bs(const RsJob& j, uint32_t k, uint32_t n, hipStream_t s) {
    if (k == 512) return launch_bs<9>(j, n, s);
    if (k == 256) return launch_bs<8>(j, n, s);
    return hipErrorInvalidValue;
}

}  // namespace cda
