// rs_gf16_bs.hip -- bitsliced Leopard GF(2^16) encode for k = 256 / 512.
//
// Restates klauspost/reedsolomon v1.12.1 leopardFF16.encode (EXT, pinned at
// /root/reference/go.mod:152; selected by reedsolomon.New when data + parity
// shards > 256, i.e. squares wider than 128): IFFT of the k data shards at
// coset k (skew[k - 1 + g + d]), then FFT to the k parity shards (skew[g + d
// - 1]), on symbols b[i] | b[i + 32] << 8 of every 64-byte block.
//
// MI355X mapping.  TWO workgroups per codeword, each over 4 of the 8 64-byte
// blocks of every shard (Leopard is independent per symbol position), and two
// workgroups per CU, so one's loads, stores, exchanges and barrier waits run
// under the other's XOR networks (k = 512: 4 waves, 256 threads, 64 KiB of
// LDS each).  A lane holds 8 "units" -- the 16 bit-planes of the 32 symbols of
// one block of one shard (128 VGPRs, bitslice16.h) -- so GF addition is one
// XOR per plane and multiplying by a butterfly constant is a compile-time XOR
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
#include <algorithm>

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

// One half-codeword (4 of the 8 blocks of every shard): codeword c of
// segment g, reading src and writing E (one square's bases).
struct NoHook {
    __device__ void operator()() const {}
};
// after_loads(): called once the codeword's loads are issued (the ticket
// kernel stores its prefetched next ticket there)
template <int LOGK, typename AfterLoads = NoHook>
__device__ __forceinline__ void bs_encode_half(const uint8_t* src, uint8_t* E, const RsSeg& g, uint32_t c,
                                               uint32_t half, u32x4* X, bool write_through = false,
                                               AfterLoads after_loads = {}) {
    constexpr int NW = 1 << (LOGK - 7);    // waves per workgroup
    constexpr int K = 1 << LOGK;
    const uint32_t tid = threadIdx.x, lane = tid & 63, b4 = lane & 3, jl = lane >> 2;
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // LOW layout: unit u of lane (b4, jl) of wave w is shard w << 7 | jl << 3 | u,
    // block 4 half + b4: uniform part (w, u) in SGPRs + a per-lane offset
    const uint32_t blk_off = 64 * (4 * half + b4);
    const uint32_t s0 = g.src_off + c * g.src_cw + (w << 7) * g.src_sh;
    const uint32_t d0 = g.dst_off + c * g.dst_cw + (w << 7) * g.dst_sh;
    const uint32_t ls = blk_off + 8 * jl * g.src_sh, ld = blk_off + 8 * jl * g.dst_sh;
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
    after_loads();
    if (g.cpy_off != kNoCopy) {   // the ODS copy into Q0 (packed entry)
        const uint32_t c0 = g.cpy_off + c * g.cpy_cw + (w << 7) * g.cpy_sh, lc = blk_off + 8 * jl * g.cpy_sh;
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
    bs16::sfor<0, 8, 1>([&](auto uu) { bs16::block_planes(R + 16 * decltype(uu)::value); });
    uint32_t m[4];
#pragma unroll
    for (int i = 0; i < 4; i++) m[i] = 0u - ((jl >> i) & 1);
    bs16::phase_low_ifft<LOGK>(R, m, w);

    // ---- exchanges ------------------------------------------------------------
    // X12 / X21 (LOW <-> M1, within each wave): unit u of lane (b4, jl) <->
    // unit jl & 7 of lane (b4, (jl & 8) | u).  Slot ((chunk * NW + w) * 8 +
    // dst unit) * 64 + (dst lane ^ (dst unit & 1) << 2): the XOR keeps the two
    // jl of an 8-lane group on distinct bank groups for writer and reader.
    auto x12 = [&](bool barrier) {
        if (barrier) __syncthreads();   // the buffer's previous readers (other waves) are done
        bs16::sfor<0, 4 / kChunksPerRound, 1>([&](auto rr) {
            constexpr int rnd = decltype(rr)::value;
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t du = jl & 7, dl = (b4 | ((jl & 8) | u) << 2) ^ ((du & 1) << 2);
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
                    lds_ld(X, ((cq * NW + w) * 8 + u) * 64 + (lane ^ ((u & 1) << 2)), R + 16 * u + 4 * q);
                });
            });
        });
    };
    // X23 / X32 (M1 <-> M2, all waves): slot (chunk * K + shard) * 4 + b4.
    //   M1 (w, jl, u): shard w << 7 | (jl >> 3) << 6 | u << 3 | jl & 7
    //   M2 (w, jl, u): shard u << (LOGK - 3) | w << 4 | jl
    auto m1_shard = [&](uint32_t u) { return w << 7 | (jl >> 3) << 6 | u << 3 | (jl & 7); };
    auto m2_shard = [&](uint32_t u) { return u << (LOGK - 3) | w << 4 | jl; };
    auto x23 = [&](bool to_m2) {
        bs16::sfor<0, 4 / kChunksPerRound, 1>([&](auto rr) {
            constexpr int rnd = decltype(rr)::value;
            __syncthreads();
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t sh = to_m2 ? m1_shard(u) : m2_shard(u);
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value;
                    lds_st(X, (cq * K + sh) * 4 + b4, R + 16 * u + 4 * (rnd * kChunksPerRound + cq));
                });
            });
            __syncthreads();
            bs16::sfor<0, 8, 1>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const uint32_t sh = to_m2 ? m2_shard(u) : m1_shard(u);
                bs16::sfor<0, kChunksPerRound, 1>([&](auto cc) {
                    constexpr int cq = decltype(cc)::value;
                    lds_ld(X, (cq * K + sh) * 4 + b4, R + 16 * u + 4 * (rnd * kChunksPerRound + cq));
                });
            });
        });
    };

    x12(false);   // the first exchange: the workgroup's LDS is untouched so far
    bs16::phase_m1_ifft<LOGK>(R, m, w);
    x23(true);
    bs16::phase_m2<LOGK>(R);
    x23(false);
    bs16::phase_m1_fft<LOGK>(R, m, w);
    x12(true);
    bs16::phase_low_fft<LOGK>(R, m, w);
    // ---- planes -> bytes, store parity -----------------------------------------
    // write_through (uniform): sc1 stores, the parity another workgroup of
    // the launch reads (rs16_bs_ticket_kernel); s_nop 1 after each: the
    // compiler does not see the store's data registers in use
    bs16::sfor<0, 8, 1>([&](auto uu) {
        constexpr int u = decltype(uu)::value;
        bs16::block_planes(R + 16 * u);
        uint32_t o = d0 + u * g.dst_sh;
        asm volatile("" : "+s"(o));
        u32x4* p = reinterpret_cast<u32x4*>(E + o + ld);
        if (write_through) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1"
                             :
                             : "v"(p + q), "v"(u32x4{R[16 * u + 4 * q], R[16 * u + 4 * q + 1], R[16 * u + 4 * q + 2],
                                                    R[16 * u + 4 * q + 3]})
                             : "memory");
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
                p[q] = u32x4{R[16 * u + 4 * q], R[16 * u + 4 * q + 1], R[16 * u + 4 * q + 2], R[16 * u + 4 * q + 3]};
        }
    });
}

template <int LOGK>
__global__ __launch_bounds__(64 << (LOGK - 7)) __attribute__((amdgpu_waves_per_eu(kWavesPerSimd))) void rs16_bs_kernel(
    const RsJob job) {
    rs_err_init(job);
    extern __shared__ u32x4 X[];
    const uint32_t cw = blockIdx.x >> 1, half = blockIdx.x & 1;
    const bool s1 = job.n_seg > 1 && cw >= job.seg[0].n_cw;
    const RsSeg& g = s1 ? job.seg[1] : job.seg[0];
    const uint32_t c = s1 ? cw - job.seg[0].n_cw : cw;
    bs_encode_half<LOGK>(job.src + (size_t)blockIdx.y * job.src_sq, job.dst + (size_t)blockIdx.y * job.dst_sq, g, c,
                         half, X);
}

// The whole extension of n squares in ONE launch (Q0 columns, Q0 rows, Q3):
// every workgroup draws a ticket; tickets [0, P) are the column
// half-codewords (Q0 -> Q2), [P, 2P) the rows (Q0 -> Q1), [2P, 3P) Q3 (Q2
// rows -> Q3), P = n * 2k.  A Q3 workgroup needs the columns of its square
// done; it polls the column counter, which every column workgroup bumps after
// publishing its parity (write-through sc1 stores drained by every wave,
// barrier, one lane's relaxed agent add: no L2 write-back), and then acquires
// (one lane's agent acquire, drain, barrier) before its plain loads (the
// hand-off recipe of the MI355X guide, inter-workgroup visibility; a release
// fence per column workgroup instead measured 15-30 % slower).  No
// deadlock whatever the dispatch order: a workgroup holding a Q3 ticket waits
// only for workgroups that drew earlier tickets, which never wait.  The one
// launch has no Q0 -> Q3 boundary: 3P items fill ceil(3P / resident) rounds
// instead of ceil(2P / resident) + ceil(P / resident).  A persistent grid (the
// resident workgroups), each drawing its next ticket while it encodes; the two
// counters (128-byte lines) are zeroed by a memset ahead of the launch.
typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr uint32_t kTicketLine = 32;   // u32 words per 128-byte line
template <int LOGK>
__global__ __launch_bounds__(64 << (LOGK - 7)) __attribute__((amdgpu_waves_per_eu(kWavesPerSimd))) void
rs16_bs_ticket_kernel(const RsJob job, const RsSeg q3, uint32_t* ctr_p, uint32_t n_sq) {
    extern __shared__ u32x4 X[];
    __shared__ uint32_t s_ticket[2];   // the next ticket, by item parity
    gu32* ctr = (gu32*)ctr_p;
    const uint32_t tid = threadIdx.x;
    const uint32_t per = 2u << LOGK, P = n_sq * per;   // half-codewords per square and phase; per phase
    if (tid == 0) s_ticket[0] = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    uint32_t t = __builtin_amdgcn_readfirstlane(s_ticket[0]);
    for (uint32_t it = 1; t < 3 * P; it ^= 1) {
        // the next ticket, drawn now and stored once the item's loads are
        // issued: its latency hides under them.  Always a later ticket than t,
        // so a waiting Q3 item never holds back a column ticket (no deadlock).
        // Slot it is written in this item and read at its end; the other slot
        // was read by every wave before this item's first barrier.
        uint32_t next = 0;
        if (tid == 0) next = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t phase = t / P, r = t - phase * P, y = r / per, x = r - y * per;
        const bool q3_item = phase == 2;
        if (q3_item) {   // Q3: wait for every column of the launch, then acquire
            if (tid == 0) {
                for (uint32_t i = 0;
                     __hip_atomic_load(ctr + kTicketLine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < P;) {
                    __builtin_amdgcn_s_sleep(8);
                    if (++i == (1u << 22)) break;   // bounded (~1 s): a wrong count ends in wrong parity, not a hang
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        } else if (phase == 0 && x == 0 && tid == 0 && job.err_init) {
            job.err_init[y] = 0xFFFFFFFFu;
        }
        uint8_t* E = job.dst + (size_t)y * job.dst_sq;
        // one call site: the encoder body is instantiated once
        bs_encode_half<LOGK>(q3_item ? E : job.src + (size_t)y * job.src_sq, E,
                             q3_item ? q3 : phase == 0 ? job.seg[1] : job.seg[0], x >> 1, x & 1, X, phase == 0,
                             [&] {
                                 if (tid == 0) s_ticket[it] = next;
                             });
        if (phase == 0) {   // publish this half-codeword's Q2 parity (sc1 stores: no release fence)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(ctr + kTicketLine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();   // the item's LDS readers are done (the next item's first exchange has no barrier)
        t = __builtin_amdgcn_readfirstlane(s_ticket[it]);
    }
}

template <int LOGK>
hipError_t launch_ticket(const RsJob& q0, const RsSeg& q3, uint32_t* ctr, uint32_t n, hipStream_t s) {
    static int grid = 0;   // resident workgroups: a persistent grid (fewer admitted just start later)
    if (!grid) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_bs_ticket_kernel<LOGK>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs16_lds_bytes<LOGK>());
        if (e != hipSuccess) return e;
        int dev = 0, cus = 0, per_cu = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rs16_bs_ticket_kernel<LOGK>, 64 << (LOGK - 7),
                                                              bs16_lds_bytes<LOGK>())) != hipSuccess)
            return e;
        grid = std::max(1, cus * std::max(1, per_cu));
    }
    const uint32_t items = 3 * n * (2u << LOGK);
    // the ticket and column counters start at zero every launch
    hipError_t e = hipMemsetAsync(ctr, 0, 2 * kTicketLine * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rs16_bs_ticket_kernel<LOGK>, dim3(std::min<uint32_t>(items, (uint32_t)grid)),
                       dim3(64 << (LOGK - 7)), bs16_lds_bytes<LOGK>(), s, q0, q3, ctr, n);
    return hipGetLastError();
}

template <int LOGK>
hipError_t launch_bs(const RsJob& j, uint32_t n, hipStream_t s) {
    const uint32_t ncw = j.seg[0].n_cw + (j.n_seg > 1 ? j.seg[1].n_cw : 0);
    static bool attr = false;   // function attribute, set once per instantiation
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(rs16_bs_kernel<LOGK>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs16_lds_bytes<LOGK>());
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(rs16_bs_kernel<LOGK>, dim3(2 * ncw, n), dim3(64 << (LOGK - 7)), bs16_lds_bytes<LOGK>(), s, j);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_rs16_bs(const RsJob& j, uint32_t k, uint32_t n, hipStream_t s) {
    if (k == 512) return launch_bs<9>(j, n, s);
    if (k == 256) return launch_bs<8>(j, n, s);
    return hipErrorInvalidValue;
}

hipError_t launch_rs16_bs_square(const RsJob& q0, const RsJob& q3, uint32_t* ctr, uint32_t k, uint32_t n,
                                 hipStream_t s) {
    // the ticket decode assumes both Q0 segments (rows, columns) and Q3 hold k codewords
    if (q0.n_seg != 2 || q0.seg[0].n_cw != k || q0.seg[1].n_cw != k || q3.n_seg != 1 || q3.seg[0].n_cw != k ||
        q3.src != q0.dst || q3.dst != q0.dst || q3.dst_sq != q0.dst_sq || !ctr || n == 0)
        return hipErrorInvalidValue;
    if (k == 512) return launch_ticket<9>(q0, q3.seg[0], ctr, n, s);
    if (k == 256) return launch_ticket<8>(q0, q3.seg[0], ctr, n, s);
    return hipErrorInvalidValue;
}

}  // namespace cda
