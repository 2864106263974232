// repair.hip -- EDS repair: Leopard erasure decode of
// EDS rows / columns on the GPU and the rsmt2d crossword driver.
//
// Restates (EXT modules, go.mod:11,152; not vendored):
//   klauspost/reedsolomon v1.12.1 leopardFF8/FF16 reconstruct (as called by
//     rsmt2d LeoRSCodec.Decode -> Reconstruct, recoverAll):
//       work index of data shard i = m + i, of parity shard i = i (m = k);
//       errLocs = FWHT(FWHT(E) * logWalsh)  -- an XOR-convolution, i.e.
//       errLoc[i] = sum_{j in E} log[i ^ j] (mod MOD; the transform size is
//       2^BITS = 1 mod MOD, so the two FWHTs compose to the identity);
//       work = received * g^errLoc (erasures 0); IFFT (skew offset 0, size
//       n = 2k); formal derivative; FFT; erased shard = work * g^-errLoc.
//   rsmt2d v0.14.0 ExtendedDataSquare.Repair: pre-repair sanity check of
//     complete rows / columns (roots and parity), then the crossword loop.
//
// The decoded symbols are unique (MDS), so any correct decoder is bit-exact
// with the reference's; tests check encode -> erase -> repair round trips and
// the reference's error outcomes (ErrByzantineData, ErrUnrepairableDataSquare).
//
// MI355X mapping: one workgroup per (codeword, 64-B column block) with the
// n x 64 B block in LDS (n = 2k <= 1024); log / exp / skew tables through L1/L2.
// Per-codeword error locators come from a separate kernel (one workgroup per
// codeword).  Every sweep decodes all decodable rows (then columns) at once;
// roots are re-verified with the regular NMT kernels.
#include <algorithm>
#include <cstring>
#include <memory>
#include <tuple>

#include "../../include/cda.h"
#include "engine.h"
#include "leopard_tables.h"
#include "sha256_dev.h"

namespace cda {

namespace {

struct FieldDev {
    const uint16_t* log;
    const uint16_t* exp;
    const uint16_t* skew;
    uint32_t bits, mod;
};

// Codeword descriptor: axis 0 = row, 1 = column; index in the EDS.
struct Cw {
    uint32_t axis, index;
};

__device__ __forceinline__ uint32_t cell_off(const Cw c, uint32_t pos, uint32_t W) {
    return c.axis == 0 ? c.index * W + pos : pos * W + c.index;
}

// errLoc[cw][i] = sum over erased work indexes j of log[i ^ j] (mod MOD).
__global__ __launch_bounds__(256) void errloc_kernel(FieldDev F, const Cw* __restrict__ cws,
                                                     const uint8_t* __restrict__ present, uint32_t k,
                                                     uint16_t* __restrict__ err) {
    extern __shared__ uint32_t erased[];   // work indexes of the erasures
    __shared__ uint32_t n_er;
    const Cw c = cws[blockIdx.x];
    const uint32_t n = 2 * k, W = 2 * k;
    if (threadIdx.x == 0) n_er = 0;
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < n; p += blockDim.x)
        if (!present[cell_off(c, p, W)]) erased[atomicAdd(&n_er, 1u)] = p ^ k;   // work index
    __syncthreads();
    const uint32_t ne = n_er;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t acc = 0;
        for (uint32_t q = 0; q < ne; q++) {
            const uint32_t j = erased[q];
            if (j != i) acc += F.log[i ^ j];
        }
        err[(size_t)blockIdx.x * n + i] = (uint16_t)(acc % F.mod);
    }
}

__device__ __forceinline__ uint32_t gmul(const FieldDev& F, uint32_t x, uint32_t L) {   // x * g^L
    if (x == 0) return 0;
    uint32_t s = F.log[x] + L;
    s = (s + (s >> F.bits)) & F.mod;
    return F.exp[s];
}

// One 64-B column block of one codeword: S symbols per shard (64 for GF(2^8),
// 32 for GF(2^16) with the lo/hi byte split of leopard's 64-byte blocks).
template <int BITS>
__global__ __launch_bounds__(256) void decode_kernel(FieldDev F, const Cw* __restrict__ cws, uint8_t* __restrict__ eds,
                                                     const uint8_t* __restrict__ present, uint32_t k,
                                                     const uint16_t* __restrict__ errloc, uint32_t shard_len) {
    constexpr uint32_t S = BITS == 8 ? 64 : 32;
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];   // work[n][S] | tmp[n][S]
    const uint32_t blocks = shard_len / 64;
    const uint32_t cwi = blockIdx.x / blocks, blk = blockIdx.x % blocks;
    const Cw c = cws[cwi];
    const uint32_t n = 2 * k, W = 2 * k, tid = threadIdx.x, nt = blockDim.x;
    const uint16_t* el = errloc + (size_t)cwi * n;
    uint16_t* work = lds;
    uint16_t* tmp = lds + n * S;
    // load: work[w(p)] = received[p] * g^errLoc (erasures 0)
    for (uint32_t it = tid; it < n * S; it += nt) {
        const uint32_t p = it / S, s = it % S, w = p ^ k;
        const uint32_t off = cell_off(c, p, W);
        uint32_t x = 0;
        if (present[off]) {
            const uint8_t* b = eds + (size_t)off * shard_len + blk * 64;
            x = BITS == 8 ? b[s] : (uint32_t)b[s] | ((uint32_t)b[s + 32] << 8);
            x = gmul(F, x, el[w]);
        }
        work[w * S + s] = (uint16_t)x;
    }
    __syncthreads();
    // IFFT (ifftDITDecoder, skew offset 0)
    for (uint32_t d = 1; d < n; d <<= 1) {
        for (uint32_t it = tid; it < (n / 2) * S; it += nt) {
            const uint32_t q = it / S, s = it % S;
            const uint32_t g = (q / d) * 2 * d, i = g + (q % d);
            const uint32_t L = F.skew[g + d - 1];
            uint32_t x = work[i * S + s], y = work[(i + d) * S + s];
            y ^= x;
            if (L != F.mod) x ^= gmul(F, y, L);
            work[i * S + s] = (uint16_t)x;
            work[(i + d) * S + s] = (uint16_t)y;
        }
        __syncthreads();
    }
    // formal derivative: the reference's in-order updates only ever read
    // original values, so new[p] = old[p] ^ sum of old[p + w] over the powers
    // of two w with floor(p / w) even and (floor(p / w) + 1) * w < n.
    for (uint32_t it = tid; it < n * S; it += nt) {
        const uint32_t p = it / S, s = it % S;
        uint32_t x = work[p * S + s];
        for (uint32_t w = 1; w < n; w <<= 1)
            if (((p / w) & 1) == 0 && (p / w + 1) * w < n) x ^= work[(p + w) * S + s];
        tmp[p * S + s] = (uint16_t)x;
    }
    __syncthreads();
    // FFT (fftDIT, skew offset 0)
    for (uint32_t d = n / 2; d >= 1; d >>= 1) {
        for (uint32_t it = tid; it < (n / 2) * S; it += nt) {
            const uint32_t q = it / S, s = it % S;
            const uint32_t g = (q / d) * 2 * d, i = g + (q % d);
            const uint32_t L = F.skew[g + d - 1];
            uint32_t x = tmp[i * S + s], y = tmp[(i + d) * S + s];
            if (L != F.mod) x ^= gmul(F, y, L);
            y ^= x;
            tmp[i * S + s] = (uint16_t)x;
            tmp[(i + d) * S + s] = (uint16_t)y;
        }
        __syncthreads();
    }
    // reveal erasures: shard = work * g^(MOD - errLoc)
    for (uint32_t it = tid; it < n * (BITS == 8 ? S : 2 * S); it += nt) {
        const uint32_t p = BITS == 8 ? it / S : it / (2 * S);
        const uint32_t off = cell_off(c, p, W);
        if (present[off]) continue;
        const uint32_t w = p ^ k;
        uint8_t* b = eds + (size_t)off * shard_len + blk * 64;
        if (BITS == 8) {
            const uint32_t s = it % S;
            b[s] = (uint8_t)gmul(F, tmp[w * S + s], F.mod - el[w]);
        } else {
            const uint32_t byte = it % (2 * S), s = byte % 32;
            const uint32_t v = gmul(F, tmp[w * S + s], F.mod - el[w]);
            b[byte] = (uint8_t)(byte < 32 ? v : v >> 8);
        }
    }
}

// GF(2^8) decode, dword form: a thread handles 4 packed symbols (one dword of
// a shard's 64-B column block) per step, and multiplies by a runtime constant
// with the 2-bit-chunk v_perm tables of all 255 logs (make_all_mul8), staged
// in LDS with the skew vector: 4 v_perm + 7 selector ops per 4 symbols instead
// of two dependent log/exp lookups per symbol.  Same algorithm and order as
// decode_kernel<8>.
constexpr Mul8All kMul8Dec = make_all_mul8(make_gf8());
__constant__ Mul8All kMul8Tab = kMul8Dec;

__device__ __forceinline__ uint32_t mul8v(uint32_t y, const uint4 T) {
    const uint32_t m = 0x03030303u;
    const uint32_t p0 = __builtin_amdgcn_perm(T.x, T.x, y & m);
    const uint32_t p1 = __builtin_amdgcn_perm(T.y, T.y, (y >> 2) & m);
    const uint32_t p2 = __builtin_amdgcn_perm(T.z, T.z, (y >> 4) & m);
    const uint32_t p3 = __builtin_amdgcn_perm(T.w, T.w, (y >> 6) & m);
    return p0 ^ p1 ^ p2 ^ p3;
}

__global__ __launch_bounds__(256) void decode8_kernel(const uint16_t* __restrict__ skew, const Cw* __restrict__ cws,
                                                      uint8_t* __restrict__ eds, const uint8_t* __restrict__ present,
                                                      uint32_t k, const uint16_t* __restrict__ errloc,
                                                      uint32_t shard_len) {
    constexpr uint32_t Q = 16;   // dwords per 64-B column block
    extern __shared__ __attribute__((aligned(16))) uint32_t lds8[];   // tab[256] uint4 | skew[256] u16 | work | tmp
    uint4* tab = reinterpret_cast<uint4*>(lds8);
    uint16_t* sk = reinterpret_cast<uint16_t*>(lds8 + 1024);
    const uint32_t n = 2 * k, W = 2 * k, tid = threadIdx.x, nt = blockDim.x;
    uint32_t* work = lds8 + 1024 + 128;
    uint32_t* tmp = work + n * Q;
    const uint32_t blocks = shard_len / 64;
    const uint32_t cwi = blockIdx.x / blocks, blk = blockIdx.x % blocks;
    const Cw c = cws[cwi];
    const uint16_t* el = errloc + (size_t)cwi * n;
    for (uint32_t i = tid; i < 256; i += nt) {
        const Mul8Chunks& t = kMul8Tab.t[i];
        tab[i] = make_uint4(t.c[0], t.c[1], t.c[2], t.c[3]);
        sk[i] = i < 255 ? skew[i] : 255;
    }
    __syncthreads();
    for (uint32_t it = tid; it < n * Q; it += nt) {
        const uint32_t p = it / Q, q = it % Q, w = p ^ k;
        const uint32_t off = cell_off(c, p, W);
        uint32_t x = 0;
        if (present[off]) {
            x = *reinterpret_cast<const uint32_t*>(eds + (size_t)off * shard_len + blk * 64 + 4 * q);
            x = mul8v(x, tab[el[w]]);
        }
        work[w * Q + q] = x;
    }
    __syncthreads();
    for (uint32_t d = 1; d < n; d <<= 1) {   // IFFT (ifftDITDecoder, skew offset 0)
        for (uint32_t it = tid; it < (n / 2) * Q; it += nt) {
            const uint32_t b = it / Q, q = it % Q;
            const uint32_t g = (b / d) * 2 * d, i = g + (b % d);
            const uint32_t L = sk[g + d - 1];
            uint32_t x = work[i * Q + q], y = work[(i + d) * Q + q];
            y ^= x;
            if (L != 255) x ^= mul8v(y, tab[L]);
            work[i * Q + q] = x;
            work[(i + d) * Q + q] = y;
        }
        __syncthreads();
    }
    for (uint32_t it = tid; it < n * Q; it += nt) {   // formal derivative (see decode_kernel)
        const uint32_t p = it / Q, q = it % Q;
        uint32_t x = work[p * Q + q];
        for (uint32_t w = 1; w < n; w <<= 1)
            if (((p / w) & 1) == 0 && (p / w + 1) * w < n) x ^= work[(p + w) * Q + q];
        tmp[p * Q + q] = x;
    }
    __syncthreads();
    for (uint32_t d = n / 2; d >= 1; d >>= 1) {   // FFT (fftDIT, skew offset 0)
        for (uint32_t it = tid; it < (n / 2) * Q; it += nt) {
            const uint32_t b = it / Q, q = it % Q;
            const uint32_t g = (b / d) * 2 * d, i = g + (b % d);
            const uint32_t L = sk[g + d - 1];
            uint32_t x = tmp[i * Q + q], y = tmp[(i + d) * Q + q];
            if (L != 255) x ^= mul8v(y, tab[L]);
            y ^= x;
            tmp[i * Q + q] = x;
            tmp[(i + d) * Q + q] = y;
        }
        __syncthreads();
    }
    for (uint32_t it = tid; it < n * Q; it += nt) {   // reveal erasures: work * g^(255 - errLoc)
        const uint32_t p = it / Q, q = it % Q;
        const uint32_t off = cell_off(c, p, W);
        if (present[off]) continue;
        const uint32_t w = p ^ k;
        *reinterpret_cast<uint32_t*>(eds + (size_t)off * shard_len + blk * 64 + 4 * q) =
            mul8v(tmp[w * Q + q], tab[255 - el[w]]);
    }
}

// Mark every cell of the listed codewords present.
__global__ void mark_kernel(const Cw* __restrict__ cws, uint32_t n_cw, uint8_t* __restrict__ present, uint32_t W) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n_cw * W) return;
    const Cw c = cws[t / W];
    present[cell_off(c, t % W, W)] = 1;
}

// Parity check of every row (blockIdx.x < W) and column: compare the k
// re-encoded parity shards with the EDS cells k..2k-1 of the vector.
__global__ __launch_bounds__(64) void parity_compare_kernel(const uint8_t* __restrict__ eds,
                                                            const uint8_t* __restrict__ parity, uint32_t k,
                                                            uint32_t* __restrict__ flags) {
    const uint32_t W = 2 * k, v = blockIdx.x, p = blockIdx.y;
    const uint32_t axis = v / W, i = v % W;
    const size_t c = axis == 0 ? (size_t)i * W + k + p : (size_t)(k + p) * W + i;
    const uint64_t* a = reinterpret_cast<const uint64_t*>(eds + c * 512);
    const uint64_t* b = reinterpret_cast<const uint64_t*>(parity + ((size_t)v * k + p) * 512);
    const bool diff = a[threadIdx.x] != b[threadIdx.x];
    if (__any(diff) && threadIdx.x == 0) atomicOr(&flags[v], 1u);
}

}  // namespace

// ---------------------------------------------------------------------------
// Engine glue
// ---------------------------------------------------------------------------
int Engine::ensure_gf8_tables() {
    if (gf8_log_.ptr) return CDA_OK;
    auto F = std::make_unique<LeoField<8>>();
    leo_build<8>(*F, 0x11D, kCantor8);
    int rc;
    for (auto [buf, src, len] : {std::tuple{&gf8_log_, (const void*)F->log, sizeof F->log},
                                 std::tuple{&gf8_exp_, (const void*)F->exp, sizeof F->exp},
                                 std::tuple{&gf8_skew_, (const void*)F->skew, sizeof F->skew}}) {
        if ((rc = check(buf->ensure_fixed(len), "hipMalloc"))) return rc;   // filled by a host copy below
        if ((rc = check(hipMemcpy(buf->ptr, src, len, hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
    }
    return CDA_OK;
}

// Copies n host bytes into the pinned staging area and returns the staged
// address (for an async H2D on s).  When the area is full, waits for s
// (the earlier copies out of it are then done) and starts over.
uint8_t* Engine::rp_stage(const void* src, size_t n, hipStream_t s, int* rc) {
    const size_t need = (n + 63) & ~(size_t)63;
    if (rp_host_used_ + need > rp_host_bytes_) {
        if ((*rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return nullptr;
        rp_host_used_ = 0;
        if (need > rp_host_bytes_) {
            if (rp_host_) (void)hipHostFree(rp_host_);
            rp_host_ = nullptr;
            rp_host_bytes_ = 0;
            const size_t cap = std::max(need, (size_t)4 << 20);
            if ((*rc = check(hipHostMalloc(&rp_host_, cap, hipHostMallocDefault), "hipHostMalloc"))) return nullptr;
            rp_host_bytes_ = cap;
        }
    }
    uint8_t* p = static_cast<uint8_t*>(rp_host_) + rp_host_used_;
    std::memcpy(p, src, n);
    rp_host_used_ += need;
    *rc = CDA_OK;
    return p;
}

int Engine::decode_codewords(uint8_t* d_eds, uint8_t* d_present, uint32_t k, uint32_t shard_len,
                             const std::vector<uint32_t>& axis_index, hipStream_t s) {
    const uint32_t n_cw = (uint32_t)axis_index.size() / 2;
    if (n_cw == 0) return CDA_OK;
    const uint32_t n = 2 * k;
    int rc;
    FieldDev F;
    if (k <= 128) {
        if ((rc = ensure_gf8_tables())) return rc;
        F = FieldDev{gf8_log_.as<uint16_t>(), gf8_exp_.as<uint16_t>(), gf8_skew_.as<uint16_t>(), 8, 255};
    } else {
        F = FieldDev{gf16_log_.as<uint16_t>(), gf16_exp_.as<uint16_t>(), gf16_skew_.as<uint16_t>(), 16, 65535};
    }
    if ((rc = check(rp_cw_.ensure((size_t)n_cw * sizeof(Cw)), "hipMalloc"))) return rc;
    if ((rc = check(rp_err_.ensure((size_t)n_cw * n * 2), "hipMalloc"))) return rc;
    const uint8_t* staged = rp_stage(axis_index.data(), (size_t)n_cw * sizeof(Cw), s, &rc);
    if (!staged) return rc;
    if ((rc = check(hipMemcpyAsync(rp_cw_.ptr, staged, (size_t)n_cw * sizeof(Cw), hipMemcpyHostToDevice, s), "H2D")))
        return rc;
    hipLaunchKernelGGL(errloc_kernel, dim3(n_cw), dim3(256), n * 4, s, F, rp_cw_.as<Cw>(), d_present, k,
                       rp_err_.as<uint16_t>());
    if ((rc = check(hipGetLastError(), "errloc"))) return rc;
    const uint32_t S = k <= 128 ? 64 : 32;
    const size_t lds = (size_t)2 * n * S * 2;
    if (k <= 128) {
        const size_t lds8 = (1024 + 128 + (size_t)2 * n * 16) * 4;
        hipLaunchKernelGGL(decode8_kernel, dim3(n_cw * (shard_len / 64)), dim3(256), lds8, s, F.skew, rp_cw_.as<Cw>(),
                           d_eds, d_present, k, rp_err_.as<uint16_t>(), shard_len);
    } else {
        if (lds > 64 * 1024 &&
            (rc = check(hipFuncSetAttribute(reinterpret_cast<const void*>(decode_kernel<16>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        "hipFuncSetAttribute")))
            return rc;
        hipLaunchKernelGGL(decode_kernel<16>, dim3(n_cw * (shard_len / 64)), dim3(256), lds, s, F, rp_cw_.as<Cw>(),
                           d_eds, d_present, k, rp_err_.as<uint16_t>(), shard_len);
    }
    if ((rc = check(hipGetLastError(), "decode"))) return rc;
    hipLaunchKernelGGL(mark_kernel, dim3((n_cw * n + 255) / 256), dim3(256), 0, s, rp_cw_.as<Cw>(), n_cw, d_present, n);
    return check(hipGetLastError(), "mark");
}

namespace {

std::string hex(const uint8_t* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; i++) {
        s += d[p[i] >> 4];
        s += d[p[i] & 15];
    }
    return s;
}

}  // namespace

// Verification of the device EDS E against the DAH (used by the sanity
// check, after the batched sweeps and by the exact replay): the roots of
// every row and column (one enqueue_dah) and the parity of every row and
// column re-encoded from its data half and compared on the device.
// bad[axis * W + i]: bit 0 = root differs, bit 1 = parity differs;
// meaningful for complete vectors only.
int Engine::repair_verify(const uint8_t* E, uint32_t k, const uint8_t* row_roots, const uint8_t* col_roots,
                          std::vector<uint8_t>& bad, hipStream_t s) {
    const uint32_t W = 2 * k, SH = kShare;
    const size_t roots_b = (size_t)W * kNode;
    int rc;
    if ((rc = check(rp_parity_.ensure((size_t)2 * W * k * SH), "hipMalloc"))) return rc;
    if ((rc = check(rp_flags_.ensure((size_t)2 * W * 4), "hipMalloc"))) return rc;
    if ((rc = enqueue_dah(E, k, 1, h_rows_.as<uint8_t>(), h_cols_.as<uint8_t>(), nullptr, err_buf_.as<uint32_t>(),
                          nullptr, s)))
        return rc;
    RsJob j{};
    j.src = E;
    j.dst = rp_parity_.as<uint8_t>();
    j.n_seg = 2;
    j.seg[0] = RsSeg{W, 0, W * SH, SH, 0, k * SH, SH};              // rows: data half = cells 0..k-1
    j.seg[1] = RsSeg{W, 0, SH, W * SH, W * k * SH, k * SH, SH};     // columns
    if ((rc = check(launch_rs(j, k, 1, gf16(k), s), "parity re-encode"))) return rc;
    if ((rc = check(hipMemsetAsync(rp_flags_.ptr, 0, (size_t)2 * W * 4, s), "hipMemsetAsync"))) return rc;
    hipLaunchKernelGGL(parity_compare_kernel, dim3(2 * W, k), dim3(64), 0, s, E, rp_parity_.as<uint8_t>(), k,
                       rp_flags_.as<uint32_t>());
    if ((rc = check(hipGetLastError(), "parity compare"))) return rc;
    // results land in pinned memory: the copies queue right behind the
    // kernels (a pageable destination makes each copy wait for the stream and
    // go through a staging blit)
    const size_t flags_b = (size_t)2 * W * 4, out_b = 2 * roots_b + flags_b;
    if (out_b > rp_out_bytes_) {
        if (rp_out_) (void)hipHostFree(rp_out_);
        rp_out_ = nullptr;
        rp_out_bytes_ = 0;
        if ((rc = check(hipHostMalloc(&rp_out_, out_b, hipHostMallocDefault), "hipHostMalloc"))) return rc;
        rp_out_bytes_ = out_b;
    }
    uint8_t* ob = static_cast<uint8_t*>(rp_out_);
    if ((rc = check(hipMemcpyAsync(ob, h_rows_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(ob + roots_b, h_cols_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(ob + 2 * roots_b, rp_flags_.ptr, flags_b, hipMemcpyDeviceToHost, s), "D2H")))
        return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    const std::vector<uint8_t> rows(ob, ob + roots_b), cols(ob + roots_b, ob + 2 * roots_b);
    std::vector<uint32_t> flags(2 * W);
    std::memcpy(flags.data(), ob + 2 * roots_b, flags_b);
    bad.assign(2 * W, 0);
    for (uint32_t axis = 0; axis < 2; axis++) {
        const uint8_t* want = axis == 0 ? row_roots : col_roots;
        const uint8_t* got = axis == 0 ? rows.data() : cols.data();
        for (uint32_t i = 0; i < W; i++)
            bad[axis * W + i] = (std::memcmp(want + (size_t)i * kNode, got + (size_t)i * kNode, kNode) ? 1 : 0) |
                                (flags[axis * W + i] ? 2 : 0);
    }
    rp_roots_.assign(rows.begin(), rows.end());
    rp_roots_.insert(rp_roots_.end(), cols.begin(), cols.end());
    return CDA_OK;
}

// rsmt2d ExtendedDataSquare.Repair on a host or device EDS (cells whose
// present[] is 0 are ignored and overwritten).  Returns CDA_OK, CDA_ERR_BYZANTINE (axis /
// index in *byz_axis / *byz_index), CDA_ERR_UNREPAIRABLE or CDA_ERR_INVALID
// ("bad root input").  The square is copied back in every one of these
// outcomes (partially repaired on an error).
//
// Fast path: sweeps that decode every decodable row at once, then every
// decodable column, up to the fixed point of "decode any vector with >= k
// cells" (unique, so the reference's row/column interleaving reaches the
// same one), then one verification of every complete vector (which covers
// the reference's pre-repair sanity check: see precheck).  When all of
// them match their roots and are codewords, each decode the reference would
// have run saw cells of that same codeword, so its result and its checks are
// the ones of the fast path (MDS uniqueness, by induction over its order).
// Otherwise the crossword is replayed from the input in the reference's
// order (for i: row i, column i) with the checks after every decode, which
// names the same first byzantine vector as rsmt2d.
int Engine::host_repair(uint8_t* eds, const uint8_t* present_in, uint32_t W, const uint8_t* row_roots,
                        const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index) {
    return repair(eds, nullptr, present_in, W, row_roots, col_roots, byz_axis, byz_index);
}

int Engine::device_repair(uint8_t* d_eds, const uint8_t* present_in, uint32_t W, const uint8_t* row_roots,
                          const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index) {
    // the square may have been written on any stream of the caller
    if (int rc = check(hipDeviceSynchronize(), "hipDeviceSynchronize")) return rc;
    return repair(nullptr, d_eds, present_in, W, row_roots, col_roots, byz_axis, byz_index);
}

// One of `eds` (host) / `d_eds` (device, repaired in place) is set.  The
// host square is staged in h_eds_; a device square keeps a pristine copy in
// rp_buf_ for the exact replay.
int Engine::repair(uint8_t* eds, uint8_t* d_eds, const uint8_t* present_in, uint32_t W, const uint8_t* row_roots,
                   const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index) {
    const uint32_t k = W / 2;
    if (W < 2 || (W & (W - 1)) || k > 512) return fail(CDA_ERR_INVALID, "EDS width must be a power of two in [2, 1024]");
    const size_t eds_b = (size_t)W * W * kShare, roots_b = (size_t)W * kNode;
    hipStream_t s = stream_;
    int rc;
    // earlier copies out of the staging area are done once s is idle
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    rp_host_used_ = 0;
    DevBuf& stage = d_eds ? rp_buf_ : h_eds_;
    if ((rc = check(stage.ensure(eds_b), "hipMalloc"))) return rc;
    if ((rc = check(rp_present_.ensure((size_t)W * W), "hipMalloc"))) return rc;
    if ((rc = check(h_rows_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_cols_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure(32), "hipMalloc"))) return rc;
    if ((rc = check(err_buf_.ensure(4), "hipMalloc"))) return rc;
    std::vector<uint8_t> present;
    uint8_t* E = d_eds ? d_eds : h_eds_.as<uint8_t>();
    bool first = true;
    auto upload = [&]() -> int {
        present.assign(present_in, present_in + (size_t)W * W);
        for (auto& v : present) v = v ? 1 : 0;
        int r;
        if (!d_eds) {
            if ((r = check(hipMemcpyAsync(E, eds, eds_b, hipMemcpyHostToDevice, s), "H2D"))) return r;
        } else if (first) {
            if ((r = check(hipMemcpyAsync(stage.ptr, E, eds_b, hipMemcpyDeviceToDevice, s), "D2D"))) return r;
        } else if ((r = check(hipMemcpyAsync(E, stage.ptr, eds_b, hipMemcpyDeviceToDevice, s), "D2D"))) {
            return r;
        }
        first = false;
        const uint8_t* staged = rp_stage(present.data(), present.size(), s, &r);
        if (!staged) return r;
        return check(hipMemcpyAsync(rp_present_.ptr, staged, present.size(), hipMemcpyHostToDevice, s), "H2D");
    };
    auto cell = [&](uint32_t axis, uint32_t i, uint32_t p) {
        return axis == 0 ? (size_t)i * W + p : (size_t)p * W + i;
    };
    auto count = [&](uint32_t axis, uint32_t i) {
        uint32_t c = 0;
        for (uint32_t p = 0; p < W; p++) c += present[cell(axis, i, p)];
        return c;
    };
    auto download = [&](int code) -> int {
        int r;
        if (!d_eds && (r = check(hipMemcpyAsync(eds, E, eds_b, hipMemcpyDeviceToHost, s), "D2H"))) return r;
        if ((r = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return r;
        return code;
    };
    auto byzantine = [&](uint32_t axis, uint32_t i) {
        if (byz_axis) *byz_axis = (int32_t)axis;
        if (byz_index) *byz_index = i;
        char buf[64];
        snprintf(buf, sizeof buf, "byzantine %s: %u", axis == 0 ? "row" : "col", i);
        const int code = fail(CDA_ERR_BYZANTINE, buf);
        const int r = download(code);
        return r == code ? code : r;
    };
    std::vector<uint8_t> bad;
    // ---- preRepairSanityCheck: every complete vector must match its root
    // ("bad root input", a plain error) and re-encode to its parity
    // (ErrByzantineData).  rsmt2d runs these checks in parallel goroutines;
    // the first failure in (index, row before column, root before parity)
    // order is reported here.  Run only on the error path: a vector complete
    // in the input keeps its cells through the sweeps, so a clean final
    // verification implies this check passed.
    auto precheck = [&]() -> int {
        int r;
        if ((r = repair_verify(E, k, row_roots, col_roots, bad, s))) return r;
        for (uint32_t i = 0; i < W; i++)
            for (uint32_t axis = 0; axis < 2; axis++) {
                if (count(axis, i) != W) continue;
                const uint8_t b = bad[axis * W + i];
                if (b & 1) {
                    char head[64];
                    snprintf(head, sizeof head, "bad root input: %s %u expected ", axis == 0 ? "row" : "col", i);
                    const uint8_t* want = (axis == 0 ? row_roots : col_roots) + (size_t)i * kNode;
                    return fail(CDA_ERR_INVALID, std::string(head) + hex(want, kNode) + " got " +
                                                     hex(rp_roots_.data() + ((size_t)axis * W + i) * kNode, kNode));
                }
                if (b & 2) return byzantine(axis, i);
            }
        return CDA_OK;
    };
    if ((rc = upload())) return rc;
    // ---- fast path: batched sweeps to the fixed point, then verification
    bool solved = false;
    for (;;) {
        bool progress = false;
        for (uint32_t axis = 0; axis < 2; axis++) {
            std::vector<uint32_t> cw;
            for (uint32_t i = 0; i < W; i++) {
                const uint32_t c = count(axis, i);
                if (c != W && c >= k) cw.push_back(axis), cw.push_back(i);
            }
            if (cw.empty()) continue;
            if ((rc = decode_codewords(E, rp_present_.as<uint8_t>(), k, kShare, cw, s))) return rc;
            for (size_t q = 1; q < cw.size(); q += 2)
                for (uint32_t p = 0; p < W; p++) present[cell(axis, cw[q], p)] = 1;
            progress = true;
        }
        solved = std::all_of(present.begin(), present.end(), [](uint8_t v) { return v != 0; });
        if (solved || !progress) break;
    }
    if ((rc = repair_verify(E, k, row_roots, col_roots, bad, s))) return rc;
    bool clean = true;
    for (uint32_t axis = 0; axis < 2 && clean; axis++)
        for (uint32_t i = 0; i < W && clean; i++)
            if (bad[axis * W + i] && count(axis, i) == W) clean = false;
    if (clean) {
        if (solved) return download(CDA_OK);
        const int code = fail(CDA_ERR_UNREPAIRABLE, "failed to solve data square");
        const int r = download(code);
        return r == code ? code : r;
    }
    // ---- error path: from the input again, the sanity check, then the exact
    // replay of solveCrossword
    if ((rc = upload())) return rc;
    if ((rc = precheck())) return rc;
    for (;;) {
        bool all = true, progress = false;
        for (uint32_t i = 0; i < W; i++)
            for (uint32_t axis = 0; axis < 2; axis++) {
                const uint32_t c = count(axis, i);
                if (c == W) continue;
                if (c < k) {
                    all = false;
                    continue;
                }
                std::vector<uint8_t> was(W);   // orthogonal vectors complete but for this one's cell
                const uint32_t ox = 1 - axis;
                for (uint32_t o = 0; o < W; o++)
                    was[o] = !present[cell(axis, i, o)] && count(ox, o) == W - 1;
                const std::vector<uint32_t> cw{axis, i};
                if ((rc = decode_codewords(E, rp_present_.as<uint8_t>(), k, kShare, cw, s))) return rc;
                for (uint32_t p = 0; p < W; p++) present[cell(axis, i, p)] = 1;
                progress = true;
                if ((rc = repair_verify(E, k, row_roots, col_roots, bad, s))) return rc;
                // the rebuilt vector against its root, then the orthogonal
                // vectors it completed against their roots and encodings
                if (bad[axis * W + i] & 1) return byzantine(axis, i);
                for (uint32_t o = 0; o < W; o++)
                    if (was[o] && bad[ox * W + o]) return byzantine(ox, o);
            }
        if (all) return download(CDA_OK);   // unreachable when the fast path failed, kept for safety
        if (!progress) {
            const int code = fail(CDA_ERR_UNREPAIRABLE, "failed to solve data square");
            const int r = download(code);
            return r == code ? code : r;
        }
    }
}

int Engine::host_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t k, uint32_t shard_len,
                           uint32_t n_codewords) {
    // rsmt2d Codec.Decode: n codewords of 2k shards x shard_len bytes,
    // contiguous; missing shards (present[] == 0) are reconstructed in place.
    if (k == 0 || (k & (k - 1)) || k > 512) return fail(CDA_ERR_UNSUPPORTED, "shard count must be a power of two <= 512");
    if (shard_len == 0 || shard_len % 64) {
        char buf[80];
        snprintf(buf, sizeof buf, "chunkSize %u must be a multiple of 64 bytes", shard_len);
        return fail(CDA_ERR_CHUNK_SIZE, buf);
    }
    const uint32_t W = 2 * k;
    std::vector<uint32_t> cw;
    for (uint32_t i = 0; i < n_codewords; i++) {
        uint32_t cnt = 0;
        for (uint32_t p = 0; p < W; p++) cnt += present[(size_t)i * W + p] ? 1 : 0;
        if (cnt < k) return fail(CDA_ERR_UNREPAIRABLE, "too few shards given");
        if (cnt < W) {
            cw.push_back(0);
            cw.push_back(i);
        }
    }
    hipStream_t s = stream_;
    const size_t b = (size_t)n_codewords * W * shard_len;
    int rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    rp_host_used_ = 0;
    if ((rc = check(rp_buf_.ensure(b), "hipMalloc"))) return rc;
    if ((rc = check(rp_present_.ensure((size_t)n_codewords * W), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(rp_buf_.ptr, shards, b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = check(hipMemcpyAsync(rp_present_.ptr, present, (size_t)n_codewords * W, hipMemcpyHostToDevice, s),
                    "H2D")))
        return rc;
    // row codewords of a "W-wide" grid: cell (i, p) = codeword i, shard p
    if ((rc = decode_codewords(rp_buf_.as<uint8_t>(), rp_present_.as<uint8_t>(), k, shard_len, cw, s))) return rc;
    if ((rc = check(hipMemcpyAsync(shards, rp_buf_.ptr, b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace cda
