// tree.hip -- standalone erasured NMT trees and generic RFC-6962 roots.
//
// Reference behaviour (paths under /root/reference):
//   * pkg/wrapper/nmt_wrapper.go:55-140: NewErasuredNamespacedMerkleTree,
//     Push (leaf namespace = data[0:29] when isQuadrantZero, else
//     ParitySharesNamespace), Root, ProveRange -- used outside
//     ComputeExtendedDataSquare by pkg/proof/proof.go:157-189,
//     pkg/inclusion/nmt_caching.go:96-109 and test/util/malicious/tree.go:46-70.
//   * nmt v0.22.0 (EXT; hasher rules copied in-tree at
//     test/util/malicious/hasher.go:186-310): computeRoot splits n leaves at
//     the largest power of two < n (RFC-6962).  Pairing adjacent nodes level by
//     level and promoting an odd last node unchanged builds the same tree, so
//     every level is one launch for all trees whatever n is.
//   * go-square/merkle HashFromByteSlices (RFC-6962, same split rule) over
//     arbitrary byte slices: (*DataAvailabilityHeader).Hash,
//     pkg/da/data_availability_header.go:92-108, for any root count / size.
//
// The square-shaped case (512-B cells, power-of-two leaf count, consecutive
// axis indexes) runs on the tuned leaf/level kernels of nmt.hip; these generic
// kernels take any cell length and leaf count (byte-addressed message build).
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

// SHA-256 of pre[0:npre] || data[0:len] (npre <= 32), big-endian state words.
__device__ void sha_generic(const uint8_t (&pre)[32], uint32_t npre, const uint8_t* __restrict__ data, uint64_t len,
                            uint32_t (&out)[8]) {
    ShaState st;
    sha_init(st);
    const uint64_t total = npre + len;
    const uint64_t n_blocks = (total + 9 + 63) / 64;
    auto byte_at = [&](uint64_t i) -> uint32_t {
        if (i < npre) return pre[i];
        if (i < total) return data[i - npre];
        if (i == total) return 0x80u;
        return 0;
    };
    const uint64_t bits = total * 8;
    for (uint64_t b = 0; b < n_blocks; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint64_t p = b * 64 + 4 * j;
            w[j] = (byte_at(p) << 24) | (byte_at(p + 1) << 16) | (byte_at(p + 2) << 8) | byte_at(p + 3);
        }
        if (b == n_blocks - 1) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha_compress(st, w);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = st.h[j];
}

// Big-endian namespace words of a cell (byte 28 in the top byte of word 7).
__device__ void ns_words(const uint8_t* cell, bool parity, uint32_t (&ns)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = 4 * j + q;
            const uint32_t byte = parity ? 0xFFu : (i < kNs ? cell[i] : 0u);
            v |= (i < kNs ? byte : 0u) << (24 - 8 * q);
        }
        ns[j] = v;
    }
}

__device__ __forceinline__ bool ns_less_w(const uint32_t (&a)[8], const uint32_t (&b)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (a[i] != b[i]) return a[i] < b[i];
    return false;
}

// One leaf per (tree, push): slot = ns || ns || sha256(0x00 || ns || cell).
// err[t] = min push position whose namespace is below the previous one.
__global__ __launch_bounds__(256) void gen_leaf_kernel(const uint8_t* __restrict__ cells, uint32_t cell_len,
                                                      uint32_t n_cells, uint32_t n_trees, uint32_t square_size,
                                                      const uint32_t* __restrict__ axis, uint8_t* __restrict__ slots,
                                                      uint32_t* __restrict__ err) {
    const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= (uint64_t)n_trees * n_cells) return;
    const uint32_t t = (uint32_t)(id / n_cells), i = (uint32_t)(id % n_cells);
    const uint32_t ax = axis[t];
    const uint8_t* cell = cells + id * cell_len;
    const bool parity = !(i < square_size && ax < square_size);   // isQuadrantZero
    uint32_t ns[8];
    ns_words(cell, parity, ns);
    uint8_t pre[32];
    pre[0] = 0x00;
#pragma unroll
    for (int j = 0; j < kNs; j++) pre[1 + j] = (uint8_t)(ns[j / 4] >> (24 - 8 * (j % 4)));
    pre[30] = pre[31] = 0;
    uint32_t d[8];
    sha_generic(pre, 1 + kNs, cell, cell_len, d);
    uint32_t out[kSlotWords];
    leaf_node_words(ns, d, out);
    store_slot(slots + id * kSlot, out);
    if (i > 0) {
        uint32_t prev[8];
        ns_words(cell - cell_len, !((i - 1) < square_size && ax < square_size), prev);
        if (ns_less_w(ns, prev)) atomicMin(err + t, i);
    }
}

// One level of every tree: parent p of tree t = HashNode(2p, 2p+1), or the
// odd last node promoted unchanged (RFC-6962 split, see the header).
__global__ __launch_bounds__(256) void gen_level_kernel(const uint8_t* __restrict__ in, uint32_t n_in,
                                                       uint8_t* __restrict__ out, uint32_t n_trees, uint64_t in_tree,
                                                       uint64_t out_tree) {
    const uint32_t n_out = (n_in + 1) / 2;
    const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= (uint64_t)n_trees * n_out) return;
    const uint32_t t = (uint32_t)(id / n_out), p = (uint32_t)(id % n_out);
    const uint8_t* l = in + t * in_tree + (uint64_t)(2 * p) * kSlot;
    uint8_t* o = out + t * out_tree + (uint64_t)p * kSlot;
    if (2 * p + 1 >= n_in) {
        const uint4* s = reinterpret_cast<const uint4*>(l);
        uint4* d = reinterpret_cast<uint4*>(o);
#pragma unroll
        for (int q = 0; q < 6; q++) d[q] = s[q];
        return;
    }
    uint32_t L[kSlotWords], R[kSlotWords], w[16];
    load_slot_be(l, L);
    load_slot_be(l + kSlot, R);
    ShaState st;
    sha_init(st);
#pragma unroll
    for (int b = 0; b < 3; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 16 * b + i);
        sha_compress(st, w);
    }
    uint32_t ow[kSlotWords];
    inner_node_words(L, R, st.h, ow);
    store_slot(o, ow);
}

// RFC-6962 leaf digests of arbitrary byte items: sha256(0x00 || item).
__global__ __launch_bounds__(256) void gen_rfc_leaf_kernel(const uint8_t* __restrict__ items,
                                                          const uint64_t* __restrict__ off, uint32_t n,
                                                          uint32_t* __restrict__ dig) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t pre[32] = {0};
    uint32_t d[8];
    sha_generic(pre, 1, items + off[i], off[i + 1] - off[i], d);
#pragma unroll
    for (int j = 0; j < 8; j++) dig[(size_t)i * 8 + j] = d[j];
}

// RFC-6962 inner levels of one tree of n digests in a single workgroup
// (pairs hashed, an odd last digest promoted); dig is overwritten.
__global__ __launch_bounds__(256) void gen_rfc_levels_kernel(uint32_t* __restrict__ dig, uint32_t n,
                                                            uint8_t* __restrict__ root) {
    for (uint32_t m = n; m > 1; m = (m + 1) / 2) {
        const uint32_t half = m / 2;
        // parents are written in place over slots 0..half-1 after all reads
        // of this level: first hash into registers, then barrier, then store
        for (uint32_t base = 0; base < half; base += blockDim.x) {
            const uint32_t p = base + threadIdx.x;
            uint32_t h[8];
            if (p < half) {
                uint32_t A[8], B[8], w[16];
#pragma unroll
                for (int j = 0; j < 8; j++) { A[j] = dig[(2 * p) * 8 + j]; B[j] = dig[(2 * p + 1) * 8 + j]; }
                ShaState st;
                sha_init(st);
#pragma unroll
                for (int b = 0; b < 2; b++) {
#pragma unroll
                    for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(A, B, 16 * b + j);
                    sha_compress(st, w);
                }
#pragma unroll
                for (int j = 0; j < 8; j++) h[j] = st.h[j];
            }
            __syncthreads();
            if (p < half) {
#pragma unroll
                for (int j = 0; j < 8; j++) dig[p * 8 + j] = h[j];
            }
            __syncthreads();
        }
        if (m & 1) {   // promote the odd last digest to slot half
            if (threadIdx.x < 8) dig[half * 8 + threadIdx.x] = dig[(m - 1) * 8 + threadIdx.x];
            __syncthreads();
        }
    }
    if (threadIdx.x < 8) reinterpret_cast<uint32_t*>(root)[threadIdx.x] = bswap32(dig[threadIdx.x]);
}

// Copy n 96-B slots at byte offsets src_off[i] of `base` into packed 90-B nodes.
__global__ __launch_bounds__(64) void gen_gather_nodes_kernel(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ src_off, uint32_t n,
                                                             uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    for (uint32_t b = threadIdx.x; b < (uint32_t)kNode; b += blockDim.x) out[(size_t)i * kNode + b] = base[src_off[i] + b];
}

// Pack tree roots (slot 0 of the last level of tree t) into 90-B roots.
__global__ __launch_bounds__(96) void gen_pack_roots_kernel(const uint8_t* __restrict__ top, uint64_t tree_stride,
                                                           uint32_t n_trees, uint8_t* __restrict__ roots) {
    const uint32_t t = blockIdx.x;
    if (t < n_trees && threadIdx.x < (uint32_t)kNode)
        roots[(size_t)t * kNode + threadIdx.x] = top[t * tree_stride + threadIdx.x];
}

const uint8_t kEmptyRoot[kNode] = {
    // NmtHasher.EmptyRoot: 0^29 || 0^29 || sha256("")
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
    0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

// Level sizes of the promoted-pairing tree over n leaves: n, ceil(n/2), ..., 1.
std::vector<uint32_t> level_counts(uint32_t n) {
    std::vector<uint32_t> c{n};
    while (c.back() > 1) c.push_back((c.back() + 1) / 2);
    return c;
}

// nmt ProveRange node order: maximal subtrees outside [start, end), depth
// first, left to right, as (level, index) of the promoted-pairing tree.
void prove_nodes(uint32_t lo, uint32_t hi, uint32_t start, uint32_t end, std::vector<std::pair<uint32_t, uint32_t>>& out) {
    if (hi <= start || lo >= end) {
        uint32_t L = 0;
        while ((1u << L) < hi - lo) L++;   // subtree [lo, hi) = node lo >> L of level L
        out.emplace_back(L, lo >> L);
        return;
    }
    if (hi - lo == 1) return;
    uint32_t k = 1;
    while (2 * k < hi - lo) k *= 2;   // largest power of two < n (RFC-6962 split)
    prove_nodes(lo, lo + k, start, end, out);
    prove_nodes(lo + k, hi, start, end, out);
}

}  // namespace

// All levels of n_trees erasured trees over host cells into tr_ (device):
// level L of tree t at tr_ + off[L] + t * count[L] * 96.  err words per tree.
int Engine::build_trees(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees,
                        uint32_t square_size, const uint32_t* axis, std::vector<uint64_t>* level_off,
                        std::vector<uint32_t>* err_out) {
    hipStream_t s = stream_;
    const std::vector<uint32_t> cnt = level_counts(n_cells);
    level_off->assign(cnt.size(), 0);
    uint64_t total = 0;
    for (size_t L = 0; L < cnt.size(); L++) {
        (*level_off)[L] = total;
        total += (uint64_t)cnt[L] * n_trees * kSlot;
    }
    const uint64_t cells_b = (uint64_t)n_trees * n_cells * cell_len;
    int rc;
    if ((rc = check(tr_cells_.ensure(cells_b + 16), "hipMalloc tree cells"))) return rc;
    if ((rc = check(tr_levels_.ensure(total), "hipMalloc tree levels"))) return rc;
    if ((rc = check(tr_axis_.ensure((size_t)n_trees * 8), "hipMalloc tree axes"))) return rc;
    uint32_t* d_axis = tr_axis_.as<uint32_t>();
    uint32_t* d_err = d_axis + n_trees;
    if ((rc = check(hipMemcpyAsync(tr_cells_.ptr, cells, cells_b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = check(hipMemcpyAsync(d_axis, axis, (size_t)n_trees * 4, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = check(hipMemsetAsync(d_err, 0xFF, (size_t)n_trees * 4, s), "hipMemsetAsync"))) return rc;
    uint8_t* lv = tr_levels_.as<uint8_t>();
    const uint64_t n_leaves = (uint64_t)n_trees * n_cells;
    hipLaunchKernelGGL(gen_leaf_kernel, dim3((uint32_t)((n_leaves + 255) / 256)), dim3(256), 0, s,
                       tr_cells_.as<uint8_t>(), cell_len, n_cells, n_trees, square_size, d_axis, lv, d_err);
    if ((rc = check(hipGetLastError(), "tree leaves"))) return rc;
    for (size_t L = 1; L < cnt.size(); L++) {
        const uint64_t work = (uint64_t)n_trees * cnt[L];
        hipLaunchKernelGGL(gen_level_kernel, dim3((uint32_t)((work + 255) / 256)), dim3(256), 0, s,
                           lv + (*level_off)[L - 1], cnt[L - 1], lv + (*level_off)[L], n_trees,
                           (uint64_t)cnt[L - 1] * kSlot, (uint64_t)cnt[L] * kSlot);
        if ((rc = check(hipGetLastError(), "tree level"))) return rc;
    }
    err_out->assign(n_trees, 0);
    if ((rc = check(hipMemcpyAsync(err_out->data(), d_err, (size_t)n_trees * 4, hipMemcpyDeviceToHost, s), "D2H")))
        return rc;
    return CDA_OK;
}

int Engine::tree_order_error(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                             const uint32_t* axis, const std::vector<uint32_t>& err, int32_t* status) {
    int rc = CDA_OK;
    for (size_t t = 0; t < err.size(); t++) {
        if (status) status[t] = err[t] == 0xFFFFFFFFu ? CDA_OK : CDA_ERR_PUSH_ORDER;
        if (err[t] == 0xFFFFFFFFu || rc != CDA_OK) continue;
        const uint32_t i = err[t];
        auto ns_hex = [&](uint32_t pos) {
            const uint8_t* c = cells + ((uint64_t)t * n_cells + pos) * cell_len;
            const bool par = !(pos < square_size && axis[t] < square_size);
            std::string h;
            char hx[3];
            for (int b = 0; b < kNs; b++) {
                snprintf(hx, sizeof hx, "%02x", par ? 0xFF : c[b]);
                h += hx;
            }
            return h;
        };
        po_axis = 0;
        po_index = axis[t];
        po_pos = i;
        rc = fail(CDA_ERR_PUSH_ORDER, "pushed data has to be lexicographically ordered by namespace IDs: last namespace: " +
                                          ns_hex(i - 1) + ", pushed: " + ns_hex(i));
    }
    return rc;
}

int Engine::nmt_axis_roots(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees,
                           uint32_t square_size, const uint32_t* axis, uint8_t* roots, int32_t* status) {
    if (n_cells == 0) {   // no pushes: NmtHasher.EmptyRoot
        for (uint32_t t = 0; t < n_trees; t++) {
            memcpy(roots + (size_t)t * kNode, kEmptyRoot, kNode);
            if (status) status[t] = CDA_OK;
        }
        return CDA_OK;
    }
    hipStream_t s = stream_;
    int rc;
    bool consecutive = true;
    for (uint32_t t = 1; t < n_trees; t++) consecutive = consecutive && axis[t] == axis[0] + t;
    if (cell_len == (uint32_t)kShare && n_cells >= 2 && is_pow2(n_cells) && consecutive && axis[0] + n_trees <= 4096 &&
        n_cells < 4096) {
        // square-shaped: the tuned leaf / level kernels of nmt.hip
        const uint64_t cells_b = (uint64_t)n_trees * n_cells * kShare, slots = (uint64_t)n_trees * n_cells * kSlot;
        if ((rc = check(tr_cells_.ensure(cells_b), "hipMalloc tree cells"))) return rc;
        if ((rc = check(tr_levels_.ensure(2 * slots), "hipMalloc tree levels"))) return rc;
        if ((rc = check(tr_axis_.ensure((size_t)n_trees * kNode + 64), "hipMalloc tree roots"))) return rc;
        uint8_t* d_roots = tr_axis_.as<uint8_t>();
        uint32_t* d_err = reinterpret_cast<uint32_t*>(d_roots + (((size_t)n_trees * kNode + 15) & ~(size_t)15));
        uint8_t* leaf = tr_levels_.as<uint8_t>();
        uint8_t* lvl = leaf + slots;
        if ((rc = check(hipMemcpyAsync(tr_cells_.ptr, cells, cells_b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
        if ((rc = check(hipMemsetAsync(d_err, 0xFF, 4, s), "hipMemsetAsync"))) return rc;
        const CellGrid g{tr_cells_.as<uint8_t>(), 0, n_trees, n_cells, n_cells, axis[0], 0, square_size};
        if ((rc = check(launch_leaves(g, 1, leaf, d_err, true, false, s), "leaf hashing"))) return rc;
        Forest f{leaf, 0, n_trees, n_cells, 1, nullptr, 0, d_roots, 0, nullptr, 0, 0};
        const uint64_t off0[1] = {0};
        if ((rc = run_forests(&f, 1, n_cells, 1, lvl, leaf, 0, off0, s))) return rc;
        uint32_t err = 0;
        if ((rc = check(hipMemcpyAsync(roots, d_roots, (size_t)n_trees * kNode, hipMemcpyDeviceToHost, s), "D2H")))
            return rc;
        if ((rc = check(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
        if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
        // err = min over the batch's violations: a single word cannot tell
        // which other trees broke push order, so a batch with any violation
        // is re-run on the generic kernels, which keep one word per tree
        // (rare: an honest square never gets here)
        if (err == 0xFFFFFFFFu) {
            if (status)
                for (uint32_t t = 0; t < n_trees; t++) status[t] = CDA_OK;
            return CDA_OK;
        }
    }
    std::vector<uint64_t> off;
    std::vector<uint32_t> err;
    if ((rc = build_trees(cells, cell_len, n_cells, n_trees, square_size, axis, &off, &err))) return rc;
    if ((rc = check(tr_roots_.ensure((size_t)n_trees * kNode), "hipMalloc tree roots"))) return rc;
    hipLaunchKernelGGL(gen_pack_roots_kernel, dim3(n_trees), dim3(96), 0, s, tr_levels_.as<uint8_t>() + off.back(),
                       (uint64_t)kSlot, n_trees, tr_roots_.as<uint8_t>());
    if ((rc = check(hipGetLastError(), "pack roots"))) return rc;
    if ((rc = check(hipMemcpyAsync(roots, tr_roots_.ptr, (size_t)n_trees * kNode, hipMemcpyDeviceToHost, s), "D2H")))
        return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    return tree_order_error(cells, cell_len, n_cells, square_size, axis, err, status);
}

int Engine::nmt_prove_range(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                            uint32_t axis, uint32_t start, uint32_t end, uint8_t* nodes, uint32_t* n_nodes,
                            uint8_t* root) {
    if (start >= end || end > n_cells) return fail(CDA_ERR_INVALID, "invalid proof range");
    hipStream_t s = stream_;
    int rc;
    std::vector<uint64_t> off;
    std::vector<uint32_t> err;
    if ((rc = build_trees(cells, cell_len, n_cells, 1, square_size, &axis, &off, &err))) return rc;
    std::vector<std::pair<uint32_t, uint32_t>> ids;
    prove_nodes(0, n_cells, start, end, ids);
    const std::vector<uint32_t> cnt = level_counts(n_cells);
    std::vector<uint64_t> src(ids.size() + 1);
    for (size_t i = 0; i < ids.size(); i++) src[i] = off[ids[i].first] + (uint64_t)ids[i].second * kSlot;
    src[ids.size()] = off.back();   // the root
    const uint32_t n = (uint32_t)src.size();
    if ((rc = check(tr_roots_.ensure((size_t)n * (kNode + 8) + 64), "hipMalloc proof nodes"))) return rc;
    uint64_t* d_src = tr_roots_.as<uint64_t>();
    uint8_t* d_out = tr_roots_.as<uint8_t>() + (size_t)n * 8;
    if ((rc = check(hipMemcpyAsync(d_src, src.data(), (size_t)n * 8, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    hipLaunchKernelGGL(gen_gather_nodes_kernel, dim3(n), dim3(64), 0, s, tr_levels_.as<uint8_t>(), d_src, n, d_out);
    if ((rc = check(hipGetLastError(), "gather nodes"))) return rc;
    std::vector<uint8_t> host((size_t)n * kNode);
    if ((rc = check(hipMemcpyAsync(host.data(), d_out, host.size(), hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    if ((rc = tree_order_error(cells, cell_len, n_cells, square_size, &axis, err, nullptr))) return rc;
    if (nodes) memcpy(nodes, host.data(), (size_t)(n - 1) * kNode);
    if (n_nodes) *n_nodes = n - 1;
    if (root) memcpy(root, host.data() + (size_t)(n - 1) * kNode, kNode);
    return CDA_OK;
}

int Engine::merkle_root(const uint8_t* items, const uint64_t* off, uint32_t n, uint8_t* out) {
    hipStream_t s = stream_;
    int rc;
    const uint64_t bytes = off[n] - off[0];
    std::vector<uint64_t> rel(n + 1);
    for (uint32_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
    if ((rc = check(tr_cells_.ensure(bytes + 16), "hipMalloc merkle items"))) return rc;
    if ((rc = check(tr_levels_.ensure((size_t)n * 32), "hipMalloc merkle digests"))) return rc;
    if ((rc = check(tr_axis_.ensure((size_t)(n + 1) * 8 + 64), "hipMalloc merkle offsets"))) return rc;
    uint64_t* d_off = tr_axis_.as<uint64_t>();
    uint8_t* d_root = reinterpret_cast<uint8_t*>(d_off + n + 1);
    if (bytes && (rc = check(hipMemcpyAsync(tr_cells_.ptr, items + off[0], bytes, hipMemcpyHostToDevice, s), "H2D")))
        return rc;
    if ((rc = check(hipMemcpyAsync(d_off, rel.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s), "H2D")))
        return rc;
    hipLaunchKernelGGL(gen_rfc_leaf_kernel, dim3((n + 255) / 256), dim3(256), 0, s, tr_cells_.as<uint8_t>(), d_off, n,
                       tr_levels_.as<uint32_t>());
    if ((rc = check(hipGetLastError(), "merkle leaves"))) return rc;
    hipLaunchKernelGGL(gen_rfc_levels_kernel, dim3(1), dim3(256), 0, s, tr_levels_.as<uint32_t>(), n, d_root);
    if ((rc = check(hipGetLastError(), "merkle levels"))) return rc;
    if ((rc = check(hipMemcpyAsync(out, d_root, 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace cda
