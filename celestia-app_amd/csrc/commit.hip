// commit.hip -- blob share commitments on the device.
//
// go-square v1.1.0 inclusion.CreateCommitment (EXT, go.mod:9) as called by
// x/blob/types/blob_tx.go:98 (ValidateBlobTx: every blob of every BlobTx in
// CheckTx / ProcessProposal) and x/blob/types/payforblob.go:53
// (CreateCommitments), with merkle.HashFromByteSlices:
//   shares = SplitBlobs(blob); w = SubTreeWidth(#shares, threshold);
//   subtree roots = NMT roots over the Merkle-mountain-range runs (sizes w,
//   ..., decreasing powers of two) of leaves ns || share;
//   commitment = RFC-6962 root of the subtree roots.
//
// MI355X mapping for a batch of blobs (plan: square_plan.cpp
// plan_commitments):
//   1. share writer (square.hip) lays every blob's sparse shares into one leaf
//      array, blob starts aligned to their w, so all subtrees are perfect
//      trees aligned to their size;
//   2. leaf_kernel (nmt.hip) hashes every leaf (9 SHA-256 blocks of
//      0x00 || ns || share -- the same leaves as the EDS Q0 cells);
//   3. one subtree_level_kernel launch per level for ALL subtrees of ALL
//      blobs: node n of level L covers leaves [n << L, (n + 1) << L); a binary
//      search over the subtree table tells whether it lies inside a subtree
//      tall enough (else the thread exits); a subtree's top node goes to its
//      root slot;
//   4. commitment_kernel: one workgroup per blob, RFC-6962 over its subtree
//      roots in LDS (odd nodes promoted, which equals the RFC split rule).
// VALU-bound like the EDS hashing: 9 compressions per share + 3 per inner node
// + 2 per subtree root and RFC node.
#include <cstring>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

using square::Tree;

// Height-0 subtrees (single share): the root is the leaf node itself.
__global__ __launch_bounds__(256) void leaf_roots_kernel(const Tree* __restrict__ trees, uint32_t n_trees,
                                                         const uint8_t* __restrict__ leaf_slots,
                                                         uint8_t* __restrict__ roots) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n_trees || trees[t].height != 0) return;
    const uint4* s = reinterpret_cast<const uint4*>(leaf_slots + (size_t)trees[t].off * kSlot);
    uint4* d = reinterpret_cast<uint4*>(roots + (size_t)t * kSlot);
#pragma unroll
    for (int q = 0; q < kSlot / 16; q++) d[q] = s[q];
}

__global__ __launch_bounds__(256) void subtree_level_kernel(const Tree* __restrict__ trees, uint32_t n_trees,
                                                            const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                            uint8_t* __restrict__ roots, uint32_t level,
                                                            uint32_t n_nodes) {
    const uint32_t n = blockIdx.x * 256 + threadIdx.x;
    if (n >= n_nodes) return;
    const uint32_t leaf0 = n << level;
    uint32_t lo = 0, hi = n_trees;   // last subtree with off <= leaf0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (trees[mid].off <= leaf0) lo = mid;
        else hi = mid;
    }
    const Tree T = trees[lo];
    if (T.off > leaf0 || T.height < level || leaf0 - T.off >= (1u << T.height)) return;
    uint32_t L[kSlotWords], R[kSlotWords], w[16];
    load_slot_be(in + (size_t)(2 * n) * kSlot, L);
    load_slot_be(in + (size_t)(2 * n + 1) * kSlot, R);
    ShaState st;
    sha_init(st);
#pragma unroll
    for (int b = 0; b < 3; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 16 * b + i);
        sha_compress(st, w);
    }
    uint32_t o[kSlotWords];
    inner_node_words(L, R, st.h, o);
    store_slot(T.height == level ? roots + (size_t)lo * kSlot : out + (size_t)n * kSlot, o);
}

__device__ __forceinline__ void rfc_inner(const uint32_t* a, const uint32_t* b, uint32_t* o) {
    uint32_t A[8], B[8], w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) { A[j] = a[j]; B[j] = b[j]; }
    ShaState st;
    sha_init(st);
#pragma unroll
    for (int q = 0; q < 2; q++) {
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(A, B, 16 * q + j);
        sha_compress(st, w);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) o[j] = st.h[j];
}

// One workgroup per blob: RFC-6962 root of its subtree roots.
__global__ __launch_bounds__(256) void commitment_kernel(const uint8_t* __restrict__ roots,
                                                         const uint32_t* __restrict__ blob_tree0, uint32_t max_trees,
                                                         uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hs[];   // [max_trees][8] | [(max_trees+1)/2][8]
    const uint32_t b = blockIdx.x;
    const uint32_t t0 = blob_tree0[b];
    uint32_t m = blob_tree0[b + 1] - t0;
    uint32_t* o = reinterpret_cast<uint32_t*>(out + (size_t)b * 32);
    if (m == 0) {   // no shares: merkle.HashFromByteSlices(nil) = sha256("")
        if (threadIdx.x == 0) {
            const uint32_t e[8] = {0x42c4b0e3u, 0x141cfc98u, 0xc8f4fb9au, 0x24b96f99u,
                                   0xe441ae27u, 0x4c939b64u, 0x1b9995a4u, 0x55b85278u};
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = e[j];
        }
        return;
    }
    uint32_t* src = hs;
    uint32_t* dst = hs + max_trees * 8;
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
        uint32_t I[kSlotWords], w[16];
        load_slot_be(roots + (size_t)(t0 + i) * kSlot, I);
        ShaState st;
        sha_init(st);
#pragma unroll
        for (int q = 0; q < 2; q++) {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = rfc_leaf_msg(I, 16 * q + j);
            sha_compress(st, w);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) src[i * 8 + j] = st.h[j];
    }
    __syncthreads();
    while (m > 1) {
        const uint32_t pairs = m / 2;
        for (uint32_t i = threadIdx.x; i < pairs; i += blockDim.x) rfc_inner(src + 16 * i, src + 16 * i + 8, dst + 8 * i);
        if ((m & 1) && threadIdx.x < 8) dst[pairs * 8 + threadIdx.x] = src[(m - 1) * 8 + threadIdx.x];
        __syncthreads();
        uint32_t* t = src;
        src = dst;
        dst = t;
        m = pairs + (m & 1);
    }
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = bswap32(src[j]);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// Engine glue
// ---------------------------------------------------------------------------
int Engine::enqueue_commitments(const square::CommitPlan& p, uint32_t n_blobs, const uint8_t* d_data, uint8_t* d_out,
                                hipStream_t s) {
    if (n_blobs == 0) return CDA_OK;
    const size_t seg_b = p.segs.size() * sizeof(square::Segment);
    const size_t tree_b = p.trees.size() * sizeof(Tree);
    const size_t bt_b = p.blob_tree0.size() * 4;
    const size_t plan_b = seg_b + tree_b + bt_b;
    int rc;
    if (sq_event_ && (rc = check(hipEventSynchronize(sq_event_), "hipEventSynchronize"))) return rc;
    if (plan_b > sq_stage_bytes_) {
        if (sq_stage_) (void)hipHostFree(sq_stage_);
        sq_stage_ = nullptr;
        sq_stage_bytes_ = 0;
        if ((rc = check(hipHostMalloc(&sq_stage_, plan_b, hipHostMallocDefault), "hipHostMalloc"))) return rc;
        sq_stage_bytes_ = plan_b;
    }
    if (!sq_event_ && (rc = check(hipEventCreateWithFlags(&sq_event_, hipEventDisableTiming), "hipEventCreate")))
        return rc;
    uint8_t* stage = static_cast<uint8_t*>(sq_stage_);
    if (seg_b) std::memcpy(stage, p.segs.data(), seg_b);
    if (tree_b) std::memcpy(stage + seg_b, p.trees.data(), tree_b);
    std::memcpy(stage + seg_b + tree_b, p.blob_tree0.data(), bt_b);
    if ((rc = check(cm_plan_.ensure(plan_b), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(cm_plan_.ptr, stage, plan_b, hipMemcpyHostToDevice, s), "H2D plan"))) return rc;
    if ((rc = check(hipEventRecord(sq_event_, s), "hipEventRecord"))) return rc;
    const square::Segment* d_segs = cm_plan_.as<square::Segment>();
    const Tree* d_trees = reinterpret_cast<const Tree*>(cm_plan_.as<uint8_t>() + seg_b);
    const uint32_t* d_bt = reinterpret_cast<const uint32_t*>(cm_plan_.as<uint8_t>() + seg_b + tree_b);
    const uint32_t N = p.n_leaves, n_trees = (uint32_t)p.trees.size();
    if (N) {
        if ((rc = check(cm_shares_.ensure((size_t)N * kShare), "hipMalloc"))) return rc;
        if ((rc = check(cm_leaf_.ensure((size_t)N * kSlot), "hipMalloc"))) return rc;
        if ((rc = check(cm_lvl_.ensure((size_t)(N / 2 + 1) * kSlot), "hipMalloc"))) return rc;
        if ((rc = check(cm_roots_.ensure((size_t)n_trees * kSlot), "hipMalloc"))) return rc;
        if ((rc = check(err_buf_.ensure(4), "hipMalloc"))) return rc;
        if ((rc = check(launch_share_writer(d_segs, (uint32_t)p.segs.size(), nullptr, d_data, cm_shares_.as<uint8_t>(),
                                            N, s),
                        "share writer")))
            return rc;
        const CellGrid g{cm_shares_.as<uint8_t>(), 0, 1, N, N, 0, 0, 0xFFFFFFFFu};
        if ((rc = check(launch_leaves(g, 1, cm_leaf_.as<uint8_t>(), err_buf_.as<uint32_t>(), false, false, s),
                        "leaves")))
            return rc;
        hipLaunchKernelGGL(leaf_roots_kernel, dim3((n_trees + 255) / 256), dim3(256), 0, s, d_trees, n_trees,
                           cm_leaf_.as<uint8_t>(), cm_roots_.as<uint8_t>());
        if ((rc = check(hipGetLastError(), "leaf roots"))) return rc;
        for (uint32_t L = 1; L <= p.max_height; L++) {
            uint8_t* in = (L - 1) % 2 == 0 ? cm_leaf_.as<uint8_t>() : cm_lvl_.as<uint8_t>();
            uint8_t* out = L % 2 == 0 ? cm_leaf_.as<uint8_t>() : cm_lvl_.as<uint8_t>();
            const uint32_t n_nodes = (uint32_t)(((uint64_t)N + (1ull << L) - 1) >> L);
            hipLaunchKernelGGL(subtree_level_kernel, dim3((n_nodes + 255) / 256), dim3(256), 0, s, d_trees, n_trees, in,
                               out, cm_roots_.as<uint8_t>(), L, n_nodes);
            if ((rc = check(hipGetLastError(), "subtree level"))) return rc;
        }
    }
    const uint32_t mt = p.max_trees ? p.max_trees : 1;
    const size_t lds = (size_t)(mt + (mt + 1) / 2) * 32;
    if (lds > 160 * 1024) return fail(CDA_ERR_UNSUPPORTED, "too many subtree roots in one blob");
    if (lds > 64 * 1024 &&
        (rc = check(hipFuncSetAttribute(reinterpret_cast<const void*>(commitment_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                    "hipFuncSetAttribute")))
        return rc;
    hipLaunchKernelGGL(commitment_kernel, dim3(n_blobs), dim3(256), lds, s, cm_roots_.as<uint8_t>(), d_bt, mt, d_out);
    return check(hipGetLastError(), "commitments");
}

int Engine::host_commitments(const square::CommitPlan& p, uint32_t n_blobs, const uint8_t* data, size_t data_len,
                             uint8_t* out) {
    hipStream_t s = stream_;
    int rc;
    if ((rc = upload_txs(data, data_len, s))) return rc;
    if ((rc = check(cm_out_.ensure((size_t)n_blobs * 32), "hipMalloc"))) return rc;
    if ((rc = enqueue_commitments(p, n_blobs, sq_txs_.as<uint8_t>(), cm_out_.as<uint8_t>(), s))) return rc;
    if ((rc = check(hipMemcpyAsync(out, cm_out_.ptr, (size_t)n_blobs * 32, hipMemcpyDeviceToHost, s), "D2H")))
        return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace cda
