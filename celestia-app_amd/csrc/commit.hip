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
//   1. every blob's sparse shares get leaf positions in one array, blob starts
//      aligned to their w, so all subtrees are perfect trees aligned to their
//      size; the host sends only the segment list (no per-subtree records);
//   2. blob_leaf_kernel finds each leaf's segment and subtree (and the first
//      leaf of each subtree writes the subtree record), then hashes the leaf
//      (9 SHA-256 blocks of 0x00 || ns || share -- the same leaves as the EDS
//      Q0 cells), building the share words straight from the blob bytes (no
//      share copy in HBM);
//   3. one subtree_level_kernel launch per level for ALL subtrees of ALL
//      blobs: node n of level L covers leaves [n << L, (n + 1) << L); the
//      per-leaf subtree table tells whether it lies inside a subtree tall
//      enough (else the thread exits).
//      A subtree's top node is hashed straight into its RFC-6962 leaf digest
//      sha256(0x00 || root) (parallel, off the per-blob serial chain); the
//      level-1 launch also does this for the single-share subtrees;
//   4. commitment_group_kernel: one wave per group of consecutive blobs,
//      RFC-6962 inner levels over those digests in LDS (odd nodes promoted,
//      equal to the RFC split rule).
// VALU-bound like the EDS hashing: 9 compressions per share + 3 per inner node
// + 2 per subtree root and RFC node.
#include "knobs.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

using square::Tree;

// RFC-6962 leaf digest sha256(0x00 || root90) of a subtree root (I = the
// root slot's big-endian words), stored as 8 state words: the commitment's
// Merkle leaves are hashed where the roots are produced, in parallel, instead
// of on the per-blob serial path.
__device__ __forceinline__ void store_rfc_leaf(const uint32_t (&I)[kSlotWords], uint32_t* __restrict__ dig) {
    uint32_t w[16];
    ShaState st;
    sha_init(st);
#pragma unroll
    for (int q = 0; q < 2; q++) {
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rfc_leaf_msg(I, 16 * q + j);
        sha_compress(st, w);
    }
    uint4* d = reinterpret_cast<uint4*>(dig);
    d[0] = make_uint4(st.h[0], st.h[1], st.h[2], st.h[3]);
    d[1] = make_uint4(st.h[4], st.h[5], st.h[6], st.h[7]);
}

// Per-leaf subtree index and the subtree list, built on the device from the
// plan's segment list (binary search per leaf, at the start of
// blob_leaf_kernel) instead of shipped over PCIe.  The subtree list is written here too: a blob's subtrees
// (inclusion.MerkleMountainRangeSizes: n >> sub_log full ones, then one per
// set bit of the remainder r, largest first) follow from its segment, and the
// first leaf of each subtree writes its record.  A remainder leaf j lies in
// the subtree of the highest bit where j and r differ (r has it set).
__device__ __forceinline__ uint32_t leaf_tables(uint32_t i, const square::Segment* __restrict__ segs, uint32_t n_segs,
                                                const uint32_t* __restrict__ seg_tree0, Tree* __restrict__ trees,
                                                uint32_t* __restrict__ leaf_tree) {
    uint32_t lo = 0, hi = n_segs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segs[mid].start <= i) lo = mid;
        else hi = mid;
    }
    const uint32_t t0 = seg_tree0[lo];
    const square::Segment* g = segs + lo;
    if (t0 == square::kNoTree || g->kind != square::kSegBlob) {
        leaf_tree[i] = square::kNoTree;
        return lo;
    }
    const uint32_t j = i - g->start, wl = g->sub_log, full = g->n >> wl;
    uint32_t q, off, h;
    if ((j >> wl) < full) {
        q = j >> wl;
        off = q << wl;
        h = wl;
    } else {
        const uint32_t base = full << wl, r = g->n - base, jr = j - base;
        h = 31u - (uint32_t)__builtin_clz(r ^ jr);
        q = full + (uint32_t)__builtin_popcount(r >> (h + 1));
        off = base + (r & ~((2u << h) - 1));
    }
    leaf_tree[i] = t0 + q;
    if (j == off) trees[t0 + q] = Tree{g->start + off, h};
    return lo;
}

// Leaf node of every blob share, hashed straight from the blob bytes (the
// sparse share is never materialised).  Message = 0x00 || ns || share (542 B,
// 9 blocks) with share = ns || info || [len BE32 if first] || data || zeros:
//   words 0..14  namespace twice + info byte (from the segment record);
//   word 15      first share: sequence length; continuation: data[0..3];
//   words 16..   4 blob bytes each, from B + 4(t - 16) where B is the blob
//                byte at message byte 64 (aligned dword loads + one v_perm
//                per word: shift and byte swap together), bytes past the
//                share's data masked to zero.
__device__ __forceinline__ uint32_t data_word(uint32_t lo, uint32_t hi, uint32_t sel, int32_t v) {
    const uint32_t x = __builtin_amdgcn_perm(hi, lo, sel);
    if (v >= 4) return x;
    if (v <= 0) return 0;
    return x & (0xFFFFFFFFu << (32 - 8 * v));
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void blob_leaf_kernel(
    const square::Segment* __restrict__ segs, uint32_t n_segs, const uint32_t* __restrict__ seg_tree0,
    Tree* __restrict__ trees, uint32_t* __restrict__ leaf_tree, const uint8_t* __restrict__ data,
    uint8_t* __restrict__ slots, uint32_t n_leaves) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_leaves) return;
    const square::Segment* g = segs + leaf_tables(i, segs, n_segs, seg_tree0, trees, leaf_tree);
    if (g->kind != square::kSegBlob) return;   // alignment gap: never read by a used node
    const uint32_t j = i - g->start, len = g->len;
    const bool first = j == 0;
    const uint32_t dbase = first ? 0u : (kShare - kNs - 5) + (j - 1) * (kShare - kNs - 1);
    const uint32_t cap = first ? kShare - kNs - 5 : kShare - kNs - 1;
    const uint32_t cnt = min(len - dbase, cap);
    const uint64_t B = g->src + dbase + (first ? 0 : 4);
    const int32_t L = (int32_t)cnt - (first ? 0 : 4);   // valid bytes from B
    const uint32_t sh = (uint32_t)(B & 3);
    const uint32_t sel = (sh << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
    // Dword indexes into `data` (batches < 16 GiB): A0 holds blob byte B; last
    // = the dword holding the share's last data byte.  Loads are branch-free:
    // each 4-dword chunk starts at min(chunk, last), so reads stay within 15
    // bytes of the last data byte (callers give 16 B of slack after the
    // buffer) and bytes past the data are masked by data_word.
    const uint32_t A0 = (uint32_t)(B >> 2);
    const uint32_t last = (uint32_t)(((int64_t)B + L - 1) >> 2);   // L >= -3 and B >= 4 when L <= 0
    const uint32_t* D = reinterpret_cast<const uint32_t*>(data);
    // one 16-byte load per chunk (dword-aligned: global loads need only
    // dword alignment), not four dword loads -- a lane's chunks lie in its
    // own share, so each load instruction touches 64 distinct cache lines
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    auto chunk = [&](uint32_t dw, uint32_t* x) {
        dw = min(dw, last);
        const u32x4a v = *reinterpret_cast<const u32x4a*>(D + dw);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    };

    uint32_t N[8];
    {
        const uint32_t* nsraw = reinterpret_cast<const uint32_t*>(g) + 7;   // Segment::ns at byte 28
#pragma unroll
        for (int k = 0; k < 8; k++) N[k] = bswap32(nsraw[k]);
    }
    const uint32_t info = (g->version << 1) | (first ? 1u : 0u);
    uint32_t w[16];
    w[0] = N[0] >> 8;
#pragma unroll
    for (int t = 1; t < 7; t++) w[t] = (N[t - 1] << 24) | (N[t] >> 8);
    w[7] = (N[6] << 24) | ((N[7] >> 24) << 16) | (N[0] >> 16);
#pragma unroll
    for (int t = 8; t < 14; t++) w[t] = (N[t - 8] << 16) | (N[t - 7] >> 16);
    w[14] = (N[6] << 16) | ((N[7] >> 24) << 8) | info;
    // R = the 17 dwords block b reads (R[0] shared with block b - 1); the next
    // block's 16 are loaded into X while the current block compresses.
    auto load16 = [&](int b, uint32_t (&X)[16]) {
        const uint32_t d0 = A0 + 16 * (b - 1) + 1;
#pragma unroll
        for (int c = 0; c < 4; c++) chunk(d0 + 4 * c, X + 4 * c);
    };
    uint32_t R0 = D[min(A0, last)], X[16];
    if (first) {
        w[15] = len;
    } else {
        const uint32_t Rm = D[A0 - 1];   // B - 4 >= the blob's first byte
        w[15] = data_word(Rm, R0, sel, L + 4);
    }
    load16(1, X);
    ShaState st;
    sha_init(st);
    sha_compress(st, w);
#pragma unroll 1
    for (int b = 1; b < 9; b++) {
        uint32_t R[17];
        R[0] = R0;
#pragma unroll
        for (int k = 0; k < 16; k++) R[k + 1] = X[k];
        if (b < 8) load16(b + 1, X);
        const int32_t o = 64 * (b - 1);
        if (b < 8) {
#pragma unroll
            for (int k = 0; k < 16; k++) w[k] = data_word(R[k], R[k + 1], sel, L - o - 4 * k);
        } else {
#pragma unroll
            for (int k = 0; k < 7; k++) w[k] = data_word(R[k], R[k + 1], sel, L - o - 4 * k);
            w[7] = data_word(R[7], R[8], sel, min(L - o - 28, 2)) | 0x8000u;   // message bytes 540..543
#pragma unroll
            for (int k = 8; k < 15; k++) w[k] = 0;
            w[15] = kLeafMsgBits;
        }
        sha_compress(st, w);
        R0 = R[16];
    }
    uint32_t out[kSlotWords];
    N[7] &= 0xFF000000u;
    leaf_node_words(N, st.h, out);
    store_slot(slots + (size_t)i * kSlot, out);
}

// Height-0 subtrees (single share): the root is the leaf node itself.
__global__ __launch_bounds__(256) void leaf_roots_kernel(const Tree* __restrict__ trees, uint32_t n_trees,
                                                         const uint8_t* __restrict__ leaf_slots,
                                                         uint32_t* __restrict__ dig) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n_trees || trees[t].height != 0) return;
    uint32_t I[kSlotWords];
    load_slot_be(leaf_slots + (size_t)trees[t].off * kSlot, I);
    store_rfc_leaf(I, dig + (size_t)t * 8);
}

__global__ __launch_bounds__(256) void subtree_level_kernel(const Tree* __restrict__ trees, uint32_t n_trees,
                                                            const uint32_t* __restrict__ leaf_tree,
                                                            const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                            uint32_t* __restrict__ dig, uint32_t level,
                                                            uint32_t n_nodes) {
    const uint32_t n = blockIdx.x * 256 + threadIdx.x;
    if (n >= n_nodes) {
        // level 1 also takes the height-0 subtrees (a single share: its RFC
        // leaf digest is of the leaf node itself), off the launch chain
        const uint32_t t = n - n_nodes;
        if (level != 1 || t >= n_trees || trees[t].height != 0) return;
        uint32_t I[kSlotWords];
        load_slot_be(in + (size_t)trees[t].off * kSlot, I);
        store_rfc_leaf(I, dig + (size_t)t * 8);
        return;
    }
    const uint32_t leaf0 = n << level;
    const uint32_t lo = leaf_tree[leaf0];   // subtree holding leaf0 (kNoTree: alignment gap)
    if (lo == square::kNoTree) return;
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
    if (T.height == level) {   // subtree root -> its RFC-6962 leaf digest
#pragma unroll
        for (int t = 0; t < kSlotWords; t++) L[t] = bswap32(o[t]);
        store_rfc_leaf(L, dig + (size_t)lo * 8);
    } else {
        store_slot(out + (size_t)n * kSlot, o);
    }
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

// One wave per blob: RFC-6962 root over its subtree roots' leaf digests (a
// blob has at most a few hundred subtrees; the chain of levels is serial, so
// a single wave per blob keeps every blob resident at once).
__global__ __launch_bounds__(64) void commitment_kernel(const uint32_t* __restrict__ dig,
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
    for (uint32_t i = threadIdx.x; i < m * 8; i += blockDim.x) src[i] = dig[(size_t)t0 * 8 + i];
    __syncthreads();
    while (m > 1) {
        const uint32_t pairs = m / 2;
        if (2 * pairs <= blockDim.x) {
            // a lane pair per parent (sha_pair_compress): the narrow levels
            // of the per-blob chain are latency-bound
            const uint32_t i = threadIdx.x >> 1;
            const bool A = threadIdx.x & 1;
            if (i < pairs) {
                uint32_t a[8], bb[8], D[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    a[j] = src[16 * i + j];
                    bb[j] = src[16 * i + 8 + j];
                }
                rfc_inner_u<true>(a, bb, D, A);
                if (!A) {
#pragma unroll
                    for (int j = 0; j < 8; j++) dst[8 * i + j] = D[j];
                }
            }
        } else {
            for (uint32_t i = threadIdx.x; i < pairs; i += blockDim.x) rfc_inner(src + 16 * i, src + 16 * i + 8, dst + 8 * i);
        }
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

// RFC-6962 levels of a group of G <= 64 consecutive blobs whose subtree-root
// digests sit in LDS (hs, blob i's at slots [bbase[i], bbase[i] + m_i)), by
// NT threads: each level's parents of all the group's blobs are one flat
// unit list (a lane pair per unit when they fit, else a lane per unit in
// passes), compacted in place at the front of each blob's slot range (every
// unit reads its two children before any unit writes; the odd node is
// promoted after the level's writes).  Wave 0's lanes i < G hold m_i / base_i
// and write blob i's commitment.
template <int NT>
__device__ __forceinline__ void group_rfc_levels(uint32_t* hs, uint32_t G, uint32_t m, uint32_t base, uint32_t b0,
                                                 uint32_t* pre, const uint32_t* bbase, uint32_t* s_total,
                                                 uint8_t* __restrict__ out, bool pair_ok) {
    const uint32_t tid = threadIdx.x;
    // blob of unit u: the first i with pre[i] > u (pre = inclusive prefix of
    // the level's parent counts)
    auto find = [&](uint32_t u) {
        if (G == 1) return 0u;
        uint32_t lo = 0, hi = G - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] > u) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    };
    for (;;) {
        const uint32_t p = m / 2;
        if (tid < 64) {
            uint32_t sc = p;
#pragma unroll
            for (int k = 1; k < 64; k <<= 1) {
                const uint32_t v = __shfl_up(sc, k, 64);
                if (tid >= (uint32_t)k) sc += v;
            }
            pre[tid] = sc;
            if (tid == 63) *s_total = sc;
        }
        const bool odd = (m & 1) && m > 1;
        uint32_t carry[8];
        if (odd) {
#pragma unroll
            for (int j = 0; j < 8; j++) carry[j] = hs[(base + m - 1) * 8 + j];
        }
        __syncthreads();
        const uint32_t total = *s_total;
        if (total == 0) break;
        if (pair_ok && 2 * total <= NT) {
            const uint32_t u = tid >> 1;
            const bool A = tid & 1;
            uint32_t D[8], slot = 0;
            if (u < total) {
                const uint32_t i = find(u);
                const uint32_t q = u - (i ? pre[i - 1] : 0u);
                const uint32_t c = (bbase[i] + 2 * q) * 8;
                uint32_t a[8], bb[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    a[j] = hs[c + j];
                    bb[j] = hs[c + 8 + j];
                }
                rfc_inner_u<true>(a, bb, D, A);
                slot = (bbase[i] + q) * 8;
            }
            __syncthreads();
            if (u < total && !A) {
#pragma unroll
                for (int j = 0; j < 8; j++) hs[slot + j] = D[j];
            }
        } else {
            // a later pass's children lie past every slot an earlier pass wrote
            for (uint32_t u0 = 0; u0 < total; u0 += NT) {
                const uint32_t u = u0 + tid;
                uint32_t D[8], slot = 0;
                if (u < total) {
                    const uint32_t i = find(u);
                    const uint32_t q = u - (i ? pre[i - 1] : 0u);
                    const uint32_t c = (bbase[i] + 2 * q) * 8;
                    rfc_inner(hs + c, hs + c + 8, D);
                    slot = (bbase[i] + q) * 8;
                }
                __syncthreads();
                if (u < total) {
#pragma unroll
                    for (int j = 0; j < 8; j++) hs[slot + j] = D[j];
                }
            }
        }
        __syncthreads();
        if (odd) {
#pragma unroll
            for (int j = 0; j < 8; j++) hs[(base + p) * 8 + j] = carry[j];
        }
        m = p + (m & 1);
        __syncthreads();
    }
    if (tid < G) {
        uint32_t* o = reinterpret_cast<uint32_t*>(out + (size_t)(b0 + tid) * 32);
        if (m == 0) {   // no shares: merkle.HashFromByteSlices(nil) = sha256("")
            const uint32_t e[8] = {0x42c4b0e3u, 0x141cfc98u, 0xc8f4fb9au, 0x24b96f99u,
                                   0xe441ae27u, 0x4c939b64u, 0x1b9995a4u, 0x55b85278u};
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = e[j];
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = bswap32(hs[base * 8 + j]);
        }
    }
}

// Blob groups: one wave takes the consecutive blobs [group_blob0[g],
// group_blob0[g + 1]) (at most 64) and runs their RFC-6962 levels together
// (group_rfc_levels), so the narrow upper levels of one blob share the
// wave's instruction stream with those of its neighbours instead of idling
// 60 of 64 lanes.
__global__ __launch_bounds__(64) void commitment_group_kernel(const uint32_t* __restrict__ dig,
                                                               const uint32_t* __restrict__ blob_tree0,
                                                               const uint32_t* __restrict__ group_blob0,
                                                               uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hs[];   // [group trees][8]
    __shared__ uint32_t pre[64], bbase[64], s_total;
    const uint32_t b0 = group_blob0[blockIdx.x], G = group_blob0[blockIdx.x + 1] - b0;
    const uint32_t lane = threadIdx.x;
    const uint32_t t_base = blob_tree0[b0], T = blob_tree0[b0 + G] - t_base;
    for (uint32_t i = lane; i < T * 8; i += 64) hs[i] = dig[(size_t)t_base * 8 + i];
    uint32_t m = 0, base = 0;
    if (lane < G) {
        base = blob_tree0[b0 + lane] - t_base;
        m = blob_tree0[b0 + lane + 1] - blob_tree0[b0 + lane];
        bbase[lane] = base;
    }
    __syncthreads();
    group_rfc_levels<64>(hs, G, m, base, b0, pre, bbase, &s_total, out, true);
}

// Small batches of small blobs (every blob at most kFusedMaxShares shares,
// at most one group per CU -- the latency case, e.g. one block's blobs in
// ProcessProposal): one 256-thread workgroup per group of consecutive blobs
// also runs the subtree
// levels, in LDS, after blob_leaf_kernel -- no launch per level, no slot
// round trips through HBM.  The group's leaf slots are loaded once
// (big-endian words); node n of level L lives at the slot of its first leaf
// (n << L), so a parent overwrites only its own left child and a level
// needs no barrier between reads and writes.  Subtree roots go straight to
// their RFC-6962 leaf digests, then group_rfc_levels.
constexpr uint32_t kFusedMaxShares = 512;
__global__ __launch_bounds__(256) void commitment_fused_kernel(const uint8_t* __restrict__ leaf_slots,
                                                               const Tree* __restrict__ trees,
                                                               const uint32_t* __restrict__ leaf_tree,
                                                               const uint32_t* __restrict__ blob_tree0,
                                                               const uint32_t* __restrict__ group_blob0,
                                                               uint8_t* __restrict__ out, uint32_t pair_ok) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    __shared__ uint32_t pre[64], bbase[64], s_total, s_maxh;
    const uint32_t tid = threadIdx.x;
    const uint32_t b0 = group_blob0[blockIdx.x], G = group_blob0[blockIdx.x + 1] - b0;
    const uint32_t T0 = blob_tree0[b0], T = blob_tree0[b0 + G] - T0;
    uint32_t L0 = 0, NL = 0;
    if (T) {
        const Tree first = trees[T0], last = trees[T0 + T - 1];
        L0 = first.off;
        NL = last.off + (1u << last.height) - L0;
    }
    uint32_t* slots = sm;                     // [NL][24] big-endian words
    uint32_t* dig = sm + NL * kSlotWords;     // [T][8] subtree roots' RFC leaf digests
    for (uint32_t i = tid; i < NL * 6; i += 256) {
        const uint4 v = *reinterpret_cast<const uint4*>(leaf_slots + (size_t)(L0 + i / 6) * kSlot + (i % 6) * 16);
        uint32_t* d = slots + (i / 6) * kSlotWords + (i % 6) * 4;
        d[0] = bswap32(v.x);
        d[1] = bswap32(v.y);
        d[2] = bswap32(v.z);
        d[3] = bswap32(v.w);
    }
    if (tid == 0) s_maxh = 0;
    __syncthreads();
    for (uint32_t t = tid; t < T; t += 256) {
        const Tree tr = trees[T0 + t];
        atomicMax(&s_maxh, tr.height);
        if (tr.height == 0) {   // a single share: the leaf is the subtree root
            uint32_t I[kSlotWords], D[8];
#pragma unroll
            for (int j = 0; j < kSlotWords; j++) I[j] = slots[(tr.off - L0) * kSlotWords + j];
            rfc_leaf_u<false>(I, D, false);
#pragma unroll
            for (int j = 0; j < 8; j++) dig[t * 8 + j] = D[j];
        }
    }
    __syncthreads();
    const uint32_t maxh = s_maxh;
    for (uint32_t L = 1; L <= maxh; L++) {
        const uint32_t n_lo = L0 >> L, cnt = ((L0 + NL - 1) >> L) - n_lo + 1;
        auto node = [&](uint32_t n, bool pair, bool A) {
            const uint32_t leaf0 = n << L;
            if (leaf0 < L0) return;
            const uint32_t lo = leaf_tree[leaf0];
            if (lo == square::kNoTree) return;
            const uint32_t h = trees[lo].height;
            if (h < L) return;
            uint32_t Lw[kSlotWords], Rw[kSlotWords], o[kSlotWords];
            const uint32_t* pl = slots + (leaf0 - L0) * kSlotWords;
            const uint32_t* pr = slots + (leaf0 + (1u << (L - 1)) - L0) * kSlotWords;
#pragma unroll
            for (int j = 0; j < kSlotWords; j++) {
                Lw[j] = pl[j];
                Rw[j] = pr[j];
            }
            if (pair) hash_node_u<true>(Lw, Rw, o, A);
            else hash_node_u<false>(Lw, Rw, o, false);
#pragma unroll
            for (int j = 0; j < kSlotWords; j++) o[j] = bswap32(o[j]);   // big-endian view
            if (h == L) {   // subtree root -> its RFC-6962 leaf digest
                uint32_t D[8];
                if (pair) rfc_leaf_u<true>(o, D, A);
                else rfc_leaf_u<false>(o, D, false);
                if (!A) {
#pragma unroll
                    for (int j = 0; j < 8; j++) dig[(lo - T0) * 8 + j] = D[j];
                }
            } else if (!A) {
                uint32_t* po = slots + (leaf0 - L0) * kSlotWords;
#pragma unroll
                for (int j = 0; j < kSlotWords; j++) po[j] = o[j];
            }
        };
        if (pair_ok && 2 * cnt <= 256) {
            if ((tid >> 1) < cnt) node(n_lo + (tid >> 1), true, tid & 1);
        } else {
            for (uint32_t i = tid; i < cnt; i += 256) node(n_lo + i, false, false);
        }
        __syncthreads();
    }
    uint32_t m = 0, base = 0;
    if (tid < G) {
        base = blob_tree0[b0 + tid] - T0;
        m = blob_tree0[b0 + tid + 1] - blob_tree0[b0 + tid];
        bbase[tid] = base;
    }
    __syncthreads();
    group_rfc_levels<256>(dig, G, m, base, b0, pre, bbase, &s_total, out, pair_ok != 0);
}

// RFC-6962 leaf digests of n 96-B slots.
__global__ __launch_bounds__(256) void slot_digest_kernel(const uint8_t* __restrict__ slots, uint32_t n,
                                                          uint32_t* __restrict__ dig) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    uint32_t I[kSlotWords];
    load_slot_be(slots + (size_t)t * kSlot, I);
    store_rfc_leaf(I, dig + (size_t)t * 8);
}

}  // namespace

hipError_t launch_slot_merkle_roots(const uint8_t* slots, const uint32_t* bt, uint32_t n_sets, uint32_t n_slots,
                                    uint32_t max_n, uint32_t* dig, uint8_t* out, hipStream_t s) {
    if (n_sets == 0) return hipSuccess;
    if (n_slots) {
        hipLaunchKernelGGL(slot_digest_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, s, slots, n_slots, dig);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint32_t mt = max_n ? max_n : 1;
    const size_t lds = (size_t)(mt + (mt + 1) / 2) * 32;
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(commitment_kernel, dim3(n_sets), dim3(64), lds, s, dig, bt, mt, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Engine glue
// ---------------------------------------------------------------------------
// CDA_COMMIT_GROUP=0: one wave per blob (commitment_kernel) instead of blob
// groups (A/B knob, read once).
static bool group_commitments() {
    static const bool on = [] {
        const char* e = test_knob("CDA_COMMIT_GROUP");
        return !(e && e[0] == '0');
    }();
    return on;
}
// CDA_COMMIT_FUSED=0: small-blob batches also take the level launches and
// commitment_group_kernel instead of commitment_fused_kernel (read per call).
static bool fuse_commitments() {
    const char* e = test_knob("CDA_COMMIT_FUSED");
    return !(e && e[0] == '0');
}

int Engine::enqueue_commitments(const square::CommitPlan& p, uint32_t n_blobs, const uint8_t* d_data, uint8_t* d_out,
                                hipStream_t s) {
    if (n_blobs == 0) return CDA_OK;
    const size_t seg_b = p.segs.size() * sizeof(square::Segment);
    const size_t st_b = p.seg_tree0.size() * 4;
    const size_t bt_b = p.blob_tree0.size() * 4;
    // Blob groups for commitment_group_kernel: consecutive blobs while the
    // group's first-level parents stay within ucap units -- 32 (one lane pair
    // each) for a small batch, enough for about one group per SIMD for a large
    // one -- and its subtree roots within tcap LDS slots.
    std::vector<uint32_t>& grp = cm_groups_;
    grp.clear();
    uint32_t max_gt = 0;
    // Small-blob batches take commitment_fused_kernel (subtree levels in LDS
    // too): groups of consecutive blobs whose leaf range (alignment gaps
    // included) stays within kFusedGroupLeaves -- a single blob up to
    // kFusedMaxShares -- sized for three workgroups per CU.
    constexpr uint32_t kFusedGroupLeaves = 384, kFusedMaxGroups = 256;
    uint32_t max_sh = 0;
    for (const auto& g : p.segs)
        if (g.kind == square::kSegBlob) max_sh = std::max(max_sh, g.n);
    bool fused = group_commitments() && fuse_commitments() && p.n_leaves && max_sh <= kFusedMaxShares;
    size_t fused_lds = 0;
    if (fused) {
        const uint32_t* bt = p.blob_tree0.data();
        size_t si = 0;
        uint32_t g0 = 0, gl0 = 0, gl1 = 0, gt = 0;
        auto close = [&]() {
            fused_lds = std::max(fused_lds, ((size_t)(gl1 - gl0) * kSlotWords + (size_t)gt * 8) * 4);
        };
        grp.push_back(0);
        for (uint32_t b = 0; b < n_blobs; b++) {
            const uint32_t nt = bt[b + 1] - bt[b];
            uint32_t s0 = 0, s1 = 0;
            if (nt) {   // the blob's segment: blobs with shares have one each, in order
                while (p.segs[si].kind != square::kSegBlob) si++;
                s0 = p.segs[si].start;
                s1 = s0 + p.segs[si].n;
                si++;
            }
            if (b > g0 && (b - g0 == 64 || (nt && gt && s1 - gl0 > kFusedGroupLeaves))) {
                close();
                grp.push_back(b);
                g0 = b;
                gl0 = gl1 = gt = 0;
            }
            if (nt) {
                if (!gt) gl0 = s0;
                gl1 = s1;
                gt += nt;
            }
        }
        grp.push_back(n_blobs);
        close();
        // a latency path: with more groups than CUs the level launches pack
        // the chip better (64 full blocks: 0.49 ms unfused, 0.67 fused)
        if (grp.size() - 1 > kFusedMaxGroups) {
            fused = false;
            grp.clear();
        }
    }
    if (!fused && group_commitments()) {
        const uint32_t* bt = p.blob_tree0.data();
        uint64_t units = 0;
        for (uint32_t b = 0; b < n_blobs; b++) units += (bt[b + 1] - bt[b]) / 2;
        // CDA_COMMIT_UCAP (read per call; tests): a larger minimum, to drive
        // the lane-per-unit passes with small batches
        const char* ue = test_knob("CDA_COMMIT_UCAP");
        const uint64_t umin = ue ? std::max(1L, std::atol(ue)) : 32;
        const uint32_t ucap = (uint32_t)std::max<uint64_t>(umin, (units + 1023) / 1024);
        const uint32_t tcap = std::max(p.max_trees, 512u);
        uint32_t g0 = 0, gu = 0, gt = 0;
        grp.push_back(0);
        for (uint32_t b = 0; b < n_blobs; b++) {
            const uint32_t nt = bt[b + 1] - bt[b];
            if (b > g0 && (b - g0 == 64 || gu + nt / 2 > ucap || gt + nt > tcap)) {
                grp.push_back(b);
                max_gt = std::max(max_gt, gt);
                g0 = b;
                gu = gt = 0;
            }
            gu += nt / 2;
            gt += nt;
        }
        grp.push_back(n_blobs);
        max_gt = std::max(max_gt, gt);
    }
    const size_t gr_b = grp.size() * 4;
    const size_t plan_b = seg_b + st_b + bt_b + gr_b;
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
    if (st_b) std::memcpy(stage + seg_b, p.seg_tree0.data(), st_b);
    std::memcpy(stage + seg_b + st_b, p.blob_tree0.data(), bt_b);
    if (gr_b) std::memcpy(stage + seg_b + st_b + bt_b, grp.data(), gr_b);
    if ((rc = check(cm_plan_.ensure(plan_b), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(cm_plan_.ptr, stage, plan_b, hipMemcpyHostToDevice, s), "H2D plan"))) return rc;
    if ((rc = check(hipEventRecord(sq_event_, s), "hipEventRecord"))) return rc;
    const square::Segment* d_segs = cm_plan_.as<square::Segment>();
    const uint32_t* d_st = reinterpret_cast<const uint32_t*>(cm_plan_.as<uint8_t>() + seg_b);
    const uint32_t* d_bt = reinterpret_cast<const uint32_t*>(cm_plan_.as<uint8_t>() + seg_b + st_b);
    const uint32_t* d_grp = reinterpret_cast<const uint32_t*>(cm_plan_.as<uint8_t>() + seg_b + st_b + bt_b);
    const uint32_t N = p.n_leaves, n_trees = p.n_trees;
    if (N) {
        if ((rc = check(cm_leaf_.ensure((size_t)N * kSlot), "hipMalloc"))) return rc;
        if ((rc = check(cm_lvl_.ensure((size_t)(N / 2 + 1) * kSlot), "hipMalloc"))) return rc;
        if ((rc = check(cm_roots_.ensure((size_t)n_trees * 32), "hipMalloc"))) return rc;   // RFC leaf digests
        if ((rc = check(cm_tables_.ensure((size_t)N * 4 + (size_t)n_trees * sizeof(Tree)), "hipMalloc"))) return rc;
        uint32_t* d_leaf_tree = cm_tables_.as<uint32_t>();
        Tree* d_trees = reinterpret_cast<Tree*>(d_leaf_tree + N);
        hipLaunchKernelGGL(blob_leaf_kernel, dim3((N + 255) / 256), dim3(256), 0, s, d_segs, (uint32_t)p.segs.size(),
                           d_st, d_trees, d_leaf_tree, d_data, cm_leaf_.as<uint8_t>(), N);
        if ((rc = check(hipGetLastError(), "blob leaves"))) return rc;
        if (fused) {
            if (fused_lds > 48 * 1024 &&
                (rc = check(hipFuncSetAttribute(reinterpret_cast<const void*>(commitment_fused_kernel),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)fused_lds),
                            "hipFuncSetAttribute")))
                return rc;
            // lane pairs cut a compression's latency but cost 1.6x its lane
            // work: kept for when the groups leave most of the chip idle
            const uint32_t n_groups = (uint32_t)grp.size() - 1, pair_ok = n_groups <= 512 ? 1u : 0u;
            hipLaunchKernelGGL(commitment_fused_kernel, dim3(n_groups), dim3(256), fused_lds, s, cm_leaf_.as<uint8_t>(),
                               d_trees, d_leaf_tree, d_bt, d_grp, d_out, pair_ok);
            return check(hipGetLastError(), "commitments");
        }
        if (p.max_height == 0) {   // else the level-1 launch hashes the height-0 subtrees too
            hipLaunchKernelGGL(leaf_roots_kernel, dim3((n_trees + 255) / 256), dim3(256), 0, s, d_trees, n_trees,
                               cm_leaf_.as<uint8_t>(), cm_roots_.as<uint32_t>());
            if ((rc = check(hipGetLastError(), "leaf roots"))) return rc;
        }
        for (uint32_t L = 1; L <= p.max_height; L++) {
            uint8_t* in = (L - 1) % 2 == 0 ? cm_leaf_.as<uint8_t>() : cm_lvl_.as<uint8_t>();
            uint8_t* out = L % 2 == 0 ? cm_leaf_.as<uint8_t>() : cm_lvl_.as<uint8_t>();
            const uint32_t n_nodes = (uint32_t)(((uint64_t)N + (1ull << L) - 1) >> L);
            const uint64_t threads = (uint64_t)n_nodes + (L == 1 ? n_trees : 0u);
            hipLaunchKernelGGL(subtree_level_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, d_trees,
                               n_trees, d_leaf_tree, in, out, cm_roots_.as<uint32_t>(), L, n_nodes);
            if ((rc = check(hipGetLastError(), "subtree level"))) return rc;
        }
    }
    if (!grp.empty()) {
        const size_t lds = (size_t)std::max(max_gt, 1u) * 32;
        if (lds > 159 * 1024) return fail(CDA_ERR_UNSUPPORTED, "too many subtree roots in one blob");
        if (lds > 64 * 1024 &&
            (rc = check(hipFuncSetAttribute(reinterpret_cast<const void*>(commitment_group_kernel),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        "hipFuncSetAttribute")))
            return rc;
        hipLaunchKernelGGL(commitment_group_kernel, dim3((uint32_t)grp.size() - 1), dim3(64), lds, s,
                           cm_roots_.as<uint32_t>(), d_bt, d_grp, d_out);
        return check(hipGetLastError(), "commitments");
    }
    const uint32_t mt = p.max_trees ? p.max_trees : 1;
    const size_t lds = (size_t)(mt + (mt + 1) / 2) * 32;
    if (lds > 160 * 1024) return fail(CDA_ERR_UNSUPPORTED, "too many subtree roots in one blob");
    if (lds > 64 * 1024 &&
        (rc = check(hipFuncSetAttribute(reinterpret_cast<const void*>(commitment_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                    "hipFuncSetAttribute")))
        return rc;
    hipLaunchKernelGGL(commitment_kernel, dim3(n_blobs), dim3(64), lds, s, cm_roots_.as<uint32_t>(), d_bt, mt, d_out);
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
