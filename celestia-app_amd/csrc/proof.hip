// proof.hip -- device-resident extended squares: NMT share-inclusion proofs
// and blob commitments from cached row-tree nodes.
//
// Reference: pkg/proof/proof.go:77-206 (NewShareInclusionProofFromEDS,
// CreateShareToRowRootProofs -> nmt ProveRange, merkle.ProofsFromByteSlices
// over rowRoots || colRoots) and pkg/inclusion/{nmt_caching.go,
// get_commit.go, paths.go} (EDSSubTreeRootCacher: every inner node of every
// row tree kept so GetCommitment can walk to the subtree roots).
//
// The reference re-hashes whole rows on the CPU for every proof.  Here the
// square is extended once and EVERYTHING the proofs read stays in HBM:
//   leaf slots      [W][W][96]            (level 0 of every row tree)
//   row levels      level L: [W][W >> L][96]
//   RFC levels      data-root tree over the 2W roots: level l: [2W >> l][32]
// A proof is then index arithmetic on the host (which nodes: nmt
// buildRangeProof's maximal subtrees outside the range, RFC aunts bottom-up)
// plus one gather launch and one copy back.
#include <algorithm>
#include <cstring>
#include <string>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

// All RFC-6962 levels of the data-root tree (n leaf digests, n a power of two)
// in one workgroup: level 0 = the leaf digests, level l has n >> l entries.
__global__ __launch_bounds__(1024) void rfc_levels_kernel(uint32_t* __restrict__ lv, uint32_t n,
                                                          uint8_t* __restrict__ root) {
    uint32_t* src = lv;
    for (uint32_t m = n / 2; m >= 1; m >>= 1) {
        uint32_t* dst = src + 2 * m * 8;
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
            uint32_t A[8], B[8], w[16];
#pragma unroll
            for (int j = 0; j < 8; j++) { A[j] = src[16 * i + j]; B[j] = src[16 * i + 8 + j]; }
            ShaState st;
            sha_init(st);
#pragma unroll
            for (int q = 0; q < 2; q++) {
#pragma unroll
                for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(A, B, 16 * q + j);
                sha_compress(st, w);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) dst[8 * i + j] = st.h[j];
        }
        __syncthreads();
        src = dst;
    }
    if (threadIdx.x < 8) reinterpret_cast<uint32_t*>(root)[threadIdx.x] = bswap32(src[threadIdx.x]);
}

// Copies of (src, len) pieces into one output buffer: one workgroup per piece.
struct Piece {
    const uint8_t* src;
    uint64_t dst;
    uint32_t len;
    uint32_t kind;   // 0 raw bytes, 1 digest words -> big-endian bytes (32 B)
};

__global__ __launch_bounds__(256) void gather_kernel(const Piece* __restrict__ pieces, uint8_t* __restrict__ out) {
    const Piece p = pieces[blockIdx.x];
    if (p.kind == 1) {
        if (threadIdx.x < 8)
            reinterpret_cast<uint32_t*>(out + p.dst)[threadIdx.x] =
                bswap32(reinterpret_cast<const uint32_t*>(p.src)[threadIdx.x]);
        return;
    }
    for (uint32_t i = threadIdx.x; i < p.len; i += blockDim.x) out[p.dst + i] = p.src[i];
}

}  // namespace

// ---------------------------------------------------------------------------
// ResidentSquare
// ---------------------------------------------------------------------------
ResidentSquare::~ResidentSquare() {
    for (DevBuf* b : {&eds, &levels, &col_a, &col_b, &roots_slots, &rfc, &rows, &cols, &root, &err, &scratch, &pieces})
        b->release();
}

uint64_t ResidentSquare::level_offset(uint32_t L) const {   // bytes into `levels`
    const uint64_t W = 2ull * k;
    uint64_t off = 0;
    for (uint32_t l = 0; l < L; l++) off += W * (W >> l) * kSlot;
    return off;
}

int Engine::square_create(const uint8_t* ods, uint32_t k, ResidentSquare* sq) {
    if (!is_pow2(k) || k > 1024) return fail(CDA_ERR_INVALID, "square width must be a power of two <= 1024");
    const uint32_t W = 2 * k;
    uint32_t logW = 0;
    while ((1u << logW) < W) logW++;
    sq->k = k;
    sq->log_w = logW;
    const size_t ods_b = (size_t)k * k * kShare, eds_b = (size_t)W * W * kShare;
    hipStream_t s = stream_;
    int rc;
    if ((rc = check(sq->eds.ensure(eds_b), "hipMalloc"))) return rc;
    if ((rc = check(sq->levels.ensure(sq->level_offset(logW + 1)), "hipMalloc"))) return rc;
    if ((rc = check(sq->col_a.ensure((size_t)W * W / 2 * kSlot), "hipMalloc"))) return rc;
    if ((rc = check(sq->col_b.ensure((size_t)W * W / 2 * kSlot), "hipMalloc"))) return rc;
    if ((rc = check(sq->roots_slots.ensure((size_t)2 * W * kSlot), "hipMalloc"))) return rc;
    if ((rc = check(sq->rfc.ensure((size_t)2 * (2 * W) * 32), "hipMalloc"))) return rc;
    if ((rc = check(sq->rows.ensure((size_t)W * kNode), "hipMalloc"))) return rc;
    if ((rc = check(sq->cols.ensure((size_t)W * kNode), "hipMalloc"))) return rc;
    if ((rc = check(sq->root.ensure(32), "hipMalloc"))) return rc;
    if ((rc = check(sq->err.ensure(4), "hipMalloc"))) return rc;
    if ((rc = check(h_ods_.ensure(ods_b), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(h_ods_.ptr, ods, ods_b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = enqueue_extend(h_ods_.as<uint8_t>(), k, 1, sq->eds.as<uint8_t>(), s))) return rc;
    if ((rc = check(hipMemsetAsync(sq->err.ptr, 0xFF, 4, s), "hipMemsetAsync"))) return rc;
    uint8_t* lv = sq->levels.as<uint8_t>();
    const CellGrid g{sq->eds.as<uint8_t>(), 0, W, W, W, 0, 0, k};
    if ((rc = check(launch_leaves(g, 1, lv, sq->err.as<uint32_t>(), true, true, s), "leaf hashing"))) return rc;
    // row forest: every level retained; column forest: ping-pong scratch
    Forest f[2]{};
    f[0] = Forest{lv, 0, W, W, 1, nullptr, 0, sq->rows.as<uint8_t>(), 0, sq->roots_slots.as<uint8_t>(), 0, 0};
    f[1] = Forest{lv, 0, W, 1, W, nullptr, 0, sq->cols.as<uint8_t>(), 0, sq->roots_slots.as<uint8_t>(), 0, W};
    uint8_t* colbuf[2] = {sq->col_a.as<uint8_t>(), sq->col_b.as<uint8_t>()};
    uint32_t L = 1;
    for (uint32_t m = W; m >= 2; m /= 2, L++) {
        f[0].out = lv + sq->level_offset(L);
        f[1].out = colbuf[L & 1];
        if ((rc = check(launch_level(f, 2, m, 1, s), "nmt level"))) return rc;
        for (int i = 0; i < 2; i++) {
            f[i].in = f[i].out;
            f[i].tree_stride = m / 2;
            f[i].node_stride = 1;
        }
    }
    // data root with every RFC-6962 level kept: leaf digests, then one workgroup
    if ((rc = check(launch_rfc_leaves(sq->roots_slots.as<uint8_t>(), 2 * W, sq->rfc.as<uint32_t>(), s), "rfc leaves")))
        return rc;
    hipLaunchKernelGGL(rfc_levels_kernel, dim3(1), dim3(1024), 0, s, sq->rfc.as<uint32_t>(), 2 * W,
                       sq->root.as<uint8_t>());
    if ((rc = check(hipGetLastError(), "rfc levels"))) return rc;
    uint32_t e = 0;
    if ((rc = check(hipMemcpyAsync(&e, sq->err.ptr, 4, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    sq->push_err = e;
    if (e != 0xFFFFFFFFu) return push_order_error(&e, 1, ods, k, false);
    return CDA_OK;
}

int Engine::square_read(ResidentSquare* sq, ResidentSquare::Part part, uint8_t* out) {
    const uint64_t W = 2ull * sq->k;
    const DevBuf* b = part == ResidentSquare::kRowRoots  ? &sq->rows
                      : part == ResidentSquare::kColRoots ? &sq->cols
                      : part == ResidentSquare::kDataRoot ? &sq->root
                                                          : &sq->eds;
    const size_t len = part == ResidentSquare::kDataRoot ? 32 : part == ResidentSquare::kEds ? W * W * kShare : W * kNode;
    int rc;
    if ((rc = check(hipMemcpyAsync(out, b->ptr, len, hipMemcpyDeviceToHost, stream_), "D2H"))) return rc;
    return check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

int Engine::square_gather(ResidentSquare* sq, const std::vector<GatherPiece>& pieces, uint8_t* out, size_t out_len) {
    int rc;
    if ((rc = square_gather_device(sq, pieces, out_len))) return rc;
    hipStream_t s = stream_;
    if ((rc = check(hipMemcpyAsync(out, sq->scratch.ptr, out_len, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

int Engine::square_gather_device(ResidentSquare* sq, const std::vector<GatherPiece>& pieces, size_t out_len) {
    hipStream_t s = stream_;
    int rc;
    if ((rc = check(sq->scratch.ensure(out_len ? out_len : 1), "hipMalloc"))) return rc;
    if (pieces.empty()) return CDA_OK;
    std::vector<Piece> P(pieces.size());
    for (size_t i = 0; i < pieces.size(); i++) {
        const GatherPiece& g = pieces[i];
        const DevBuf* b = g.buf == GatherPiece::kEds      ? &sq->eds
                          : g.buf == GatherPiece::kLevels ? &sq->levels
                          : g.buf == GatherPiece::kRfc    ? &sq->rfc
                          : g.buf == GatherPiece::kRows   ? &sq->rows
                                                          : &sq->roots_slots;
        P[i] = Piece{b->as<uint8_t>() + g.src, g.dst, g.len, g.buf == GatherPiece::kRfc ? 1u : 0u};
    }
    if ((rc = check(sq->pieces.ensure(P.size() * sizeof(Piece)), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(sq->pieces.ptr, P.data(), P.size() * sizeof(Piece), hipMemcpyHostToDevice, s),
                    "H2D pieces")))
        return rc;
    hipLaunchKernelGGL(gather_kernel, dim3((uint32_t)P.size()), dim3(256), 0, s, sq->pieces.as<Piece>(),
                       sq->scratch.as<uint8_t>());
    if ((rc = check(hipGetLastError(), "gather"))) return rc;
    // `P` is pageable: make sure the copy has left it before returning
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

// ---------------------------------------------------------------------------
// Share inclusion proof (pkg/proof/proof.go:77-206)
// ---------------------------------------------------------------------------
namespace {

// nmt buildRangeProof on a perfect tree of `width` leaves: the maximal
// subtrees outside [s, e), depth-first, left to right, as (level, index).
void range_proof_nodes(uint32_t lo, uint32_t hi, uint32_t s, uint32_t e, uint32_t level,
                       std::vector<std::pair<uint32_t, uint32_t>>& out) {
    if (hi <= s || lo >= e) {
        out.emplace_back(level, lo >> level);
        return;
    }
    if (hi - lo == 1) return;   // a leaf inside the range
    const uint32_t mid = (lo + hi) / 2;
    range_proof_nodes(lo, mid, s, e, level - 1, out);
    range_proof_nodes(mid, hi, s, e, level - 1, out);
}

uint32_t log2u(uint32_t x) {
    uint32_t l = 0;
    while ((1u << l) < x) l++;
    return l;
}

}  // namespace

int Engine::square_share_proof(ResidentSquare* sq, uint32_t start, uint32_t end, ShareProofOut* o) {
    const uint32_t k = sq->k, W = 2 * k, logW = sq->log_w;
    if (start >= end || end > k * k) return fail(CDA_ERR_INVALID, "share range out of the original square");
    const uint32_t startRow = start / k, endRow = (end - 1) / k;
    const uint32_t startLeaf = start % k, endLeaf = (end - 1) % k;
    const uint32_t nrows = endRow - startRow + 1, maxn = 2 * logW, naunts = log2u(2 * W);
    // staging layout: shares | nodes [nrows][maxn][90] | roots [nrows][90] | leaf hash [nrows][32] | aunts
    const size_t sh_b = (size_t)(end - start) * kShare;
    const size_t nd_off = sh_b, rt_off = nd_off + (size_t)nrows * maxn * kNode;
    const size_t lh_off = rt_off + (size_t)nrows * kNode, au_off = lh_off + (size_t)nrows * 32;
    const size_t total = au_off + (size_t)nrows * naunts * 32;
    std::vector<GatherPiece> pieces;
    size_t sh_at = 0;
    // RFC level offsets (entries) of the data-root tree over 2W items
    std::vector<uint64_t> rfc_off(naunts + 1, 0);
    for (uint32_t l = 0; l < naunts; l++) rfc_off[l + 1] = rfc_off[l] + ((2ull * W) >> l);
    for (uint32_t i = 0; i < nrows; i++) {
        const uint32_t r = startRow + i;
        const uint32_t s0 = i == 0 ? startLeaf : 0;
        const uint32_t e0 = (i == nrows - 1 ? endLeaf : k - 1) + 1;
        o->nmt_start[i] = (int32_t)s0;
        o->nmt_end[i] = (int32_t)e0;
        pieces.push_back(GatherPiece{GatherPiece::kEds, ((uint64_t)r * W + s0) * kShare, sh_at, (e0 - s0) * kShare});
        sh_at += (size_t)(e0 - s0) * kShare;
        std::vector<std::pair<uint32_t, uint32_t>> nodes;
        range_proof_nodes(0, W, s0, e0, logW, nodes);
        o->nmt_count[i] = (uint32_t)nodes.size();
        for (size_t q = 0; q < nodes.size(); q++) {
            const uint32_t L = nodes[q].first, p = nodes[q].second;
            const uint64_t src = sq->level_offset(L) + ((uint64_t)r * (W >> L) + p) * kSlot;
            pieces.push_back(GatherPiece{GatherPiece::kLevels, src, nd_off + ((size_t)i * maxn + q) * kNode, kNode});
        }
        pieces.push_back(GatherPiece{GatherPiece::kRows, (uint64_t)r * kNode, rt_off + (size_t)i * kNode, kNode});
        pieces.push_back(GatherPiece{GatherPiece::kRfc, (uint64_t)r * 32, lh_off + (size_t)i * 32, 32});
        uint32_t idx = r;   // merkle.ProofsFromByteSlices: aunts bottom-up
        for (uint32_t l = 0; l < naunts; l++, idx >>= 1)
            pieces.push_back(GatherPiece{GatherPiece::kRfc, (rfc_off[l] + (idx ^ 1)) * 32,
                                         au_off + ((size_t)i * naunts + l) * 32, 32});
    }
    std::vector<uint8_t> buf(total);
    int rc;
    if ((rc = square_gather(sq, pieces, buf.data(), total))) return rc;
    o->start_row = startRow;
    o->end_row = endRow;
    if (o->shares) std::memcpy(o->shares, buf.data(), sh_b);
    if (o->nmt_nodes) std::memcpy(o->nmt_nodes, buf.data() + nd_off, (size_t)nrows * maxn * kNode);
    if (o->row_roots) std::memcpy(o->row_roots, buf.data() + rt_off, (size_t)nrows * kNode);
    if (o->row_leaf_hash) std::memcpy(o->row_leaf_hash, buf.data() + lh_off, (size_t)nrows * 32);
    if (o->row_aunts) std::memcpy(o->row_aunts, buf.data() + au_off, (size_t)nrows * naunts * 32);
    return CDA_OK;
}

// ---------------------------------------------------------------------------
// EDSSubTreeRootCacher.getSubTreeRoot (pkg/inclusion/nmt_caching.go:111-124,
// walk :51-78): the node of row tree `row` reached from its root by `walk`
// (0 = WalkLeft, 1 = WalkRight).  The cache holds inner nodes only, so a walk
// may end on a leaf but not continue below one.
// ---------------------------------------------------------------------------
int Engine::square_subtree_root(ResidentSquare* sq, uint32_t row, const uint8_t* walk, uint32_t walk_len,
                                uint8_t* out) {
    const uint32_t W = 2 * sq->k, logW = sq->log_w;
    if (row >= W)
        return fail(CDA_ERR_INVALID,
                    "row exceeds range of cache: max " + std::to_string(W) + " got " + std::to_string(row));
    const uint32_t d = std::min(walk_len, logW);
    uint32_t pos = 0;
    for (uint32_t i = 0; i < d; i++) pos = 2 * pos + (walk[i] ? 1u : 0u);
    const uint32_t L = logW - d;
    // the levels below the root are kept per row tree; the root itself is the row root
    const GatherPiece piece = L == logW
                                  ? GatherPiece{GatherPiece::kRows, (uint64_t)row * kNode, 0, kNode}
                                  : GatherPiece{GatherPiece::kLevels,
                                                sq->level_offset(L) + ((uint64_t)row * (W >> L) + pos) * kSlot, 0, kNode};
    int rc;
    if ((rc = square_gather(sq, {piece}, out, kNode))) return rc;
    if (walk_len > logW) {   // walk(leaf, rest): the leaf is not in the cache -- Go's %v of its bytes
        std::string msg = "did not find sub tree root: [";
        for (uint32_t i = 0; i < kNode; i++) msg += (i ? " " : "") + std::to_string(out[i]);
        return fail(CDA_ERR_INVALID, msg + "]");
    }
    return CDA_OK;
}

// ---------------------------------------------------------------------------
// GetCommitment from the cached row trees (pkg/inclusion/get_commit.go,
// paths.go): subtree roots of the blob's rows, RFC-6962 over them.
// ---------------------------------------------------------------------------
namespace {

struct Coord {
    int depth, position;
};

// paths.go calculateSubTreeRootCoordinates (restated: climb from the leftmost
// leaf while the node is a left child above minDepth and its range fits).
std::vector<Coord> subtree_coords(int maxDepth, int minDepth, int start, int end) {
    std::vector<Coord> coords;
    int leafCursor = start;
    Coord node{maxDepth, start}, lastNode = node;
    int lastLeaf = leafCursor, range = 1;
    auto reset = [&]() {
        lastNode = node;
        lastLeaf = leafCursor;
        node = Coord{maxDepth, leafCursor};
        range = 1;
    };
    for (;;) {
        if (leafCursor + 1 == end) {
            coords.push_back(node);
            return coords;
        } else if (leafCursor + 1 > end) {
            coords.push_back(lastNode);
            leafCursor = lastLeaf + 1;
            reset();
        } else if (!(node.position % 2 == 0 && node.depth > minDepth)) {
            coords.push_back(node);
            leafCursor++;
            reset();
        } else {
            lastLeaf = leafCursor;
            lastNode = node;
            leafCursor += range;
            range *= 2;
            node = Coord{node.depth - 1, node.position / 2};
        }
    }
}

}  // namespace

int Engine::square_blob_commitments(ResidentSquare* sq, const uint32_t* starts, const uint32_t* lens, uint32_t n,
                                    uint32_t threshold, uint8_t* out) {
    if (n == 0) return CDA_OK;
    if (threshold == 0) return fail(CDA_ERR_INVALID, "subtree root threshold must be positive");
    const uint32_t k = sq->k, W = 2 * k;
    const int maxDepth = (int)log2u(k);
    std::vector<GatherPiece> pieces;
    std::vector<uint32_t> bt{0};
    uint32_t max_n = 0;
    for (uint32_t b = 0; b < n; b++) {
        const uint64_t len = lens[b];
        if (len == 0 || starts[b] + len > (uint64_t)k * k)
            return fail(CDA_ERR_INVALID, "cannot get commitment for blob that doesn't fit in square");
        const uint32_t w = square::subtree_width((uint32_t)len, threshold);
        const uint64_t start = (starts[b] + w - 1) / w * w;   // inclusion.NextShareIndex
        if (start + len > (uint64_t)k * k)
            return fail(CDA_ERR_INVALID, "cannot get commitment for blob that doesn't fit in square");
        const uint32_t startRow = (uint32_t)(start / k), endRow = (uint32_t)((start + len - 1) / k);
        const int nsi = (int)(start % k), nei = (int)(start + len - (uint64_t)endRow * k);
        const int minDepth = maxDepth - (int)log2u(w);
        uint32_t cnt = 0;
        for (uint32_t r = startRow; r <= endRow; r++) {
            const int s0 = r == startRow ? nsi : 0, e0 = r == endRow ? nei : (int)k;
            for (const Coord& c : subtree_coords(maxDepth, minDepth, s0, e0)) {
                // depth d of the ODS half of the row tree = level maxDepth - d of the full row tree
                const uint32_t L = (uint32_t)(maxDepth - c.depth);
                const uint64_t src = sq->level_offset(L) + ((uint64_t)r * (W >> L) + (uint32_t)c.position) * kSlot;
                pieces.push_back(GatherPiece{GatherPiece::kLevels, src, (uint64_t)pieces.size() * kSlot, kSlot});
                cnt++;
            }
        }
        bt.push_back(bt.back() + cnt);
        max_n = std::max(max_n, cnt);
    }
    const uint32_t n_slots = bt.back();
    int rc;
    if ((rc = square_gather_device(sq, pieces, (size_t)n_slots * kSlot))) return rc;
    hipStream_t s = stream_;
    if ((rc = check(cm_roots_.ensure((size_t)n_slots * 32 + 32), "hipMalloc"))) return rc;
    if ((rc = check(cm_plan_.ensure(bt.size() * 4), "hipMalloc"))) return rc;
    if ((rc = check(cm_out_.ensure((size_t)n * 32), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(cm_plan_.ptr, bt.data(), bt.size() * 4, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = check(launch_slot_merkle_roots(sq->scratch.as<uint8_t>(), cm_plan_.as<uint32_t>(), n, n_slots, max_n,
                                             cm_roots_.as<uint32_t>(), cm_out_.as<uint8_t>(), s),
                    "commitment roots")))
        return rc;
    if ((rc = check(hipMemcpyAsync(out, cm_out_.ptr, (size_t)n * 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace cda
