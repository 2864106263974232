// square_plan.h -- data-square construction (txs -> ODS layout), host side.
//
// Restates go-square v1.1.0 square.Construct / square.Build (EXT, pinned at
// /root/reference/go.mod:9; not vendored).  The builder and Export sequence is
// visible in the reference's malicious copy,
// test/util/malicious/out_of_order_builder.go:24-161 (Build, Construct, the
// Export body minus its blob swap); share formats follow
// specs/src/specs/shares.md and data_square_layout.md.  Call sites:
// app/prepare_proposal.go:50 (Build), app/process_proposal.go:122 and
// app/extend_block.go:16 (Construct).
//
// The layout is inherently serial (a cursor over blobs in namespace order), so
// it is planned on the host in O(#txs + #blobs).  The plan is a list of
// segments in square order; the share bytes themselves are written by the
// GPU share writer (square.hip) straight into the HBM-resident ODS that the
// extension kernels consume.  Compact (tx / PFB) shares are small and are
// produced here.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace cda {
namespace square {

constexpr uint32_t kShare = 512;
constexpr uint32_t kNs = 29;

enum SegKind : uint32_t {
    kSegCompact = 0,    // n shares copied from Plan::compact (tx then PFB compact shares)
    kSegPadding = 1,    // n padding shares: ns || info(version, start) || 0x00000000 || zeros
    kSegBlob = 2,       // n sparse shares of one blob
};

// One contiguous run of shares.  Device-visible (plain POD, 64 B).
struct Segment {
    uint32_t kind;
    uint32_t start;        // first share index in the square
    uint32_t n;            // share count
    uint32_t version;      // share version (info byte = version << 1 | sequence start)
    uint64_t src;          // kSegCompact: byte offset in the compact buffer; kSegBlob: byte offset of the blob data in the tx buffer
    uint32_t len;          // kSegBlob: blob data length (sequence length)
    uint8_t ns[kNs];       // namespace (kSegPadding / kSegBlob)
    uint8_t sub_log;       // CommitPlan kSegBlob: log2(subtree width)
    uint8_t pad_[6];
};
static_assert(sizeof(Segment) == 64, "Segment is 64 bytes");

struct Plan {
    uint32_t square_size = 0;          // k
    std::vector<Segment> segs;         // in square order, covering [0, k*k)
    std::vector<uint8_t> compact;      // compact shares (tx then PFB), 512 B each
    std::vector<uint32_t> kept;        // Build: indexes of the txs in the square (normal txs, then blob txs)
    std::vector<uint32_t> share_indexes;   // per PFB (square order) per blob: start share (IndexWrapper.share_indexes)
    std::vector<uint32_t> share_index_pfb; // PFB ordinal of each entry of share_indexes
    uint32_t n_blobs = 0;
    // builder.FindTxShareRange per kept tx (normal txs, then PFBs): shares
    // [unit_start, unit_end) of the square; equal units (same bytes, same
    // writer) all report the last one's range, as the go-square splitters key
    // their range maps by the tx hash (shares.CompactShareSplitter.ShareRanges)
    std::vector<uint32_t> unit_start, unit_end;
    uint32_t n_normal = 0;             // kept normal txs (units [0, n_normal) are in the tx namespace)
};

enum Mode { kConstruct = 0, kBuild = 1 };

// Share-writer hint granularity: hint[i] = segment holding share i * kHintShares.
constexpr uint32_t kHintShares = 16;

// Plans the square for n txs (tx i = txs[off[i], off[i+1])).  Returns 0, or -1
// with the go-square error text in *err.
int plan(const uint8_t* txs, const uint64_t* off, uint32_t n, uint32_t max_square_size, uint32_t threshold, Mode mode,
         Plan* out, std::string* err);

// ---- blob share commitments (go-square v1.1.0 inclusion.CreateCommitment) ----
// Every blob's sparse shares are laid out in one leaf array, each blob starting
// at a multiple of its subtree width w, so every Merkle-mountain-range subtree
// (sizes w, ..., then decreasing powers of two) is a perfect tree aligned to
// its size: level L of all subtrees of all blobs is then one pairwise pass.
struct Tree {
    uint32_t off;      // first leaf (multiple of 1 << height)
    uint32_t height;   // log2(size)
};
// The subtree list itself (n_trees Tree records, blob order then MMR order) is
// not built here: it follows from each blob segment's start, share count and
// sub_log, and the device writes it (commit.hip leaf_tables_kernel).
constexpr uint32_t kNoTree = 0xFFFFFFFFu;
struct CommitPlan {
    uint32_t n_leaves = 0;             // leaf array length (blobs + alignment gaps)
    uint32_t max_height = 0;
    uint32_t max_trees = 0;            // most subtree roots of one blob
    uint32_t n_trees = 0;              // all subtrees of all blobs
    std::vector<Segment> segs;         // share layout of the leaf array (blob segments + gaps)
    std::vector<uint32_t> seg_tree0;   // first tree of each segment's blob (kNoTree for gaps)
    std::vector<uint32_t> blob_tree0;  // first tree of blob i (n + 1 entries: prefix sums)
};
// Subtrees of a blob of n shares with width 1 << sub_log
// (inclusion.MerkleMountainRangeSizes): n >> sub_log of full width, then one per
// set bit of the remainder, largest first.
inline uint32_t mmr_tree_count(uint32_t n, uint32_t sub_log) {
    return (n >> sub_log) + (uint32_t)__builtin_popcount(n & ((1u << sub_log) - 1));
}
// namespaces: n * 29 bytes; data_off: n + 1 offsets into the blob data;
// share_versions: n bytes or NULL (all 0).  *out is reused: its vectors keep
// their capacity from call to call.
int plan_commitments(const uint8_t* namespaces, const uint64_t* data_off, const uint8_t* share_versions, uint32_t n,
                     uint32_t threshold, CommitPlan* out, std::string* err);

// Helpers shared with tests and other components (go-square inclusion / shares).
uint32_t round_up_pow2(uint32_t x);
uint32_t blob_min_square_size(uint32_t share_count);
uint32_t subtree_width(uint32_t share_count, uint32_t threshold);
uint32_t sparse_shares_needed(uint32_t len);

}  // namespace square
}  // namespace cda
