// nmt.hip -- namespaced Merkle roots of every EDS row/column and the data root.
//
// Reference behaviour (paths under /root/reference):
//   * rsmt2d computeRoots (EXT v0.14.0), called from
//     pkg/da/data_availability_header.go:45,49: one tree per row and column,
//     W = 2k leaves pushed in order.
//   * pkg/wrapper/nmt_wrapper.go:93-140: leaf namespace = share[0:29] in Q0,
//     ParitySharesNamespace (0xFF*29) elsewhere; :97-99 short-data error.
//   * nmt v0.22.0 (EXT; hasher rules copied in-tree at
//     test/util/malicious/hasher.go:186-310): HashLeaf, HashNode,
//     computeNsRange with IgnoreMaxNamespace(true); Push rejects a namespace
//     smaller than the previous one (ErrInvalidPushOrder).
//   * pkg/da/data_availability_header.go:92-108 -> go-square/merkle
//     HashFromByteSlices (RFC-6962) over rowRoots || colRoots.
//
// MI355X mapping.  The quadrant test is symmetric in (row, col), so a cell's
// leaf node is identical in its row tree and its column tree: it is hashed
// once (4k^2 leaf hashes instead of the reference's 8k^2).  One thread per
// leaf / per parent node; each NMT level of all 4k trees of every square in
// the batch is one launch.  SHA-256 is pure 32-bit VALU work (no MFMA).
#include "knobs.h"
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "cda_kernels.h"
#include "sha256_dev.h"
#include "leaf_dev.h"

namespace cda {

namespace {

constexpr size_t SH = 512;

// Tuning knobs (override with -D).  Measured on MI355X (profiles/r01_sha_sweep.txt):
// the SHA kernels are VALU-issue-bound; 3-5 waves/SIMD run within 1 %, more
// waves (forced spills or no prefetch) and non-temporal loads are slower.
#ifndef CDA_LEAF_WAVES
#define CDA_LEAF_WAVES 4
#endif
#ifndef CDA_LEVEL_WAVES
#define CDA_LEVEL_WAVES 4
#endif

__device__ __forceinline__ void load_chunk(const uint4* p, uint32_t (&w)[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 v = p[q];
        w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
__device__ __forceinline__ void bswap16(uint32_t (&w)[16]) {
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = bswap32(w[i]);
}

// Row-only push-order check over a grid of Q0 cells (config 5: the rank that
// owns a block of ODS rows checks them whole).
__global__ __launch_bounds__(256) void row_order_kernel(const CellGrid g, uint32_t* __restrict__ err) {
    const uint32_t cell = blockIdx.x * 256 + threadIdx.x;
    if (cell >= g.rows * g.cols) return;
    const uint32_t r = cell / g.cols, c = cell % g.cols;
    const uint32_t gr = g.row0 + r, gc = g.col0 + c;
    if (gr >= g.k || gc + 1 >= g.k || c + 1 >= g.cols) return;
    const uint8_t* E = g.base + blockIdx.y * g.sq;
    uint32_t me[8], nb[8];
    load_ns_be(E + ((size_t)r * g.row_stride + c) * SH, me);
    load_ns_be(E + ((size_t)r * g.row_stride + c + 1) * SH, nb);
    if (ns_less(nb, me)) atomicMin(err + blockIdx.y, (0u << 24) | (gr << 12) | (gc + 1));
}

// One virtual block (bx = 256-cell group, by = square) of the leaf launch:
// one cell per thread (leaf_dev.h leaf_cell).
__device__ __forceinline__ void leaf_block(const CellGrid& g, uint8_t* __restrict__ slots, uint32_t* __restrict__ err,
                                           int check_rows, int check_cols, uint32_t bx, uint32_t by,
                                           uint32_t (*ns_lds)[8]) {
    const uint32_t cell = bx * 256 + threadIdx.x;
    if (cell >= g.rows * g.cols) return;
    leaf_cell(g, slots, err, check_rows, check_cols, by, cell / g.cols, cell % g.cols, ns_lds[threadIdx.x]);
}

// Lane-pair leaves (round 5), for leaf launches of at most half a wave per
// SIMD of cells (k <= 64 squares): two lanes per cell run one instruction
// stream (sha_pair_compress: 1 040 instead of ~1 430 instructions per
// compression on the chain), so twice the SIMDs hold a wave.  One k = 64
// square 0.155 -> 0.150 ms (leaves 31 -> 28 us); at one k = 128 square (one
// wave per SIMD either way) the two pair waves per SIMD share its issue and
// the leaves take 34 -> 42 us, so 65 536-cell launches stay one lane per
// cell (profiles/r05/leaf_pair_ab.txt).  Both
// lanes of a pair load the same bytes and build the same message words; the
// e-side lane stores the slot and runs the push-order check.  No parity
// mid-state (block 0 of a parity leaf runs all 64 rounds).  128 cells per
// 256-thread workgroup.
__global__ __launch_bounds__(256) void leaf_pair_kernel(const CellGrid g, uint8_t* __restrict__ slots,
                                                        uint32_t* __restrict__ err, int check_rows, int check_cols,
                                                        uint32_t nbx) {
    const uint32_t bx = blockIdx.x % nbx, by = blockIdx.x / nbx;
    const uint32_t cell = bx * 128 + (threadIdx.x >> 1);
    if (cell >= g.rows * g.cols) return;   // both lanes of a pair leave together
    const bool A = threadIdx.x & 1;
    const size_t sq = by;
    const uint32_t r = cell / g.cols, c = cell % g.cols;
    const uint32_t gr = g.row0 + r, gc = g.col0 + c, k = g.k;
    const bool parity = !(gr < k && gc < k);
    const uint8_t* cellp = g.base + sq * g.sq + ((size_t)r * g.row_stride + c) * SH;
    const uint4* src = reinterpret_cast<const uint4*>(cellp);

    Sha<true> h;
    h.init(A);
    uint32_t cur[16], tail[8], w[16], nsw[8];
    load_raw16(src, cur);
    if (parity) {
#pragma unroll
        for (int i = 0; i < 8; i++) nsw[i] = 0xFFFFFFFFu;
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) nsw[i] = bswap32(cur[i]);
        nsw[7] &= 0xFF000000u;
        if (!A) leaf_order_check(g, cellp, nsw, err + sq, check_rows, check_cols, r, c, gr, gc);
    }
    uint32_t nxt[16];
    load_raw16(src + 4, nxt);
#pragma unroll
    for (int i = 8; i < 16; i++) w[i] = body_word(cur[i - 8], cur[i - 7]);
    if (parity) {
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = kLeafParityHead[i];
        w[7] = __builtin_amdgcn_perm(cur[0], cur[0], 0x0D0D0001u);
    } else {
        w[0] = __builtin_amdgcn_perm(cur[0], cur[0], 0x0C000102u);
#pragma unroll
        for (int i = 1; i < 7; i++) w[i] = __builtin_amdgcn_perm(cur[i], cur[i - 1], 0x03040506u);
        w[7] = __builtin_amdgcn_perm(cur[7], cur[6], 0x03040C0Cu) | __builtin_amdgcn_perm(cur[0], cur[0], 0x0C0C0001u);
    }
    h.compress(w, A);
#pragma unroll
    for (int i = 0; i < 8; i++) tail[i] = cur[8 + i];
#pragma unroll 1
    for (int b = 1; b < 8; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) cur[i] = nxt[i];
        if (b < 7) load_raw16(src + 4 * (b + 1), nxt);
#pragma unroll
        for (int t = 0; t < 7; t++) w[t] = body_word(tail[t], tail[t + 1]);
        w[7] = body_word(tail[7], cur[0]);
#pragma unroll
        for (int t = 8; t < 16; t++) w[t] = body_word(cur[t - 8], cur[t - 7]);
#pragma unroll
        for (int i = 0; i < 8; i++) tail[i] = cur[8 + i];
        h.compress(w, A);
    }
#pragma unroll
    for (int t = 0; t < 7; t++) w[t] = body_word(tail[t], tail[t + 1]);
    w[7] = __builtin_amdgcn_perm(tail[7], tail[7], 0x02030C0Cu) | 0x8000u;
#pragma unroll
    for (int t = 8; t < 15; t++) w[t] = 0;
    w[15] = kLeafMsgBits;
    h.compress(w, A);
    uint32_t D[8], out[kSlotWords];
    h.digest(A, D);
    leaf_node_words(nsw, D, out);
    if (!A) store_slot(slots + (sq * (size_t)g.rows * g.cols + cell) * kSlot, out);
}

// The hash launches run a 1-D grid over virtual blocks b = by * nbx + bx: one
// block per workgroup when the grid covers them all, or a capped persistent
// grid (CDA_HASH_WG_PER_CU workgroups per CU) whose workgroups stride over
// them -- then the hash kernels hold a fixed share of every CU and leave room
// for the batch pipeline's RS workgroups (engine.hip enqueue_extend_dah).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CDA_LEAF_WAVES))) void leaf_kernel(
    const CellGrid g, uint8_t* __restrict__ slots, uint32_t* __restrict__ err, int check_rows, int check_cols,
    uint32_t nbx, uint32_t nblocks) {
    __shared__ __attribute__((aligned(16))) uint32_t ns_lds[256][8];
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
        leaf_block(g, slots, err, check_rows, check_cols, b % nbx, b / nbx, ns_lds);
}

// ---------------------------------------------------------------------------
// One NMT level of up to two forests (blockIdx.z).  Thread -> (tree, parent):
// parents of one tree are adjacent threads when nodes are adjacent slots
// (node_stride == 1), otherwise adjacent threads take the same parent of
// adjacent trees (tree_stride == 1, e.g. column trees over a row-major grid),
// so slot loads stay coalesced either way.
// ---------------------------------------------------------------------------
struct Forest2 {
    Forest f[2];
};

// HashNode of two big-endian child slots -> parent slot (little-endian words,
// as stored).  Block 0 = 0x01 || L[0:63]: a parity left child makes words
// 0..13 constant, so those nodes start from the precomputed mid-state (MID).
// The branch is worth it only where a wave's parents are all of one kind
// (level_kernel orders them so); otherwise both paths run (MID = false).
template <bool MID = true>
__device__ __forceinline__ void hash_node(const uint32_t (&L)[kSlotWords], const uint32_t (&R)[kSlotWords],
                                          uint32_t (&o)[kSlotWords]) {
    uint32_t w[16];
    ShaState st;
    sha_init(st);
    // (Writing the parity branch's constant 0xFF words of blocks 1-2 as
    // literals saves ~1.5% of its rotations but duplicates blocks 1-2 per
    // branch: ~8.2k instead of ~5.5k instructions, past the instruction cache
    // a CU pair shares -- not taken.)
    if (MID && is_parity_min(L)) {
        w[14] = node_msg(L, R, 14);
        w[15] = node_msg(L, R, 15);
        sha_compress_from<kNodeParityRounds>(st, kNodeParityMid, kNodeParityHead, w);
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, i);
        sha_compress(st, w);
    }
#pragma unroll
    for (int b = 1; b < 3; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 16 * b + i);
        sha_compress(st, w);
    }
    inner_node_words(L, R, st.h, o);
}

// One virtual block (bx = 256-parent group, by = square, bz = forest).
__device__ __forceinline__ void level_block(const Forest2& fs, uint32_t n_in, uint32_t bx, uint32_t by, uint32_t bz) {
    const Forest& F = fs.f[bz];
    const uint32_t n_out = n_in / 2;
    const uint32_t idx = bx * 256 + threadIdx.x;
    if (idx >= F.n_trees * n_out) return;
    const size_t sq = by;
    uint32_t t, p;
    if (F.node_stride == 1) {
        // all trees' left-half parents first, then the right halves: a wave
        // then never mixes parents with a data and a parity left child (the
        // mid-state branch below stays uniform); runs of n_out/2 parents of
        // one tree remain adjacent, so slot loads stay coalesced
        if (n_out >= 2) {
            const uint32_t hn = n_out / 2, per = F.n_trees * hn;
            const uint32_t h = idx / per, r = idx % per;
            t = r / hn; p = h * hn + r % hn;
        } else {
            t = idx; p = 0;
        }
    } else {
        p = idx / F.n_trees; t = idx % F.n_trees;
    }
    const uint8_t* base = F.in + sq * F.in_sq;
    const uint8_t* l = base + ((size_t)t * F.tree_stride + (size_t)(2 * p) * F.node_stride) * kSlot;
    const uint8_t* rr = l + (size_t)F.node_stride * kSlot;
    uint32_t L[kSlotWords], R[kSlotWords];
    load_slot_be(l, L);
    load_slot_be(rr, R);
    uint32_t o[kSlotWords];
    hash_node(L, R, o);
    if (n_out == 1) {
        if (F.roots) {
            uint16_t* d16 = reinterpret_cast<uint16_t*>(F.roots + sq * F.roots_sq + (size_t)t * kNode);
#pragma unroll
            for (int i = 0; i < kNode / 2; i++) d16[i] = (uint16_t)(o[i / 2] >> (16 * (i & 1)));
        }
        if (F.root_slots) store_slot(F.root_slots + sq * F.rslot_sq + (size_t)(F.root0 + t) * kSlot, o);
    } else {
        store_slot(F.out + sq * F.out_sq + ((size_t)t * n_out + p) * kSlot, o);
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CDA_LEVEL_WAVES))) void level_kernel(
    const Forest2 fs, uint32_t n_in, uint32_t nbx, uint32_t nsq, uint32_t nblocks) {
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const uint32_t bx = b % nbx, r = b / nbx;
        level_block(fs, n_in, bx, r % nsq, r / nsq);
    }
}

// ---------------------------------------------------------------------------
// Fused subtree levels (latency-shaped jobs: k = 256 / 512 squares, a few per
// call).  Where a job's levels drop from many waves per SIMD to one within a
// few launches (k = 512, one square: 16, 8, 4, 2, 1), the per-level launches
// pay a drain tail and a boundary each, and the last ones run below one wave
// per SIMD.  Here ONE lane takes a whole S-leaf subtree of one tree and hashes
// its S - 1 nodes in post order -- one node per loop iteration, the same
// instruction stream for every lane, so the loop is uniform -- and the job
// holds >= 1 wave per SIMD (the host picks S = n_in / top with top from
// top_fuse_nodes, so lanes = n * 2W * top >= 65 536).  A lone wave issues an
// instruction every ~4.25 cycles, about the rate of a SIMD saturated with the
// same mixed stream, so these chains run at the wide
// launches' compression rate without their tails.  Each iteration loads its
// operands (a leaf pair, or a stored left sibling) at use: 141 VGPRs, three
// waves per SIMD, whose loads hide behind each other's hashing -- against
// round 3's first form, which loaded them one iteration ahead as raw words
// (189 VGPRs, two waves per SIMD; tools/probes/subtree_prefetch.patch): config 4's
// levels 14.06 -> 13.90 ms, one k = 512 square unchanged (profiles/r03ar/).
// Pending left siblings go to a per-lane stack in the forest's output buffer
// behind the subtree roots (written and read by the same lane).  A wave is
// 64 consecutive trees of one subtree index, so the parity mid-state branch
// of hash_node stays uniform.
// ---------------------------------------------------------------------------
// (Register-sized for 4 waves per SIMD -- 128 VGPRs, a few spills -- where a
// launch holds between 3 and 4 waves per SIMD, e.g. config 4's 128-square
// shard: 2 % slower in an interleaved A/B, profiles/r04/
// r04o_fused_root_wide_subtree4_ab.txt; tools/probes/top_root_fused_subtree4.patch.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void subtree_kernel(
    const Forest2 fs, uint32_t n_in, uint32_t slog, uint32_t nbx, uint32_t nsq, uint32_t nblocks) {
    const uint32_t S = 1u << slog;
    const uint32_t top = n_in >> slog;   // subtree roots per tree
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const uint32_t bx = b % nbx, r = b / nbx;
        const size_t sq = r % nsq;
        const Forest& F = fs.f[r / nsq];
        const uint32_t lanes = F.n_trees * top;
        const uint32_t idx = bx * 256 + threadIdx.x;
        if (idx >= lanes) continue;
        const uint32_t t = idx % F.n_trees, s = idx / F.n_trees;
        const uint8_t* in = F.in + sq * F.in_sq + ((size_t)t * F.tree_stride + (size_t)s * S * F.node_stride) * kSlot;
        const size_t leaf_step = (size_t)F.node_stride * kSlot;
        uint8_t* out = F.out + sq * F.out_sq;
        // pending left sibling at level l (1 .. slog-1): one slot per lane and
        // level behind the `lanes` subtree-root slots
        auto stack_slot = [&](uint32_t l) -> uint8_t* {
            return out + ((size_t)lanes + (size_t)(l - 1) * lanes + idx) * kSlot;
        };
        uint32_t cur[kSlotWords];
        auto load_raw = [](const uint8_t* p, uint4 (&q)[6]) {
            const uint4* v = reinterpret_cast<const uint4*>(p);
#pragma unroll
            for (int i = 0; i < 6; i++) q[i] = v[i];
        };
        auto be = [](const uint4 (&q)[6], uint32_t (&w)[kSlotWords]) {
#pragma unroll
            for (int i = 0; i < 6; i++) {
                w[4 * i] = bswap32(q[i].x); w[4 * i + 1] = bswap32(q[i].y);
                w[4 * i + 2] = bswap32(q[i].z); w[4 * i + 3] = bswap32(q[i].w);
            }
        };
        uint32_t j = 0, lvl = 0, pos = 0;   // next leaf pair; level / index of cur
#pragma unroll 1
        for (uint32_t it = 0; it + 1 < S; it++) {
            const bool merge = it > 0 && (pos & 1);
            const uint8_t* pa = merge ? stack_slot(lvl) : in + (size_t)(2 * j) * leaf_step;
            const uint8_t* pb = merge ? pa : in + (size_t)(2 * j + 1) * leaf_step;
            uint4 a[6], b[6];
            load_raw(pa, a);
            load_raw(pb, b);
            uint32_t L[kSlotWords], R[kSlotWords];
            be(a, L);
            be(b, R);
            if (merge) {
#pragma unroll
                for (int i = 0; i < kSlotWords; i++) R[i] = bswap32(cur[i]);
            }
            const uint32_t nlvl = merge ? lvl + 1 : 1u, npos = merge ? pos >> 1 : j;
            if (!merge) j++;
            hash_node(L, R, cur);
            if (!(npos & 1) && nlvl < slog) store_slot(stack_slot(nlvl), cur);
            lvl = nlvl;
            pos = npos;
        }
        if (top == 1) {   // whole trees: the roots, as level_kernel's last level writes them
            if (F.roots) {
                uint16_t* d16 = reinterpret_cast<uint16_t*>(F.roots + sq * F.roots_sq + (size_t)t * kNode);
#pragma unroll
                for (int i = 0; i < kNode / 2; i++) d16[i] = (uint16_t)(cur[i / 2] >> (16 * (i & 1)));
            }
            if (F.root_slots) store_slot(F.root_slots + sq * F.rslot_sq + (size_t)(F.root0 + t) * kSlot, cur);
        } else {
            store_slot(out + ((size_t)t * top + s) * kSlot, cur);
        }
    }
}

// Data root from n leaf digests (rfc_leaf_kernel, or the group digests of
// tree_top_kernel): one workgroup per square; the first inner level reads
// global memory, later levels ping-pong in LDS.  A level of m <= 128 parents
// (at most a wave per SIMD of lane pairs) runs a lane pair per parent, wider
// levels a thread per parent.
template <bool PAIR>
__device__ __forceinline__ void data_root_level(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                uint32_t m) {
    const uint32_t step = PAIR ? blockDim.x / 2 : blockDim.x;
    const bool A = PAIR && (threadIdx.x & 1);
    for (uint32_t i = PAIR ? threadIdx.x / 2 : threadIdx.x; i < m; i += step) {
        uint32_t a[8], b[8], D[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a[j] = in[(2 * i) * 8 + j];
            b[j] = in[(2 * i + 1) * 8 + j];
        }
        rfc_inner_u<PAIR>(a, b, D, A);
        if (!A) {
#pragma unroll
            for (int j = 0; j < 8; j++) out[i * 8 + j] = D[j];
        }
    }
}

// Largest data-root level run on lane pairs: 128 parents (256 lanes, a wave
// per SIMD), or 256 in launches of few squares (kPairMaxParentsSmall, 512
// lanes: a k = 512 square's first level; data root 0.055 -> 0.049 ms,
// profiles/r05/data_root_pairs_ab.txt -- at config 4's 1 024 squares the
// 512-thread launch made the stage 0.143 -> 0.209 ms, so not there).
constexpr uint32_t kPairMaxParents = 128;
constexpr uint32_t kPairMaxParentsSmall = 256;
constexpr uint32_t kPairSmallSquares = 8;   // launches of <= this many squares

// 16 rounds [R0, R0 + 16) of a lane-pair compression over precomputed
// K + W words (v: the pair's 4 state words, as in sha_pair_compress).
template <int R0>
__device__ __forceinline__ void pair_rounds16(uint32_t (&v)[4], const uint32_t (&kw)[16], bool A) {
    const uint32_t r1 = A ? 2u : 6u, r2 = A ? 13u : 11u, r3 = A ? 22u : 25u;
    const uint32_t mA = pair_mask();
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t S = xor3(__builtin_amdgcn_alignbit(v[0], v[0], r1), __builtin_amdgcn_alignbit(v[0], v[0], r2),
                                __builtin_amdgcn_alignbit(v[0], v[0], r3));
        const uint32_t F = pair_chmaj(v[0], v[1], v[2], mA);
        const uint32_t Y = pair_sel(v[3] + kw[i], 0u);
        const uint32_t T = add3(S, F, Y);
        const uint32_t nv = pair_add(T, pair_sel(T, v[3]));
        v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = nv;
    }
}

// Schedule words [T0, T0 + 16) (T0 >= 16) of one block into kw[T0 .. T0+16)
// as K + W (w: the 16-word ring, updated in place).
template <int T0>
__device__ __forceinline__ void schedule16_kw(uint32_t (&w)[16], uint32_t* kw) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    uint4* q = reinterpret_cast<uint4*>(kw + T0);
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        uint32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int t = T0 + i + r;
            const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            const uint32_t wi = add3(w[t & 15], s0, w[(t - 7) & 15]) + s1;
            w[t & 15] = wi;
            v[r] = K[t] + wi;
        }
        q[i / 4] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// One data-root level of m <= 32 parents with schedule helpers: wave 0 holds
// the parents' lane pairs, and one lane of waves 1.. per parent computes the
// message schedule of its block 0 (16 words at a time, through LDS, one
// barrier per 16 rounds) while the pair runs the rounds; block 1 comes from
// kRfcPad.  The pair's chain then carries no schedule work at all (DESIGN.md
// 3.5: the chain costs its wave's instruction count).  Every thread of the
// workgroup must call this (it holds barriers).
constexpr uint32_t kDrKwRow = 68;   // 64 words + 4 of padding (bank spread)
__device__ __forceinline__ void data_root_level_helped(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint32_t m, uint32_t (*kwb)[kDrKwRow]) {
    constexpr uint32_t K[64] = CDA_SHA_K;
    const bool A = threadIdx.x & 1;
    const uint32_t i = threadIdx.x / 2, hi = threadIdx.x - 64;
    const bool rounds = threadIdx.x < 64 && i < m;
    const bool helper = threadIdx.x >= 64 && hi < m;
    const uint32_t p = rounds ? i : hi;
    uint32_t a[8], b[8], w[16];
    if (rounds || helper) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a[j] = in[(2 * p) * 8 + j];
            b[j] = in[(2 * p + 1) * 8 + j];
        }
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(a, b, j);
    }
    ShaPair st;
    sha_pair_init(st, A);
    uint32_t v[4] = {st.h[0], st.h[1], st.h[2], st.h[3]};
    uint32_t kw[16];
    // block 1's K + W row (kRfcPad), streamed 16 words at a time
    const uint4* row = reinterpret_cast<const uint4*>(kRfcPad.kw[(rounds ? b[7] : 0u) & 0xFFu]);
    uint4 nx[4];
    if (rounds) {
#pragma unroll
        for (int t = 0; t < 16; t++) kw[t] = K[t] + w[t];
        pair_rounds16<0>(v, kw, A);
    } else if (helper) {
        schedule16_kw<16>(w, kwb[hi]);
    }
    __syncthreads();
    auto phase = [&](auto R0c) {
        constexpr int R0 = decltype(R0c)::value;
        if (rounds) {
            const uint4* q = reinterpret_cast<const uint4*>(&kwb[i][R0]);
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint4 x = q[c];
                kw[4 * c] = x.x; kw[4 * c + 1] = x.y; kw[4 * c + 2] = x.z; kw[4 * c + 3] = x.w;
            }
            pair_rounds16<R0>(v, kw, A);
        } else if (helper && R0 + 16 < 64) {
            schedule16_kw<(R0 + 16 < 64 ? R0 + 16 : 48)>(w, kwb[hi]);
        }
    };
    phase(std::integral_constant<int, 16>{});
    __syncthreads();
    phase(std::integral_constant<int, 32>{});
    __syncthreads();
    if (rounds) {
#pragma unroll
        for (int c = 0; c < 4; c++) nx[c] = row[c];   // in flight during rounds 48..63
    }
    phase(std::integral_constant<int, 48>{});
    if (rounds) {
        st.h[0] += v[0]; st.h[1] += v[1]; st.h[2] += v[2]; st.h[3] += v[3];
        v[0] = st.h[0]; v[1] = st.h[1]; v[2] = st.h[2]; v[3] = st.h[3];
        auto block1 = [&](auto Cc) {
            constexpr int C = decltype(Cc)::value;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                kw[4 * c] = nx[c].x; kw[4 * c + 1] = nx[c].y; kw[4 * c + 2] = nx[c].z; kw[4 * c + 3] = nx[c].w;
            }
            if constexpr (C < 3) {
#pragma unroll
                for (int c = 0; c < 4; c++) nx[c] = row[4 * (C + 1) + c];
            }
            pair_rounds16<16 * C>(v, kw, A);
        };
        block1(std::integral_constant<int, 0>{});
        block1(std::integral_constant<int, 1>{});
        block1(std::integral_constant<int, 2>{});
        block1(std::integral_constant<int, 3>{});
        st.h[0] += v[0]; st.h[1] += v[1]; st.h[2] += v[2]; st.h[3] += v[3];
        uint32_t D[8];
        sha_pair_digest(st, A, D);
        if (!A) {
#pragma unroll
            for (int j = 0; j < 8; j++) out[i * 8 + j] = D[j];
        }
    }
}

// The data root's inner levels over the n digests at D (global memory, or
// LDS in the fused tree top): the first level writes src, later levels
// ping-pong src / dst (LDS, room for n/2 and n/4 digests; dst may be D's LDS
// once the first level has read it).  A level of m <= 128 parents (at most a
// wave per SIMD of lane pairs) runs a lane pair per parent, wider levels a
// thread per parent; pair_ok == 2: schedule helpers in levels of <= 32
// parents.  Thread 0 writes the square's data root and its push-order status
// (status_kernel, fused: one launch less).  Every thread of the workgroup
// calls this (barriers).
__device__ __forceinline__ void data_root_levels(const uint32_t* D, uint32_t n, uint32_t* src, uint32_t* dst,
                                                 uint32_t (*kwb)[kDrKwRow], uint32_t pair_ok, uint8_t* data_root,
                                                 const uint32_t* err, int32_t* status) {
    for (uint32_t m = n / 2; m >= 1; m >>= 1) {
        const uint32_t* in = m == n / 2 ? D : src;
        uint32_t* out = m == n / 2 ? src : dst;
        if ((pair_ok & 0xFF) == 2 && m <= 32 && blockDim.x >= 128)
            data_root_level_helped(in, out, m, kwb);
        else if ((pair_ok & 0xFF) && m <= (pair_ok >> 8 ? pair_ok >> 8 : kPairMaxParents) && 2 * m <= blockDim.x)
            data_root_level<true>(in, out, m);
        else
            data_root_level<false>(in, out, m);
        __syncthreads();
        if (m != n / 2) {
            uint32_t* t = src;
            src = dst;
            dst = t;
        }
    }
    if (threadIdx.x == 0) {
        uint32_t* o = reinterpret_cast<uint32_t*>(data_root);
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = bswap32(src[j]);
        if (status) *status = *err == 0xFFFFFFFFu ? 0 : -3;   // CDA_OK / CDA_ERR_PUSH_ORDER
    }
}

// ---------------------------------------------------------------------------
// Fused top of the trees (latency-bound part: fewer parents than the chip has
// wave slots).  One workgroup takes tpw trees and runs every remaining level
// in LDS, no launch per level: the first level reads the trees' input slots
// from global memory, later levels ping-pong between two LDS halves.  The
// root goes out packed (90 B) and as a 96-B slot like level_kernel's.  If
// dig is set, the workgroup also starts the data root: the RFC-6962 leaf
// digests of its tpw roots (consecutive items of rowRoots || colRoots) and
// `rfc_levels` inner levels over them, one digest per 2^rfc_levels roots to
// dig[sq][item >> rfc_levels] -- the data root's throughput-heavy first levels
// spread over all workgroups instead of one per square.  PAIR: a lane pair
// per parent (kTopThreads pairs).
// ---------------------------------------------------------------------------
constexpr uint32_t kTopThreads = 128;   // parents per workgroup: tpw = 256 / n_in trees x n_in / 2

// flags: kTopHelpers -- schedule-helper waves in the narrow levels (PAIR);
// kTopWide -- the first level runs a thread per parent over 2 kTopThreads
// parents (tpw = 4 kTopThreads / n_in trees), the rest as lane pairs: one
// launch covers a level that has more parents than the lane pairs fit in a
// wave per SIMD (n_in >= 8).
constexpr uint32_t kTopHelpers = 1, kTopWide = 2;
template <bool PAIR>
__global__ __launch_bounds__(PAIR ? 2 * kTopThreads : kTopThreads) void tree_top_kernel(
    const Forest2 fs, uint32_t n_in, uint32_t tpw, uint32_t* __restrict__ dig, uint32_t n_dig, uint32_t rfc_levels,
    uint32_t flags) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][kTopThreads][kSlotWords];
    // schedule helpers (PAIR, levels of <= 64 parents): K + W of blocks 1 and
    // 2 of unit u's node at kwb[u][block - 1][t] (rows padded 4 words so the
    // units' 16-B reads spread over the banks)
    constexpr uint32_t kKwRow = 2 * 64 + 4;
    __shared__ __attribute__((aligned(16))) uint32_t kwb[PAIR ? 64 : 1][kKwRow];
    // kTopWide: the first level's 2 kTopThreads nodes, in kwb (the second
    // level has 128 parents, no helpers: kwb is free until the third)
    static_assert(!PAIR || 64 * kKwRow >= 2 * kTopThreads * kSlotWords, "wide level output must fit in kwb");
    uint32_t* wide_out = &kwb[0][0];
    const bool helpers = flags & kTopHelpers;
    const bool wide = PAIR && (flags & kTopWide);
    const size_t sq = blockIdx.y;
    const uint32_t n_trees = fs.f[0].n_trees + fs.f[1].n_trees;
    const uint32_t u = PAIR ? threadIdx.x >> 1 : threadIdx.x;   // unit (parent) index
    const bool A = PAIR && (threadIdx.x & 1);
    const bool writer = !A;                                    // one store per unit
    uint32_t o[kSlotWords];
    uint32_t cur = 0;
    if (wide) {   // first level: a thread per parent, from global memory into wide_out
        const uint32_t half = n_in / 2, j = threadIdx.x / half, p = threadIdx.x % half;
        const uint32_t g = blockIdx.x * tpw + j;
        if (j < tpw && g < n_trees) {
            const bool f1 = g >= fs.f[0].n_trees;
            const Forest& F = fs.f[f1 ? 1 : 0];
            const uint32_t t = f1 ? g - fs.f[0].n_trees : g;
            const uint8_t* l = F.in + sq * F.in_sq + ((size_t)t * F.tree_stride + (size_t)(2 * p) * F.node_stride) * kSlot;
            uint32_t L[kSlotWords], R[kSlotWords], w1[kSlotWords];
            load_slot_be(l, L);
            load_slot_be(l + (size_t)F.node_stride * kSlot, R);
            hash_node_u<false>(L, R, w1, false);
#pragma unroll
            for (int i = 0; i < kSlotWords; i++) wide_out[threadIdx.x * kSlotWords + i] = w1[i];
        }
        __syncthreads();
    }
    for (uint32_t m = wide ? n_in / 2 : n_in; m >= 2; m /= 2) {
        const uint32_t half = m / 2;
        const uint32_t j = u / half, p = u % half;   // tree j of this workgroup, parent p
        const uint32_t g = blockIdx.x * tpw + j;
        // this level's input nodes: node q of tree j at in_lds[(j * m + q) * kSlotWords]
        const uint32_t* in_lds = wide && m == n_in / 2 ? wide_out : &buf[cur][0][0];
        if (PAIR && helpers && m < n_in && tpw * half <= 64) {
            // At most two waves of parents: waves 2 and 3 would idle, so they
            // compute the message schedules of blocks 1 and 2 of every node
            // (one lane per block) while waves 0-1 run block 0; the parents'
            // lane pairs then run blocks 1 and 2 rounds-only (sha_pair_compress_kw:
            // the chain of dependent compressions is the critical wave's
            // instruction count).
            Sha<true> h;
            const bool work = threadIdx.x < 128 && j < tpw && g < n_trees;
            uint32_t L[kSlotWords], R[kSlotWords];
            if (threadIdx.x >= 128) {
                const uint32_t hi = threadIdx.x - 128, hu = hi >> 1, hb = 1 + (hi & 1);
                const uint32_t hj = hu / half, hp = hu % half;
                if (hj < tpw && blockIdx.x * tpw + hj < n_trees) {
#pragma unroll
                    for (int i = 0; i < kSlotWords; i++) {
                        L[i] = bswap32(in_lds[(hj * m + 2 * hp) * kSlotWords + i]);
                        R[i] = bswap32(in_lds[(hj * m + 2 * hp + 1) * kSlotWords + i]);
                    }
                    // the block index must be a compile-time constant in
                    // node_msg (a run-time one indexes L / R dynamically:
                    // private memory)
                    uint32_t w[16];
                    if (hb == 1) {
#pragma unroll
                        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 16 + i);
                    } else {
#pragma unroll
                        for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, 32 + i);
                    }
                    sha_schedule_kw(w, &kwb[hu][64 * (hb - 1)]);
                }
            } else if (work) {
#pragma unroll
                for (int i = 0; i < kSlotWords; i++) {
                    L[i] = bswap32(in_lds[(j * m + 2 * p) * kSlotWords + i]);
                    R[i] = bswap32(in_lds[(j * m + 2 * p + 1) * kSlotWords + i]);
                }
                h.init(A);
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; i++) w[i] = node_msg(L, R, i);
                h.compress(w, A);
            }
            __syncthreads();   // the helpers' schedules are in kwb
            if (work) {
#pragma unroll
                for (int b = 0; b < 2; b++) {
                    uint4 kw[16];
                    const uint4* row = reinterpret_cast<const uint4*>(&kwb[u][64 * b]);
#pragma unroll
                    for (int q = 0; q < 16; q++) kw[q] = row[q];
                    sha_pair_compress_kw(h.st, kw, A);
                }
                uint32_t D[8];
                h.digest(A, D);
                inner_node_words(L, R, D, o);
                if (m > 2 && writer) {
#pragma unroll
                    for (int i = 0; i < kSlotWords; i++) buf[cur ^ 1][u][i] = o[i];
                }
            }
        } else if (j < tpw && g < n_trees) {
            uint32_t L[kSlotWords], R[kSlotWords];
            if (m == n_in) {
                const bool f1 = g >= fs.f[0].n_trees;
                const Forest& F = fs.f[f1 ? 1 : 0];
                const uint32_t t = f1 ? g - fs.f[0].n_trees : g;
                const uint8_t* l =
                    F.in + sq * F.in_sq + ((size_t)t * F.tree_stride + (size_t)(2 * p) * F.node_stride) * kSlot;
                load_slot_be(l, L);
                load_slot_be(l + (size_t)F.node_stride * kSlot, R);
            } else {
#pragma unroll
                for (int i = 0; i < kSlotWords; i++) {
                    L[i] = bswap32(in_lds[(j * m + 2 * p) * kSlotWords + i]);
                    R[i] = bswap32(in_lds[(j * m + 2 * p + 1) * kSlotWords + i]);
                }
            }
            hash_node_u<PAIR>(L, R, o, A);
            if (m > 2 && writer) {
#pragma unroll
                for (int i = 0; i < kSlotWords; i++) buf[cur ^ 1][u][i] = o[i];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    // unit j < tpw holds tree j's root slot in o
    const uint32_t g = blockIdx.x * tpw + u;
    const bool has = u < tpw && g < n_trees;
    uint32_t D[8];
    if (has) {
        const bool f1 = g >= fs.f[0].n_trees;
        const Forest& F = fs.f[f1 ? 1 : 0];
        const uint32_t t = f1 ? g - fs.f[0].n_trees : g;
        if (writer && F.roots) {
            uint16_t* d16 = reinterpret_cast<uint16_t*>(F.roots + sq * F.roots_sq + (size_t)t * kNode);
#pragma unroll
            for (int i = 0; i < kNode / 2; i++) d16[i] = (uint16_t)(o[i / 2] >> (16 * (i & 1)));
        }
        if (writer && F.root_slots) store_slot(F.root_slots + sq * F.rslot_sq + (size_t)(F.root0 + t) * kSlot, o);
        if (dig) {
            uint32_t I[kSlotWords];
#pragma unroll
            for (int i = 0; i < kSlotWords; i++) I[i] = bswap32(o[i]);
            rfc_leaf_u<PAIR>(I, D, A);
        }
    }
    if (!dig) return;
    // rfc_levels inner levels over this workgroup's tpw digests (the host only
    // asks for them when every workgroup holds tpw trees): unit u < cnt holds
    // digest u of the current level
    uint32_t* dl = &buf[0][0][0];   // [unit][8]
    uint32_t cnt = tpw;
    for (uint32_t lv = 0; lv < rfc_levels; lv++) {
        if (u < cnt && writer) {
#pragma unroll
            for (int i = 0; i < 8; i++) dl[u * 8 + i] = D[i];
        }
        __syncthreads();
        cnt /= 2;
        if (u < cnt) {
            uint32_t a[8], b[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                a[i] = dl[(2 * u) * 8 + i];
                b[i] = dl[(2 * u + 1) * 8 + i];
            }
            rfc_inner_u<PAIR>(a, b, D, A);
        }
        __syncthreads();
    }
    if (has && writer && u < cnt) {
        uint4* d = reinterpret_cast<uint4*>(dig + (sq * n_dig + ((blockIdx.x * tpw) >> rfc_levels) + u) * 8);
        d[0] = make_uint4(D[0], D[1], D[2], D[3]);
        d[1] = make_uint4(D[4], D[5], D[6], D[7]);
    }
}

// ---------------------------------------------------------------------------
// Data root: RFC-6962 over the 2W root slots (rows then columns); 2W is a
// power of two so the tree is perfect.  One 256-thread block per square.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void data_root_kernel(const uint8_t* __restrict__ root_slots, uint32_t n,
                                                       uint8_t* __restrict__ data_roots) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hs[];   // ping [n][8] | pong [n/2][8]
    const size_t sq = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t I[kSlotWords], w[16];
        load_slot_be(root_slots + (sq * n + i) * (size_t)kSlot, I);
        ShaState st;
        sha_init(st);
#pragma unroll
        for (int b = 0; b < 2; b++) {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = rfc_leaf_msg(I, 16 * b + j);
            sha_compress(st, w);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) hs[i * 8 + j] = st.h[j];
    }
    __syncthreads();
    uint32_t* src = hs;
    uint32_t* dst = hs + n * 8;
    for (uint32_t m = n / 2; m >= 1; m >>= 1) {
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
            uint32_t A[8], B[8], w[16];
#pragma unroll
            for (int j = 0; j < 8; j++) { A[j] = src[(2 * i) * 8 + j]; B[j] = src[(2 * i + 1) * 8 + j]; }
            ShaState st;
            sha_init(st);
#pragma unroll
            for (int b = 0; b < 2; b++) {
#pragma unroll
                for (int j = 0; j < 16; j++) w[j] = rfc_inner_msg(A, B, 16 * b + j);
                sha_compress(st, w);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) dst[i * 8 + j] = st.h[j];
        }
        __syncthreads();
        uint32_t* t = src; src = dst; dst = t;
    }
    if (threadIdx.x == 0) {
        uint32_t* o = reinterpret_cast<uint32_t*>(data_roots + sq * 32);
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = bswap32(src[j]);
    }
}

// RFC-6962 leaf digests sha256(0x00 || root) of n 96-B root slots (one thread
// each, 2 compressions), 8 big-endian-valued words per digest.
__global__ __launch_bounds__(256) void rfc_leaf_kernel(const uint8_t* __restrict__ slots, uint32_t n,
                                                      uint32_t* __restrict__ dig) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t I[kSlotWords], w[16];
    load_slot_be(slots + (size_t)i * kSlot, I);
    ShaState st;
    sha_init(st);
#pragma unroll
    for (int b = 0; b < 2; b++) {
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rfc_leaf_msg(I, 16 * b + j);
        sha_compress(st, w);
    }
    uint4* d = reinterpret_cast<uint4*>(dig + (size_t)i * 8);
    d[0] = make_uint4(st.h[0], st.h[1], st.h[2], st.h[3]);
    d[1] = make_uint4(st.h[4], st.h[5], st.h[6], st.h[7]);
}

__global__ __launch_bounds__(512) void data_root_digest_kernel(const uint32_t* __restrict__ dig, uint32_t n,
                                                               uint8_t* __restrict__ data_roots,
                                                               const uint32_t* __restrict__ err,
                                                               int32_t* __restrict__ status, uint32_t pair_ok) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hs[];   // [n/2][8] | [n/4][8]
    __shared__ __attribute__((aligned(16))) uint32_t kwb[32][kDrKwRow];   // schedule helpers' K + W
    const size_t sq = blockIdx.x;
    data_root_levels(dig + sq * (size_t)n * 8, n, hs, hs + (n / 2) * 8, kwb, pair_ok, data_roots + sq * 32,
                     err + sq, status ? status + sq : nullptr);
}

__global__ void status_kernel(const uint32_t* __restrict__ err, uint32_t n, int32_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) status[i] = err[i] == 0xFFFFFFFFu ? 0 : -3;   // CDA_OK / CDA_ERR_PUSH_ORDER
}

__global__ void slots_to_roots_kernel(const uint8_t* __restrict__ slots, uint32_t n, uint8_t* __restrict__ rows,
                                      uint8_t* __restrict__ cols, uint32_t w) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n * (kNode / 2)) return;
    const uint32_t node = i / (kNode / 2), h = i % (kNode / 2);
    const uint16_t v = reinterpret_cast<const uint16_t*>(slots + (size_t)node * kSlot)[h];
    uint8_t* dst = node < w ? rows + (size_t)node * kNode : cols + (size_t)(node - w) * kNode;
    reinterpret_cast<uint16_t*>(dst)[h] = v;
}

}  // namespace

hipError_t launch_slots_to_roots(const uint8_t* slots, uint32_t n, uint8_t* rows, uint8_t* cols, uint32_t w,
                                 hipStream_t s) {
    hipLaunchKernelGGL(slots_to_roots_kernel, dim3((n * (kNode / 2) + 255) / 256), dim3(256), 0, s, slots, n, rows,
                       cols, w);
    return hipGetLastError();
}

hipError_t launch_status(const uint32_t* err, uint32_t n, int32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(status_kernel, dim3((n + 255) / 256), dim3(256), 0, s, err, n, status);
    return hipGetLastError();
}

hipError_t launch_row_order(const CellGrid& g, uint32_t n, uint32_t* err, hipStream_t s) {
    dim3 grid((g.rows * g.cols + 255) / 256, n);
    hipLaunchKernelGGL(row_order_kernel, grid, dim3(256), 0, s, g, err);
    return hipGetLastError();
}

// Occupancy limiter (tuning / co-run experiments): CDA_HASH_LDS=N reserves N
// bytes of (unused) LDS per hash workgroup, so at most 160 KiB / N of them
// share a CU -- e.g. 98304 leaves room for exactly one 256-thread workgroup
// (one wave per SIMD) next to a 64 KiB RS workgroup.
static size_t hash_lds(const void* fn) {
    static long v = -2;
    if (v == -2) {
        const char* e = test_knob("CDA_HASH_LDS");
        v = e ? atol(e) : 0;
    }
    if (v > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v);
    return v > 0 ? (size_t)v : 0;
}

// CUs of the current device (all devices of a process are MI355X).
static uint32_t device_cus() {
    static const uint32_t cus = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            return 0u;
        return (uint32_t)c;
    }();
    return cus;
}

// Workgroups of a hash launch over `nblocks` virtual blocks: all of them, or
// CDA_HASH_WG_PER_CU x the device's CUs (persistent; tuning / batch pipeline).
static uint32_t hash_grid(uint32_t nblocks) {
    static const uint32_t cap = [] {
        const char* e = test_knob("CDA_HASH_WG_PER_CU");
        const int per = e ? atoi(e) : 0;
        return per > 0 ? (uint32_t)per * device_cus() : 0u;
    }();
    return cap && nblocks > cap ? cap : nblocks;
}

// CDA_LEAF_PAIR_MAX: cells per launch up to which the lane-pair leaf kernel
// runs (default 32 768 = half a wave per SIMD of one-lane cells; 0 = never).
static uint64_t leaf_pair_max() {
    static const uint64_t v = [] {
        const char* e = test_knob("CDA_LEAF_PAIR_MAX");
        return e ? strtoull(e, nullptr, 10) : 32768ull;
    }();
    return v;
}

hipError_t launch_leaves(const CellGrid& g, uint32_t n, uint8_t* slots, uint32_t* err, bool check_rows,
                         bool check_cols, hipStream_t s) {
    const uint64_t cells = (uint64_t)g.rows * g.cols * n;
    if (cells > 0 && cells <= leaf_pair_max() && pair_sha_enabled()) {
        const uint32_t nbx2 = (g.rows * g.cols + 127) / 128;
        hipLaunchKernelGGL(leaf_pair_kernel, dim3(nbx2 * n), dim3(256), 0, s, g, slots, err, check_rows ? 1 : 0,
                           check_cols ? 1 : 0, nbx2);
        return hipGetLastError();
    }
    const uint32_t nbx = (g.rows * g.cols + 255) / 256, nblocks = nbx * n;
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(leaf_kernel, dim3(hash_grid(nblocks)), dim3(256),
                       hash_lds(reinterpret_cast<const void*>(leaf_kernel)), s, g, slots, err, check_rows ? 1 : 0,
                       check_cols ? 1 : 0, nbx, nblocks);
    return hipGetLastError();
}

hipError_t launch_level(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n, hipStream_t s) {
    if (n_forest < 1 || n_forest > 2 || n_in < 2) return hipErrorInvalidValue;
    Forest2 fs{};
    uint32_t maxw = 0;
    for (uint32_t i = 0; i < n_forest; i++) {
        fs.f[i] = f[i];
        maxw = maxw > f[i].n_trees * (n_in / 2) ? maxw : f[i].n_trees * (n_in / 2);
    }
    const uint32_t nbx = (maxw + 255) / 256, nblocks = nbx * n * n_forest;
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(level_kernel, dim3(hash_grid(nblocks)), dim3(256),
                       hash_lds(reinterpret_cast<const void*>(level_kernel)), s, fs, n_in, nbx, n, nblocks);
    return hipGetLastError();
}

hipError_t launch_subtrees(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t top, uint32_t n, hipStream_t s) {
    if (n_forest < 1 || n_forest > 2 || top < 1 || n_in % top) return hipErrorInvalidValue;
    const uint32_t S = n_in / top;
    if (S < 4 || (S & (S - 1))) return hipErrorInvalidValue;
    Forest2 fs{};
    uint32_t maxw = 0;
    for (uint32_t i = 0; i < n_forest; i++) {
        fs.f[i] = f[i];
        maxw = std::max(maxw, f[i].n_trees * top);
    }
    const uint32_t nbx = (maxw + 255) / 256, nblocks = nbx * n * n_forest;
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(subtree_kernel, dim3(nblocks), dim3(256), 0, s, fs, n_in, (uint32_t)__builtin_ctz(S), nbx, n,
                       nblocks);
    return hipGetLastError();
}

// CDA_TOP_PAIR=0 (A/B knob): one thread per parent in the tree tops and the
// data root instead of the lane-pair compression.
bool pair_sha_enabled() {
    static const bool v = [] {
        const char* e = test_knob("CDA_TOP_PAIR");
        return !(e && atoi(e) == 0);
    }();
    return v;
}

// data_root_levels' mode: 0 a thread per parent, 1 lane pairs, 2 lane pairs +
// schedule helpers (CDA_DR_HELPERS=0: no helpers; CDA_TOP_PAIR=0: no pairs)
static uint32_t data_root_mode() {
    static const bool dr_helpers = [] {
        const char* e = test_knob("CDA_DR_HELPERS");
        return !(e && atoi(e) == 0);
    }();
    return pair_sha_enabled() ? (dr_helpers ? 2u : 1u) : 0u;
}

hipError_t launch_tree_top(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n, uint32_t* dig,
                           uint32_t n_items, hipStream_t s, uint32_t* n_dig_out, bool wide) {
    wide = wide && pair_sha_enabled();
    if (n_forest < 1 || n_forest > 2 || n_in < (wide ? 8u : 2u) || n_in > (wide ? 4 : 2) * kTopThreads ||
        (n_in & (n_in - 1)))
        return hipErrorInvalidValue;
    Forest2 fs{};
    uint32_t trees = 0;
    for (uint32_t i = 0; i < n_forest; i++) {
        fs.f[i] = f[i];
        trees += f[i].n_trees;
    }
    const uint32_t tpw = (wide ? 4 : 2) * kTopThreads / n_in;   // trees per workgroup
    // RFC-6962 levels inside the workgroups: while every workgroup holds tpw
    // of the n_items (a power of two) roots and at least 2 digests per square
    // remain for data_root_digest_kernel
    uint32_t lv = 0;
    if (dig && trees == n_items && (n_items & (n_items - 1)) == 0 && tpw <= n_items)
        while ((2u << lv) <= tpw && (n_items >> (lv + 1)) >= 2) lv++;
    static const bool rfc_in_top = [] {   // CDA_TOP_RFC=0: leaf digests only (A/B knob)
        const char* e = test_knob("CDA_TOP_RFC");
        return !(e && atoi(e) == 0);
    }();
    if (!rfc_in_top) lv = 0;
    const uint32_t n_dig = n_items >> lv;
    if (n_dig_out) *n_dig_out = n_dig;
    // lane pairs while they still fit in a wave per SIMD (1024 SIMDs); wide:
    // the caller's choice (a thread per parent in the first level)
    const uint64_t parents = (uint64_t)n * trees * (n_in / 2);
    const bool pair = wide || (pair_sha_enabled() && 2 * parents <= 65536);
    const dim3 grid((trees + tpw - 1) / tpw, n);
    // CDA_TOP_HELPERS=0 (A/B knob): no schedule-helper waves in the narrow levels
    static const uint32_t helpers = [] {
        const char* e = test_knob("CDA_TOP_HELPERS");
        return e && atoi(e) == 0 ? 0u : kTopHelpers;
    }();
    if (pair)
        hipLaunchKernelGGL(tree_top_kernel<true>, grid, dim3(2 * kTopThreads), 0, s, fs, n_in, tpw, dig, n_dig, lv,
                           helpers | (wide ? kTopWide : 0u));
    else
        hipLaunchKernelGGL(tree_top_kernel<false>, grid, dim3(kTopThreads), 0, s, fs, n_in, tpw, dig, n_dig, lv, 0u);
    return hipGetLastError();
}

hipError_t launch_data_root(const uint8_t* root_slots, uint32_t n_items, uint32_t n, uint8_t* data_roots,
                            hipStream_t s) {
    if (n_items < 2 || (n_items & (n_items - 1))) return hipErrorInvalidValue;
    const size_t lds = (size_t)3 * (n_items / 2) * 32;   // ping-pong: n + n/2 digests
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(data_root_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(data_root_kernel, dim3(n), dim3(256), lds, s, root_slots, n_items, data_roots);
    return hipGetLastError();
}

hipError_t launch_data_root_slots(const uint8_t* root_slots, uint32_t n_items, uint32_t n, uint32_t* dig,
                                  uint8_t* data_roots, hipStream_t s, const uint32_t* err, int32_t* status) {
    if (n_items < 2 || n_items > 4096 || (n_items & (n_items - 1))) return hipErrorInvalidValue;
    const uint32_t total = n_items * n;
    hipLaunchKernelGGL(rfc_leaf_kernel, dim3((total + 255) / 256), dim3(256), 0, s, root_slots, total, dig);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_data_root_digests(dig, n_items, n, data_roots, s, err, status);
}

hipError_t launch_rfc_leaves(const uint8_t* slots, uint32_t n, uint32_t* dig, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rfc_leaf_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slots, n, dig);
    return hipGetLastError();
}

hipError_t launch_data_root_digests(const uint32_t* dig, uint32_t n_items, uint32_t n, uint8_t* data_roots,
                                    hipStream_t s, const uint32_t* err, int32_t* status) {
    if (n_items < 2 || n_items > 4096 || (n_items & (n_items - 1))) return hipErrorInvalidValue;
    const size_t lds = (size_t)(n_items / 2 + n_items / 4) * 32;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(data_root_digest_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    // a thread per first-level parent (<= 512: more would cap the kernel at
    // 128 VGPRs and spill the helpers' registers), and room for the lane pairs
    const uint32_t pmax = n <= kPairSmallSquares ? kPairMaxParentsSmall : kPairMaxParents;
    uint32_t threads = std::min<uint32_t>(n_items / 2, 512);
    threads = std::max<uint32_t>(threads, std::min<uint32_t>(n_items, 2 * pmax));
    threads = std::max<uint32_t>((threads + 63) / 64 * 64, 64);
    // mode in the low byte, the largest pair level above it
    const uint32_t mode = data_root_mode() | pmax << 8;
    hipLaunchKernelGGL(data_root_digest_kernel, dim3(n), dim3(threads), lds, s, dig, n_items, data_roots,
                       status ? err : nullptr, status, mode);
    return hipGetLastError();
}

}  // namespace cda
