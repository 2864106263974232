// leaf_dev.h -- NMT leaf hashing of one EDS cell (device code), shared by the
// leaf launch (nmt.hip leaf_kernel) and the fused GF(2^8) encode + leaf
// launch (rs_gf8_bs.hip rs8_leaf_kernel).
//
// Reference: nmt HashLeaf (EXT v0.22.0; in-tree copy
// /root/reference/test/util/malicious/hasher.go:186-310) over the erasured
// wrapper's leaf (/root/reference/pkg/wrapper/nmt_wrapper.go:93-140):
// 0x00 || ns || share, ns = share[0:29] in Q0 and ParitySharesNamespace
// (0xFF * 29) elsewhere; nmt Push rejects a namespace below its predecessor
// (ErrInvalidPushOrder), checked here for the Q0 rows and columns.
#pragma once
#include "cda_kernels.h"
#include "sha256_dev.h"

namespace cda {

// ---------------------------------------------------------------------------
// Q0 push-order check (nmt ErrInvalidPushOrder on any row or column of Q0).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_ns_be(const uint8_t* cell, uint32_t (&ns)[8]) {
    const uint4* p = reinterpret_cast<const uint4*>(cell);
    const uint4 a = p[0], b = p[1];
    ns[0] = bswap32(a.x); ns[1] = bswap32(a.y); ns[2] = bswap32(a.z); ns[3] = bswap32(a.w);
    ns[4] = bswap32(b.x); ns[5] = bswap32(b.y); ns[6] = bswap32(b.z); ns[7] = bswap32(b.w) & 0xFF000000u;
}
// a < b lexicographically over the 29 namespace bytes
__device__ __forceinline__ bool ns_less(const uint32_t (&a)[8], const uint32_t (&b)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (a[i] != b[i]) return a[i] < b[i];
    return false;
}

// ---------------------------------------------------------------------------
// Leaf hashing: one thread per EDS cell, 9 SHA-256 blocks of
// 0x00 || ns || share.  The share is streamed in 64-B chunks of raw
// little-endian words; every big-endian message word is ONE v_perm_b32 of two
// raw words (byte swap and the 30-byte message offset folded together).  Only
// the upper half of the previous chunk (8 words) is carried between blocks.
// 125 VGPRs, four waves per SIMD (CDA_LEAF_WAVES); at five the compiler fits
// 96 VGPRs only by spilling 34 values.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_raw16(const uint4* p, uint32_t (&w)[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 v = p[q];
        w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
// Big-endian message word from share bytes 4j+2 .. 4j+5 (raw words j, j+1).
__device__ __forceinline__ uint32_t body_word(uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x02030405u); }

// Push-order check of a Q0 cell against its right / lower neighbour (fused
// into the leaf launch: this cell's namespace is in nsw).
__device__ __forceinline__ void leaf_order_check(const CellGrid& g, const uint8_t* cellp, const uint32_t (&nsw)[8],
                                                 uint32_t* err, int check_rows, int check_cols, uint32_t r, uint32_t c,
                                                 uint32_t gr, uint32_t gc) {
    const uint32_t k = g.k;
    uint32_t nb[8];
    uint32_t key = 0xFFFFFFFFu;
    if (check_rows && gc + 1 < k && c + 1 < g.cols) {
        load_ns_be(cellp + kShare, nb);
        if (ns_less(nb, nsw)) key = min(key, (0u << 24) | (gr << 12) | (gc + 1));
    }
    if (check_cols && gr + 1 < k && r + 1 < g.rows) {
        load_ns_be(cellp + (size_t)g.row_stride * kShare, nb);
        if (ns_less(nb, nsw)) key = min(key, (1u << 24) | (gc << 12) | (gr + 1));
    }
    if (key != 0xFFFFFFFFu) atomicMin(err, key);
}

// The leaf node of cell (r, c) of square sq of grid g, stored to its 96-B
// slot slots[sq][r][c].  ns_slot: 8 words of LDS that hold this cell's
// namespace between the first chunk and the leaf node (Q0 cells).  Round 5:
// the namespace used to be reloaded from global memory after the ninth block
// and the neighbours' namespaces read there too -- lines long evicted by then,
// ~1.2x the algorithmic bytes at the fabric (r04s / r05m PMC); now the check
// runs while the neighbours' first chunks are in flight in the same wave / the
// next workgroup, and the own namespace waits in LDS: the launch's FETCH_SIZE
// -5 %, WRITE_SIZE -20 % (its six spilled values gone, 128 -> 125 VGPRs), time
// equal (VALU-bound; profiles/r05/leaf_ns_ab.txt).
__device__ __forceinline__ void leaf_cell(const CellGrid& g, uint8_t* __restrict__ slots, uint32_t* __restrict__ err,
                                          int check_rows, int check_cols, size_t sq, uint32_t r, uint32_t c,
                                          uint32_t* ns_slot) {
    const uint32_t cell = r * g.cols + c;
    const uint32_t gr = g.row0 + r, gc = g.col0 + c, k = g.k;
    const bool parity = !(gr < k && gc < k);
    const uint8_t* E = g.base + sq * g.sq;
    const uint8_t* cellp = E + ((size_t)r * g.row_stride + c) * kShare;
    const uint4* src = reinterpret_cast<const uint4*>(cellp);

    ShaState st;
    sha_init(st);
    uint32_t cur[16], tail[8], w[16];
    load_raw16(src, cur);
    if (!parity) {
        uint32_t nsw[8];
#pragma unroll
        for (int i = 0; i < 8; i++) nsw[i] = bswap32(cur[i]);
        nsw[7] &= 0xFF000000u;
        uint4* o = reinterpret_cast<uint4*>(ns_slot);
        o[0] = make_uint4(nsw[0], nsw[1], nsw[2], nsw[3]);
        o[1] = make_uint4(nsw[4], nsw[5], nsw[6], nsw[7]);
        leaf_order_check(g, cellp, nsw, err + sq, check_rows, check_cols, r, c, gr, gc);
    }
    uint32_t nxt[16];   // the next 64-B chunk in flight during each block
    load_raw16(src + 4, nxt);
    // block 0: 0x00 || ns(29) || share[0:34]; a parity leaf's first 7 words
    // are constant, so it starts from the precomputed mid-state
#pragma unroll
    for (int i = 8; i < 16; i++) w[i] = body_word(cur[i - 8], cur[i - 7]);
    if (parity) {
        w[7] = __builtin_amdgcn_perm(cur[0], cur[0], 0x0D0D0001u);
        sha_compress_from<kLeafParityRounds>(st, kLeafParityMid, kLeafParityHead, w);
    } else {
        w[0] = __builtin_amdgcn_perm(cur[0], cur[0], 0x0C000102u);
#pragma unroll
        for (int i = 1; i < 7; i++) w[i] = __builtin_amdgcn_perm(cur[i], cur[i - 1], 0x03040506u);
        w[7] = __builtin_amdgcn_perm(cur[7], cur[6], 0x03040C0Cu) | __builtin_amdgcn_perm(cur[0], cur[0], 0x0C0C0001u);
        sha_compress(st, w);
    }
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
        sha_compress(st, w);
    }
    // block 8: share words 120..127 then padding (542-B message)
#pragma unroll
    for (int t = 0; t < 7; t++) w[t] = body_word(tail[t], tail[t + 1]);
    w[7] = __builtin_amdgcn_perm(tail[7], tail[7], 0x02030C0Cu) | 0x8000u;
#pragma unroll
    for (int t = 8; t < 15; t++) w[t] = 0;
    w[15] = kLeafMsgBits;
    sha_compress(st, w);

    // namespace (big-endian words): saved in LDS, 8 VGPRs not live here
    uint32_t nsw[8];
    if (parity) {
#pragma unroll
        for (int i = 0; i < 8; i++) nsw[i] = 0xFFFFFFFFu;
    } else {
        const uint4* q = reinterpret_cast<const uint4*>(ns_slot);
        const uint4 a = q[0], b = q[1];
        nsw[0] = a.x; nsw[1] = a.y; nsw[2] = a.z; nsw[3] = a.w;
        nsw[4] = b.x; nsw[5] = b.y; nsw[6] = b.z; nsw[7] = b.w;
    }
    uint32_t out[kSlotWords];
    leaf_node_words(nsw, st.h, out);
    store_slot(slots + (sq * (size_t)g.rows * g.cols + cell) * kSlot, out);
}

}  // namespace cda
