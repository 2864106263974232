// split_layout.h -- the buffer arithmetic of config 5 (one square over G
// ranks; comm.hip split_extend_dah), host + device.
//
// Rank g holds R = k/G ODS rows and, after the all-to-all, C = W/G EDS
// columns (W = 2k).  Every offset the split uses is computed here, by the
// group_rows kernel on the device and by split_extend_dah on the host, and
// exported through cda_split_layout / cda_split_offsets (include/cda.h) so a
// CPU test can replay the G > 1 exchange over in-memory buffers with the very
// same arithmetic (tests/test_split_layout.py; unmeasured on hardware).
//
//   send buffer [G][R][C][512]: piece h = the sender's R rows restricted to
//     columns [h*C, h*C + C), sent to rank h;
//   column block [W][C][512]: EDS rows of the receiver's C columns; the piece
//     received from rank g lands at byte g * piece = rows g*R .. g*R + R - 1,
//     i.e. ODS rows in order: rows 0..k-1 after the all-to-all, rows k..W-1
//     written by the column encode;
//   slot area (96-B node slots): [C] column roots, [W] row subtree nodes of
//     this rank's columns, then (rank 0) the gathered [G][W] row subtrees and
//     [G*C = W] column roots in rank order, then the push-order word;
//   combine (rank 0): row tree r = the G subtree nodes (g, r) at g*W + r of
//     the gathered [G][W], i.e. leaves of a G-leaf tree.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SPLIT_HD __host__ __device__ __forceinline__
#else
#define SPLIT_HD inline
#endif

namespace cda {

struct SplitLayout {
    static constexpr uint32_t kShareB = 512, kSlotB = 96;
    uint32_t k, G, W, R, C;

    SPLIT_HD SplitLayout(uint32_t k_, uint32_t g_) : k(k_), G(g_), W(2 * k_), R(k_ / g_), C(2 * k_ / g_) {}
    // k a power of two <= 1024, G a power of two dividing k
    SPLIT_HD bool valid() const { return k && !(k & (k - 1)) && G && !(G & (G - 1)) && k % G == 0 && k <= 1024; }

    SPLIT_HD uint64_t piece() const { return (uint64_t)R * C * kShareB; }           // one rank pair's block
    SPLIT_HD uint64_t send_bytes() const { return piece() * G; }
    SPLIT_HD uint64_t col_block_bytes() const { return (uint64_t)W * C * kShareB; }
    // send layout: row-block cell (r, col), r < R, col < W
    SPLIT_HD uint64_t send_off(uint32_t r, uint32_t col) const {
        const uint32_t h = col / C, c = col % C;
        return (((uint64_t)h * R + r) * C + c) * kShareB;
    }
    SPLIT_HD uint64_t send_piece_off(uint32_t h) const { return (uint64_t)h * piece(); }   // piece for rank h
    SPLIT_HD uint64_t recv_piece_off(uint32_t g) const { return (uint64_t)g * piece(); }   // piece from rank g
    // column block: EDS row `row` (< W), local column c (< C)
    SPLIT_HD uint64_t block_off(uint32_t row, uint32_t c) const { return ((uint64_t)row * C + c) * kShareB; }
    // slot area, bytes
    SPLIT_HD uint64_t col_slots_off() const { return 0; }
    SPLIT_HD uint64_t row_sub_off() const { return (uint64_t)C * kSlotB; }
    SPLIT_HD uint64_t own_slots() const { return (uint64_t)(C + W) * kSlotB; }
    SPLIT_HD uint64_t gather_sub_off(uint32_t h) const { return own_slots() + (uint64_t)h * W * kSlotB; }
    SPLIT_HD uint64_t gather_col_off(uint32_t h) const {
        return own_slots() + (uint64_t)G * W * kSlotB + (uint64_t)h * C * kSlotB;
    }
    SPLIT_HD uint64_t err_off() const { return own_slots() + (uint64_t)G * W * kSlotB + (uint64_t)W * kSlotB; }
    SPLIT_HD uint64_t slots_bytes() const { return err_off() + 64; }
    // combine: slot index of rank g's subtree node of row r in the gathered [G][W]
    SPLIT_HD uint64_t combine_slot(uint32_t g, uint32_t r) const { return (uint64_t)g * W + r; }
};

}  // namespace cda
