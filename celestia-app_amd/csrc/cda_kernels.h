// cda_kernels.h -- launch interface of the HIP kernels (engine <-> kernels).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cda {

// Phase of the 2-D extension (rsmt2d erasureExtendSquare schedule):
//   kPhaseQ0: codewords 0..k-1 = ODS rows (Q0->Q1, also copies Q0 into the EDS),
//             codewords k..2k-1 = ODS columns (Q0->Q2);
//   kPhaseQ3: codewords 0..k-1 = EDS rows k..2k-1 (Q2->Q3).
enum RsPhase : int { kPhaseQ0 = 0, kPhaseQ3 = 1 };

// GF(2^8) Leopard encode of whole squares (k <= 128).
hipError_t launch_rs8(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t n_squares, int phase,
                      hipStream_t stream);
// GF(2^8) encode of an arbitrary list of codewords: n_code codewords of k
// shards x len bytes, contiguous (rsmt2d Codec.Encode compatibility).
hipError_t launch_rs8_flat(const uint8_t* data, uint8_t* parity, uint32_t k, uint32_t len, uint32_t n_code,
                           hipStream_t stream);

// GF(2^16) tables uploaded once per context.
struct Gf16Dev {
    const uint16_t* log;   // 65536
    const uint16_t* exp;   // 65536
    const uint16_t* skew;  // 65535
    // Per-k multiply tables for the register-resident encoder (k = 256, 512):
    // chunk[idx][16] = 2-bit-chunk v_perm tables of the constant skew[idx]
    // (all zero when skew[idx] is the modulus, i.e. "multiply by zero").
    const uint32_t* chunk = nullptr;
    uint32_t chunk_k = 0;
};
hipError_t launch_rs16(const Gf16Dev& t, const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t n_squares,
                       int phase, hipStream_t stream);
hipError_t launch_rs16_flat(const Gf16Dev& t, const uint8_t* data, uint8_t* parity, uint32_t k, uint32_t len,
                            uint32_t n_code, hipStream_t stream);

// Q0 namespace order check: err[s] = min over violations of
// (axis << 24 | axis_index << 12 | push_position), 0xFFFFFFFF when ordered.
hipError_t launch_order_check(const uint8_t* eds, uint32_t k, uint32_t n_squares, uint32_t* err,
                              hipStream_t stream);
// err word -> CDA_OK (0) / CDA_ERR_PUSH_ORDER (-3) per square.
hipError_t launch_status(const uint32_t* err, uint32_t n_squares, int32_t* status, hipStream_t stream);
// NMT leaf hashing: one 96-B leaf slot per EDS cell, [n][W][W]; also runs the
// Q0 push-order check (same err encoding as launch_order_check).
hipError_t launch_leaves(const uint8_t* eds, uint32_t k, uint32_t n_squares, uint8_t* leaf_slots, uint32_t* err,
                         hipStream_t stream);
// One NMT level for all 2W trees of every square.  `in_leaf` selects the
// level-0 addressing (row tree t = leaf row t, column tree t = leaf column t);
// otherwise `in` is [n][2W][n_in] slots (rows then columns).  Output is
// [n][2W][n_in/2] slots; when n_in == 2 the roots are written as packed
// 90-byte nodes to row_roots/col_roots ([n][W][90]) and as 96-B slots to
// root_slots ([n][2W][96], rows then columns) instead.
hipError_t launch_level(const uint8_t* in, bool in_leaf, uint32_t W, uint32_t n_in, uint32_t n_squares,
                        uint8_t* out, uint8_t* row_roots, uint8_t* col_roots, uint8_t* root_slots,
                        hipStream_t stream);
// RFC-6962 data root of rows || cols per square (reads root_slots).
hipError_t launch_data_root(const uint8_t* root_slots, uint32_t W, uint32_t n_squares, uint8_t* data_roots,
                            hipStream_t stream);

}  // namespace cda
