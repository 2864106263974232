// cda_kernels.h -- launch interface of the HIP kernels (engine <-> kernels).
//
// All kernels address shares through small descriptors of byte offsets so the
// same code serves whole squares (configs 1-4), the row/column blocks of a
// square split across GPUs (config 5) and rsmt2d Codec.Encode batches.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cda {

constexpr uint32_t kNoCopy = 0xFFFFFFFFu;

// One group of codewords: codeword c, shard i lives at
//   base + off + c*cw + i*sh   (bytes; offsets are per square and < 4 GiB).
// `cpy_*` optionally stores the data shards unchanged (ODS -> EDS Q0 copy).
struct RsSeg {
    uint32_t n_cw;
    uint32_t src_off, src_cw, src_sh;
    uint32_t dst_off, dst_cw, dst_sh;
    uint32_t cpy_off = kNoCopy, cpy_cw = 0, cpy_sh = 0;
};
// Up to two segments per launch (e.g. rows and columns of Q0 in one grid);
// blockIdx.y selects the square: src + y*src_sq, dst + y*dst_sq.
struct RsJob {
    const uint8_t* src;
    uint8_t* dst;           // parity and copy destination
    uint64_t src_sq, dst_sq;
    RsSeg seg[2];
    uint32_t n_seg;
    // optional: err_init[y] = 0xFFFFFFFF for every square y of the launch
    // (the push-order words of the hashing that follows, set by the RS launch
    // instead of a separate fill)
    uint32_t* err_init = nullptr;
    // GF(2^16) bitsliced encoder: raise the wave priority (s_setprio) while a
    // workgroup loads and while it stores (Engine::enqueue_extend, batches of
    // <= CDA_RS16_PRIO_MAX squares)
    uint32_t prio = 0;
};
#if defined(__HIPCC__)
__device__ __forceinline__ void rs_err_init(const RsJob& job) {
    if (job.err_init && blockIdx.x == 0 && threadIdx.x == 0) job.err_init[blockIdx.y] = 0xFFFFFFFFu;
}
#endif

// GF(2^16) tables uploaded once per context.
struct Gf16Dev {
    const uint16_t* log;   // 65536
    const uint16_t* exp;   // 65536
    const uint16_t* skew;  // 65535
};

// Leopard encode of every codeword of `job` for n_squares squares; k data
// shards of 512 B per codeword (GF(2^8) for k <= 128, GF(2^16) above).
hipError_t launch_rs(const RsJob& job, uint32_t k, uint32_t n_squares, const Gf16Dev& gf16, hipStream_t stream);
// Bitsliced GF(2^16) encode of every codeword of `job` (k = 256 or 512).
hipError_t launch_rs16_bs(const RsJob& job, uint32_t k, uint32_t n_squares, hipStream_t stream);
// rsmt2d Codec.Encode of n_code contiguous codewords of k shards x len bytes.
hipError_t launch_rs8_flat(const uint8_t* data, uint8_t* parity, uint32_t k, uint32_t len, uint32_t n_code,
                           hipStream_t stream);
hipError_t launch_rs16_flat(const Gf16Dev& t, const uint8_t* data, uint8_t* parity, uint32_t k, uint32_t len,
                            uint32_t n_code, hipStream_t stream);

// Square phases (rsmt2d erasureExtendSquare): Q0->Q1 rows + Q0->Q2 columns
// (with the Q0 copy), then Q2->Q3 rows.
RsJob square_job_q0(const uint8_t* ods, uint8_t* eds, uint32_t k);
RsJob square_job_q0_inplace(uint8_t* eds, uint32_t k);
RsJob square_job_q3(uint8_t* eds, uint32_t k);

// A grid of EDS cells seen by the hash kernels: cell (r, c) of square y at
//   base + y*sq + (r*row_stride + c)*512, global coordinates (row0 + r, col0 + c),
// quadrant Q0 when row0+r < k and col0+c < k.
struct CellGrid {
    const uint8_t* base;
    uint64_t sq;            // bytes per square
    uint32_t rows, cols, row_stride;
    uint32_t row0, col0, k;
};

// NMT leaf hashing: one 96-B leaf slot per grid cell, slots[y][r][c].  Also
// checks nmt push order inside Q0: along rows if check_rows (both cells in the
// grid) and along columns if check_cols.  err[y] = min over violations of
// (axis << 24 | axis_index << 12 | push_position) in global coordinates.
hipError_t launch_leaves(const CellGrid& g, uint32_t n_squares, uint8_t* slots, uint32_t* err, bool check_rows,
                         bool check_cols, hipStream_t stream);
// Push-order check of Q0 rows only, for a block of ODS rows held in
// row-major order (config 5: each rank checks the rows it owns).
hipError_t launch_row_order(const CellGrid& g, uint32_t n_squares, uint32_t* err, hipStream_t stream);

// A forest of NMT trees over 96-B slots: node i of tree t of square y at
//   in + y*in_sq + (t*tree_stride + i*node_stride)*96.
// One level halves every tree: parent p of tree t goes to
//   out + y*out_sq + (t*n_in/2 + p)*96;
// when n_in == 2 the tree roots are written instead as packed 90-B nodes to
// roots + y*roots_sq + t*90 (if roots) and as 96-B slots to
// root_slots + y*rslot_sq + (root0 + t)*96 (if root_slots).
struct Forest {
    const uint8_t* in;
    uint64_t in_sq;
    uint32_t n_trees, tree_stride, node_stride;
    uint8_t* out;
    uint64_t out_sq;
    uint8_t* roots;
    uint64_t roots_sq;
    uint8_t* root_slots;
    uint64_t rslot_sq;
    uint32_t root0;
};
// One level of up to two forests with the same n_in (blockIdx.z selects).
hipError_t launch_level(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n_squares, hipStream_t stream);
// The levels of up to two forests from n_in down to `top` nodes per tree in
// ONE launch: a lane per (n_in / top)-leaf subtree hashes its nodes in post
// order (nmt.hip subtree_kernel); roots to out + y*out_sq + (t*top + s)*96,
// with per-lane stacks behind them (n_trees*top*log2(n_in/top) slots per
// forest and square in all); top == 1: the trees' roots to roots /
// root_slots, as launch_level's last level writes them.  n_in / top a power
// of two >= 4.
hipError_t launch_subtrees(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t top, uint32_t n_squares,
                           hipStream_t stream);
// Every remaining level of up to two forests of n_in (<= 256) nodes per tree
// in one launch (a workgroup takes 256 / n_in trees, levels in LDS; wide: 8 <=
// n_in <= 512, 512 / n_in trees, the first level a thread per parent, the
// rest lane pairs -- for a first level too wide for lane pairs); the roots go to
// roots / root_slots as in launch_level, and if dig is non-NULL the first
// levels of the data root over the n_items roots per square: RFC-6962 leaf
// digests and, where every workgroup holds a power-of-two group of roots,
// inner levels over the group; *n_dig_out (<= n_items) digests per square go
// to dig[sq][.] for launch_data_root_digests.
// Lane-pair SHA-256 in the tree tops and the data root (CDA_TOP_PAIR=0: off).
bool pair_sha_enabled();
hipError_t launch_tree_top(const Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n_squares, uint32_t* dig,
                           uint32_t n_items, hipStream_t stream, uint32_t* n_dig_out = nullptr, bool wide = false);
// RFC-6962 data root over n_items 96-B root slots per square (power of two).
hipError_t launch_data_root(const uint8_t* root_slots, uint32_t n_items, uint32_t n_squares, uint8_t* data_roots,
                            hipStream_t stream);
// The same from the root slots in two wide launches: RFC-6962 leaf digests
// (one thread per root, into `digests`: n_items*n_squares*32 B of scratch),
// then one workgroup per square for the inner levels (n_items a power of two
// <= 4096).
// err / status (optional): also writes status[sq] = CDA_OK / CDA_ERR_PUSH_ORDER
// from the push-order word err[sq] (status_kernel fused into the last launch).
hipError_t launch_data_root_slots(const uint8_t* root_slots, uint32_t n_items, uint32_t n_squares,
                                  uint32_t* digests, uint8_t* data_roots, hipStream_t stream,
                                  const uint32_t* err = nullptr, int32_t* status = nullptr);
// RFC-6962 leaf digests sha256(0x00 || slot[0:90]) of n slots (8 words each).
hipError_t launch_rfc_leaves(const uint8_t* slots, uint32_t n, uint32_t* digests, hipStream_t stream);
hipError_t launch_data_root_digests(const uint32_t* digests, uint32_t n_items, uint32_t n_squares,
                                    uint8_t* data_roots, hipStream_t stream, const uint32_t* err = nullptr,
                                    int32_t* status = nullptr);
// Pack n_slots 96-B root slots (rows then columns) into 90-B roots.
hipError_t launch_slots_to_roots(const uint8_t* slots, uint32_t n_slots, uint8_t* rows, uint8_t* cols, uint32_t w,
                                 hipStream_t stream);
// err word -> CDA_OK (0) / CDA_ERR_PUSH_ORDER (-3) per square.
hipError_t launch_status(const uint32_t* err, uint32_t n_squares, int32_t* status, hipStream_t stream);

}  // namespace cda
