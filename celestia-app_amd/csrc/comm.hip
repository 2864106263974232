// comm.hip -- multi-GPU inside the library.
//
//   * Config 5 (one k = 512 square over G GPUs): each rank's context joins an
//     RCCL communicator (cda_comm_init); cda_extend_dah_split then runs the
//     whole split on the rank's stream -- row encode of the rank's ODS rows
//     straight into the all-to-all send layout, one grouped ncclSend/ncclRecv
//     all-to-all over xGMI into the column block, column encode + hashing,
//     one grouped gather of the 96-B subtree / column-root slots and a MIN
//     reduce of the push-order word to rank 0, which finishes the row trees
//     and the data root.  A cgo host needs no torch.distributed.
//   * Config 4 (independent squares): cda_extend_dah_multi splits a host batch
//     over several contexts (one per device) and runs them on host threads --
//     no collective at all.
// Reference call sites: app/process_proposal.go:138-152 (block replay),
// pkg/da/data_availability_header.go:44-75.
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

// [R][W] row block -> [G][R][C] send layout (dst g = columns [g*C, g*C+C)):
// one thread per 16 bytes.
__global__ __launch_bounds__(256) void group_rows_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        uint32_t R, uint32_t W, uint32_t C) {
    constexpr uint32_t V = kShare / 16;   // uint4 per share
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint64_t)R * W * V) return;
    const uint32_t v = (uint32_t)(i % V);
    const uint64_t cell = i / V;
    const uint32_t r = (uint32_t)(cell / W), col = (uint32_t)(cell % W);
    const uint32_t g = col / C, c = col % C;
    dst[(((uint64_t)g * R + r) * C + c) * V + v] = src[i];
}

int nccl_check(Engine& e, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return CDA_OK;
    return e.fail(CDA_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

int Engine::enqueue_split_rows_send(const uint8_t* d_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                                    uint32_t parts, uint8_t* d_send, uint32_t* d_err, hipStream_t s) {
    const uint32_t W = 2 * k;
    if (parts == 0 || (parts & (parts - 1)) || parts > W || n_rows == 0)
        return fail(CDA_ERR_INVALID, "bad split: parts must be a power of two <= 2k");
    const uint32_t C = W / parts;
    int rc;
    if (parts == 1) return enqueue_split_rows(d_rows, k, n_rows, row0, d_send, d_err, s);   // [1][R][W] = [R][W]
    if ((rc = check(split_blk_.ensure((size_t)n_rows * W * kShare), "hipMalloc row block"))) return rc;
    if ((rc = enqueue_split_rows(d_rows, k, n_rows, row0, split_blk_.as<uint8_t>(), d_err, s))) return rc;
    const uint64_t n16 = (uint64_t)n_rows * W * (kShare / 16);
    hipLaunchKernelGGL(group_rows_kernel, dim3((uint32_t)((n16 + 255) / 256)), dim3(256), 0, s,
                       split_blk_.as<uint4>(), reinterpret_cast<uint4*>(d_send), n_rows, W, C);
    return check(hipGetLastError(), "group rows");
}

int comm_unique_id(uint8_t* id) {
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return CDA_ERR_DEVICE;
    memcpy(id, &uid, sizeof uid);
    return CDA_OK;
}

int Engine::comm_init(int rank, int world, const uint8_t* id) {
    if (world < 1 || rank < 0 || rank >= world) return fail(CDA_ERR_INVALID, "bad rank / world size");
    if (comm_) {
        (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
        comm_ = nullptr;
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclComm_t c = nullptr;
    int rc;
    if ((rc = nccl_check(*this, ncclCommInitRank(&c, world, uid, rank), "ncclCommInitRank"))) return rc;
    comm_ = c;
    rank_ = rank;
    world_ = world;
    return CDA_OK;
}

void Engine::comm_destroy() {
    if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
    rank_ = 0;
    world_ = 0;
}

int Engine::split_extend_dah(const uint8_t* d_rows, uint32_t k, uint8_t* d_col_block, uint8_t* d_row_roots,
                             uint8_t* d_col_roots, uint8_t* d_root, uint32_t* d_err, hipStream_t s) {
    if (!comm_) return fail(CDA_ERR_INVALID, "no communicator: call cda_comm_init first");
    const uint32_t G = (uint32_t)world_, W = 2 * k;
    if (k == 0 || (k & (k - 1)) || (G & (G - 1)) || k % G) return fail(CDA_ERR_INVALID, "world size must divide k");
    const uint32_t R = k / G, C = W / G;
    const size_t piece = (size_t)R * C * kShare;   // one rank pair's all-to-all block
    ncclComm_t comm = static_cast<ncclComm_t>(comm_);
    int rc;
    if (G > 1 && (rc = check(split_send_.ensure(piece * G), "hipMalloc send"))) return rc;
    uint8_t* block = d_col_block;
    if (!block) {
        if ((rc = check(split_col_.ensure((size_t)W * C * kShare), "hipMalloc column block"))) return rc;
        block = split_col_.as<uint8_t>();
    }
    // slots: this rank's column roots [C] and row subtrees [W]; rank 0 also
    // the gathered [G][W] subtrees and [W] column roots (rank order)
    const size_t own = (size_t)(C + W) * kSlot, all = (size_t)G * (C + W) * kSlot;
    if ((rc = check(split_slots_.ensure(own + all), "hipMalloc slots"))) return rc;
    uint8_t* col_slots = split_slots_.as<uint8_t>();
    uint8_t* row_sub = col_slots + (size_t)C * kSlot;
    uint8_t* g_sub = col_slots + own;                        // [G][W][96]
    uint8_t* g_col = g_sub + (size_t)G * W * kSlot;          // [G*C = W][96]
    if ((rc = check(hipMemsetAsync(d_err, 0xFF, 4, s), "hipMemsetAsync"))) return rc;
    if (G == 1) {
        // one rank: the row block IS rows 0..k-1 of the (whole) column block
        if ((rc = enqueue_split_rows_send(d_rows, k, R, 0, 1, block, d_err, s))) return rc;
    } else {
        // 1. rows -> [G][R][C] send layout
        if ((rc = enqueue_split_rows_send(d_rows, k, R, (uint32_t)rank_ * R, G, split_send_.as<uint8_t>(), d_err,
                                          s)))
            return rc;
        // 2. all-to-all: piece h goes to rank h; rank g's piece lands at rows
        //    g*R..g*R+R-1 of the column block
        if ((rc = nccl_check(*this, ncclGroupStart(), "ncclGroupStart"))) return rc;
        for (uint32_t h = 0; h < G; h++) {
            if ((rc = nccl_check(*this,
                                 ncclSend(split_send_.as<uint8_t>() + h * piece, piece, ncclUint8, (int)h, comm, s),
                                 "ncclSend")))
                return rc;
            if ((rc = nccl_check(*this, ncclRecv(block + h * piece, piece, ncclUint8, (int)h, comm, s), "ncclRecv")))
                return rc;
        }
        if ((rc = nccl_check(*this, ncclGroupEnd(), "ncclGroupEnd"))) return rc;
    }
    // 3. columns: Q2|Q3 parity, leaves, column roots, row subtrees
    if ((rc = enqueue_split_cols(block, k, C, (uint32_t)rank_ * C, col_slots, row_sub, d_err, s))) return rc;
    // 4. gather the slots on rank 0 and reduce the push-order word
    if ((rc = nccl_check(*this, ncclGroupStart(), "ncclGroupStart"))) return rc;
    if (rank_ == 0) {
        for (uint32_t h = 0; h < G; h++) {
            if ((rc = nccl_check(*this, ncclRecv(g_sub + (size_t)h * W * kSlot, (size_t)W * kSlot, ncclUint8, (int)h,
                                                 comm, s),
                                 "ncclRecv")))
                return rc;
            if ((rc = nccl_check(*this, ncclRecv(g_col + (size_t)h * C * kSlot, (size_t)C * kSlot, ncclUint8, (int)h,
                                                 comm, s),
                                 "ncclRecv")))
                return rc;
        }
    }
    if ((rc = nccl_check(*this, ncclSend(row_sub, (size_t)W * kSlot, ncclUint8, 0, comm, s), "ncclSend"))) return rc;
    if ((rc = nccl_check(*this, ncclSend(col_slots, (size_t)C * kSlot, ncclUint8, 0, comm, s), "ncclSend"))) return rc;
    if ((rc = nccl_check(*this, ncclGroupEnd(), "ncclGroupEnd"))) return rc;
    if ((rc = nccl_check(*this, ncclReduce(d_err, d_err, 1, ncclUint32, ncclMin, 0, comm, s), "ncclReduce")))
        return rc;
    // 5. rank 0: top log2(G) levels of every row tree, roots, data root
    if (rank_ == 0) return enqueue_split_combine(g_sub, G, k, g_col, d_row_roots, d_col_roots, d_root, s);
    return CDA_OK;
}

}  // namespace cda
