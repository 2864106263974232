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
#include "knobs.h"
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"
#include "split_layout.h"

namespace cda {

namespace {

// [R][W] row block -> [G][R][C] send layout (SplitLayout::send_off): one
// thread per 16 bytes.
__global__ __launch_bounds__(256) void group_rows_kernel(const uint4* __restrict__ src, uint8_t* __restrict__ dst,
                                                        const SplitLayout L) {
    constexpr uint32_t V = kShare / 16;   // uint4 per share
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint64_t)L.R * L.W * V) return;
    const uint32_t v = (uint32_t)(i % V);
    const uint64_t cell = i / V;
    const uint32_t r = (uint32_t)(cell / L.W), col = (uint32_t)(cell % L.W);
    reinterpret_cast<uint4*>(dst + L.send_off(r, col))[v] = src[i];
}

// CDA_COMM_FAULT (tests only, read at every split call): make one step fail
// as if RCCL or the device had failed there -- "a2a" (the all-to-all group),
// "gather" (the gather group), "local" (this rank's column stage), "alloc"
// (this rank's scratch allocation in the agreement round).  Lets the GPU
// tests drive every error path at world size 1.
bool comm_fault(const char* where) {
    const char* e = test_knob("CDA_COMM_FAULT");
    return e && strcmp(e, where) == 0;
}

}  // namespace

int Engine::enqueue_split_rows_send(const uint8_t* d_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                                    uint32_t parts, uint8_t* d_send, uint32_t* d_err, hipStream_t s) {
    const uint32_t W = 2 * k;
    if (parts == 0 || (parts & (parts - 1)) || parts > W || n_rows == 0)
        return fail(CDA_ERR_INVALID, "bad split: parts must be a power of two <= 2k");
    int rc;
    if (parts == 1) return enqueue_split_rows(d_rows, k, n_rows, row0, d_send, d_err, s);   // [1][R][W] = [R][W]
    if ((rc = check(split_blk_.ensure((size_t)n_rows * W * kShare), "hipMalloc row block"))) return rc;
    if ((rc = enqueue_split_rows(d_rows, k, n_rows, row0, split_blk_.as<uint8_t>(), d_err, s))) return rc;
    // the layout of a split into `parts` column groups, with this call's row
    // count (cda_split_rows_send callers may pass any R)
    SplitLayout L(k, parts);
    L.R = n_rows;
    const uint64_t n16 = (uint64_t)n_rows * W * (kShare / 16);
    hipLaunchKernelGGL(group_rows_kernel, dim3((uint32_t)((n16 + 255) / 256)), dim3(256), 0, s,
                       split_blk_.as<uint4>(), d_send, L);
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
    comm_destroy();
    // the agreement round's words (split_extend_dah): preset 0 and 1, so the
    // all-reduce needs no copy that could fail before it
    int rc;
    if ((rc = check(comm_flag_.ensure_fixed(16), "hipMalloc agreement words"))) return rc;
    const int32_t preset[4] = {0, 1, 0, 0};
    if ((rc = check(hipMemcpy(comm_flag_.ptr, preset, sizeof preset, hipMemcpyHostToDevice), "hipMemcpy agreement words")))
        return rc;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRank(&c, world, uid, rank);
    if (r != ncclSuccess) return fail(CDA_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    {
        std::lock_guard<std::mutex> g(comm_mu_);
        comm_ = c;
    }
    rank_ = rank;
    world_ = world;
    comm_k_ = 0;
    return CDA_OK;
}

// cda_comm_abort may run on a watchdog thread while another thread is inside
// split_extend_dah.  comm_ changes only under comm_mu_, every RCCL post (group
// start, send / recv / reduce) runs under it after re-reading comm_, and the
// blocking steps (ncclGroupEnd -- it may wait for peers while it connects --
// and stream syncs) run unlocked and re-read comm_ when they return.  So a
// post never sees a freed communicator, and an abort during a blocking step
// releases it (ncclCommAbort stops the queued collectives) and the call
// returns CDA_ERR_COMM without touching the communicator again.
void* Engine::take_comm() {
    std::lock_guard<std::mutex> g(comm_mu_);
    void* c = comm_;
    comm_ = nullptr;
    return c;
}

bool Engine::comm_alive() {
    std::lock_guard<std::mutex> g(comm_mu_);
    return comm_ != nullptr;
}

void Engine::comm_destroy() {
    if (void* c = take_comm()) (void)ncclCommDestroy(static_cast<ncclComm_t>(c));
    rank_ = 0;
    world_ = 0;
    comm_k_ = 0;
}

// An RCCL call failed: the communicator may hold half-posted operations, so it
// is aborted (ncclCommAbort also stops this rank's queued collective kernels)
// and released.  Peers blocked in the same collective are released by their
// own host calling cda_comm_abort (e.g. on a timeout), as NCCL prescribes.
int Engine::comm_fail(const char* what, int result) {
    std::string msg = std::string(what) + ": " + ncclGetErrorString(static_cast<ncclResult_t>(result)) +
                      " (communicator aborted; every rank must call cda_comm_init again)";
    if (void* c = take_comm()) (void)ncclCommAbort(static_cast<ncclComm_t>(c));
    rank_ = 0;
    world_ = 0;
    comm_k_ = 0;
    return fail(CDA_ERR_COMM, msg);
}

// The communicator's own view (ncclCommUserRank / ncclCommCount), so a host
// can report the world size RCCL actually formed.
int Engine::comm_size(int* rank, int* world) {
    std::lock_guard<std::mutex> g(comm_mu_);
    if (!comm_) return fail(CDA_ERR_INVALID, "no communicator: call cda_comm_init first");
    ncclComm_t c = static_cast<ncclComm_t>(comm_);
    ncclResult_t r = ncclCommCount(c, world);
    if (r == ncclSuccess) r = ncclCommUserRank(c, rank);
    if (r != ncclSuccess) return fail(CDA_ERR_COMM, std::string("ncclCommCount: ") + ncclGetErrorString(r));
    return CDA_OK;
}

int Engine::comm_abort() {
    if (void* c = take_comm()) (void)ncclCommAbort(static_cast<ncclComm_t>(c));
    return CDA_OK;
}

static int aborted(Engine& e, const char* what) {
    return e.fail(CDA_ERR_COMM, std::string(what) + ": the communicator was aborted during the call (cda_comm_abort)");
}

// One RCCL group: the posts under comm_mu_, ncclGroupEnd unlocked.  A group
// is always closed, even after a failed post.
int Engine::comm_group(const char* what, const std::function<int(void*)>& post) {
    ncclResult_t first;
    bool opened = false;
    {
        std::lock_guard<std::mutex> g(comm_mu_);
        if (!comm_) return aborted(*this, what);
        first = ncclGroupStart();
        if (first == ncclSuccess) {
            opened = true;
            first = static_cast<ncclResult_t>(post(comm_));
        }
    }
    const ncclResult_t end = opened ? ncclGroupEnd() : ncclSuccess;
    if (!comm_alive()) return aborted(*this, what);
    if (first != ncclSuccess) return comm_fail(what, first);
    if (end != ncclSuccess) return comm_fail(what, end);
    return CDA_OK;
}

// Config 5 on this rank.  Error discipline (every rank must leave every
// collective it entered, or its peers block forever):
//   * checks that depend only on k and the world size fail on every rank alike
//     before any collective;
//   * scratch is allocated when k changes, followed by one agreement
//     all-reduce (MIN of an ok flag -- one of two preset device words, so no
//     copy precedes it -- read back on the host): if any rank could not
//     allocate, every rank returns CDA_ERR_OOM and the communicator stays
//     usable;
//   * a local failure after that (a kernel launch, bad per-rank buffers) does
//     not return early: the rank stops its own compute, poisons its push-order
//     word with 0 (never a valid violation word: positions start at 1), takes
//     part in the remaining collectives and returns its error at the end;
//     rank 0 reads the MIN-reduced word back, and when it is 0 (a peer
//     failed) skips the combine and returns CDA_ERR_DEVICE;
//   * an RCCL call that fails closes its group (ncclGroupEnd), aborts the
//     communicator and returns CDA_ERR_COMM; so does an abort by another
//     thread (cda_comm_abort) while the call waits in a collective.
int Engine::split_extend_dah(const uint8_t* d_rows, uint32_t k, uint8_t* d_col_block, uint8_t* d_row_roots,
                             uint8_t* d_col_roots, uint8_t* d_root, uint32_t* d_err, hipStream_t s) {
    if (!comm_alive()) return fail(CDA_ERR_INVALID, "no communicator: call cda_comm_init first");
    const uint32_t G = (uint32_t)world_, W = 2 * k;
    const SplitLayout L(k, G);   // every offset below (split_layout.h, pinned at G > 1 by a CPU replay)
    if (!L.valid()) return fail(CDA_ERR_INVALID, "world size must divide k (a power of two <= 1024)");
    const uint32_t R = L.R, C = L.C;
    const size_t piece = L.piece();   // one rank pair's all-to-all block
    int rc;
    // -- scratch + agreement (only when k changes; k is the same on every rank) --
    if (comm_k_ != k) {
        int ok = 1;
        if (comm_fault("alloc")) ok = 0;
        if (ok && G > 1 && split_send_.ensure(L.send_bytes()) != hipSuccess) ok = 0;
        if (ok && split_col_.ensure(L.col_block_bytes()) != hipSuccess) ok = 0;
        if (ok && split_slots_.ensure(L.slots_bytes()) != hipSuccess) ok = 0;
        // the column stage's leaf / level slots too, so no buffer grows (and
        // synchronises) once the collectives are queued
        if (ok && leaf_.ensure((size_t)W * C * kSlot) != hipSuccess) ok = 0;
        if (ok && lvl_.ensure((size_t)W * C * kSlot) != hipSuccess) ok = 0;
        (void)hipGetLastError();
        int32_t* words = comm_flag_.as<int32_t>();
        if ((rc = comm_group("ncclAllReduce (allocation agreement)", [&](void* c) {
                 return (int)ncclAllReduce(words + (ok ? 1 : 0), words + 2, 1, ncclInt32, ncclMin,
                                           static_cast<ncclComm_t>(c), s);
             })))
            return rc;
        int32_t h_ok = 0;
        if ((rc = check(hipMemcpyAsync(&h_ok, words + 2, 4, hipMemcpyDeviceToHost, s), "D2H agreement word"))) return rc;
        if (comm_fault("stall")) {   // tests: wait here as if a peer never arrived, until aborted
            for (int i = 0; i < 30000 && comm_alive(); i++) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        const hipError_t se = hipStreamSynchronize(s);
        if (!comm_alive()) return aborted(*this, "allocation agreement");
        if ((rc = check(se, "hipStreamSynchronize"))) return rc;
        if (!h_ok)
            return fail(CDA_ERR_OOM, ok ? "a peer rank could not allocate its split scratch"
                                        : "split scratch allocation failed on this rank");
        comm_k_ = k;
    }
    uint8_t* block = d_col_block ? d_col_block : split_col_.as<uint8_t>();
    // slots: this rank's column roots [C] and row subtrees [W]; rank 0 also
    // the gathered [G][W] subtrees and [W] column roots (rank order)
    uint8_t* slots = split_slots_.as<uint8_t>();
    uint8_t* col_slots = slots + L.col_slots_off();
    uint8_t* row_sub = slots + L.row_sub_off();
    uint8_t* g_sub = slots + L.gather_sub_off(0);            // [G][W][96]
    uint8_t* g_col = slots + L.gather_col_off(0);            // [G*C = W][96]
    // the push-order word: the caller's, or library scratch when it passed none
    uint32_t* err = d_err ? d_err : reinterpret_cast<uint32_t*>(slots + L.err_off());
    int local = CDA_OK;                                      // first local failure
    std::string local_msg;
    auto local_fail = [&](int code, const std::string& msg) {
        if (local == CDA_OK) {
            local = code;
            local_msg = msg;
        }
    };
    if (!d_rows || !d_err) local_fail(CDA_ERR_INVALID, "null buffer");
    if (rank_ == 0 && (!d_row_roots || !d_col_roots || !d_root)) local_fail(CDA_ERR_INVALID, "null buffer");
    if (hipMemsetAsync(err, local ? 0x00 : 0xFF, 4, s) != hipSuccess) return comm_fail("hipMemsetAsync", ncclUnhandledCudaError);
    // a local step: runs only while this rank is healthy; a failure poisons
    // the push-order word and keeps the rank in the collectives
    auto step = [&](auto&& f) -> bool {
        if (local != CDA_OK) return true;
        const int e = f();
        if (e == CDA_OK) return true;
        local_fail(e, last_error());
        return hipMemsetAsync(err, 0x00, 4, s) == hipSuccess;
    };
    if (G == 1) {
        // one rank: the row block IS rows 0..k-1 of the (whole) column block
        if (!step([&] { return enqueue_split_rows_send(d_rows, k, R, 0, 1, block, err, s); }))
            return comm_fail("poison", ncclUnhandledCudaError);
    } else {
        // 1. rows -> [G][R][C] send layout
        if (!step([&] {
                return enqueue_split_rows_send(d_rows, k, R, (uint32_t)rank_ * R, G, split_send_.as<uint8_t>(), err, s);
            }))
            return comm_fail("poison", ncclUnhandledCudaError);
        // 2. all-to-all: piece h goes to rank h; rank g's piece lands at rows
        //    g*R..g*R+R-1 of the column block
        if ((rc = comm_group("all-to-all", [&](void* cv) -> int {
                 if (comm_fault("a2a")) return (int)ncclInternalError;
                 ncclComm_t comm = static_cast<ncclComm_t>(cv);
                 for (uint32_t h = 0; h < G; h++) {
                     ncclResult_t q = ncclSend(split_send_.as<uint8_t>() + L.send_piece_off(h), piece, ncclUint8, (int)h,
                                               comm, s);
                     if (q != ncclSuccess) return (int)q;
                     if ((q = ncclRecv(block + L.recv_piece_off(h), piece, ncclUint8, (int)h, comm, s)) != ncclSuccess)
                         return (int)q;
                 }
                 return (int)ncclSuccess;
             })))
            return rc;
    }
    // 3. columns: Q2|Q3 parity, leaves, column roots, row subtrees
    if (!step([&] {
            if (comm_fault("local")) return fail(CDA_ERR_DEVICE, "column stage: injected fault (CDA_COMM_FAULT=local)");
            return enqueue_split_cols(block, k, C, (uint32_t)rank_ * C, col_slots, row_sub, err, s);
        }))
        return comm_fail("poison", ncclUnhandledCudaError);
    if (comm_fault("peer") && hipMemsetAsync(err, 0x00, 4, s) != hipSuccess)   // tests: as if a peer had failed
        return comm_fail("poison", ncclUnhandledCudaError);
    // 4. gather the slots on rank 0 and reduce the push-order word
    if ((rc = comm_group("gather", [&](void* cv) -> int {
             if (comm_fault("gather")) return (int)ncclInternalError;
             ncclComm_t comm = static_cast<ncclComm_t>(cv);
             ncclResult_t q;
             if (rank_ == 0) {
                 for (uint32_t h = 0; h < G; h++) {
                     if ((q = ncclRecv(slots + L.gather_sub_off(h), (size_t)W * kSlot, ncclUint8, (int)h, comm, s)) !=
                         ncclSuccess)
                         return (int)q;
                     if ((q = ncclRecv(slots + L.gather_col_off(h), (size_t)C * kSlot, ncclUint8, (int)h, comm, s)) !=
                         ncclSuccess)
                         return (int)q;
                 }
             }
             if ((q = ncclSend(row_sub, (size_t)W * kSlot, ncclUint8, 0, comm, s)) != ncclSuccess) return (int)q;
             return (int)ncclSend(col_slots, (size_t)C * kSlot, ncclUint8, 0, comm, s);
         })))
        return rc;
    if ((rc = comm_group("ncclReduce", [&](void* cv) {
             return (int)ncclReduce(err, err, 1, ncclUint32, ncclMin, 0, static_cast<ncclComm_t>(cv), s);
         })))
        return rc;
    if (local != CDA_OK) return fail(local, local_msg);
    if (rank_ != 0) return CDA_OK;
    // 5. rank 0: a peer that failed left 0 in the reduced word -- nothing valid
    //    to combine; otherwise the top log2(G) levels of every row tree, the
    //    roots and the data root
    uint32_t word = 0;
    if ((rc = check(hipMemcpyAsync(&word, err, 4, hipMemcpyDeviceToHost, s), "D2H push-order word"))) return rc;
    const hipError_t se = hipStreamSynchronize(s);
    if (!comm_alive()) return aborted(*this, "ncclReduce");
    if ((rc = check(se, "hipStreamSynchronize"))) return rc;
    if (word == 0)
        return fail(CDA_ERR_DEVICE,
                    "a peer rank failed its local stage (MIN-reduced push-order word 0): roots not written");
    return enqueue_split_combine(g_sub, G, k, g_col, d_row_roots, d_col_roots, d_root, s);
}

}  // namespace cda
