// engine.h -- device runtime behind the C ABI: one context per GPU, owning a
// HIP stream, the GF(2^16) tables and grow-only scratch buffers, and the
// enqueue logic of the whole ODS -> EDS -> roots -> data-root pipeline.
#pragma once
#include "knobs.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "cda_kernels.h"
#include "square_plan.h"

namespace cda {

// Page-locks a caller's host buffer for the duration of a call (RAII), so
// its copies are plain DMA: both PCIe directions then run at once (a pageable
// copy goes through the runtime's staging and serialises with the other
// direction).  A buffer that cannot be registered -- e.g. one the caller
// registered itself -- is used as it is.  Measured: a 16-square k = 128 batch
// with its EDS returned 1 200 -> 1 880 squares/s, one square 1.25 -> 0.79 ms
// (profiles/r02_host_buffers.txt).  CDA_HOST_REGISTER=0 turns it off.
// The streams that may still copy from / to the buffer are drained before it
// is unregistered (already idle on the normal path, which synchronises).
struct HostPin {
    void* p = nullptr;
    hipStream_t s0, s1;
    HostPin(bool on, const void* q, size_t bytes, hipStream_t a, hipStream_t b) : s0(a), s1(b) {
        if (!on || !q || !bytes) return;
        // already page-locked (hipHostMalloc / registered by the caller): nothing to do
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, q) == hipSuccess && attr.type == hipMemoryTypeHost) return;
        (void)hipGetLastError();
        if (hipHostRegister(const_cast<void*>(q), bytes, hipHostRegisterDefault) == hipSuccess)
            p = const_cast<void*>(q);
        else
            (void)hipGetLastError();
    }
    ~HostPin() {
        if (!p) return;
        (void)hipStreamSynchronize(s0);
        (void)hipStreamSynchronize(s1);
        (void)hipHostUnregister(p);
    }
    HostPin(const HostPin&) = delete;
    HostPin& operator=(const HostPin&) = delete;
};


// square.hip: writes n_shares shares of a square::Plan / CommitPlan layout.
// hint (optional): segment index of every kHintShares-th share.
hipError_t launch_share_writer(const square::Segment* segs, uint32_t n_segs, const uint32_t* hint,
                               const uint8_t* compact, const uint8_t* txs, uint8_t* ods, uint32_t n_shares,
                               hipStream_t s);

// Device scratch that only grows.  Inside a context call (between
// Engine::order_begin and order_end) growth is stream-ordered: the old buffer
// is released with hipFreeAsync on the call's stream -- which already waits
// for every earlier call of the context -- and the new one comes from
// hipMallocAsync on it, so device entry points stay enqueue-only (no device
// synchronisation).  Outside a call (context set-up) plain hipMalloc / hipFree.
// A pooled buffer is usable in the call stream's order only: a host-side copy
// into it (hipMemcpy on the null stream) is not ordered after the allocation,
// so buffers filled from the host once (tables, preset words) use
// ensure_fixed (plain hipMalloc, never pooled).
// release(): inside a call, stream-ordered on the call's stream; outside a
// call (destructors) the owner first drains every stream that may still use
// the buffer (Engine::drain), then frees.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    bool pooled = false;   // allocated by hipMallocAsync
    hipError_t ensure(size_t n);
    hipError_t ensure_fixed(size_t n);
    void release();
    template <class T>
    T* as() const { return reinterpret_cast<T*>(ptr); }
};

// commit.hip: RFC-6962 root (merkle.HashFromByteSlices) of each set of 96-B
// node slots: set b = slots [bt[b], bt[b+1]) (bt in device memory, n_sets + 1
// entries, at most max_n per set); dig = scratch, 8 words per slot.
hipError_t launch_slot_merkle_roots(const uint8_t* slots, const uint32_t* bt, uint32_t n_sets, uint32_t n_slots,
                                    uint32_t max_n, uint32_t* dig, uint8_t* out, hipStream_t s);

// A square kept in HBM after extension (proof.hip): the EDS, every level of
// every row tree (level 0 = the W x W leaf slots, level L = [W][W >> L] 96-B
// slots), the roots and all RFC-6962 levels of the data-root tree.
struct ResidentSquare {
    enum Part { kRowRoots, kColRoots, kDataRoot, kEds };
    uint32_t k = 0, log_w = 0, push_err = 0xFFFFFFFFu;
    DevBuf eds, levels, col_a, col_b, roots_slots, rfc, rows, cols, root, err, scratch, pieces;
    uint64_t level_offset(uint32_t L) const;
    ~ResidentSquare();
};
// One copy out of a resident square (byte offsets into the named buffer).
struct GatherPiece {
    enum Buf : uint32_t { kEds = 0, kLevels = 1, kRfc = 2, kRows = 3, kRootSlots = 4 };
    uint32_t buf;
    uint64_t src, dst;
    uint32_t len;
};

// comm.hip: ncclGetUniqueId into 128 bytes (CDA_OK / CDA_ERR_DEVICE).
int comm_unique_id(uint8_t* id);

class Engine {
  public:
    explicit Engine(int device);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    int init();                        // CDA_OK or CDA_ERR_*
    std::mutex& mutex() { return mu_; }
    const std::string& last_error() const { return err_; }
    void clear_error() { err_.clear(); }
    int fail(int code, const std::string& msg) { err_ = msg; return code; }
    hipStream_t stream() const { return stream_; }
    int device() const { return device_; }

    // Scratch ordering.  The context's scratch buffers (leaf/level slots,
    // digests, error words, staging) are shared by every call, and a device
    // entry point only enqueues on the caller's stream.  Each call therefore
    // starts with order_begin(s) -- s waits for the GPU work of the previous
    // call, whatever stream it ran on -- and ends with order_end(s), which
    // records that point.  The mutex orders the enqueues, the event orders the
    // GPU work, so two calls on two streams never touch the scratch at once.
    // order_begin returns CDA_OK, or CDA_ERR_DEVICE when the previous call's
    // work can be neither waited for on s nor on the host.
    int order_begin(hipStream_t s);
    void order_end(hipStream_t s);
    // Wait on the host until every stream the context owns (stream_, the copy,
    // hash-split, pipeline and CU-mask streams) is idle.  Called after a failed
    // call: a call joins its side streams back to the call stream only on its
    // success path, and an early error return would otherwise leave side-stream
    // work that reads the scratch unordered before the next call's
    // stream-ordered frees.  Returns the first error.
    int drain_streams();
    // drain_streams + the last call's end on the caller's stream (order_ev_):
    // nothing of the context runs any more (destructors, resident squares).
    int drain();
    // The last call's end on the caller's stream only (order_ev_): every call
    // joins its side streams on success and a failed call drained them
    // (capi.hip guarded), so this covers all GPU work any call queued.
    int wait_last_call();
    // Test build only (CDA_FAULT, read at init by libcda_test.so; knobs.h): an injected error at a named point
    // after GPU work was enqueued -- "dah_part" (enqueue_dah's side part, after
    // its leaves and levels), "pipe_chunk" (host_pipeline, after chunk 1's
    // compute), "extend_chunk" (the RS pipeline, after chunk 0's RS).  Fires
    // once per context, so the follow-up calls of a test run clean.
    bool fault_at(const char* where) {
        if (!kTestBuild || fault_.empty() || fault_ != where) return false;
        fault_.clear();
        return true;
    }
    // n push-order error words of a device entry point (context scratch), or
    // NULL when the allocation fails.
    uint32_t* err_words(uint32_t n) {
        void* before = dev_err_.ptr;
        if (dev_err_.ensure((size_t)n * 4) != hipSuccess) {
            dev_err_n_ = 0;
            return nullptr;
        }
        if (dev_err_.ptr != before) dev_err_n_ = 0;   // a regrown buffer holds no batch's words
        return dev_err_.as<uint32_t>();
    }
    // The push-order words belong to the last device batch of n squares
    // (cda_extend_dah_device / _inplace_device): device_push_order_detail
    // reads square sq's word after that batch's work completed.
    // n = 0: the last device batch failed to enqueue (no words to read)
    void set_device_batch(uint32_t n) { dev_err_n_ = n; }
    int device_push_order_detail(uint32_t sq, int32_t* axis, uint32_t* index, uint32_t* pos);

    // Enqueue the full path for n squares of width k (device pointers).
    // d_err: n u32 words (min-encoded push-order violation, ~0 = ordered);
    // d_status (optional): n int32 CDA_OK / CDA_ERR_PUSH_ORDER.
    int enqueue_extend_dah(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds, uint8_t* d_rows,
                           uint8_t* d_cols, uint8_t* d_roots, uint32_t* d_err, int32_t* d_status, hipStream_t s);
    // Size the device batch calls' scratch for n squares of width k, so later
    // calls up to that size never grow (and synchronise) a buffer.
    int reserve(uint32_t k, uint32_t n);
    // RS extension only (ExtendShares).
    // err_init (optional): n push-order words set to ~0 by the first RS launch.
    int enqueue_extend(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds, hipStream_t s,
                       uint32_t* err_init = nullptr);
    // Roots + data root of existing EDSs.
    // err_ready: d_err already holds ~0 words (enqueue_extend's err_init).
    int enqueue_dah(const uint8_t* d_eds, uint32_t k, uint32_t n, uint8_t* d_rows, uint8_t* d_cols, uint8_t* d_roots,
                    uint32_t* d_err, int32_t* d_status, hipStream_t s, bool err_ready = false);
    int enqueue_rs(const uint8_t* d_data, uint8_t* d_parity, uint32_t k, uint32_t len, uint32_t n, hipStream_t s);

    // Config 5: one square split across ranks (cda_split_* in include/cda.h).
    int enqueue_split_rows(const uint8_t* d_rows, uint32_t k, uint32_t n_rows, uint32_t row0, uint8_t* d_block,
                           uint32_t* d_err, hipStream_t s);
    int enqueue_split_cols(uint8_t* d_block, uint32_t k, uint32_t n_cols, uint32_t col0, uint8_t* d_col_slots,
                           uint8_t* d_row_sub, uint32_t* d_err, hipStream_t s);
    int enqueue_split_combine(const uint8_t* d_row_sub, uint32_t parts, uint32_t k, const uint8_t* d_col_slots,
                              uint8_t* d_rows, uint8_t* d_cols, uint8_t* d_root, hipStream_t s);

    // Config 5 inside the library (comm.hip): the row block written straight
    // into the all-to-all send layout [parts][R][C][512], an RCCL
    // communicator per context, and the whole split on the caller's stream.
    int enqueue_split_rows_send(const uint8_t* d_rows, uint32_t k, uint32_t n_rows, uint32_t row0, uint32_t parts,
                                uint8_t* d_send, uint32_t* d_err, hipStream_t s);
    int comm_init(int rank, int world, const uint8_t* id);
    void comm_destroy();
    int comm_size(int* rank, int* world);   // ncclCommUserRank / ncclCommCount of the live communicator
    int comm_abort();   // ncclCommAbort (e.g. from a host watchdog after a peer failed)
    int comm_rank() const { return rank_; }
    int split_extend_dah(const uint8_t* d_rows, uint32_t k, uint8_t* d_col_block, uint8_t* d_row_roots,
                         uint8_t* d_col_roots, uint8_t* d_root, uint32_t* d_err, hipStream_t s);

    // Host-buffer helpers (copy in, run, copy out, synchronise).
    // eds_mode (include/cda.h CDA_EDS_*): the whole EDS with Q0 copied on the
    // host (FULL), the whole EDS without Q0 (SKIP_Q0: the caller's Q0 cells
    // alias its shares), or packed parity [n][Q1 k x k | rows k..2k-1] (PARITY).
    int host_extend_dah(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, uint8_t* rows, uint8_t* cols,
                        uint8_t* roots, int32_t* status, int eds_mode = 0);
    int host_extend(const uint8_t* ods, uint32_t k, uint8_t* eds);
    int host_dah(const uint8_t* eds, uint32_t k, uint8_t* rows, uint8_t* cols, uint8_t* root);
    int host_rs(const uint8_t* data, uint32_t k, uint32_t len, uint32_t n, uint8_t* parity);
    int host_data_root(const uint8_t* rows, const uint8_t* cols, uint32_t w, uint8_t* root);

    // Square construction (square.hip): the layout is planned on the host
    // (square_plan.cpp), the shares are written on the device.
    // d_txs: the transaction bytes the plan's offsets refer to, with >= 16
    // bytes of readable slack after the end.
    int enqueue_square(const square::Plan& p, const uint8_t* d_txs, uint8_t* d_ods, hipStream_t s);
    int host_square(const square::Plan& p, const uint8_t* txs, size_t txs_len, uint8_t* ods);
    int host_construct_extend_dah(const square::Plan& p, const uint8_t* txs, size_t txs_len, uint8_t* eds,
                                  uint8_t* rows, uint8_t* cols, uint8_t* root);

    // Blob share commitments (commit.hip).  d_data: blob bytes the plan's
    // offsets refer to (>= 16 readable bytes of slack); d_out: n_blobs * 32.
    // Host plan reused by every commitment call (its vectors keep their
    // capacity; the engine mutex serialises callers).
    square::CommitPlan& commit_plan() { return cm_host_plan_; }
    int enqueue_commitments(const square::CommitPlan& p, uint32_t n_blobs, const uint8_t* d_data, uint8_t* d_out,
                            hipStream_t s);
    int host_commitments(const square::CommitPlan& p, uint32_t n_blobs, const uint8_t* data, size_t data_len,
                         uint8_t* out);

    // Resident squares and proofs (proof.hip).
    int square_create(const uint8_t* ods, uint32_t k, ResidentSquare* sq);
    int square_gather(ResidentSquare* sq, const std::vector<GatherPiece>& pieces, uint8_t* out, size_t out_len);
    int square_gather_device(ResidentSquare* sq, const std::vector<GatherPiece>& pieces, size_t out_len);
    int square_read(ResidentSquare* sq, ResidentSquare::Part part, uint8_t* out);   // synchronous D2H
    struct ShareProofOut {
        uint8_t* shares;
        uint32_t start_row, end_row;
        int32_t* nmt_start;
        int32_t* nmt_end;
        uint32_t* nmt_count;
        uint8_t* nmt_nodes;       // [rows][2 log2(2k)][90]
        uint8_t* row_roots;       // [rows][90]
        uint8_t* row_leaf_hash;   // [rows][32]
        uint8_t* row_aunts;       // [rows][log2(4k)][32]
    };
    int square_share_proof(ResidentSquare* sq, uint32_t start, uint32_t end, ShareProofOut* out);
    int square_subtree_root(ResidentSquare* sq, uint32_t row, const uint8_t* walk, uint32_t walk_len, uint8_t* out);
    int square_blob_commitments(ResidentSquare* sq, const uint32_t* starts, const uint32_t* lens, uint32_t n,
                                uint32_t threshold, uint8_t* out);

    // Repair (repair.hip): rsmt2d ExtendedDataSquare.Repair and Codec.Decode.
    int host_repair(uint8_t* eds, const uint8_t* present, uint32_t w, const uint8_t* row_roots,
                    const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index);
    int device_repair(uint8_t* d_eds, const uint8_t* present, uint32_t w, const uint8_t* row_roots,
                      const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index);
    int repair(uint8_t* eds, uint8_t* d_eds, const uint8_t* present, uint32_t w, const uint8_t* row_roots,
               const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index);
    int host_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t k, uint32_t shard_len, uint32_t n_codewords);

    // Standalone erasured NMT trees and generic RFC-6962 roots (tree.hip).
    int nmt_axis_roots(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees,
                       uint32_t square_size, const uint32_t* axis, uint8_t* roots, int32_t* status);
    int nmt_prove_range(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                        uint32_t axis, uint32_t start, uint32_t end, uint8_t* nodes, uint32_t* n_nodes,
                        uint8_t* root);
    int merkle_root(const uint8_t* items, const uint64_t* off, uint32_t n, uint8_t* out);

    // Stage timing with HIP events on the launch stream (bench / profiling).
    enum Stage { kStageRsQ0 = 0, kStageRsQ3, kStageOrder, kStageLeaves, kStageLevels, kStageDataRoot, kNumStages };
    void set_profiling(bool on) { profiling_ = on; }
    int collect_stage_times(double* ms, uint32_t* counts, int n);

    uint32_t dev_err_n_ = 0;   // squares of the last device batch (their push-order words in dev_err_)
    int32_t po_axis = -1;
    uint32_t po_index = 0, po_pos = 0;

  private:
    int check(hipError_t e, const char* what);
    // stages enqueued since the context's work was last seen complete (for
    // attributing asynchronous device faults; see check())
    static constexpr size_t kMaxPending = 48;
    std::vector<const char*> pending_;
    bool sync_check_ = false;   // CDA_SYNC_CHECK: synchronise after every stage
    void note_stage(const char* what);
    std::string pending_stages() const;
    // levels of the forests down to `stop` nodes per tree (f[i].in then
    // describes that level); stop = 1 runs them all
    // (subtrees: the first levels may run as one fused subtree launch, after
    // which the ping-pong parity no longer follows the level count -- only for
    // callers that take f[i].in as it comes back)
    int run_forests(Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n, uint8_t* bufA, uint8_t* bufB,
                    uint64_t buf_sq, const uint64_t* out_off, hipStream_t s, uint32_t stop = 1,
                    bool subtrees = false);
    int subtree_min_ = 8;   // CDA_SUBTREE: fused subtree levels of >= this many leaves (0 = off)
    uint64_t subtree_lanes_ = 0;   // CDA_SUBTREE_LANES: lanes a subtree launch must hold (0 = by tree size)
    uint32_t rs16_prio_max_ = 4;   // CDA_RS16_PRIO_MAX: squares per launch up to which RsJob::prio is set (k >= 256)
    bool rs8_prio_ = true;         // CDA_RS8_PRIO=0: no RsJob::prio for the GF(2^8) bitsliced encoder
    uint32_t top_fuse_nodes(uint32_t W, uint32_t n, bool* wide = nullptr) const;
    int top_fuse_ = -1;   // CDA_TOP_FUSE (tuning / A-B): -1 auto, 0 off, N = nodes per tree
    int top_wide_ = 2;    // CDA_TOP_WIDE: levels the tree top absorbs below the lane-pair level
    int push_order_error(const uint32_t* err_words, uint32_t n, const uint8_t* host_q0_src, uint32_t k,
                         bool src_is_eds);
    std::string fault_;   // CDA_FAULT (tests only)

    struct Mark {
        int stage;
        hipEvent_t a, b;
    };
    void mark_begin(int stage, hipStream_t s);
    void mark_end(hipStream_t s);
    bool profiling_ = false;
    std::vector<Mark> marks_;
    std::vector<hipEvent_t> event_pool_;
    double stage_ms_[kNumStages] = {};
    uint32_t stage_n_[kNumStages] = {};
    hipEvent_t take_event();

    int device_;
    hipStream_t stream_ = nullptr;
    // host-buffer calls: device-to-host copies of the parity quadrants run on
    // copy_out_ while stream_ hashes (ev_rs_: RS done, ev_out_: copies done)
    hipStream_t copy_out_ = nullptr;
    hipEvent_t ev_rs_ = nullptr, ev_out_ = nullptr;
    // eds_mode PARITY: d_par = device staging of n packed parity squares
    int enqueue_parity_d2h(const uint8_t* d_eds, uint32_t k, uint32_t n, uint8_t* eds, hipStream_t from,
                           hipEvent_t ready, hipEvent_t done, int eds_mode = 0, uint8_t* d_par = nullptr);
    // Big host-buffer batches (host_extend_dah, n > 2 chunks): chunks of
    // squares through a ring of kPipeSlots device slots, H2D on copy_in_,
    // extension + hashing on stream_, parity D2H on copy_out_, so chunk i+1
    // goes up while chunk i computes and chunk i-1 comes down.
    static constexpr uint32_t kPipeSlots = 3;
    hipStream_t copy_in_ = nullptr;
    hipEvent_t pipe_in_[kPipeSlots] = {}, pipe_rs_[kPipeSlots] = {}, pipe_d2h_[kPipeSlots] = {},
               pipe_comp_[kPipeSlots] = {};
    uint32_t host_pipe_chunk_ = 0;   // CDA_HOST_PIPE_CHUNK: squares per chunk (0 = auto: ~256 MiB of ODS)
    int host_pipeline(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, uint8_t* rows, uint8_t* cols,
                      uint8_t* roots, int32_t* status, uint32_t chunk, int eds_mode);
    DevBuf h_par_;   // packed-parity staging (eds_mode PARITY)
    static void copy_q0(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds);
    hipEvent_t order_ev_ = nullptr;   // end of the last call's GPU work
    bool order_used_ = false;
    // Second stream of a call: half of a batch's hash stages (enqueue_dah), or
    // the batch pipeline's RS chunks (enqueue_extend_dah, CDA_PIPELINE_CHUNK).
    hipStream_t aux_stream_ = nullptr;
    std::vector<hipEvent_t> sync_events_;
    uint32_t pipeline_chunk_ = 0;   // squares per chunk (0 = auto)
    int hash_split_ = -1;           // CDA_HASH_SPLIT: hash the batch in this many parts on as many streams (0/1 = off, -1 = auto)
    static constexpr uint32_t kMaxHashParts = 4;
    uint32_t host_chunk_ = 4;       // CDA_HOST_CHUNK: squares per H2D/RS/D2H chunk of a host-buffer batch
    bool host_full_d2h_ = false;    // CDA_HOST_FULL_D2H: EDS back as one contiguous copy (no host Q0 copy)
    bool host_register_ = true;     // CDA_HOST_REGISTER: page-lock the caller's buffers for the call (0 = off)
    hipStream_t split_streams_[kMaxHashParts - 2] = {};
    // CDA_RS_CUS=N (batch pipeline): chunk i > 0's RS on a stream masked to N
    // CUs, the chunks' hashing on the complement (no CU runs both kernels:
    // their instruction streams slow each other down on a shared SIMD)
    uint32_t rs_cus_ = 0;
    hipStream_t rs_cu_stream_ = nullptr, hash_cu_stream_ = nullptr;
    int make_cu_streams();
    int split_stream(uint32_t i, hipStream_t* out);
    hipEvent_t sync_event(size_t i);
    int dah_prepare(uint32_t W, uint32_t n, uint32_t* d_err, hipStream_t s);
    void dah_forests(uint32_t W, uint8_t* d_rows, uint8_t* d_cols, Forest (&f)[2]);
    int dah_chunk(const uint8_t* d_eds, uint32_t k, uint32_t i0, uint32_t m, uint32_t stop, uint32_t* d_err,
                  const Forest (&f)[2], Forest (&post)[2], hipStream_t s, bool subtrees = false);
    int dah_finish(uint32_t k, uint32_t i0, uint32_t n, uint32_t from, const Forest (&f)[2], uint8_t* d_roots,
                   uint32_t* d_err, int32_t* d_status, hipStream_t s);
    int enqueue_extend_dah_serial(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds, uint8_t* d_rows,
                                  uint8_t* d_cols, uint8_t* d_roots, uint32_t* d_err, int32_t* d_status,
                                  hipStream_t s);
    std::mutex mu_;
    std::string err_;
    DevBuf gf16_log_, gf16_exp_, gf16_skew_;
    Gf16Dev gf16(uint32_t k) const;
    DevBuf leaf_, lvl_, root_slots_, dig_, err_buf_, dev_err_;
    DevBuf h_ods_, h_eds_, h_rows_, h_cols_, h_roots_;   // device staging for host-buffer calls
    // square construction: device plan (segments + compact shares), device
    // copy of host txs, pinned staging for the plan and its copy-done event
    DevBuf sq_plan_, sq_txs_;
    DevBuf cm_plan_, cm_tables_, cm_leaf_, cm_lvl_, cm_roots_, cm_out_;   // commitments
    square::CommitPlan cm_host_plan_;
    std::vector<uint32_t> cm_groups_;   // commitment blob groups (host side)
    void* sq_stage_ = nullptr;
    size_t sq_stage_bytes_ = 0;
    hipEvent_t sq_event_ = nullptr;
    int upload_txs(const uint8_t* txs, size_t len, hipStream_t s);
    // repair: GF(2^8) tables (GF(2^16) ones are shared with the encoder),
    // codeword list, error locators, presence map, parity check scratch
    DevBuf gf8_log_, gf8_exp_, gf8_skew_, rp_cw_, rp_err_, rp_present_, rp_parity_, rp_buf_, rp_flags_;
    // pinned staging of repair's small uploads (presence map, codeword lists):
    // copies stay asynchronous; the cursor restarts after a stream sync
    void* rp_host_ = nullptr;
    size_t rp_host_bytes_ = 0, rp_host_used_ = 0;
    void* rp_out_ = nullptr;   // pinned landing area of repair_verify's results
    size_t rp_out_bytes_ = 0;
    uint8_t* rp_stage(const void* src, size_t n, hipStream_t s, int* rc);
    std::vector<uint8_t> rp_roots_;
    // standalone trees: host cells, all tree levels, axis indexes / error words, roots
    DevBuf tr_cells_, tr_levels_, tr_axis_, tr_roots_;
    DevBuf rs_pad_;   // Codec.Encode of a non-power-of-two shard count
    // config 5 in the library: RCCL communicator (ncclComm_t), row block,
    // send buffer, column block, slots
    // comm_mu_ guards comm_ and every non-blocking RCCL post; cda_comm_abort
    // takes comm_ under it, so no post touches an aborted communicator, while
    // the blocking calls (ncclGroupEnd, stream syncs) run unlocked and re-read
    // comm_ after they return (comm.hip).
    void* comm_ = nullptr;
    std::mutex comm_mu_;
    int rank_ = 0, world_ = 0;
    uint32_t comm_k_ = 0;   // k whose split scratch every rank agreed on (0 = none yet)
    // comm_flag_: the agreement round's words, allocated by comm_init: [0] = 0,
    // [1] = 1 (the all-reduce sends one of them, so nothing can fail before
    // it), [2] = the MIN result
    DevBuf split_blk_, split_send_, split_col_, split_slots_, comm_flag_;
    int comm_fail(const char* what, int nccl_result);
    void* take_comm();   // comm_ = nullptr under comm_mu_; returns the old value
    bool comm_alive();
    int comm_group(const char* what, const std::function<int(void*)>& post);
    int build_trees(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees, uint32_t square_size,
                    const uint32_t* axis, std::vector<uint64_t>* level_off, std::vector<uint32_t>* err_out);
    int tree_order_error(const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                         const uint32_t* axis, const std::vector<uint32_t>& err, int32_t* status);   // roots of the last repair_verify (rows then columns)
    int ensure_gf8_tables();
    int repair_verify(const uint8_t* d_eds, uint32_t k, const uint8_t* row_roots, const uint8_t* col_roots,
                      std::vector<uint8_t>& bad, hipStream_t s);
    // Leopard decode of codewords (axis, index pairs) of a grid of 2k x 2k
    // cells of shard_len bytes; marks them present.
    int decode_codewords(uint8_t* d_cells, uint8_t* d_present, uint32_t k, uint32_t shard_len,
                         const std::vector<uint32_t>& axis_index, hipStream_t s);
};

}  // namespace cda
