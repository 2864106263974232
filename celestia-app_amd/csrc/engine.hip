// engine.hip -- implementation of cda::Engine (see engine.h).
//
// Pipeline per batch of n squares of width k (W = 2k), all on one stream:
//   1. RS phase Q0: rows Q0->Q1 (+ Q0 copy into the EDS) and columns Q0->Q2
//   2. RS phase Q3: rows Q2->Q3                     (rsmt2d erasureExtendSquare)
//   3. leaf hashing, one per EDS cell               (NmtHasher.HashLeaf), fused
//      with the Q0 namespace push-order check       (nmt Push, ErrInvalidPushOrder)
//   4. log2(W) NMT levels over all 2W trees         (NmtHasher.HashNode)
//   5. RFC-6962 data root                           (DataAvailabilityHeader.Hash)
#include "knobs.h"
#include "engine.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include "../../include/cda.h"
#include "leopard_tables.h"
#include "sha256_dev.h"
#include "split_layout.h"

namespace cda {

// the stream of the context call running on this thread (order_begin / order_end)
static thread_local bool tl_in_call = false;
static thread_local hipStream_t tl_call_stream = nullptr;

hipError_t DevBuf::ensure(size_t n) {
    if (n <= bytes && ptr) return hipSuccess;
    const size_t want = n < 256 ? 256 : n;
    if (tl_in_call) {
        // Growing inside a call: work queued earlier (this call's, or an
        // earlier call's -- the call stream waits for those) may still read the
        // old buffer, so it is freed in stream order after that work; no sync.
        if (ptr) {
            if (pooled) (void)hipFreeAsync(ptr, tl_call_stream);
            else (void)hipFree(ptr);   // a set-up allocation (never regrown in practice)
        }
        ptr = nullptr;
        bytes = 0;
        hipError_t e = hipMallocAsync(&ptr, want, tl_call_stream);
        if (e != hipSuccess) {
            ptr = nullptr;
            return e;
        }
        pooled = true;
        bytes = want;
        return hipSuccess;
    }
    return ensure_fixed(n);
}

hipError_t DevBuf::ensure_fixed(size_t n) {
    if (n <= bytes && ptr && !pooled) return hipSuccess;
    const size_t want = n < 256 ? 256 : n;
    release();
    hipError_t e = hipMalloc(&ptr, want);
    if (e != hipSuccess) {
        ptr = nullptr;
        bytes = 0;
        return e;
    }
    pooled = false;
    bytes = want;
    return hipSuccess;
}

void DevBuf::release() {
    if (ptr) {
        if (pooled && tl_in_call) {
            (void)hipFreeAsync(ptr, tl_call_stream);   // after the call's work, in stream order
        } else if (pooled) {
            // outside a call: the owner drained the streams that used it
            (void)hipFreeAsync(ptr, nullptr);
            (void)hipStreamSynchronize(nullptr);
        } else {
            (void)hipFree(ptr);
        }
    }
    ptr = nullptr;
    bytes = 0;
    pooled = false;
}

Engine::Engine(int device) : device_(device) {}

Engine::~Engine() {
    if (device_ >= 0) (void)hipSetDevice(device_);
    // every stream that may still read a buffer -- the context's own and the
    // last caller's (order_ev_) -- is idle before anything goes back to the
    // pool (round 4: pooled buffers were freed on the null stream, which does
    // not order against the context's non-blocking streams)
    (void)drain();
    for (DevBuf* b : {&gf16_log_, &gf16_exp_,
                      &gf16_skew_, &leaf_, &lvl_, &root_slots_, &dig_, &err_buf_, &dev_err_, &h_ods_, &h_eds_,
                      &h_rows_, &h_cols_, &h_roots_, &sq_plan_, &sq_txs_, &cm_plan_, &cm_tables_,
                      &cm_leaf_, &cm_lvl_, &cm_roots_, &cm_out_, &gf8_log_, &gf8_exp_, &gf8_skew_, &rp_cw_,
                      &rp_err_, &rp_present_, &rp_parity_, &rp_buf_, &rp_flags_, &tr_cells_, &tr_levels_,
                      &tr_axis_, &tr_roots_, &rs_pad_, &split_blk_, &split_send_, &split_col_, &split_slots_,
                      &comm_flag_, &h_par_})
        b->release();
    if (sq_event_) (void)hipEventSynchronize(sq_event_), (void)hipEventDestroy(sq_event_);
    if (sq_stage_) (void)hipHostFree(sq_stage_);
    if (rp_host_) (void)hipHostFree(rp_host_);
    if (rp_out_) (void)hipHostFree(rp_out_);
    for (Mark& m : marks_) {
        if (m.a) (void)hipEventDestroy(m.a);
        if (m.b) (void)hipEventDestroy(m.b);
    }
    for (hipEvent_t e : event_pool_) (void)hipEventDestroy(e);
    for (hipEvent_t e : sync_events_) (void)hipEventDestroy(e);
    comm_destroy();
    if (order_ev_) (void)hipEventDestroy(order_ev_);
    if (ev_rs_) (void)hipEventDestroy(ev_rs_);
    if (ev_out_) (void)hipEventDestroy(ev_out_);
    for (hipEvent_t* e : {pipe_in_, pipe_rs_, pipe_d2h_, pipe_comp_})
        for (uint32_t i = 0; i < kPipeSlots; i++)
            if (e[i]) (void)hipEventDestroy(e[i]);
    if (copy_in_) (void)hipStreamDestroy(copy_in_);
    if (copy_out_) (void)hipStreamDestroy(copy_out_);
    if (stream_) (void)hipStreamDestroy(stream_);
    if (aux_stream_) (void)hipStreamDestroy(aux_stream_);
    if (rs_cu_stream_) (void)hipStreamDestroy(rs_cu_stream_);
    if (hash_cu_stream_) (void)hipStreamDestroy(hash_cu_stream_);
    for (hipStream_t q : split_streams_)
        if (q) (void)hipStreamDestroy(q);
}

// Kernel faults surface asynchronously: at the next launch, copy or
// synchronisation of the context, whatever stage that is.  check() therefore
// keeps the stages enqueued since the context's work was last seen complete
// (pending_), and an asynchronous fault names them instead of blaming the
// stage that happened to detect it.  CDA_SYNC_CHECK=1 synchronises after every
// successful stage, so a fault is reported by the stage that raised it.
static bool async_fault(hipError_t e) {
    return e == hipErrorIllegalAddress || e == hipErrorLaunchTimeOut || e == hipErrorAssert ||
           e == hipErrorLaunchFailure;
}

static bool is_sync_point(const char* what) {
    return strncmp(what, "hipStreamSynchronize", 20) == 0 || strncmp(what, "hipEventSynchronize", 19) == 0 ||
           strncmp(what, "hipDeviceSynchronize", 20) == 0;
}

void Engine::note_stage(const char* what) {
    if (is_sync_point(what)) {   // everything enqueued before completed cleanly
        pending_.clear();
        return;
    }
    if (!pending_.empty() && strcmp(pending_.back(), what) == 0) return;
    if (pending_.size() >= kMaxPending) pending_.erase(pending_.begin());
    pending_.push_back(what);
}

std::string Engine::pending_stages() const {
    std::string s;
    for (const char* p : pending_) {
        if (!s.empty()) s += " -> ";
        s += p;
    }
    return s.empty() ? std::string("none recorded") : s;
}

int Engine::check(hipError_t e, const char* what) {
    if (e == hipSuccess) {
        if (sync_check_ && !is_sync_point(what)) {
            const hipError_t f = hipDeviceSynchronize();
            if (f != hipSuccess) {
                (void)hipGetLastError();
                return fail(CDA_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(f) +
                                                " (CDA_SYNC_CHECK: raised by this stage)");
            }
            pending_.clear();
            return CDA_OK;
        }
        note_stage(what);
        return CDA_OK;
    }
    std::string msg = std::string(what) + ": " + hipGetErrorString(e);
    if (async_fault(e))
        msg += " (asynchronous device fault, detected here but raised by GPU work of this context not yet seen "
               "complete; stages enqueued since, oldest first: " +
               pending_stages() + "; set CDA_SYNC_CHECK=1 to name the faulting stage)";
    (void)hipGetLastError();  // clear sticky launch error state
    return fail(e == hipErrorOutOfMemory ? CDA_ERR_OOM : CDA_ERR_DEVICE, msg);
}

int Engine::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(CDA_ERR_DEVICE, "no HIP device available");
    if (device_ < 0) {
        if (hipGetDevice(&device_) != hipSuccess) return fail(CDA_ERR_DEVICE, "hipGetDevice failed");
    }
    if (device_ >= n) return fail(CDA_ERR_INVALID, "device ordinal out of range");
    int rc;
    if ((rc = check(hipSetDevice(device_), "hipSetDevice"))) return rc;
    if ((rc = check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate"))) return rc;
    if ((rc = check(hipEventCreateWithFlags(&order_ev_, hipEventDisableTiming), "hipEventCreate"))) return rc;
    if ((rc = check(hipStreamCreateWithFlags(&copy_out_, hipStreamNonBlocking), "hipStreamCreate"))) return rc;
    if ((rc = check(hipEventCreateWithFlags(&ev_rs_, hipEventDisableTiming), "hipEventCreate"))) return rc;
    if ((rc = check(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming), "hipEventCreate"))) return rc;
    if ((rc = check(hipStreamCreateWithFlags(&copy_in_, hipStreamNonBlocking), "hipStreamCreate"))) return rc;
    for (hipEvent_t* e : {pipe_in_, pipe_rs_, pipe_d2h_, pipe_comp_})
        for (uint32_t i = 0; i < kPipeSlots; i++)
            if ((rc = check(hipEventCreateWithFlags(&e[i], hipEventDisableTiming), "hipEventCreate"))) return rc;
    // CDA_RS_PRIORITY (tuning): priority of the pipeline's RS stream (HIP: a
    // lower value is a higher priority).
    if (const char* env = test_knob("CDA_RS_PRIORITY")) {
        if ((rc = check(hipStreamCreateWithPriority(&aux_stream_, hipStreamNonBlocking, atoi(env)), "hipStreamCreate")))
            return rc;
    } else if ((rc = check(hipStreamCreateWithFlags(&aux_stream_, hipStreamNonBlocking), "hipStreamCreate"))) {
        return rc;
    }
    if (const char* env = deploy_knob("CDA_PIPELINE_CHUNK")) pipeline_chunk_ = (uint32_t)strtoul(env, nullptr, 10);
    if (const char* env = test_knob("CDA_HASH_SPLIT")) hash_split_ = atoi(env);
    if (const char* env = test_knob("CDA_HOST_CHUNK")) host_chunk_ = (uint32_t)strtoul(env, nullptr, 10);
    if (const char* env = deploy_knob("CDA_HOST_PIPE_CHUNK")) host_pipe_chunk_ = (uint32_t)strtoul(env, nullptr, 10);
    if (const char* env = test_knob("CDA_HOST_FULL_D2H")) host_full_d2h_ = atoi(env) != 0;
    if (const char* env = deploy_knob("CDA_HOST_REGISTER")) host_register_ = atoi(env) != 0;
    if (const char* env = test_knob("CDA_TOP_FUSE")) top_fuse_ = atoi(env);
    if (const char* env = test_knob("CDA_TOP_WIDE")) top_wide_ = atoi(env);
    if (const char* env = test_knob("CDA_SUBTREE")) subtree_min_ = atoi(env);
    if (const char* env = test_knob("CDA_SUBTREE_LANES")) subtree_lanes_ = strtoull(env, nullptr, 10);
    if (const char* env = test_knob("CDA_RS16_PRIO_MAX")) rs16_prio_max_ = (uint32_t)strtoul(env, nullptr, 10);
    if (const char* env = test_knob("CDA_RS8_PRIO")) rs8_prio_ = atoi(env) != 0;
    if (const char* env = test_knob("CDA_RS_CUS")) rs_cus_ = (uint32_t)strtoul(env, nullptr, 10);
    if (const char* env = deploy_knob("CDA_SYNC_CHECK")) sync_check_ = atoi(env) != 0;
    if (const char* env = test_knob("CDA_FAULT")) fault_ = env;
    // GF(2^16) tables (leopard.go initLUTs / initFFT), built on the host once.
    auto F = std::make_unique<LeoField<16>>();
    leo_build<16>(*F, 0x1002D, kCantor16);
    if ((rc = check(gf16_log_.ensure_fixed(sizeof F->log), "hipMalloc"))) return rc;
    if ((rc = check(gf16_exp_.ensure_fixed(sizeof F->exp), "hipMalloc"))) return rc;
    if ((rc = check(gf16_skew_.ensure_fixed(sizeof F->skew), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpy(gf16_log_.ptr, F->log, sizeof F->log, hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
    if ((rc = check(hipMemcpy(gf16_exp_.ptr, F->exp, sizeof F->exp, hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
    if ((rc = check(hipMemcpy(gf16_skew_.ptr, F->skew, sizeof F->skew, hipMemcpyHostToDevice), "hipMemcpy")))
        return rc;
    return CDA_OK;
}

Gf16Dev Engine::gf16(uint32_t k) const {
    (void)k;   // k = 256 / 512 use compile-time networks (rs_gf16_bs.hip); the tables serve other k
    return Gf16Dev{gf16_log_.as<uint16_t>(), gf16_exp_.as<uint16_t>(), gf16_skew_.as<uint16_t>()};
}

static bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

// Nodes per tree at which the NMT levels switch from one wide launch per level
// to tree_top_kernel (0 = never): the first level whose parents, over all 2W
// trees of the n squares, fill less than one wave per SIMD of the chip
// (1024 SIMDs x 64 lanes) -- lane pairs from there -- and then up to
// top_wide_ (CDA_TOP_WIDE) levels more, while the lane pairs of the level
// below the first fit in two waves per SIMD: the first of them runs a thread
// per parent inside the tree top (*wide), which saves their per-level
// launches (drain tail + boundary each).  CDA_TOP_FUSE=0 disables, =N forces
// N (not wide).
uint32_t Engine::top_fuse_nodes(uint32_t W, uint32_t n, bool* wide) const {
    if (wide) *wide = false;
    if (top_fuse_ >= 0) return (uint32_t)top_fuse_ <= W && top_fuse_ <= 256 ? (uint32_t)top_fuse_ : 0;
    for (uint32_t m = W; m >= 2; m /= 2) {
        if ((uint64_t)n * 2 * W * (m / 2) >= 65536) continue;
        if (m > 256) return 0;
        uint32_t t = m;
        // the wide first level runs lane pairs above it: none without pairs
        // (a one-thread-per-parent top holds at most 256 nodes)
        const int widen = pair_sha_enabled() ? top_wide_ : 0;
        for (int e = 0; e < widen && 2 * t <= W && 2 * t <= 512 && 2 * t >= 8 &&
                        2 * (uint64_t)n * 2 * W * (t / 2) <= 131072;
             e++)
            t *= 2;
        if (wide) *wide = t > m;
        return t;
    }
    return 0;
}

int Engine::order_begin(hipStream_t s) {
    tl_in_call = true;
    tl_call_stream = s;
    if (!order_used_) return CDA_OK;
    // the previous calls' work is complete (without a fault): nothing of it can
    // surface later, and there is nothing to order after (no wait packet ahead
    // of this call's first launch: the latency path's calls find it complete)
    if (hipEventQuery(order_ev_) == hipSuccess) {
        pending_.clear();
        return CDA_OK;
    }
    if (hipStreamWaitEvent(s, order_ev_, 0) == hipSuccess) return CDA_OK;
    // the wait could not be enqueued: wait on the host instead (a fault of the
    // previous work surfaces here, named by check())
    (void)hipGetLastError();
    return check(hipEventSynchronize(order_ev_), "hipEventSynchronize (previous call's work)");
}

int Engine::drain_streams() {
    int first = CDA_OK;
    auto sync = [&](hipStream_t q) {
        if (!q) return;
        const hipError_t e = hipStreamSynchronize(q);
        if (e != hipSuccess && first == CDA_OK) first = check(e, "hipStreamSynchronize (drain)");
        else if (e != hipSuccess) (void)hipGetLastError();
    };
    for (hipStream_t q : {stream_, copy_in_, copy_out_, aux_stream_, rs_cu_stream_, hash_cu_stream_}) sync(q);
    for (hipStream_t q : split_streams_) sync(q);
    return first;
}

int Engine::wait_last_call() {
    if (order_used_ && order_ev_) return check(hipEventSynchronize(order_ev_), "hipEventSynchronize (last call)");
    return CDA_OK;
}

int Engine::drain() {
    int rc = drain_streams();
    const int w = wait_last_call();
    return rc != CDA_OK ? rc : w;
}

void Engine::order_end(hipStream_t s) {
    tl_in_call = false;
    if (order_ev_ && hipEventRecord(order_ev_, s) == hipSuccess) order_used_ = true;
}

hipEvent_t Engine::take_event() {
    if (!event_pool_.empty()) {
        hipEvent_t e = event_pool_.back();
        event_pool_.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void Engine::mark_begin(int stage, hipStream_t s) {
    if (!profiling_) return;
    Mark m{stage, take_event(), take_event()};
    if (m.a) (void)hipEventRecord(m.a, s);
    marks_.push_back(m);
}

void Engine::mark_end(hipStream_t s) {
    if (!profiling_ || marks_.empty()) return;
    if (marks_.back().b) (void)hipEventRecord(marks_.back().b, s);
}

int Engine::collect_stage_times(double* ms, uint32_t* counts, int n) {
    for (Mark& m : marks_) {
        if (m.a && m.b && hipEventSynchronize(m.b) == hipSuccess) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, m.a, m.b) == hipSuccess) {
                stage_ms_[m.stage] += t;
                stage_n_[m.stage] += 1;
            }
        }
        if (m.a) event_pool_.push_back(m.a);
        if (m.b) event_pool_.push_back(m.b);
    }
    marks_.clear();
    for (int i = 0; i < n && i < kNumStages; i++) {
        if (ms) ms[i] = stage_ms_[i];
        if (counts) counts[i] = stage_n_[i];
        stage_ms_[i] = 0;
        stage_n_[i] = 0;
    }
    return CDA_OK;
}

int Engine::enqueue_extend(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds, hipStream_t s,
                           uint32_t* err_init) {
    if (!pow2(k) || k > 1024) return fail(CDA_ERR_INVALID, "square width must be a power of two <= 1024");
    int rc;
    const Gf16Dev t = gf16(k);
    mark_begin(kStageRsQ0, s);
    // d_ods == NULL: in place, the ODS is already in Q0 of d_eds
    RsJob q0 = d_ods ? square_job_q0(d_ods, d_eds, k) : square_job_q0_inplace(d_eds, k);
    RsJob q3 = square_job_q3(d_eds, k);
    q0.err_init = err_init;
    q0.prio = q3.prio = (k >= 256 ? n <= rs16_prio_max_ : rs8_prio_) ? 1u : 0u;
    if ((rc = check(launch_rs(q0, k, n, t, s), "rs Q0"))) return rc;
    mark_end(s);
    mark_begin(kStageRsQ3, s);
    if ((rc = check(launch_rs(q3, k, n, t, s), "rs Q3"))) return rc;
    mark_end(s);
    return CDA_OK;
}

// Run every level of `f` (n_forest forests of n_in leaves each) ping-ponging
// between two scratch buffers; the first level reads f[i].in.
int Engine::run_forests(Forest* f, uint32_t n_forest, uint32_t n_in, uint32_t n, uint8_t* bufA, uint8_t* bufB,
                        uint64_t buf_sq, const uint64_t* out_off, hipStream_t s, uint32_t stop, bool subtrees) {
    uint8_t* out = bufA;
    int rc;
    // The first levels as one fused subtree launch (nmt.hip subtree_kernel):
    // a lane per (n_in / sub)-leaf subtree, sub the smallest node count >= stop
    // at which the launch holds `want` lanes (default two waves per
    // SIMD: a lone wave per SIMD issues at ~5.4 cycles per instruction on this
    // chain, two interleave to the saturated rate); the levels from sub down
    // to stop then run as per-level launches.  With stop = 1 (big batches: no
    // tree top) and sub = 1 a lane hashes a whole tree and the launch writes
    // the roots itself (config 4: levels 15.8 -> 14.1 ms, profiles/r03ab/,
    // r03ak/).  Roots and per-lane stacks need n_trees * sub * log2(n_in /
    // sub) slots of each forest's output region.  With the batch split over
    // two streams (n <= 256) each launch holds only its part's lanes, so the
    // lane bound is per launch.
    uint32_t m0 = n_in;
    if (subtrees && subtree_min_ > 0 && stop >= 1 && n_in % stop == 0) {
        uint64_t per_node = 0;   // lanes per subtree root per tree
        for (uint32_t i = 0; i < n_forest; i++) per_node += (uint64_t)n * f[i].n_trees;
        uint32_t sub = stop;
        // default target: 524288 lanes (8 waves per SIMD, 2.67 rounds at the
        // kernel's 3 waves per SIMD, the shape of config 4's whole-tree launch)
        // for trees of <= 512 leaves -- config 4's per-GPU shards of 64 / 128
        // / 256 squares +4-5 % over 131072 lanes on two streams (round 5,
        // profiles/r05/subtree_lanes_ab.txt); 262144 for trees of >= 1024
        // leaves (k >= 512: one k = 512 square 1.096 -> 1.087 ms, 8- instead
        // of 16-leaf subtrees; profiles/r03at/).  Subtrees keep >= 8 leaves
        // (CDA_SUBTREE); a batch too small to reach the target still takes the
        // fused launch when it holds 131072 lanes.
        const uint64_t want = subtree_lanes_ ? subtree_lanes_ : n_in >= 1024 ? 262144u : 524288u;
        // launch_subtrees needs subtrees of >= 4 leaves: a smaller CDA_SUBTREE
        // setting means per-level launches, not a failing launch
        const uint32_t min_leaves = (uint32_t)std::max(subtree_min_, 4);
        while (sub < n_in && 2 * (uint64_t)sub * min_leaves <= n_in && per_node * sub < want) sub *= 2;
        bool fits = per_node * sub >= std::min<uint64_t>(want, 131072) && sub < n_in && n_in / sub >= min_leaves;
        const uint32_t slog = fits ? (uint32_t)__builtin_ctz(n_in / sub) : 0;
        for (uint32_t i = 0; i < n_forest && fits; i++) {
            const uint64_t need = (uint64_t)f[i].n_trees * sub * slog * kSlot;
            const uint64_t room = n_forest > 1 ? out_off[1] - out_off[0] : buf_sq;
            fits = need <= room && f[i].n_trees % 64 == 0;
        }
        if (fits) {
            for (uint32_t i = 0; i < n_forest; i++) {
                f[i].out = out + out_off[i];
                f[i].out_sq = buf_sq;
            }
            if ((rc = check(launch_subtrees(f, n_forest, n_in, sub, n, s), "nmt subtrees"))) return rc;
            for (uint32_t i = 0; i < n_forest; i++) {
                f[i].in = out + out_off[i];
                f[i].in_sq = buf_sq;
                f[i].tree_stride = sub;
                f[i].node_stride = 1;
            }
            out = bufB;
            m0 = sub;
        }
    }
    for (uint32_t m = m0; m >= 2 && m > stop; m /= 2) {
        for (uint32_t i = 0; i < n_forest; i++) {
            f[i].out = out + out_off[i];
            f[i].out_sq = buf_sq;
        }
        if ((rc = check(launch_level(f, n_forest, m, n, s), "nmt level"))) return rc;
        for (uint32_t i = 0; i < n_forest; i++) {   // next level reads this one
            f[i].in = out + out_off[i];
            f[i].in_sq = buf_sq;
            f[i].tree_stride = m / 2;
            f[i].node_stride = 1;
        }
        out = out == bufA ? bufB : bufA;
    }
    return CDA_OK;
}

// enqueue_dah in pieces.  The serial path runs them back to back; the batch
// pipeline (enqueue_extend_dah) hashes each chunk as soon as its RS is done
// (dah_chunk) and runs the latency-bound rest once for the whole batch
// (dah_finish).
// d_err == NULL: the push-order words are already set (enqueue_extend's err_init).
int Engine::dah_prepare(uint32_t W, uint32_t n, uint32_t* d_err, hipStream_t s) {
    const uint64_t slots_sq = (uint64_t)W * W * kSlot;
    int rc;
    if ((rc = check(leaf_.ensure(slots_sq * n), "hipMalloc leaf slots"))) return rc;
    if ((rc = check(lvl_.ensure(slots_sq * n), "hipMalloc level slots"))) return rc;
    if ((rc = check(root_slots_.ensure((size_t)n * 2 * W * kSlot), "hipMalloc root slots"))) return rc;
    if ((rc = check(dig_.ensure((size_t)n * 2 * W * 32), "hipMalloc digests"))) return rc;
    return d_err ? check(hipMemsetAsync(d_err, 0xFF, (size_t)n * 4, s), "hipMemsetAsync") : CDA_OK;
}

int Engine::reserve(uint32_t k, uint32_t n) {
    int rc;
    if (!err_words(n)) return fail(CDA_ERR_OOM, "hipMalloc err words");
    if ((rc = dah_prepare(2 * k, n, nullptr, stream_))) return rc;
    return check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

// Row trees: leaves (t, i); column trees: leaves (i, t) of the same leaf grid.
// Roots go packed to d_rows / d_cols and as 96-B slots (rows then columns) to
// root_slots_ for the data root.
void Engine::dah_forests(uint32_t W, uint8_t* d_rows, uint8_t* d_cols, Forest (&f)[2]) {
    const uint64_t slots_sq = (uint64_t)W * W * kSlot;
    f[0] = Forest{leaf_.as<uint8_t>(), slots_sq, W, W, 1, nullptr, 0, d_rows, (uint64_t)W * kNode,
                  root_slots_.as<uint8_t>(), (uint64_t)2 * W * kSlot, 0};
    f[1] = Forest{leaf_.as<uint8_t>(), slots_sq, W, 1, W, nullptr, 0, d_cols, (uint64_t)W * kNode,
                  root_slots_.as<uint8_t>(), (uint64_t)2 * W * kSlot, W};
}

// Leaves and the NMT levels down to `stop` nodes per tree of squares
// [i0, i0 + m).  f: the batch's forests from dah_forests; on return `post`
// describes (for the whole batch) the level the chunk stopped at.
int Engine::dah_chunk(const uint8_t* d_eds, uint32_t k, uint32_t i0, uint32_t m, uint32_t stop, uint32_t* d_err,
                      const Forest (&f)[2], Forest (&post)[2], hipStream_t s, bool subtrees) {
    const uint32_t W = 2 * k;
    const uint64_t slots_sq = (uint64_t)W * W * kSlot, eds_sq = (uint64_t)W * W * kShare;
    int rc;
    mark_begin(kStageLeaves, s);
    const CellGrid g{d_eds + i0 * eds_sq, eds_sq, W, W, W, 0, 0, k};
    if ((rc = check(launch_leaves(g, m, leaf_.as<uint8_t>() + i0 * slots_sq, d_err + i0, true, true, s),
                    "leaf hashing")))
        return rc;
    mark_end(s);
    Forest fc[2] = {f[0], f[1]};
    for (int i = 0; i < 2; i++) {
        fc[i].in += i0 * fc[i].in_sq;
        if (fc[i].roots) fc[i].roots += i0 * fc[i].roots_sq;
        if (fc[i].root_slots) fc[i].root_slots += i0 * fc[i].rslot_sq;
    }
    if (W > stop) {
        mark_begin(kStageLevels, s);
        const uint64_t off[2] = {0, slots_sq / 2};
        if ((rc = run_forests(fc, 2, W, m, lvl_.as<uint8_t>() + i0 * slots_sq, leaf_.as<uint8_t>() + i0 * slots_sq,
                              slots_sq, off, s, stop, subtrees)))
            return rc;
        mark_end(s);
    }
    for (int i = 0; i < 2; i++) {
        post[i] = fc[i];
        post[i].in -= i0 * fc[i].in_sq;
        post[i].roots = f[i].roots;
        post[i].root_slots = f[i].root_slots;
    }
    return CDA_OK;
}

// The levels below `from` nodes per tree (f = dah_chunk's post), the fused
// tree top and the data root (which also writes d_status), for squares
// [i0, i0 + n) of the batch (d_roots, d_err, d_status: batch base pointers).
int Engine::dah_finish(uint32_t k, uint32_t i0, uint32_t n, uint32_t from, const Forest (&fb)[2], uint8_t* d_roots,
                       uint32_t* d_err, int32_t* d_status, hipStream_t s) {
    const uint32_t W = 2 * k;
    const uint64_t slots_sq = (uint64_t)W * W * kSlot;
    int rc;
    Forest f[2] = {fb[0], fb[1]};
    for (int i = 0; i < 2; i++) {
        f[i].in += i0 * f[i].in_sq;
        if (f[i].roots) f[i].roots += i0 * f[i].roots_sq;
        if (f[i].root_slots) f[i].root_slots += i0 * f[i].rslot_sq;
    }
    uint32_t* dig = dig_.as<uint32_t>() + (size_t)i0 * 2 * W * 8;
    uint8_t* rslots = root_slots_.as<uint8_t>() + (size_t)i0 * 2 * W * kSlot;
    if (d_roots) d_roots += (size_t)i0 * 32;
    d_err += i0;
    if (d_status) d_status += i0;
    // Wide per-level launches while a level has at least a wave per SIMD of
    // parents; the latency-bound rest of the trees (and the data root's RFC
    // leaf digests) in one tree_top_kernel launch.
    // (from == 1: the chunks already produced the roots -- no tree top)
    bool wide = false;
    uint32_t top = from > 1 ? top_fuse_nodes(W, n, &wide) : 0;
    uint32_t n_dig = 2 * W;   // digests per square the tree top leaves for the data root
    if (top > from) {
        top = from;
        wide = false;
    }
    if (from > 1) {
        const uint32_t stop = top ? top : 1;
        mark_begin(kStageLevels, s);
        if (from > stop) {
            // the chunks ran ctz(W) - ctz(from) levels, the first into lvl_
            const bool in_lvl = ((__builtin_ctz(W) - __builtin_ctz(from)) & 1) != 0;
            uint8_t* a = (in_lvl ? leaf_.as<uint8_t>() : lvl_.as<uint8_t>()) + i0 * slots_sq;
            uint8_t* b = (in_lvl ? lvl_.as<uint8_t>() : leaf_.as<uint8_t>()) + i0 * slots_sq;
            const uint64_t off[2] = {0, slots_sq / 2};
            if ((rc = run_forests(f, 2, from, n, a, b, slots_sq, off, s, stop))) return rc;
        }
        if (top && (rc = check(launch_tree_top(f, 2, top, n, d_roots ? dig : nullptr, 2 * W, s, &n_dig, wide),
                               "nmt tree top")))
            return rc;
        mark_end(s);
    }
    // the data-root launch also writes the per-square push-order status
    if (d_roots && top) {
        mark_begin(kStageDataRoot, s);
        if ((rc = check(launch_data_root_digests(dig, n_dig, n, d_roots, s, d_err, d_status), "data root")))
            return rc;
        mark_end(s);
    } else if (d_roots) {   // NULL: roots only (repair verification needs no data root)
        mark_begin(kStageDataRoot, s);
        if ((rc = check(launch_data_root_slots(rslots, 2 * W, n, dig, d_roots, s, d_err, d_status), "data root")))
            return rc;
        mark_end(s);
    }
    if (!d_roots && d_status && (rc = check(launch_status(d_err, n, d_status, s), "status"))) return rc;
    return CDA_OK;
}

int Engine::enqueue_dah(const uint8_t* d_eds, uint32_t k, uint32_t n, uint8_t* d_rows, uint8_t* d_cols,
                        uint8_t* d_roots, uint32_t* d_err, int32_t* d_status, hipStream_t s, bool err_ready) {
    if (!pow2(k) || k > 1024) return fail(CDA_ERR_INVALID, "square width must be a power of two <= 1024");
    const uint32_t W = 2 * k;
    int rc;
    if ((rc = dah_prepare(W, n, err_ready ? nullptr : d_err, s))) return rc;
    Forest f[2], post[2];
    dah_forests(W, d_rows, d_cols, f);
    const uint32_t top = top_fuse_nodes(W, n);
    const uint32_t stop = top ? top : 1;
    // The leaves and wide levels of the parts of a batch (CDA_HASH_SPLIT of
    // them, default 2) run on their own streams, so one part's level launches
    // fill the chip while another's last partial round of workgroups drains
    // (levels 3-8 of a k = 128 batch lose 10-60 % to that tail alone;
    // profiles/r02_hash_split.txt).  CDA_HASH_SPLIT=0 turns it off; stage
    // profiling (bench's separate stage pass) uses the one-stream schedule so
    // every stage's events time its own kernels.
    // auto: two parts up to 256 squares (+0.3-1.8 % at 128, profiles/r02_hash_split.txt), one above --
    // at config 4's 1024 squares per launch the level tails no longer matter (21 465 split vs 21 528
    // one stream, profiles/r03a/bench_split0.json), and one stream keeps every launch of a kernel the
    // same shape, so per-launch profiler counters divide by a known square count
    // k >= 256: one stream -- a k = 512 square's levels already fill the chip
    // (its subtree launch holds 262 144 lanes), and half-size launches on two
    // streams ran slower: k = 512 x 4 0.996 -> 0.945 ms per square, x 16
    // 0.888 -> 0.874 with one stream (profiles/r05/k512_pipeline_hashsplit_ab.txt)
    // Round 5: one stream from 64 squares up as well -- with the subtree
    // launch's 524288-lane target (run_forests) one launch fills the chip, and
    // 64 / 128 / 256 squares ran 4-5 % faster on one stream
    // (profiles/r05/subtree_lanes_ab.txt); two parts stay for small batches,
    // whose latency-bound tails the second stream overlaps.
    const uint32_t want = hash_split_ >= 0 ? (uint32_t)hash_split_ : (n < 64 && k <= 128 ? 2u : 1u);
    const uint32_t parts = std::min<uint32_t>(std::min<uint32_t>(want, n), kMaxHashParts);
    if (parts > 1 && !profiling_) {
        hipEvent_t go = sync_event(0);
        if (!go || !sync_event(parts)) return fail(CDA_ERR_DEVICE, "hipEventCreate failed");
        if ((rc = check(hipEventRecord(go, s), "hipEventRecord"))) return rc;
        // part p: squares [p n / parts, (p + 1) n / parts); part 0 on the
        // caller's stream.  Each part also finishes its own trees and data
        // roots, so one part's latency-bound data root runs under another's
        // levels.
        // Every side part that started is joined back to s on every return
        // path, the error returns included: a part that failed half-way may
        // have queued leaves / levels reading the scratch, and the next call
        // orders itself after s only.
        int err = CDA_OK;
        uint32_t joined_from = parts;   // side parts [joined_from, parts) recorded their end on sync_event(p)
        for (uint32_t p = parts; p-- > 0;) {
            const uint32_t i0 = p * n / parts, i1 = (p + 1) * n / parts;
            hipStream_t q = s;
            if (p) {
                if ((rc = split_stream(p - 1, &q))) {
                    err = rc;
                    break;
                }
                if ((rc = check(hipStreamWaitEvent(q, go, 0), "hipStreamWaitEvent"))) {   // nothing queued on q
                    err = rc;
                    break;
                }
            }
            Forest pp[2];
            rc = dah_chunk(d_eds, k, i0, i1 - i0, stop, d_err, f, pp, q, true);
            if (!rc) rc = dah_finish(k, i0, i1 - i0, stop, pp, d_roots, d_err, d_status, q);
            if (!rc && p && fault_at("dah_part"))
                rc = fail(CDA_ERR_DEVICE, "enqueue_dah: injected fault after a side part's hashing (CDA_FAULT=dah_part)");
            if (p) {
                if (hipEventRecord(sync_event(p), q) == hipSuccess) {
                    joined_from = p;
                } else {   // cannot join by event: wait for the part on the host
                    (void)hipGetLastError();
                    (void)hipStreamSynchronize(q);
                    if (!rc) rc = fail(CDA_ERR_DEVICE, "hipEventRecord failed (hash split join)");
                }
            }
            if (rc) {
                err = rc;
                break;
            }
        }
        for (uint32_t p = joined_from; p < parts; p++) {
            if (hipStreamWaitEvent(s, sync_event(p), 0) == hipSuccess) continue;
            (void)hipGetLastError();
            hipStream_t q = nullptr;
            if (split_stream(p - 1, &q) == CDA_OK) (void)hipStreamSynchronize(q);
            if (!err) err = fail(CDA_ERR_DEVICE, "hipStreamWaitEvent failed (hash split join)");
        }
        return err;
    }
    if ((rc = dah_chunk(d_eds, k, 0, n, stop, d_err, f, post, s, true))) return rc;
    return dah_finish(k, 0, n, stop, post, d_roots, d_err, d_status, s);
}

// ---------------------------------------------------------------------------
// Config 5: one square split across G ranks (see include/cda.h cda_split_*).
// ---------------------------------------------------------------------------
int Engine::enqueue_split_rows(const uint8_t* d_rows, uint32_t k, uint32_t n_rows, uint32_t row0, uint8_t* d_block,
                               uint32_t* d_err, hipStream_t s) {
    if (!pow2(k) || k > 1024 || n_rows == 0 || row0 + n_rows > k)
        return fail(CDA_ERR_INVALID, "bad row block");
    const uint32_t W = 2 * k, SH = kShare;
    int rc;
    const CellGrid g{d_rows, 0, n_rows, k, k, row0, 0, k};
    if ((rc = check(launch_row_order(g, 1, d_err, s), "row order"))) return rc;
    RsJob j{};
    j.src = d_rows;
    j.dst = d_block;
    j.n_seg = 1;
    j.seg[0] = RsSeg{n_rows, 0, k * SH, SH, k * SH, W * SH, SH, 0, W * SH, SH};
    return check(launch_rs(j, k, 1, gf16(k), s), "rs rows");
}

int Engine::enqueue_split_cols(uint8_t* d_block, uint32_t k, uint32_t n_cols, uint32_t col0, uint8_t* d_col_slots,
                               uint8_t* d_row_sub, uint32_t* d_err, hipStream_t s) {
    const uint32_t W = 2 * k, SH = kShare;
    if (!pow2(k) || k > 1024 || !pow2(n_cols) || n_cols < 2 || col0 + n_cols > W)
        return fail(CDA_ERR_INVALID, "bad column block");
    int rc;
    RsJob j{};
    j.src = d_block;
    j.dst = d_block;
    j.n_seg = 1;
    j.seg[0] = RsSeg{n_cols, 0, SH, n_cols * SH, k * n_cols * SH, SH, n_cols * SH};
    if ((rc = check(launch_rs(j, k, 1, gf16(k), s), "rs cols"))) return rc;
    const uint64_t slots = (uint64_t)W * n_cols * kSlot;
    if ((rc = check(leaf_.ensure(slots), "hipMalloc leaf slots"))) return rc;
    if ((rc = check(lvl_.ensure(slots), "hipMalloc level slots"))) return rc;
    const CellGrid g{d_block, 0, W, n_cols, n_cols, 0, col0, k};
    if ((rc = check(launch_leaves(g, 1, leaf_.as<uint8_t>(), d_err, true, true, s), "leaf hashing"))) return rc;
    // row subtrees: W trees of n_cols leaves -> one 96-B slot per row
    // (ping-pong between the two halves of the level buffer; leaves untouched)
    Forest fr{leaf_.as<uint8_t>(), 0, W, n_cols, 1, nullptr, 0, nullptr, 0, d_row_sub, 0, 0};
    const uint64_t off0[1] = {0};
    if ((rc = run_forests(&fr, 1, n_cols, 1, lvl_.as<uint8_t>(), lvl_.as<uint8_t>() + slots / 2, 0, off0, s)))
        return rc;
    // column trees: n_cols trees of W leaves; after their first level the leaf
    // buffer is free and becomes the second ping-pong buffer
    Forest fc{leaf_.as<uint8_t>(), 0, n_cols, 1, n_cols, nullptr, 0, nullptr, 0, d_col_slots, 0, 0};
    return run_forests(&fc, 1, W, 1, lvl_.as<uint8_t>(), leaf_.as<uint8_t>(), 0, off0, s);
}

int Engine::enqueue_split_combine(const uint8_t* d_row_sub, uint32_t parts, uint32_t k, const uint8_t* d_col_slots,
                                  uint8_t* d_rows, uint8_t* d_cols, uint8_t* d_root, hipStream_t s) {
    const uint32_t W = 2 * k;
    if (!pow2(k) || !pow2(parts) || parts > W) return fail(CDA_ERR_INVALID, "bad split");
    int rc;
    if ((rc = check(root_slots_.ensure((size_t)2 * W * kSlot), "hipMalloc root slots"))) return rc;
    if ((rc = check(lvl_.ensure((size_t)W * parts * kSlot), "hipMalloc level slots"))) return rc;
    if ((rc = check(leaf_.ensure((size_t)W * parts * kSlot), "hipMalloc leaf slots"))) return rc;
    uint8_t* rs = root_slots_.as<uint8_t>();
    if (parts == 1) {
        if ((rc = check(hipMemcpyAsync(rs, d_row_sub, (size_t)W * kSlot, hipMemcpyDeviceToDevice, s), "copy")))
            return rc;
    } else {
        // row tree r: nodes (g, r) of the gathered [parts][W] -> top
        // log2(parts) levels (SplitLayout::combine_slot: tree stride 1, node stride W)
        const SplitLayout L(k, parts);
        const uint32_t tstride = (uint32_t)(L.combine_slot(0, 1) - L.combine_slot(0, 0));
        const uint32_t nstride = (uint32_t)(L.combine_slot(1, 0) - L.combine_slot(0, 0));
        Forest fr{d_row_sub, 0, W, tstride, nstride, nullptr, 0, nullptr, 0, rs, 0, 0};
        const uint64_t off0[1] = {0};
        if ((rc = run_forests(&fr, 1, parts, 1, lvl_.as<uint8_t>(), leaf_.as<uint8_t>(), 0, off0, s))) return rc;
    }
    if ((rc = check(hipMemcpyAsync(rs + (size_t)W * kSlot, d_col_slots, (size_t)W * kSlot, hipMemcpyDeviceToDevice, s),
                    "copy")))
        return rc;
    if ((rc = check(launch_slots_to_roots(rs, 2 * W, d_rows, d_cols, W, s), "pack roots"))) return rc;
    return check(launch_data_root(rs, 2 * W, 1, d_root, s), "data root");
}

int Engine::enqueue_extend_dah_serial(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds,
                                      uint8_t* d_rows, uint8_t* d_cols, uint8_t* d_roots, uint32_t* d_err,
                                      int32_t* d_status, hipStream_t s) {
    // the first RS launch also sets the push-order words (no separate fill)
    int rc = enqueue_extend(d_ods, k, n, d_eds, s, d_err);
    if (rc) return rc;
    return enqueue_dah(d_eds, k, n, d_rows, d_cols, d_roots, d_err, d_status, s, true);
}

// Stream i of the hash split: the context's second stream, then lazily
// created ones.
int Engine::split_stream(uint32_t i, hipStream_t* out) {
    if (i == 0) {
        *out = aux_stream_;
        return CDA_OK;
    }
    hipStream_t& q = split_streams_[i - 1];
    if (!q) {
        int rc;
        if ((rc = check(hipStreamCreateWithFlags(&q, hipStreamNonBlocking), "hipStreamCreate"))) return rc;
    }
    *out = q;
    return CDA_OK;
}

hipEvent_t Engine::sync_event(size_t i) {
    while (sync_events_.size() <= i) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        sync_events_.push_back(e);
    }
    return sync_events_[i];
}

// The RS / hash CU partition of CDA_RS_CUS: RS on CUs (33 j) mod ncu, j < N --
// spread over the XCDs whether the mask bits run XCD-major or CU-major.
int Engine::make_cu_streams() {
    if (rs_cu_stream_) return CDA_OK;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_) != hipSuccess || ncu <= 0 ||
        rs_cus_ >= (uint32_t)ncu)
        return fail(CDA_ERR_INVALID, "the RS CU partition must be below the device's CU count");
    std::vector<uint32_t> rs((ncu + 31) / 32, 0u), hs((ncu + 31) / 32, 0u);
    for (uint32_t j = 0; j < rs_cus_; j++) {
        const uint32_t b = (33u * j) % (uint32_t)ncu;
        rs[b / 32] |= 1u << (b % 32);
    }
    for (int b = 0; b < ncu; b++)
        if (!(rs[b / 32] >> (b % 32) & 1)) hs[b / 32] |= 1u << (b % 32);
    int rc;
    if ((rc = check(hipExtStreamCreateWithCUMask(&rs_cu_stream_, (uint32_t)rs.size(), rs.data()), "cu mask stream")))
        return rc;
    return check(hipExtStreamCreateWithCUMask(&hash_cu_stream_, (uint32_t)hs.size(), hs.data()), "cu mask stream");
}

// Batch pipeline.  The batch is cut into chunks of c squares; chunk i's RS
// extension runs on aux_stream_ and its leaves and wide NMT levels on the
// caller's stream after an event, so the RS of chunk i+1 (memory-bound: its
// half-footprint kernel leaves room for hash waves on every CU) runs under the
// SHA-256 of chunk i (VALU-bound).  The narrow levels, the tree tops and the
// data roots -- latency-bound -- run once for the whole batch at the end.
// aux_stream_ starts after the work already queued on `s` and `s` waits for
// every chunk's RS before hashing it, so the call keeps single-stream
// semantics for the caller.  Events are re-recorded by later calls only after
// hipStreamWaitEvent has captured them (HIP semantics).
int Engine::enqueue_extend_dah(const uint8_t* d_ods, uint32_t k, uint32_t n, uint8_t* d_eds, uint8_t* d_rows,
                               uint8_t* d_cols, uint8_t* d_roots, uint32_t* d_err, int32_t* d_status,
                               hipStream_t s) {
    if (!pow2(k) || k > 1024) return fail(CDA_ERR_INVALID, "square width must be a power of two <= 1024");
    const uint32_t c = pipeline_chunk_ ? pipeline_chunk_ : n;
    if (c >= n) return enqueue_extend_dah_serial(d_ods, k, n, d_eds, d_rows, d_cols, d_roots, d_err, d_status, s);
    const uint32_t W = 2 * k;
    const uint64_t ods_sq = (uint64_t)k * k * kShare, eds_sq = (uint64_t)W * W * kShare;
    const uint32_t n_chunks = (n + c - 1) / c;
    // per chunk: the levels whose parents (over the chunk's 2W trees) fill at
    // least a wave per SIMD (1024 SIMDs x 64 lanes)
    uint32_t stop = 1;
    for (uint32_t m = W; m >= 2; m /= 2)
        if ((uint64_t)c * 2 * W * (m / 2) < 65536) {
            stop = m;
            break;
        }
    int rc;
    const bool cu_split = rs_cus_ > 0 && !profiling_;
    if (cu_split && (rc = make_cu_streams())) return rc;
    // RS chunks: on aux_stream_, or (CU split) chunk 0 on the whole chip (s)
    // and the rest on the RS CUs; hashing on s, or on the complement CUs
    hipStream_t rs_q = cu_split ? rs_cu_stream_ : aux_stream_;
    hipStream_t hq = cu_split ? hash_cu_stream_ : s;
    hipEvent_t start = sync_event(0);
    if (!start || !sync_event(n_chunks + 1)) return fail(CDA_ERR_DEVICE, "hipEventCreate failed");
    if ((rc = dah_prepare(W, n, d_err, s))) return rc;
    if (cu_split) {
        if ((rc = enqueue_extend(d_ods, k, c, d_eds, s))) return rc;
        if ((rc = check(hipEventRecord(sync_event(1), s), "hipEventRecord"))) return rc;
    }
    if ((rc = check(hipEventRecord(start, s), "hipEventRecord"))) return rc;
    if ((rc = check(hipStreamWaitEvent(rs_q, start, 0), "hipStreamWaitEvent"))) return rc;
    for (uint32_t i = cu_split ? 1 : 0; i < n_chunks; i++) {
        const uint32_t i0 = i * c, m = (i0 + c <= n) ? c : n - i0;
        if ((rc = enqueue_extend(d_ods ? d_ods + i0 * ods_sq : nullptr, k, m, d_eds + i0 * eds_sq, rs_q)))
            return rc;   // rs_q is joined by the caller's drain (guarded_on)
        if (fault_at("extend_chunk"))
            return fail(CDA_ERR_DEVICE, "enqueue_extend_dah: injected fault after a chunk's RS (CDA_FAULT=extend_chunk)");
        hipEvent_t ev = sync_event(1 + i);
        if ((rc = check(hipEventRecord(ev, rs_q), "hipEventRecord"))) return rc;
    }
    Forest f[2], post[2];
    dah_forests(W, d_rows, d_cols, f);
    for (uint32_t i = 0; i < n_chunks; i++) {
        const uint32_t i0 = i * c, m = (i0 + c <= n) ? c : n - i0;
        if ((rc = check(hipStreamWaitEvent(hq, sync_event(1 + i), 0), "hipStreamWaitEvent"))) return rc;
        Forest p[2];
        if ((rc = dah_chunk(d_eds, k, i0, m, stop, d_err, f, p, hq))) return rc;
        if (i == 0) {
            post[0] = p[0];
            post[1] = p[1];
        }
    }
    if (cu_split) {   // the latency-bound rest on the whole chip, in order on s
        hipEvent_t done = sync_event(n_chunks + 1);
        if ((rc = check(hipEventRecord(done, hq), "hipEventRecord"))) return rc;
        if ((rc = check(hipStreamWaitEvent(s, done, 0), "hipStreamWaitEvent"))) return rc;
    }
    return dah_finish(k, 0, n, stop, post, d_roots, d_err, d_status, s);
}

int Engine::enqueue_rs(const uint8_t* d_data, uint8_t* d_parity, uint32_t k, uint32_t len, uint32_t n,
                       hipStream_t s) {
    if (len % 64) {
        char buf[96];
        snprintf(buf, sizeof buf, "chunkSize %u must be a multiple of 64 bytes", len);
        return fail(CDA_ERR_CHUNK_SIZE, buf);
    }
    if (k == 0) return fail(CDA_ERR_UNSUPPORTED, "no shards");
    if (k > 1024) return fail(CDA_ERR_UNSUPPORTED, "more than 2048 shards");
    if (!pow2(k)) {
        // klauspost leopardFF8/16 encode with dataShards = parityShards = k:
        // m = ceilPow2(k); the IFFT reads k data shards and zeros up to m
        // (ifftDITEncoder's mtrunc), the FFT's first k outputs are the parity.
        // Same result: encode the zero-padded m-shard codeword, keep k shards.
        uint32_t m = 1;
        while (m < k) m <<= 1;
        const size_t in_cw = (size_t)k * len, pad_cw = (size_t)m * len;
        int rc;
        if ((rc = check(rs_pad_.ensure(2 * pad_cw * n), "hipMalloc rs padding"))) return rc;
        uint8_t* pad_in = rs_pad_.as<uint8_t>();
        uint8_t* pad_out = pad_in + pad_cw * n;
        if ((rc = check(hipMemsetAsync(pad_in, 0, pad_cw * n, s), "hipMemsetAsync"))) return rc;
        if ((rc = check(hipMemcpy2DAsync(pad_in, pad_cw, d_data, in_cw, in_cw, n, hipMemcpyDeviceToDevice, s),
                        "copy")))
            return rc;
        if ((rc = enqueue_rs(pad_in, pad_out, m, len, n, s))) return rc;
        return check(hipMemcpy2DAsync(d_parity, in_cw, pad_out, pad_cw, in_cw, n, hipMemcpyDeviceToDevice, s), "copy");
    }
    if (k == 1)
        return check(hipMemcpyAsync(d_parity, d_data, (size_t)len * n, hipMemcpyDeviceToDevice, s), "copy");
    if (k <= 128) return check(launch_rs8_flat(d_data, d_parity, k, len, n, s), "rs8 flat");
    return check(launch_rs16_flat(gf16(k), d_data, d_parity, k, len, n, s), "rs16 flat");
}

// cda_push_order_detail_at: the decoded push-order word of square sq of the
// last device batch, once that batch's GPU work (the call's end event) is done.
int Engine::device_push_order_detail(uint32_t sq, int32_t* axis, uint32_t* index, uint32_t* pos) {
    if (sq >= dev_err_n_) return fail(CDA_ERR_INVALID, "square index beyond the last device batch");
    int rc;
    if (order_used_ && order_ev_ && (rc = check(hipEventSynchronize(order_ev_), "hipEventSynchronize (last call)")))
        return rc;
    uint32_t w = 0xFFFFFFFFu;
    if ((rc = check(hipMemcpyAsync(&w, dev_err_.as<uint32_t>() + sq, 4, hipMemcpyDeviceToHost, stream_),
                    "hipMemcpyAsync push-order word")))
        return rc;
    if ((rc = check(hipStreamSynchronize(stream_), "hipStreamSynchronize"))) return rc;
    if (w == 0xFFFFFFFFu) {
        *axis = -1;
        *index = *pos = 0;
    } else {
        *axis = (int32_t)(w >> 24);
        *index = (w >> 12) & 0xFFF;
        *pos = w & 0xFFF;
    }
    return CDA_OK;
}

// Build the reference's error text for the first violating square.
int Engine::push_order_error(const uint32_t* err_words, uint32_t n, const uint8_t* src, uint32_t k,
                             bool src_is_eds) {
    for (uint32_t sq = 0; sq < n; sq++) {
        const uint32_t e = err_words[sq];
        if (e == 0xFFFFFFFFu) continue;
        po_axis = (int32_t)(e >> 24);
        po_index = (e >> 12) & 0xFFF;
        po_pos = e & 0xFFF;
        const uint32_t w = src_is_eds ? 2 * k : k;
        const uint8_t* base = src + (size_t)sq * w * w * kShare;
        auto cell = [&](uint32_t pos) {
            const uint32_t r = po_axis == 0 ? po_index : pos, c = po_axis == 0 ? pos : po_index;
            return base + ((size_t)r * w + c) * kShare;
        };
        std::string msg = "pushed data has to be lexicographically ordered by namespace IDs: last namespace: ";
        char hx[3];
        const uint8_t* last = cell(po_pos - 1);
        const uint8_t* pushed = cell(po_pos);
        for (int i = 0; i < kNs; i++) { snprintf(hx, sizeof hx, "%02x", last[i]); msg += hx; }
        msg += ", pushed: ";
        for (int i = 0; i < kNs; i++) { snprintf(hx, sizeof hx, "%02x", pushed[i]); msg += hx; }
        return fail(CDA_ERR_PUSH_ORDER, msg);
    }
    return CDA_OK;
}

// Host-buffer extension.  The EDS goes back over PCIe as its three parity
// quadrants only: Q0 IS the caller's ODS, so the host copies it itself while
// the GPU works (24 instead of 32 MiB over the link per k = 128 square), and
// the parity copies start as soon as the RS launches finish, on copy_out_,
// overlapping the NMT hashing on stream_.
// Host copy of the ODS rows into Q0 of the caller's EDS, on a few host
// threads (one core copies ~10 GB/s: a 16-square k = 128 batch's 128 MiB
// would outlast the PCIe copies it runs beside).  CDA_HOST_THREADS caps them.
void Engine::copy_q0(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds) {
    const size_t row = (size_t)k * kShare, W = 2 * (size_t)k;
    const size_t rows = (size_t)n * k;
    static const unsigned cap = [] {
        const char* e = deploy_knob("CDA_HOST_THREADS");
        const unsigned hw = std::thread::hardware_concurrency();
        unsigned v = e ? (unsigned)atoi(e) : 8u;
        if (hw && v > hw) v = hw;
        return v ? v : 1u;
    }();
    const unsigned nt = (unsigned)std::min<size_t>(cap, std::max<size_t>(1, rows * row / (2u << 20)));
    // streaming stores (CDA_HOST_NT, default on): the EDS rows are not read
    // back here, so skip the read-for-ownership of every destination line
    static const bool nt_stores = [] {
        const char* e = test_knob("CDA_HOST_NT");
        return e ? atoi(e) != 0 : true;
    }();
    auto part = [&](unsigned t) {
        for (size_t i = rows * t / nt; i < rows * (t + 1) / nt; i++) {
            const size_t sq = i / k, r = i % k;
            uint8_t* dst = eds + (sq * W * W + r * W) * kShare;
            const uint8_t* src = ods + i * row;
            if (!nt_stores || ((uintptr_t)dst | (uintptr_t)src) & 15) {
                memcpy(dst, src, row);
                continue;
            }
            for (size_t o = 0; o < row; o += 64) {   // rows are whole shares (512 B)
                const __m128i a = _mm_load_si128((const __m128i*)(src + o)),
                              b = _mm_load_si128((const __m128i*)(src + o + 16)),
                              c = _mm_load_si128((const __m128i*)(src + o + 32)),
                              d = _mm_load_si128((const __m128i*)(src + o + 48));
                _mm_stream_si128((__m128i*)(dst + o), a);
                _mm_stream_si128((__m128i*)(dst + o + 16), b);
                _mm_stream_si128((__m128i*)(dst + o + 32), c);
                _mm_stream_si128((__m128i*)(dst + o + 48), d);
            }
        }
        _mm_sfence();
    };
    std::vector<std::thread> th;
    unsigned started = 1;   // parts [0, started) have a thread (part 0: the caller)
    try {
        th.reserve(nt);
        for (unsigned t = 1; t < nt; t++, started++) th.emplace_back(part, t);
    } catch (...) {   // no more threads (std::system_error) or memory: copy the rest here
    }
    part(0);
    for (unsigned t = started; t < nt; t++) part(t);
    for (auto& x : th) x.join();
}

// Packed parity of n squares (eds_mode PARITY): per square Q1 as k rows of k
// shares, then EDS rows k..2k-1 (Q2 | Q3) whole -- 3 k^2 shares, contiguous,
// so the chunk's parity leaves in ONE linear device-to-host copy instead of a
// strided Q1 copy and a linear Q2 | Q3 copy per square (each copy costs a
// ~30 us turnaround on the DMA engine, profiles/r04/host_pipe_trace.txt).
// One thread per 16 bytes.
__global__ __launch_bounds__(256) void pack_parity_kernel(const uint8_t* __restrict__ eds, uint8_t* __restrict__ par,
                                                         uint32_t k, uint64_t total16) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total16) return;
    constexpr uint32_t V = kShare / 16;
    const uint64_t W = 2 * (uint64_t)k, per_sq = 3 * (uint64_t)k * k * V;
    const uint64_t sq = i / per_sq, j = i % per_sq;
    const uint64_t q1 = (uint64_t)k * k * V;
    uint64_t src;   // in uint4 units within the square
    if (j < q1) {
        const uint64_t cell = j / V, r = cell / k, c = cell % k;
        src = (r * W + k + c) * V + j % V;
    } else {
        src = (uint64_t)k * W * V + (j - q1);
    }
    reinterpret_cast<uint4*>(par)[i] = reinterpret_cast<const uint4*>(eds + sq * W * W * kShare)[src];
}

int Engine::enqueue_parity_d2h(const uint8_t* d_eds, uint32_t k, uint32_t n, uint8_t* eds, hipStream_t from,
                               hipEvent_t ready, hipEvent_t done, int eds_mode, uint8_t* d_par) {
    const size_t W = 2 * (size_t)k, sq_b = W * W * kShare, half = k * W * kShare;
    int rc;
    const size_t par_b = (size_t)n * 3 * k * k * kShare;
    if (eds_mode == CDA_EDS_PARITY) {
        // pack on the compute stream right behind the RS (a few hundred us per
        // 32 squares, where the compute stream has slack against the copies),
        // so the copy stream runs nothing but back-to-back linear copies
        const uint64_t total16 = par_b / 16;
        hipLaunchKernelGGL(pack_parity_kernel, dim3((uint32_t)((total16 + 255) / 256)), dim3(256), 0, from, d_eds,
                           d_par, k, total16);
        if ((rc = check(hipGetLastError(), "pack parity"))) return rc;
    }
    if ((rc = check(hipEventRecord(ready, from), "hipEventRecord"))) return rc;
    if ((rc = check(hipStreamWaitEvent(copy_out_, ready, 0), "hipStreamWaitEvent"))) return rc;
    if (eds_mode == CDA_EDS_PARITY) {
        if ((rc = check(hipMemcpyAsync(eds, d_par, par_b, hipMemcpyDeviceToHost, copy_out_), "D2H parity"))) return rc;
        return check(hipEventRecord(done, copy_out_), "hipEventRecord");
    }
    if (host_full_d2h_ && eds_mode == CDA_EDS_FULL) {   // the whole EDS back as one contiguous copy (Q0 included)
        if ((rc = check(hipMemcpyAsync(eds, d_eds, n * sq_b, hipMemcpyDeviceToHost, copy_out_), "D2H EDS"))) return rc;
        return check(hipEventRecord(done, copy_out_), "hipEventRecord");
    }
    // Q1 (rows 0..k-1, columns k..2k-1: strided) as 2-D copies, Q2|Q3 (rows
    // k..2k-1) linear (a second stream for the Q1 copies measured no faster:
    // profiles/r04/host_d2h_streams.txt)
    for (uint32_t sq = 0; sq < n; sq++) {
        if ((rc = check(hipMemcpy2DAsync(eds + sq * sq_b + k * kShare, W * kShare, d_eds + sq * sq_b + k * kShare,
                                         W * kShare, (size_t)k * kShare, k, hipMemcpyDeviceToHost, copy_out_),
                        "D2H Q1")))
            return rc;
        if ((rc = check(hipMemcpyAsync(eds + sq * sq_b + half, d_eds + sq * sq_b + half, half, hipMemcpyDeviceToHost,
                                       copy_out_),
                        "D2H Q2|Q3")))
            return rc;
    }
    return check(hipEventRecord(done, copy_out_), "hipEventRecord");
}

// Big batches from host buffers (config 4 through the C ABI as a Go caller
// would drive it: pkg/da/data_availability_header.go:65-75 takes host shares,
// returns a host EDS).  Chunk i (slot i % kPipeSlots):
//   copy_in_ : wait until chunk i - slots finished computing (its ODS slot is
//              free), H2D of the chunk's ODS                        -> pipe_in_
//   stream_  : wait for the H2D, and for chunk i - slots's parity to have left
//              the EDS slot; RS                                      -> pipe_rs_
//   copy_out_: wait for the RS, D2H of the three parity quadrants     -> pipe_d2h_
//   stream_  : leaves, levels, roots and data roots of the chunk    -> pipe_comp_
// so the H2D of chunk i+1, the compute of chunk i and the D2H of chunk i-1
// run at once (PCIe is full duplex); the host copies Q0 (= the caller's ODS)
// on its own threads meanwhile.
int Engine::host_pipeline(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, uint8_t* rows, uint8_t* cols,
                          uint8_t* roots, int32_t* status, uint32_t c, int eds_mode) {
    const uint32_t W = 2 * k;
    const size_t ods_sq = (size_t)k * k * kShare, eds_sq = (size_t)W * W * kShare, root_sq = (size_t)W * kNode;
    const bool packed = eds && eds_mode == CDA_EDS_PARITY;
    const size_t out_sq = packed ? 3 * ods_sq : eds_sq;   // bytes per square of the caller's eds buffer
    int rc;
    if ((rc = check(h_ods_.ensure(kPipeSlots * c * ods_sq), "hipMalloc"))) return rc;
    if ((rc = check(h_eds_.ensure(kPipeSlots * c * eds_sq), "hipMalloc"))) return rc;
    if (packed && (rc = check(h_par_.ensure(kPipeSlots * c * 3 * ods_sq), "hipMalloc"))) return rc;
    if ((rc = check(h_rows_.ensure(n * root_sq), "hipMalloc"))) return rc;
    if ((rc = check(h_cols_.ensure(n * root_sq), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure((size_t)n * 32), "hipMalloc"))) return rc;
    if ((rc = check(err_buf_.ensure((size_t)n * 4), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    // the buffers' allocation (stream-ordered on s) precedes the copies
    if ((rc = check(hipEventRecord(pipe_comp_[0], s), "hipEventRecord"))) return rc;
    if ((rc = check(hipStreamWaitEvent(copy_in_, pipe_comp_[0], 0), "hipStreamWaitEvent"))) return rc;
    HostPin pin_ods(host_register_, ods, (size_t)n * ods_sq, copy_in_, s),
        pin_eds(host_register_, eds, (size_t)n * out_sq, s, copy_out_);
    uint32_t* err = err_buf_.as<uint32_t>();
    for (uint32_t i = 0, i0 = 0; i0 < n; i++, i0 += c) {
        const uint32_t m = std::min(c, n - i0), slot = i % kPipeSlots;
        uint8_t* d_ods = h_ods_.as<uint8_t>() + slot * c * ods_sq;
        uint8_t* d_eds = h_eds_.as<uint8_t>() + slot * c * eds_sq;
        if (i >= kPipeSlots && (rc = check(hipStreamWaitEvent(copy_in_, pipe_comp_[slot], 0), "hipStreamWaitEvent")))
            return rc;
        if ((rc = check(hipMemcpyAsync(d_ods, ods + i0 * ods_sq, m * ods_sq, hipMemcpyHostToDevice, copy_in_), "H2D")))
            return rc;
        if ((rc = check(hipEventRecord(pipe_in_[slot], copy_in_), "hipEventRecord"))) return rc;
        if ((rc = check(hipStreamWaitEvent(s, pipe_in_[slot], 0), "hipStreamWaitEvent"))) return rc;
        if (eds && i >= kPipeSlots && (rc = check(hipStreamWaitEvent(s, pipe_d2h_[slot], 0), "hipStreamWaitEvent")))
            return rc;
        if ((rc = enqueue_extend(d_ods, k, m, d_eds, s, err + i0))) return rc;
        if (eds && (rc = enqueue_parity_d2h(d_eds, k, m, eds + i0 * out_sq, s, pipe_rs_[slot], pipe_d2h_[slot],
                                            eds_mode, packed ? h_par_.as<uint8_t>() + slot * c * 3 * ods_sq : nullptr)))
            return rc;
        if ((rc = enqueue_dah(d_eds, k, m, h_rows_.as<uint8_t>() + i0 * root_sq, h_cols_.as<uint8_t>() + i0 * root_sq,
                              h_roots_.as<uint8_t>() + (size_t)i0 * 32, err + i0, nullptr, s, true)))
            return rc;
        if ((rc = check(hipEventRecord(pipe_comp_[slot], s), "hipEventRecord"))) return rc;
        // (an error return leaves copies queued on copy_in_ / copy_out_: the
        // caller's drain (guarded_on) waits for them before the call returns)
        if (i == 1 && fault_at("pipe_chunk"))
            return fail(CDA_ERR_DEVICE, "host_pipeline: injected fault after chunk 1 (CDA_FAULT=pipe_chunk)");
    }
    if ((rc = check(hipMemcpyAsync(rows, h_rows_.ptr, n * root_sq, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(cols, h_cols_.ptr, n * root_sq, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(roots, h_roots_.ptr, (size_t)n * 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    std::vector<uint32_t> words(n);
    if ((rc = check(hipMemcpyAsync(words.data(), err, (size_t)n * 4, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if (eds && eds_mode == CDA_EDS_FULL && !host_full_d2h_) copy_q0(ods, k, n, eds);   // host work while the GPU runs
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    if (eds && (rc = check(hipStreamSynchronize(copy_out_), "hipStreamSynchronize"))) return rc;
    if (status)
        for (uint32_t i = 0; i < n; i++) status[i] = words[i] == 0xFFFFFFFFu ? CDA_OK : CDA_ERR_PUSH_ORDER;
    return push_order_error(words.data(), n, ods, k, false);
}

int Engine::host_extend_dah(const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, uint8_t* rows, uint8_t* cols,
                            uint8_t* roots, int32_t* status, int eds_mode) {
    if (eds_mode != CDA_EDS_FULL && eds_mode != CDA_EDS_SKIP_Q0 && eds_mode != CDA_EDS_PARITY)
        return fail(CDA_ERR_INVALID, "unknown eds_mode");
    const uint32_t W = 2 * k;
    const size_t ods_b = (size_t)n * k * k * kShare, eds_b = (size_t)n * W * W * kShare;
    const size_t roots_b = (size_t)n * W * kNode;
    const bool packed = eds && eds_mode == CDA_EDS_PARITY;
    {   // big batches: the chunk pipeline (chunk ~ 256 MiB of ODS: 32 squares at k = 128)
        const size_t ods_sq = (size_t)k * k * kShare;
        const uint32_t c = host_pipe_chunk_ ? host_pipe_chunk_ : (uint32_t)std::max<size_t>(1, (256u << 20) / ods_sq);
        if (n > 2 * c) return host_pipeline(ods, k, n, eds, rows, cols, roots, status, c, eds_mode);
    }
    int rc;
    if ((rc = check(h_ods_.ensure(ods_b), "hipMalloc"))) return rc;
    if ((rc = check(h_eds_.ensure(eds_b), "hipMalloc"))) return rc;
    if ((rc = check(h_rows_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_cols_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure((size_t)n * 32), "hipMalloc"))) return rc;
    if ((rc = check(err_buf_.ensure((size_t)n * 4), "hipMalloc"))) return rc;
    if (packed && (rc = check(h_par_.ensure(3 * ods_b), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    HostPin pin_ods(host_register_, ods, ods_b, stream_, copy_out_),
        pin_eds(host_register_, eds, packed ? 3 * ods_b : eds_b, stream_, copy_out_);
    // With the EDS going back, the batch moves in chunks: chunk i+1's ODS goes
    // up while chunk i's parity comes down (PCIe is full duplex); without
    // chunks every H2D would precede every D2H.  CDA_HOST_CHUNK (squares,
    // 0 = whole batch).
    const size_t ods_sq = (size_t)k * k * kShare, eds_sq = (size_t)W * W * kShare;
    const uint32_t c = eds && host_chunk_ && n > host_chunk_ ? host_chunk_ : n;
    for (uint32_t i0 = 0; i0 < n; i0 += c) {
        const uint32_t m = std::min(c, n - i0);
        if ((rc = check(hipMemcpyAsync(h_ods_.as<uint8_t>() + i0 * ods_sq, ods + i0 * ods_sq, m * ods_sq,
                                       hipMemcpyHostToDevice, s),
                        "H2D")))
            return rc;
        if ((rc = enqueue_extend(h_ods_.as<uint8_t>() + i0 * ods_sq, k, m, h_eds_.as<uint8_t>() + i0 * eds_sq, s,
                                 err_buf_.as<uint32_t>() + i0)))
            return rc;
        if (eds && (rc = enqueue_parity_d2h(h_eds_.as<uint8_t>() + i0 * eds_sq, k, m,
                                            eds + i0 * (packed ? 3 * ods_sq : eds_sq), s, ev_rs_, ev_out_, eds_mode,
                                            packed ? h_par_.as<uint8_t>() + i0 * 3 * ods_sq : nullptr)))
            return rc;
    }
    if ((rc = enqueue_dah(h_eds_.as<uint8_t>(), k, n, h_rows_.as<uint8_t>(), h_cols_.as<uint8_t>(),
                          h_roots_.as<uint8_t>(), err_buf_.as<uint32_t>(), nullptr, s, true)))
        return rc;
    if ((rc = check(hipMemcpyAsync(rows, h_rows_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(cols, h_cols_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(roots, h_roots_.ptr, (size_t)n * 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    std::vector<uint32_t> err(n);
    if ((rc = check(hipMemcpyAsync(err.data(), err_buf_.ptr, (size_t)n * 4, hipMemcpyDeviceToHost, s), "D2H")))
        return rc;
    if (eds && eds_mode == CDA_EDS_FULL && !host_full_d2h_) copy_q0(ods, k, n, eds);   // host work while the GPU runs
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    if (eds && (rc = check(hipEventSynchronize(ev_out_), "hipEventSynchronize"))) return rc;
    if (status)
        for (uint32_t i = 0; i < n; i++) status[i] = err[i] == 0xFFFFFFFFu ? CDA_OK : CDA_ERR_PUSH_ORDER;
    return push_order_error(err.data(), n, ods, k, false);
}

int Engine::host_extend(const uint8_t* ods, uint32_t k, uint8_t* eds) {
    const uint32_t W = 2 * k;
    const size_t ods_b = (size_t)k * k * kShare, eds_b = (size_t)W * W * kShare;
    int rc;
    if ((rc = check(h_ods_.ensure(ods_b), "hipMalloc"))) return rc;
    if ((rc = check(h_eds_.ensure(eds_b), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    HostPin pin_ods(host_register_, ods, ods_b, stream_, copy_out_),
        pin_eds(host_register_, eds, eds_b, stream_, copy_out_);
    if ((rc = check(hipMemcpyAsync(h_ods_.ptr, ods, ods_b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = enqueue_extend(h_ods_.as<uint8_t>(), k, 1, h_eds_.as<uint8_t>(), s))) return rc;
    if ((rc = enqueue_parity_d2h(h_eds_.as<uint8_t>(), k, 1, eds, s, ev_rs_, ev_out_))) return rc;
    copy_q0(ods, k, 1, eds);
    return check(hipEventSynchronize(ev_out_), "hipEventSynchronize");
}

int Engine::host_dah(const uint8_t* eds, uint32_t k, uint8_t* rows, uint8_t* cols, uint8_t* root) {
    const uint32_t W = 2 * k;
    const size_t eds_b = (size_t)W * W * kShare, roots_b = (size_t)W * kNode;
    int rc;
    if ((rc = check(h_eds_.ensure(eds_b), "hipMalloc"))) return rc;
    if ((rc = check(h_rows_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_cols_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure(32), "hipMalloc"))) return rc;
    if ((rc = check(err_buf_.ensure(4), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    HostPin pin_eds(host_register_, eds, eds_b, stream_, copy_out_);
    if ((rc = check(hipMemcpyAsync(h_eds_.ptr, eds, eds_b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = enqueue_dah(h_eds_.as<uint8_t>(), k, 1, h_rows_.as<uint8_t>(), h_cols_.as<uint8_t>(),
                          h_roots_.as<uint8_t>(), err_buf_.as<uint32_t>(), nullptr, s)))
        return rc;
    uint32_t err = 0;
    if ((rc = check(hipMemcpyAsync(rows, h_rows_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(cols, h_cols_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(root, h_roots_.ptr, 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(&err, err_buf_.ptr, 4, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    return push_order_error(&err, 1, eds, k, true);
}

int Engine::host_rs(const uint8_t* data, uint32_t k, uint32_t len, uint32_t n, uint8_t* parity) {
    const size_t b = (size_t)n * k * len;
    int rc;
    if ((rc = check(h_ods_.ensure(b), "hipMalloc"))) return rc;
    if ((rc = check(h_eds_.ensure(b), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    if ((rc = check(hipMemcpyAsync(h_ods_.ptr, data, b, hipMemcpyHostToDevice, s), "H2D"))) return rc;
    if ((rc = enqueue_rs(h_ods_.as<uint8_t>(), h_eds_.as<uint8_t>(), k, len, n, s))) return rc;
    if ((rc = check(hipMemcpyAsync(parity, h_eds_.ptr, b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

int Engine::host_data_root(const uint8_t* rows, const uint8_t* cols, uint32_t w, uint8_t* root) {
    // Pack the 90-B roots into 96-B slots (rows then columns) and reuse the
    // device RFC-6962 kernel.
    std::vector<uint8_t> slots((size_t)2 * w * kSlot, 0);
    for (uint32_t i = 0; i < w; i++) {
        memcpy(&slots[(size_t)i * kSlot], rows + (size_t)i * kNode, kNode);
        memcpy(&slots[(size_t)(w + i) * kSlot], cols + (size_t)i * kNode, kNode);
    }
    int rc;
    if ((rc = check(root_slots_.ensure(slots.size()), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure(32), "hipMalloc"))) return rc;
    hipStream_t s = stream_;
    if ((rc = check(hipMemcpyAsync(root_slots_.ptr, slots.data(), slots.size(), hipMemcpyHostToDevice, s), "H2D")))
        return rc;
    if ((rc = check(launch_data_root(root_slots_.as<uint8_t>(), 2 * w, 1, h_roots_.as<uint8_t>(), s), "data root")))
        return rc;
    if ((rc = check(hipMemcpyAsync(root, h_roots_.ptr, 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace cda
