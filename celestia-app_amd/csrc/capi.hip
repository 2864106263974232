// capi.hip -- extern "C" entry points of libcda.so (declared in include/cda.h).
// Each function validates arguments the way the reference does, locks the
// context and forwards to cda::Engine.  No C++ exception or abort crosses the
// ABI.
#include <cmath>
#include <cstring>
#include <new>
#include <thread>
#include <utility>

#include "../../include/cda.h"
#include "engine.h"
#include "split_layout.h"

struct cda_ctx {
    cda::Engine eng;
    explicit cda_ctx(int dev) : eng(dev) {}
};

struct cda_square {
    cda_ctx* ctx;
    cda::ResidentSquare sq;
};

namespace {

// pkg/da/data_availability_header.go SquareSize + IsPowerOfTwo; a power of
// two that is not a square (8 shares) passes ExtendShares' check and fails in
// rsmt2d's newDataSquare instead
bool square_width(uint32_t n_shares, uint32_t* k) {
    if (n_shares == 0 || (n_shares & (n_shares - 1))) return false;
    uint32_t w = 1;
    while ((uint64_t)w * w < n_shares) w <<= 1;
    if ((uint64_t)w * w != n_shares) return false;
    *k = w;
    return true;
}

// The last call's error text and push-order details, per calling thread.  The
// context's own copy is overwritten by the next call on it (from any thread),
// so cda_last_error / cda_push_order_detail read this snapshot instead.
struct ThreadError {
    std::string msg;
    int32_t axis = -1;
    uint32_t index = 0, pos = 0;
};
thread_local ThreadError tl_err;

// A context may be driven from any OS thread (Go moves goroutines between
// threads): its device becomes current for the call and the caller's device
// is restored afterwards.
struct DeviceScope {
    int prev = -1, want;
    explicit DeviceScope(int d) : want(d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceScope() {
        if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
    }
};

// Lock the context, make its device current, order the call's GPU work after
// the previous call's (Engine::order_begin / order_end on the stream the call
// enqueues on: `stream`, or the context's private stream for host-buffer
// calls), run f and publish the error to the calling thread.
template <class F>
int guarded_on(cda_ctx* ctx, const hipStream_t* stream, F&& f) {
    if (!ctx) {
        tl_err.msg = "null context";
        return CDA_ERR_INVALID;
    }
    cda::Engine& e = ctx->eng;
    std::lock_guard<std::mutex> g(e.mutex());
    DeviceScope dev(e.device());
    e.clear_error();
    const hipStream_t s = stream ? *stream : e.stream();
    int rc;
    try {
        rc = e.order_begin(s);
        if (rc == CDA_OK) rc = f(e);
    } catch (const std::bad_alloc&) {
        rc = e.fail(CDA_ERR_OOM, "host allocation failed");
    } catch (...) {
        rc = e.fail(CDA_ERR_DEVICE, "unexpected exception");
    }
    // A failed call may have returned before joining its side streams (hash
    // split parts, RS chunks, the host pipeline's copies): wait for them here,
    // so nothing the call queued can still read a buffer that the next call
    // frees in stream order, or a host buffer the caller frees on return.
    // (Push-order results are complete answers, not failures.)
    if (rc != CDA_OK && rc != CDA_ERR_PUSH_ORDER) {
        const std::string msg = e.last_error();
        (void)e.drain_streams();
        e.fail(rc, msg);   // keep the call's own error text
    }
    e.order_end(s);
    tl_err.msg = e.last_error();
    if (rc == CDA_ERR_PUSH_ORDER) {
        tl_err.axis = e.po_axis;
        tl_err.index = e.po_index;
        tl_err.pos = e.po_pos;
    }
    return rc;
}

template <class F>
int guarded(cda_ctx* ctx, F&& f) {
    return guarded_on(ctx, nullptr, std::forward<F>(f));
}

// Device entry points enqueue on the caller's stream (NULL = HIP's default).
template <class F>
int guarded_stream(cda_ctx* ctx, void* stream, F&& f) {
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return guarded_on(ctx, &s, [&](cda::Engine& e) { return f(e, s); });
}

// The error of a share count square_width rejects: ExtendShares' own
// (data_availability_header.go:67-69), or rsmt2d's for a power of two that is
// not a square (newDataSquare, EXT v0.14.0).
int not_pow2(cda::Engine& e, uint32_t n) {
    if (n && !(n & (n - 1))) return e.fail(CDA_ERR_INVALID, "number of chunks must be a square number");
    char buf[96];
    snprintf(buf, sizeof buf, "number of shares is not a power of 2: got %u", n);
    return e.fail(CDA_ERR_NOT_POW2, buf);
}

int plan_square(const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs, uint32_t max_square_size,
                uint32_t threshold, int mode, cda::square::Plan* p, std::string* err) {
    if (mode != CDA_SQUARE_CONSTRUCT && mode != CDA_SQUARE_BUILD) {
        *err = "unknown square construction mode";
        return -1;
    }
    for (uint32_t i = 0; i < n_txs; i++)
        if (tx_off[i + 1] < tx_off[i]) {
            *err = "tx offsets must be non-decreasing";
            return -1;
        }
    return cda::square::plan(txs, tx_off, n_txs, max_square_size, threshold,
                             mode == CDA_SQUARE_BUILD ? cda::square::kBuild : cda::square::kConstruct, p, err);
}

}  // namespace

extern "C" {

const char* cda_version(void) { return cda::kTestBuild ? "cda 0.1.0 gfx950 test-build" : "cda 0.1.0 gfx950"; }

int cda_ctx_create(int device, cda_ctx** out) {
    if (!out) return CDA_ERR_INVALID;
    *out = nullptr;
    cda_ctx* c = new (std::nothrow) cda_ctx(device);
    if (!c) return CDA_ERR_OOM;
    int rc = c->eng.init();
    if (rc) {
        delete c;
        return rc;
    }
    *out = c;
    return CDA_OK;
}

int cda_ctx_destroy(cda_ctx* ctx) {
    delete ctx;
    return CDA_OK;
}

const char* cda_last_error(cda_ctx* ctx) {
    (void)ctx;   // per calling thread: the message of this thread's last call (include/cda.h)
    return tl_err.msg.c_str();
}

int cda_extend_shares(cda_ctx* ctx, const uint8_t* ods, uint32_t n_shares, uint8_t* eds) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        uint32_t k;
        if (!square_width(n_shares, &k)) return not_pow2(e, n_shares);
        if (!ods || !eds) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_extend(ods, k, eds);
    });
}

int cda_dah_from_eds(cda_ctx* ctx, const uint8_t* eds, uint32_t w, uint8_t* row_roots, uint8_t* col_roots,
                     uint8_t* data_root) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (w < 2 || (w & (w - 1))) return e.fail(CDA_ERR_INVALID, "EDS width must be a power of two >= 2");
        if (!eds || !row_roots || !col_roots || !data_root) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_dah(eds, w / 2, row_roots, col_roots, data_root);
    });
}

int cda_extend_dah(cda_ctx* ctx, const uint8_t* ods, uint32_t n_shares, uint8_t* eds, uint8_t* row_roots,
                   uint8_t* col_roots, uint8_t* data_root) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        uint32_t k;
        if (!square_width(n_shares, &k)) return not_pow2(e, n_shares);
        if (!ods || !row_roots || !col_roots || !data_root) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_extend_dah(ods, k, 1, eds, row_roots, col_roots, data_root, nullptr);
    });
}

int cda_extend_dah_batch(cda_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, uint8_t* row_roots,
                         uint8_t* col_roots, uint8_t* data_roots, int32_t* status) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (k == 0 || (k & (k - 1))) return not_pow2(e, k * k);
        if (n == 0) return CDA_OK;
        if (!ods || !row_roots || !col_roots || !data_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_extend_dah(ods, k, n, eds, row_roots, col_roots, data_roots, status);
    });
}

int cda_extend_dah_batch_ex(cda_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t n, uint8_t* eds, int eds_mode,
                            uint8_t* row_roots, uint8_t* col_roots, uint8_t* data_roots, int32_t* status) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (k == 0 || (k & (k - 1))) return not_pow2(e, k * k);
        if (eds_mode != CDA_EDS_FULL && eds_mode != CDA_EDS_SKIP_Q0 && eds_mode != CDA_EDS_PARITY)
            return e.fail(CDA_ERR_INVALID, "unknown eds_mode");
        if (n == 0) return CDA_OK;
        if (!ods || !row_roots || !col_roots || !data_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_extend_dah(ods, k, n, eds, row_roots, col_roots, data_roots, status, eds_mode);
    });
}

int cda_extend_dah_device(cda_ctx* ctx, const void* d_ods, uint32_t k, uint32_t n, void* d_eds, void* d_row_roots,
                          void* d_col_roots, void* d_data_roots, int32_t* d_status, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (k == 0 || (k & (k - 1))) return not_pow2(e, k * k);
        if (n == 0) return CDA_OK;
        if (!d_ods || !d_eds || !d_row_roots || !d_col_roots || !d_data_roots)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        uint32_t* err = e.err_words(n);
        if (!err) return e.fail(CDA_ERR_OOM, "hipMalloc err words");
        const int rc = e.enqueue_extend_dah(static_cast<const uint8_t*>(d_ods), k, n, static_cast<uint8_t*>(d_eds),
                                            static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                            static_cast<uint8_t*>(d_data_roots), err, d_status, s);
        e.set_device_batch(rc == CDA_OK ? n : 0);
        return rc;
    });
}

int cda_reserve(cda_ctx* ctx, uint32_t k, uint32_t n) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (k == 0 || (k & (k - 1)) || k > 1024) return not_pow2(e, k * k);
        return e.reserve(k, n);
    });
}

int cda_extend_dah_inplace_device(cda_ctx* ctx, uint32_t k, uint32_t n, void* d_eds, void* d_row_roots,
                                  void* d_col_roots, void* d_data_roots, int32_t* d_status, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (k == 0 || (k & (k - 1))) return not_pow2(e, k * k);
        if (n == 0) return CDA_OK;
        if (!d_eds || !d_row_roots || !d_col_roots || !d_data_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        uint32_t* err = e.err_words(n);
        if (!err) return e.fail(CDA_ERR_OOM, "hipMalloc err words");
        const int rc = e.enqueue_extend_dah(nullptr, k, n, static_cast<uint8_t*>(d_eds),
                                            static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                            static_cast<uint8_t*>(d_data_roots), err, d_status, s);
        e.set_device_batch(rc == CDA_OK ? n : 0);
        return rc;
    });
}

int cda_rs_encode(cda_ctx* ctx, const uint8_t* data, uint32_t n_shards, uint32_t shard_len, uint32_t n_codewords,
                  uint8_t* parity) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (n_codewords == 0) return CDA_OK;
        if (!data || !parity) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_rs(data, n_shards, shard_len, n_codewords, parity);
    });
}

int cda_data_root(cda_ctx* ctx, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t w, uint8_t* data_root) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!data_root) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (w == 0) {  // merkle.HashFromByteSlices(nil) = sha256("")
            static const uint8_t empty[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                              0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                              0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
            memcpy(data_root, empty, 32);
            return CDA_OK;
        }
        if (w & (w - 1)) return e.fail(CDA_ERR_UNSUPPORTED, "root count must be a power of two");
        if (!row_roots || !col_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_data_root(row_roots, col_roots, w, data_root);
    });
}

int cda_push_order_detail(cda_ctx* ctx, int32_t* axis, uint32_t* index, uint32_t* position) {
    if (!ctx) return CDA_ERR_INVALID;
    if (axis) *axis = tl_err.axis;
    if (index) *index = tl_err.index;
    if (position) *position = tl_err.pos;
    return CDA_OK;
}

int cda_push_order_detail_at(cda_ctx* ctx, uint32_t square, int32_t* axis, uint32_t* index, uint32_t* position) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!axis || !index || !position) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.device_push_order_detail(square, axis, index, position);
    });
}

int cda_split_rows(cda_ctx* ctx, const void* d_ods_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                   void* d_row_block, uint32_t* d_err, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (!d_ods_rows || !d_row_block || !d_err) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.enqueue_split_rows(static_cast<const uint8_t*>(d_ods_rows), k, n_rows, row0,
                                    static_cast<uint8_t*>(d_row_block), d_err, s);
    });
}

int cda_split_cols(cda_ctx* ctx, void* d_col_block, uint32_t k, uint32_t n_cols, uint32_t col0,
                   void* d_col_root_slots, void* d_row_subtree_slots, uint32_t* d_err, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (!d_col_block || !d_col_root_slots || !d_row_subtree_slots || !d_err)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.enqueue_split_cols(static_cast<uint8_t*>(d_col_block), k, n_cols, col0,
                                    static_cast<uint8_t*>(d_col_root_slots), static_cast<uint8_t*>(d_row_subtree_slots),
                                    d_err, s);
    });
}

int cda_split_combine(cda_ctx* ctx, const void* d_row_subtree_slots, uint32_t parts, uint32_t k,
                      const void* d_col_root_slots, void* d_row_roots, void* d_col_roots, void* d_data_root,
                      void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (!d_row_subtree_slots || !d_col_root_slots || !d_row_roots || !d_col_roots || !d_data_root)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.enqueue_split_combine(static_cast<const uint8_t*>(d_row_subtree_slots), parts, k,
                                       static_cast<const uint8_t*>(d_col_root_slots),
                                       static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                       static_cast<uint8_t*>(d_data_root), s);
    });
}

int cda_square_tx_share_range(cda_ctx* ctx, const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs,
                              uint32_t max_square_size, uint32_t threshold, uint32_t tx_index, uint32_t* start,
                              uint32_t* end, int* is_pfb) {
    // Host-only (no device work): usable without a context.
    auto run = [&](std::string* err) -> int {
        if (!start || !end || (n_txs && (!txs || !tx_off))) {
            *err = "null buffer";
            return CDA_ERR_INVALID;
        }
        cda::square::Plan p;
        if (plan_square(txs, tx_off, n_txs, max_square_size, threshold, CDA_SQUARE_CONSTRUCT, &p, err))
            return CDA_ERR_SQUARE;
        if (tx_index >= p.unit_start.size()) {
            char b[64];
            snprintf(b, sizeof b, "txIndex %u out of range", tx_index);
            *err = b;
            return CDA_ERR_INVALID;
        }
        *start = p.unit_start[tx_index];
        *end = p.unit_end[tx_index];
        if (is_pfb) *is_pfb = tx_index >= p.n_normal;
        return CDA_OK;
    };
    if (!ctx) {
        tl_err.msg.clear();
        try {
            return run(&tl_err.msg);
        } catch (const std::bad_alloc&) {
            tl_err.msg = "host allocation failed";
            return CDA_ERR_OOM;
        }
    }
    return guarded(ctx, [&](cda::Engine& e) -> int {
        std::string err;
        const int rc = run(&err);
        return rc ? e.fail(rc, err) : CDA_OK;
    });
}

int cda_square_layout(cda_ctx* ctx, const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs,
                      uint32_t max_square_size, uint32_t threshold, int mode, uint32_t* square_size, uint32_t* kept,
                      uint32_t* n_kept, uint32_t* share_indexes, uint32_t share_index_cap, uint32_t* n_share_indexes) {
    // Host-only (no device work): usable without a context.
    auto run = [&](std::string* err) -> int {
        if (!square_size || (n_txs && (!txs || !tx_off))) {
            *err = "null buffer";
            return CDA_ERR_INVALID;
        }
        cda::square::Plan p;
        if (plan_square(txs, tx_off, n_txs, max_square_size, threshold, mode, &p, err)) return CDA_ERR_SQUARE;
        *square_size = p.square_size;
        if (kept) {
            memcpy(kept, p.kept.data(), p.kept.size() * 4);
            if (n_kept) *n_kept = (uint32_t)p.kept.size();
        }
        if (n_share_indexes) *n_share_indexes = (uint32_t)p.share_indexes.size();
        if (share_indexes) {
            if (p.share_indexes.size() > share_index_cap) {
                *err = "share_indexes capacity too small";
                return CDA_ERR_INVALID;
            }
            memcpy(share_indexes, p.share_indexes.data(), p.share_indexes.size() * 4);
        }
        return CDA_OK;
    };
    if (!ctx) {
        tl_err.msg.clear();
        try {
            return run(&tl_err.msg);
        } catch (const std::bad_alloc&) {
            tl_err.msg = "host allocation failed";
            return CDA_ERR_OOM;
        }
    }
    return guarded(ctx, [&](cda::Engine& e) -> int {
        std::string err;
        const int rc = run(&err);
        return rc ? e.fail(rc, err) : CDA_OK;
    });
}

int cda_square_construct(cda_ctx* ctx, const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs,
                         uint32_t max_square_size, uint32_t threshold, int mode, uint8_t* ods, size_t ods_capacity,
                         uint32_t* square_size, uint32_t* kept, uint32_t* n_kept) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!ods || !square_size || (n_txs && (!txs || !tx_off))) return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::square::Plan p;
        std::string err;
        if (plan_square(txs, tx_off, n_txs, max_square_size, threshold, mode, &p, &err))
            return e.fail(CDA_ERR_SQUARE, err);
        *square_size = p.square_size;
        if (kept) {
            memcpy(kept, p.kept.data(), p.kept.size() * 4);
            if (n_kept) *n_kept = (uint32_t)p.kept.size();
        }
        if ((size_t)p.square_size * p.square_size * CDA_SHARE_SIZE > ods_capacity)
            return e.fail(CDA_ERR_INVALID, "ods capacity too small for the square");
        return e.host_square(p, txs, n_txs ? tx_off[n_txs] : 0, ods);
    });
}

int cda_construct_extend_dah(cda_ctx* ctx, const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs,
                             uint32_t max_square_size, uint32_t threshold, int mode, uint8_t* eds, size_t eds_capacity,
                             uint8_t* row_roots, uint8_t* col_roots, size_t roots_capacity, uint8_t* data_root,
                             uint32_t* square_size, uint32_t* kept, uint32_t* n_kept) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!row_roots || !col_roots || !data_root || !square_size || (n_txs && (!txs || !tx_off)))
            return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::square::Plan p;
        std::string err;
        if (plan_square(txs, tx_off, n_txs, max_square_size, threshold, mode, &p, &err))
            return e.fail(CDA_ERR_SQUARE, err);
        *square_size = p.square_size;
        if (kept) {
            memcpy(kept, p.kept.data(), p.kept.size() * 4);
            if (n_kept) *n_kept = (uint32_t)p.kept.size();
        }
        const size_t w = 2 * (size_t)p.square_size;
        if (w * CDA_NMT_ROOT_SIZE > roots_capacity) return e.fail(CDA_ERR_INVALID, "roots capacity too small");
        if (eds && w * w * CDA_SHARE_SIZE > eds_capacity) return e.fail(CDA_ERR_INVALID, "eds capacity too small");
        return e.host_construct_extend_dah(p, txs, n_txs ? tx_off[n_txs] : 0, eds, row_roots, col_roots, data_root);
    });
}

int cda_square_construct_device(cda_ctx* ctx, const uint8_t* txs, const uint64_t* tx_off, uint32_t n_txs,
                                const void* d_txs, uint32_t max_square_size, uint32_t threshold, int mode,
                                void* d_ods, size_t ods_capacity, uint32_t* square_size, uint32_t* kept,
                                uint32_t* n_kept, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (!d_ods || !square_size || (n_txs && (!txs || !tx_off || !d_txs)))
            return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::square::Plan p;
        std::string err;
        if (plan_square(txs, tx_off, n_txs, max_square_size, threshold, mode, &p, &err))
            return e.fail(CDA_ERR_SQUARE, err);
        *square_size = p.square_size;
        if (kept) {
            memcpy(kept, p.kept.data(), p.kept.size() * 4);
            if (n_kept) *n_kept = (uint32_t)p.kept.size();
        }
        if ((size_t)p.square_size * p.square_size * CDA_SHARE_SIZE > ods_capacity)
            return e.fail(CDA_ERR_INVALID, "ods capacity too small for the square");
        return e.enqueue_square(p, static_cast<const uint8_t*>(d_txs), static_cast<uint8_t*>(d_ods), s);
    });
}

int cda_blob_commitments(cda_ctx* ctx, const uint8_t* namespaces, const uint8_t* data, const uint64_t* data_off,
                         const uint8_t* share_versions, uint32_t n, uint32_t threshold, uint8_t* commitments) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (n == 0) return CDA_OK;
        if (!namespaces || !data_off || !commitments || (data_off[n] > data_off[0] && !data))
            return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::square::CommitPlan& p = e.commit_plan();
        std::string err;
        if (cda::square::plan_commitments(namespaces, data_off, share_versions, n, threshold, &p, &err))
            return e.fail(CDA_ERR_SQUARE, err);
        return e.host_commitments(p, n, data, (size_t)data_off[n], commitments);
    });
}

int cda_blob_commitments_device(cda_ctx* ctx, const uint8_t* namespaces, const uint64_t* data_off,
                                const uint8_t* share_versions, uint32_t n, uint32_t threshold, const void* d_data,
                                void* d_commitments, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (n == 0) return CDA_OK;
        if (!namespaces || !data_off || !d_commitments || (data_off[n] > data_off[0] && !d_data))
            return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::square::CommitPlan& p = e.commit_plan();
        std::string err;
        if (cda::square::plan_commitments(namespaces, data_off, share_versions, n, threshold, &p, &err))
            return e.fail(CDA_ERR_SQUARE, err);
        return e.enqueue_commitments(p, n, static_cast<const uint8_t*>(d_data), static_cast<uint8_t*>(d_commitments),
                                     s);
    });
}

int cda_square_create(cda_ctx* ctx, const uint8_t* ods, uint32_t n_shares, cda_square** out) {
    if (!out) return CDA_ERR_INVALID;
    *out = nullptr;
    return guarded(ctx, [&](cda::Engine& e) -> int {
        uint32_t k;
        if (!square_width(n_shares, &k)) return not_pow2(e, n_shares);
        if (!ods) return e.fail(CDA_ERR_INVALID, "null buffer");
        cda_square* h = new cda_square{ctx, {}};
        const int rc = e.square_create(ods, k, &h->sq);
        if (rc != CDA_OK && rc != CDA_ERR_PUSH_ORDER) {
            delete h;
            return rc;
        }
        *out = h;   // a push-order failure still leaves the EDS (as ExtendShares does)
        return rc;
    });
}

int cda_square_destroy(cda_square* sq) {
    if (!sq) return CDA_OK;
    std::lock_guard<std::mutex> g(sq->ctx->eng.mutex());
    DeviceScope dev(sq->ctx->eng.device());
    // no queued work of the context reads the square any more: the square's
    // calls end with the context's end event, and waiting for that (not every
    // context stream) leaves unrelated in-flight batch work alone
    (void)sq->ctx->eng.wait_last_call();
    delete sq;
    return CDA_OK;
}

int cda_square_dah(cda_square* sq, uint32_t* k, uint8_t* row_roots, uint8_t* col_roots, uint8_t* data_root,
                   uint8_t* eds) {
    if (!sq) return CDA_ERR_INVALID;
    return guarded(sq->ctx, [&](cda::Engine& e) -> int {
        if (k) *k = sq->sq.k;
        int rc;
        if (row_roots && (rc = e.square_read(&sq->sq, cda::ResidentSquare::kRowRoots, row_roots))) return rc;
        if (col_roots && (rc = e.square_read(&sq->sq, cda::ResidentSquare::kColRoots, col_roots))) return rc;
        if (data_root && (rc = e.square_read(&sq->sq, cda::ResidentSquare::kDataRoot, data_root))) return rc;
        if (eds && (rc = e.square_read(&sq->sq, cda::ResidentSquare::kEds, eds))) return rc;
        return CDA_OK;
    });
}

int cda_square_share_proof(cda_square* sq, uint32_t start, uint32_t end, uint8_t* shares, uint32_t* start_row,
                           uint32_t* end_row, int32_t* nmt_start, int32_t* nmt_end, uint32_t* nmt_count,
                           uint8_t* nmt_nodes, uint8_t* row_roots, uint8_t* row_leaf_hash, uint8_t* row_aunts) {
    if (!sq) return CDA_ERR_INVALID;
    return guarded(sq->ctx, [&](cda::Engine& e) -> int {
        if (!nmt_start || !nmt_end || !nmt_count || !start_row || !end_row)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        cda::Engine::ShareProofOut o{shares, 0, 0, nmt_start, nmt_end, nmt_count, nmt_nodes, row_roots,
                                     row_leaf_hash, row_aunts};
        const int rc = e.square_share_proof(&sq->sq, start, end, &o);
        *start_row = o.start_row;
        *end_row = o.end_row;
        return rc;
    });
}

int cda_square_blob_commitments(cda_square* sq, const uint32_t* starts, const uint32_t* share_lens, uint32_t n,
                                uint32_t threshold, uint8_t* commitments) {
    if (!sq) return CDA_ERR_INVALID;
    return guarded(sq->ctx, [&](cda::Engine& e) -> int {
        if (n && (!starts || !share_lens || !commitments)) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.square_blob_commitments(&sq->sq, starts, share_lens, n, threshold, commitments);
    });
}

int cda_square_subtree_root(cda_square* sq, uint32_t row, const uint8_t* walk, uint32_t walk_len, uint8_t* root) {
    if (!sq) return CDA_ERR_INVALID;
    return guarded(sq->ctx, [&](cda::Engine& e) -> int {
        if (!root || (walk_len && !walk)) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.square_subtree_root(&sq->sq, row, walk, walk_len, root);
    });
}

int cda_repair(cda_ctx* ctx, uint8_t* eds, const uint8_t* present, uint32_t w, const uint8_t* row_roots,
               const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!eds || !present || !row_roots || !col_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (byz_axis) *byz_axis = -1;
        return e.host_repair(eds, present, w, row_roots, col_roots, byz_axis, byz_index);
    });
}

int cda_repair_device(cda_ctx* ctx, void* d_eds, const uint8_t* present, uint32_t w, const uint8_t* row_roots,
                      const uint8_t* col_roots, int32_t* byz_axis, uint32_t* byz_index) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!d_eds || !present || !row_roots || !col_roots) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (byz_axis) *byz_axis = -1;
        return e.device_repair(static_cast<uint8_t*>(d_eds), present, w, row_roots, col_roots, byz_axis, byz_index);
    });
}

int cda_rs_decode(cda_ctx* ctx, uint8_t* shards, const uint8_t* present, uint32_t n_shards, uint32_t shard_len,
                  uint32_t n_codewords) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (n_codewords == 0) return CDA_OK;
        if (!shards || !present) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.host_rs_decode(shards, present, n_shards, shard_len, n_codewords);
    });
}

int cda_nmt_axis_roots(cda_ctx* ctx, const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees,
                       uint32_t square_size, const uint32_t* axis_index, uint8_t* roots, int32_t* status) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (n_trees == 0) return CDA_OK;
        if (square_size == 0) return e.fail(CDA_ERR_INVALID, "cannot create a ErasuredNamespacedMerkleTree of squareSize == 0");
        if (!roots || !axis_index || (n_cells && !cells)) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (cell_len < CDA_NAMESPACE_SIZE) return e.fail(CDA_ERR_INVALID, "data is too short to contain namespace ID");
        for (uint32_t t = 0; t < n_trees; t++) {
            // wrapper Push (pkg/wrapper/nmt_wrapper.go:94-96)
            if ((uint64_t)axis_index[t] + 1 > 2ull * square_size || (uint64_t)n_cells > 2ull * square_size) {
                char buf[160];
                snprintf(buf, sizeof buf, "pushed past predetermined square size: boundary at %llu index at %u %u",
                         2ull * square_size, axis_index[t], n_cells > 2 * square_size ? 2 * square_size : n_cells - 1);
                return e.fail(CDA_ERR_INVALID, buf);
            }
        }
        return e.nmt_axis_roots(cells, cell_len, n_cells, n_trees, square_size, axis_index, roots, status);
    });
}

int cda_nmt_axis_root(cda_ctx* ctx, const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                      uint32_t axis_index, uint8_t* root) {
    return cda_nmt_axis_roots(ctx, cells, cell_len, n_cells, 1, square_size, &axis_index, root, nullptr);
}

int cda_nmt_prove_range(cda_ctx* ctx, const uint8_t* cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                        uint32_t axis_index, uint32_t start, uint32_t end, uint8_t* nodes, uint32_t* n_nodes,
                        uint8_t* root) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (square_size == 0) return e.fail(CDA_ERR_INVALID, "cannot create a ErasuredNamespacedMerkleTree of squareSize == 0");
        if (!cells || !n_nodes) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (cell_len < CDA_NAMESPACE_SIZE) return e.fail(CDA_ERR_INVALID, "data is too short to contain namespace ID");
        if ((uint64_t)axis_index + 1 > 2ull * square_size || (uint64_t)n_cells > 2ull * square_size)
            return e.fail(CDA_ERR_INVALID, "pushed past predetermined square size");
        return e.nmt_prove_range(cells, cell_len, n_cells, square_size, axis_index, start, end, nodes, n_nodes, root);
    });
}

int cda_merkle_root(cda_ctx* ctx, const uint8_t* items, const uint64_t* off, uint32_t n, uint8_t* out) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!out) return e.fail(CDA_ERR_INVALID, "null buffer");
        if (n == 0) {   // merkle.HashFromByteSlices(nil) = sha256("")
            static const uint8_t empty[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                              0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                              0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
            memcpy(out, empty, 32);
            return CDA_OK;
        }
        if (!off || (off[n] > off[0] && !items)) return e.fail(CDA_ERR_INVALID, "null buffer");
        for (uint32_t i = 0; i < n; i++)
            if (off[i + 1] < off[i]) return e.fail(CDA_ERR_INVALID, "item offsets must be non-decreasing");
        return e.merkle_root(items, off, n, out);
    });
}

int cda_comm_unique_id(uint8_t* id) {
    if (!id) return CDA_ERR_INVALID;
    tl_err.msg.clear();
    int rc = cda::comm_unique_id(id);
    if (rc) tl_err.msg = "ncclGetUniqueId failed";
    return rc;
}

int cda_comm_init(cda_ctx* ctx, int rank, int world, const uint8_t* id) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!id) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.comm_init(rank, world, id);
    });
}

int cda_comm_destroy(cda_ctx* ctx) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        e.comm_destroy();
        return CDA_OK;
    });
}

int cda_comm_size(cda_ctx* ctx, int* rank, int* world) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!rank || !world) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.comm_size(rank, world);
    });
}

int cda_comm_abort(cda_ctx* ctx) {
    // no context lock: a watchdog thread may call this while another thread
    // is blocked inside a collective on the same context
    if (!ctx) return CDA_ERR_INVALID;
    DeviceScope dev(ctx->eng.device());
    return ctx->eng.comm_abort();
}

int cda_split_rows_send(cda_ctx* ctx, const void* d_ods_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                        uint32_t parts, void* d_send, uint32_t* d_err, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        if (!d_ods_rows || !d_send || !d_err) return e.fail(CDA_ERR_INVALID, "null buffer");
        return e.enqueue_split_rows_send(static_cast<const uint8_t*>(d_ods_rows), k, n_rows, row0, parts,
                                         static_cast<uint8_t*>(d_send), d_err, s);
    });
}

int cda_extend_dah_split(cda_ctx* ctx, const void* d_ods_rows, uint32_t k, void* d_col_block, void* d_row_roots,
                         void* d_col_roots, void* d_data_root, uint32_t* d_err, void* stream) {
    return guarded_stream(ctx, stream, [&](cda::Engine& e, hipStream_t s) -> int {
        // per-rank buffer checks happen inside, after this rank has taken part
        // in every collective (an early return here would leave the peers
        // blocked in the all-to-all)
        return e.split_extend_dah(static_cast<const uint8_t*>(d_ods_rows), k, static_cast<uint8_t*>(d_col_block),
                                  static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                  static_cast<uint8_t*>(d_data_root), d_err, s);
    });
}

int cda_split_layout(uint32_t k, uint32_t world, cda_split_layout_t* out) {
    if (!out) return CDA_ERR_INVALID;
    const cda::SplitLayout L(k, world ? world : 1);
    if (!world || !L.valid() || world > 2 * k) return CDA_ERR_INVALID;
    *out = cda_split_layout_t{L.k, L.G, L.W, L.R, L.C, L.piece(), L.send_bytes(), L.col_block_bytes(),
                              L.col_slots_off(), L.row_sub_off(), L.gather_sub_off(0), L.gather_col_off(0),
                              L.err_off(), L.slots_bytes()};
    return CDA_OK;
}

int cda_split_offsets(uint32_t k, uint32_t world, int what, uint32_t n, const uint32_t* a, const uint32_t* b,
                      uint64_t* off) {
    if (!world || !off || (n && !a)) return CDA_ERR_INVALID;
    const cda::SplitLayout L(k, world);
    if (!L.valid()) return CDA_ERR_INVALID;
    // (a, b) ranges per kind; b must be given where the kind reads it
    uint32_t amax, bmax = 1;
    switch (what) {
        case CDA_SPLIT_SEND: amax = L.R; bmax = L.W; break;
        case CDA_SPLIT_BLOCK: amax = L.W; bmax = L.C; break;
        case CDA_SPLIT_COMBINE: amax = L.G; bmax = L.W; break;
        case CDA_SPLIT_SEND_PIECE: case CDA_SPLIT_RECV_PIECE: case CDA_SPLIT_GATHER_SUB: case CDA_SPLIT_GATHER_COL:
            amax = L.G; break;
        default: return CDA_ERR_INVALID;
    }
    if (n && bmax > 1 && !b) return CDA_ERR_INVALID;
    for (uint32_t i = 0; i < n; i++)
        if (a[i] >= amax || (bmax > 1 && b[i] >= bmax)) return CDA_ERR_INVALID;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t x = a[i], y = bmax > 1 ? b[i] : 0;
        switch (what) {
            case CDA_SPLIT_SEND: off[i] = L.send_off(x, y); break;
            case CDA_SPLIT_SEND_PIECE: off[i] = L.send_piece_off(x); break;
            case CDA_SPLIT_RECV_PIECE: off[i] = L.recv_piece_off(x); break;
            case CDA_SPLIT_BLOCK: off[i] = L.block_off(x, y); break;
            case CDA_SPLIT_GATHER_SUB: off[i] = L.gather_sub_off(x); break;
            case CDA_SPLIT_GATHER_COL: off[i] = L.gather_col_off(x); break;
            case CDA_SPLIT_COMBINE: off[i] = L.combine_slot(x, y); break;
            default: return CDA_ERR_INVALID;
        }
    }
    return CDA_OK;
}

int cda_extend_dah_multi(cda_ctx* const* ctxs, uint32_t n_ctx, const uint8_t* ods, uint32_t k, uint32_t n,
                         uint8_t* eds, uint8_t* row_roots, uint8_t* col_roots, uint8_t* data_roots, int32_t* status) {
    tl_err.msg.clear();
    if (!ctxs || n_ctx == 0) {
        tl_err.msg = "no contexts";
        return CDA_ERR_INVALID;
    }
    if (n == 0) return CDA_OK;
    const uint32_t W = 2 * k;
    const size_t ods_sq = (size_t)k * k * CDA_SHARE_SIZE, eds_sq = (size_t)W * W * CDA_SHARE_SIZE;
    const size_t roots_sq = (size_t)W * CDA_NMT_ROOT_SIZE;
    std::vector<int> rcs(n_ctx, CDA_OK);
    std::vector<std::string> msgs(n_ctx);
    std::vector<std::thread> th;
    uint32_t first = 0;
    try {
        for (uint32_t d = 0; d < n_ctx; d++) {
            // context d: squares [first, first + m), config 4's contiguous shard
            const uint32_t m = n / n_ctx + (d < n % n_ctx ? 1 : 0);
            if (m == 0) continue;
            th.emplace_back([=, &rcs, &msgs] {
                rcs[d] = cda_extend_dah_batch(ctxs[d], ods + first * ods_sq, k, m,
                                              eds ? eds + first * eds_sq : nullptr, row_roots + first * roots_sq,
                                              col_roots + first * roots_sq, data_roots + (size_t)first * 32,
                                              status ? status + first : nullptr);
                msgs[d] = tl_err.msg;   // the worker thread's error text
            });
            first += m;
        }
    } catch (...) {
        for (auto& t : th) t.join();
        tl_err.msg = "thread creation failed";
        return CDA_ERR_DEVICE;
    }
    for (auto& t : th) t.join();
    // the first device error wins over push-order (reported per square in status)
    int rc = CDA_OK;
    for (uint32_t d = 0; d < n_ctx; d++) {
        if (rcs[d] != CDA_OK && (rc == CDA_OK || rc == CDA_ERR_PUSH_ORDER) && rc != rcs[d]) {
            rc = rcs[d];
            tl_err.msg = msgs[d];
        }
    }
    return rc;
}

int cda_set_profiling(cda_ctx* ctx, int enable) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        e.set_profiling(enable != 0);
        return CDA_OK;
    });
}

int cda_stage_times(cda_ctx* ctx, double* ms, uint32_t* counts, int n_stages) {
    return guarded(ctx, [&](cda::Engine& e) -> int { return e.collect_stage_times(ms, counts, n_stages); });
}

}  // extern "C"
