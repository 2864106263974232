// capi.hip -- extern "C" entry points of libcda.so (declared in include/cda.h).
// Each function validates arguments the way the reference does, locks the
// context and forwards to cda::Engine.  No C++ exception or abort crosses the
// ABI.
#include <cmath>
#include <cstring>
#include <new>

#include "../../include/cda.h"
#include "engine.h"

struct cda_ctx {
    cda::Engine eng;
    explicit cda_ctx(int dev) : eng(dev) {}
};

namespace {

// pkg/da/data_availability_header.go SquareSize + IsPowerOfTwo
bool square_width(uint32_t n_shares, uint32_t* k) {
    if (n_shares == 0 || (n_shares & (n_shares - 1))) return false;
    uint32_t w = 1;
    while ((uint64_t)w * w < n_shares) w <<= 1;
    if ((uint64_t)w * w != n_shares) return false;   // e.g. 8 shares: power of two, not a square
    *k = w;
    return true;
}

template <class F>
int guarded(cda_ctx* ctx, F&& f) {
    if (!ctx) return CDA_ERR_INVALID;
    try {
        std::lock_guard<std::mutex> g(ctx->eng.mutex());
        ctx->eng.clear_error();
        return f(ctx->eng);
    } catch (const std::bad_alloc&) {
        return ctx->eng.fail(CDA_ERR_OOM, "host allocation failed");
    } catch (...) {
        return ctx->eng.fail(CDA_ERR_DEVICE, "unexpected exception");
    }
}

int not_pow2(cda::Engine& e, uint32_t n) {
    char buf[96];
    snprintf(buf, sizeof buf, "number of shares is not a power of 2: got %u", n);
    return e.fail(CDA_ERR_NOT_POW2, buf);
}

}  // namespace

extern "C" {

const char* cda_version(void) { return "cda 0.1.0 gfx950"; }

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

const char* cda_last_error(cda_ctx* ctx) { return ctx ? ctx->eng.last_error().c_str() : "null context"; }

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

int cda_extend_dah_device(cda_ctx* ctx, const void* d_ods, uint32_t k, uint32_t n, void* d_eds, void* d_row_roots,
                          void* d_col_roots, void* d_data_roots, int32_t* d_status, void* stream) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (k == 0 || (k & (k - 1))) return not_pow2(e, k * k);
        if (n == 0) return CDA_OK;
        if (!d_ods || !d_eds || !d_row_roots || !d_col_roots || !d_data_roots)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        static thread_local cda::DevBuf err;   // per-thread err words (device)
        hipError_t he = err.ensure((size_t)n * 4);
        if (he != hipSuccess) return e.fail(CDA_ERR_OOM, "hipMalloc err words");
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = default stream
        return e.enqueue_extend_dah(static_cast<const uint8_t*>(d_ods), k, n, static_cast<uint8_t*>(d_eds),
                                    static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                    static_cast<uint8_t*>(d_data_roots), err.as<uint32_t>(), d_status, s);
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
    if (axis) *axis = ctx->eng.po_axis;
    if (index) *index = ctx->eng.po_index;
    if (position) *position = ctx->eng.po_pos;
    return CDA_OK;
}

int cda_split_rows(cda_ctx* ctx, const void* d_ods_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                   void* d_row_block, uint32_t* d_err, void* stream) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!d_ods_rows || !d_row_block || !d_err) return e.fail(CDA_ERR_INVALID, "null buffer");
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = default stream
        return e.enqueue_split_rows(static_cast<const uint8_t*>(d_ods_rows), k, n_rows, row0,
                                    static_cast<uint8_t*>(d_row_block), d_err, s);
    });
}

int cda_split_cols(cda_ctx* ctx, void* d_col_block, uint32_t k, uint32_t n_cols, uint32_t col0,
                   void* d_col_root_slots, void* d_row_subtree_slots, uint32_t* d_err, void* stream) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!d_col_block || !d_col_root_slots || !d_row_subtree_slots || !d_err)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = default stream
        return e.enqueue_split_cols(static_cast<uint8_t*>(d_col_block), k, n_cols, col0,
                                    static_cast<uint8_t*>(d_col_root_slots), static_cast<uint8_t*>(d_row_subtree_slots),
                                    d_err, s);
    });
}

int cda_split_combine(cda_ctx* ctx, const void* d_row_subtree_slots, uint32_t parts, uint32_t k,
                      const void* d_col_root_slots, void* d_row_roots, void* d_col_roots, void* d_data_root,
                      void* stream) {
    return guarded(ctx, [&](cda::Engine& e) -> int {
        if (!d_row_subtree_slots || !d_col_root_slots || !d_row_roots || !d_col_roots || !d_data_root)
            return e.fail(CDA_ERR_INVALID, "null buffer");
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = default stream
        return e.enqueue_split_combine(static_cast<const uint8_t*>(d_row_subtree_slots), parts, k,
                                       static_cast<const uint8_t*>(d_col_root_slots),
                                       static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                       static_cast<uint8_t*>(d_data_root), s);
    });
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
