// square.hip -- data-square construction on the device: the share writer and
// the Engine glue for square.Construct / square.Build (+ extend + DAH).
//
// The host plans the layout (square_plan.cpp: go-square v1.1.0 Builder /
// Export / WriteSquare); this file writes the k*k shares into HBM:
//   compact segments  tx and PFB compact shares, built on the host (small);
//   padding segments  ns || info(version, start) || 0x00000000 || zeros
//                     (shares.md "Padding"; reserved, namespace and tail);
//   blob segments     sparse shares: first = ns || info(v, 1) || len (BE32)
//                     || data[0:478], continuation j = ns || info(v, 0) ||
//                     data[478 + 482(j-1) : ...], zero-padded (shares.md
//                     "Share Format", SparseShareSplitter.Write).
// One wave per share, 8 bytes per lane, so every share is one coalesced
// 512-B store; blob bytes come straight from the transaction buffer (aligned
// dword loads + v_alignbyte for the arbitrary source offset), so the ODS is
// produced in HBM without a host-side copy of the payload.  HBM-bound:
// algorithmic bytes = payload read + k*k*512 written.
#include <cstring>

#include "../../include/cda.h"
#include "engine.h"
#include "sha256_dev.h"

namespace cda {

namespace {

using square::Segment;

__global__ __launch_bounds__(256) void share_writer_kernel(const Segment* __restrict__ segs, uint32_t n_segs,
                                                           const uint32_t* __restrict__ hint,
                                                           const uint8_t* __restrict__ compact,
                                                           const uint8_t* __restrict__ txs, uint8_t* __restrict__ ods,
                                                           uint32_t n_shares) {
    const uint32_t s = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (s >= n_shares) return;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = 0;   // last segment with start <= s
    if (hint) {        // segment of share (s / kHintShares) * kHintShares, then a short forward scan
        lo = hint[s / square::kHintShares];
        while (lo + 1 < n_segs && segs[lo + 1].start <= s) lo++;
    } else {
        uint32_t hi = n_segs;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (segs[mid].start <= s) lo = mid;
            else hi = mid;
        }
    }
    const Segment& g = segs[lo];
    const uint32_t j = s - g.start;
    const uint32_t p0 = 8 * lane;
    uint2 v;
    if (g.kind == square::kSegCompact) {
        v = *reinterpret_cast<const uint2*>(compact + g.src + (size_t)j * square::kShare + p0);
    } else {
        const bool blob = g.kind == square::kSegBlob;
        const bool first = !blob || j == 0;             // padding shares are sequence starts (length 0)
        const uint32_t hdr = first ? square::kNs + 5 : square::kNs + 1;
        const uint32_t seq = blob ? g.len : 0;
        const uint32_t dbase = j == 0 ? 0 : (square::kShare - square::kNs - 5) + (j - 1) * (square::kShare - square::kNs - 1);
        uint32_t w0 = 0, w1 = 0;
        if (p0 >= hdr) {
            const uint32_t d0 = p0 - hdr + dbase;
            if (blob && d0 < seq) {
                const uint64_t base = g.src + d0;
                const uint32_t sh = (uint32_t)(base & 3);
                const uint32_t* q = reinterpret_cast<const uint32_t*>(txs + (base & ~uint64_t(3)));
                const uint32_t x0 = q[0], x1 = q[1], x2 = q[2];
                w0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
                w1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
                const uint32_t valid = seq - d0;   // blob bytes left in this 8-byte window
                if (valid < 4) {
                    w0 &= (1u << (8 * valid)) - 1;
                    w1 = 0;
                } else if (valid < 8) {
                    w1 &= (1u << (8 * (valid - 4))) - 1;
                }
            }
        } else {   // lanes covering the header (bytes 0..39)
            const uint32_t info = (g.version << 1) | (first ? 1u : 0u);
            uint32_t b8[8];
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint32_t p = p0 + b;
                uint32_t x = 0;
                if (p < square::kNs) x = g.ns[p];
                else if (p == square::kNs) x = info;
                else if (first && p < square::kNs + 5) x = (seq >> (8 * (square::kNs + 4 - p))) & 0xFF;
                else if (blob && p >= hdr) {
                    const uint32_t d = p - hdr + dbase;
                    if (d < seq) x = txs[g.src + d];
                }
                b8[b] = x;
            }
            w0 = b8[0] | b8[1] << 8 | b8[2] << 16 | b8[3] << 24;
            w1 = b8[4] | b8[5] << 8 | b8[6] << 16 | b8[7] << 24;
        }
        v = make_uint2(w0, w1);
    }
    *reinterpret_cast<uint2*>(ods + (size_t)s * square::kShare + p0) = v;
}

}  // namespace

hipError_t launch_share_writer(const Segment* segs, uint32_t n_segs, const uint32_t* hint, const uint8_t* compact,
                               const uint8_t* txs, uint8_t* ods, uint32_t n_shares, hipStream_t s) {
    if (n_shares == 0 || n_segs == 0) return hipSuccess;
    hipLaunchKernelGGL(share_writer_kernel, dim3((n_shares + 3) / 4), dim3(256), 0, s, segs, n_segs, hint, compact, txs,
                       ods, n_shares);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Engine glue
// ---------------------------------------------------------------------------
int Engine::enqueue_square(const square::Plan& p, const uint8_t* d_txs, uint8_t* d_ods, hipStream_t s) {
    const size_t seg_b = p.segs.size() * sizeof(Segment);
    const size_t plan_b = seg_b + p.compact.size();
    int rc;
    // The plan goes through an engine-owned pinned buffer so the copy stays
    // asynchronous; the previous call's copy must have left it first.
    if (sq_event_ && (rc = check(hipEventSynchronize(sq_event_), "hipEventSynchronize"))) return rc;
    if (plan_b > sq_stage_bytes_) {
        if (sq_stage_) (void)hipHostFree(sq_stage_);
        sq_stage_ = nullptr;
        sq_stage_bytes_ = 0;
        if ((rc = check(hipHostMalloc(&sq_stage_, plan_b, hipHostMallocDefault), "hipHostMalloc"))) return rc;
        sq_stage_bytes_ = plan_b;
    }
    if (!sq_event_ && (rc = check(hipEventCreateWithFlags(&sq_event_, hipEventDisableTiming), "hipEventCreate")))
        return rc;
    std::memcpy(sq_stage_, p.segs.data(), seg_b);
    if (!p.compact.empty()) std::memcpy(static_cast<uint8_t*>(sq_stage_) + seg_b, p.compact.data(), p.compact.size());
    if ((rc = check(sq_plan_.ensure(plan_b), "hipMalloc"))) return rc;
    if ((rc = check(hipMemcpyAsync(sq_plan_.ptr, sq_stage_, plan_b, hipMemcpyHostToDevice, s), "H2D plan"))) return rc;
    if ((rc = check(hipEventRecord(sq_event_, s), "hipEventRecord"))) return rc;
    const uint32_t n_shares = p.square_size * p.square_size;
    return check(launch_share_writer(sq_plan_.as<Segment>(), (uint32_t)p.segs.size(), nullptr,
                                     sq_plan_.as<uint8_t>() + seg_b, d_txs, d_ods, n_shares, s),
                 "share writer");
}

int Engine::upload_txs(const uint8_t* txs, size_t len, hipStream_t s) {
    int rc;
    // 16 bytes of slack: the writer's aligned dword loads may run past the
    // last blob byte (the loaded bytes are masked off).
    if ((rc = check(sq_txs_.ensure(len + 16), "hipMalloc"))) return rc;
    if (len && (rc = check(hipMemcpyAsync(sq_txs_.ptr, txs, len, hipMemcpyHostToDevice, s), "H2D txs"))) return rc;
    return CDA_OK;
}

int Engine::host_square(const square::Plan& p, const uint8_t* txs, size_t txs_len, uint8_t* ods) {
    const size_t ods_b = (size_t)p.square_size * p.square_size * kShare;
    hipStream_t s = stream_;
    int rc;
    if ((rc = check(h_ods_.ensure(ods_b), "hipMalloc"))) return rc;
    if ((rc = upload_txs(txs, txs_len, s))) return rc;
    if ((rc = enqueue_square(p, sq_txs_.as<uint8_t>(), h_ods_.as<uint8_t>(), s))) return rc;
    if ((rc = check(hipMemcpyAsync(ods, h_ods_.ptr, ods_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    return check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

int Engine::host_construct_extend_dah(const square::Plan& p, const uint8_t* txs, size_t txs_len, uint8_t* eds,
                                      uint8_t* rows, uint8_t* cols, uint8_t* root) {
    const uint32_t k = p.square_size, W = 2 * k;
    const size_t ods_b = (size_t)k * k * kShare, eds_b = (size_t)W * W * kShare, roots_b = (size_t)W * kNode;
    hipStream_t s = stream_;
    int rc;
    if ((rc = check(h_ods_.ensure(ods_b), "hipMalloc"))) return rc;
    if ((rc = check(h_eds_.ensure(eds_b), "hipMalloc"))) return rc;
    if ((rc = check(h_rows_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_cols_.ensure(roots_b), "hipMalloc"))) return rc;
    if ((rc = check(h_roots_.ensure(32), "hipMalloc"))) return rc;
    if ((rc = check(err_buf_.ensure(4), "hipMalloc"))) return rc;
    if ((rc = upload_txs(txs, txs_len, s))) return rc;
    if ((rc = enqueue_square(p, sq_txs_.as<uint8_t>(), h_ods_.as<uint8_t>(), s))) return rc;
    if ((rc = enqueue_extend_dah(h_ods_.as<uint8_t>(), k, 1, h_eds_.as<uint8_t>(), h_rows_.as<uint8_t>(),
                                 h_cols_.as<uint8_t>(), h_roots_.as<uint8_t>(), err_buf_.as<uint32_t>(), nullptr, s)))
        return rc;
    if (eds && (rc = check(hipMemcpyAsync(eds, h_eds_.ptr, eds_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(rows, h_rows_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(cols, h_cols_.ptr, roots_b, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipMemcpyAsync(root, h_roots_.ptr, 32, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    uint32_t err = 0;
    if ((rc = check(hipMemcpyAsync(&err, err_buf_.ptr, 4, hipMemcpyDeviceToHost, s), "D2H"))) return rc;
    if ((rc = check(hipStreamSynchronize(s), "hipStreamSynchronize"))) return rc;
    if (err == 0xFFFFFFFFu) return CDA_OK;
    // A namespace out of order in Q0 (e.g. a blob in a reserved namespace):
    // fetch the ODS once to name the offending namespaces.
    std::vector<uint8_t> ods(ods_b);
    if ((rc = check(hipMemcpy(ods.data(), h_ods_.ptr, ods_b, hipMemcpyDeviceToHost), "D2H"))) return rc;
    return push_order_error(&err, 1, ods.data(), k, false);
}

}  // namespace cda
