// square_plan.cpp -- go-square v1.1.0 square.Construct / square.Build layout
// (see square_plan.h for the reference pointers).
//
// Pieces and the go-square functions they restate:
//   proto decoding       blob.UnmarshalBlobTx (google.golang.org/protobuf
//                        semantics: a known field with an unexpected wire type
//                        is kept as an unknown field, proto3 strings must be
//                        UTF-8, empty proto3 bytes decode to nil)
//   CompactCounter       shares.CompactShareCounter Add / Revert / Size
//   compact_shares       shares.CompactShareSplitter WriteTx / Export
//                        (reserved bytes = offset of the first unit that
//                        starts in the share; sequence length in share 0)
//   plan                 square.NewBuilder / AppendTx / AppendBlobTx /
//                        Export / WriteSquare and square.Build
//                        (out_of_order_builder.go:24-57, 63-161 minus the swap)
#include "square_plan.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string_view>
#include <unordered_map>

namespace cda {
namespace square {

namespace {

constexpr uint32_t kFirstCompact = kShare - kNs - 1 - 4 - 4;   // 474: FirstCompactShareContentSize
constexpr uint32_t kContCompact = kShare - kNs - 1 - 4;        // 478: ContinuationCompactShareContentSize
constexpr uint32_t kFirstSparse = kShare - kNs - 1 - 4;        // 478: FirstSparseShareContentSize
constexpr uint32_t kContSparse = kShare - kNs - 1;             // 482: ContinuationSparseShareContentSize
// worstCaseShareIndexes: every index is priced at the upper-bound share count
// (128 * 128); any index below 2^21 is a 3-byte varint, so the price does not
// depend on the exact bound.
constexpr uint32_t kWorstCaseShareIndex = 128 * 128;

const uint8_t kTxNs[kNs] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01};
const uint8_t kPfbNs[kNs] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x04};
const uint8_t kReservedPadNs[kNs] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF};
const uint8_t kTailPadNs[kNs] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE};

// ---------------------------------------------------------------- protobuf
struct Span {
    const uint8_t* p = nullptr;
    size_t n = 0;
    bool present = false;
};

bool get_varint(const uint8_t* b, size_t n, size_t& i, uint64_t& v) {
    v = 0;
    for (int k = 0; k < 10; k++) {
        if (i >= n) return false;
        const uint8_t c = b[i++];
        if (k == 9 && c > 1) return false;   // overflows 64 bits
        v |= (uint64_t)(c & 0x7F) << (7 * k);
        if (!(c & 0x80)) return true;
    }
    return false;
}

bool get_tag(const uint8_t* b, size_t n, size_t& i, uint32_t& num, uint32_t& wt) {
    uint64_t t;
    if (!get_varint(b, n, i, t)) return false;
    num = (uint32_t)(t >> 3);
    wt = (uint32_t)(t & 7);
    return (t >> 3) >= 1 && (t >> 3) <= 0x1FFFFFFF;
}

bool skip_value(const uint8_t* b, size_t n, size_t& i, uint32_t num, uint32_t wt, int depth = 0) {
    uint64_t v;
    switch (wt) {
        case 0: return get_varint(b, n, i, v);
        case 1: if (n - i < 8) return false; i += 8; return true;
        case 5: if (n - i < 4) return false; i += 4; return true;
        case 2:
            if (!get_varint(b, n, i, v) || v > n - i) return false;
            i += (size_t)v;
            return true;
        case 3: {   // group: fields until the matching end-group tag
            if (depth > 100) return false;
            for (;;) {
                uint32_t fn, fw;
                if (!get_tag(b, n, i, fn, fw)) return false;
                if (fw == 4) return fn == num;
                if (!skip_value(b, n, i, fn, fw, depth + 1)) return false;
            }
        }
        default: return false;   // stray end-group, reserved wire types
    }
}

bool get_bytes(const uint8_t* b, size_t n, size_t& i, Span& out) {
    uint64_t len;
    if (!get_varint(b, n, i, len) || len > n - i) return false;
    out.p = b + i;
    out.n = (size_t)len;
    out.present = len > 0;   // proto3 implicit-presence bytes: empty -> nil
    i += (size_t)len;
    return true;
}

bool valid_utf8(const uint8_t* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const uint8_t c = s[i];
        if (c < 0x80) { i++; continue; }
        int len;
        uint32_t cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return false;
        if (n - i < (size_t)len) return false;
        for (int k = 1; k < len; k++) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
            return false;
        if (cp >= 0xD800 && cp <= 0xDFFF) return false;
        i += len;
    }
    return true;
}

struct BlobRec {
    Span ns_id, data;
    uint32_t share_version = 0, ns_version = 0;
};

// v1.BlobProto{namespace_id = 1; data = 2; share_version = 3; namespace_version = 4}
bool parse_blob(const uint8_t* b, size_t n, BlobRec& out) {
    size_t i = 0;
    while (i < n) {
        uint32_t fn, wt;
        if (!get_tag(b, n, i, fn, wt)) return false;
        uint64_t v;
        if (fn == 1 && wt == 2) {
            if (!get_bytes(b, n, i, out.ns_id)) return false;
        } else if (fn == 2 && wt == 2) {
            if (!get_bytes(b, n, i, out.data)) return false;
        } else if (fn == 3 && wt == 0) {
            if (!get_varint(b, n, i, v)) return false;
            out.share_version = (uint32_t)v;
        } else if (fn == 4 && wt == 0) {
            if (!get_varint(b, n, i, v)) return false;
            out.ns_version = (uint32_t)v;
        } else if (!skip_value(b, n, i, fn, wt)) {
            return false;
        }
    }
    return true;
}

struct BlobTxRec {
    Span inner;
    std::vector<BlobRec> blobs;
};

// blob.UnmarshalBlobTx: v1.BlobTx{tx = 1; repeated BlobProto blobs = 2;
// string type_id = 3}; a blob tx iff it decodes and type_id == "BLOB".
bool unmarshal_blob_tx(const uint8_t* b, size_t n, BlobTxRec& out) {
    size_t i = 0;
    Span type_id;
    while (i < n) {
        uint32_t fn, wt;
        if (!get_tag(b, n, i, fn, wt)) return false;
        if (fn == 1 && wt == 2) {
            if (!get_bytes(b, n, i, out.inner)) return false;
        } else if (fn == 2 && wt == 2) {
            Span m;
            if (!get_bytes(b, n, i, m)) return false;
            BlobRec r;
            if (!parse_blob(m.p, m.n, r)) return false;
            out.blobs.push_back(r);
        } else if (fn == 3 && wt == 2) {
            if (!get_bytes(b, n, i, type_id)) return false;
            if (!valid_utf8(type_id.p, type_id.n)) return false;
        } else if (!skip_value(b, n, i, fn, wt)) {
            return false;
        }
    }
    return type_id.n == 4 && std::memcmp(type_id.p, "BLOB", 4) == 0;
}

uint32_t varint_len(uint64_t x) {
    uint32_t n = 1;
    while (x >= 0x80) { x >>= 7; n++; }
    return n;
}

void put_varint(std::vector<uint8_t>& o, uint64_t x) {
    while (x >= 0x80) { o.push_back((uint8_t)(x | 0x80)); x >>= 7; }
    o.push_back((uint8_t)x);
}

// v1.IndexWrapper{tx = 1; repeated uint32 share_indexes = 2 (packed); string
// type_id = 3 = "INDX"}, deterministic field order, empty fields omitted.
void marshal_index_wrapper(const Span& tx, const uint32_t* idx, size_t n_idx, std::vector<uint8_t>& o) {
    o.clear();
    if (tx.n) {
        o.push_back(0x0A);
        put_varint(o, tx.n);
        o.insert(o.end(), tx.p, tx.p + tx.n);
    }
    if (n_idx) {
        size_t packed = 0;
        for (size_t j = 0; j < n_idx; j++) packed += varint_len(idx[j]);
        o.push_back(0x12);
        put_varint(o, packed);
        for (size_t j = 0; j < n_idx; j++) put_varint(o, idx[j]);
    }
    o.push_back(0x1A);
    o.push_back(4);
    o.insert(o.end(), {'I', 'N', 'D', 'X'});
}

size_t index_wrapper_size(size_t tx_len, size_t n_blobs) {
    size_t s = 0;
    if (tx_len) s += 1 + varint_len(tx_len) + tx_len;
    if (n_blobs) {
        const size_t packed = n_blobs * varint_len(kWorstCaseShareIndex);
        s += 1 + varint_len(packed) + packed;
    }
    return s + 6;
}

// ------------------------------------------------------- share accounting
struct CompactCounter {   // shares.CompactShareCounter
    int64_t shares = 0, remainder = 0, last_shares = 0, last_remainder = 0;
    int64_t add(uint64_t data_len) {
        int64_t d = (int64_t)(data_len + varint_len(data_len));
        last_remainder = remainder;
        last_shares = shares;
        if (shares == 0) {
            if (d >= (int64_t)kFirstCompact - remainder) {
                d -= (int64_t)kFirstCompact - remainder;
                shares++;
                remainder = 0;
            } else {
                remainder += d;
                d = 0;
            }
        }
        if (d >= (int64_t)kContCompact - remainder) {
            d -= (int64_t)kContCompact - remainder;
            shares++;
            remainder = 0;
        } else {
            remainder += d;
            d = 0;
        }
        if (d > 0) {
            shares += d / kContCompact;
            remainder = d % kContCompact;
        }
        int64_t diff = shares - last_shares;
        if (last_remainder == 0 && remainder > 0) diff++;
        else if (last_remainder > 0 && remainder == 0) diff--;
        return diff;
    }
    void revert() { shares = last_shares; remainder = last_remainder; }
    int64_t size() const { return remainder == 0 ? shares : shares + 1; }
};

// CompactShareSplitter: units are varint-delimited; appends whole shares.
// ranges (optional): per unit, WriteTx's recorded range -- from the share the
// unit starts in (the number of completed shares before it) to Count() after
// it (completed shares, plus the pending one if it holds data).
void compact_shares(const uint8_t* ns, const std::vector<Span>& units, std::vector<uint8_t>& out, uint32_t* n_out,
                    std::vector<uint32_t>* r_start = nullptr, std::vector<uint32_t>* r_end = nullptr) {
    *n_out = 0;
    if (units.empty()) return;
    const size_t base = out.size();
    std::vector<uint8_t> cur;
    size_t res_at = 0;
    bool reserved_set = false;
    uint64_t total = 0;
    auto start_share = [&](bool first) {
        cur.assign(ns, ns + kNs);
        cur.push_back(first ? 1 : 0);   // info byte: version 0, sequence start
        if (first) cur.insert(cur.end(), 4, 0);
        res_at = cur.size();
        cur.insert(cur.end(), 4, 0);
        reserved_set = false;
    };
    auto flush = [&]() {
        cur.resize(kShare, 0);
        out.insert(out.end(), cur.begin(), cur.end());
        (*n_out)++;
    };
    start_share(true);
    std::vector<uint8_t> unit;
    for (const Span& u : units) {
        unit.clear();
        put_varint(unit, u.n);
        unit.insert(unit.end(), u.p, u.p + u.n);
        total += unit.size();
        if (!reserved_set) {
            const uint32_t at = (uint32_t)cur.size();
            cur[res_at + 0] = (uint8_t)(at >> 24);
            cur[res_at + 1] = (uint8_t)(at >> 16);
            cur[res_at + 2] = (uint8_t)(at >> 8);
            cur[res_at + 3] = (uint8_t)at;
            reserved_set = true;
        }
        if (r_start) r_start->push_back(*n_out);
        size_t off = 0;
        while (off < unit.size()) {
            const size_t room = kShare - cur.size();
            const size_t take = std::min(room, unit.size() - off);
            cur.insert(cur.end(), unit.begin() + off, unit.begin() + off + take);
            off += take;
            if (cur.size() == kShare) {
                flush();
                start_share(false);
            }
        }
        if (r_end) r_end->push_back(*n_out + (cur.size() > res_at + 4 ? 1u : 0u));
    }
    if (cur.size() > res_at + 4) flush();
    uint8_t* first = out.data() + base;
    first[kNs + 1] = (uint8_t)(total >> 24);
    first[kNs + 2] = (uint8_t)(total >> 16);
    first[kNs + 3] = (uint8_t)(total >> 8);
    first[kNs + 4] = (uint8_t)total;
}

struct Element {   // square.Element
    uint32_t pfb, blob;
    const uint8_t* ns_id;
    uint32_t ns_id_len;
    uint8_t ns_version;   // uint8(namespace_version)
    uint32_t share_version;
    const uint8_t* data;
    uint32_t len;
    uint32_t num_shares, max_padding;
};

int ns_compare(const Element& a, const Element& b) {   // bytes.Compare(Namespace().Bytes())
    if (a.ns_version != b.ns_version) return a.ns_version < b.ns_version ? -1 : 1;
    const uint32_t m = std::min(a.ns_id_len, b.ns_id_len);
    const int c = m ? std::memcmp(a.ns_id, b.ns_id, m) : 0;
    if (c) return c;
    return a.ns_id_len == b.ns_id_len ? 0 : (a.ns_id_len < b.ns_id_len ? -1 : 1);
}

std::string fmt(const char* f, long long a, long long b = 0, long long c = 0) {
    char buf[256];
    snprintf(buf, sizeof buf, f, a, b, c);
    return buf;
}

}  // namespace

uint32_t round_up_pow2(uint32_t x) {
    uint32_t r = 1;
    while (r < x) r <<= 1;
    return r;
}

uint32_t blob_min_square_size(uint32_t share_count) {   // inclusion.BlobMinSquareSize
    uint32_t s = 0;
    while ((uint64_t)s * s < share_count) s++;           // ceil(sqrt)
    return round_up_pow2(s);
}

uint32_t subtree_width(uint32_t share_count, uint32_t threshold) {   // inclusion.SubTreeWidth
    uint32_t s = share_count / threshold + (share_count % threshold ? 1 : 0);
    return std::min(round_up_pow2(s), blob_min_square_size(share_count));
}

uint32_t sparse_shares_needed(uint32_t len) {   // shares.SparseSharesNeeded
    if (len == 0) return 0;
    if (len < kFirstSparse) return 1;
    return 1 + (len - kFirstSparse + kContSparse - 1) / kContSparse;
}

int plan(const uint8_t* txs, const uint64_t* off, uint32_t n, uint32_t max_ss, uint32_t threshold, Mode mode,
         Plan* out, std::string* err) {
    Plan& P = *out;
    P = Plan{};
    if (max_ss == 0 || (max_ss & (max_ss - 1))) {
        *err = "max square size must be a power of two";
        return -1;
    }
    if (threshold == 0) {
        *err = "subtree root threshold must be positive";
        return -1;
    }
    const int64_t cap = (int64_t)max_ss * max_ss;
    CompactCounter tx_counter, pfb_counter;
    int64_t current = 0;
    std::vector<Span> normal;
    std::vector<uint32_t> normal_idx, blob_idx;
    std::vector<Span> pfb_inner;
    std::vector<uint32_t> pfb_nblobs;
    std::vector<Element> elems;
    bool seen_blob = false;
    for (uint32_t t = 0; t < n; t++) {
        const uint8_t* p = txs + off[t];
        const size_t len = (size_t)(off[t + 1] - off[t]);
        BlobTxRec btx;
        if (unmarshal_blob_tx(p, len, btx)) {
            seen_blob = true;
            const int64_t pfb_diff = pfb_counter.add(index_wrapper_size(btx.inner.n, btx.blobs.size()));
            int64_t max_blob_shares = 0;
            std::vector<Element> es;
            for (uint32_t b = 0; b < btx.blobs.size(); b++) {
                const BlobRec& r = btx.blobs[b];
                Element e;
                e.pfb = (uint32_t)pfb_inner.size();
                e.blob = b;
                e.ns_id = r.ns_id.p;
                e.ns_id_len = (uint32_t)r.ns_id.n;
                e.ns_version = (uint8_t)r.ns_version;
                e.share_version = r.share_version;
                e.data = r.data.p;
                e.len = (uint32_t)r.data.n;
                e.num_shares = sparse_shares_needed(e.len);
                e.max_padding = subtree_width(e.num_shares, threshold) - 1;
                max_blob_shares += e.num_shares + e.max_padding;
                es.push_back(e);
            }
            if (current + pfb_diff + max_blob_shares <= cap) {
                current += pfb_diff + max_blob_shares;
                elems.insert(elems.end(), es.begin(), es.end());
                pfb_inner.push_back(btx.inner);
                pfb_nblobs.push_back((uint32_t)btx.blobs.size());
                blob_idx.push_back(t);
            } else {
                pfb_counter.revert();
                if (mode == kConstruct) {
                    *err = fmt("not enough space to append blob tx at index %lld", t);
                    return -1;
                }
            }
        } else {
            if (mode == kConstruct && seen_blob) {
                *err = fmt("normal transaction at index %lld can not be appended after blob tx", t);
                return -1;
            }
            const int64_t diff = tx_counter.add(len);
            if (current + diff <= cap) {
                current += diff;
                normal.push_back(Span{p, len, len > 0});
                normal_idx.push_back(t);
            } else {
                tx_counter.revert();
                if (mode == kConstruct) {
                    *err = fmt("not enough space to append tx at index %lld", t);
                    return -1;
                }
            }
        }
    }
    P.kept = normal_idx;
    P.kept.insert(P.kept.end(), blob_idx.begin(), blob_idx.end());
    P.n_blobs = (uint32_t)elems.size();

    // ---- Export -----------------------------------------------------------
    if (normal.empty() && pfb_inner.empty()) {   // EmptySquare: one tail padding share
        P.square_size = 1;
        Segment s{};
        s.kind = kSegPadding;
        s.start = 0;
        s.n = 1;
        std::memcpy(s.ns, kTailPadNs, kNs);
        P.segs.push_back(s);
        return 0;
    }
    const uint32_t ss = blob_min_square_size((uint32_t)current);
    std::stable_sort(elems.begin(), elems.end(),
                     [](const Element& a, const Element& b) { return ns_compare(a, b) < 0; });
    uint32_t n_tx_shares = 0, n_pfb_shares = 0;
    std::vector<uint32_t> tx_s, tx_e, pfb_s, pfb_e;
    compact_shares(kTxNs, normal, P.compact, &n_tx_shares, &tx_s, &tx_e);

    std::vector<std::vector<uint32_t>> pfb_idx(pfb_inner.size());
    for (size_t i = 0; i < pfb_inner.size(); i++) pfb_idx[i].assign(pfb_nblobs[i], 0);
    int64_t non_reserved_start = tx_counter.size() + pfb_counter.size();
    int64_t cursor = non_reserved_start, end_of_last = non_reserved_start;
    struct BlobSeg {
        const Element* e;
        uint32_t padding_before;
    };
    std::vector<BlobSeg> bsegs;
    uint32_t writer_count = 0;   // shares written by the sparse splitter so far
    for (size_t i = 0; i < elems.size(); i++) {
        const Element& e = elems[i];
        const uint32_t w = subtree_width(e.num_shares, threshold);
        cursor = (cursor + w - 1) / w * w;                                  // inclusion.NextShareIndex
        if (i == 0) non_reserved_start = cursor;
        const int64_t padding = cursor - end_of_last;
        if (padding > (int64_t)e.max_padding) {
            *err = fmt("blob has %lld padding shares, but %lld was the max possible", padding, e.max_padding);
            return -1;
        }
        pfb_idx[e.pfb][e.blob] = (uint32_t)cursor;
        if (i > 0 && padding > 0 && writer_count == 0) {
            *err = "writing padding into sparse shares: cannot write namespace padding shares on an empty "
                   "SparseShareSplitter";
            return -1;
        }
        // SparseShareSplitter.Write: share version and namespace validation
        if ((uint8_t)e.share_version != 0) {
            *err = fmt("writing blob into sparse shares: unsupported share version: %lld", (uint8_t)e.share_version);
            return -1;
        }
        if (e.ns_version != 0 && e.ns_version != 255) {
            *err = fmt("writing blob into sparse shares: unsupported namespace version %lld", e.ns_version);
            return -1;
        }
        if (e.ns_id_len != kNs - 1) {
            *err = fmt("writing blob into sparse shares: unsupported namespace id length: id must be %lld bytes but it "
                       "was %lld bytes",
                       kNs - 1, e.ns_id_len);
            return -1;
        }
        if (e.ns_version == 0) {
            for (int z = 0; z < 18; z++)
                if (e.ns_id[z]) {
                    *err = "writing blob into sparse shares: unsupported namespace id with version 0: ID must start "
                           "with 18 leading zeros";
                    return -1;
                }
        }
        bsegs.push_back(BlobSeg{&e, i > 0 ? (uint32_t)padding : 0u});
        writer_count += (i > 0 ? (uint32_t)padding : 0u) + e.num_shares;
        cursor += e.num_shares;
        end_of_last = cursor;
    }

    std::vector<std::vector<uint8_t>> iws(pfb_inner.size());
    std::vector<Span> pfb_units;
    for (size_t i = 0; i < pfb_inner.size(); i++) {
        marshal_index_wrapper(pfb_inner[i], pfb_idx[i].data(), pfb_idx[i].size(), iws[i]);
        pfb_units.push_back(Span{iws[i].data(), iws[i].size(), true});
        for (uint32_t v : pfb_idx[i]) {
            P.share_indexes.push_back(v);
            P.share_index_pfb.push_back((uint32_t)i);
        }
    }
    compact_shares(kPfbNs, pfb_units, P.compact, &n_pfb_shares, &pfb_s, &pfb_e);
    // FindTxShareRange: the tx writer's ranges, then the PFB writer's offset by
    // the tx writer's share count; a repeated unit reports its last copy's range
    auto ranges = [&](const std::vector<Span>& units, const std::vector<uint32_t>& s0, const std::vector<uint32_t>& e0,
                      uint32_t base) {
        std::unordered_map<std::string_view, size_t> last;
        for (size_t i = 0; i < units.size(); i++)
            last[std::string_view(reinterpret_cast<const char*>(units[i].p), units[i].n)] = i;
        for (size_t i = 0; i < units.size(); i++) {
            const size_t j = last[std::string_view(reinterpret_cast<const char*>(units[i].p), units[i].n)];
            P.unit_start.push_back(base + s0[j]);
            P.unit_end.push_back(base + e0[j]);
        }
    };
    ranges(normal, tx_s, tx_e, 0);
    ranges(pfb_units, pfb_s, pfb_e, n_tx_shares);
    P.n_normal = (uint32_t)normal.size();
    if (pfb_counter.size() < (int64_t)n_pfb_shares) {
        *err = fmt("pfbCounter.Size() < pfbTxWriter.Count(): %lld < %lld", pfb_counter.size(), n_pfb_shares);
        return -1;
    }

    // ---- WriteSquare --------------------------------------------------------
    const int64_t total = (int64_t)ss * ss;
    const int64_t padding_start = n_tx_shares + n_pfb_shares;
    if (non_reserved_start < padding_start) {
        *err = fmt("writing square: nonReservedStart %lld is too small to fit all PFBs and txs", non_reserved_start);
        return -1;
    }
    const int64_t end_of_blobs = non_reserved_start + writer_count;
    if (total < end_of_blobs) {
        *err = fmt("writing square: square size %lld is too small to fit all blobs", total);
        return -1;
    }
    uint32_t at = 0;
    auto add = [&](uint32_t kind, uint32_t cnt, const uint8_t* ns, uint64_t src, uint32_t len) {
        if (!cnt) return;
        Segment s{};
        s.kind = kind;
        s.start = at;
        s.n = cnt;
        s.src = src;
        s.len = len;
        if (ns) std::memcpy(s.ns, ns, kNs);
        P.segs.push_back(s);
        at += cnt;
    };
    add(kSegCompact, n_tx_shares + n_pfb_shares, nullptr, 0, 0);
    add(kSegPadding, (uint32_t)(non_reserved_start - padding_start), kReservedPadNs, 0, 0);
    const uint8_t* last_ns = nullptr;
    std::vector<uint8_t> ns_store(bsegs.size() * kNs);
    for (size_t i = 0; i < bsegs.size(); i++) {
        const Element& e = *bsegs[i].e;
        uint8_t* ns = ns_store.data() + i * kNs;
        ns[0] = e.ns_version;
        std::memcpy(ns + 1, e.ns_id, kNs - 1);
        add(kSegPadding, bsegs[i].padding_before, last_ns, 0, 0);   // NamespacePaddingShares(last share's ns)
        add(kSegBlob, e.num_shares, ns, (uint64_t)(e.data - txs), e.len);
        if (e.num_shares) last_ns = ns;
    }
    add(kSegPadding, (uint32_t)(total - end_of_blobs), kTailPadNs, 0, 0);
    P.square_size = ss;
    return 0;
}

// inclusion.CreateCommitment layout for a batch of blobs: SplitBlobs (sparse
// shares), SubTreeWidth, MerkleMountainRangeSizes.  Validation follows
// SparseShareSplitter.Write (share version, namespace.New).
int plan_commitments(const uint8_t* namespaces, const uint64_t* data_off, const uint8_t* share_versions, uint32_t n,
                     uint32_t threshold, CommitPlan* out, std::string* err) {
    CommitPlan& P = *out;
    P.n_leaves = P.max_height = P.max_trees = P.n_trees = 0;
    P.segs.clear();
    P.seg_tree0.clear();
    P.blob_tree0.clear();
    if (threshold == 0) {
        *err = "subtree root threshold must be positive";
        return -1;
    }
    P.blob_tree0.reserve(n + 1);
    P.segs.reserve(2 * (size_t)n);
    P.seg_tree0.reserve(2 * (size_t)n);
    uint64_t cursor = 0;
    for (uint32_t b = 0; b < n; b++) {
        P.blob_tree0.push_back(P.n_trees);
        const uint8_t* ns = namespaces + (size_t)b * kNs;
        const uint8_t ver = share_versions ? share_versions[b] : 0;
        if (ver != 0) {
            *err = fmt("blob %lld: unsupported share version: %lld", b, ver);
            return -1;
        }
        if (ns[0] != 0 && ns[0] != 255) {
            *err = fmt("blob %lld: unsupported namespace version %lld", b, ns[0]);
            return -1;
        }
        if (ns[0] == 0)
            for (int z = 1; z < 19; z++)
                if (ns[z]) {
                    *err = fmt("blob %lld: unsupported namespace id with version 0: ID must start with 18 leading "
                               "zeros",
                               b);
                    return -1;
                }
        if (data_off[b + 1] < data_off[b]) {
            *err = "blob offsets must be non-decreasing";
            return -1;
        }
        const uint64_t len = data_off[b + 1] - data_off[b];
        if (len > 0xFFFFFFFFull) {
            *err = "blob too large";
            return -1;
        }
        const uint32_t n_sh = sparse_shares_needed((uint32_t)len);
        if (n_sh == 0) continue;   // nil data: no shares, commitment = sha256("")
        const uint32_t w = subtree_width(n_sh, threshold);
        const uint64_t start = (cursor + w - 1) / w * w;
        if (start > cursor) {   // alignment gap (never hashed into a used node)
            Segment g{};
            g.kind = kSegPadding;
            g.start = (uint32_t)cursor;
            g.n = (uint32_t)(start - cursor);
            P.segs.push_back(g);
            P.seg_tree0.push_back(kNoTree);
        }
        Segment s{};
        s.kind = kSegBlob;
        s.start = (uint32_t)start;
        s.n = n_sh;
        s.version = ver;
        s.src = data_off[b];
        s.len = (uint32_t)len;
        std::memcpy(s.ns, ns, kNs);
        uint32_t sub_log = 0;
        while ((1u << sub_log) < w) sub_log++;
        s.sub_log = (uint8_t)sub_log;
        P.segs.push_back(s);
        P.seg_tree0.push_back(P.n_trees);
        const uint32_t nt = mmr_tree_count(n_sh, sub_log);   // inclusion.MerkleMountainRangeSizes
        const uint32_t top = (n_sh >> sub_log) ? sub_log : 31u - (uint32_t)__builtin_clz(n_sh);
        P.max_height = std::max(P.max_height, top);
        P.n_trees += nt;
        P.max_trees = std::max(P.max_trees, nt);
        cursor = start + n_sh;
        if (cursor > 0x7FFFFFFFull) {
            *err = "blob batch too large";
            return -1;
        }
    }
    P.blob_tree0.push_back(P.n_trees);
    P.n_leaves = (uint32_t)cursor;
    return 0;
}

}  // namespace square
}  // namespace cda
