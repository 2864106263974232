"""Square construction (txs -> ODS) -- TEST INFRASTRUCTURE ONLY (oracle).

Restates go-square v1.1.0 ``square.Construct`` (EXT module pinned at
/root/reference/go.mod:9; not vendored) from the specs under
/root/reference/specs/src/specs/: data_square_layout.md (blob share
commitment rules, padding), shares.md (share format, compact and sparse
shares, padding shares), namespace.md (reserved namespaces) and
data_structures.md (IndexWrapper / BlobTx).  Call sites in the reference:
app/prepare_proposal.go:50, app/process_proposal.go:122, app/extend_block.go:16.

Its only job here is to pin the Leopard GF(2^8) restatement with real data:
mainnet block 408 (x/blob/test/testdata/block_response.json, k = 32) has a
data root that depends on real (non-constant) Reed-Solomon parity.
"""
from __future__ import annotations

import base64
import json
import math

SHARE_SIZE = 512
NS_SIZE = 29
SUBTREE_ROOT_THRESHOLD = 64          # pkg/appconsts/v1/app_consts.go

TX_NS = b"\x00" * 28 + b"\x01"
PFB_NS = b"\x00" * 28 + b"\x04"
PRIMARY_RESERVED_PADDING_NS = b"\x00" * 28 + b"\xff"
TAIL_PADDING_NS = b"\xff" * 28 + b"\xfe"


# ---------------------------------------------------------------- protobuf
def _varint(buf: bytes, i: int):
    x, s = 0, 0
    while True:
        b = buf[i]
        i += 1
        x |= (b & 0x7F) << s
        s += 7
        if b < 0x80:
            return x, i


def _enc_varint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fields(buf: bytes):
    i = 0
    while i < len(buf):
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            n, i = _varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ValueError("unsupported wire type")
        yield fn, wt, v


def unmarshal_blob_tx(tx: bytes):
    """go-square tx.UnmarshalBlobTx: BlobTx{tx=1, blobs=2, type_id=3 == "BLOB"}."""
    try:
        inner, blobs, type_id = b"", [], b""
        for fn, wt, v in _fields(tx):
            if fn == 1 and wt == 2:
                inner = v
            elif fn == 2 and wt == 2:
                blob = {"namespace_id": b"", "data": b"", "share_version": 0, "namespace_version": 0}
                for bf, bw, bv in _fields(v):
                    if bf == 1:
                        blob["namespace_id"] = bv
                    elif bf == 2:
                        blob["data"] = bv
                    elif bf == 3:
                        blob["share_version"] = bv
                    elif bf == 4:
                        blob["namespace_version"] = bv
                blobs.append(blob)
            elif fn == 3 and wt == 2:
                type_id = v
    except Exception:
        return None
    if type_id != b"BLOB":
        return None
    return inner, blobs


def marshal_index_wrapper(tx: bytes, share_indexes) -> bytes:
    """IndexWrapper{tx=1, share_indexes=2 (packed), type_id=3 = "INDX"} (gogoproto order)."""
    out = bytearray()
    if tx:
        out += b"\x0a" + _enc_varint(len(tx)) + tx
    if share_indexes:
        packed = b"".join(_enc_varint(x) for x in share_indexes)
        out += b"\x12" + _enc_varint(len(packed)) + packed
    out += b"\x1a\x04INDX"
    return bytes(out)


# ------------------------------------------------------------------ shares
def _info_byte(version: int, start: bool) -> int:
    return (version << 1) | (1 if start else 0)


def compact_shares(ns: bytes, units) -> list:
    """CompactShareSplitter: varint-delimited units, reserved bytes = offset
    of the first unit starting in the share (shares.md "Transaction Shares")."""
    shares = []
    cur = None
    reserved_set = False

    def new_share(first: bool):
        b = bytearray(ns + bytes([_info_byte(0, first)]))
        if first:
            b += b"\x00" * 4           # sequence length, filled at export
        res_at = len(b)
        b += b"\x00" * 4               # reserved bytes
        return b, res_at

    res_at = 0
    total = 0
    for u in units:
        data = _enc_varint(len(u)) + u
        total += len(data)
        if cur is None:
            cur, res_at = new_share(True)
            reserved_set = False
        if not reserved_set:
            cur[res_at:res_at + 4] = len(cur).to_bytes(4, "big")
            reserved_set = True
        while data:
            room = SHARE_SIZE - len(cur)
            cur += data[:room]
            data = data[room:]
            if len(cur) == SHARE_SIZE:
                shares.append(cur)
                cur, res_at = new_share(False)
                reserved_set = False
    if cur is not None and len(cur) > res_at + 4:
        cur += b"\x00" * (SHARE_SIZE - len(cur))
        shares.append(cur)
    if shares:
        shares[0][NS_SIZE + 1:NS_SIZE + 5] = total.to_bytes(4, "big")
    return [bytes(s) for s in shares]


def compact_share_ranges(units) -> list:
    """CompactShareSplitter.WriteTx's recorded share range per unit, as
    (start, end): start = the shares completed before the unit is written,
    end = Count() after it (completed shares + the pending one if it holds
    data).  The splitter keys its range map by the tx hash, so equal units
    all report the range of the last one written (ShareRanges)."""
    out, done, fill = [], 0, None      # fill: bytes in the pending share (None: no share yet)
    for u in units:
        n = len(_enc_varint(len(u))) + len(u)
        if fill is None:
            fill = NS_SIZE + 1 + 4 + 4          # first share: ns, info, sequence length, reserved
        start = done
        while n:
            take = min(SHARE_SIZE - fill, n)
            fill += take
            n -= take
            if fill == SHARE_SIZE:
                done += 1
                fill = NS_SIZE + 1 + 4          # continuation: ns, info, reserved
        header = NS_SIZE + 1 + 4 + (4 if done == 0 else 0)
        out.append((start, done + (1 if fill > header else 0)))
    last = {bytes(u): i for i, u in enumerate(units)}
    return [out[last[bytes(u)]] for u in units]


def find_tx_share_range(txs, tx_index: int, max_square_size: int = 128,
                        threshold: int = SUBTREE_ROOT_THRESHOLD):
    """go-square builder.FindTxShareRange after square.Construct's layout
    (pkg/proof/proof.go:22-49): (start, end, is_pfb) of kept tx tx_index --
    normal txs in the tx namespace's compact shares, then blob txs as their
    IndexWrapper in the PFB namespace's, offset by the tx shares."""
    _, _, kept, share_idx = builder(txs, max_square_size, threshold, "construct")
    normal, pfbs, at = [], [], 0
    for t in kept:
        bt = unmarshal_blob_tx(txs[t])
        if bt is None:
            normal.append(txs[t])
        else:
            inner, bl = bt
            pfbs.append(marshal_index_wrapper(inner, share_idx[at:at + len(bl)]))
            at += len(bl)
    if tx_index >= len(normal) + len(pfbs):
        raise ValueError(f"txIndex {tx_index} out of range")
    if tx_index < len(normal):
        s, e = compact_share_ranges(normal)[tx_index]
        return s, e, False
    n_tx = len(compact_shares(TX_NS, normal))
    s, e = compact_share_ranges(pfbs)[tx_index - len(normal)]
    return n_tx + s, n_tx + e, True


def sparse_shares(ns: bytes, data: bytes, version: int = 0) -> list:
    out = []
    first = bytearray(ns + bytes([_info_byte(version, True)]) + len(data).to_bytes(4, "big"))
    room = SHARE_SIZE - len(first)
    first += data[:room]
    data = data[room:]
    out.append(first)
    while data:
        s = bytearray(ns + bytes([_info_byte(version, False)]))
        room = SHARE_SIZE - len(s)
        s += data[:room]
        data = data[room:]
        out.append(s)
    return [bytes(s) + b"\x00" * (SHARE_SIZE - len(s)) for s in out]


def padding_share(ns: bytes) -> bytes:
    s = ns + bytes([_info_byte(0, True)]) + b"\x00" * 4
    return s + b"\x00" * (SHARE_SIZE - len(s))


def sparse_share_count(n_bytes: int) -> int:
    if n_bytes <= SHARE_SIZE - NS_SIZE - 5:
        return 1
    rest = n_bytes - (SHARE_SIZE - NS_SIZE - 5)
    return 1 + -(-rest // (SHARE_SIZE - NS_SIZE - 1))


# ----------------------------------------------------------------- layout
def round_up_pow2(x: int) -> int:
    r = 1
    while r < x:
        r <<= 1
    return r


def blob_min_square_size(share_count: int) -> int:
    return round_up_pow2(int(math.ceil(math.sqrt(share_count))))


def subtree_width(share_count: int, threshold: int = SUBTREE_ROOT_THRESHOLD) -> int:
    s = share_count // threshold + (1 if share_count % threshold else 0)
    return min(round_up_pow2(s), blob_min_square_size(share_count))


def next_share_index(cursor: int, blob_share_len: int, threshold: int = SUBTREE_ROOT_THRESHOLD) -> int:
    w = subtree_width(blob_share_len, threshold)
    return -(-cursor // w) * w


FIRST_COMPACT_CONTENT = SHARE_SIZE - NS_SIZE - 1 - 4 - 4        # 474
CONT_COMPACT_CONTENT = SHARE_SIZE - NS_SIZE - 1 - 4             # 478
WORST_CASE_SHARE_INDEX = 128 * 128                               # worstCaseShareIndexes


class CompactShareCounter:
    """go-square shares.CompactShareCounter (share-count estimate)."""

    def __init__(self):
        self.shares = 0
        self.remainder = 0
        self.last = (0, 0)

    def revert(self):
        self.shares, self.remainder = self.last

    def add(self, data_len: int) -> int:
        """Returns the change of size() (the Go counter's diff)."""
        before = self.size()
        self.last = (self.shares, self.remainder)
        data_len += len(_enc_varint(data_len))
        if self.shares == 0:
            if data_len >= FIRST_COMPACT_CONTENT - self.remainder:
                data_len -= FIRST_COMPACT_CONTENT - self.remainder
                self.shares += 1
                self.remainder = 0
            else:
                self.remainder += data_len
                data_len = 0
        if data_len >= CONT_COMPACT_CONTENT - self.remainder:
            data_len -= CONT_COMPACT_CONTENT - self.remainder
            self.shares += 1
            self.remainder = 0
        else:
            self.remainder += data_len
            data_len = 0
        if data_len > 0:
            self.shares += data_len // CONT_COMPACT_CONTENT
            self.remainder = data_len % CONT_COMPACT_CONTENT
        return self.size() - before

    def size(self) -> int:
        return self.shares if self.remainder == 0 else self.shares + 1


def construct(txs, square_size: int, threshold: int = SUBTREE_ROOT_THRESHOLD) -> list:
    """square.Construct (Builder.AppendTx / AppendBlobTx / Export / WriteSquare)
    for the block's own square size."""
    normal, pfbs, blobs = [], [], []
    tx_counter, pfb_counter = CompactShareCounter(), CompactShareCounter()
    for tx in txs:
        bt = unmarshal_blob_tx(tx)
        if bt is None:
            if pfbs:
                raise ValueError("normal tx can not be appended after blob tx")
            normal.append(tx)
            tx_counter.add(len(tx))
        else:
            inner, bl = bt
            pidx = len(pfbs)
            pfbs.append([inner, [0] * len(bl)])
            pfb_counter.add(len(marshal_index_wrapper(inner, [WORST_CASE_SHARE_INDEX] * len(bl))))
            for bi, b in enumerate(bl):
                ns = bytes([b["namespace_version"]]) + b["namespace_id"]
                blobs.append((ns, b["data"], b["share_version"], pidx, bi))
    blobs.sort(key=lambda e: e[0])               # sort.SliceStable by namespace
    tx_shares = compact_shares(TX_NS, normal)
    cursor = tx_counter.size() + pfb_counter.size()
    non_reserved_start = cursor
    layout = []
    for i, (ns, data, ver, pidx, bi) in enumerate(blobs):
        n = sparse_share_count(len(data))
        cursor = next_share_index(cursor, n, threshold)
        if i == 0:
            non_reserved_start = cursor
        pfbs[pidx][1][bi] = cursor
        layout.append((cursor, ns, data, ver))
        cursor += n
    pfb_shares = compact_shares(PFB_NS, [marshal_index_wrapper(t, idx) for t, idx in pfbs])
    total = square_size * square_size
    square = list(tx_shares) + list(pfb_shares)
    if layout:
        square += [padding_share(PRIMARY_RESERVED_PADDING_NS)] * (non_reserved_start - len(square))
        prev_ns = None
        for pos, ns, data, ver in layout:
            if len(square) < pos:
                square += [padding_share(prev_ns)] * (pos - len(square))
            square += sparse_shares(ns, data, ver)
            prev_ns = ns
    if len(square) > total:
        raise ValueError("square size too small to fit all blobs")
    square += [padding_share(TAIL_PADDING_NS)] * (total - len(square))
    return square


def load_block(path: str):
    d = json.load(open(path))["block"]
    txs = [base64.b64decode(t) for t in d["data"]["txs"]]
    k = int(d["data"]["square_size"])
    data_hash = base64.b64decode(d["header"]["data_hash"])
    return txs, k, data_hash


# ------------------------------------------------- builder (Construct / Build)
def _valid_blob_namespace(ns_version: int, ns_id: bytes) -> bool:
    """namespace.New checks run by SparseShareSplitter.Write."""
    if ns_version not in (0, 255) or len(ns_id) != NS_SIZE - 1:
        return False
    return ns_version != 0 or ns_id[:18] == b"\x00" * 18


def builder(txs, max_square_size: int = 128, threshold: int = SUBTREE_ROOT_THRESHOLD, mode: str = "construct"):
    """go-square square.Construct (mode "construct") / square.Build ("build"):
    NewBuilder + AppendTx / AppendBlobTx (worst-case share accounting, canFit
    against max_square_size^2) + Export (square size = BlobMinSquareSize of the
    worst-case total) + WriteSquare.  Structure as in the reference's copy,
    test/util/malicious/out_of_order_builder.go:24-161.

    Returns (shares, square_size, kept tx indexes, share indexes per blob in
    PFB order); raises ValueError with go-square's message."""
    cap = max_square_size * max_square_size
    txc, pfbc = CompactShareCounter(), CompactShareCounter()
    current = 0
    normal, normal_idx, blob_idx, pfbs, elems = [], [], [], [], []
    seen_blob = False
    for t, tx in enumerate(txs):
        bt = unmarshal_blob_tx(tx)
        if bt is not None:
            seen_blob = True
            inner, bl = bt
            diff = pfbc.add(len(marshal_index_wrapper(inner, [WORST_CASE_SHARE_INDEX] * len(bl))))
            es, worst = [], 0
            for bi, b in enumerate(bl):
                n = sparse_share_count(len(b["data"])) if b["data"] else 0
                maxpad = subtree_width(n, threshold) - 1
                worst += n + maxpad
                ns_version = b["namespace_version"] & 0xFF
                es.append(dict(ns=bytes([ns_version]) + b["namespace_id"], ns_version=ns_version,
                               ns_id=b["namespace_id"], data=b["data"], ver=b["share_version"],
                               pfb=len(pfbs), bi=bi, n=n, maxpad=maxpad))
            if current + diff + worst <= cap:
                current += diff + worst
                elems += es
                pfbs.append([inner, [0] * len(bl)])
                blob_idx.append(t)
            else:
                pfbc.revert()
                if mode == "construct":
                    raise ValueError(f"not enough space to append blob tx at index {t}")
        else:
            if mode == "construct" and seen_blob:
                raise ValueError(f"normal transaction at index {t} can not be appended after blob tx")
            diff = txc.add(len(tx))
            if current + diff <= cap:
                current += diff
                normal.append(tx)
                normal_idx.append(t)
            else:
                txc.revert()
                if mode == "construct":
                    raise ValueError(f"not enough space to append tx at index {t}")
    kept = normal_idx + blob_idx
    if not normal and not pfbs:
        return [padding_share(TAIL_PADDING_NS)], 1, kept, []
    ss = blob_min_square_size(current)
    elems.sort(key=lambda e: e["ns"])                       # stable
    tx_shares = compact_shares(TX_NS, normal)
    cursor = end_of_last = non_reserved_start = txc.size() + pfbc.size()
    blob_part = []
    for i, e in enumerate(elems):
        cursor = next_share_index(cursor, e["n"], threshold)
        if i == 0:
            non_reserved_start = cursor
        padding = cursor - end_of_last
        if padding > e["maxpad"]:
            raise ValueError(f"blob has {padding} padding shares, but {e['maxpad']} was the max possible")
        pfbs[e["pfb"]][1][e["bi"]] = cursor
        if i > 0 and padding:
            if not blob_part:
                raise ValueError("cannot write namespace padding shares on an empty SparseShareSplitter")
            blob_part += [padding_share(blob_part[-1][:NS_SIZE])] * padding
        if e["ver"] & 0xFF != 0:
            raise ValueError(f"unsupported share version: {e['ver'] & 0xFF}")
        if not _valid_blob_namespace(e["ns_version"], e["ns_id"]):
            raise ValueError("invalid blob namespace")
        if e["n"]:
            blob_part += sparse_shares(e["ns"], e["data"], 0)
        cursor += e["n"]
        end_of_last = cursor
    pfb_shares = compact_shares(PFB_NS, [marshal_index_wrapper(t, idx) for t, idx in pfbs])
    total = ss * ss
    if non_reserved_start < len(tx_shares) + len(pfb_shares):
        raise ValueError("nonReservedStart is too small to fit all PFBs and txs")
    square = list(tx_shares) + list(pfb_shares)
    square += [padding_share(PRIMARY_RESERVED_PADDING_NS)] * (non_reserved_start - len(square))
    square += blob_part
    if len(square) > total:
        raise ValueError(f"square size {total} is too small to fit all blobs")
    square += [padding_share(TAIL_PADDING_NS)] * (total - len(square))
    return square, ss, kept, [i for _, idx in pfbs for i in idx]
