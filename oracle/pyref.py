"""Python restatement of the celestia-app DA hot path -- TEST INFRASTRUCTURE ONLY.

This module is part of the oracle: it is imported only by tests/, by the
fixture generator (oracle/gen_golden.py) and by __graft_entry__.smoke() as a
checker.  The product path (celestia-app_amd/) never imports it.

What it restates (reference files are under /root/reference):

* ``ods -> eds``: rsmt2d v0.14.0 ``ComputeExtendedDataSquare`` /
  ``erasureExtendSquare`` (EXT module, not vendored; schedule per
  specs/src/specs/data_structures.md:306-310): Q0->Q1 rows, Q0->Q2 columns,
  Q2->Q3 rows, called from pkg/da/data_availability_header.go:65-75.
* Leopard RS encode: klauspost/reedsolomon v1.12.1 ``leopardFF8.encode`` /
  ``leopardFF16.encode`` (EXT, not vendored; restated from the published
  algorithm -- SURVEY.md Appendix A), codec chosen by
  pkg/appconsts/global_consts.go:92 (rsmt2d.NewLeoRSCodec ->
  reedsolomon.New(k, k, WithLeopardGF(true))).
* NMT: pkg/wrapper/nmt_wrapper.go:93-140 (namespace prefixing, quadrant
  test) and the nmt hasher rules copied in-tree at
  test/util/malicious/hasher.go:161-310 (HashLeaf / HashNode / computeNsRange /
  EmptyRoot) with IgnoreMaxNamespace(true).
* DAH: pkg/da/data_availability_header.go:44-108 and go-square/merkle
  ``HashFromByteSlices`` (RFC-6962).

Pinning: NMT + DAH are pinned by the reference's golden hashes
(pkg/da/data_availability_header_test.go:15-66); RS GF(2^8) is additionally
pinned by mainnet block 408 (x/blob/test/testdata/block_response.json) via
oracle/square.py; RS GF(2^16) is checked only intrinsically (Lagrange
interpolation cross-check, MDS) -- "parity unpinned" for k > 128.
"""
from __future__ import annotations

import hashlib
from functools import lru_cache

import numpy as np

SHARE_SIZE = 512          # pkg/appconsts/global_consts.go:29
NAMESPACE_SIZE = 29       # pkg/appconsts/global_consts.go:26
NMT_NODE_SIZE = 2 * NAMESPACE_SIZE + 32
PARITY_NS = b"\xff" * NAMESPACE_SIZE   # go-square namespace.ParitySharesNamespace
LEAF_PREFIX = b"\x00"
NODE_PREFIX = b"\x01"

# ---------------------------------------------------------------------------
# Leopard field tables (klauspost/reedsolomon v1.12.1 leopard8.go initLUTs8 /
# leopard.go initLUTs)
# ---------------------------------------------------------------------------
CANTOR8 = (1, 214, 152, 146, 86, 200, 88, 230)
CANTOR16 = (0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
            0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E)


class Field:
    def __init__(self, bits: int, poly: int, cantor):
        self.bits = bits
        self.order = 1 << bits
        self.mod = self.order - 1
        order, mod = self.order, self.mod
        exp = [0] * order
        log = [0] * order
        state = 1
        for i in range(mod):           # LFSR: exp[] temporarily holds discrete logs
            exp[state] = i
            state <<= 1
            if state >= order:
                state ^= poly
        exp[0] = mod
        log[0] = 0                     # Cantor-basis coordinates -> poly-basis value
        for i in range(bits):
            width = 1 << i
            for j in range(width):
                log[j + width] = log[j] ^ cantor[i]
        for i in range(order):
            log[i] = exp[log[i]]
        for i in range(order):
            exp[log[i]] = i
        exp[mod] = exp[0]
        self.exp = exp
        self.log = log
        self.exp_np = np.array(exp, dtype=np.int64)
        self.log_np = np.array(log, dtype=np.int64)
        self.skew = self._init_fft()

    def add_mod(self, a: int, b: int) -> int:
        s = a + b
        return (s + (s >> self.bits)) & self.mod

    def mul_log(self, a: int, log_b: int) -> int:
        if a == 0:
            return 0
        return self.exp[self.add_mod(self.log[a], log_b)]

    def _init_fft(self):
        # leopard initFFT8 / initFFT
        bits, mod, log = self.bits, self.mod, self.log
        temp = [1 << i for i in range(1, bits)]
        skew = [0] * mod
        for m in range(bits - 1):
            step = 1 << (m + 1)
            skew[(1 << m) - 1] = 0
            for i in range(m, bits - 1):
                s = 1 << (i + 1)
                for j in range((1 << m) - 1, s, step):
                    skew[j + s] = skew[j] ^ temp[i]
            temp[m] = mod - log[self.mul_log(temp[m], log[temp[m] ^ 1])]
            for i in range(m + 1, bits - 1):
                temp[i] = self.mul_log(temp[i], self.add_mod(log[temp[i] ^ 1], temp[m]))
        return [log[s] for s in skew]

    # vectorised multiply of a symbol array by exp(log_m)
    def mul_np(self, y: np.ndarray, log_m: int) -> np.ndarray:
        lg = self.log_np[y] + log_m
        lg = (lg + (lg >> self.bits)) & self.mod
        out = self.exp_np[lg]
        out[y == 0] = 0
        return out


@lru_cache(maxsize=None)
def gf8() -> Field:
    return Field(8, 0x11D, CANTOR8)


@lru_cache(maxsize=None)
def gf16() -> Field:
    return Field(16, 0x1002D, CANTOR16)


def field_for(k: int) -> Field:
    # reedsolomon.New: total shards > 256 -> leopardFF16, else (WithLeopardGF) FF8
    return gf8() if 2 * k <= 256 else gf16()


def _encode_symbols(F: Field, w: np.ndarray) -> np.ndarray:
    """Leopard encode, data shards == parity shards == m (a power of two).

    ``w`` has shape (m, lanes) of field symbols (int64).  Radix-2 restatement of
    ifftDITEncoder (coset m) followed by fftDIT (coset 0); upstream fuses the
    layers two at a time (ifftDIT4/fftDIT4) in the identical order.
    """
    m = w.shape[0]
    w = w.copy()
    skew, mod = F.skew, F.mod
    d = 1
    while d < m:                                   # IFFT, decimation in time
        for g in range(0, m, 2 * d):
            L = skew[m - 1 + g + d]
            x = w[g:g + d]
            y = w[g + d:g + 2 * d]
            y ^= x
            if L != mod:
                x ^= F.mul_np(y, L)
        d <<= 1
    d = m >> 1
    while d >= 1:                                  # FFT
        for g in range(0, m, 2 * d):
            L = skew[g + d - 1]
            x = w[g:g + d]
            y = w[g + d:g + 2 * d]
            if L != mod:
                x ^= F.mul_np(y, L)
            y ^= x
        d >>= 1
    return w


def leopard_encode(data: np.ndarray) -> np.ndarray:
    """rsmt2d LeoRSCodec.Encode: k shards (k, L) uint8 -> k parity shards."""
    data = np.asarray(data, dtype=np.uint8)
    k, L = data.shape
    if L % 64:
        raise ValueError(f"chunkSize {L} must be a multiple of 64 bytes")
    if k == 1:
        return data.copy()
    if k & (k - 1):
        # klauspost leopardFF8/16 encode with dataShards == parityShards == k
        # (rsmt2d LeoRSCodec.Encode of a non-power-of-two shard count, e.g.
        # pkg/wrapper/nmt_wrapper_test.go:152-180): m = ceilPow2(k), the IFFT
        # reads the k data shards and zeros up to m (ifftDITEncoder's mtrunc),
        # the first k FFT outputs are the parity.
        m = 1 << (k - 1).bit_length()
        pad = np.zeros((m, L), dtype=np.uint8)
        pad[:k] = data
        return leopard_encode(pad)[:k]
    F = field_for(k)
    if F.bits == 8:
        out = _encode_symbols(F, data.astype(np.int64))
        return out.astype(np.uint8)
    # GF(2^16): within each 64-byte block symbol i = b[i] | b[i+32] << 8
    blk = data.reshape(k, L // 64, 2, 32).astype(np.int64)
    sym = blk[:, :, 0, :] | (blk[:, :, 1, :] << 8)
    out = _encode_symbols(F, sym.reshape(k, -1)).reshape(k, L // 64, 32)
    res = np.empty((k, L // 64, 2, 32), dtype=np.uint8)
    res[:, :, 0, :] = out & 0xFF
    res[:, :, 1, :] = out >> 8
    return res.reshape(k, L)


def extend_square(ods: np.ndarray) -> np.ndarray:
    """ods (k, k, S) uint8 -> eds (2k, 2k, S); rsmt2d erasureExtendSquare."""
    k = ods.shape[0]
    S = ods.shape[2]
    eds = np.zeros((2 * k, 2 * k, S), dtype=np.uint8)
    eds[:k, :k] = ods
    for i in range(k):                       # Q0 -> Q1 (rows)
        eds[i, k:] = leopard_encode(eds[i, :k])
    for j in range(k):                       # Q0 -> Q2 (columns)
        eds[k:, j] = leopard_encode(eds[:k, j])
    for i in range(k, 2 * k):                # Q2 -> Q3 (rows)
        eds[i, k:] = leopard_encode(eds[i, :k])
    return eds


# ---------------------------------------------------------------------------
# NMT (test/util/malicious/hasher.go:161-310, pkg/wrapper/nmt_wrapper.go:93-140)
# ---------------------------------------------------------------------------
def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def nmt_hash_leaf(ndata: bytes) -> bytes:
    ns = ndata[:NAMESPACE_SIZE]
    return ns + ns + sha256(LEAF_PREFIX + ndata)


def nmt_hash_node(left: bytes, right: bytes) -> bytes:
    lmin, lmax = left[:NAMESPACE_SIZE], left[NAMESPACE_SIZE:2 * NAMESPACE_SIZE]
    rmin, rmax = right[:NAMESPACE_SIZE], right[NAMESPACE_SIZE:2 * NAMESPACE_SIZE]
    mx = lmax if rmin == PARITY_NS else rmax       # IgnoreMaxNamespace(true)
    return lmin + mx + sha256(NODE_PREFIX + left + right)


def nmt_empty_root() -> bytes:
    return b"\x00" * (2 * NAMESPACE_SIZE) + sha256(b"")


def _split_point(n: int) -> int:
    # largest power of two strictly less than n (RFC-6962)
    k = 1
    while k * 2 < n:
        k *= 2
    return k


def nmt_root_from_nodes(nodes) -> bytes:
    n = len(nodes)
    if n == 0:
        return nmt_empty_root()
    if n == 1:
        return nodes[0]
    k = _split_point(n)
    return nmt_hash_node(nmt_root_from_nodes(nodes[:k]), nmt_root_from_nodes(nodes[k:]))


class PushOrderError(ValueError):
    pass


def erasured_leaves(cells, k: int, axis_index: int, blind: bool = False):
    """ErasuredNamespacedMerkleTree.Push for every cell of one row/column.
    blind: test/util/malicious/tree.go:18-26 BlindTree (ForceAddLeaf: no
    namespace-order check; the malicious hasher above checks no sibling order
    either), the tree the reference's fraud tests build unordered squares with."""
    leaves = []
    last_ns = None
    for share_index, cell in enumerate(cells):
        cell = bytes(cell)
        if len(cell) < NAMESPACE_SIZE:
            raise ValueError("data is too short to contain namespace ID")
        ns = cell[:NAMESPACE_SIZE] if (share_index < k and axis_index < k) else PARITY_NS
        if not blind and last_ns is not None and ns < last_ns:
            raise PushOrderError(
                "pushed data has to be lexicographically ordered by namespace IDs: "
                f"last namespace: {last_ns.hex()}, pushed: {ns.hex()}")
        last_ns = ns
        leaves.append(nmt_hash_leaf(ns + cell))
    return leaves


def axis_root(cells, k: int, axis_index: int, blind: bool = False) -> bytes:
    return nmt_root_from_nodes(erasured_leaves(cells, k, axis_index, blind))


# ---------------------------------------------------------------------------
# RFC-6962 merkle (go-square/merkle HashFromByteSlices)
# ---------------------------------------------------------------------------
def merkle_root(items) -> bytes:
    n = len(items)
    if n == 0:
        return sha256(b"")
    if n == 1:
        return sha256(LEAF_PREFIX + items[0])
    k = _split_point(n)
    return sha256(NODE_PREFIX + merkle_root(items[:k]) + merkle_root(items[k:]))


def dah_from_eds(eds: np.ndarray, blind: bool = False):
    """NewDataAvailabilityHeader; blind: over malicious.NewConstructor's trees."""
    W = eds.shape[0]
    k = W // 2
    rows = [axis_root(eds[i], k, i, blind) for i in range(W)]
    cols = [axis_root(eds[:, j], k, j, blind) for j in range(W)]
    return rows, cols, merkle_root(rows + cols)


def extend_and_dah(ods: np.ndarray):
    eds = extend_square(ods)
    rows, cols, root = dah_from_eds(eds)
    return eds, rows, cols, root


# ---------------------------------------------------------------------------
# Inputs
# ---------------------------------------------------------------------------
def tail_padding_share() -> bytes:
    # specs/src/specs/shares.md:71-81, namespace.md:83 (TAIL_PADDING_NAMESPACE)
    ns = b"\xff" + b"\xff" * 27 + b"\xfe"
    return ns + b"\x01" + b"\x00" * 4 + b"\x00" * (SHARE_SIZE - NAMESPACE_SIZE - 5)


def constant_shares(count: int) -> np.ndarray:
    """pkg/da/data_availability_header_test.go:247-263 generateShares."""
    ns1 = b"\x00" + b"\x00" * 18 + b"\x01" * 10     # MustNewV0(Repeat(1, 10))
    share = ns1 + b"\xff" * (SHARE_SIZE - NAMESPACE_SIZE)
    return np.frombuffer(share * count, dtype=np.uint8).reshape(count, SHARE_SIZE).copy()


MASK64 = (1 << 64) - 1


def splitmix64_bytes(seed: int, n: int) -> bytes:
    """Successive little-endian outputs of SplitMix64 (gamma 0x9E3779B97F4A7C15)."""
    cnt = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed & MASK64) + np.arange(1, cnt + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:n]


SEED_BASE = 0xCE1E57A0


def random_namespaced_square(k: int, square_index: int = 0) -> np.ndarray:
    """SURVEY.md 8(d) synthetic square; mirrors test/util/testfactory/common.go:36-46.

    Stream = splitmix64(seed); per share draw 10 namespace-id bytes (re-draw
    while the first 9 are zero: primary-reserved / not a blob namespace, see
    testfactory/namespace.go:15-28) then 483 payload bytes.  Shares are sorted
    bytewise and laid out row-major.  Returns (k*k, 512) uint8.
    """
    n = k * k
    # draw generously; each share consumes 10 (+10 per redraw) + 483 bytes
    need = n * 493 + 4096
    stream = splitmix64_bytes(SEED_BASE + square_index, need)
    shares = []
    pos = 0
    for _ in range(n):
        while True:
            nid = stream[pos:pos + 10]
            pos += 10
            if any(nid[:9]):
                break
        payload = stream[pos:pos + 483]
        pos += 483
        shares.append(b"\x00" + b"\x00" * 18 + nid + payload)
    shares.sort()
    return np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(n, SHARE_SIZE).copy()


def ods_from_shares(shares: np.ndarray) -> np.ndarray:
    n = shares.shape[0]
    k = int(round(n ** 0.5))
    assert k * k == n
    return shares.reshape(k, k, SHARE_SIZE)
