"""Python restatement of EDS repair -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/ (and fixture scripts) as the checker for
celestia-app_amd's cda_rs_decode / cda_repair; the product path never
imports it.

Restates (EXT modules, not vendored in /root/reference; pins go.mod:11,13):

* klauspost/reedsolomon v1.12.1 ``leopardFF8.reconstruct`` /
  ``leopardFF16.reconstruct`` (rsmt2d LeoRSCodec.Decode -> Reconstruct):
  erasure flags -> FWHT -> x logWalsh -> FWHT (error-locator logs), work =
  received * g^errLoc, IFFT (skew offset 0), formal derivative, FFT, erased
  shard = work * g^-errLoc.  Work index of data shard i is m + i, of parity
  shard i is i (m = number of parity shards = k).
* celestiaorg/rsmt2d v0.14.0 ``ExtendedDataSquare.Repair``:
  preRepairSanityCheck (complete rows / columns must match their roots and
  their parity must re-encode) followed by solveCrossword, which loops
  ``for i: solveCrosswordRow(i); solveCrosswordCol(i)`` until solved or no
  progress (ErrUnrepairableDataSquare).  A rebuilt vector whose root
  differs, or an orthogonal vector it completes whose root or encoding
  differs, is ErrByzantineData{axis, index}.  rsmt2d's Repair is called by
  celestia-node after sampling (specs/src/specs/data_structures.md:283-294).

Parity pin: decoding is unique (MDS), so the reference's reconstructed bytes
are the original EDS bytes; the tests check erase -> repair round trips
against oracle-extended squares, including block 408's real square.
"""
from __future__ import annotations

import numpy as np

import pyref

ROW, COL = 0, 1


class ErrByzantineData(Exception):
    def __init__(self, axis: int, index: int):
        super().__init__(f"byzantine {'row' if axis == ROW else 'col'}: {index}")
        self.axis, self.index = axis, index


class ErrUnrepairableDataSquare(Exception):
    def __init__(self):
        super().__init__("failed to solve data square")


class ErrBadRoot(Exception):
    pass


def _fwht_mod(a: np.ndarray, mod: int) -> np.ndarray:
    """leopard fwht(data, order, order) with exact arithmetic mod MOD."""
    a = a.copy()
    n = a.shape[0]
    d = 1
    while d < n:
        v = a.reshape(-1, 2, d)
        x, y = v[:, 0, :].copy(), v[:, 1, :].copy()
        v[:, 0, :] = (x + y) % mod
        v[:, 1, :] = (x - y) % mod
        d <<= 1
    return a


_LOG_WALSH = {}


def _log_walsh(F: pyref.Field) -> np.ndarray:
    # initFFT: logWalsh = logLUT with logWalsh[0] = 0, then fwht
    if F.bits not in _LOG_WALSH:
        lw = F.log_np.copy()
        lw[0] = 0
        _LOG_WALSH[F.bits] = _fwht_mod(lw, F.mod)
    return _LOG_WALSH[F.bits]


def error_locator_logs(F: pyref.Field, erased_work_indexes) -> np.ndarray:
    err = np.zeros(F.order, dtype=np.int64)
    for i in erased_work_indexes:
        err[i] = 1
    err = _fwht_mod(err, F.mod)
    err = (err * _log_walsh(F)) % F.mod
    return _fwht_mod(err, F.mod)


def _decode_symbols(F: pyref.Field, sym: np.ndarray, present: np.ndarray) -> np.ndarray:
    """sym: (2k, lanes) symbols in rsmt2d order (data then parity)."""
    n = sym.shape[0]
    m = n // 2
    work_of = lambda p: p + m if p < m else p - m   # data i -> m + i, parity i -> i
    erased = [work_of(p) for p in range(n) if not present[p]]
    el = error_locator_logs(F, erased)
    work = np.zeros_like(sym)
    for p in range(n):
        if present[p]:
            work[work_of(p)] = F.mul_np(sym[p], int(el[work_of(p)]))
    skew, mod = F.skew, F.mod
    d = 1
    while d < n:                                   # ifftDITDecoder, skew offset 0
        for g in range(0, n, 2 * d):
            L = skew[g + d - 1]
            x, y = work[g:g + d], work[g + d:g + 2 * d]
            y ^= x
            if L != mod:
                x ^= F.mul_np(y, L)
        d <<= 1
    for i in range(1, n):                          # formal derivative
        w = ((i ^ (i - 1)) + 1) >> 1
        work[i - w:i] ^= work[i:i + w]
    d = n >> 1
    while d >= 1:                                  # fftDIT
        for g in range(0, n, 2 * d):
            L = skew[g + d - 1]
            x, y = work[g:g + d], work[g + d:g + 2 * d]
            if L != mod:
                x ^= F.mul_np(y, L)
            y ^= x
        d >>= 1
    out = sym.copy()
    for p in range(n):
        if not present[p]:
            w = work_of(p)
            out[p] = F.mul_np(work[w], mod - int(el[w]))
    return out


def leopard_reconstruct(shards: np.ndarray, present) -> np.ndarray:
    """Codec.Decode: shards (2k, L) uint8 (missing rows ignored) -> all 2k."""
    shards = np.asarray(shards, dtype=np.uint8)
    present = np.asarray(present, dtype=bool)
    n, L = shards.shape
    k = n // 2
    if present.sum() < k:
        raise ErrUnrepairableDataSquare()
    if present.all():
        return shards.copy()
    F = pyref.field_for(k)
    if F.bits == 8:
        return _decode_symbols(F, shards.astype(np.int64), present).astype(np.uint8)
    blk = shards.reshape(n, L // 64, 2, 32).astype(np.int64)
    sym = (blk[:, :, 0, :] | (blk[:, :, 1, :] << 8)).reshape(n, -1)
    out = _decode_symbols(F, sym, present).reshape(n, L // 64, 32)
    res = np.empty((n, L // 64, 2, 32), dtype=np.uint8)
    res[:, :, 0, :] = out & 0xFF
    res[:, :, 1, :] = out >> 8
    return res.reshape(n, L)


def repair(eds: np.ndarray, present: np.ndarray, row_roots, col_roots) -> np.ndarray:
    """rsmt2d ExtendedDataSquare.Repair in the reference's visiting order."""
    eds = np.array(eds, dtype=np.uint8, copy=True)
    present = np.array(present, dtype=bool, copy=True)
    W = eds.shape[0]
    k = W // 2

    def vec(axis, i):
        return eds[i] if axis == ROW else eds[:, i]

    def pres(axis, i):
        return present[i] if axis == ROW else present[:, i]

    def root(axis, i):
        return pyref.axis_root(vec(axis, i), k, i)

    def want(axis, i):
        return bytes(row_roots[i] if axis == ROW else col_roots[i])

    def encoding_ok(axis, i):
        v = vec(axis, i)
        return np.array_equal(pyref.leopard_encode(v[:k]), v[k:])

    # preRepairSanityCheck
    for i in range(W):
        for axis in (ROW, COL):
            if pres(axis, i).all():
                got = root(axis, i)
                if got != want(axis, i):
                    raise ErrBadRoot(f"bad root input: {'row' if axis == ROW else 'col'} {i} expected "
                                     f"{want(axis, i).hex()} got {got.hex()}")
                if not encoding_ok(axis, i):
                    raise ErrByzantineData(axis, i)

    def solve(axis, i):
        p = pres(axis, i)
        if p.all():
            return True, False
        if p.sum() < k:
            return False, False
        rebuilt = leopard_reconstruct(vec(axis, i), p)
        try:
            got = pyref.axis_root(rebuilt, k, i)
        except pyref.PushOrderError:
            raise ErrByzantineData(axis, i)
        if got != want(axis, i):
            raise ErrByzantineData(axis, i)
        ox = COL if axis == ROW else ROW
        newly = np.nonzero(~p)[0]
        # orthogonal vectors this rebuild completes
        for o in newly:
            op = pres(ox, o).copy()
            op[i] = True
            if op.all():
                ov = vec(ox, o).copy()
                ov[i] = rebuilt[o]
                try:
                    ogot = pyref.axis_root(ov, k, o)
                except pyref.PushOrderError:
                    raise ErrByzantineData(ox, o)
                if ogot != want(ox, o) or not np.array_equal(pyref.leopard_encode(ov[:k]), ov[k:]):
                    raise ErrByzantineData(ox, o)
        if axis == ROW:
            eds[i] = rebuilt
            present[i] = True
        else:
            eds[:, i] = rebuilt
            present[:, i] = True
        return True, True

    while True:
        solved, progress = True, False
        for i in range(W):
            for axis in (ROW, COL):
                s, p = solve(axis, i)
                solved &= s
                progress |= p
        if solved:
            return eds
        if not progress:
            raise ErrUnrepairableDataSquare()
