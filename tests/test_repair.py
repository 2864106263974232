"""EDS repair and Leopard decode.

Reference: rsmt2d v0.14.0 ExtendedDataSquare.Repair / Codec.Decode ->
klauspost/reedsolomon v1.12.1 leopard reconstruct (EXT, go.mod:11,13), as
restated in oracle/repair.py.

Checks:
  * CPU: the restated decoder reconstructs every erasure pattern of k lost
    shards (GF(2^8) and GF(2^16)), and the restated Repair round-trips
    oracle-extended squares, including mainnet block 408's (k=32), and
    reports rsmt2d's error outcomes;
  * GPU: cda_rs_decode equals the oracle (and the original codeword) for
    every field size and erasure shape; cda_repair returns the oracle's
    square, and for byzantine / unrepairable / bad-root inputs the same
    outcome as the oracle's replay in the reference's visiting order
    (axis and index of the byzantine vector included).  k=512 is checked by
    the erase -> repair round trip (size-independent property).
"""
import gzip
import os

import numpy as np
import pytest

import coracle
import repair as orp

HERE = os.path.dirname(os.path.abspath(__file__))


def block408_eds():
    with gzip.open(os.path.join(HERE, "golden", "block408_ods.bin.gz")) as f:
        ods = np.frombuffer(f.read(), dtype=np.uint8).reshape(-1, 512).copy()
    eds, rows, cols, root = coracle.extend_dah(ods)
    k = int(round(ods.shape[0] ** 0.5))
    return eds.reshape(2 * k, 2 * k, 512), [bytes(r) for r in rows], [bytes(c) for c in cols], root


def small_eds(k, seed=3):
    ods = coracle.random_square(k, seed)
    eds, rows, cols, root = coracle.extend_dah(ods)
    return eds.reshape(2 * k, 2 * k, 512), [bytes(r) for r in rows], [bytes(c) for c in cols]


def erasure_patterns(k, rng):
    n = 2 * k
    pats = [np.r_[np.zeros(k, bool), np.ones(k, bool)],      # all data lost
            np.r_[np.ones(k, bool), np.zeros(k, bool)],      # all parity lost
            np.ones(n, bool)]
    pats[2][0] = False                                        # one shard lost
    for _ in range(2):
        p = np.ones(n, bool)
        p[rng.choice(n, k, replace=False)] = False           # exactly k left
        pats.append(p)
    return pats


def run_oracle(eds, present, rows, cols):
    try:
        return "ok", orp.repair(np.where(present[..., None], eds, 0), present, rows, cols)
    except orp.ErrByzantineData as e:
        return ("byz", e.axis, e.index), None
    except orp.ErrUnrepairableDataSquare:
        return "unrep", None
    except orp.ErrBadRoot:
        return "badroot", None


# ------------------------------------------------------------------ CPU tests
@pytest.mark.parametrize("k,L", [(1, 64), (2, 64), (4, 128), (16, 512), (128, 64), (256, 64), (512, 64)])
def test_oracle_decode_round_trip(k, L):
    rng = np.random.default_rng(k)
    data = rng.integers(0, 256, (k, L), dtype=np.uint8)
    cw = np.concatenate([data, coracle.leopard_encode(data)])
    for p in erasure_patterns(k, rng):
        out = orp.leopard_reconstruct(np.where(p[:, None], cw, 0), p)
        assert np.array_equal(out, cw)


def test_oracle_decode_too_few():
    cw = np.zeros((8, 64), np.uint8)
    p = np.zeros(8, bool)
    p[:3] = True
    with pytest.raises(orp.ErrUnrepairableDataSquare):
        orp.leopard_reconstruct(cw, p)


def test_oracle_repair_block408():
    """Real data (k=32): Q0 lost, or a random half of the cells lost."""
    eds, rows, cols, root = block408_eds()
    W = eds.shape[0]
    k = W // 2
    p = np.ones((W, W), bool)
    p[:k, :k] = False
    assert np.array_equal(orp.repair(np.where(p[..., None], eds, 0), p, rows, cols), eds)


@pytest.mark.parametrize("k", [1, 2, 4])
def test_oracle_repair_outcomes(k):
    eds, rows, cols = small_eds(k)
    W = 2 * k
    rng = np.random.default_rng(10 + k)
    p = rng.random((W, W)) < 0.6
    out, rep = run_oracle(eds, p, rows, cols)
    assert out in ("ok", "unrep")
    if out == "ok":
        assert np.array_equal(rep, eds)
    p = np.zeros((W, W), bool)
    p[0, 0] = True    # one cell: enough only for k = 1
    assert run_oracle(eds, p, rows, cols)[0] == ("ok" if k == 1 else "unrep")
    bad = eds.copy()
    bad[0, 0, 100] ^= 1
    assert run_oracle(bad, np.ones((W, W), bool), rows, cols)[0] == "badroot"


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("k,L", [(1, 512), (2, 64), (4, 512), (16, 128), (32, 512), (64, 512), (128, 512),
                                 (256, 128), (512, 64)])
def test_rs_decode_matches_oracle(ctx, k, L):
    from celestia_da import rsmt2d
    rng = np.random.default_rng(100 + k)
    codec = rsmt2d.LeoRSCodec(ctx)
    pats = erasure_patterns(k, rng)
    n = len(pats)
    data = rng.integers(0, 256, (n, k, L), dtype=np.uint8)
    cws = np.stack([np.concatenate([d, coracle.leopard_encode(d)]) for d in data])
    pres = np.stack(pats)
    shards = np.where(pres[..., None], cws, 0).astype(np.uint8)
    codec.decode_batch(shards, pres)
    for i in range(n):
        assert np.array_equal(shards[i], cws[i]), i
        if k <= 128 or i < 2:
            assert np.array_equal(orp.leopard_reconstruct(np.where(pres[i][:, None], cws[i], 0), pres[i]), shards[i])


@pytest.mark.gpu
def test_codec_decode_api(ctx):
    from celestia_da import UnrepairableError, rsmt2d
    codec = rsmt2d.LeoRSCodec(ctx)
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, (8, 512), dtype=np.uint8)
    full = [r.tobytes() for r in np.concatenate([data, codec.encode(data)])]
    holes = [s if i % 2 else None for i, s in enumerate(full)]
    assert codec.decode(holes) == full
    with pytest.raises(UnrepairableError):
        codec.decode([full[0]] + [None] * 15)


def gpu_repair(ctx, eds, present, rows, cols):
    from celestia_da import ByzantineDataError, CdaError, UnrepairableError, rsmt2d, wrapper
    W = eds.shape[0]
    sq = rsmt2d.new_extended_data_square_with_missing(eds, present, rsmt2d.LeoRSCodec(ctx),
                                                     wrapper.new_constructor(W // 2))
    try:
        sq.repair(rows, cols, present)
        return "ok", sq.array()
    except ByzantineDataError as e:
        return ("byz", e.axis, e.index), None
    except UnrepairableError:
        return "unrep", None
    except CdaError as e:
        assert "bad root input" in str(e)
        return "badroot", None


@pytest.mark.gpu
def test_repair_block408(ctx):
    eds, rows, cols, root = block408_eds()
    W = eds.shape[0]
    rng = np.random.default_rng(408)
    for p in (np.pad(np.zeros((W // 2, W // 2), bool), ((0, W // 2), (0, W // 2)), constant_values=True),
              rng.random((W, W)) < 0.55):
        out, rep = gpu_repair(ctx, eds, p, rows, cols)
        assert out == "ok"
        assert np.array_equal(rep, eds)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 4, 8])
def test_repair_random_patterns_match_oracle(ctx, k):
    eds, rows, cols = small_eds(k, 5)
    W = 2 * k
    rng = np.random.default_rng(1000 + k)
    for trial in range(6):
        p = rng.random((W, W)) < (0.35 + 0.1 * trial)
        want, rep_o = run_oracle(eds, p, rows, cols)
        got, rep_g = gpu_repair(ctx, eds, p, rows, cols)
        assert got == want, (trial, got, want)
        if want == "ok":
            assert np.array_equal(rep_g, eds) and np.array_equal(rep_o, eds)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 4, 8])
def test_repair_byzantine_matches_oracle(ctx, k):
    """Corrupted cells that only a decode can expose: the GPU names the same
    byzantine (axis, index) as the oracle's replay in rsmt2d's order."""
    eds, rows, cols = small_eds(k, 6)
    W = 2 * k
    rng = np.random.default_rng(2000 + k)
    seen = set()
    for trial in range(8):
        bad = eds.copy()
        r, c = rng.integers(0, W, 2)
        bad[r, c, rng.integers(0, 512)] ^= 1 + rng.integers(0, 255)
        p = rng.random((W, W)) < 0.7
        p[r, c] = True
        p[r, (c + 1 + rng.integers(0, W - 1)) % W] = False   # row r and column c incomplete
        p[(r + 1 + rng.integers(0, W - 1)) % W, c] = False
        want, _ = run_oracle(bad, p, rows, cols)
        got, _ = gpu_repair(ctx, bad, p, rows, cols)
        assert got == want, (trial, got, want)
        seen.add(want if isinstance(want, str) else want[0])
    assert "byz" in seen


@pytest.mark.gpu
def test_repair_bad_root_and_unrepairable(ctx):
    eds, rows, cols = small_eds(4, 7)
    W = 8
    bad = eds.copy()
    bad[1, 2, 77] ^= 0x40
    assert gpu_repair(ctx, bad, np.ones((W, W), bool), rows, cols)[0] == "badroot"
    p = np.zeros((W, W), bool)
    p[:3, :] = True    # three full rows: no column has k = 4 cells
    assert gpu_repair(ctx, eds, p, rows, cols)[0] == "unrep"


@pytest.mark.gpu
@pytest.mark.parametrize("k", [64, 128])
def test_repair_matches_oracle_eds(ctx, k):
    eds, rows, cols = small_eds(k, 9)
    W = 2 * k
    rng = np.random.default_rng(k)
    p = rng.random((W, W)) < 0.5
    out, rep = gpu_repair(ctx, eds, p, rows, cols)
    assert out == "ok" and np.array_equal(rep, eds)


@pytest.mark.gpu
def test_repair_k512_round_trip(ctx):
    """GF(2^16), 512 MiB EDS: Q0 erased -> repaired square equals the GPU
    extension it came from, and its roots equal the DAH."""
    from celestia_da import da, testfactory
    k, W = 512, 1024
    ods = testfactory.random_square(k, 0)
    sq = da.extend_shares(ods)
    dah = da.new_data_availability_header(sq)
    eds = sq.array().copy()
    p = np.ones((W, W), bool)
    p[:k, :k] = False
    out, rep = gpu_repair(ctx, eds, p, dah.row_roots, dah.column_roots)
    assert out == "ok"
    assert np.array_equal(rep[:k, :k].reshape(-1, 512), ods)
    assert np.array_equal(rep, sq.array())


def device_repair(ctx, eds, present, rows, cols):
    """cda_repair_device on an HBM-resident copy of the square."""
    import ctypes as C

    import torch

    from celestia_da._lib import ptr
    W = eds.shape[0]
    e = np.where(np.asarray(present, bool)[..., None], eds, 0).astype(np.uint8)
    d = torch.from_numpy(e.reshape(-1)).to("cuda")
    p = np.ascontiguousarray(present, dtype=np.uint8)
    rb = np.frombuffer(b"".join(bytes(r) for r in rows), dtype=np.uint8)
    cb = np.frombuffer(b"".join(bytes(c) for c in cols), dtype=np.uint8)
    ax, ix = C.c_int32(-1), C.c_uint32(0)
    rc = ctx.lib.cda_repair_device(ctx.h, d.data_ptr(), ptr(p), W, ptr(rb), ptr(cb), C.byref(ax), C.byref(ix))
    out = d.cpu().numpy().reshape(W, W, 512)
    if rc == 0:
        return "ok", out
    if rc == -9:
        return ("byz", ax.value, ix.value), None
    if rc == -10:
        return "unrep", None
    assert rc == -6 and "bad root input" in ctx.lib.cda_last_error(ctx.h).decode()
    return "badroot", None


@pytest.mark.gpu
@pytest.mark.parametrize("k", [4, 16, 128])
def test_repair_device_matches_host(ctx, k):
    """The HBM-resident entry point gives the host entry point's outcome and
    square for ordinary, byzantine, unrepairable and bad-root inputs."""
    eds, rows, cols = small_eds(k, 12)
    W = 2 * k
    rng = np.random.default_rng(3000 + k)
    cases = []
    for trial in range(3):
        cases.append((eds, rng.random((W, W)) < (0.4 + 0.15 * trial)))
    q0 = np.ones((W, W), bool)
    q0[:k, :k] = False
    cases.append((eds, q0))
    bad = eds.copy()
    bad[1, 2, 77] ^= 0x40
    cases.append((bad, np.ones((W, W), bool)))                # bad root input
    p = np.ones((W, W), bool)
    p[0, 1] = False
    cases.append((bad, p))                                    # decode exposes the corruption
    none = np.zeros((W, W), bool)
    none[: max(1, k - 1), :] = True
    cases.append((eds, none))                                 # unrepairable
    for i, (sq, p) in enumerate(cases):
        h = gpu_repair(ctx, sq, p, rows, cols)
        d = device_repair(ctx, sq, p, rows, cols)
        assert h[0] == d[0], (i, h[0], d[0])
        if h[0] == "ok":
            assert np.array_equal(h[1], d[1]) and np.array_equal(d[1], eds)
