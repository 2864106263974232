"""Mirror of the reference's fraud tooling for unordered squares
(test/util/malicious).

malicious.ExtendShares (tree.go:60-71) extends with the default codec and
builds every row / column tree as a BlindTree (tree.go:18-58: ForceAddLeaf,
no namespace-order check, and the malicious hasher, hasher.go:161-310, which
checks no sibling order either); OutOfOrderPrepareProposal
(out_of_order_prepare.go:18-83) then takes da.NewDataAvailabilityHeader of
that square.  libcda.so computes exactly those roots in its normal
submission -- the hashing never depends on the order check, which only sets
the push-order status -- so the blind DAH is the honest call's output with
CDA_ERR_PUSH_ORDER accepted instead of raised.  An honest caller uses
celestia_da.da, which raises PushOrderError for such a square.
"""
from __future__ import annotations

import numpy as np

from . import da
from ._lib import CDA_ERR_PUSH_ORDER, NMT_ROOT_SIZE, SHARE_SIZE, default_context, ptr


def extend_shares_dah(s, ctx=None):
    """malicious.ExtendShares + da.NewDataAvailabilityHeader over its trees:
    (EDS as a (2k, 2k, 512) array, DataAvailabilityHeader with the blind
    roots and their hash), in one GPU submission.  s: the k*k shares."""
    ctx = ctx or default_context()
    n = len(s)
    if not da.is_power_of_two(n):
        raise ValueError(f"number of shares is not a power of 2: got {n}")
    k = da.square_size(n)
    ods = np.frombuffer(b"".join(bytes(x) for x in s), dtype=np.uint8)
    if ods.size != n * SHARE_SIZE:
        raise ValueError(f"shares must be {SHARE_SIZE} bytes each")
    W = 2 * k
    eds = np.empty((W, W, SHARE_SIZE), dtype=np.uint8)
    rows = np.empty(W * NMT_ROOT_SIZE, dtype=np.uint8)
    cols = np.empty(W * NMT_ROOT_SIZE, dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    rc = ctx.lib.cda_extend_dah(ctx.h, ptr(ods), n, ptr(eds), ptr(rows), ptr(cols), ptr(root))
    if rc != CDA_ERR_PUSH_ORDER:   # the order status is the only error a blind tree ignores
        ctx.check(rc)

    def roots(a):
        return [a[i * NMT_ROOT_SIZE:(i + 1) * NMT_ROOT_SIZE].tobytes() for i in range(W)]
    dah = da.DataAvailabilityHeader(roots(rows), roots(cols))
    dah._hash = root.tobytes()
    return eds, dah
