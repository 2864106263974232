"""Run cda_repair_device a few times on one k=128 square (for rocprofv3)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "celestia-app_amd"))
from celestia_da import Context, da, testfactory  # noqa: E402
from celestia_da._lib import ptr  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pattern = sys.argv[2] if len(sys.argv) > 2 else "q0"
W = 2 * k
ctx = Context(0)
ods = testfactory.random_square(k, 7)
sq = da.extend_shares(ods)
dah = da.new_data_availability_header(sq)
full = np.ascontiguousarray(sq.array())
rows = np.frombuffer(b"".join(dah.row_roots), dtype=np.uint8)
cols = np.frombuffer(b"".join(dah.column_roots), dtype=np.uint8)
p = np.ones((W, W), np.uint8)
if pattern == "q0":
    p[:k, :k] = 0
else:
    rng = np.random.default_rng(5)
    for r in range(W):
        p[r, rng.choice(W, k, replace=False)] = 0
er = torch.from_numpy(np.where(p[..., None].astype(bool), full, 0).astype(np.uint8).reshape(-1)).to("cuda")
d = torch.empty_like(er)
for _ in range(5):
    d.copy_(er)
    torch.cuda.synchronize()
    ax, ix = C.c_int32(-1), C.c_uint32(0)
    ctx.check(ctx.lib.cda_repair_device(ctx.h, d.data_ptr(), ptr(p), W, ptr(rows), ptr(cols), C.byref(ax),
                                        C.byref(ix)))
assert np.array_equal(d.cpu().numpy().reshape(W, W, 512), full)
print("ok")
