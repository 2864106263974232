"""Can RS's memory traffic hide under the VALU-bound hash stages?

Runs, on one GPU, (A) the hash stages alone (libcda variant whose RS kernel is
a no-op: CDA_LIB=tools/var/probe4/libcda.so), (B) a plain device-to-device copy
moving the RS stage's bytes per step (48 MiB per k=128 square read+written),
and (C) both at once on two streams.  C close to max(A, B) means a
small-footprint RS kernel co-running with hashing would hide its traffic;
C close to A + B means it would not.  Timing diagnostic only (wrong roots).
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "celestia-app_amd"))
from celestia_da import Context  # noqa: E402

k, B, W, SH = 128, 128, 256, 512
steps = int(os.environ.get("STEPS", "10"))
dev = torch.device("cuda", 0)
ctx = Context(0)
eds = torch.randint(0, 255, (B * W * W * SH,), dtype=torch.uint8, device=dev)
rows = torch.empty(B * W * 90, dtype=torch.uint8, device=dev)
cols = torch.empty_like(rows)
roots = torch.empty(B * 32, dtype=torch.uint8, device=dev)
status = torch.empty(B, dtype=torch.int32, device=dev)
copy_bytes = int(os.environ.get("COPY_MIB_PER_SQUARE", "24")) * B * (1 << 20)   # read + write = 2x
src = torch.empty(copy_bytes // 4, dtype=torch.int32, device=dev)
dst = torch.empty_like(src)
s_hash = torch.cuda.Stream(dev)
s_copy = torch.cuda.Stream(dev)


def hash_step():
    ctx.extend_dah_inplace_device(k, B, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), s_hash.cuda_stream)


def copy_step():
    with torch.cuda.stream(s_copy):
        dst.copy_(src)


def timed(fns):
    for f in fns:
        f()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(steps):
        for f in fns:
            f()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) / steps * 1e3


a = timed([hash_step])
b = timed([copy_step])
c = timed([hash_step, copy_step])
print(f"hash alone {a:.3f} ms/step, copy alone {b:.3f} ms/step ({2 * copy_bytes / b / 1e9:.2f} TB/s), "
      f"both {c:.3f} ms/step; sum {a + b:.3f}, max {max(a, b):.3f}; hidden fraction of copy "
      f"{(a + b - c) / b:.2f}")
