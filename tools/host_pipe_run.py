"""Config-4 host pipeline leg on its own (bench.py host_pipeline_rates), for
timelines: n squares (default 256) from page-locked host buffers through one
cda_extend_dah_batch call, with and without the EDS returned.
Usage: python tools/host_pipe_run.py [n] [reps]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from celestia_da import Context, testfactory  # noqa: E402
from celestia_da._lib import ptr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
k, W, SH = 128, 256, 512
ctx = Context(0)
h_ods = torch.empty((n, k * k * SH), dtype=torch.uint8, pin_memory=True)
for j0, part in testfactory.random_squares(k, range(n)):
    h_ods[j0:j0 + part.shape[0]].copy_(torch.from_numpy(part.reshape(part.shape[0], -1)))
h_eds = torch.empty((n, W * W * SH), dtype=torch.uint8, pin_memory=True)
rows = np.empty((n, W * 90), dtype=np.uint8)
cols = np.empty((n, W * 90), dtype=np.uint8)
roots = np.empty((n, 32), dtype=np.uint8)
st = np.zeros(n, dtype=np.int32)


def tp(t):
    return C.cast(C.c_void_p(t.data_ptr()), C.POINTER(C.c_ubyte))


for with_eds in (False, True):
    for r in range(reps):
        a = time.perf_counter()
        ctx.check(ctx.lib.cda_extend_dah_batch(ctx.h, tp(h_ods), k, n, tp(h_eds) if with_eds else None, ptr(rows),
                                               ptr(cols), ptr(roots), st.ctypes.data_as(C.POINTER(C.c_int32))))
        t = time.perf_counter() - a
        gb = n * (3 if with_eds else 1) * k * k * SH / t / 1e9
        print(f"eds={with_eds} rep {r}: {t * 1e3:.1f} ms  {n / t:.0f} squares/s  {gb:.1f} GB/s", flush=True)

# check: every square's EDS and data root against the device path (HBM-resident
# extend_dah_device of the same ODS, one square at a time for a sample)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
bad = 0
for i in sorted({0, 1, n // 2, n - 1}):
    o = h_ods[i].to(dev)
    e = torch.empty(W * W * SH, dtype=torch.uint8, device=dev)
    rr = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    cc = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    g = torch.empty(32, dtype=torch.uint8, device=dev)
    ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), rr.data_ptr(), cc.data_ptr(), g.data_ptr(), None, s)
    torch.cuda.synchronize(dev)
    ok = torch.equal(e.cpu(), h_eds[i]) and bytes(g.cpu().numpy()) == bytes(roots[i])
    bad += not ok
print(f"check: {4 - bad if n > 3 else n} sampled squares match the device path (EDS bytes + data root)"
      + ("" if bad == 0 else f"; {bad} DIFFER"), flush=True)
sys.exit(1 if bad else 0)
