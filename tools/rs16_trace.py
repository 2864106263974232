"""Per-workgroup timeline of rs16_cw_kernel<512> from a CDA_RS16_TRACE build
(tools/rs16_trace.sh): n k=512 squares in place, one traced step; prints the
phase durations (median / p10 / p90, us) of both RS launches and, per CU, the
gap between one workgroup's end and the next one's start.

usage: python tools/rs16_trace.py LIB [n_squares]"""
import ctypes as C
import os
import sys

import numpy as np

LIB = os.path.abspath(sys.argv[1])
os.environ["CDA_LIB"] = LIB
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "celestia-app_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from celestia_da import testfactory  # noqa: E402
from celestia_da._lib import Context  # noqa: E402

SLOTS, WGS, Q2 = 12, 16384, 8192
k, W, SH = 512, 1024, 512
dev = torch.device("cuda:0")
ctx = Context(0)
ods = np.stack([testfactory.random_square(k, i) for i in range(N)])
d_eds = torch.zeros(N * W * W * SH, dtype=torch.uint8, device=dev)
d_eds.view(N, W, W, SH)[:, :k, :k] = torch.from_numpy(ods).to(dev).view(N, k, k, SH)
d_rows = torch.empty(N * W * 90, dtype=torch.uint8, device=dev)
d_cols = torch.empty_like(d_rows)
d_roots = torch.empty(N * 32, dtype=torch.uint8, device=dev)
d_status = torch.empty(N, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
for _ in range(3):
    ctx.extend_dah_inplace_device(k, N, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(), d_roots.data_ptr(),
                                  d_status.data_ptr(), stream)
torch.cuda.synchronize()
# clock calibration: the same device clock around a timed step
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
ctx.extend_dah_inplace_device(k, N, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(), d_roots.data_ptr(),
                              d_status.data_ptr(), stream)
ev1.record()
torch.cuda.synchronize()
step_ms = ev0.elapsed_time(ev1)
assert N <= 8, "trace buffer holds 8 squares"
buf = np.zeros((WGS, SLOTS, 16), dtype=np.uint64)
lib = C.CDLL(LIB)
assert lib.cda_debug_rs16_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
raw = os.environ.get("TRACE_SAVE")
if raw:
    np.save(raw, np.concatenate([buf[:1024 * N], buf[Q2:Q2 + 512 * N]]))
us = 0.01   # s_memrealtime: 100 MHz (tools/var/clk calibration: 99.9-100.0 MHz)
names = ["tables", "passA(+loads)", "xchg1", "passB", "xchg2", "passA'", "stores"]
q = lambda d: f"med {np.median(d):7.2f}  p10 {np.percentile(d, 10):7.2f}  p90 {np.percentile(d, 90):7.2f}"
for label, lo, n in (("Q0 launch", 0, 1024 * N), ("Q2 launch", Q2, 512 * N)):
    t = buf[lo:lo + n].astype(np.int64)           # [wg][slot][wave]
    start, end = t[:, 0, :].min(1), t[:, 7, :].max(1)
    t0 = start.min()
    print(f"== {label}: {n} workgroups, span {(end.max() - t0) * us:.1f} us")
    for nm, a_ in zip(names, range(7)):
        d = (t[:, a_ + 1, :] - t[:, a_, :]) * us
        print(f"  {nm:14s} per wave {q(d)}")
    if t[:, 10, :].any():
        print(f"  {'loads landed':14s} per wave {q((t[:, 10, :] - t[:, 1, :]) * us)}  (after tables)")
    print(f"  wave spread at each mark (max-min over the 16 waves), med: " +
          " ".join(f"{np.median((t[:, s_, :].max(1) - t[:, s_, :].min(1)) * us):.2f}" for s_ in range(8)))
    print(f"  workgroup total {q((end - start) * us)}")
    hw = t[:, 9, 0]
    xcc = (hw >> 32) & 0xF
    hid = hw & 0xFFFFFFFF
    cu = (xcc << 16) | (((hid >> 13) & 0x7) << 8) | (((hid >> 12) & 1) << 4) | ((hid >> 8) & 0xF)
    gaps, per = [], []
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        o = idx[np.argsort(start[idx])]
        per.append(len(o))
        gaps += list((start[o[1:]] - end[o[:-1]]) * us)
    gaps = np.array(gaps) if gaps else np.zeros(1)
    print(f"  CUs {len(per)}, wg/CU {min(per)}-{max(per)}; gap end->next start {q(gaps)} us")
    busy = sum(((end - start) * us).tolist())
    print(f"  CU occupancy: sum of workgroup times / (CUs x span) = {busy / (len(per) * (end.max() - t0) * us):.3f}")
