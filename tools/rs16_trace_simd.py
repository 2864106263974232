"""Offline analysis of a saved rs16 trace (TRACE_SAVE=... tools/rs16_trace.py):
per workgroup and SIMD, the VALU-idle time implied by the barriers -- at each
exchange the SIMD waits from its own last wave's arrival to the workgroup's
last arrival -- and the phase a SIMD spends with no wave computing.

usage: python tools/rs16_trace_simd.py trace.npy n_squares"""
import sys

import numpy as np

t = np.load(sys.argv[1]).astype(np.int64)      # [wg][slot][wave]
N = int(sys.argv[2])
us = 0.01
simd = (t[:, 9, :] >> 4) & 3                   # HW_ID SIMD_ID per wave
for label, sl in (("Q0", slice(0, 1024 * N)), ("Q2", slice(1024 * N, 1536 * N))):
    x, sm = t[sl], simd[sl]
    n = len(x)
    start = x[:, 0, :].min(1)
    end = x[:, 7, :].max(1)
    tot = (end - start) * us
    out = {}
    # the barrier before each exchange: arrival = slot 2 (xchg1) / slot 4 (xchg2);
    # the tables barrier: arrival = slot 1 is after it, so use slot 0 -> 1 whole
    for nm, arr in (("xchg1", 2), ("xchg2", 4), ("end", 7)):
        last = x[:, arr, :].max(1)
        idle = []
        for s_ in range(4):
            m = sm == s_
            a = np.where(m, x[:, arr, :], 0).max(1)
            idle.append((last - a) * us)
        out[nm] = np.mean(idle, axis=0)
    # exchange duration with every wave out of compute: last arrival -> first
    # wave's next mark
    x1 = (x[:, 3, :].min(1) - x[:, 2, :].max(1)) * us
    x2 = (x[:, 5, :].min(1) - x[:, 4, :].max(1)) * us
    tb = (x[:, 1, :].min(1) - x[:, 0, :].min(1)) * us
    print(f"{label}: {n} wg, total med {np.median(tot):.2f} us")
    print(f"  tables (no compute)                     med {np.median(tb):.2f}")
    print(f"  SIMD idle before xchg1 barrier (mean/SIMD) med {np.median(out['xchg1']):.2f}")
    print(f"  xchg1 all waves out of compute           med {np.median(x1):.2f}")
    print(f"  SIMD idle before xchg2 barrier            med {np.median(out['xchg2']):.2f}")
    print(f"  xchg2 all waves out of compute           med {np.median(x2):.2f}")
    print(f"  SIMD idle at the end (last wave of wg)    med {np.median(out['end']):.2f}")
    for s_ in range(8):
        pass
    pa = (x[:, 2, :] - x[:, 1, :]) * us
    print(f"  pass A per wave med {np.median(pa):.2f}; pass B {np.median((x[:, 4, :] - x[:, 3, :]) * us):.2f};"
          f" pass A' {np.median((x[:, 6, :] - x[:, 5, :]) * us):.2f}")
    # SIMD-level busy span in each compute pass: first wave start -> last wave end per SIMD
    for nm, a_, b_ in (("A", 1, 2), ("B", 3, 4), ("A'", 5, 6)):
        spans = []
        for s_ in range(4):
            m = sm == s_
            lo = np.where(m, x[:, a_, :], np.iinfo(np.int64).max).min(1)
            hi = np.where(m, x[:, b_, :], 0).max(1)
            spans.append((hi - lo) * us)
        print(f"  pass {nm:2s}: SIMD span (first start -> last end) med {np.median(np.mean(spans, axis=0)):.2f}")
