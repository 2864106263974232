#!/usr/bin/env python3
"""Phase timeline of the latency chain's tree top and data root (configs 2
and 3) from a timing-probe build (PATCH=tools/probes/top_trace.patch
tools/build_variant.sh toptrace -DCDA_TOP_TRACE; run with CDA_LIB=<that>/libcda.so): workgroup (0, 0)'s thread 0
stamps s_memtime / s_memrealtime (100 MHz) at every level boundary of
tree_top_kernel and data_root_digest_kernel.  Prints per-phase deltas."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))


def main():
    import torch
    from celestia_da import Context, testfactory, _lib
    L = _lib.load()
    fn = L.cda_debug_top_trace
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_uint]
    fn.restype = C.c_int
    buf = (C.c_ulonglong * 128)()
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    for k in (128, 512):
        W = 2 * k
        o = torch.from_numpy(testfactory.random_square(k, 0)).to(dev)
        e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
        r = torch.empty(W * 90, dtype=torch.uint8, device=dev)
        c = torch.empty(W * 90, dtype=torch.uint8, device=dev)
        g = torch.empty(32, dtype=torch.uint8, device=dev)
        for rep in range(6):
            fn(buf, 128)   # drain
            ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(), None, s)
            torch.cuda.synchronize()
            n = fn(buf, 128)
        v = list(buf[:n])
        ticks, real = v[0::2], v[1::2]
        print(f"k={k}: {n // 2} marks; tree top then data root (WG 0, thread 0)")
        mhz = (ticks[-1] - ticks[0]) / max(1, (real[-1] - real[0])) * 100.0
        print(f"  s_memtime rate {mhz:.0f} MHz (against the 100 MHz real-time clock)")
        for i in range(1, len(ticks)):
            print(f"  mark {i:2d}: +{(real[i] - real[i - 1]) / 100.0:7.2f} us  ({ticks[i] - ticks[i - 1]:7d} clk)")
        print(f"  total {(real[-1] - real[0]) / 100.0:.2f} us")
        del o, e


if __name__ == "__main__":
    main()
