#!/usr/bin/env python3
"""Phase timeline of rs16_half_kernel<512> from a timing-probe build
(PATCH=tools/probes/rs16_phases.patch tools/build_variant.sh rs16ph
-DCDA_RS16_PHASES; run with CDA_LIB=<that>):
thread 0 of the grid's workgroups 0, 1 and its last two stamps s_memtime
(shader cycles) at: start, tables staged + codeword loaded, pass A done,
A->B exchange done, pass B done, B->A exchange done, pass A' (and its
stores) issued.  One k = 512 square; the
sampled launch is the LAST RS launch of the call (Q2 -> Q3: 1024 workgroups,
so "last" = 1022/1023, a second-round start)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))


def main():
    import torch
    from celestia_da import Context, testfactory, _lib
    L = _lib.load()
    fn = L.cda_debug_rs16_phases
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 32)()
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    k, W = 512, 1024
    o = torch.from_numpy(testfactory.random_square(k, 0)).to(dev)
    e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
    r = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    c = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    g = torch.empty(32, dtype=torch.uint8, device=dev)
    names = ["staged+loaded", "pass A", "xchg A->B", "pass B", "xchg B->A", "pass A'+stores"]
    for rep in range(5):
        ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(), None, s)
        torch.cuda.synchronize()
        fn(buf)
        v = list(buf)
        rows = []
        for slot, wg in enumerate(("0", "1", "last-1", "last")):
            t = v[8 * slot: 8 * slot + 7]
            d = [t[i + 1] - t[i] for i in range(6)]
            rows.append(f"  wg {wg:>6}: " + "  ".join(f"{n} {x:6d}" for n, x in zip(names, d)) + f"  total {t[6] - t[0]}")
        print(f"rep {rep} (shader cycles)")
        print("\n".join(rows))


if __name__ == "__main__":
    main()
