#!/usr/bin/env python3
"""Check the GF(2^16) codeword kernels for reads of SGPRs whose inline-asm
scalar load is still in flight.

rs_gf16.hip issues the next butterfly group's table load (`sload16`) from
inline asm and waits for it explicitly one group later, so the compiler does
not know the destination SGPRs are written asynchronously.  Any instruction
that reads or writes those SGPRs (a spill, a copy) between the load and the
next `s_waitcnt lgkmcnt(0)` would see stale data.  This compiles the file to
gfx950 assembly and scans every rs16_cw_kernel / rs16_half_kernel
instantiation.

Usage: python tools/check_sload_hazards.py  (exit 1 on a hazard)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "celestia-app_amd", "csrc", "rs_gf16.hip")


def sregs(text: str) -> set:
    out = set()
    for a, b in re.findall(r"s\[(\d+):(\d+)\]", text):
        out |= set(range(int(a), int(b) + 1))
    out |= {int(a) for a in re.findall(r"\bs(\d+)\b", text)}
    return out


def scan(asm: str) -> dict:
    res = {}
    for m in re.finditer(r"^(_ZN3cda\w*rs16_(?:cw|half)_kernel\w*):(.*?)s_endpgm", asm, re.S | re.M):
        pending, loads, hazards = set(), 0, []
        for ln in m.group(2).splitlines():
            t = ln.split(";")[0].strip()
            if not t or t.startswith(".") or t.endswith(":"):
                continue
            if t.startswith("s_waitcnt") and "lgkmcnt(0)" in t:
                pending = set()
                continue
            op, _, args = t.partition(" ")
            parts = [p.strip() for p in args.split(",")] if args else []
            if op.startswith("s_load"):
                if sregs(",".join(parts[1:])) & pending:
                    hazards.append(t)
                pending |= sregs(parts[0])
                loads += 1
                continue
            touched = sregs(",".join(parts))
            if touched & pending:
                hazards.append(t)
        res[m.group(1)] = (loads, hazards)
    return res


def main() -> int:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "rs_gf16.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950",
                               "--cuda-device-only", "-S", SRC, "-o", out])
        asm = open(out).read()
    res = scan(asm)
    bad = 0
    for name, (loads, hz) in res.items():
        print(f"{name}: {loads} scalar loads, {len(hz)} hazards")
        for t in hz[:5]:
            print("   ", t)
        bad += len(hz)
    if not res:
        print("no rs16 codeword kernel found")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
