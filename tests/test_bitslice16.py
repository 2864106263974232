"""CPU checks of the bitsliced GF(2^16) encoder (rs_gf16_bs.hip, bitslice16.h).

* test_host_schedule: tools/bs16_host_test.cpp compiled with g++ -- the
  constexpr field (Leopard's Cantor-basis representation without tables) equals
  leo_build<16>'s tables for 200 000 products, the whole skew vector (65 535
  entries), the networks and the linear split of the skew (skew_part /
  tbasis); then the kernel's whole schedule -- three layouts, the LDS
  exchanges, the masked lane terms and the uniform wave terms -- is emulated
  lane by lane for k = 256 and k = 512 and compared byte for byte with a scalar
  Leopard encoder (klauspost/reedsolomon v1.12.1 leopardFF16.encode, EXT,
  go.mod:152).  The GPU tests (test_gpu_parity k = 256 / 512, k512.json)
  check the kernel itself.
* test_kernel_is_full_rate: the gfx950 ISA of rs16_bs_kernel holds no
  half-rate VALU op beyond a few prologue address computations (v_perm, v_alignbit, 64-bit shifts, 3-operand adds/ors,
  bfi -- DESIGN.md 3.1: one in the stream makes every instruction issue at
  4 cycles), within 168 VGPRs (three waves per SIMD) and with at most a
  few dozen spilled values.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "celestia-app_amd", "csrc")
HALF_RATE = ("v_perm_b32", "v_alignbit_b32", "v_alignbyte_b32", "v_lshrrev_b64", "v_lshlrev_b64", "v_add3_u32",
             "v_or3_b32", "v_bfi_b32", "v_lshl_or_b32", "v_and_or_b32", "v_lshl_add_u32", "v_xad_u32")


@pytest.mark.skipif(not shutil.which("g++"), reason="g++ not available")
def test_host_schedule():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "bs16_host_test")
        subprocess.run(["g++", "-O2", "-std=c++20", "-I", CSRC, os.path.join(ROOT, "tools", "bs16_host_test.cpp"),
                        "-o", exe], check=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bitsliced schedule k=512: 0 differing" in r.stdout
    assert "bitsliced schedule k=256: 0 differing" in r.stdout


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_kernel_is_full_rate():
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
                        "--cuda-device-only", "-S", os.path.join(CSRC, "rs_gf16_bs.hip"), "-o", asm],
                       check=True, timeout=600)
        s = open(asm).read()
    kernels = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w*rs16_bs_kernel\w*):", s, re.M)]
    assert len(kernels) == 2, [k for _, k in kernels]
    for pos, name in kernels:
        body = s[pos:s.index(".Lfunc_end", pos)]
        ops = re.findall(r"^\s+(v_\w+)", body, re.M)
        # a handful of address ops (prologue, exchange slots) are harmless; the
        # networks must have none
        bad = [o for o in ops if o.startswith(HALF_RATE)]
        assert len(bad) <= 0.005 * len(ops), (name, sorted(set(bad)), len(bad), len(ops))
        assert len(ops) > 5000, (name, len(ops))   # the networks are really there
        meta = s[s.index(".Lfunc_end", pos):]
        vg = int(re.search(r"NumVgprs: (\d+)", meta).group(1))
        scratch = int(re.search(r"ScratchSize: (\d+)", meta).group(1))
        # three waves per SIMD (168 VGPRs); the few dozen long-lived values the
        # register cap spills (addresses, lane masks) are reloaded once per
        # phase, not inside the networks
        n_scratch = len(re.findall(r"^\s+scratch_(?:load|store)", body, re.M))
        assert vg <= 168 and scratch <= 256 and n_scratch <= 0.02 * len(ops), (name, vg, scratch, n_scratch)
