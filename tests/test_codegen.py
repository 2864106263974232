"""Codegen guard for the GF(2^16) encoder's inline-asm table prefetch
(rs_gf16.hip sload16): no instruction may touch the destination SGPRs of an
in-flight scalar load before its explicit wait (tools/check_sload_hazards.py).
CPU only: hipcc cross-compiles gfx950 assembly here."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_no_scalar_load_hazards():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_sload_hazards.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("rs16_cw_kernelILi512", "rs16_half_kernelILi512"):
        line = next(ln for ln in r.stdout.splitlines() if name in ln)
        assert line.endswith(" 0 hazards"), line
