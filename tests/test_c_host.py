"""libcda.so from plain C (tests/c_host/cda_host_smoke.c): the header compiles
as C -- what cgo's C compiler sees -- and, on a GPU, a C program with no
Python or torch in its process reproduces the reference's golden data roots
and error texts through the C ABI alone."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "celestia-app_amd")
SRC = os.path.join(ROOT, "tests", "c_host", "cda_host_smoke.c")


def _build(out: str) -> str:
    exe = os.path.join(out, "cda_host_smoke")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
                           "-L", PKG, "-lcda", f"-Wl,-rpath,{PKG}", "-o", exe])
    return exe


def test_header_is_c_and_links(tmp_path):
    exe = _build(str(tmp_path))
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_c_host_golden_roots_and_errors(tmp_path):
    exe = _build(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("c host ok"), r.stdout
