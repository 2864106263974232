"""CPU checks of the C ABI: libcda.so loads and exports every symbol that
include/cda.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cda.h")
LIB = os.path.join(ROOT, "celestia-app_amd", "libcda.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(cda_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "celestia-app_amd"), "-j8"])
    return ctypes.CDLL(LIB)


def test_header_declares_api():
    names = declared()
    assert "cda_extend_shares" in names and "cda_extend_dah_device" in names
    assert len(names) >= 14


def test_every_declared_symbol_exported(lib):
    for name in declared():
        assert hasattr(lib, name), name


def test_python_binding_covers_header():
    import celestia_da._lib as L
    assert sorted(L.EXPORTED) == declared()


def test_version_and_no_device_error(lib):
    lib.cda_version.restype = ctypes.c_char_p
    assert lib.cda_version().startswith(b"cda ")
    import celestia_da
    if os.environ.get("HIP_VISIBLE_DEVICES") == "" or not os.path.exists("/dev/kfd"):
        with pytest.raises(celestia_da.CdaError):
            celestia_da.Context()


def test_no_oracle_in_product():
    """The product package never imports the oracle (checker only)."""
    pkg = os.path.join(ROOT, "celestia-app_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "coracle" not in txt and "pyref" not in txt and "liboracle" not in txt, f
