"""Contexts of the test build (libcda_test.so) with test knobs set.

libcda.so reads only the deployer knobs of csrc/knobs.h; fault injection
(CDA_FAULT, CDA_COMM_FAULT) and the A/B schedule switches the parity tests use
to reach every alternative schedule are read only by the test build, which
__graft_entry__.build() makes beside the product library from the same
sources (-DCDA_TESTING)."""
import os

import pytest

from celestia_da import _lib

DEPLOY_KNOBS = ("CDA_SYNC_CHECK", "CDA_HOST_THREADS", "CDA_HOST_REGISTER", "CDA_HOST_PIPE_CHUNK",
                "CDA_PIPELINE_CHUNK")


def lib_path_for_tests() -> str:
    if not os.path.exists(_lib.TEST_LIB_PATH):
        pytest.fail(f"test build missing: {_lib.TEST_LIB_PATH} (make -C celestia-app_amd test-lib)")
    return _lib.TEST_LIB_PATH


def ctx_with(env: dict, test_build: bool = True):
    """A context created while `env` is set (knobs are read at creation);
    on the test build unless every knob is a deployer knob and test_build is
    False."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        path = lib_path_for_tests() if test_build else None
        return _lib.Context(int(os.environ.get("CDA_DEVICE", "-1")), lib_path=path)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
