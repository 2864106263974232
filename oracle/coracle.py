"""ctypes binding for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg.  Never imported by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
NODE = 90
SHARE = 512

_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u8p = C.POINTER(C.c_uint8)
        L.oracle_extend.argtypes = [u8p, C.c_uint32, u8p]
        L.oracle_roots.argtypes = [u8p, C.c_uint32, u8p, u8p, C.POINTER(C.c_int), C.POINTER(C.c_uint32)]
        L.oracle_data_root.argtypes = [u8p, u8p, C.c_uint32, u8p]
        L.oracle_extend_dah.argtypes = [u8p, C.c_uint32, u8p, u8p, u8p, u8p]
        L.oracle_cpu_baseline.argtypes = [u8p, C.c_uint32, u8p, u8p, u8p, u8p, C.c_int]
        L.oracle_random_square.argtypes = [C.c_uint32, C.c_uint64, u8p]
        L.oracle_leopard_encode.argtypes = [u8p, u8p, C.c_uint32, C.c_uint32]
        L.oracle_table.argtypes = [C.c_int, C.c_int]
        L.oracle_table.restype = C.POINTER(C.c_uint16)
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def random_square(k: int, square_index: int = 0) -> np.ndarray:
    ods = np.empty((k * k, SHARE), dtype=np.uint8)
    lib().oracle_random_square(k, square_index, _p(ods))
    return ods


def leopard_encode(data: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    k, L = data.shape
    par = np.empty_like(data)
    rc = lib().oracle_leopard_encode(_p(data), _p(par), k, L)
    if rc:
        raise ValueError(f"chunkSize {L} must be a multiple of 64 bytes")
    return par


def extend(ods: np.ndarray) -> np.ndarray:
    ods = np.ascontiguousarray(ods, dtype=np.uint8).reshape(-1, SHARE)
    k = int(round(ods.shape[0] ** 0.5))
    eds = np.empty((4 * k * k, SHARE), dtype=np.uint8)
    rc = lib().oracle_extend(_p(ods), k, _p(eds))
    if rc:
        raise ValueError(f"oracle_extend rc={rc}")
    return eds


class PushOrderError(ValueError):
    pass


def roots(eds: np.ndarray, k: int):
    eds = np.ascontiguousarray(eds, dtype=np.uint8)
    W = 2 * k
    rows = np.empty((W, NODE), dtype=np.uint8)
    cols = np.empty((W, NODE), dtype=np.uint8)
    ax = C.c_int(-1)
    idx = C.c_uint32(0)
    rc = lib().oracle_roots(_p(eds), k, _p(rows), _p(cols), C.byref(ax), C.byref(idx))
    if rc == -3:
        raise PushOrderError(f"push order violated on {'col' if ax.value else 'row'} {idx.value}")
    return rows, cols


def data_root(rows: np.ndarray, cols: np.ndarray) -> bytes:
    out = np.empty(32, dtype=np.uint8)
    lib().oracle_data_root(_p(np.ascontiguousarray(rows)), _p(np.ascontiguousarray(cols)), rows.shape[0], _p(out))
    return out.tobytes()


def extend_dah(ods: np.ndarray):
    ods = np.ascontiguousarray(ods, dtype=np.uint8).reshape(-1, SHARE)
    k = int(round(ods.shape[0] ** 0.5))
    W = 2 * k
    eds = np.empty((W * W, SHARE), dtype=np.uint8)
    rows = np.empty((W, NODE), dtype=np.uint8)
    cols = np.empty((W, NODE), dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    rc = lib().oracle_extend_dah(_p(ods), k, _p(eds), _p(rows), _p(cols), _p(root))
    if rc == -3:
        raise PushOrderError("push order violated")
    if rc:
        raise ValueError(f"oracle_extend_dah rc={rc}")
    return eds, rows, cols, root.tobytes()


def cpu_baseline(ods: np.ndarray, nthreads: int):
    ods = np.ascontiguousarray(ods, dtype=np.uint8).reshape(-1, SHARE)
    k = int(round(ods.shape[0] ** 0.5))
    W = 2 * k
    eds = np.empty((W * W, SHARE), dtype=np.uint8)
    rows = np.empty((W, NODE), dtype=np.uint8)
    cols = np.empty((W, NODE), dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    rc = lib().oracle_cpu_baseline(_p(ods), k, _p(eds), _p(rows), _p(cols), _p(root), nthreads)
    if rc:
        raise ValueError(f"oracle_cpu_baseline rc={rc}")
    return eds, rows, cols, root.tobytes()


def table(bits: int, which: str) -> np.ndarray:
    n = {("log", 8): 256, ("exp", 8): 256, ("skew", 8): 255,
         ("log", 16): 65536, ("exp", 16): 65536, ("skew", 16): 65535}[(which, bits)]
    ptr = lib().oracle_table(bits, {"log": 0, "exp": 1, "skew": 2}[which])
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy()
