"""Shared fixtures.  `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X.

The oracle (oracle/liboracle.so) is test infrastructure only: it is loaded
here as the checker, never by the product package.
"""
import ctypes
import fcntl
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libhiccl_ref.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "runtime_probe: records the HIP runtime's behaviour; runs after every "
                                       "other test, so that under -x it never keeps the parity tests from running")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: it.get_closest_marker("runtime_probe") is not None)  # stable: order kept otherwise


def make(directory, *targets):
    """`make -C directory targets` under a lock file, so that test workers
    (pytest -n) never run make on the same targets at once (a header edited
    since the last build sends every worker into the same rebuild)."""
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", directory, *targets], check=True, stdout=subprocess.DEVNULL)


def _build_oracle():
    if not os.path.exists(ORACLE_SO):
        make(os.path.join(ROOT, "oracle"), "liboracle.so")


class Oracle:
    """ctypes view of oracle/reduce_oracle.c."""

    def __init__(self, path=ORACLE_SO):
        self.lib = ctypes.CDLL(path)
        for name in ("oracle_reduce_f32", "oracle_reduce_f64", "oracle_reduce_u64", "oracle_reduce_i32",
                     "oracle_reduce_bf16", "oracle_reduce_bf16_accf32"):
            f = getattr(self.lib, name)
            f.restype = None
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        for name in ("oracle_fill_uniform_f32", "oracle_fill_uniform_bf16", "oracle_fill_uniform_f64"):
            f = getattr(self.lib, name)
            f.restype = None
            f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t]
        for name in ("oracle_sample_sum_f32", "oracle_sample_sum_bf16"):
            f = getattr(self.lib, name)
            f.restype = None
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int]
        self.lib.oracle_num_threads.restype = ctypes.c_int

    _FN = {np.dtype(np.float32): "oracle_reduce_f32", np.dtype(np.float64): "oracle_reduce_f64",
           np.dtype(np.uint64): "oracle_reduce_u64", np.dtype(np.int64): "oracle_reduce_u64",
           np.dtype(np.int32): "oracle_reduce_i32", np.dtype(np.uint16): "oracle_reduce_bf16"}

    def reduce(self, inputs, count=None, dtype=None, wide=False):
        """inputs: (n, count) array or list of 1-D arrays.  Returns out."""
        rows = [np.ascontiguousarray(r) for r in inputs]
        if dtype is None:
            dtype = rows[0].dtype if rows else np.float32
        dtype = np.dtype(dtype)
        if count is None:
            count = len(rows[0]) if rows else 0
        out = np.empty(count, dtype)
        tab = (ctypes.c_void_p * max(1, len(rows)))(*[r.ctypes.data for r in rows])
        fn = "oracle_reduce_bf16_accf32" if wide else self._FN[dtype]
        getattr(self.lib, fn)(out.ctypes.data, tab, len(rows), count)
        return out

    def fill(self, n, count, seed, dtype=np.float32, first=0):
        x = np.empty((n, count), dtype)
        fn = {np.dtype(np.float32): "oracle_fill_uniform_f32", np.dtype(np.uint16): "oracle_fill_uniform_bf16",
              np.dtype(np.float64): "oracle_fill_uniform_f64"}[np.dtype(dtype)]
        for k in range(n):
            getattr(self.lib, fn)(x[k].ctypes.data, count, seed, k, first)
        return x

    def sample_sum(self, idx, seed, n, bf16=False):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.empty(len(idx), np.uint16 if bf16 else np.float32)
        fn = self.lib.oracle_sample_sum_bf16 if bf16 else self.lib.oracle_sample_sum_f32
        fn(out.ctypes.data, idx.ctypes.data, len(idx), seed, n)
        return out


@pytest.fixture(scope="session")
def oracle():
    _build_oracle()
    return Oracle()


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    cases = {}
    for key in z.files:
        case, part = key.rsplit("/", 1)
        cases.setdefault(case, {})[part] = z[key]
    return cases


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


def bits_equal(a, b, float_nan_any=True):
    """Bitwise equality; NaN outputs compare by NaN-ness only (payload and sign
    of a NaN differ between x86 and gfx950)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if not float_nan_any:  # exact bits, NaN payloads included
        return a.dtype == b.dtype and a.tobytes() == b.tobytes()
    if a.dtype.kind == "f":
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb):
            return False
        ua = a.view(np.uint32 if a.dtype == np.float32 else np.uint64)
        ub = b.view(np.uint32 if b.dtype == np.float32 else np.uint64)
        return bool(np.array_equal(ua[~na], ub[~nb]))
    if a.dtype == np.uint16:  # bf16 bits
        na = ((a & 0x7F80) == 0x7F80) & ((a & 0x7F) != 0)
        nb = ((b & 0x7F80) == 0x7F80) & ((b & 0x7F) != 0)
        if not np.array_equal(na, nb):
            return False
        return bool(np.array_equal(a[~na], b[~nb]))
    return bool(np.array_equal(a, b))


def first_mismatch(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype.kind == "f":
        ua = a.view(np.uint32 if a.dtype == np.float32 else np.uint64)
        ub = b.view(np.uint32 if b.dtype == np.float32 else np.uint64)
        bad = np.nonzero((ua != ub) & ~(np.isnan(a) & np.isnan(b)))[0]
    else:
        bad = np.nonzero(a != b)[0]
    if len(bad) == 0:
        return "no mismatch"
    i = bad[0]
    return f"{len(bad)} mismatches, first at {i}: got {a[i]!r} expected {b[i]!r}"
