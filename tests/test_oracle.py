"""CPU tier: the oracle is pinned to the reference before anything trusts it.

* fixtures are intact (sha256 in manifest.json);
* oracle/liboracle.so (the C restatement of source/compute.h:14-23)
  reproduces every committed fixture bit for bit -- the f32 / f64 / size_t
  fixtures were produced by the REFERENCE's own reduce_kernel compiled from
  /root/reference (tests/golden/make_golden.py);
* where the compiled reference is present (build container), it is re-run
  (bf16: reduce_kernel<__hip_bfloat16>, on the fixtures and on inputs drawn
  from every bf16 bit pattern);
* an independent numpy restatement (sequential adds in list order) agrees;
* the synthetic-input generator matches a numpy restatement of the hash.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, REF_SO, bits_equal, first_mismatch, load_golden

DTYPES = {"reduce_f32": np.float32, "reduce_f64": np.float64, "reduce_u64": np.uint64,
          "reduce_bf16": np.uint16, "reduce_i32": np.int32}


def test_manifest_hashes(manifest):
    for fname, meta in manifest["files"].items():
        with open(os.path.join(GOLDEN, fname), "rb") as fh:
            assert hashlib.sha256(fh.read()).hexdigest() == meta["sha256"], fname
    assert manifest["files"]["reduce_f32.npz"]["pinned_by"] == "reference"
    assert manifest["files"]["reduce_u64.npz"]["pinned_by"] == "reference"
    assert manifest["files"]["reduce_bf16.npz"]["pinned_by"] == "reference"
    assert manifest["files"]["reduce_i32.npz"]["pinned_by"] == "reference"


@pytest.mark.parametrize("name", sorted(DTYPES))
def test_oracle_matches_golden(oracle, name):
    cases = load_golden(name)
    assert cases
    for case, d in cases.items():
        x, y = d["in"], d["out"]
        got = oracle.reduce(list(x), count=len(y), dtype=y.dtype)
        assert bits_equal(got, y, float_nan_any=False), f"{name}/{case}: {first_mismatch(got, y)}"


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="compiled reference only in the build container")
@pytest.mark.parametrize("name,fn", [("reduce_f32", "ref_reduce_f32"), ("reduce_f64", "ref_reduce_f64"),
                                     ("reduce_u64", "ref_reduce_u64"), ("reduce_i32", "ref_reduce_i32")])
def test_reference_rerun_matches_golden(name, fn):
    ref = ctypes.CDLL(REF_SO)
    f = getattr(ref, fn)
    f.restype = None
    for case, d in load_golden(name).items():
        x, y = d["in"], d["out"]
        out = np.empty_like(y)
        rows = [np.ascontiguousarray(r) for r in x]
        tab = (ctypes.c_void_p * max(1, len(rows)))(*[r.ctypes.data for r in rows])
        f(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(len(y)), tab, ctypes.c_int(len(rows)))
        assert out.tobytes() == y.tobytes(), case


REF16_SO = os.path.join(os.path.dirname(REF_SO), "libhiccl_ref_bf16.so")


STAMP = os.path.join(os.path.dirname(REF_SO), "BUILT_FROM_REFERENCE")


def _ref16():
    if not os.path.exists(REF16_SO):
        if os.path.exists(STAMP):
            pytest.fail("tree built from the reference but oracle/_ref/libhiccl_ref_bf16.so is missing")
        pytest.skip("compiled reference only in the build container")
    f = ctypes.CDLL(REF16_SO).ref_reduce_bf16
    f.restype = None

    def run(x, count):
        out = np.full(count, 0x7F7F, np.uint16)
        rows = [np.ascontiguousarray(r) for r in x]
        tab = (ctypes.c_void_p * max(1, len(rows)))(*[r.ctypes.data for r in rows])
        f(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(count), tab, ctypes.c_int(len(rows)))
        return out
    return run


def test_reference_bf16_rerun_matches_golden():
    """reduce_kernel<__hip_bfloat16> (compute.h:14-23 with ROCm's host bf16
    type, oracle/build_ref.sh) reproduces every bf16 fixture bit for bit."""
    run = _ref16()
    for case, d in load_golden("reduce_bf16").items():
        assert run(d["in"], len(d["out"])).tobytes() == d["out"].tobytes(), case


def test_oracle_bf16_vs_reference_every_bit_pattern(oracle):
    """Inputs drawn from all 65,536 bf16 bit patterns (NaN, Inf, denormals,
    signed zeros), 0-19 inputs: the restatement equals reduce_kernel<
    __hip_bfloat16> on every element (a NaN output's payload aside)."""
    run = _ref16()
    rng = np.random.default_rng(5)
    for _ in range(60):
        n, c = int(rng.integers(0, 20)), int(rng.integers(1, 3000))
        x = rng.integers(0, 1 << 16, size=(n, c), dtype=np.uint32).astype(np.uint16)
        want = run(list(x), c)
        got = oracle.reduce(list(x), count=c, dtype=np.uint16)
        assert bits_equal(got, want), (n, c, first_mismatch(got, want))


def _numpy_sequential(x, dtype):
    acc = np.zeros(x.shape[1], dtype)
    with np.errstate(all="ignore"):
        for k in range(x.shape[0]):
            acc = (acc + x[k]).astype(dtype)
    return acc


def test_numpy_restatement_f32(oracle):
    for case, d in load_golden("reduce_f32").items():
        got = _numpy_sequential(d["in"], np.float32) if d["in"].shape[0] else np.zeros(len(d["out"]), np.float32)
        assert bits_equal(got, d["out"]), case


def _bf16_to_f32(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def _f32_to_bf16(f):
    u = f.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(f)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def test_numpy_restatement_bf16(oracle):
    """bf16 semantics: f32 add, round to bf16 after every add."""
    for case, d in load_golden("reduce_bf16").items():
        x = d["in"]
        acc = np.zeros(x.shape[1], np.uint16)
        with np.errstate(all="ignore"):
            for k in range(x.shape[0]):
                acc = _f32_to_bf16(_bf16_to_f32(acc) + _bf16_to_f32(x[k]))
        assert bits_equal(acc, d["out"]), case


def test_summation_order_is_list_order(oracle):
    # 1e8 + 1 - 1e8 = 0 in f32, while 1e8 - 1e8 + 1 = 1: order is observable.
    x = np.array([[1e8], [1.0], [-1e8]], np.float32)
    assert oracle.reduce(list(x))[0] == 0.0
    assert oracle.reduce(list(x[[0, 2, 1]]))[0] == 1.0


def test_zero_sign_semantics(oracle):
    x = np.array([[-0.0, -0.0]], np.float32)
    out = oracle.reduce(list(x))
    assert out.view(np.uint32).tolist() == [0, 0]  # +0: acc starts at +0 (compute.h:17)
    assert oracle.reduce([], count=3, dtype=np.float32).tolist() == [0.0, 0.0, 0.0]


M64 = (1 << 64) - 1


def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def test_generator_matches_python_restatement(oracle):
    seed, n, count = 1234, 3, 97
    x = oracle.fill(n, count, seed, first=5)
    for k in range(n):
        key = _splitmix64(seed ^ (k << 48))
        for i in range(count):
            h = _splitmix64((key + 5 + i) & M64)
            v = np.float32(h >> 40) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
            assert x[k, i] == v


def test_sample_sum_consistent(oracle):
    seed, n, count = 77, 8, 5000
    x = oracle.fill(n, count, seed)
    full = oracle.reduce(list(x))
    idx = np.array([0, 1, 2, 999, 4097, 4999], np.uint64)
    assert bits_equal(oracle.sample_sum(idx, seed, n), full[idx.astype(np.int64)])
    xb = oracle.fill(n, count, seed, dtype=np.uint16)
    fullb = oracle.reduce(list(xb), dtype=np.uint16)
    assert bits_equal(oracle.sample_sum(idx, seed, n, bf16=True), fullb[idx.astype(np.int64)])
