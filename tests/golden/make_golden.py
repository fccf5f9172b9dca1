#!/usr/bin/env python3
"""Generate the committed golden fixtures for the bucket-reduction stage.

TEST INFRASTRUCTURE.  Run in the build container (where /root/reference
exists):

    make -C oracle            # liboracle.so + _ref/libhiccl_ref.so
    python tests/golden/make_golden.py

Expected outputs come from the REFERENCE ITSELF: HiCCL's CPU
``reduce_kernel<T>`` (source/compute.h:14-23), compiled unmodified from the
reference tree by oracle/build_ref.sh into oracle/_ref/libhiccl_ref.so.  The
CPU restatement (oracle/liboracle.so) is run on every case too and must agree
bit for bit -- this is what pins the oracle.  The reference's drivers use
size_t / float; for bf16 the same reduce_kernel<T> is instantiated with ROCm's
own host bf16 type, __hip_bfloat16 (oracle/_ref/libhiccl_ref_bf16.so, see
oracle/build_ref.sh), and must agree with the restatement bit for bit (NaN
outputs: NaN-ness only -- the payload of a NaN is not part of the contract).

Each fixture file is an .npz of plain numeric arrays (no pickles):
  <case>/in   (n, count) inputs in summation order
  <case>/out  (count,)   expected output
plus manifest.json with per-file sha256, the generator parameters and which
library produced the expected outputs.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SEED = 1234

COUNTS = [0, 1, 63, 64, 65, 255, 256, 257, 4099]
NS = [1, 2, 3, 4, 7, 8, 64]


def load_libs():
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libhiccl_ref.so"))
    ref16 = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libhiccl_ref_bf16.so"))
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    return ref, ref16, ora


def bf16_nan(a):
    return ((a & 0x7F80) == 0x7F80) & ((a & 0x7F) != 0)


def ptr_table(arrs):
    t = (ctypes.c_void_p * max(1, len(arrs)))()
    for k, a in enumerate(arrs):
        t[k] = a.ctypes.data
    return t


def run(lib, fn, dtype, inputs, count):
    out = np.full(count, 0x7F, dtype=dtype) if dtype != np.float32 else np.full(count, np.nan, np.float32)
    rows = [np.ascontiguousarray(r) for r in inputs]
    tab = ptr_table(rows)
    f = getattr(lib, fn)
    f.restype = None
    if fn.startswith("ref_"):  # (out, count, in, n) -- compute.h:14-15 signature
        f(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(count), tab, ctypes.c_int(len(rows)))
    else:  # oracle (out, in, n, count)
        f(ctypes.c_void_p(out.ctypes.data), tab, ctypes.c_int(len(rows)), ctypes.c_size_t(count))
    return out


def fill_uniform(ora, n, count, seed=SEED):
    x = np.empty((n, count), np.float32)
    f = ora.oracle_fill_uniform_f32
    f.restype = None
    for k in range(n):
        f(ctypes.c_void_p(x[k].ctypes.data), ctypes.c_size_t(count), ctypes.c_uint64(seed),
          ctypes.c_uint32(k), ctypes.c_size_t(0))
    return x


def special_f32():
    """Columns that pin zero signs, NaN/Inf, denormals, overflow and order."""
    inf, nan = np.float32(np.inf), np.float32(np.nan)
    big = np.float32(np.finfo(np.float32).max)
    den = np.float32(1e-45)  # smallest denormal
    cols = [
        (-0.0, -0.0, -0.0),          # -> +0 (acc starts at +0)
        (0.0, -0.0, -0.0),
        (inf, -inf, 1.0),            # NaN
        (nan, 1.0, 1.0),
        (1.0, nan, inf),
        (inf, 1.0, 1.0),
        (-inf, -1.0, 0.0),
        (den, den, -den),            # denormal arithmetic, no flush
        (den * 3, -den, den * 7),
        (1.1754942e-38, 1.1754942e-38, 0.0),
        (big, big, -big),            # overflow to inf before the cancel
        (-big, -big, big),
        (1e30, -1e30, 1.0),
        (1e8, 1.0, -1e8),            # order-sensitive: 0, not 1
        (16777216.0, 1.0, 1.0),      # 2^24 + 1 + 1 rounds twice
        (1.0, 16777216.0, 1.0),
        (0.1, 0.2, 0.3),
        (-0.1, 0.1, -0.0),
        (3.4e38, 3.4e38, 3.4e38),
        (1.0, -1.0, -0.0),
    ]
    x = np.array(cols, dtype=np.float32).T.copy()  # (3, ncols)
    return x


def wide_range(rng, n, count):
    mant = rng.uniform(1.0, 2.0, size=(n, count))
    expo = rng.integers(-40, 40, size=(n, count))
    sign = rng.choice([-1.0, 1.0], size=(n, count))
    return (sign * mant * np.exp2(expo)).astype(np.float32)


def f32_to_bf16_bits(x):
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    nan = np.isnan(x)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


def main():
    ref, ref16, ora = load_libs()
    rng = np.random.default_rng(SEED)
    manifest = {"seed": SEED, "generator": "tests/golden/make_golden.py",
                "reference": "source/compute.h:14-23 reduce_kernel<T> (oracle/_ref/libhiccl_ref.so; bf16: "
                             "reduce_kernel<__hip_bfloat16>, oracle/_ref/libhiccl_ref_bf16.so)",
                "files": {}}

    def check(name, dtype, ref_fn, ora_fn, inputs, count):
        exp = run(ref16 if ref_fn == "ref_reduce_bf16" else ref, ref_fn, dtype, inputs, count)
        got = run(ora, ora_fn, dtype, inputs, count)
        if ref_fn == "ref_reduce_bf16":
            na, ng = bf16_nan(exp), bf16_nan(got)
            if not (np.array_equal(na, ng) and np.array_equal(exp[~na], got[~ng])):
                raise SystemExit(f"oracle disagrees with the reference on {name}")
        elif exp.tobytes() != got.tobytes():
            raise SystemExit(f"oracle disagrees with the reference on {name}")
        return exp

    # ---- f32
    cases = {}
    for n in NS:
        for c in COUNTS:
            if n == 64 and c > 257:
                continue
            x = fill_uniform(ora, n, c)
            cases[f"rand_n{n}_c{c}"] = (x, check(f"rand_n{n}_c{c}", np.float32, "ref_reduce_f32",
                                                  "oracle_reduce_f32", list(x), c))
    for n in (2, 3, 8, 16):
        x = wide_range(rng, n, 4099)
        cases[f"wide_n{n}"] = (x, check(f"wide_n{n}", np.float32, "ref_reduce_f32", "oracle_reduce_f32",
                                        list(x), 4099))
    x = special_f32()
    cases["special_n3"] = (x, check("special", np.float32, "ref_reduce_f32", "oracle_reduce_f32", list(x),
                                    x.shape[1]))
    x1 = x[:1].copy()
    cases["special_n1"] = (x1, check("special_n1", np.float32, "ref_reduce_f32", "oracle_reduce_f32",
                                     list(x1), x.shape[1]))
    x0 = np.zeros((0, 5), np.float32)
    cases["empty_n0_c5"] = (x0, check("n0", np.float32, "ref_reduce_f32", "oracle_reduce_f32", [], 5))
    save("reduce_f32", cases, manifest, "reference")

    # ---- f64
    cases = {}
    for n in (1, 2, 3, 8):
        for c in (1, 65, 257, 4099):
            x = rng.uniform(-1, 1, size=(n, c)).astype(np.float64) * np.exp2(rng.integers(-60, 60, size=(n, c)))
            cases[f"rand_n{n}_c{c}"] = (x, check("f64", np.float64, "ref_reduce_f64", "oracle_reduce_f64",
                                                  list(x), c))
    save("reduce_f64", cases, manifest, "reference")

    # ---- size_t: the reference's own known-answer pattern (bench.h:80-82:
    # sendbuf[i] = i; rank p contributes element p*count + i), and wrap-around.
    cases = {}
    for n in (2, 3, 8):
        c = 4099
        x = np.stack([np.arange(c, dtype=np.uint64) + np.uint64(k * c) for k in range(n)])
        cases[f"kat_n{n}"] = (x, check("u64", np.uint64, "ref_reduce_u64", "oracle_reduce_u64", list(x), c))
    x = rng.integers(0, 2**64 - 1, size=(4, 1031), dtype=np.uint64)
    cases["wrap_n4"] = (x, check("u64wrap", np.uint64, "ref_reduce_u64", "oracle_reduce_u64", list(x), 1031))
    save("reduce_u64", cases, manifest, "reference")

    # ---- int32: small values, and full-range values whose sums wrap
    cases = {}
    for n in (1, 2, 3, 8):
        x = rng.integers(-1000, 1000, size=(n, 4099), dtype=np.int64).astype(np.int32)
        cases[f"small_n{n}"] = (x, check("i32", np.int32, "ref_reduce_i32", "oracle_reduce_i32", list(x), 4099))
    x = rng.integers(-2**31, 2**31, size=(5, 1031), dtype=np.int64).astype(np.int32)
    cases["wrap_n5"] = (x, check("i32wrap", np.int32, "ref_reduce_i32", "oracle_reduce_i32", list(x), 1031))
    save("reduce_i32", cases, manifest, "reference")

    # ---- bf16: reduce_kernel<__hip_bfloat16>
    cases = {}
    for n in (1, 2, 3, 8, 16):
        for c in (1, 7, 8, 9, 257, 4099):
            xf = fill_uniform(ora, n, c)
            x = f32_to_bf16_bits(xf * np.float32(n))  # spread magnitudes a little
            cases[f"rand_n{n}_c{c}"] = (x, check("bf16", np.uint16, "ref_reduce_bf16", "oracle_reduce_bf16",
                                                  list(x), c))
    sp = f32_to_bf16_bits(special_f32())
    cases["special_n3"] = (sp, check("bf16sp", np.uint16, "ref_reduce_bf16", "oracle_reduce_bf16", list(sp),
                                        sp.shape[1]))
    save("reduce_bf16", cases, manifest, "reference")

    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print("wrote", sorted(manifest["files"]))


def save(name, cases, manifest, pinned_by):
    arrs = {}
    for k, (x, y) in cases.items():
        arrs[f"{k}/in"] = x
        arrs[f"{k}/out"] = y
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrs)
    manifest["files"][f"{name}.npz"] = {"sha256": sha(path), "cases": len(cases), "pinned_by": pinned_by}


if __name__ == "__main__":
    sys.exit(main())
