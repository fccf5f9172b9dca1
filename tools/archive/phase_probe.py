#!/usr/bin/env python3
"""Drive tools/libphase_probe.so (bench-only, see phase_probe.hip): fresh
8 x 1 GiB fp32 buckets under several allocation modes; per bucket the product
kernel (hiccl_reduce) and the input-phased / slab variants, median of 5 HIP-
event timings, plus a bit-compare of every variant's output with the
product's.  One JSON line per (alloc mode, bucket, kernel)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hiccl_amd  # noqa: E402
from hiccl_amd import _lib as L  # noqa: E402

P = ctypes.CDLL(os.path.join(ROOT, "tools", "libphase_probe.so"))
vp = ctypes.c_void_p
P.pp_run.restype = ctypes.c_int
P.pp_run.argtypes = [ctypes.c_int] * 6 + [vp, ctypes.c_int, vp, ctypes.c_uint64, vp]
P.pp_alloc.restype = ctypes.c_int
P.pp_alloc.argtypes = [ctypes.POINTER(vp), ctypes.c_uint64, ctypes.c_int]
P.pp_diff.restype = ctypes.c_longlong
P.pp_diff.argtypes = [vp, vp, ctypes.c_uint64]
P.pp_granularity.restype = ctypes.c_uint64

H = None
if os.path.exists(os.path.join(ROOT, "tools", "libhbm_probe.so")):
    H = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
    H.probe_run.restype = ctypes.c_int
    H.probe_run.argtypes = [ctypes.c_int] * 7 + [vp, ctypes.c_int, vp, ctypes.c_uint64, vp]

N, COUNT = 8, 1 << 28
NB = COUNT * 4


def timeit(fn, reps=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        ev.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def alloc(mode):
    p = vp()
    rc = P.pp_alloc(ctypes.byref(p), NB, mode)
    if rc != 0:
        raise RuntimeError(f"pp_alloc mode {mode}: rc={rc}")
    return p.value


def main():
    modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2").split(",")]
    buckets = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    # (kind, block, param, depth, nt, grid); kind 0 phase (runtime n), 1 slab, 2 phase_n (n = 8)
    # kind 12: (12, block, U, C, per_wave, grid)
    variants = [(11, 256, 4, 0, 1, 256), (12, 256, 4, 2, 0, 256), (12, 256, 4, 4, 0, 256),
                (12, 256, 4, 8, 0, 256), (12, 256, 2, 4, 0, 256), (12, 256, 2, 8, 0, 256),
                (12, 256, 4, 4, 1, 256), (12, 256, 4, 2, 1, 256), (11, 256, 4, 0, 1, 256)]
    g = P.pp_granularity()
    print(json.dumps({"vmm_granularity_min": g >> 32, "vmm_granularity_rec": g & 0xffffffff}), flush=True)
    stream = torch.cuda.current_stream()
    sh = vp(stream.cuda_stream)
    keep = []
    for mode in modes:
        for b in range(buckets):
            try:
                ins = [alloc(mode) for _ in range(N)]
                out, ref = alloc(mode), alloc(mode)
            except RuntimeError as e:
                print(json.dumps({"alloc": mode, "error": str(e)}), flush=True)
                break
            keep.append(ins + [out, ref])
            for k, p in enumerate(ins):
                L.check(L.lib().hiccl_fill_uniform(0, vp(p), COUNT, 1234, k, 0, sh), "fill")
            tab = (vp * N)(*ins)
            prod = lambda: L.check(L.lib().hiccl_reduce(0, vp(ref), tab, N, COUNT, sh), "reduce")
            ms = timeit(prod)
            row = {"alloc": mode, "bucket": b, "kernel": "product", "ms": round(ms, 4),
                   "GBps": round(9 * NB / ms / 1e6, 1), "base": hex(ins[0])}
            print(json.dumps(row), flush=True)
            for (kind, block, param, depth, nt, grid) in variants:
                fn = lambda: P.pp_run(kind, block, param, depth, nt, grid, tab, N, vp(out), NB, sh)
                rc = fn()
                if rc != 0:
                    print(json.dumps({"kind": kind, "block": block, "param": param, "rc": rc}), flush=True)
                    continue
                ms = timeit(fn)
                torch.cuda.synchronize()
                diff = P.pp_diff(vp(out), vp(ref), NB) if not (kind == 4 and depth < 16 and depth & 1) else None
                print(json.dumps({"alloc": mode, "bucket": b,
                                  "kernel": ["phase", "slab", "phase_n", "phase_lds", "phase_x", "phase_flat", "phase_pipe", "phase_sync", "phase_q", "phase_dyn", "wave_dyn", "wg_dyn", "multi_dyn"][kind], "block": block,
                                  "param": param, "depth": depth, "nt": nt, "grid": grid, "ms": round(ms, 4),
                                  "GBps": round(9 * NB / ms / 1e6, 1), "mismatch_words": diff}), flush=True)
            if H is not None:
                for g in (256, 1024):
                    fn = lambda: H.probe_run(2, 256, 4, 2, 2, 0, g, tab, N, vp(out), NB, sh)
                    ms = timeit(fn)
                    print(json.dumps({"alloc": mode, "bucket": b, "kernel": "write_only(hbm_probe)", "grid": g,
                                      "ms": round(ms, 4), "GBps": round(NB / ms / 1e6, 1)}), flush=True)
                fn = lambda: H.probe_run(1, 256, 4, 2, 2, 0, 256, tab, N, vp(out), NB, sh)
                ms = timeit(fn)
                print(json.dumps({"alloc": mode, "bucket": b, "kernel": "read_only_tile(hbm_probe)",
                                  "ms": round(ms, 4), "GBps": round(N * NB / ms / 1e6, 1)}), flush=True)
            ms = timeit(prod)
            print(json.dumps({"alloc": mode, "bucket": b, "kernel": "product(again)", "ms": round(ms, 4),
                              "GBps": round(9 * NB / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
