#!/usr/bin/env python3
"""Drive tools/libhbm_probe.so: achievable HBM rates for the reduction's
access mix on this MI355X (bench-only; see hbm_probe.hip).  Prints one JSON
line per (mode, variant, grid), best first per mode."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
LIB.probe_run.restype = ctypes.c_int
LIB.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_void_p]


def timeit(fn, reps=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        ts.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ts])) * 1e-3


def stagger_main(n):
    """Same geometry, buffers whose bases are staggered by k*S bytes."""
    nbytes = 1 << 30
    pad = 64 << 20
    raw = [torch.empty((nbytes + pad) // 4, device="cuda").uniform_() for _ in range(n + 1)]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = []
    for S in (0, 256, 4096 + 256, 65536 + 4096 + 256, (1 << 20) + 65536 + 4096 + 256, 3 * (1 << 20) + 12288 + 768):
        ptrs = [raw[k].data_ptr() + (k * S) % pad for k in range(n)]
        outp = raw[n].data_ptr() + (n * S) % pad
        tab = (ctypes.c_void_p * n)(*ptrs)
        for (block, unroll, al, as_, order, grid) in ((256, 4, 2, 2, 0, 192), (256, 4, 2, 2, 0, 256),
                                                     (1024, 4, 2, 16, 0, 1024), (256, 2, 2, 0, 0, 1024),
                                                     (256, 4, 2, 2, 2, 256), (256, 8, 2, 2, 2, 256),
                                                     (512, 4, 2, 2, 2, 256)):
            for mode in (0, 1):
                def fn():
                    rc = LIB.probe_run(mode, block, unroll, al, as_, order, grid, tab, n, ctypes.c_void_p(outp),
                                       nbytes, stream)
                    assert rc == 0, rc
                t = min(timeit(fn) for _ in range(3))
                moved = (n + 1) * nbytes if mode == 0 else n * nbytes
                rows.append({"stagger": S, "mode": ["mix", "read"][mode], "block": block, "unroll": unroll,
                             "aux_load": al, "aux_store": as_, "order": order, "grid": grid,
                             "GBps": round(moved / t / 1e9, 1)})
    for r in rows:
        print(json.dumps(r))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nbytes = 1 << 30
    ins = [torch.empty(nbytes // 4, device="cuda").uniform_() for _ in range(n)]
    out = torch.empty(nbytes // 4, device="cuda")
    tab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = []

    def run(mode, block, unroll, al, as_, order, grid, reps=2):
        def fn():
            rc = LIB.probe_run(mode, block, unroll, al, as_, order, grid, tab, n,
                               ctypes.c_void_p(out.data_ptr()), nbytes, stream)
            assert rc == 0, rc
        t = min(timeit(fn) for _ in range(reps))
        moved = {0: (n + 1) * nbytes, 1: n * nbytes, 2: nbytes, 3: (n + 1) * nbytes}[mode]
        rows.append({"mode": ["mix", "read", "write", "mix_ldsdma"][mode], "n": n, "block": block,
                     "unroll": unroll, "aux_load": al, "aux_store": as_, "order": order, "grid": grid,
                     "ms": round(t * 1e3, 4), "GBps": round(moved / t / 1e9, 1)})

    # 1) mix: geometry x policy
    for block in (256, 512, 1024):
        for unroll in (1, 2, 4, 8):
            if block * unroll > 4096:
                continue
            for grid in (128, 192, 256, 384, 512, 1024):
                for al in (0, 2):
                    run(0, block, unroll, al, 0, 0, grid)
    print("geometry done", file=sys.stderr, flush=True)
    best = sorted([r for r in rows if r["mode"] == "mix"], key=lambda r: -r["GBps"])[:6]
    for b in best:  # 2) policies and order around the best geometries
        for al in (0, 2, 16):
            for as_ in (0, 2, 16, 17):
                for order in (0, 1):
                    run(0, b["block"], b["unroll"], al, as_, order, b["grid"])
    print("policy done", file=sys.stderr, flush=True)
    for block, unroll in ((256, 4), (512, 2), (256, 8)):  # 3) read-only / write-only ceilings
        for grid in (256, 512, 1024):
            run(1, block, unroll, 2, 0, 0, grid)
            run(2, block, unroll, 0, 0, 0, grid)
    for grid in (256, 512):
        run(3, 256, 1, 2, 0, 0, grid)
    for mode in ("mix", "read", "write", "mix_ldsdma"):
        sel = sorted([r for r in rows if r["mode"] == mode], key=lambda r: -r["GBps"])
        for r in sel[:8]:
            print(json.dumps(r))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "stagger":
        stagger_main(int(sys.argv[1]))
    else:
        main()
