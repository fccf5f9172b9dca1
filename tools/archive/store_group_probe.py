#!/usr/bin/env python3
"""Grouped-store probe (Next 2): does writing in bursts
of G tiles per workgroup move the C2 read/write mix (8 x 1 GiB read + 1 GiB
written) closer to the serial read-only + write-only bound?

tools/libhbm_probe.so mode 4 (XOR instead of add, nt loads and stores) on
the C2 bucket shape, each (U, G, grid) interleaved over rounds on the same
buffers, with the read-only (mode 1) and write-only (mode 2) rates of the
same buffers.  Writes JSON lines to stdout.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

LIB = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
LIB.probe_run.restype = ctypes.c_int
LIB.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_void_p]


def main():
    n, count = 8, 1 << 28
    ins = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(n)]
    out = torch.empty(count, dtype=torch.float32, device="cuda")
    for t in ins:
        t.fill_(1.0)
    tab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbytes = count * 4

    def runner(mode, unroll, order, grid):
        def fn():
            rc = LIB.probe_run(mode, 256, unroll, 2, 2, order, grid, tab, n, ctypes.c_void_p(out.data_ptr()),
                               nbytes, st)
            if rc:
                raise RuntimeError(f"probe_run rc {rc}")
        return fn

    variants = [("read_only", 1, 4, 0, 256, n), ("write_only", 2, 4, 0, 256, 1)]
    for u, g in ((4, 1), (4, 2), (2, 2), (2, 4), (1, 4), (1, 8)):
        for grid in (256, 512, 1024):
            variants.append((f"mix_u{u}_g{g}_grid{grid}", 4, u, g, grid, n + 1))
    res = {v[0]: [] for v in variants}
    for _ in range(3):
        for name, mode, u, g, grid, streams in variants:
            _, ms = bench.time_launches(runner(mode, u, g, grid), 10, 3)
            res[name].append(float(np.median(ms)))
    t = {name: float(np.median(v)) for name, v in res.items()}
    read_rate = n * nbytes / (t["read_only"] * 1e-3)
    write_rate = nbytes / (t["write_only"] * 1e-3)
    serial_ms = (n * nbytes / read_rate + nbytes / write_rate) * 1e3
    print(json.dumps({"read_only_GBps": round(read_rate / 1e9, 1), "write_only_GBps": round(write_rate / 1e9, 1),
                      "serial_ms": round(serial_ms, 4)}), flush=True)
    for name, mode, u, g, grid, streams in variants[2:]:
        print(json.dumps({"variant": name, "unroll": u, "group": g, "grid": grid, "ms": round(t[name], 4),
                          "GBps": round((n + 1) * nbytes / (t[name] * 1e-3) / 1e9, 1),
                          "frac_of_serial": round(serial_ms / t[name], 4)}), flush=True)


if __name__ == "__main__":
    main()
