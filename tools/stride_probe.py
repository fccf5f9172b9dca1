"""Relative-placement probe (round 6): the 8-stream read rate as a function
of the stride between the streams inside ONE allocation.

Separate allocations put config 2's inputs at arbitrary relative physical
placements and their joint read rate moves by ~9 % with it
(profiles/r06r_placement_swap.jsonl); inside one large allocation the
relative placement is the virtual one (as far as the allocation is
physically contiguous), so sweeping the stride maps which relative offsets
the HBM address interleave serves well.  For each of `--pools` fresh pools
and each stride S: tools/libhbm_probe.so's read-only kernel over 8 streams
of `--mib` MiB at base + k * S, median of `--reps`, interleaved rounds.
  usage: python tools/stride_probe.py [--pools 2] [--mib 256] [--reps 10] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP = ctypes.CDLL("libamdhip64.so.7")
HIP.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
HIP.hipFree.argtypes = [ctypes.c_void_p]
MiB, KiB = 1 << 20, 1 << 10
N = 8


def timed(fn, reps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pools", type=int, default=2)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.init()
    B = args.mib * MiB
    strides = {"1x": B, "1x+4K": B + 4 * KiB, "1x+64K": B + 64 * KiB, "1x+1M": B + MiB, "1x+2M": B + 2 * MiB,
               "1x+8M": B + 8 * MiB, "1x+32M": B + 32 * MiB, "1.25x": B * 5 // 4, "1.5x": B * 3 // 2, "2x": 2 * B,
               "3x": 3 * B, "4x": 4 * B, "8x": 8 * B}
    span = max(strides.values()) * (N - 1) + B
    probe = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
    probe.probe_run.restype = ctypes.c_int
    probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_uint64, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for p in range(args.pools):
        base = ctypes.c_void_p()
        if HIP.hipMalloc(ctypes.byref(base), span) != 0:
            print(json.dumps({"pool": p, "error": f"hipMalloc({span}) failed"}), flush=True)
            break
        fns = {}
        for name, S in strides.items():
            tab = (ctypes.c_void_p * N)(*[base.value + k * S for k in range(N)])
            fns[name] = (lambda tab=tab: probe.probe_run(1, 256, 4, 2, 2, 0, 256, tab, N, tab[0], B, st))
        for fn in fns.values():
            timed(fn, 2)
        ms = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, fn in fns.items():
                ms[k] += timed(fn, args.reps)
        rates = {k: round(N * B / (np.median(v) * 1e-3) / 1e9, 1) for k, v in ms.items()}
        print(json.dumps({"pool": p, "base_GiB": round(base.value / 2**30, 3), "mib_per_stream": args.mib,
                          "read_GBps_by_stride": rates}), flush=True)
        for k, v in rates.items():
            out.setdefault(k, []).append(v)
        HIP.hipFree(base)
    print(json.dumps({"summary": "8-stream read-only GB/s by stride, per pool", **out}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
