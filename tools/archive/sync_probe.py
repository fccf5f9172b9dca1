#!/usr/bin/env python3
"""Host wait after a launch: hipStreamSynchronize vs polling hipStreamQuery.

The reference's Compute<T>::wait (compute.h:107-117) and the transport's wait
block in hipStreamSynchronize once per pipeline step.  This probe times one
config-5 step's plan (four 2-input and one 4-input compute of 2^18 floats) as
start + wait on the host clock, waiting by (a) hipStreamSynchronize and (b) a
hipStreamQuery spin, interleaved; plus the kernel alone by HIP events.  One
JSON line per variant.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hiccl_amd  # noqa: E402

DEV = "cuda:0"


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamQuery.restype = ctypes.c_int
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.restype = ctypes.c_int
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    comp = hiccl_amd.Compute(torch.float32, device=0)
    keep = []
    for n in (2, 2, 2, 2, 4):
        ins = [torch.rand(1 << 18, device=DEV) for _ in range(n)]
        out = torch.empty(1 << 18, device=DEV)
        comp.add(ins, out, 1 << 18, compid=0)
        keep.append((ins, out))
    s = ctypes.c_void_p(comp.stream_handle())
    lib = hiccl_amd._lib.lib()
    plan = comp._plan

    def launch():
        assert lib.hiccl_reduce_plan_launch(plan, s) == 0

    def wait_sync():
        assert hip.hipStreamSynchronize(s) == 0

    def wait_spin():
        while True:
            rc = hip.hipStreamQuery(s)
            if rc == 0:
                return
            assert rc == 600, rc  # hipErrorNotReady

    for _ in range(50):
        launch()
        wait_sync()
    res = {"sync": [], "spin": []}
    for _ in range(20):
        for name, w in (("sync", wait_sync), ("spin", wait_spin)):
            for _ in range(25):
                t0 = time.perf_counter()
                launch()
                w()
                res[name].append(time.perf_counter() - t0)
    ev = []
    st = torch.cuda.ExternalStream(comp.stream_handle(), device=DEV)
    for _ in range(200):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        launch()
        b.record(st)
        ev.append((a, b))
    torch.cuda.synchronize()
    kern = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
    for name, v in res.items():
        print(json.dumps({"probe": "host_wait", "wait": name, "step": "C5 step plan (4 x n=2 + 1 x n=4, 2^18 fp32)",
                          "median_us": round(float(np.median(v)) * 1e6, 2),
                          "p10_us": round(float(np.percentile(v, 10)) * 1e6, 2),
                          "p90_us": round(float(np.percentile(v, 90)) * 1e6, 2),
                          "kernel_us_events": round(kern, 2)}), flush=True)
    comp.close()


if __name__ == "__main__":
    main()
