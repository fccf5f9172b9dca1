#!/usr/bin/env python3
"""C2 with every input shifted 1-3 elements: the reduction under each load
cache policy (nt = the default; plain loads keep the 128-B lines two
neighbouring wave loads share in L2), interleaved, aligned buckets beside.
One JSON line per (case, policy, round)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import hiccl_amd  # noqa: E402

n, count = 8, 1 << 28
for rnd in range(2):
    for name, offs in (("aligned", [0] * n), ("shifted", [1 + k % 3 for k in range(n)])):
        bases = [torch.empty(count + 4, dtype=torch.float32, device="cuda") for _ in range(n)]
        ins = [b[o:o + count] for b, o in zip(bases, offs)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, bench.SEED, k)
        out = torch.empty(count, dtype=torch.float32, device="cuda")
        for pol, cfg in (("nt loads", None), ("plain loads", dict(nontemporal=1)),
                         ("plain loads, plain stores", dict(nontemporal=1, store_policy=1))):
            _, ms = bench.time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), 10, 3)
            t = float(np.median(ms)) * 1e-3
            print(json.dumps({"round": rnd, "case": name, "offsets": offs, "policy": pol,
                              "sample_ok": bench.sample_check(out, n, count),
                              "GBps": round(9 * count * 4 / t / 1e9, 1)}), flush=True)
        del bases, ins, out
        torch.cuda.empty_cache()
