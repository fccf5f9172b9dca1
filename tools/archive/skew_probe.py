"""Does the relative displacement of the inputs matter for a FIXED physical
allocation?  One pool per trial set; inputs at k*1GiB + s_k*4MiB for several
patterns s; kernel median by HIP events.  (Placement study)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hiccl_amd  # noqa: E402

n, count = 8, 1 << 28
GiB, MiB = 1 << 30, 1 << 20
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
patterns = [[0] * n] + [list(rng.integers(0, 4, n)) for _ in range(9)] + [[0] * n]


def timeit(out, ins, reps=10):
    for _ in range(3):
        hiccl_amd.reduce(out, ins)
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(s)
        hiccl_amd.reduce(out, ins)
        b.record(s)
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]


for pool_id in range(3):
    pool = torch.empty((n * GiB + 16 * MiB) // 4, dtype=torch.float32, device="cuda")
    out = torch.empty(count, dtype=torch.float32, device="cuda")
    for pat in patterns:
        ins = [pool[(k * GiB + int(pat[k]) * 4 * MiB) // 4:][:count] for k in range(n)]
        ms = timeit(out, ins)
        print(json.dumps({"pool": pool_id, "skew_4MiB": [int(v) for v in pat], "kernel_ms": round(ms, 4),
                          "GBps": round(9 * count * 4 / ms / 1e6, 1)}), flush=True)
    del pool, out, ins
    torch.cuda.empty_cache()
