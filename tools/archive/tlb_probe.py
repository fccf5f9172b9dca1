"""Placement study: several fresh 8 x 1 GiB buckets (separate allocations,
as bench.py makes them); per bucket the median kernel time.  Run under
rocprofv3 --pmc with translation counters to correlate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hiccl_amd  # noqa: E402

n, count = 8, 1 << 28
keep = []
for b in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    ins = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, 1234, k)
    out = torch.empty(count, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(4):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        hiccl_amd.reduce(out, ins)
        e.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e))
    print(json.dumps({"bucket": b, "kernel_ms": [round(t, 4) for t in ts],
                      "GBps": round(9 * count * 4 / sorted(ts)[2] / 1e6, 1),
                      "ptrs": [hex(t.data_ptr()) for t in ins[:2]] + [hex(out.data_ptr())]}), flush=True)
    keep.append((ins, out))  # keep allocated: each bucket gets fresh memory
