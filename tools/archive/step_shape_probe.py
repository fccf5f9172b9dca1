"""The C5 step kernel's shape under write-through stores (round 6).

The step's batched reduction (4 computes of n = 2 and one of n = 4, 2^18
f32 each: 12 MiB read, 5 MiB written) was shaped in
round 2 with nt stores (TILE, unroll 2, 4 workgroups per CU:
profiles/r02c_plan_sweep.jsonl).  Round 5 made its stores write-through.
This probe times the plan under several shapes -- queued (events around
200 back-to-back launches) -- in interleaved rounds, every shape's outputs
compared bit for bit with the default's.
    python tools/step_shape_probe.py > gpurun_out/<tag>_step_shape.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hiccl_amd  # noqa: E402

SHAPES = {
    "default": None,
    "u4_bpc1": dict(engine=1, unroll=4, blocks_per_cu=1),
    "u4_bpc2": dict(engine=1, unroll=4, blocks_per_cu=2),
    "u4_bpc4": dict(engine=1, unroll=4, blocks_per_cu=4),
    "u2_bpc1": dict(engine=1, unroll=2, blocks_per_cu=1),
    "u2_bpc2": dict(engine=1, unroll=2, blocks_per_cu=2),
    "u2_grid320": dict(engine=1, unroll=2, grid=320),
    "u2_grid160": dict(engine=1, unroll=2, grid=160),
    "phase": dict(engine=2),
}


def queued_us(comp, n=200):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(n):
        comp.enqueue(s)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    dev = torch.cuda.current_device()
    c = 1 << 18
    bufs = [torch.empty(c, device="cuda") for _ in range(12)]
    for k, t in enumerate(bufs):
        hiccl_amd.fill_uniform(t, 1234, k)
    comps, outs = {}, {}
    for name, cfg in SHAPES.items():
        o = [torch.empty(c, device="cuda") for _ in range(5)]
        comp = hiccl_amd.Compute(torch.float32, device=dev, config=cfg)
        for j in range(4):
            comp.add([bufs[2 * j], bufs[2 * j + 1]], o[j], c, compid=0)
        comp.add(bufs[8:12], o[4], c, compid=0)
        comp.start()
        comp.wait()
        comps[name], outs[name] = comp, o
    exact = {k: all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(v, outs["default"]))
             for k, v in outs.items()}
    us = {k: [] for k in comps}
    for _ in range(5):
        for k, comp in comps.items():
            us[k].append(queued_us(comp))
    base = float(np.median(us["default"]))
    for k in comps:
        m = float(np.median(us[k]))
        print(json.dumps({"shape": k, "config": SHAPES[k], "engine": comps[k].engine(),
                          "store_policy": comps[k].store_policy(), "queued_us_median": round(m, 3),
                          "us_per_round": [round(x, 3) for x in us[k]], "over_default": round(m / base, 4),
                          "frac_of_8TBs": round(17 * (1 << 20) / (m * 1e-6) / 8e12, 4),
                          "bit_exact": exact[k]}), flush=True)
    for comp in comps.values():
        comp.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
