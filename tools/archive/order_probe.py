"""Tile-order probe (round 6): does interleaving the TILE engine's units over
2^L stretches of the bucket (hiccl_reduce_config_t.order) change config 2's
kernel time, and its spread over allocations?

Several config-2 buckets (8 x 2^28 fp32 + output): separate allocations as
bench.py makes them, plus one pool carved at exactly 1 GiB stride (every
input's tile t at the same offset mod 1 GiB).  For each bucket, interleaved
rounds over the orders, `reps` queued launches each (HIP events on the launch
stream); every order's output compared bit for bit with the linear order's.
One JSON line per bucket and order, then a summary line.
  usage: python tools/order_probe.py [--buckets 3] [--rounds 5] [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hiccl_amd  # noqa: E402

N, COUNT, SEED = 8, 1 << 28, 1234
ORDERS = (0, 2, 4, 8, 16, 64, 256)


def bucket_separate():
    ins = [torch.empty(COUNT, device="cuda") for _ in range(N)]
    return ins, torch.empty(COUNT, device="cuda"), None


def bucket_pool():
    pool = torch.empty((N + 1) * COUNT, device="cuda")
    ins = [pool[k * COUNT:(k + 1) * COUNT] for k in range(N)]
    return ins, pool[N * COUNT:], pool


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
    ap.add_argument("--buckets", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--orders", default=",".join(map(str, ORDERS)))
    args = ap.parse_args()
    orders = [int(o) for o in args.orders.split(",")]
    kinds = ["separate"] * args.buckets + ["pool_1GiB_stride"]
    summary = {o: [] for o in orders}
    for b, kind in enumerate(kinds):
        ins, out, keep = bucket_separate() if kind == "separate" else bucket_pool()
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, SEED, k)
        ref = torch.empty(COUNT, device="cuda")
        hiccl_amd.reduce(ref, ins)
        torch.cuda.synchronize()
        fns = {o: (lambda o=o: hiccl_amd.reduce(out, ins, config=dict(order=o) if o else None)) for o in orders}
        exact = {}
        for o, fn in fns.items():
            fn()
            torch.cuda.synchronize()
            exact[o] = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            timed(fn, 2)
        ms = {o: [] for o in orders}
        for _ in range(args.rounds):
            for o, fn in fns.items():
                ms[o] += timed(fn, args.reps)
        base = float(np.mean(ms[orders[0]]))
        for o in orders:
            m = float(np.mean(ms[o]))
            summary[o].append(m / base)
            print(json.dumps({"bucket": b, "kind": kind, "order": o, "kernel_ms_mean": round(m, 4),
                              "kernel_ms_median": round(float(np.median(ms[o])), 4),
                              "frac_of_8TBs": round(9 * COUNT * 4 / (m * 1e-3) / 8e12, 4),
                              "over_first_order": round(m / base, 4), "bit_exact_vs_linear": exact[o]}), flush=True)
        del ins, out, keep, ref
        torch.cuda.empty_cache()
    print(json.dumps({"summary": "time over the first order, per bucket",
                      **{str(o): [round(x, 4) for x in v] for o, v in summary.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
