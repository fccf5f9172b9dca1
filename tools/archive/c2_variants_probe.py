"""Config-2 kernel variants on the bucket layout (round 6).  With the
bucket's fixed physical placement (hiccl_bucket_alloc; spread between
instances <= 0.5 %) small differences between kernel shapes are measurable
on one box; earlier sweeps ran on separate allocations, whose placement
lottery (up to 9 %) was larger than most of the differences they looked
for.  Interleaved rounds over the variants on each bucket, every variant's
output compared bit for bit with the default's.
  usage: python tools/c2_variants_probe.py [--buckets 2] [--rounds 5] [--reps 10]
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
VARIANTS = {
    "default": None,
    "tile_u4_bpc2": dict(engine=1, unroll=4, blocks_per_cu=2),
    "tile_u2_bpc2": dict(engine=1, unroll=2, blocks_per_cu=2),
    "tile_u8": dict(engine=1, unroll=8),
    "tile_u4_b512": dict(engine=1, unroll=4, block=512),
    "tile_u4_grab2": dict(engine=1, unroll=4, grab=2),
    "tile_u4_static": dict(engine=1, unroll=4, schedule=1),
    "phase": dict(engine=2),
    "write_through": dict(store_policy=4),
    "tile_u4_grid192": dict(engine=1, unroll=4, grid=192),
    "tile_u4_bpc3": dict(engine=1, unroll=4, blocks_per_cu=3),
    # fewer bytes in flight (r06i: more in flight lost 12-29 %)
    "tile_u2": dict(engine=1, unroll=2, blocks_per_cu=1, schedule=2),
    "tile_u1": dict(engine=1, unroll=1, blocks_per_cu=1, schedule=2),
    "tile_u4_grid240": dict(engine=1, unroll=4, grid=240),
    "tile_u4_grid224": dict(engine=1, unroll=4, grid=224),
    "tile_u4_drain": dict(engine=1, unroll=4, drain=1),
}


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
    ap.add_argument("--buckets", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    variants = {k: v for k, v in VARIANTS.items() if not args.only or k in args.only.split(",") or k == "default"}
    buckets = []
    for _ in range(args.buckets):
        ins, out = hiccl_amd.bucket(N, COUNT)
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, SEED, k)
        buckets.append((ins, out))
    ref = torch.empty(COUNT, device="cuda")
    hiccl_amd.reduce(ref, buckets[0][0])
    torch.cuda.synchronize()
    summary = {}
    for b, (ins, out) in enumerate(buckets):
        fns = {k: (lambda c=c: hiccl_amd.reduce(out, ins, config=c)) for k, c in variants.items()}
        exact = {}
        for k, fn in fns.items():
            fn()
            torch.cuda.synchronize()
            exact[k] = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            timed(fn, 2)
        ms = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, fn in fns.items():
                ms[k] += timed(fn, args.reps)
        base = float(np.mean(ms["default"]))
        for k in fns:
            m = float(np.mean(ms[k]))
            summary.setdefault(k, []).append(round(m / base, 4))
            print(json.dumps({"bucket": b, "variant": k, "config": variants[k], "kernel_ms_mean": round(m, 4),
                              "frac_of_8TBs": round(9 * COUNT * 4 / (m * 1e-3) / 8e12, 4),
                              "over_default": round(m / base, 4), "bit_exact": exact[k]}), flush=True)
    print(json.dumps({"summary": "time over the default, per bucket", **summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
