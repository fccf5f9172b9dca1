"""Which buffer makes a separate-allocation bucket slow? (round 6)

Allocates several config-2 buckets as separate torch buffers (bench.py's
rounds 1-5 layout), times each, then takes the slowest (S) and the fastest
(F) and times hybrids: S's inputs with F's output, F's inputs with S's
output, and S with one input at a time replaced by F's same-index input.
Also the 8-stream read-only probe (tools/libhbm_probe.so, mode 1) on S's and
F's inputs.  Every hybrid's output is compared bit for bit with the
reference output (every bucket holds the same generated inputs).
  usage: python tools/placement_swap_probe.py [--buckets 6] [--reps 10] [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hiccl_amd  # noqa: E402

N, COUNT, SEED = 8, 1 << 28, 1234


def timed(fn, reps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def mean_ms(fns, reps, rounds):
    """Interleaved rounds over the named launches; mean ms each."""
    for fn in fns.values():
        timed(fn, 2)
    ms = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            ms[k] += timed(fn, reps)
    return {k: round(float(np.mean(v)), 4) for k, v in ms.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--engines", action="store_true",
                    help="also every bucket under the phased engine and the static tile schedule")
    args = ap.parse_args()
    buckets = []
    for _ in range(args.buckets):
        ins = [torch.empty(COUNT, device="cuda") for _ in range(N)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, SEED, k)
        buckets.append((ins, torch.empty(COUNT, device="cuda")))
    ref = torch.empty(COUNT, device="cuda")
    hiccl_amd.reduce(ref, buckets[0][0])
    torch.cuda.synchronize()
    t = mean_ms({b: (lambda b=b: hiccl_amd.reduce(buckets[b][1], buckets[b][0])) for b in range(len(buckets))},
                args.reps, args.rounds)
    print(json.dumps({"buckets_ms": t}), flush=True)
    if args.engines:
        cfgs = {"phase": dict(engine=2), "tile_static": dict(engine=1, unroll=4, schedule=1)}
        fns = {f"{b}:{k}": (lambda b=b, c=c: hiccl_amd.reduce(buckets[b][1], buckets[b][0], config=c))
               for b in range(len(buckets)) for k, c in cfgs.items()}
        print(json.dumps({"buckets_engines_ms": mean_ms(fns, args.reps, args.rounds)}), flush=True)
    s = max(t, key=t.get)
    f = min(t, key=t.get)
    (si, so), (fi, fo) = buckets[s], buckets[f]
    hy = {"S": (si, so), "F": (fi, fo), "S_inputs+F_output": (si, fo), "F_inputs+S_output": (fi, so)}
    for k in range(N):
        hy[f"S_with_F_input{k}"] = ([fi[j] if j == k else si[j] for j in range(N)], fo)
    fns = {name: (lambda i=i, o=o: hiccl_amd.reduce(o, i)) for name, (i, o) in hy.items()}
    res = mean_ms(fns, args.reps, args.rounds)
    exact = {}
    for name, (i, o) in hy.items():
        hiccl_amd.reduce(o, i)
        torch.cuda.synchronize()
        exact[name] = bool(torch.equal(o.view(torch.int32), ref.view(torch.int32)))
    probe = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
    probe.probe_run.restype = ctypes.c_int
    probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_uint64, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    reads = {}
    for name, (i, o) in (("S", (si, so)), ("F", (fi, fo))):
        tab = (ctypes.c_void_p * N)(*[x.data_ptr() for x in i])
        fn = lambda: probe.probe_run(1, 256, 4, 2, 2, 0, 256, tab, N, ctypes.c_void_p(o.data_ptr()),  # noqa: E731
                                     COUNT * 4, st)
        timed(fn, 2)
        reads[name] = round(N * COUNT * 4 / (np.median(timed(fn, args.reps)) * 1e-3) / 1e9, 1)
    print(json.dumps({"slow_bucket": s, "fast_bucket": f, "hybrids_ms": res, "bit_exact": exact,
                      "read_only_8stream_GBps": reads}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
