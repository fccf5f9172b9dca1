#!/usr/bin/env python3
"""Does the C5 step kernel pay for dirty L2 lines at its kernel boundary?

The C5 step's batched reduction (4 computes of n = 2 and one of n = 4,
2^18 f32 each at scale 1: 12 MiB read, 5 MiB written; DESIGN.md section 5
M11) costs ~3.4 us per eager launch beyond its bytes, and the MI355X price
table (MI355X_MICROARCH.md "boundary") adds B / 6 TB/s to a kernel boundary
when the predecessor leaves B bytes dirty.  nt stores are not write-through:
the step's 5 MiB of outputs may sit dirty in the XCD L2s until the
end-of-kernel release writes them back.  This probe times the same plan
with nt stores (store_policy 2) and with system-scope write-through
stores (store_policy 4: the peer-store form, sc0 sc1), queued (events around 200 back-to-back launches) and as
one hipGraph of 200 launches, at scales 1/4 .. 16, interleaved rounds; and
the step's copies (5 x 1 MiB byte plans) the same way.  Both policies must
give the same bits.  One JSON line per scale, then a summary.

    python tools/step_store_probe.py > gpurun_out/<tag>_step_store.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench as B  # noqa: E402
import hiccl_amd  # noqa: E402


def step_plan(dev, bufs, outs, c, peer):
    # explicit store forms: 2 nt, 4 write-through (round 5's default picks
    # by size; this probe is what set it)
    comp = hiccl_amd.Compute(torch.float32, device=dev, config=dict(store_policy=4 if peer else 2))
    for j in range(4):
        comp.add([bufs[2 * j], bufs[2 * j + 1]], outs[j], c, compid=0)
    comp.add(bufs[8:12], outs[4], c, compid=0)
    assert comp.store_policy() == (4 if peer else 2)
    return comp


def copy_plan(dev, src, dst, nbytes, peer):
    cp = hiccl_amd.Compute(torch.uint8, device=dev, config=dict(store_policy=4 if peer else 2))
    for a, b in zip(src, dst):
        cp.add([a.view(torch.uint8)], b.view(torch.uint8), nbytes, compid=0)
    assert cp.store_policy() == (4 if peer else 2)
    return cp


def graph_us(fn, n=200):
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        cs = torch.cuda.current_stream()
        with torch.cuda.graph(g, stream=cs):
            for _ in range(n):
                fn(cs)
    v = []
    for _ in range(5):
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        v.append(a.elapsed_time(b) * 1e3 / n)
    return float(np.median(v))


def main():
    dev = torch.cuda.current_device()
    stream = torch.cuda.current_stream()
    scales = (0.25, 0.5, 1, 2, 4, 8, 16)
    cases = {}
    for f in scales:
        c = int((1 << 18) * f)
        bufs = [torch.empty(c, device="cuda") for _ in range(12)]
        for k, t in enumerate(bufs):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        outs = {p: [torch.empty(c, device="cuda") for _ in range(5)] for p in (0, 1)}
        src = [torch.empty(c, device="cuda") for _ in range(5)]
        for k, t in enumerate(src):
            hiccl_amd.fill_uniform(t, B.SEED, 20 + k)
        dst = {p: [torch.empty(c, device="cuda") for _ in range(5)] for p in (0, 1)}
        cases[f] = {"c": c, "bufs": bufs, "outs": outs, "src": src, "dst": dst,
                    "red": {p: step_plan(dev, bufs, outs[p], c, p) for p in (0, 1)},
                    "cp": {p: copy_plan(dev, src, dst[p], c * 4, p) for p in (0, 1)}}
    res = {(f, kind, p): [] for f in scales for kind in ("red", "cp") for p in (0, 1)}
    for _ in range(5):
        for f in scales:
            for kind in ("red", "cp"):
                for p in (0, 1):
                    plan = cases[f][kind][p]
                    res[(f, kind, p)].append(B.time_queued(lambda: plan.enqueue(stream), 200, 10) * 1e3)
    torch.cuda.synchronize()
    rows = []
    for f in scales:
        cs_ = cases[f]
        c = cs_["c"]
        ok = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(cs_["outs"][0], cs_["outs"][1]))
        ok = ok and all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(cs_["dst"][0], cs_["src"]))
        ok = ok and all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(cs_["dst"][1], cs_["src"]))
        ref = torch.empty(c, device="cuda")
        hiccl_amd.reduce(ref, cs_["bufs"][8:12])
        ok = ok and torch.equal(ref.view(torch.int32), cs_["outs"][0][4].view(torch.int32))
        red_b, cp_b = 17 * c * 4, 10 * c * 4
        row = {"mode": "step_store", "scale": f, "count": c, "bits_ok": bool(ok), "reduce_bytes": red_b,
               "copy_bytes": cp_b}
        for kind, nb in (("red", red_b), ("cp", cp_b)):
            for p, name in ((0, "nt"), (1, "wt")):
                t = float(np.median(res[(f, kind, p)]))
                row[f"{kind}_{name}_us"] = round(t, 3)
                row[f"{kind}_{name}_GBps"] = round(nb / t * 1e-3, 1)
        if f == 1:
            for kind in ("red", "cp"):
                for p, name in ((0, "nt"), (1, "wt")):
                    plan = cs_[kind][p]
                    plan.enqueue(stream)  # uploaded before the capture
                    torch.cuda.synchronize()
                    row[f"{kind}_{name}_graph_us"] = round(graph_us(lambda s_, pl=plan: pl.enqueue(s_)), 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    one = rows[scales.index(1)]
    print(json.dumps({"summary": "step_store", "device": torch.cuda.get_device_properties(0).name,
                      "reduce_wt_over_nt_scale1": round(one["red_wt_us"] / one["red_nt_us"], 4),
                      "copy_wt_over_nt_scale1": round(one["cp_wt_us"] / one["cp_nt_us"], 4),
                      "reduce_wt_over_nt": {str(r["scale"]): round(r["red_wt_us"] / r["red_nt_us"], 4) for r in rows},
                      "copy_wt_over_nt": {str(r["scale"]): round(r["cp_wt_us"] / r["cp_nt_us"], 4) for r in rows},
                      "all_bits_ok": all(r["bits_ok"] for r in rows)}), flush=True)
    for f in scales:
        for kind in ("red", "cp"):
            for p in (0, 1):
                cases[f][kind][p].close()
    oneshot()
    return 0


def oneshot():
    """One-shot hiccl_reduce calls (the single-compute kernel) of n inputs x
    1-64 MiB: nt vs write-through stores (store_policy 2 / 4) and the default
    (0: by size), queued, interleaved rounds; the same bits."""
    stream = torch.cuda.current_stream()
    rows = []
    for n in (2, 8):
        for mib in (1, 4, 16, 32, 64):
            c = (mib << 20) // 4
            ins = [torch.empty(c, device="cuda") for _ in range(n)]
            for k, t in enumerate(ins):
                hiccl_amd.fill_uniform(t, B.SEED, k)
            outs = {k: torch.empty(c, device="cuda") for k in ("nt", "wt", "auto")}
            cfgs = {"nt": dict(store_policy=2), "wt": dict(store_policy=4), "auto": None}
            res = {k: [] for k in cfgs}
            for _ in range(5):
                for k, cfg in cfgs.items():
                    res[k].append(B.time_queued(lambda: hiccl_amd.reduce(outs[k], ins, config=cfg, stream=stream),
                                                100, 5) * 1e3)
            torch.cuda.synchronize()
            ok = all(torch.equal(outs["nt"].view(torch.int32), outs[k].view(torch.int32)) for k in ("wt", "auto"))
            nb = (n + 1) * c * 4
            row = {"mode": "oneshot_store", "n": n, "mib_per_input": mib, "bits_ok": bool(ok)}
            for k in cfgs:
                t = float(np.median(res[k]))
                row[f"{k}_us"] = round(t, 3)
                row[f"{k}_GBps"] = round(nb / t * 1e-3, 1)
            row["wt_over_nt"] = round(row["wt_us"] / row["nt_us"], 4)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del ins, outs
    return rows


if __name__ == "__main__":
    sys.exit(main())
