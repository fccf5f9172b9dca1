#!/usr/bin/env python3
"""Where does write-through stop paying?  Round 5 stores write-through when a
launch writes <= 32 MiB (kWtMaxBytes), set from the C5 step shape scaled
1/4x-16x (tools/step_store_probe.py: reductions still 3-6 % faster at 40
and 80 MiB written, byte copies 4-5 % slower at 80 MiB).  This probe times
larger launches with both store forms (store_policy 2 nt / 4 write-through),
interleaved rounds, events around each launch (median), same bits:
  * one-shot reductions of 8 inputs writing 32 / 64 / 128 / 256 MiB
    (C4's 64 MiB-per-input bucket is the 64 MiB row; C3 n = 8 the 256 MiB);
  * the same buckets as plans of 1 MiB computes (C4's structure);
  * one-shot reductions of 2 inputs writing 64 / 256 MiB (few inputs: the
    write share is a third of the bytes);
  * byte copies of 48 / 64 / 128 MiB (the transport's).
One JSON line per case.

    python tools/store_threshold_probe.py > gpurun_out/<tag>_store_threshold.jsonl
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

FORMS = {"nt": 2, "wt": 4}


def timed(fns, steps=10, warmup=3, rounds=5):
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            _, ms = B.time_launches(fn, steps, warmup)
            res[k].append(float(np.median(ms)))
    return {k: float(np.median(v)) for k, v in res.items()}


def row(kind, n, mib, nbytes, t, ok, extra=None):
    r = {"mode": "store_threshold", "kind": kind, "n": n, "mib_written": mib, "bits_ok": bool(ok)}
    for k, v in t.items():
        r[f"{k}_us"] = round(v * 1e3, 2)
        r[f"{k}_GBps"] = round(nbytes / (v * 1e-3) / 1e9, 1)
    r["wt_over_nt"] = round(t["wt"] / t["nt"], 4)
    r.update(extra or {})
    print(json.dumps(r), flush=True)


def c3(stream):
    """Config 3's buckets (n x 256 MiB, 256 MiB written) in both forms."""
    c = (256 << 20) // 4
    for n in (2, 3, 4, 8, 16, 32, 64):
        ins = [torch.empty(c, device="cuda") for _ in range(n)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        outs = {f: torch.empty(c, device="cuda") for f in FORMS}
        fns = {f: (lambda f=f: hiccl_amd.reduce(outs[f], ins, config=dict(store_policy=FORMS[f]), stream=stream))
               for f in FORMS}
        t = timed(fns)
        torch.cuda.synchronize()
        ok = torch.equal(outs["nt"].view(torch.int32), outs["wt"].view(torch.int32))
        row("c3_oneshot", n, 256, (n + 1) * c * 4, t, ok)
        del ins, outs
        torch.cuda.empty_cache()


def big(stream):
    """Config 2's bucket (8 x 1 GiB) and 2 x 1 GiB / 8 x 512 MiB: AUTO (TILE
    on the dynamic schedule at C2) and the phased engine, each with nt and
    write-through stores; wide tiles (AUTO at 2 x 1 GiB) have nt only."""
    for n, mib in ((8, 1024), (8, 512), (2, 1024)):
        c = (mib << 20) // 4
        ins = [torch.empty(c, device="cuda") for _ in range(n)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        out = {}
        variants = {"auto_nt": dict(store_policy=2), "phase_nt": dict(store_policy=2, engine=2),
                    "phase_wt": dict(store_policy=4, engine=2), "tile4_nt": dict(store_policy=2, engine=1, unroll=4),
                    "tile4_wt": dict(store_policy=4, engine=1, unroll=4)}
        if n == 8:
            variants["auto_wt"] = dict(store_policy=4)
        for k in variants:
            out[k] = torch.empty(c, device="cuda")
        fns = {k: (lambda k=k: hiccl_amd.reduce(out[k], ins, config=variants[k], stream=stream)) for k in variants}
        t = timed(fns, steps=10, warmup=2, rounds=5)
        torch.cuda.synchronize()
        ok = all(torch.equal(out["auto_nt"].view(torch.int32), v.view(torch.int32)) for v in out.values())
        nb = (n + 1) * c * 4
        r = {"mode": "store_threshold", "kind": "big", "n": n, "mib_written": mib, "bits_ok": bool(ok)}
        for k, v in t.items():
            r[f"{k}_ms"] = round(v, 4)
            r[f"{k}_frac"] = round(nb / (v * 1e-3) / 1e9 / 8000.0, 4)
        print(json.dumps(r), flush=True)
        del ins, out
        torch.cuda.empty_cache()


def split(stream):
    """Config 2's bucket (8 x 1 GiB, one set of allocations) reduced by one
    launch, or by 2 / 4 / 8 launches over consecutive element ranges (views
    of the same buffers), each in its default store form (a quarter or an
    eighth writes <= 256 MiB: write-through) and the quarters also nt;
    whole-bucket time between events around the launches, interleaved
    rounds, same bits."""
    n, c = 8, 1 << 28
    ins = [torch.empty(c, device="cuda") for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, B.SEED, k)
    outs = {}

    def parts(k, cfg=None):
        out = outs.setdefault((k, str(cfg)), torch.empty(c, device="cuda"))
        step = c // k

        def run():
            for j in range(k):
                lo = j * step
                hiccl_amd.reduce(out[lo:lo + step], [x[lo:lo + step] for x in ins], config=cfg, stream=stream)
        return run
    fns = {"one": parts(1), "halves": parts(2), "quarters": parts(4), "quarters_nt": parts(4, dict(store_policy=2)),
           "eighths": parts(8)}
    t = timed(fns, steps=10, warmup=2, rounds=5)
    torch.cuda.synchronize()
    ref = outs[(1, "None")]
    ok = all(torch.equal(ref.view(torch.int32), v.view(torch.int32)) for v in outs.values())
    nb = (n + 1) * c * 4
    r = {"mode": "store_threshold", "kind": "c2_split", "bits_ok": bool(ok)}
    for k, v in t.items():
        r[f"{k}_ms"] = round(v, 4)
        r[f"{k}_frac"] = round(nb / (v * 1e-3) / 1e9 / 8000.0, 4)
    print(json.dumps(r), flush=True)


def engines(stream):
    """Config 3's few-input buckets (n x 256 MiB) with the round-5 default
    store form (write-through at this size): AUTO against the TILE engine
    (static and dynamic) and the phased engine, interleaved rounds -- does
    AUTO's engine choice, set with nt stores, still hold?"""
    c = (256 << 20) // 4
    variants = {"auto": None, "tile": dict(engine=1), "tile_dyn": dict(engine=1, schedule=2),
                "phase": dict(engine=2)}
    ns = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else (2, 3, 4, 8)
    for n in ns:
        ins = [torch.empty(c, device="cuda") for _ in range(n)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        outs = {v: torch.empty(c, device="cuda") for v in variants}
        fns = {v: (lambda v=v: hiccl_amd.reduce(outs[v], ins, config=variants[v], stream=stream)) for v in variants}
        t = timed(fns)
        torch.cuda.synchronize()
        ok = all(torch.equal(outs["auto"].view(torch.int32), o.view(torch.int32)) for o in outs.values())
        nb = (n + 1) * c * 4
        r = {"mode": "store_threshold", "kind": "c3_engines", "n": n, "bits_ok": bool(ok)}
        for k, v in t.items():
            r[f"{k}_GBps"] = round(nb / (v * 1e-3) / 1e9, 1)
        print(json.dumps(r), flush=True)
        del ins, outs
        torch.cuda.empty_cache()


def c4(stream):
    """Config 4's batched plans (8 inputs in 1 MiB computes, one launch) at
    16 / 64 / 256 MiB per input, f32 and bf16, nt against write-through,
    interleaved rounds, same bits."""
    for dtype in (torch.float32, torch.bfloat16):
        esz = torch.tensor([], dtype=dtype).element_size()
        for mib in (16, 64, 256):
            c = (mib << 20) // esz
            ins = [torch.empty(c, dtype=dtype, device="cuda") for _ in range(8)]
            for k, t in enumerate(ins):
                hiccl_amd.fill_uniform(t, B.SEED, k)
            outs = {f: torch.empty(c, dtype=dtype, device="cuda") for f in FORMS}
            plans = {}
            step = (1 << 20) // esz
            for f in FORMS:
                comp = hiccl_amd.Compute(dtype, device=torch.cuda.current_device(), config=dict(store_policy=FORMS[f]))
                for off in range(0, c, step):
                    comp.add([(x, off) for x in ins], (outs[f], off), min(step, c - off), compid=0)
                plans[f] = comp
            t = timed({f: (lambda p=p: p.start(stream=stream)) for f, p in plans.items()})
            torch.cuda.synchronize()
            bits = torch.int16 if dtype == torch.bfloat16 else torch.int32
            ok = torch.equal(outs["nt"].view(bits), outs["wt"].view(bits))
            row("c4_plan", 8, mib, 9 * c * esz, t, ok, {"dtype": str(dtype).split(".")[-1],
                                                         "engine": plans["nt"].engine()})
            for p in plans.values():
                p.close()
            del ins, outs
            torch.cuda.empty_cache()


def c4_engines(stream):
    """Config 4's batched f32 plans (8 inputs in 1 MiB computes) at 16 / 64 /
    256 MiB per input with the default store form: AUTO against each engine,
    interleaved rounds, same bits."""
    variants = {"auto": None, "tile": dict(engine=1), "tile_dyn": dict(engine=1, schedule=2), "phase": dict(engine=2)}
    dtype = torch.bfloat16 if len(sys.argv) > 2 and sys.argv[2] == "bf16" else torch.float32
    esz = torch.tensor([], dtype=dtype).element_size()
    bits = torch.int16 if dtype == torch.bfloat16 else torch.int32
    for mib in (16, 64, 256):
        c = (mib << 20) // esz
        ins = [torch.empty(c, dtype=dtype, device="cuda") for _ in range(8)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        outs = {v: torch.empty(c, dtype=dtype, device="cuda") for v in variants}
        plans = {}
        step = (1 << 20) // esz
        for v, cfg in variants.items():
            comp = hiccl_amd.Compute(dtype, device=torch.cuda.current_device(), config=cfg)
            for off in range(0, c, step):
                comp.add([(x, off) for x in ins], (outs[v], off), min(step, c - off), compid=0)
            plans[v] = comp
        t = timed({v: (lambda p=p: p.start(stream=stream)) for v, p in plans.items()})
        torch.cuda.synchronize()
        ok = all(torch.equal(outs["auto"].view(bits), o.view(bits)) for o in outs.values())
        r = {"mode": "store_threshold", "kind": "c4_engines", "dtype": str(dtype).split(".")[-1], "mib_per_input": mib,
             "bits_ok": bool(ok), "auto_engine": plans["auto"].engine(), "store_policy": plans["auto"].store_policy()}
        for k, v in t.items():
            r[f"{k}_GBps"] = round(9 * c * esz / (v * 1e-3) / 1e9, 1)
        print(json.dumps(r), flush=True)
        for p in plans.values():
            p.close()
        del ins, outs
        torch.cuda.empty_cache()


def c2_loads(stream):
    """Config 2's bucket (8 x 1 GiB) as a one-compute plan with the default
    loads (nt) and with system-scope loads (the peer-load form, sc0 sc1:
    another path through the caches), each with nt and write-through
    stores, against the one-shot launch; interleaved rounds, same bits."""
    n, c = 8, 1 << 28
    ins = [torch.empty(c, device="cuda") for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, B.SEED, k)
    outs, plans = {}, {}
    for name, peer, cfg in (("plan_nt", 0, dict(store_policy=2)), ("plan_sysload", 2, dict(store_policy=2)),
                            ("plan_sysload_wt", 2, dict(store_policy=4)), ("plan_wt", 0, dict(store_policy=4))):
        outs[name] = torch.empty(c, device="cuda")
        comp = hiccl_amd.Compute(torch.float32, device=torch.cuda.current_device(), config=dict(cfg, engine=1, unroll=4))
        if peer:
            comp.set_peer(peer)
        comp.add(ins, outs[name], c, compid=0)
        plans[name] = comp
    outs["oneshot"] = torch.empty(c, device="cuda")
    fns = {k: (lambda p=p: p.start(stream=stream)) for k, p in plans.items()}
    fns["oneshot"] = lambda: hiccl_amd.reduce(outs["oneshot"], ins, stream=stream)
    t = timed(fns, steps=10, warmup=2, rounds=5)
    torch.cuda.synchronize()
    ok = all(torch.equal(outs["oneshot"].view(torch.int32), o.view(torch.int32)) for o in outs.values())
    nb = (n + 1) * c * 4
    r = {"mode": "store_threshold", "kind": "c2_loads", "bits_ok": bool(ok)}
    for k, v in t.items():
        r[f"{k}_ms"] = round(v, 4)
        r[f"{k}_frac"] = round(nb / (v * 1e-3) / 1e9 / 8000.0, 4)
    print(json.dumps(r), flush=True)
    for p in plans.values():
        p.close()


def main():
    stream = torch.cuda.current_stream()
    if len(sys.argv) > 1 and sys.argv[1] == "c2loads":
        c2_loads(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "c4eng":
        c4_engines(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "c4":
        c4(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "engines":
        engines(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "split":
        split(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "c3":
        c3(stream)
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "big":
        big(stream)
        return 0
    for n, mibs in ((8, (32, 64, 128, 256)), (2, (64, 256))):
        for mib in mibs:
            c = (mib << 20) // 4
            ins = [torch.empty(c, device="cuda") for _ in range(n)]
            for k, t in enumerate(ins):
                hiccl_amd.fill_uniform(t, B.SEED, k)
            outs = {f: torch.empty(c, device="cuda") for f in FORMS}
            fns = {f: (lambda f=f: hiccl_amd.reduce(outs[f], ins, config=dict(store_policy=FORMS[f]),
                                                    stream=stream)) for f in FORMS}
            t = timed(fns)
            torch.cuda.synchronize()
            ok = torch.equal(outs["nt"].view(torch.int32), outs["wt"].view(torch.int32))
            row("oneshot", n, mib, (n + 1) * c * 4, t, ok)
            if n == 8:
                plans = {}
                for f in FORMS:
                    comp = hiccl_amd.Compute(torch.float32, device=torch.cuda.current_device(),
                                             config=dict(store_policy=FORMS[f]))
                    step = (1 << 20) // 4
                    for off in range(0, c, step):
                        comp.add([(x, off) for x in ins], (outs[f], off), min(step, c - off), compid=0)
                    plans[f] = comp
                t = timed({f: (lambda p=p: p.start(stream=stream)) for f, p in plans.items()})
                torch.cuda.synchronize()
                ok = torch.equal(outs["nt"].view(torch.int32), outs["wt"].view(torch.int32))
                row("plan_1MiB_computes", n, mib, (n + 1) * c * 4, t, ok,
                    {"engine": plans["nt"].engine(), "computes": mib})
                for p in plans.values():
                    p.close()
            del ins, outs
            torch.cuda.empty_cache()
    for mib in (48, 64, 128):
        nb = mib << 20
        src = torch.randint(0, 256, (nb,), dtype=torch.uint8, device="cuda")
        dst = {f: torch.empty(nb, dtype=torch.uint8, device="cuda") for f in FORMS}
        fns = {f: (lambda f=f: hiccl_amd.reduce(dst[f], [src], config=dict(store_policy=FORMS[f]), stream=stream))
               for f in FORMS}
        t = timed(fns)
        torch.cuda.synchronize()
        ok = all(torch.equal(d, src) for d in dst.values())
        row("byte_copy", 1, mib, 2 * nb, t, ok)
        del src, dst
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
