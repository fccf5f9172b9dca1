#!/usr/bin/env python3
"""Closed tuning probes moved out of bench.py (round 5): kernel-variant
sweeps, schedule sweeps, the engine crossover, plan overhead, the C5-step
kernel at 1/8x-16x, config-2 input/output offsets and config 3's relative
input placement.  Their answers are in DESIGN.md section 5 and the
profiles/r0* files it cites; kept for reproducibility, not run by the
driver or the tests.  Run from the repo root:

    python tools/archive/bench_probes.py --mode schedsweep --sweepset fewn
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench as B  # noqa: E402
import hiccl_amd  # noqa: E402
from hiccl_amd import _lib as L  # noqa: E402

def sweep(args):
    """Interleaved A/B of kernel variants in one process (rule 24), with the
    no-arithmetic 8R+1W probe (tools/libhbm_probe.so) as the ceiling row."""
    n, count = args.n, 1 << args.log2count
    ins, out = B.make_bucket(n, count)
    variants = [dict(engine=1), dict(engine=1, grid=192), dict(engine=1, block=512, unroll=4, grid=512)]
    for shape in ((512, 16), (1024, 4), (512, 8), (1024, 8), (256, 16)):
        for grid in (0, 512):
            variants.append(dict(engine=2, block=shape[0], unroll=shape[1], grid=grid))
    for nt, store in ((1, 1), (1, 2), (2, 1), (2, 3)):
        variants.append(dict(engine=2, nontemporal=nt, store_policy=store))
    probe = None
    pso = os.path.join(ROOT, "tools", "libhbm_probe.so")
    if os.path.exists(pso):
        probe = ctypes.CDLL(pso)
        probe.probe_run.restype = ctypes.c_int
        probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                         ctypes.c_uint64, ctypes.c_void_p]
        tab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for g in (192, 256):
            variants.append(dict(probe=True, block=256, unroll=4, nontemporal=2, store_policy=2, grid=g))

    def runner(v):
        if v.get("probe"):
            return lambda: probe.probe_run(0, 256, 4, 2, 2, 0, v["grid"], tab, n, ctypes.c_void_p(out.data_ptr()),
                                           count * 4, st)
        return lambda: hiccl_amd.reduce(out, ins, config=v)

    res = {i: [] for i in range(len(variants))}
    for rnd in range(3):
        for i, v in enumerate(variants):
            try:
                _, ms = B.time_launches(runner(v), 5, 2)
            except Exception as e:  # unsupported combination
                B.log("skip", v, e)
                continue
            res[i].append(float(np.median(ms)))
        B.log(f"sweep round {rnd} done")
    bytes_step = (n + 1) * count * 4
    rows = []
    for i, v in enumerate(variants):
        if res[i]:
            t = float(np.median(res[i]))
            rows.append((bytes_step / t / 1e6, t, v))
    rows.sort(key=lambda r: -r[0])
    for gbps, t, v in rows:
        print(json.dumps({"GBps": round(gbps, 1), "ms": round(t, 4), "frac": round(gbps / B.HBM_PEAK_GBPS, 4), **v}))
    return 0

def c3_offsets(args):
    """Config 3 with few inputs: does where the inputs sit relative to each
    other move the rate?  n in {2, 3, 4, 8} x 2^26 fp32; input k is a view
    starting k x `off` bytes into a padded allocation (off = 0, 4 KiB,
    64 KiB, 1 MiB + 4 KiB), so element i of every input no longer shares its
    address bits below the offset with the other inputs; AUTO and every
    engine form that leads somewhere, interleaved rounds, one set of
    allocations per n (the same physical pages for every offset)."""
    count = 1 << 26
    offs = (0, 4 << 10, 64 << 10, (1 << 20) + (4 << 10))
    forms = [("auto", None), ("phase", dict(engine=2, schedule=1)), ("tile_u4_static", dict(engine=1, schedule=1))]
    for n in (2, 3, 4, 8):
        pad = (n - 1) * max(offs) // 4 + 64
        raw = [torch.empty(count + pad, device="cuda") for _ in range(n)]
        out = torch.empty(count, device="cuda")
        res = {}
        for rnd in range(args.rounds):
            for off in offs:
                ins = [raw[k][k * off // 4:k * off // 4 + count] for k in range(n)]
                if rnd == 0:
                    for k, t in enumerate(ins):
                        hiccl_amd.fill_uniform(t, B.SEED + off, k)
                for name, cfg in forms:
                    _, ms = B.time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), args.steps, args.warmup)
                    res.setdefault((off, name), []).append(float(np.median(ms)))
                if rnd == 0:
                    torch.cuda.synchronize()
                    res[(off, "ok")] = B.sample_check(out, n, count, seed=B.SEED + off)
        alg = (n + 1) * count * 4
        row = {"mode": "c3offsets", "n": n, "count": count}
        for off in offs:
            row[f"off{off}"] = {name: round(alg / (float(np.median(res[(off, name)])) * 1e-3) / 1e9, 1)
                                for name, _ in forms}
            row[f"off{off}"]["sample_exact"] = res[(off, "ok")]
        print(json.dumps(row), flush=True)
        del raw, out
        torch.cuda.empty_cache()
    return 0

def schedsweep(args):
    """Static vs dynamic unit schedule (and grab size) for both engines,
    fp32, interleaved rounds.  Default cases n = 2/4/8/16 at 256 MiB and
    1 GiB per input; --n N --log2count L: that shape on 3 fresh buckets."""
    cases = ((2, 256), (2, 1024), (4, 256), (4, 1024), (8, 256), (8, 1024), (16, 256))
    if args.buckets:
        cases = ((args.n, (1 << args.log2count) * 4 >> 20),) * args.buckets
    elif args.xmib:
        ns = [int(v) for v in args.xn.split(",")] if args.xn else [args.n]
        cases = tuple((n, int(m)) for n in ns for m in args.xmib.split(","))
    variants = [("tile_static", dict(engine=1, schedule=1)), ("tile_dyn_g1", dict(engine=1, schedule=2, grab=1)),
                ("tile512_dyn_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=4)),
                ("tile_dyn_g2", dict(engine=1, schedule=2, grab=2)),
                ("phase_static", dict(engine=2, schedule=1)), ("phase_dyn_g1", dict(engine=2, schedule=2, grab=1)),
                ("auto", None)]
    if args.sweepset == "occupancy":  # C2-shaped: workgroups per CU / tile shape on the dynamic schedule
        variants = [("auto", None),
                    ("t256x4_bpc2_g1", dict(engine=1, schedule=2, grab=1, blocks_per_cu=2)),
                    ("t256x4_bpc2_g2", dict(engine=1, schedule=2, grab=2, blocks_per_cu=2)),
                    ("t512x2_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=2)),
                    ("t512x2_bpc2_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=2, blocks_per_cu=2)),
                    ("t256x2_bpc2_g2", dict(engine=1, schedule=2, grab=2, unroll=2, blocks_per_cu=2)),
                    ("t256x2_g2", dict(engine=1, schedule=2, grab=2, unroll=2)),
                    ("t256x4_g1_drain", dict(engine=1, schedule=2, grab=1, drain=1))]
    if args.sweepset == "small":  # few tiles per workgroup: more workgroups / smaller tiles
        variants = [("auto", None),
                    ("t256x4_bpc2", dict(engine=1, blocks_per_cu=2)),
                    ("t256x4_bpc4", dict(engine=1, blocks_per_cu=4)),
                    ("t256x2", dict(engine=1, unroll=2)),
                    ("t256x2_bpc2", dict(engine=1, unroll=2, blocks_per_cu=2)),
                    ("t256x1_bpc4", dict(engine=1, unroll=1, blocks_per_cu=4)),
                    ("t256x4_dyn", dict(engine=1, schedule=2, grab=1)),
                    ("phase", dict(engine=2))]
    if args.sweepset == "bf16occ":  # bf16 tile: hide the packed accumulator's VALU time
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_dyn_bpc2", dict(engine=1, schedule=2, blocks_per_cu=2)),
                    ("tile_dyn_bpc2_u2", dict(engine=1, schedule=2, blocks_per_cu=2, unroll=2)),
                    ("tile_dyn_b512u2", dict(engine=1, schedule=2, block=512, unroll=2)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_bpc2", dict(engine=2, schedule=1, blocks_per_cu=2))]
    if args.sweepset == "widetile":  # few inputs: wide TILE tiles (32 packets per lane in flight)
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("tile_u4_static", dict(engine=1, schedule=1)),
                    ("tile_u8_static", dict(engine=1, unroll=8, schedule=1)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u16_static", dict(engine=1, unroll=16, schedule=1)),
                    ("tile_u16_dyn", dict(engine=1, unroll=16, schedule=2, grab=1))]
    if args.sweepset == "widedyn":  # wide tiles on the dynamic schedule vs AUTO, larger buckets
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("tile_u4_dyn", dict(engine=1, unroll=4, schedule=2)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u8_dyn_g2", dict(engine=1, unroll=8, schedule=2, grab=2)),
                    ("tile_u16_dyn", dict(engine=1, unroll=16, schedule=2, grab=1))]
    if args.sweepset == "c3":  # config 3 per n: engine / occupancy / tile size
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_dyn_bpc2", dict(engine=1, schedule=2, blocks_per_cu=2)),
                    ("tile_dyn_u2_bpc2", dict(engine=1, schedule=2, unroll=2, blocks_per_cu=2)),
                    ("tile_static", dict(engine=1, schedule=1)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2))]
    if args.sweepset == "fewn":  # config 3's few-input buckets (n = 2-4): every engine form, interleaved
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2)),
                    ("tile_u4_static", dict(engine=1, schedule=1)),
                    ("tile_u4_dyn", dict(engine=1, schedule=2)),
                    ("tile_u8_static", dict(engine=1, unroll=8, schedule=1)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u4_static_bpc2", dict(engine=1, schedule=1, blocks_per_cu=2))]
    if args.sweepset == "phaseshapes":  # the phased engine's chunk shapes (block x packets per lane)
        variants = [("auto", None),
                    ("p512x16", dict(engine=2, block=512, unroll=16)),
                    ("p1024x8", dict(engine=2, block=1024, unroll=8)),
                    ("p512x8", dict(engine=2, block=512, unroll=8)),
                    ("p1024x4", dict(engine=2, block=1024, unroll=4)),
                    ("p256x16", dict(engine=2, block=256, unroll=16)),
                    ("p256x16_bpc2", dict(engine=2, block=256, unroll=16, blocks_per_cu=2))]
    if args.sweepset == "xover":  # engine x schedule crossover (sets AUTO)
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_static", dict(engine=1, schedule=1)),
                    ("tile_bpc4_static", dict(engine=1, schedule=1, blocks_per_cu=4)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2))]
    for n, mib in cases:
        sdt = {"bf16": torch.bfloat16, "bf16wide": torch.bfloat16, "f64": torch.float64, "u64": torch.int64,
               "i32": torch.int32}.get(args.sweepdtype, torch.float32)
        wide = args.sweepdtype == "bf16wide"  # f32 accumulation (HICCL_ACC_WIDE) in every variant
        esz = torch.tensor([], dtype=sdt).element_size()
        count = (mib << 20) // esz
        ins, out = B.make_bucket(n, count, sdt)
        res = {}
        for rnd in range(5):
            for name, cfg in variants:
                if wide:
                    cfg = dict(cfg or {}, acc=1)
                try:
                    _, ms = B.time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), max(args.steps, 10),
                                          args.warmup)
                except hiccl_amd.HicclError:  # a shape this type does not have (f64 / u64: block 256 only)
                    res[name] = None
                    continue
                res.setdefault(name, []).append(float(np.median(ms)))
        row = {"mode": "schedsweep", "n": n, "mib_per_input": mib}
        for name, v in res.items():
            if v is None:
                row[name] = None
                continue
            t = float(np.median(v)) * 1e-3
            row[name] = round((n + 1) * count * esz / t / 1e9, 1)
        row["dtype"] = str(sdt).split(".")[-1]
        if sdt in (torch.float64, torch.int64, torch.int32):  # in-order sum on the device (f64 adds, wrap-around ints)
            acc = torch.zeros_like(out)
            for t in ins:
                acc = acc + t
            iv = torch.int32 if sdt == torch.int32 else torch.int64
            row["parity_sample_ok"] = bool(torch.equal(acc.view(iv), out.view(iv)))
        elif wide:  # one f32 accumulation, rounded once
            acc = torch.zeros(out.shape, dtype=torch.float32, device=out.device)
            for t in ins:
                acc = acc + t.float()
            row["parity_sample_ok"] = bool(torch.equal(acc.to(torch.bfloat16).view(torch.int16), out.view(torch.int16)))
        else:
            row["parity_sample_ok"] = B.sample_check(out, n, count, bf16=(sdt == torch.bfloat16))
        print(json.dumps(row), flush=True)
        del ins, out
        torch.cuda.empty_cache()
    return 0

def planvs(args):
    """Plan-kernel overhead on the C2 bucket: one-shot launch vs a plan of
    1, 1024 (1 MiB) and 8192 (128 KiB) computes, interleaved rounds."""
    n, count = 8, 1 << 28
    ins, out = B.make_bucket(n, count)
    stream = torch.cuda.current_stream()
    plans = {}
    for name, ncomp, eng in (("plan_1", 1, 0), ("plan_1024", 1024, 0), ("plan_8192", 8192, 0),
                             ("plan_1024_tile", 1024, 1)):
        comp = hiccl_amd.Compute(torch.float32, device=torch.cuda.current_device(), engine=eng)
        off = 0
        for b in range(ncomp):
            c = count // ncomp + (1 if b < count % ncomp else 0)
            comp.add([(t, off) for t in ins], (out, off), c, compid=0)
            off += c
        plans[name] = comp
    runs = {"single": lambda: hiccl_amd.reduce(out, ins)}
    for name, comp in plans.items():
        runs[name] = (lambda c: (lambda: c.start(stream=stream)))(comp)
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, fn in runs.items():
            _, ms = B.time_launches(fn, max(args.steps, 10), args.warmup)
            res[k].append(float(np.median(ms)))
    for k, v in res.items():
        t = float(np.median(v)) * 1e-3
        eng = plans[k].engine() if k in plans else None
        print(json.dumps({"mode": "planvs", "run": k, "engine": eng, "kernel_ms": round(t * 1e3, 4),
                          "GBps": round(9 * count * 4 / t / 1e9, 1)}), flush=True)
    ok = B.sample_check(out, n, count)
    print(json.dumps({"mode": "planvs", "parity_sample_ok": ok}), flush=True)
    for comp in plans.values():
        comp.close()
    return 0

def crossover(args):
    """Engine crossover: one-shot reduce of n = 2/4/8 inputs, 1-512 MiB per
    input, f32 and bf16, TILE vs PHASE (sets the AUTO threshold)."""
    dtypes = {"f32": (torch.float32,), "bf16": (torch.bfloat16,), "f64": (torch.float64,), "u64": (torch.int64,),
              "i32": (torch.int32,), "wide": (torch.float32, torch.float64, torch.int64, torch.int32)}.get(
                  args.xdtype, (torch.float32, torch.bfloat16))
    mibs = [int(m) for m in args.xmib.split(",")] if args.xmib else (1, 4, 16, 32, 64, 128, 256, 512)
    ns = [int(m) for m in args.xn.split(",")] if args.xn else (2, 4, 8)
    for dtype in dtypes:
        esz = torch.tensor([], dtype=dtype).element_size()
        for n in ns:
            for mib in mibs:
                count = (mib << 20) // esz
                ins, out = B.make_bucket(n, count, dtype)
                row = {"mode": "crossover", "dtype": str(dtype).split(".")[-1], "n": n, "mib_per_input": mib}
                for eng, name in ((1, "tile"), (2, "phase"), (0, "auto")):
                    _, ms = B.time_launches(lambda: hiccl_amd.reduce(out, ins, config=dict(engine=eng)),
                                          max(args.steps, 10), args.warmup)
                    t = float(np.median(ms)) * 1e-3
                    row[name + "_GBps"] = round((n + 1) * count * esz / t / 1e9, 1)
                print(json.dumps(row), flush=True)
                del ins, out
                torch.cuda.empty_cache()
    return 0

def stepscale(args):
    """The C5 step's batched reduction (4 computes of n = 2 and one of n = 4,
    2^18 f32 each at scale 1) at scales 1/8 ... 16, one
    plan launch each, queued GPU time per launch (events around 200
    back-to-back launches), interleaved rounds.  A least-squares fit
    t = t0 + bytes / rate over the scales splits a launch into a fixed part
    (dispatch, first-byte latency, drain) and a bandwidth part; at scale 1
    it says how far the step kernel is from its HBM roofline and why."""
    scales = (0.125, 0.25, 0.5, 1, 2, 4, 8, 16)
    base = 1 << 18
    dev = torch.cuda.current_device()
    cases = {}
    keep = []
    for f in scales:
        c = int(base * f)
        bufs = [torch.empty(c, device="cuda") for _ in range(12)]
        for k, t in enumerate(bufs):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        outs = [torch.empty(c, device="cuda") for _ in range(5)]
        comp = hiccl_amd.Compute(torch.float32, device=dev)
        for j in range(4):
            comp.add([bufs[2 * j], bufs[2 * j + 1]], outs[j], c, compid=0)
        comp.add(bufs[8:12], outs[4], c, compid=0)
        keep.append((bufs, outs))
        cases[f] = (comp, 17 * c * 4)  # 12 inputs read + 5 outputs written
    stream = torch.cuda.current_stream()
    res = {f: [] for f in scales}
    for _ in range(5):
        for f in scales:
            comp = cases[f][0]
            res[f].append(B.time_queued(lambda: comp.enqueue(stream), 200, 10) * 1e3)
    xs = np.array([cases[f][1] for f in scales], dtype=np.float64)
    ys = np.array([float(np.median(res[f])) for f in scales])  # us
    A = np.vstack([np.ones_like(xs), xs]).T
    (t0, slope), *_ = np.linalg.lstsq(A, ys, rcond=None)
    rate_GBps = (1.0 / slope) * 1e6 / 1e9  # slope: us per byte
    rows = [{"scale": f, "algorithmic_bytes": int(cases[f][1]), "queued_us": round(float(y), 3),
             "GBps": round(cases[f][1] / y * 1e6 / 1e9, 1), "fit_us": round(float(t0 + slope * cases[f][1]), 3),
             "engine": cases[f][0].engine()}
            for f, y in zip(scales, ys)]
    # the same launches with the engine / occupancy pinned (what AUTO chose
    # against the alternatives, per scale)
    variants = {"tile": dict(engine=1), "tile_bpc2": dict(engine=1, blocks_per_cu=2),
                "tile_bpc4": dict(engine=1, blocks_per_cu=4), "phase": dict(engine=2)}
    for name, cfg in variants.items():
        vt = {f: [] for f in scales}
        for _ in range(3):
            for f in scales:
                comp = cases[f][0]
                comp.set_config(cfg)
                vt[f].append(B.time_queued(lambda: comp.enqueue(stream), 200, 10) * 1e3)
        for r, f in zip(rows, scales):
            r[name + "_us"] = round(float(np.median(vt[f])), 3)
    for f in scales:
        cases[f][0].set_config({})
    ok = True
    for f in scales:
        bufs, outs = keep[scales.index(f)]
        ref = torch.empty_like(outs[0])
        hiccl_amd.reduce(ref, [bufs[0], bufs[1]])
        ok = ok and torch.equal(ref.view(torch.int32), outs[0].view(torch.int32))
    torch.cuda.synchronize()
    # the kernel boundary alone: one 64-lane wave per launch (hiccl_counter_add),
    # back to back on the same stream
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    lib = L.lib()
    st = ctypes.c_void_p(stream.cuda_stream)
    empty = [B.time_queued(lambda: lib.hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1, st), 200, 10) * 1e3
             for _ in range(5)]
    # the same 200 launches, and 200 C5-step plan launches (scale 1, static
    # schedule inside a capture), as ONE hipGraph replay: the boundary
    # between graph nodes
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    comp1 = cases[1][0]
    comp1.enqueue(stream)  # re-uploads after the variants' set_config (an upload cannot be captured)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        cs = torch.cuda.current_stream()
        with torch.cuda.graph(g1, stream=cs):
            for _ in range(200):
                lib.hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1, ctypes.c_void_p(cs.cuda_stream))
        with torch.cuda.graph(g2, stream=cs):
            for _ in range(200):
                comp1.enqueue(cs)
    graph_us = {}
    for name, g in (("one_wave_kernel_graph_us", g1), ("scale1_graph_us", g2)):
        v = []
        for _ in range(5):
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            v.append(a.elapsed_time(b) * 1e3 / 200)
        graph_us[name] = round(float(np.median(v)), 3)
    del g1, g2
    one = rows[scales.index(1)]
    print(json.dumps({"mode": "stepscale", "shape": "4 x (n=2) + 1 x (n=4) computes of scale x 2^18 f32, one plan launch",
                      "rows": rows, "fit_fixed_us": round(float(t0), 3), "fit_rate_GBps": round(rate_GBps, 1),
                      "scale1_fixed_share": round(float(t0) / one["queued_us"], 3),
                      "scale1_frac_of_8TBps": round(one["GBps"] / 8000.0, 3),
                      "one_wave_kernel_us": round(float(np.median(empty)), 3), **graph_us,
                      "bits_ok": bool(ok)}), flush=True)
    for comp, _ in cases.values():
        comp.close()
    return 0

def c2variants(args):
    """Config 2 variants: the README's count 1e9/sizeof(T)
    = 2.5e8 (tail handling), and the 2^28 bucket with every input shifted by
    1-3 elements and the output by 0 or 1 (the mutual misalignment partition()
    produces)."""
    n = 8
    cases = [("readme_count", 250_000_000, [0] * n, 0),
             ("inputs_shifted", 1 << 28, [1 + k % 3 for k in range(n)], 0),
             ("inputs_and_output_shifted", 1 << 28, [1 + k % 3 for k in range(n)], 1),
             ("inputs_common_shift", 1 << 28, [1] * n, 0),
             ("output_shifted", 1 << 28, [0] * n, 1)]
    for name, count, in_off, out_off in cases:
        bases = [torch.empty(count + 4, dtype=torch.float32, device="cuda") for _ in range(n)]
        ins = [b[o:o + count] for b, o in zip(bases, in_off)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, B.SEED, k)
        obase = torch.empty(count + 4, dtype=torch.float32, device="cuda")
        out = obase[out_off:out_off + count]
        torch.cuda.synchronize()
        out.fill_(float("nan"))
        _, ms = B.time_launches(lambda: hiccl_amd.reduce(out, ins), args.steps, args.warmup)
        t = float(np.median(ms)) * 1e-3
        b = (n + 1) * count * 4
        print(json.dumps({"config": "C2", "variant": name, "count": count, "input_offsets": in_off,
                          "output_offset": out_off, "parity_sample_ok": B.sample_check(out, n, count),
                          "kernel_ms": round(t * 1e3, 4), "GBps": round(b / t / 1e9, 1),
                          "frac_hbm": round(b / t / 1e9 / B.HBM_PEAK_GBPS, 4)}), flush=True)
        del bases, ins, obase, out
        torch.cuda.empty_cache()
    return 0

MODES = {"sweep": sweep, "c3offsets": c3_offsets, "schedsweep": schedsweep, "planvs": planvs,
         "crossover": crossover, "stepscale": stepscale, "c2variants": c2variants}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", required=True, choices=sorted(MODES))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--log2count", type=int, default=28)
    ap.add_argument("--engine", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweepdtype", default="f32", help="schedsweep: f32 | bf16 | bf16wide | f64 | u64 | i32")
    ap.add_argument("--sweepset", default="", help="schedsweep: '' | occupancy | small | bf16occ | widetile | "
                                                   "widedyn | c3 | fewn | phaseshapes | xover")
    ap.add_argument("--xdtype", default="both", help="crossover: f32 | bf16 | both | f64 | u64 | i32 | wide")
    ap.add_argument("--xmib", default="", help="crossover / schedsweep: comma list of MiB per input")
    ap.add_argument("--xn", default="", help="crossover / schedsweep: comma list of input counts")
    ap.add_argument("--buckets", type=int, default=0, help="schedsweep: this many fresh --n x 2^--log2count buckets")
    args = ap.parse_args()
    return MODES[args.mode](args)


if __name__ == "__main__":
    sys.exit(main())
