#!/usr/bin/env python3
"""Batched-plan kernel (k_reduce_plan) on the shapes Comm<T> runs per step.

  (a) C4 at 16 MiB per input: n = 8, 16 computes of 1 MiB, f32 and bf16
  (b) C4 bf16 at 1 GiB per input: n = 8, 1024 computes of 1 MiB, against the
      one-shot launch of the same bucket (interleaved)
  (d) C4 f32 at 4 GiB per input: n = 8, 4096 computes of 1 MiB (byte
      offsets past 2^32 inside one batched plan), against the one-shot
      launch of the same bucket (interleaved)
  (c) a C5-shaped step: four n = 2 and one n = 4 computes of 2^18 f32
      (collectives/main.cpp:151-155 with {1,4,2}, 1 GiB per rank,
      pipedepth 128: reduce.h:134-170 emission per batch)

Per shape: per-launch HIP-event time (median) and the queued time (one event
pair around back-to-back launches), algorithmic GB/s (n + 1) * count * esz,
and a sampled bitwise check against the oracle generator.  --sweep adds
plan configurations (hiccl_reduce_plan_set_config) interleaved with the
default.  Run under rocprofv3 for kernel durations (tools/profile_plans.sh).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hiccl_amd  # noqa: E402
import bench  # noqa: E402

SEED = 1234
MIB = 1 << 20


def partitioned_plan(dtype, n, count, depth, config=None, engine=0):
    ins, out = bench.make_bucket(n, count, dtype)
    comp = hiccl_amd.Compute(dtype, device=torch.cuda.current_device(), engine=engine, config=config)
    off = 0
    for b in range(depth):  # reduce.h:401-415 partition()
        c = count // depth + (1 if b < count % depth else 0)
        comp.add([(t, off) for t in ins], (out, off), c, compid=0)
        off += c
    return comp, ins, out


def c5_step(config=None):
    """Four 2-input and one 4-input computes of 2^18 floats: inputs are the
    rank's send buffer chunk and freshly allocated receive buffers."""
    count = 1 << 18
    comp = hiccl_amd.Compute(torch.float32, device=torch.cuda.current_device(), config=config)
    keep = []
    k = 0
    outs = []
    for n in (2, 2, 2, 2, 4):
        ins = []
        for _ in range(n):
            t = torch.empty(count, device="cuda")
            hiccl_amd.fill_uniform(t, SEED, k)
            k += 1
            ins.append(t)
        out = torch.empty(count, device="cuda")
        comp.add(ins, out, count, compid=0)
        keep += ins
        outs.append((out, n, k - n))
    torch.cuda.synchronize()
    return comp, keep, outs


def timeit(fn, steps, warmup):
    _, ms = bench.time_launches(fn, steps, warmup)
    q = bench.time_queued(fn, max(steps, 20), 2)
    return float(np.median(ms)), q


def run_shape(name, comp, nbytes, steps, warmup, rounds, variants, stream):
    res = {}
    for _ in range(rounds):
        for vname, c in variants:
            _, ms = bench.time_launches(lambda: c.start(stream=stream), steps, warmup)
            q = bench.time_queued(lambda: c.start(stream=stream), max(steps, 20), 2)
            r = res.setdefault(vname, {"ev": [], "q": []})
            r["ev"].append(float(np.median(ms)))
            r["q"].append(q)
    for vname, c in variants:
        ev, q = float(np.median(res[vname]["ev"])), float(np.median(res[vname]["q"]))
        print(json.dumps({"shape": name, "variant": vname, "engine": c.engine(), "bytes": nbytes,
                          "event_us": round(ev * 1e3, 2), "queued_us": round(q * 1e3, 2),
                          "event_GBps": round(nbytes / ev / 1e6, 1), "queued_GBps": round(nbytes / q / 1e6, 1)}),
              flush=True)


SWEEP = [("t_u4_bpc1", dict(engine=1, unroll=4, blocks_per_cu=1)),
         ("t_u4_bpc2", dict(engine=1, unroll=4, blocks_per_cu=2)),
         ("t_u4_bpc3", dict(engine=1, unroll=4, blocks_per_cu=3)),
         ("t_u4_bpc4", dict(engine=1, unroll=4, blocks_per_cu=4)),
         ("t_u2_bpc2", dict(engine=1, unroll=2, blocks_per_cu=2)),
         ("t_u2_bpc4", dict(engine=1, unroll=2, blocks_per_cu=4)),
         ("t_u2_bpc6", dict(engine=1, unroll=2, blocks_per_cu=6)),
         ("t_u1_bpc4", dict(engine=1, unroll=1, blocks_per_cu=4)),
         ("t_u1_bpc8", dict(engine=1, unroll=1, blocks_per_cu=8)),
         ("phase", dict(engine=2))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="a,b,c")
    ap.add_argument("--sweep", action="store_true")
    args = ap.parse_args()
    stream = torch.cuda.current_stream()
    shapes = args.shapes.split(",")

    def variants_for(make):
        v = [("auto", make(None))]
        if args.sweep:
            v += [(k, make(cfg)) for k, cfg in SWEEP]
        return v

    if "launch" in shapes:
        # launch overhead on the 16 MiB shape: plan launch (+ completion event),
        # plan enqueue (no event), the one-shot launch, a 1-compute plan
        count = 16 * MIB // 4
        comp, ins, out = partitioned_plan(torch.float32, 8, count, 16)
        one, _, _ = partitioned_plan(torch.float32, 8, count, 1)
        runs = {"plan16_launch": lambda: comp.start(stream=stream), "plan16_enqueue": lambda: comp.enqueue(stream),
                "plan1_enqueue": lambda: one.enqueue(stream), "oneshot": lambda: hiccl_amd.reduce(out, ins),
                "plan16_launch_sync": lambda: (comp.start(stream=stream), comp.wait())}
        res = {}
        for _ in range(args.rounds):
            for k, fn in runs.items():
                ev, q = timeit(fn, args.steps, args.warmup)
                res.setdefault(k, []).append((ev, q))
        for k, v in res.items():
            ev, q = float(np.median([x[0] for x in v])), float(np.median([x[1] for x in v]))
            print(json.dumps({"shape": "launch_16MiB_f32", "variant": k, "event_us": round(ev * 1e3, 2),
                              "queued_us": round(q * 1e3, 2), "queued_GBps": round(9 * count * 4 / q / 1e6, 1)}),
                  flush=True)
        comp.close()
        one.close()
    if "a" in shapes:
        for dtype, dn in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            esz = 2 if dtype == torch.bfloat16 else 4
            count = 16 * MIB // esz
            made = {}

            def make(cfg, dtype=dtype, count=count):
                comp, ins, out = partitioned_plan(dtype, 8, count, 16, cfg)
                made.setdefault("bufs", []).append((ins, out))
                return comp
            vs = variants_for(make)
            run_shape(f"a_C4_{dn}_16MiB_x16", vs[0][1], 9 * count * esz, args.steps, args.warmup, args.rounds, vs,
                      stream)
            ok = [bench.sample_check(out, 8, count, bf16=(dtype == torch.bfloat16)) for ins, out in made["bufs"]]
            print(json.dumps({"shape": f"a_C4_{dn}_16MiB_x16", "parity_sample_ok": all(ok)}), flush=True)
            for _, c in vs:
                c.close()
            del made
            torch.cuda.empty_cache()
    if "b" in shapes:
        count = 1024 * MIB // 2
        comp, ins, out = partitioned_plan(torch.bfloat16, 8, count, 1024)
        vs = [("plan_1024", comp)]
        if args.sweep:
            for k, cfg in (("plan_1024_tile_dyn", dict(engine=1, schedule=2)), ("plan_1024_phase", dict(engine=2))):
                c = hiccl_amd.Compute(torch.bfloat16, device=torch.cuda.current_device(), config=cfg)
                off = 0
                for b in range(1024):
                    cc = count // 1024 + (1 if b < count % 1024 else 0)
                    c.add([(t, off) for t in ins], (out, off), cc, compid=0)
                    off += cc
                vs.append((k, c))
        nbytes = 9 * count * 2
        res = {}
        for _ in range(args.rounds):
            for vname, c in vs:
                _, ms = bench.time_launches(lambda: c.start(stream=stream), args.steps, args.warmup)
                res.setdefault(vname, []).append(float(np.median(ms)))
            _, ms = bench.time_launches(lambda: hiccl_amd.reduce(out, ins), args.steps, args.warmup)
            res.setdefault("oneshot", []).append(float(np.median(ms)))
        for vname, v in res.items():
            t = float(np.median(v))
            eng = dict(vs).get(vname)
            print(json.dumps({"shape": "b_C4_bf16_1GiB_x1024", "variant": vname,
                              "engine": eng.engine() if eng else None, "event_us": round(t * 1e3, 1),
                              "event_GBps": round(nbytes / t / 1e6, 1)}), flush=True)
        print(json.dumps({"shape": "b_C4_bf16_1GiB_x1024",
                          "parity_sample_ok": bench.sample_check(out, 8, count, bf16=True)}), flush=True)
        for _, c in vs:
            c.close()
        del ins, out
        torch.cuda.empty_cache()
    if "d" in shapes:
        count = 4096 * MIB // 4
        comp, ins, out = partitioned_plan(torch.float32, 8, count, 4096)
        nbytes = 9 * count * 4
        res = {}
        for _ in range(args.rounds):
            _, ms = bench.time_launches(lambda: comp.start(stream=stream), args.steps, args.warmup)
            res.setdefault("plan_4096", []).append(float(np.median(ms)))
            _, ms = bench.time_launches(lambda: hiccl_amd.reduce(out, ins), args.steps, args.warmup)
            res.setdefault("oneshot", []).append(float(np.median(ms)))
        comp.start(stream=stream)
        torch.cuda.synchronize()
        for vname, v in res.items():
            t = float(np.median(v))
            print(json.dumps({"shape": "d_C4_f32_4GiB_x4096", "variant": vname,
                              "engine": comp.engine() if vname.startswith("plan") else None,
                              "event_us": round(t * 1e3, 1), "event_GBps": round(nbytes / t / 1e6, 1)}), flush=True)
        print(json.dumps({"shape": "d_C4_f32_4GiB_x4096",
                          "parity_sample_ok": bench.sample_check(out, 8, count)}), flush=True)
        comp.close()
        del ins, out
        torch.cuda.empty_cache()
    if "c" in shapes:
        made = []

        def make(cfg):
            comp, keep, outs = c5_step(cfg)
            made.append((keep, outs))
            return comp
        vs = variants_for(make)
        nbytes = (4 * 3 + 5) * (1 << 18) * 4
        run_shape("c_C5_step_4x2_1x4_2^18", vs[0][1], nbytes, args.steps, args.warmup, args.rounds, vs, stream)
        ok = True
        for keep, outs in made:
            for out, n, k0 in outs:
                idx = np.random.default_rng(n).integers(0, 1 << 18, 512).astype(np.uint64)
                # inputs k0..k0+n-1 of the generator: shift the key by summing by hand
                got = out[torch.from_numpy(idx.astype(np.int64)).cuda()].cpu().numpy()
                exp = np.zeros(len(idx), np.float32)  # in-order f32 sum on the host (compute.h:14-23)
                for j in range(n):
                    t = keep[k0 + j][torch.from_numpy(idx.astype(np.int64)).cuda()].cpu().numpy()
                    exp = (exp + t).astype(np.float32)
                ok = ok and bool(np.array_equal(got.view(np.uint32), exp.view(np.uint32)))
        print(json.dumps({"shape": "c_C5_step_4x2_1x4_2^18", "parity_sample_ok": ok}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
