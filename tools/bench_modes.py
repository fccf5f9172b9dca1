#!/usr/bin/env python3
"""bench.py's secondary modes (configs 3 and 4, the host-memory round trip,
the C5 pipeline step, config 3 against config 2 on one box), dispatched from
bench.py (`--nway`, `--chunks`, `--roundtrip`, `--c3vsc2`, `--progstep`).
They share bench.py's buckets, timers and ceilings (imported as `B`) and
print one JSON line per case; the driver's line is bench.py's default run.
"""
import ctypes
import json
import os

import numpy as np
import torch

import bench as B
import hiccl_amd
from hiccl_amd import _lib as L

def nway(args):
    """Config 3: N in 2..64 inputs x 2^26 fp32 (256 MiB each)."""
    count = 1 << 26
    copy_gbps = B.copy_ceiling()
    for n in (2, 3, 4, 8, 16, 32, 64):
      ins, out = B.make_bucket(n, count)
      # the box's bound for this read/write mix on these very buckets
      read_gbps = B.mix_ceiling(ins, out, count, mode=1)
      write_gbps = B.mix_ceiling(ins, out, count, mode=2)
      for eng in (0, 1):  # auto (= phase at this size), tile
        cfg = dict(engine=eng) if eng else None
        _, ms = B.time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), args.steps, args.warmup)
        t = float(np.median(ms)) * 1e-3
        b = (n + 1) * count * 4
        print(json.dumps({"config": "C3", "engine": ["auto", "tile"][eng], "n": n, "count": count,
                          "kernel_ms": round(t * 1e3, 4),
                          "GBps": round(b / t / 1e9, 1), "frac_hbm": round(b / t / 1e9 / B.HBM_PEAK_GBPS, 4),
                          "read_GBps": round(n * count * 4 / t / 1e9, 1),
                          "frac_of_copy": round(b / t / 1e9 / copy_gbps, 4),
                          "serial_rw_model": B.serial_rw_model(n * count * 4, count * 4, read_gbps, copy_gbps, t, write_gbps)}),
              flush=True)
      del ins, out
      torch.cuda.empty_cache()
    return 0

def c3_vs_c2(args):
    """Config 3 per n on ONE box with config 2 as the control: C2 (8 x 2^28)
    and C3 n in {2, 3, 4, 8, 16, 32, 64} x 2^26 fp32, every bucket allocated
    once, then `--rounds` interleaved rounds (C2, then each n, `--steps`
    launches each, AUTO).  Per n: GB/s (median over rounds of the per-round
    median kernel time), its ratio to the same round's C2, and the serial
    read/write model on its own buckets (the box's read-only and write-only
    probe rates: R / read + W / write, roofline.serial_rw_model) -- so a
    gap between n is either the box's HBM bound for that n's buckets or
    named.  One JSON line per bucket, then a summary line."""
    sizes = [("C2", 8, 1 << 28)] + [("C3", n, 1 << 26) for n in (2, 3, 4, 8, 16, 32, 64)]
    copy_gbps = B.copy_ceiling()
    buckets = []
    for cfg, n, count in sizes:
        ins, out = B.make_bucket(n, count, seed=B.SEED + 17 * n + (count >> 26))
        read = B.mix_ceiling(ins, out, count, mode=1)
        write = B.mix_ceiling(ins, out, count, mode=2)
        buckets.append({"config": cfg, "n": n, "count": count, "ins": ins, "out": out, "read": read, "write": write,
                        "ms": []})
        B.log(f"c3vsc2: {cfg} n={n} allocated, probes read {read} write {write} GB/s")
    for rnd in range(args.rounds):
        for b in buckets:
            _, ms = B.time_launches(lambda: hiccl_amd.reduce(b["out"], b["ins"]), args.steps, args.warmup)
            b["ms"].append(float(np.median(ms)))
        B.log(f"c3vsc2: round {rnd} done")
    c2 = buckets[0]
    c2_rates = [(c2["n"] + 1) * c2["count"] * 4 / (t * 1e-3) / 1e9 for t in c2["ms"]]
    rows = []
    for b in buckets:
        n, count = b["n"], b["count"]
        alg = (n + 1) * count * 4
        rates = [alg / (t * 1e-3) / 1e9 for t in b["ms"]]
        t = float(np.median(b["ms"])) * 1e-3
        ok = B.sample_check(b["out"], n, count, seed=B.SEED + 17 * n + (count >> 26))
        row = {"config": b["config"], "n": n, "count": count, "kernel_ms": round(t * 1e3, 4),
               "GBps": round(alg / t / 1e9, 1), "frac_hbm": round(alg / t / 1e9 / B.HBM_PEAK_GBPS, 4),
               "GBps_per_round": [round(r, 1) for r in rates],
               "ratio_to_c2": round(float(np.median([r / c for r, c in zip(rates, c2_rates)])), 4),
               "read_probe_GBps": round(b["read"], 1) if b["read"] else None,
               "write_probe_GBps": round(b["write"], 1) if b["write"] else None,
               "serial_rw_model": B.serial_rw_model(n * count * 4, count * 4, b["read"], copy_gbps, t, b["write"]),
               "sample_exact": ok}
        rows.append(row)
        print(json.dumps(row), flush=True)
    c3 = [r for r in rows if r["config"] == "C3"]
    print(json.dumps({"summary": "c3_vs_c2", "rounds": args.rounds, "steps": args.steps, "copy_GBps": round(copy_gbps, 1),
                      "c2_GBps": rows[0]["GBps"], "c2_model_frac": (rows[0]["serial_rw_model"] or {}).get("frac_write_probe"),
                      "c3_ratio_to_c2": {r["n"]: r["ratio_to_c2"] for r in c3},
                      "c3_model_frac": {r["n"]: (r["serial_rw_model"] or {}).get("frac_write_probe") for r in c3},
                      "device": torch.cuda.get_device_properties(0).name}), flush=True)
    return 0

def chunks(args):
    """Config 4: fp32/bf16, 16 MiB..4 GiB per input, split into 1 MiB computes
    (pipedepth = bytes / 1 MiB, reduce.h:406 split), batched plan launch vs
    one launch per compute (the reference structure, compute.h:88-91)."""
    n = 8
    for dtype in (torch.float32, torch.bfloat16):
        esz = torch.tensor([], dtype=dtype).element_size()
        for mib in (16, 64, 256, 1024, 4096):
            count = (mib << 20) // esz
            free, _ = torch.cuda.mem_get_info()
            if (n + 1) * count * esz * 1.05 > free:
                B.log(f"chunks: skip {mib} MiB ({dtype}): not enough memory")
                continue
            ins, out = B.make_bucket(n, count, dtype)
            depth = max(1, (mib << 20) // (1 << 20))
            comp = hiccl_amd.Compute(dtype, device=torch.cuda.current_device(), engine=args.engine)
            off = 0
            for b in range(depth):  # partition(): count/numbatch + (b < count%numbatch)
                c = count // depth + (1 if b < count % depth else 0)
                comp.add([(t, off) for t in ins], (out, off), c, compid=0)
                off += c
            stream = torch.cuda.current_stream()
            res, queued = {}, {}
            for mode in ("batched", "each"):
                launch = (lambda m=mode: comp.start(stream=stream, each=(m == "each")))
                _, ms = B.time_launches(launch, args.steps, args.warmup)
                res[mode] = float(np.median(ms)) * 1e-3
                queued[mode] = B.time_queued(launch, max(args.steps, 20), 2) * 1e-3
            b = (n + 1) * count * esz
            ok = B.sample_check(out, n, count, bf16=(dtype == torch.bfloat16))
            print(json.dumps({"config": "C4", "dtype": str(dtype).split(".")[-1], "mib_per_input": mib,
                              "parity_sample_ok": ok, "engine": comp.engine(),
                              "computes": depth, "batched_ms": round(res["batched"] * 1e3, 4),
                              "batched_GBps": round(b / res["batched"] / 1e9, 1),
                              "each_ms": round(res["each"] * 1e3, 4),
                              "each_GBps": round(b / res["each"] / 1e9, 1),
                              "queued_batched_GBps": round(b / queued["batched"] / 1e9, 1),
                              "queued_each_GBps": round(b / queued["each"] / 1e9, 1)}), flush=True)
            comp.close()
            del ins, out
            torch.cuda.empty_cache()
    return 0

def host_sum(host_in):
    """In-order fp32 sum on the host (torch adds two tensors element-wise in
    fp32 with round-to-nearest: the reference's acc += in[k][i] order)."""
    exp = torch.zeros_like(host_in[0])
    for h in host_in:
        exp = exp + h
    return exp

def roundtrip(args):
    """Inputs and output in pinned host memory: H2D of N inputs + kernel + D2H
    (serial, and chunk-pipelined over 3 streams)."""
    n, count = args.n, 1 << args.log2count
    host_in = [torch.empty(count, dtype=torch.float32).pin_memory() for _ in range(n)]
    for k, h in enumerate(host_in):
        h.copy_(torch.from_numpy(np.random.default_rng(k).uniform(-1, 1, count).astype(np.float32)))
    host_out = torch.empty(count, dtype=torch.float32).pin_memory()
    dev_in = [torch.empty(count, device="cuda") for _ in range(n)]
    dev_out = torch.empty(count, device="cuda")

    def serial():
        for h, d in zip(host_in, dev_in):
            d.copy_(h, non_blocking=True)
        hiccl_amd.reduce(dev_out, dev_in)
        host_out.copy_(dev_out, non_blocking=True)

    nchunk = 16
    streams = [torch.cuda.Stream() for _ in range(3)]
    csz = count // nchunk

    def pipelined():
        cur = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(cur)
        for c in range(nchunk):
            s = streams[c % 3]
            lo = c * csz
            hi = count if c == nchunk - 1 else lo + csz
            with torch.cuda.stream(s):
                for h, d in zip(host_in, dev_in):
                    d[lo:hi].copy_(h[lo:hi], non_blocking=True)
                hiccl_amd.reduce(dev_out[lo:], [d[lo:] for d in dev_in], count=hi - lo, stream=s)
                host_out[lo:hi].copy_(dev_out[lo:hi], non_blocking=True)
        for s in streams:
            cur.wait_stream(s)

    pipes = {f"host_pipe_{mib}MiB_d{d}": hiccl_amd.HostPipe(torch.float32, chunk_bytes=mib << 20, depth=d)
             for mib, d in ((64, 3), (32, 4), (128, 2))}
    legs = [("serial", serial), ("pipelined", pipelined)]
    expect = host_sum(host_in)
    legs += [(k, (lambda p=p: p.reduce(host_out, host_in))) for k, p in pipes.items()]
    # the store form each leg's reduction launches take (hiccl_reduce_auto_choice_ex:
    # write-through by size up to 256 MiB written per launch, else nt)
    launch_count = {"serial": count, "pipelined": csz,
                    **{k: p_mib << 20 >> 2 for k, p_mib in zip(pipes, (64, 32, 128))}}
    form = {k: {2: "nt", 4: "write-through"}[hiccl_amd.auto_choice(torch.float32, c, n)["store_policy"]]
            for k, c in launch_count.items()}
    out = {}
    for name, fn in legs:
        host_out.zero_()
        wall, _ = B.time_launches(fn, 5, 2)
        t = wall / 5
        out[name] = {"s": round(t, 4), "GBps_alg": round((n + 1) * count * 4 / t / 1e9, 2),
                     "elements_per_launch": launch_count[name], "store_form": form[name]}
        if name.startswith("host_pipe"):
            out[name]["parity_ok"] = bool(torch.equal(host_out.view(torch.int32), expect.view(torch.int32)))
    for p in pipes.values():
        p.close()
    # device-only reference, and the link alone: the n inputs H2D, the output D2H
    _, ms = B.time_launches(lambda: hiccl_amd.reduce(dev_out, dev_in), 10, 3)
    out["kernel_only_GBps"] = round((n + 1) * count * 4 / (np.median(ms) * 1e-3) / 1e9, 1)
    wall, _ = B.time_launches(lambda: [d.copy_(h, non_blocking=True) for h, d in zip(host_in, dev_in)], 3, 1)
    out["h2d_only_GBps"] = round(n * count * 4 * 3 / wall / 1e9, 2)
    wall, _ = B.time_launches(lambda: host_out.copy_(dev_out, non_blocking=True), 3, 1)
    out["d2h_only_GBps"] = round(count * 4 * 3 / wall / 1e9, 2)
    pipelined()
    torch.cuda.synchronize()
    exp = expect
    out["parity_ok"] = bool(torch.equal(exp.view(torch.int32), host_out.view(torch.int32)))
    print(json.dumps({"mode": "roundtrip", "n": n, "count": count, **out,
                      "pcie_bytes": (n + 1) * count * 4}), flush=True)
    return 0

def progstep(args):
    """One C5 pipeline step on one GPU, without peers: the step's enqueue
    sequence -- a ready phase, the transport's copies (five 1 MiB byte
    copies), a done phase, the reductions (4 x n=2 + 1 x n=4 computes of
    2^18 f32, the {1,4,2} step shape), a tail phase --
    as separate launches (k_sigwait_phases + plan kernels: 5 kernels, the
    round-2 stream-ordered path) and as programs (each phase folded into the
    launch of the batch after it: 2 kernels + the tail phase, which in a
    pipeline folds into the next step's first program); queued GPU time per
    step (events around 200 back-to-back steps), interleaved rounds.  The
    phases signal and await this process's own flags (always satisfied)."""
    c = 1 << 18
    dev = torch.cuda.current_device()
    bufs = [torch.empty(c, device="cuda") for _ in range(12)]
    for k, t in enumerate(bufs):
        hiccl_amd.fill_uniform(t, B.SEED, k)
    outs = [torch.empty(c, device="cuda") for _ in range(5)]
    comp = hiccl_amd.Compute(torch.float32, device=dev)
    for j in range(4):
        comp.add([bufs[2 * j], bufs[2 * j + 1]], outs[j], c, compid=0)
    comp.add(bufs[8:12], outs[4], c, compid=0)
    src = [torch.empty(c, device="cuda") for _ in range(5)]
    dst = [torch.empty(c, device="cuda") for _ in range(5)]
    cp = hiccl_amd.Compute(torch.uint8, device=dev)
    for a, b in zip(src, dst):
        cp.add([a.view(torch.uint8)], b.view(torch.uint8), c * 4, compid=0)
    flags = torch.zeros(16, dtype=torch.int32, device="cuda")
    f = [flags.data_ptr() + 4 * i for i in range(3)]
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    st = ctypes.c_void_p(stream.cuda_stream)
    lib = L.lib()
    epoch = [0]

    def phase(flag, e):
        tab = (ctypes.c_void_p * 1)(flag)
        L.check(lib.hiccl_signal_wait(tab, 1, tab, 1, e, ctypes.c_void_p(err.data_ptr()), 10.0, st), "signal_wait")

    def separate():
        epoch[0] += 1
        phase(f[0], epoch[0])
        cp.enqueue(stream)
        phase(f[1], epoch[0])
        comp.enqueue(stream)
        phase(f[2], epoch[0])

    def build(phase_flag, plan):
        pr = hiccl_amd.Program(torch.float32, device=dev)
        if phase_flag is not None:
            pr.add_signal([phase_flag], [phase_flag])
        if plan is not None:
            pr.add_plan(plan)
        return pr

    p_copy, p_comp, p_tail = build(f[0], cp), build(f[1], comp), build(f[2], None)

    def program():
        epoch[0] += 1
        for pr in (p_copy, p_comp, p_tail):
            pr.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)

    def program_tail_folded():  # the tail phase rides in the next step's first program, as in a pipeline
        epoch[0] += 1
        p_copy.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)
        p_comp.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)

    def tokens(mode, fn):  # run fn with the token protocol `mode` (HICCL_PROG_FENCES, read at each launch)
        def run():
            os.environ["HICCL_PROG_FENCES"] = mode
            try:
                fn()
            finally:
                os.environ.pop("HICCL_PROG_FENCES", None)
        return run

    def separate_nophase():
        cp.enqueue(stream)
        comp.enqueue(stream)

    q_copy, q_comp = build(None, cp), build(None, comp)

    def program_nophase():
        q_copy.launch(stream=stream)
        q_comp.launch(stream=stream)

    # unsuffixed: the library's default token protocol (fenced); _light:
    # HICCL_PROG_FENCES=light
    runs = {"separate": separate, "separate_light": tokens("light", separate), "program": program,
            "program_tail_folded": program_tail_folded,
            "program_tail_folded_light": tokens("light", program_tail_folded),
            "separate_no_phases": separate_nophase, "program_no_phases": program_nophase}
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(B.time_queued(fn, 200, 10) * 1e3)
    # The same steps captured into one hipGraph of 200 steps and replayed, as
    # HICCL_GRAPH=1 runs a pipeline: every phase's epoch is e + *ctr, ctr
    # bumped by the graph's first node (a kernel boundary between graph
    # nodes costs less than between eager launches: tools/archive/bench_probes.py --mode stepscale).
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    cptr = ctypes.c_void_p(ctr.data_ptr())
    erp = ctypes.c_void_p(err.data_ptr())

    def phase_dev(flag, e, s_):
        tab = (ctypes.c_void_p * 1)(flag)
        L.check(lib.hiccl_signal_wait_dev(tab, 1, tab, 1, e, cptr, erp, 10.0, s_), "signal_wait_dev")

    side = torch.cuda.Stream()
    graphs = {}
    for name in ("separate_graph", "separate_light_graph", "program_tail_folded_graph",
                 "program_tail_folded_light_graph", "separate_no_phases_graph", "program_no_phases_graph"):
        if "_light" in name:
            os.environ["HICCL_PROG_FENCES"] = "light"  # read at each launch: the capture keeps it
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            cs = torch.cuda.current_stream()
            s_ = ctypes.c_void_p(cs.cuda_stream)
            with torch.cuda.graph(g, stream=cs):
                L.check(lib.hiccl_counter_add(cptr, 1, s_), "counter_add")
                for i in range(200):
                    e = 1000 + i
                    if name in ("separate_graph", "separate_light_graph"):
                        phase_dev(f[0], e, s_)
                        cp.enqueue(cs)
                        phase_dev(f[1], e, s_)
                        comp.enqueue(cs)
                        phase_dev(f[2], e, s_)
                    elif name in ("program_tail_folded_graph", "program_tail_folded_light_graph"):
                        p_copy.launch([e], epoch_dev=ctr.data_ptr(), err=err.data_ptr(), timeout_s=10.0, stream=cs)
                        p_comp.launch([e], epoch_dev=ctr.data_ptr(), err=err.data_ptr(), timeout_s=10.0, stream=cs)
                    elif name == "separate_no_phases_graph":
                        cp.enqueue(cs)
                        comp.enqueue(cs)
                    else:
                        q_copy.launch(stream=cs)
                        q_comp.launch(stream=cs)
        graphs[name] = g
        os.environ.pop("HICCL_PROG_FENCES", None)
    for name, g in graphs.items():
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
        res[name] = v
    del graphs
    ref = torch.empty(c, device="cuda")
    ok = True
    for j in range(4):
        hiccl_amd.reduce(ref, [bufs[2 * j], bufs[2 * j + 1]])
        ok = ok and torch.equal(ref.view(torch.int32), outs[j].view(torch.int32))
    hiccl_amd.reduce(ref, bufs[8:12])
    ok = ok and torch.equal(ref.view(torch.int32), outs[4].view(torch.int32))
    ok = ok and all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(src, dst))
    torch.cuda.synchronize()
    mib = 1 << 20
    alg = (12 + 5) * mib + (5 + 5) * mib  # reductions: 12 MiB read + 5 written; copies: 5 MiB read + 5 written
    row = {"mode": "progstep", "err": int(err.item()), "bits_ok": bool(ok), "algorithmic_bytes": alg,
           "default_tokens": "fenced" if lib.hiccl_token_mode() == L.HICCL_TOKENS_FENCED else "light"}
    for k, v in res.items():
        row[k + "_us"] = round(float(np.median(v)), 3)
    row["saved_us_per_step"] = round(row["separate_us"] - row["program_us"], 3)
    print(json.dumps(row), flush=True)
    for pr in (p_copy, p_comp, p_tail, q_copy, q_comp):
        pr.close()
    return 0
