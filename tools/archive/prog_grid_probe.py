#!/usr/bin/env python3
"""Fenced step programs: does a smaller grid make the gate hand-off cheaper?

Round 5 closed the gate hand-off of a program's non-zero workgroups with an
agent-scope acquire fence (k_program), which invalidates the workgroup's XCD
L2: ~8 us per C5 step at the default grid of 4 workgroups per CU
(profiles/r05a_progstep.jsonl).  The MI355X price table's barrier-xcd row
(4.1 / 5.9 / 9.7 us at 256 / 512 / 1024 workgroups) says that cost scales
with the workgroups that acquire.  This probe runs one C5 step as two
programs (ready phase + the five 1 MiB copies; done phase + the 4 x n=2 +
1 x n=4 reductions of 2^18 f32; the tail phase folded into the next step, as
in a pipeline) with hiccl_program_set_max_workgroups 0 (default), 512, 256
and 128, fenced and light tokens, queued (events around 200 back-to-back
steps), interleaved rounds, outputs checked bit for bit.  The phases signal
and await this process's own flags (always satisfied).

    python tools/prog_grid_probe.py > gpurun_out/<tag>_prog_grid.jsonl
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


def main():
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
    for k, t in enumerate(src):
        hiccl_amd.fill_uniform(t, B.SEED, 40 + k)
    dst = [torch.empty(c, device="cuda") for _ in range(5)]
    cp = hiccl_amd.Compute(torch.uint8, device=dev)
    for a, b in zip(src, dst):
        cp.add([a.view(torch.uint8)], b.view(torch.uint8), c * 4, compid=0)
    flags = torch.zeros(16, dtype=torch.int32, device="cuda")
    f = [flags.data_ptr() + 4 * i for i in range(2)]
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    epoch = [0]
    progs = {}
    for wg in (0, 512, 256, 128):
        pair = []
        for flag, plan in ((f[0], cp), (f[1], comp)):
            pr = hiccl_amd.Program(torch.float32, device=dev)
            pr.add_signal([flag], [flag])
            pr.add_plan(plan)
            if wg:
                pr.set_max_workgroups(wg)
            pair.append(pr)
        progs[wg] = pair

    def step(pair, mode):
        def run():
            os.environ["HICCL_PROG_FENCES"] = mode
            try:
                epoch[0] += 1
                for pr in pair:
                    pr.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)
            finally:
                os.environ.pop("HICCL_PROG_FENCES", None)
        return run

    runs = {(wg, mode): step(pair, mode) for wg, pair in progs.items() for mode in ("full", "light")}
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(B.time_queued(fn, 200, 10) * 1e3)
    torch.cuda.synchronize()
    ok = int(err.item()) == 0
    ref = torch.empty(c, device="cuda")
    for j in range(4):
        hiccl_amd.reduce(ref, [bufs[2 * j], bufs[2 * j + 1]])
        ok = ok and torch.equal(ref.view(torch.int32), outs[j].view(torch.int32))
    hiccl_amd.reduce(ref, bufs[8:12])
    ok = ok and torch.equal(ref.view(torch.int32), outs[4].view(torch.int32))
    ok = ok and all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(src, dst))
    row = {"mode": "prog_grid", "bits_ok": bool(ok), "err": int(err.item()),
           "reduction_units": progs[0][1].units(), "copy_units": progs[0][0].units()}
    for (wg, mode), v in res.items():
        row[f"wg{wg or 'default'}_{'fenced' if mode == 'full' else 'light'}_us"] = round(float(np.median(v)), 3)
    print(json.dumps(row), flush=True)
    for pair in progs.values():
        for pr in pair:
            pr.close()
    comp.close()
    cp.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
