#!/usr/bin/env python3
"""Summarise tools/profile_plans.sh output (gpurun_out/prof_<tag>/) into
profiles/<tag>_plan_profile.json: per reduction-kernel shape (kernel name x
grid size, in launch order), the rocprofv3 kernel-trace duration (median of
the dispatches), and the PMC counters of the separate --pmc passes per
dispatch (median): FETCH_SIZE x 2 + WRITE_SIZE = HBM bytes (the gfx950
corrections of MI355X_MICROARCH.md's HBM section: FETCH_SIZE counts half of a
16-B/lane streaming read; both in KiB), SQ_* wave/instruction counts.

    python tools/plan_pmc_summary.py <tag> [shape-label algorithmic-bytes]

The optional pair names the shape of every launch of a single-shape run
(tools/plan_shapes.py --shapes d), whose grid the table below cannot tell
from shape b's.
"""
import csv
import glob
import json
import os
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = {  # grid threads -> (shape, algorithmic bytes per launch): tools/plan_shapes.py
    262144: ("a: C4 16 MiB/input x 16 computes, n = 8 (f32 then bf16)", 9 * 16 << 20),
    65536: ("b: C4 bf16 1 GiB/input x 1024 computes, n = 8 (plan and one-shot)", 9 * 1024 << 20),
    81920: ("c: C5 step, 4 x (n = 2) + 1 x (n = 4) computes of 2^18 f32 (U = 4)", (4 * 3 + 5) * (1 << 18) * 4),
    163840: ("c: C5 step, 4 x (n = 2) + 1 x (n = 4) computes of 2^18 f32 (U = 2)", (4 * 3 + 5) * (1 << 18) * 4),
}


def kname(r):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def grid_of(r):
    for k in ("Grid_Size", "Grid_Size_X"):
        if k in r and r[k]:
            return int(r[k])
    return 0


def main():
    tag = sys.argv[1]
    d = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    trace = glob.glob(os.path.join(d, "stats", "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(trace)) if "k_reduce" in r["Kernel_Name"]]
    durs = {}
    for r in rows:
        key = (kname(r), grid_of(r))
        durs.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    counters = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "k_reduce" not in r["Kernel_Name"]:
                continue
            key = (kname(r), grid_of(r))
            counters.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = []
    for key, ds in durs.items():
        name, grid = key
        shape, alg = SHAPES.get(grid, ("?", None))
        if len(sys.argv) > 3:
            shape, alg = sys.argv[2], int(sys.argv[3])
        c = {k: st.median(v) for k, v in counters.get(key, {}).items()}
        rec = {"kernel": name, "grid_threads": grid, "shape": shape, "dispatches": len(ds),
               "duration_us_median": round(st.median(ds), 3), "duration_us_min": round(min(ds), 3),
               "algorithmic_bytes": alg,
               "GBps_at_median": round(alg / (st.median(ds) * 1e3), 1) if alg else None}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            rec.update({"fetch_size_kib": c["FETCH_SIZE"], "write_size_kib": c["WRITE_SIZE"], "hbm_bytes": hbm,
                        "traffic_over_algorithmic": round(hbm / alg, 4) if alg else None})
        for k in sorted(c):
            if k.startswith("SQ_"):
                rec[k] = c[k]
        out.append(rec)
    res = {"tag": tag, "source": "tools/profile_plans.sh (rocprofv3 --kernel-trace --stats; --pmc passes apart)",
           "shapes": out}
    path = os.path.join(ROOT, "profiles", f"{tag}_plan_profile.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
