#!/usr/bin/env python3
"""Summarise tools/c3_pmc.sh output (gpurun_out/c3pmc/n<N>/) into
profiles/<tag>_c3_pmc.json: per n, the reduction kernel (k_reduce_single
shape = the engine AUTO picked), its rocprofv3 average duration and rate,
HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
MI355X_MICROARCH.md), and the SQ occupancy / stall fractions.

    python tools/c3_pmc_summary.py <tag> [n ...]   (default: every n measured)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MATCH = "k_reduce_single"


def one(path_glob):
    f = glob.glob(path_glob, recursive=True)
    return f[0] if f else None


def counters(path):
    acc = {}
    for r in csv.DictReader(open(path)):
        if MATCH not in r["Kernel_Name"]:
            continue
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag = sys.argv[1]
    res = {"tag": tag, "workload": "C3: n inputs x 2^26 fp32 (256 MiB/input), AUTO engine, bench.py --n N --log2count 26",
           "per_n": {}}
    only = {int(x) for x in sys.argv[2:]}
    for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "c3pmc", "n*")), key=lambda p: int(p.rsplit("n", 1)[1])):
        n = int(d.rsplit("n", 1)[1])
        if only and n not in only:
            continue
        count = 1 << 26
        alg = (n + 1) * count * 4
        row = {"algorithmic_bytes_per_launch": alg}
        st = one(os.path.join(d, "stats", "**", "*kernel_stats.csv"))
        if st:
            for r in csv.DictReader(open(st)):
                if MATCH in r["Name"]:
                    ns = float(r["AverageNs"])
                    row.update({"kernel": r["Name"].split("k_reduce_single")[1][:60], "calls": int(r["Calls"]),
                                "avg_ns": ns, "GBps": round(alg / ns, 1), "frac_of_8TBps": round(alg / ns / 8000, 4)})
        fe = one(os.path.join(d, "fetch", "**", "*counter_collection.csv"))
        wr = one(os.path.join(d, "write", "**", "*counter_collection.csv"))
        if fe and wr:
            rb = 2 * counters(fe).get("FETCH_SIZE", 0) * 1024
            wb = counters(wr).get("WRITE_SIZE", 0) * 1024
            row.update({"hbm_read_bytes": rb, "hbm_write_bytes": wb,
                        "traffic_over_algorithmic": round((rb + wb) / alg, 5)})
        sq = one(os.path.join(d, "sq", "**", "*counter_collection.csv"))
        if sq:
            c = counters(sq)
            wc = c.get("SQ_WAVE_CYCLES") or 0
            row["sq"] = {k: c[k] for k in sorted(c)}
            if wc:
                row["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
                row["wait_inst_any_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
                row["active_inst_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            if c.get("SQ_BUSY_CYCLES") and row.get("avg_ns"):
                row["waves_per_busy_cycle"] = round(c.get("SQ_WAVES", 0) / c["SQ_BUSY_CYCLES"], 6)
        res["per_n"][str(n)] = row
    path = os.path.join(ROOT, "profiles", f"{tag}_c3_pmc.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
