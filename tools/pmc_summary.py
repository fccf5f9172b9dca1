#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of bench.py into profiles/<tag>_pmc.json.

    python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv>
        <kernel_stats.csv> <tag> [n_inputs] [log2count]

HBM bytes per launch of the reduction kernel, corrected as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes for gfx950:
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports exactly half of the
bytes of a wide coalesced streaming read (16 B/lane), so it is doubled;
WRITE_SIZE reads 16-B streaming stores exactly.  The two counters come from
separate passes (TCC slots), averaged over the dispatches of the kernel.
"""
import csv
import json
import os
import sys


def mean_counter(path, counter, match):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and match in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, stats_csv, tag = sys.argv[1:5]
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    log2c = int(sys.argv[6]) if len(sys.argv) > 6 else 28
    count = 1 << log2c
    match = "k_reduce_single"
    fetch_kib, nf = mean_counter(fetch_csv, "FETCH_SIZE", match)
    write_kib, nw = mean_counter(write_csv, "WRITE_SIZE", match)
    read_bytes = 2 * fetch_kib * 1024  # gfx950: FETCH_SIZE = 1/2 of a 16-B/lane stream
    write_bytes = write_kib * 1024
    alg = (n + 1) * count * 4
    stats = [r for r in csv.DictReader(open(stats_csv)) if match in r["Name"]]
    avg_ns = float(stats[0]["AverageNs"]) if stats else None
    out = {
        "tag": tag, "kernel": stats[0]["Name"] if stats else match, "n_inputs": n, "count": count,
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib, "dispatches": [nf, nw],
        "hbm_read_bytes_per_launch": read_bytes, "hbm_write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes, "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / alg,
        "rocprof_avg_kernel_ns": avg_ns,
        "rocprof_GBps": alg / avg_ns if avg_ns else None,
        "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                  "FETCH_SIZE x2 per the gfx950 correction)",
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", f"{tag}_pmc.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
