#!/usr/bin/env python3
"""Per-process kernel-trace summary of tools/trace_c5_prog.sh output:
kernel count, span and busy time of the second half of each process's trace
(steady state: graph replays), and per kernel name the count and median
duration.
    python tools/trace_summary.py gpurun_out/trace_<TAG> [label]
"""
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d)
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        rows = rows[len(rows) // 2:]
        if not rows:
            continue
        t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
        print(f"{label:28s} pid {f.split(os.sep)[-3] if f.count(os.sep) > 2 else '?'}: {len(rows)} kernels, "
              f"span {(t1 - t0) / 1e3:.0f} us, busy {busy / 1e3:.0f} us")
        by = {}
        for r in rows:
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
            by.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for name, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
            print(f"    {name:34s} n={len(v):6d} median {statistics.median(v):8.2f} us")


if __name__ == "__main__":
    main()
