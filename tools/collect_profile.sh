#!/usr/bin/env bash
# Summarise gpurun_out/prof_<tag>/ (written by tools/profile.sh on the GPU
# box) into the committed profiles/: <tag>_kernel_stats.csv (rocprofv3
# --stats), <tag>_kernel_trace.csv (reduction-kernel rows of the trace),
# <tag>_pmc.json (HBM bytes per launch, tools/pmc_summary.py) and
# <tag>_bench_under_rocprof.jsonl.
#   usage (here): tools/collect_profile.sh <tag>
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1
d=gpurun_out/prof_$tag
stats=$(find "$d/stats" -name '*kernel_stats.csv' | head -1)
trace=$(find "$d/stats" -name '*kernel_trace.csv' | head -1)
fetch=$(find "$d/fetch" -name '*counter_collection.csv' | head -1)
write=$(find "$d/write" -name '*counter_collection.csv' | head -1)
python3 tools/pmc_summary.py "$fetch" "$write" "$stats" "$tag" > /dev/null
cp "$stats" "profiles/${tag}_kernel_stats.csv"
{ head -1 "$trace"; grep k_reduce "$trace" || true; } > "profiles/${tag}_kernel_trace.csv"
grep -h '^{' "$d/stats.log" > "profiles/${tag}_bench_under_rocprof.jsonl" || true
cat "profiles/${tag}_pmc.json"
