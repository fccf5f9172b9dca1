#!/usr/bin/env bash
# HBM traffic of the misaligned C2 run (input k 1 + k mod 3 elements off a
# 16-B boundary, bench.c2_misaligned): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (MI355X_MICROARCH.md HBM recipe).  Raw output in
# gpurun_out/pmc_mis/; summarise with tools/pmc_summary.py.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_mis
rm -rf "$out"; mkdir -p "$out"
prog='import bench, json; print(json.dumps(bench.c2_misaligned(8, 1 << 28, 5, 2)))'
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 -c "$prog" > "$out/stats.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 -c "$prog" > "$out/fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 -c "$prog" > "$out/write.log" 2>&1
ls -R "$out" | head -20
