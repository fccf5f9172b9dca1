#!/usr/bin/env bash
# Config 3 per n: for n in 3 4 8 16 64 inputs x 2^26 fp32,
# one rocprofv3 --kernel-trace --stats pass, then FETCH_SIZE, WRITE_SIZE and
# the SQ occupancy / stall counters in separate --pmc passes (never combined
# with tracing).  Raw output: gpurun_out/c3pmc/n<N>/{stats,fetch,write,sq};
# summarise here with tools/c3_pmc_summary.py.
#   usage (on the GPU box): tools/c3_pmc.sh [n ...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ns=${*:-3 4 8 16 64}
for n in $ns; do
  out=gpurun_out/c3pmc/n$n
  rm -rf "$out"; mkdir -p "$out"
  args=(--n "$n" --log2count 26 --no-cpu --no-misaligned)
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 bench.py "${args[@]}" --steps 10 --warmup 3 > "$out/stats.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py "${args[@]}" --steps 4 --warmup 1 > "$out/fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 bench.py "${args[@]}" --steps 4 --warmup 1 > "$out/write.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY --output-format csv -d "$out/sq" -o run -- \
    python3 bench.py "${args[@]}" --steps 4 --warmup 1 > "$out/sq.log" 2>&1
  echo "c3pmc: n=$n done"
done
