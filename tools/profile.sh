#!/usr/bin/env bash
# rocprofv3 evidence for the bench's dominant kernel (MI355X_MICROARCH.md HBM
# recipe): one --kernel-trace --stats run, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (never combined with tracing).  Raw output lands in
# gpurun_out/prof_<tag>/ (the only directory gpurun brings back); summarise
# it into profiles/ locally with tools/collect_profile.sh <tag>.
#   usage (on the GPU box): tools/profile.sh <tag> [bench args...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
  python3 bench.py --no-cpu --no-misaligned --steps 20 --warmup 5 "$@" > "$out/stats.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 bench.py --no-cpu --no-misaligned --steps 5 --warmup 2 "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 bench.py --no-cpu --no-misaligned --steps 5 --warmup 2 "$@" > "$out/write.log" 2>&1
ls -R "$out" | head -40
