#!/usr/bin/env bash
# rocprofv3 evidence for the batched plan kernel (k_reduce_plan) on the shapes
# Comm<T> runs per step (tools/plan_shapes.py: C4 16 MiB f32/bf16, C4 bf16
# 1 GiB, a C5-shaped step).  One --kernel-trace --stats pass, then counters in
# separate --pmc passes (never combined with tracing; <= 4 TCC per pass:
# FETCH_SIZE and WRITE_SIZE apart), per MI355X_MICROARCH.md's recipe.
#   usage (on the GPU box): tools/profile_plans.sh <tag> [shapes, default a,b,c]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1
out=gpurun_out/prof_$tag
rm -rf "$out"; mkdir -p "$out"
run="python3 tools/plan_shapes.py --steps 10 --warmup 3 --rounds 1 --shapes ${2:-a,b,c}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
  $run > "$out/stats.log" 2>&1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc --output-format csv -d "$out/pmc$i" -o run -- \
    $run > "$out/pmc$i.log" 2>&1
done
ls -R "$out" | head -40
