#!/usr/bin/env bash
# Kernel traces of the 2-rank all-reduce composition on one GPU (pipedepth
# 128), one rocprofv3 per rank under mpirun: where a step's time goes.
#   usage (GPU box): tools/trace_c5_2rank.sh TAG STREAM_ORDERED(0|force) GRAPH(0|1)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 HICCL_STREAM_ORDERED=$2 HICCL_GRAPH=$3
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
out=gpurun_out/trace_$1
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 120 "$mpirun" -np 2 rocprofv3 --kernel-trace --output-format csv -d "$out/%pid%" -o run -- \
  build/collectives_hip_f32 8 1048576 1 1 128 2 3 2 ipc > "$out/log.txt" 2>&1
