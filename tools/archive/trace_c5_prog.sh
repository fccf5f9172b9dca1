#!/usr/bin/env bash
# Kernel traces of the 2-rank all-reduce composition on one GPU (pipedepth
# 128, stream-ordered forced, graph + fused), one rocprofv3 per rank under
# mpirun, with step programs on (HICCL_STEP_PROGRAM=1) or off (0): kernels
# per pipeline step and their durations.
#   usage (GPU box): tools/trace_c5_prog.sh TAG PROGRAM(0|1) [LOG2COUNT]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
lc=${3:-23}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 GPU_MAX_HW_QUEUES=2 HICCL_SIGNAL_TIMEOUT=20
export HICCL_STREAM_ORDERED=force HICCL_GRAPH=1 HICCL_FUSED_GATHER=1 HICCL_STEP_PROGRAM=$2
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
out=gpurun_out/trace_$1
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 150 "$mpirun" -np 2 rocprofv3 --kernel-trace --output-format csv -d "$out/%pid%" -o run -- \
  build/collectives_hip_f32 8 $((1 << lc)) 1 1 128 2 5 2 ipc > "$out/log.txt" 2>&1
