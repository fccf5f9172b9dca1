#!/usr/bin/env bash
# A/B of step programs (one launch per pipeline step, HICCL_STEP_PROGRAM=1,
# the default) against one launch per element (HICCL_STEP_PROGRAM=0) on ONE
# GPU (ranks share it: stream-ordered forced, hardware queues lowered): the
# all-reduce composition, pipedepth 128, stream-ordered eager and graph +
# fused, interleaved rounds.  Same shape as profiles/r02j_c5_ab_phases.jsonl
# (2 ranks: 64 MiB per rank, flat IPC).  One JSON record per run.
#   usage (GPU box): tools/c5_prog_ab.sh OUT.jsonl RANKS LOG2COUNT [ROUNDS]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1 ranks=$2 lc=$3 rounds=${4:-2}
exe=build/collectives_hip_f32
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
hier=$ranks libs=ipc
if [ "$ranks" -ge 4 ]; then hier="1,$((ranks / 2)),2" libs="mpi,ipc,ipc"; fi
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 GPU_MAX_HW_QUEUES=2 HICCL_SIGNAL_TIMEOUT=20
for r in $(seq "$rounds"); do
  for prog in 1 0; do
    for mode in eager graph_fused; do
      if [ $mode = eager ]; then g=0 f=0; else g=1 f=1; fi
      tmp=$(mktemp /tmp/c5ab.XXXXXX.json)
      HICCL_DRIVER_JSON=$tmp HICCL_STREAM_ORDERED=force HICCL_GRAPH=$g HICCL_FUSED_GATHER=$f HICCL_STEP_PROGRAM=$prog \
        timeout -k 10 120 "$mpirun" -np "$ranks" "$exe" 8 $((1 << lc)) 1 1 128 2 10 "$hier" "$libs" > /dev/null
      python3 -c "import json,sys; r=json.load(open('$tmp')); r.update(step_program=$prog, run='$mode', round=$r); print(json.dumps(r))" | tee -a "$out"
      rm -f "$tmp"
    done
  done
done
