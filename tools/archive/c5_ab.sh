#!/usr/bin/env bash
# A/B of two builds of the collectives driver on one GPU (ranks share it, so
# stream-ordered mode is forced and the hardware queues lowered): the
# all-reduce composition, pipedepth 128, stream-ordered eager and
# graph + fused.  Each run writes one JSON record (HICCL_DRIVER_JSON).
#   usage: tools/c5_ab.sh OUT.jsonl RANKS LOG2COUNT EXE_A EXE_B [ROUNDS]
set -eu
out=$1 ranks=$2 lc=$3 a=$4 b=$5 rounds=${6:-2}
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
hier=$ranks libs=ipc
if [ "$ranks" -ge 4 ]; then hier="1,$((ranks / 2)),2" libs="mpi,ipc,ipc"; fi
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 GPU_MAX_HW_QUEUES=2 HICCL_SIGNAL_TIMEOUT=20
for r in $(seq "$rounds"); do
  for exe in "$a" "$b"; do
    for mode in eager graph_fused; do
      if [ $mode = eager ]; then g=0 f=0; else g=1 f=1; fi
      tmp=$(mktemp /tmp/c5ab.XXXXXX.json)
      HICCL_DRIVER_JSON=$tmp HICCL_STREAM_ORDERED=force HICCL_GRAPH=$g HICCL_FUSED_GATHER=$f \
        timeout -k 10 120 "$mpirun" -np "$ranks" "$exe" 8 $((1 << lc)) 1 1 128 2 10 "$hier" "$libs" > /dev/null
      python3 -c "import json,sys; r=json.load(open('$tmp')); r.update(exe='$(basename "$exe")', run='$mode', round=$r); print(json.dumps(r))" | tee -a "$out"
      rm -f "$tmp"
    done
  done
done
