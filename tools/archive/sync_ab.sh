#!/usr/bin/env bash
# Host-driven all-reduce (pipedepth 128) under each HICCL_SYNC wait policy,
# interleaved rounds; one JSON record per run.
#   usage: tools/sync_ab.sh OUT.jsonl RANKS LOG2COUNT [ROUNDS]
set -eu
out=$1 ranks=$2 lc=$3 rounds=${4:-3}
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 HICCL_STREAM_ORDERED=0
for r in $(seq "$rounds"); do
  for sync in auto spin yield blocking; do
    tmp=$(mktemp /tmp/syncab.XXXXXX.json)
    HICCL_DRIVER_JSON=$tmp HICCL_SYNC=$sync \
      timeout -k 10 120 "$mpirun" -np "$ranks" build/collectives_hip_f32 8 $((1 << lc)) 1 1 128 2 10 "$ranks" ipc > /dev/null
    python3 -c "import json; r=json.load(open('$tmp')); r.update(sync='$sync', round=$r); print(json.dumps({k: r[k] for k in ('sync','round','ranks','collective_ms_min','collective_ms_median','kat')}))" | tee -a "$out"
    rm -f "$tmp"
  done
done
