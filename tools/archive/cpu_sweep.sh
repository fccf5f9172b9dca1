#!/usr/bin/env bash
# CPU baseline thread placement on the GPU box's host: the reference's CPU
# reduce_kernel over the config-2 bucket (bench.py --cpu-leg) under several
# OMP_NUM_THREADS / OMP_PROC_BIND / OMP_PLACES settings.
#   usage (on the box): tools/cpu_sweep.sh > gpurun_out/cpu_sweep.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for t in 16 32; do
  for bind in "" spread close; do
    for places in "" cores threads; do
      [ -z "$bind" ] && [ -n "$places" ] && continue
      env -u OMP_PROC_BIND -u OMP_PLACES OMP_NUM_THREADS=$t ${bind:+OMP_PROC_BIND=$bind} ${places:+OMP_PLACES=$places} \
        timeout -k 5 120 python3 bench.py --cpu-leg --n 8 --log2count 28 --cpu-budget 3 \
        | sed "s/^{/{\"omp\": \"t=$t bind=${bind:-unset} places=${places:-unset}\", /"
    done
  done
done
