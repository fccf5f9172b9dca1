#!/usr/bin/env bash
# HICCL_IPC_RETIRED_MAX=0 (every released IPC mapping closed at once): the
# README all-reduce with fresh buffers and communicators per round, RUNS
# times; counts runs that passed, stopped loudly at the init probe, or
# printed a FAILED round (a silent miss -- must stay 0).
#   usage: tools/cap0_soak.sh RUNS NP ROUNDS
set -u
runs=$1 np=$2 rounds=$3
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
export HSA_ENABLE_IPC_MODE_LEGACY=0 HICCL_IPC_RETIRED_MAX=0 HICCL_STREAM_ORDERED=0
pass=0 loud=0 silent=0 other=0
for i in $(seq "$runs"); do
  out=$(timeout -k 5 60 "$mpirun" -np "$np" build/readme_example_hip 250000 3 "$rounds" 2>&1)
  rc=$?
  if grep -q FAILED <<< "$out"; then silent=$((silent + 1)); echo "$out" > "gpurun_out/cap0_silent_$i.txt"
  elif [ $rc -eq 0 ]; then pass=$((pass + 1))
  elif grep -q "does not reach it" <<< "$out"; then loud=$((loud + 1))
  else other=$((other + 1)); echo "$out" | tail -20 > "gpurun_out/cap0_other_$i.txt"; fi
done
echo "{\"runs\": $runs, \"ranks\": $np, \"rounds\": $rounds, \"passed\": $pass, \"probe_stopped\": $loud, \"silent_wrong\": $silent, \"other\": $other}"
