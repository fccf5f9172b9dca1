#!/usr/bin/env bash
# Repeat the README all-reduce example (fresh communicator per round) RUNS
# times under the given transport env; stop at the first failing run.
#   usage: tools/readme_repeat.sh RUNS NP ROUNDS [VAR=VALUE ...]
set -u
runs=$1 np=$2 rounds=$3; shift 3
export HSA_ENABLE_IPC_MODE_LEGACY=0 HICCL_SIGNAL_TIMEOUT=10 "$@"
mpirun=$(command -v mpirun || echo /opt/conda/bin/mpirun)
for i in $(seq "$runs"); do
  out=$(timeout -k 5 60 "$mpirun" -np "$np" build/readme_example_hip "${COUNT:-250000}" 3 "$rounds" 2>&1)
  rc=$?
  fails=$(grep -c FAILED <<< "$out")
  echo "run $i rc=$rc failed_rounds=$fails"
  if [ $rc -ne 0 ]; then echo "$out" > "gpurun_out/readme_fail_$$.txt"; grep -E "wrong|FAILED|hiccl" <<< "$out" | head -20; exit $rc; fi
done
