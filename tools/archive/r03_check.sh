#!/usr/bin/env bash
# Round-3 GPU check pass (gpurun): program kernels, the single-GPU step A/B,
# the IPC reproducer, the C++ stack under MPI (stream-ordered cases run on
# programs), and the 2-rank C5 A/B of programs vs separate launches.  Every
# step has its own time limit; the first failure ends the pass.
#   usage (GPU box): tools/r03_check.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
mkdir -p gpurun_out
py="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 300 $py --timeout 120 tests/test_program_gpu.py > "gpurun_out/${tag}_program.log" 2>&1
echo "check: program tests passed"
timeout -k 10 120 python bench.py --progstep > "gpurun_out/${tag}_progstep.jsonl" 2>&1
echo "check: progstep done"
timeout -k 10 240 $py --timeout 200 tests/test_ipc_reuse_gpu.py > "gpurun_out/${tag}_ipc.log" 2>&1
echo "check: ipc reproducer done"
timeout -k 10 700 $py --timeout 200 tests/test_mpi_gpu.py tests/test_c5_leg_gpu.py tests/test_reference_driver.py \
  > "gpurun_out/${tag}_mpi.log" 2>&1
echo "check: mpi tests passed"
timeout -k 10 400 tools/c5_prog_ab.sh "gpurun_out/${tag}_c5_prog_ab.jsonl" 2 23 2 > "gpurun_out/${tag}_ab.log" 2>&1
echo "check: c5 a/b done"
