#!/usr/bin/env bash
# Round-3 measurement pass on one MI355X (gpurun): the headline bench line,
# its rocprofv3 trace + PMC (tools/profile.sh), config 3 per n (PMC passes,
# tools/c3_pmc.sh, and an interleaved engine / occupancy sweep).  Every step
# has its own time limit; the first failure ends the pass.
#   usage (GPU box): tools/r03_measure.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > "gpurun_out/${tag}_bench.jsonl" 2> "gpurun_out/${tag}_bench.err"
echo "measure: bench done"
timeout -k 10 600 tools/profile.sh "$tag"
echo "measure: profile done"
timeout -k 10 900 tools/c3_pmc.sh
echo "measure: c3 pmc done"
timeout -k 10 600 python3 bench.py --schedsweep --sweepset c3 --xn 3,4,8,16,64 --xmib 256 --steps 10 --warmup 3 \
  > "gpurun_out/${tag}_c3_sweep.jsonl" 2> "gpurun_out/${tag}_c3_sweep.err"
echo "measure: c3 sweep done"
