#!/usr/bin/env bash
# Round-4 measurement pass on one MI355X (gpurun).  Every step has its own
# time limit and the first failure ends the pass (set -e):
#   gputest    the whole -m gpu suite, one process, per-test timeouts
#   bench      the headline line (C2, CPU baseline with its spread)
#   c3vsc2     C3 per n interleaved with C2 on this one box (verdict r3 item 3)
#   roundtrip  host-resident buckets on the current code (verdict r3 item 4)
#   progstep   one C5 step's enqueue cost, default (fenced) vs light tokens
#   usage (GPU box): tools/r04_measure.sh TAG [steps...]   (default: all four)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1
shift
steps=${*:-gputest bench c3vsc2 roundtrip}
mkdir -p gpurun_out
for s in $steps; do
  case $s in
    gputest)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
        --durations 30 > "gpurun_out/${tag}_gputest.log" 2>&1 ;;
    bench)
      timeout -k 10 300 python3 bench.py > "gpurun_out/${tag}_bench.jsonl" 2> "gpurun_out/${tag}_bench.err" ;;
    c3vsc2)
      timeout -k 10 400 python3 bench.py --c3vsc2 --rounds 5 --steps 10 --warmup 3 \
        > "gpurun_out/${tag}_c3_vs_c2.jsonl" 2> "gpurun_out/${tag}_c3_vs_c2.err" ;;
    progstep)
      timeout -k 10 300 python3 bench.py --progstep > "gpurun_out/${tag}_progstep.jsonl" 2> "gpurun_out/${tag}_progstep.err" ;;
    roundtrip)
      timeout -k 10 400 python3 bench.py --roundtrip > "gpurun_out/${tag}_roundtrip.jsonl" \
        2> "gpurun_out/${tag}_roundtrip.err" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "measure: $s done"
done
