#!/usr/bin/env bash
# Config-5 rehearsal on one MI355X (2 ranks share the device):
#   tools/c5_rehearsal.sh <stream 0|1> <fused 0|1> [ranks] [count] [pipedepth] [hier] [libs]
# all-reduce (pattern 8) of float, warmup 2, 5 timed iterations.
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
MPIRUN=$(command -v mpirun || echo /opt/conda/bin/mpirun)
# more than 4 ranks on the one GPU: 2 hardware queues each
if [ "${3:-2}" -gt 4 ]; then export GPU_MAX_HW_QUEUES=2; fi
export HSA_ENABLE_IPC_MODE_LEGACY=0 HICCL_STREAM_ORDERED=$1 HICCL_FUSED_GATHER=$2 HICCL_SIGNAL_TIMEOUT=30
cd /tmp && exec "$MPIRUN" -np "${3:-2}" "$ROOT/build/collectives_hip_f32" 8 "${4:-134217728}" 1 1 "${5:-128}" 2 5 \
  "${6:-${3:-2}}" "${7:-ipc}"
