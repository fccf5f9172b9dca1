#!/usr/bin/env bash
# tools/gpurun_call.sh TAG TIMEOUT 'COMMAND' -- one gpurun call, logged.
#
# Runs COMMAND once on the GPU box (no retry: a call gpurun could not place,
# exit 3, is tried again by hand) and keeps two records under gpurun_out/:
#   TAG_call.log      everything gpurun printed for the call
#   TAG_attempts.log  one line per attempt: the time, gpurun's exit code and
#                     its own "status=... rc=... charged=..." line, so a fault,
#                     a kill at the limit or an abort is never hidden behind a
#                     later successful attempt
set -uo pipefail
[ $# -eq 3 ] || { echo "usage: $0 TAG TIMEOUT_S 'COMMAND'" >&2; exit 64; }
tag=$1 limit=$2 cmd=$3
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/gpurun_out"
log="$root/gpurun_out/${tag}_call.log"
att="$root/gpurun_out/${tag}_attempts.log"
n=$(( $( [ -f "$att" ] && wc -l < "$att" || echo 0) + 1 ))
cd "$root"
/usr/local/graft/bin/gpurun --timeout "$limit" -- "$cmd" > "$log.tmp" 2>&1
rc=$?
cat "$log.tmp" >> "$log"
status=$(grep -m1 -o 'status=.*' "$log.tmp" || echo "no status line")
rm -f "$log.tmp"
echo "$(date -u +%FT%TZ) attempt $n gpurun_rc $rc $status" >> "$att"
tail -n 40 "$log"
exit $rc
