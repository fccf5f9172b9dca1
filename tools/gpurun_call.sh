#!/usr/bin/env bash
# tools/gpurun_call.sh TAG TIMEOUT 'COMMAND' -- one gpurun call, logged.
#
# Runs COMMAND once on the GPU box (no retry: a call gpurun could not place,
# exit 3, is tried again by hand) and keeps records under gpurun_out/:
#   TAG_call.log      everything gpurun printed for the call (appended)
#   TAG_attempts.log  one line per attempt: the time, gpurun's exit code and
#                     its own "status=... rc=... charged=..." line, so a fault,
#                     a kill at the limit or an abort is never hidden behind a
#                     later successful attempt
#   TAG_aN_*          after an attempt N whose status is not ok: every
#                     gpurun_out/ entry naming TAG that the attempt pulled back
#                     (and gpurun's verdict, TAG_aN_last_call.json) renamed,
#                     so a retry into the same file names cannot overwrite the
#                     failure (r05w / r05ae lost theirs)
# (HICCL_GPURUN names another client: the CPU tier's stub, tests/test_tools.py)
set -uo pipefail
[ $# -eq 3 ] || { echo "usage: $0 TAG TIMEOUT_S 'COMMAND'" >&2; exit 64; }
tag=$1 limit=$2 cmd=$3
root=$(cd "$(dirname "$0")/.." && pwd)
out="$root/gpurun_out"
mkdir -p "$out"
log="$out/${tag}_call.log"
att="$out/${tag}_attempts.log"
prev=$(grep -c ' gpurun_rc ' "$att" 2>/dev/null)
n=$(( ${prev:-0} + 1 ))
# what gpurun_out/ holds under this tag before the call (name size mtime): an
# entry the call adds or changes is one the attempt pulled back
snap() { find "$out" -maxdepth 1 -mindepth 1 -name "*${tag}*" -printf '%f %s %T@\n' | sort; }
before=$(snap)
cd "$root"
"${HICCL_GPURUN:-/usr/local/graft/bin/gpurun}" --timeout "$limit" -- "$cmd" > "$log.tmp" 2>&1
rc=$?
cat "$log.tmp" >> "$log"
status=$(grep -m1 -o 'status=.*' "$log.tmp" || echo "no status line")
rm -f "$log.tmp"
echo "$(date -u +%FT%TZ) attempt $n gpurun_rc $rc $status" >> "$att"
case "$status" in
  status=ok*) ;;
  *)
    kept=0
    for f in "$out"/*"$tag"*; do
      [ -e "$f" ] || continue
      b=$(basename "$f")
      case "$b" in "${tag}_call.log"|"${tag}_attempts.log"|"${tag}"_a[0-9]*) continue ;; esac
      grep -qxF "$(find "$f" -maxdepth 0 -printf '%f %s %T@')" <<< "$before" && continue
      mv "$f" "$out/${tag}_a${n}_${b#"${tag}"_}" && kept=$((kept + 1))
    done
    [ -f "$out/.last_call.json" ] && cp "$out/.last_call.json" "$out/${tag}_a${n}_last_call.json"
    echo "$(date -u +%FT%TZ) attempt $n kept $kept pulled entries as ${tag}_a${n}_*" >> "$att"
    ;;
esac
tail -n 40 "$log"
exit $rc
