#!/bin/bash
# The one GPU-box call runner (replaces the per-call gpu_r3_* / gpu_r4_* scripts of earlier rounds).
#   gpurun -- 'OUT=name bash scripts/gpu_steps.sh "tests|600|python -u -m pytest -q tests -m gpu" "bench|240|python -u bench.py"'
# Each argument is "name|seconds|command". Every step runs under its own `timeout -k 10`, writes
# gpurun_out/$OUT/<name>.log and one "name rc=N" line to gpurun_out/$OUT/summary.txt. A crash, abort
# or time limit (rc > 1) ends the call there (no further GPU step after a fault); a plain test
# failure (pytest rc 1) does not. Output of a JSON bench line is copied into the summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O="gpurun_out/${OUT:-steps}"
mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name $(date +%T)" >> "$O/summary.txt"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc" >> "$O/summary.txt"
  grep -h '^{"metric"' "$O/$name.log" >> "$O/summary.txt" 2>/dev/null
  tail -3 "$O/$name.log" | cut -c1-300
  echo "[steps] $name rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
