#!/bin/bash
# Kernel trace of scripts/bn_probe.py, summarised per kernel and grid (scripts/bn_probe_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${OUT:-bnprof}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/scripts/bn_probe.py" > "$O/run.log" 2>&1 || exit $?
f=$(find "$O/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/bn_probe_summary.py" "$f" > "$O/summary.txt" || exit $?
rm -rf "$O/trace"
