#!/bin/bash
# Kernel sequence of one GPT-2 bench step (eager), scripts/step_sequence.py -> gpurun_out/$OUT/seq.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${OUT:-stepseq}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --graph 0 > "$O/step.log" 2>&1 || exit $?
f=$(find "$O/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/step_sequence.py" "$f" > "$O/seq.txt" || exit $?
python3 "$R/scripts/prof_summary.py" "$f" > "$O/step.txt" || exit $?
rm -rf "$O/trace"
