#!/bin/bash
# Per-kernel trace of the GPT-2-small bench step (eager, so every kernel is its own dispatch) for
# the fused-MLP path and the library path; summaries by scripts/prof_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/profstep"
cd /tmp && export TMPDIR=/tmp
for mode in fused lib; do
  VCX_MLP=$mode timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/profstep/$mode" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 2 --graph 0 > "$R/gpurun_out/profstep/$mode.log" 2>&1 || exit $?
  f=$(find "$R/gpurun_out/profstep/$mode" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/prof_summary.py" "$f" > "$R/gpurun_out/profstep/$mode.txt" || exit $?
  rm -f "$f"
done
