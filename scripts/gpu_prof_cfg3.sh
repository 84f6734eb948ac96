#!/bin/bash
# Kernel trace of the BASELINE config-3 step (ResNet-50 local-SGD + top-k EF, B=128, 224^2) with a
# category table (scripts/prof_categories.py): conv fwd / dgrad / wgrad vs GEMM vs BN vs other.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${OUT:-cfg3prof}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench_configs.py" --configs 3 --steps 3 > "$O/run.log" 2>&1 || exit $?
f=$(find "$O/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/prof_categories.py" "$f" 80 > "$O/categories.txt" || exit $?
rm -f "$f"
