#!/bin/bash
# Kernel-trace profile of the 1-GPU bench (eager) + attention PMC counters (separate runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
echo "[gpu_prof] kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
    python3 "$R/bench.py" --steps 4 --warmup 3 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/prof.log" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
if [ "${PMC:-1}" = "1" ]; then
  echo "[gpu_prof] attention PMC"
  timeout -k 10 900 bash $R/scripts/attn_pmc.sh
fi
