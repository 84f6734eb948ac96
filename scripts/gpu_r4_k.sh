# round 4, GPU call K: kernel trace of BASELINE config 5 (Llama-3-8B sharded AdamW + PowerSGD rank 4, one peer,
# B=2x2048) -- where the step's time goes now (round 1's table: profiles/r1_cfg5_llama3_8b_kernel_stats.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/k"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/k/cfg5" -o run -- \
    python3 "$R/bench_configs.py" --configs 5 --steps 4 > "$R/gpurun_out/k/cfg5.log" 2>&1 || exit $?
f=$(find "$R/gpurun_out/k/cfg5" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/prof_summary.py" "$f" > "$R/gpurun_out/k/cfg5.txt" || exit $?
rm -f "$f"
