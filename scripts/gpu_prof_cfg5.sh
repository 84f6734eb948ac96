#!/bin/bash
# Kernel trace of the BASELINE config-5 step (Llama-3-8B sharded optimizer + PowerSGD, B=2x2048, one peer),
# summarised per kernel name over the whole run (2 warmup + 2 timed steps and the model's init).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${OUT:-cfg5prof}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench_configs.py" --configs 5 --steps 4 > "$O/run.log" 2>&1 || exit $?
f=$(find "$O/trace" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$O/step.txt" <<'PY' || exit $?
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    agg[r["Kernel_Name"][:90]][0] += 1
    agg[r["Kernel_Name"][:90]][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"whole run (4 steps + init): {tot / 1e3:.2f} ms kernel time, {len(rows)} kernels")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:45]:
    print(f"{v[1] / 1e3:9.3f} ms {v[1] / tot * 100:5.1f}% {v[0]:5d}x  {k}")
PY
rm -rf "$O/trace"
