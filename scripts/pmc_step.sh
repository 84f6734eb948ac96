#!/bin/bash
# Hardware counters for every kernel of the GPT-2-small bench step (eager, 2 timed steps), one counter set
# per rocprofv3 run (gfx950 slots per pass: 8 SQ, 4 TCC -- FETCH_SIZE takes 3, WRITE_SIZE 2 --, 2 GRBM):
#   p1 FETCH_SIZE + GRBM_GUI_ACTIVE, p2 WRITE_SIZE + GRBM_GUI_ACTIVE,
#   p3 MFMA / VALU / LDS instruction + wave-cycle set + GRBM_GUI_ACTIVE, p4 wait / issue-stall set.
# Summarise with  python scripts/pmc_summary.py gpurun_out/pmc_step
# PMC_PROG=<script under the repo root> [PMC_ARGS=...] PMC_OUT=<name> profile another program instead.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PMC_OUT:-pmc_step}
mkdir -p "$OUT"
ARGS=${PMC_ARGS-"--steps 2 --warmup 1 --graph 0"}
[ -n "$PMC_PROG" ] && [ -z "$PMC_ARGS" ] && ARGS=""
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $set"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/${PMC_PROG:-bench.py}" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$R/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.txt" || exit $?
rm -rf "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4  # raw CSVs are large; the summary keeps the numbers
exit 0
