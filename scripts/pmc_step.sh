#!/bin/bash
# Hardware counters for every kernel of the GPT-2-small bench step (eager, 2 timed steps), one
# counter set per rocprofv3 run: HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes, they share
# the TCC counter slots) and the MFMA / LDS / wave activity set. Summarise with
#   python scripts/pmc_summary.py gpurun_out/pmc_step
# PMC_PROG=<script under the repo root> and PMC_OUT=<name> profile another program instead
# (e.g. PMC_PROG=scripts/compress_only.py PMC_OUT=pmc_compress).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PMC_OUT:-pmc_step}
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --graph 0"
[ -n "$PMC_PROG" ] && ARGS=""
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $set"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/${PMC_PROG:-bench.py}" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
exit 0
