#!/bin/bash
# Kernel trace + counters for the compression kernels (scripts/compress_only.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_compress
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o v -- \
    python3 "$R/scripts/compress_only.py" > "$OUT/trace.log" 2>&1 || exit $?
i=0
for set in "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $set"
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/scripts/compress_only.py" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
exit 0
