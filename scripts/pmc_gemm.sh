#!/bin/bash
# Counter passes over a GEMM probe script (default scripts/conv3x3_probe.py: MIOpen vs gemm_wg weight gradients);
# summarise with: python scripts/pmc_summary.py gpurun_out/$PMC_OUT
#   PMC_OUT=pmc_conv bash scripts/pmc_gemm.sh [probe.py [args...]]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PMC_OUT:-pmc_gemm}
PROBE=${1:-scripts/conv3x3_probe.py}
shift || true
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $set"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/$PROBE" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$R/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.txt" || exit $?
rm -rf "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4  # the raw counter CSVs exceed what gpurun copies back; the summary keeps the numbers
exit 0
