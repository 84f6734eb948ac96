#!/bin/bash
# Counter passes over scripts/gemm_pmc_cmp.py (hand-written gemm_nt vs the library GEMM).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gemm_cmp
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU" "FETCH_SIZE"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $set"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/scripts/gemm_pmc_cmp.py" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
exit 0
