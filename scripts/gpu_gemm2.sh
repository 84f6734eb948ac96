#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/gemm
O=gpurun_out/gemm
cp tuning/tunableop_gfx950.csv $O/old0.csv
PROBE_SPLITS=2,4,8,16 PROBE_TAG=split PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/old%d.csv \
  timeout -k 10 400 python scripts/gemm_probe.py > $O/split.log 2>&1; rc=$?
tail -1 $O/split.log; exit $rc
