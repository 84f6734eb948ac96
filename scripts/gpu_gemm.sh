#!/bin/bash
# GEMM selection study: library defaults vs the committed TunableOp table vs a retune with a
# rotating buffer (cold caches, as in a training step). Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/gemm
O=gpurun_out/gemm
echo "[gemm] library defaults"
PROBE_TAG=default timeout -k 10 300 python scripts/gemm_probe.py > $O/default.log 2>&1; rc=$?
tail -1 $O/default.log; [ $rc -ne 0 ] && exit $rc
echo "[gemm] committed table"
cp tuning/tunableop_gfx950.csv $O/old0.csv
PROBE_TAG=table PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/old%d.csv \
  timeout -k 10 300 python scripts/gemm_probe.py > $O/table.log 2>&1; rc=$?
tail -1 $O/table.log; [ $rc -ne 0 ] && exit $rc
echo "[gemm] retune, rotating buffer ${ROT:-1024} MB"
PROBE_TAG=tuning PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/new%d.csv \
  PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=${ROT:-1024} timeout -k 10 1200 python scripts/gemm_probe.py > $O/tuning.log 2>&1; rc=$?
tail -1 $O/tuning.log; [ $rc -ne 0 ] && exit $rc
echo "[gemm] retuned table"
PROBE_TAG=retuned PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/new%d.csv \
  timeout -k 10 300 python scripts/gemm_probe.py > $O/retuned.log 2>&1; rc=$?
tail -1 $O/retuned.log; exit $rc
