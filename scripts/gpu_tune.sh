#!/bin/bash
# GPU tests + hipBLASLt/rocBLAS GEMM selection (TunableOp) for the bench shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/tune
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_gfx950.csv
for B in ${BATCHES:-64}; do
  VCX_TUNABLEOP=off timeout -k 10 900 python bench.py --steps 2 --warmup 1 --batch $B > gpurun_out/tune/tune_b$B.log 2>&1 || exit $?
  tail -1 gpurun_out/tune/tune_b$B.log | cut -c1-200
done
unset PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_FILENAME PYTORCH_TUNABLEOP_ENABLED
