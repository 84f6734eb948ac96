#!/bin/bash
# Re-tune the library GEMM selection (TunableOp: every hipBLASLt + rocBLAS solution timed per
# shape) for the CURRENT bench step, then A/B the old table, the new table and no table, each
# twice, interleaved, in this one session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/tune
echo "[retune] tuning"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_gfx950.csv \
  VCX_TUNABLEOP=off timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --graph 0 > gpurun_out/tune/tune.log 2>&1
rc=$?; tail -2 gpurun_out/tune/tune.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
ls gpurun_out/tune; wc -l gpurun_out/tune/*.csv
NEW=$(ls gpurun_out/tune/tunableop_gfx950*.csv | head -1)
AB="old:VCX_TUNABLEOP=on new:VCX_TUNABLEOP_FILE=$NEW off:VCX_TUNABLEOP=off" ROUNDS=2 bash scripts/gpu_ab.sh
