#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/tune
timeout -k 10 300 python bench.py --steps 8 --warmup 4 > gpurun_out/tune/base.log 2>&1 && tail -1 gpurun_out/tune/base.log &&
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv \
  timeout -k 10 900 python bench.py --steps 8 --warmup 4 > gpurun_out/tune/tune.log 2>&1 && tail -1 gpurun_out/tune/tune.log &&
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv \
  timeout -k 10 300 python bench.py --steps 8 --warmup 4 > gpurun_out/tune/tuned.log 2>&1 && tail -1 gpurun_out/tune/tuned.log &&
timeout -k 10 300 python bench.py --steps 8 --warmup 4 --batch 64 > gpurun_out/tune/b64.log 2>&1 && tail -1 gpurun_out/tune/b64.log
