#!/bin/bash
# wgrad token-split probe, round 2: retune the committed power-of-two entries beside S = 13..15
set -o pipefail
mkdir -p gpurun_out/s
export TMPDIR=/tmp
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30
timeout -k 10 900 python -u scripts/wgrad_split_probe.py gpurun_out/s/tuned.csv --retune qkv=12,13,14,15,16 proj=14,16,20 fc=10,14,16 fc2=8,14,16 lm=2,4 > gpurun_out/s/probe.log 2>&1
