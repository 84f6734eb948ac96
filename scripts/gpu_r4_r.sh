#!/bin/bash
# wgrad token-split probe (scripts/wgrad_split_probe.py)
set -o pipefail
mkdir -p gpurun_out/r
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/wgrad_split_probe.py gpurun_out/r/tuned.csv > gpurun_out/r/probe.log 2>&1
