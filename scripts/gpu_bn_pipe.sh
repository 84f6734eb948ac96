#!/bin/bash
# BN reduction variants (VCX_BN_REDUCE; the default w512p against the round-6 w512q): correctness under the candidate, per-kernel times per shape
# (scripts/bn_prof.sh), then config 3 interleaved against the default.
set -o pipefail
CAND=${CAND:-w512p}
O=gpurun_out/${OUT:-bnpipe}
mkdir -p "$O"
VCX_BN_REDUCE=$CAND timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k "batchnorm or resnet" > "$O/tests.log" 2>&1 || exit $?
for v in w512q ${ARMS:-$CAND}; do VCX_BN_REDUCE=$v OUT=${OUT:-bnpipe}/$v bash scripts/bn_prof.sh || exit $?; done
for i in 1 2; do for v in w512q $CAND; do echo "$v $(VCX_BN_REDUCE=$v timeout -k 10 200 python bench_configs.py --configs 3 --steps 10 2>/dev/null | tail -1)" >> "$O/cfg3.log" || exit $?; done; done
