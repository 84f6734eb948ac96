#!/bin/bash
# Round-3 A/B on one box: LayerNorm forward kernels (VCX_LN_FWD4) and the fused MLP (VCX_MLP) on the
# GPT-2-small headline bench and GPT-2-medium (config 4); the touched kernels' GPU tests first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_train_gpu.py tests/test_gemm_ps_gpu.py tests/test_gpt2_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  VCX_LN_FWD4=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b_ln$v.log 2>&1 || exit $?
  echo "ln_fwd4=$v $(grep -o '"value": [0-9.]*' $O/b_ln$v.log)"
done
for m in fused lib; do
  VCX_MLP=$m timeout -k 10 300 python -u bench_configs.py --configs 4 > $O/c4_$m.log 2>&1 || exit $?
  echo "config4 mlp=$m $(grep -o '"samples_per_s": [0-9.]*' $O/c4_$m.log)"
done
