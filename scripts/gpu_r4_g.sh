# round 4, GPU call G: pipelined attention forward (tests + A/B), every GEMM of the GPT-2 step by shape,
# the whole GPU test suite, and two 1-GPU bench runs. Each step has its own limit; a crash ends it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g || exit 1
O=gpurun_out/g
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
step attn_tests 300 $PT -x tests/test_attention_gpu.py
step attn_variants 300 python -u scripts/attn_variants.py
step gemm_shapes 400 python -u scripts/gemm_step_shapes.py
step gpu_suite 900 $PT tests/ -m gpu
step bench1 300 python -u bench.py
step bench2 300 python -u bench.py
