# round 4, GPU call O: attention backward block order (VCX_ATTN_BWD_ORDER=1: every (batch, head)'s heaviest
# blocks first) -- tests under it, kernel A/B and bench A/B, interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/o || exit 1
O=gpurun_out/o
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step attn_tests_o1 300 env VCX_ATTN_BWD_ORDER=1 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_gpt2_gpu.py
for i in 1 2; do
  step attn_o0_$i 200 env VCX_ATTN_BWD_ORDER=0 python -u scripts/attn_variants.py
  step attn_o1_$i 200 env VCX_ATTN_BWD_ORDER=1 python -u scripts/attn_variants.py
done
for i in 1 2; do
  step bench_o0_$i 240 env VCX_ATTN_BWD_ORDER=0 python -u bench.py
  step bench_o1_$i 240 env VCX_ATTN_BWD_ORDER=1 python -u bench.py
done
