# round 4, GPU call T: the per-shape weight-gradient split table (config.wgrad_splits, qkv S = 14 with a
# leftover partial): its GPU tests, then interleaved 1-GPU bench runs, table on (default) vs off.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/t || exit 1
O=gpurun_out/t
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_train_gpu.py -k "wgrad" -m gpu
for i in 1 2 3; do
  step bench_on$i 240 python -u bench.py
  step bench_off$i 240 env VCX_WGRAD_SPLITS= python -u bench.py
done
grep -h '"metric"' $O/bench_*.log >> $O/summary.txt
