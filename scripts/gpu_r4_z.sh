# round 4, GPU call Z: ResNet launch reductions (BN zero-at-rest workspace + flat-grad dgamma/dbeta, 1x1 conv
# weight grads into the flat .grad, channels-last weight segments, MIOpen Find): the whole GPU suite, config 3
# twice, the GPT-2 bench once, a config-3 kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/z || exit 1
O=gpurun_out/z
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step gpu_suite 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu
grep -q " passed" $O/gpu_suite.log && ! grep -q " failed" $O/gpu_suite.log || exit 1
step cfg3_a 400 python -u bench_configs.py --configs 3 --steps 10
step cfg3_b 400 python -u bench_configs.py --configs 3 --steps 10
step bench 240 python -u bench.py
grep -h '"config"\|"metric"' $O/cfg3_*.log $O/bench.log >> $O/summary.txt
export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench_configs.py --configs 3 --steps 4
