# round 4, GPU call Y: BN kernels with a zero-at-rest workspace (finalize in the stats kernel's last block,
# dgamma / dbeta added into the flat .grad): model GPU tests, then ResNet-50 config 3 default vs MIOpen Find
# (cudnn.benchmark), interleaved, then a kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/y || exit 1
O=gpurun_out/y
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py -m gpu
grep -q " passed" $O/tests.log && ! grep -q " failed" $O/tests.log || exit 1
BENCHMARK='import runpy, sys, torch; torch.backends.cudnn.benchmark = True; sys.argv = ["bench_configs.py", "--configs", "3", "--steps", "10"]; runpy.run_path("bench_configs.py", run_name="__main__")'
for i in 1 2; do
  step default$i 400 python -u bench_configs.py --configs 3 --steps 10
  step find$i 600 python -u -c "$BENCHMARK"
done
grep -h '"config"' $O/default*.log $O/find*.log >> $O/summary.txt
export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench_configs.py --configs 3 --steps 4
