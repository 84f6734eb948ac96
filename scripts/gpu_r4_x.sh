# round 4, GPU call X: ResNet-50 (config 3) with MIOpen's default (immediate-mode) solver choice vs
# torch.backends.cudnn.benchmark (MIOpen Find per convolution shape), interleaved; then a kernel trace of the
# default arm.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/x || exit 1
O=gpurun_out/x
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
BENCHMARK='import runpy, sys, torch; torch.backends.cudnn.benchmark = True; sys.argv = ["bench_configs.py", "--configs", "3", "--steps", "10"]; runpy.run_path("bench_configs.py", run_name="__main__")'
for i in 1 2; do
  step default$i 400 python -u bench_configs.py --configs 3 --steps 10
  step find$i 600 python -u -c "$BENCHMARK"
done
grep -h '"config"' $O/default*.log $O/find*.log >> $O/summary.txt
export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench_configs.py --configs 3 --steps 4
