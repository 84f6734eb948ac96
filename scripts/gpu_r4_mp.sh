# round 4, GPU call MP: HIP stem max-pool (uint8 window index, gather backward): model tests, then config 3 twice.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mp || exit 1
O=gpurun_out/mp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py -m gpu
grep -q " passed" $O/tests.log && ! grep -q " failed" $O/tests.log || exit 1
step cfg3_a 300 python -u bench_configs.py --configs 3 --steps 10
step cfg3_b 300 python -u bench_configs.py --configs 3 --steps 10
grep -h '"config"' $O/cfg3_*.log >> $O/summary.txt
