# round 4, final GPU call (after the stem max-pool): the whole GPU test suite, smoke(), two 1-GPU bench runs, BASELINE configs 3/4/5, and the
# 8-rank RCCL rehearsal of the driver's multi-GPU path (bench direct, drop inside the all-to-all, kill-2-then-rejoin).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final3 || exit 1
O=gpurun_out/final3
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step gpu_suite 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench1 240 python -u bench.py
step bench2 240 python -u bench.py
step configs 600 python -u bench_configs.py --configs 3,4,5
ONLY="bench_n8_direct drop_collective_n8 drop_kill2_rejoin_n8" step rccl8 900 bash scripts/gpu_rccl8_rehearsal.sh
grep -h '"metric"\|"config"' $O/bench1.log $O/bench2.log $O/configs.log >> $O/summary.txt
