# round 4, GPU call W: the bench step replayed as one hipGraph (default) vs eager launches, interleaved on one box.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/w || exit 1
O=gpurun_out/w
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
for i in 1 2 3; do
  step graph$i 240 python -u bench.py
  step eager$i 240 python -u bench.py --graph 0
done
for f in graph1 eager1 graph2 eager2 graph3 eager3; do echo "$f $(grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $O/$f.log)"; done >> $O/summary.txt
