# round 4, GPU call L: TunableOp-tune the GPT-2 step's library GEMMs including the token-split batched
# weight gradients (scripts/tune_gemms.py), then interleaved 1-GPU bench runs: committed results file vs
# the freshly tuned one vs weight gradients on a side stream (VCX_ASYNC_WGRAD=1).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/l || exit 1
O=gpurun_out/l
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step tune 600 python -u scripts/tune_gemms.py $O/tunableop_gfx950.csv
[ -f $O/tunableop_gfx950.csv ] || exit 1
for i in 1 2; do
  step bench_old$i 240 python -u bench.py
  step bench_new$i 240 env VCX_TUNABLEOP_FILE=$GRAFT_REPO_ROOT/$O/tunableop_gfx950.csv python -u bench.py
  step bench_async$i 240 env VCX_ASYNC_WGRAD=1 python -u bench.py
done
