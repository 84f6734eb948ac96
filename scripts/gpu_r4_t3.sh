# round 4, GPU call T3: TunableOp-tune the GEMMs of BASELINE config 4 (GPT-2-medium) on top of the committed table
# (configs 4 + 5 together did not finish in 900 s: Llama-3-8B's shapes tune slowly), then config 4 with the committed
# table vs the extended one, interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/t3 || exit 1
O=gpurun_out/t3
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10
step tune 700 python -u scripts/tune_config_gemms.py $O/tunableop_gfx950.csv 4
unset PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS
[ -f $O/tunableop_gfx950.csv ] || exit 1
for i in 1 2; do
  step old$i 200 python -u bench_configs.py --configs 4
  step new$i 200 env VCX_TUNABLEOP_FILE=$GRAFT_REPO_ROOT/$O/tunableop_gfx950.csv python -u bench_configs.py --configs 4
done
for f in old1 new1 old2 new2; do grep -h '"config"' $O/$f.log | sed "s/^/$f /"; done >> $O/summary.txt
