# round 4, GPU call T2: TunableOp-tune the ResNet-50 step's library GEMMs, then config 3 with the committed table
# vs the extended one, interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/t2 || exit 1
O=gpurun_out/t2
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step tune 700 python -u scripts/tune_config_gemms.py $O/tunableop_gfx950.csv
[ -f $O/tunableop_gfx950.csv ] || exit 1
for i in 1 2; do
  step old$i 300 python -u bench_configs.py --configs 3 --steps 10
  step new$i 300 env VCX_TUNABLEOP_FILE=$GRAFT_REPO_ROOT/$O/tunableop_gfx950.csv python -u bench_configs.py --configs 3 --steps 10
done
for f in old1 new1 old2 new2; do echo "$f $(grep -h '"config"' $O/$f.log)"; done >> $O/summary.txt
