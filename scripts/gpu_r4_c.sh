# round 4, GPU call C: headline bench (1 GPU) + GPT-2 step kernel table; the rest of the 8-rank rehearsal
# (butterfly / ring averaging, one of 8 peers SIGKILLed inside the all-to-all, kill 2 of 8 then rejoin)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c || exit 1
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> gpurun_out/c/summary.txt
  timeout -k 10 "$secs" "$@" > gpurun_out/c/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/c/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step bench1 300 python -u bench.py --steps 20 --warmup 8
step bench1b 300 python -u bench.py --steps 20 --warmup 8
step profstep 400 bash scripts/gpu_prof_step.sh
step attn_pmc 300 bash scripts/attn_pmc.sh
ONLY="bench_n8_butterfly bench_n8_ring drop_collective_n8 drop_kill2_rejoin_n8" timeout -k 10 900 bash scripts/gpu_rccl8_rehearsal.sh
