# The driver's 8-GPU path rehearsed at P = 8 on ONE GPU (VERDICT r3 missing #2/#3): 8 RCCL ranks, one
# NCCL_HOSTID each (scripts/rccl_rehearsal_launch.py; the communicators run over loopback sockets, the
# c10d/RCCL code paths are the ones the 8-GPU run takes). bench.py with the direct / butterfly / ring
# averaging, bench_drop with one of 8 peers SIGKILLed inside the all-to-all, and config 4's kill-2-then-
# rejoin at 8 peers (per-joiner admission time). Each step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rccl8
mkdir -p $O
L="python -u scripts/rccl_rehearsal_launch.py"
B="python -u bench.py --steps 8 --warmup 4 --batch 8"
step() {  # name, seconds, command... (ONLY="name1 name2": run just those)
  local name=$1 secs=$2
  shift 2
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  echo "== $name $(date +%T)" | tee -a $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -h '"metric"' $O/$name.log $O/$name/rank0.out 2>/dev/null | tail -n 1 >> $O/summary.txt
  echo "rc=$rc" | tee -a $O/summary.txt
  return $rc
}
step bench_n8_direct 420 $L --nproc 8 --timeout 400 --log-dir $O/bench_n8_direct -- $B --gpus 8 --algo direct &&
step bench_n8_butterfly 420 $L --nproc 8 --timeout 400 --log-dir $O/bench_n8_butterfly -- $B --gpus 8 --algo butterfly &&
step bench_n8_ring 420 $L --nproc 8 --timeout 400 --log-dir $O/bench_n8_ring -- $B --gpus 8 --algo ring &&
step drop_collective_n8 420 python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 \
  --steps 16 --warmup 4 --fault collective --lease 2.0 --timeout 380 --json-out $O/drop_collective_n8.json &&
step drop_kill2_rejoin_n8 480 python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 \
  --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 440 \
  --json-out $O/drop_kill2_rejoin_n8.json
