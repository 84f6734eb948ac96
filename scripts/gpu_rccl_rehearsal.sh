# RCCL multi-rank rehearsal on a one-GPU box (scripts/rccl_rehearsal_launch.py: one NCCL_HOSTID per
# rank, loopback sockets). Runs the headline bench at 2/4 ranks over every averaging algorithm and
# the elastic drop bench with RCCL communicators (abort inside the all-to-all, SIGSTOP, kill-2 +
# rejoin). ONLY=drop runs the drop steps alone. Each step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rccl
mkdir -p $O
L="python -u scripts/rccl_rehearsal_launch.py"
B="python -u bench.py --steps 8 --warmup 4 --batch 4 --seq 256"
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "== $name" | tee -a $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -h '"metric"' $O/$name.log $O/$name/rank0.out 2>/dev/null | tail -n 1 >> $O/summary.txt
  echo "rc=$rc" | tee -a $O/summary.txt
  return $rc
}
{ [ "$ONLY" = drop ] || {
step bench_n2_direct_graph 240 $L --nproc 2 --timeout 220 --log-dir $O/bench_n2_direct_graph -- $B --gpus 2 --algo direct &&
step bench_n4_direct_graph 300 $L --nproc 4 --timeout 280 --log-dir $O/bench_n4_direct_graph -- $B --gpus 4 --algo direct &&
step bench_n4_butterfly 300 $L --nproc 4 --timeout 280 --log-dir $O/bench_n4_butterfly -- $B --gpus 4 --algo butterfly &&
step bench_n3_ring 300 $L --nproc 3 --timeout 280 --log-dir $O/bench_n3_ring -- $B --gpus 3 --algo ring &&
step bench_n3_rsag 300 $L --nproc 3 --timeout 280 --log-dir $O/bench_n3_rsag -- $B --gpus 3 --algo rs_ag; }; } &&
step drop_collective_n3 300 python -u bench_drop.py --peers 3 --backend nccl --model gpt2-tiny --batch 4 --seq 128 \
  --steps 16 --warmup 4 --fault collective --lease 2.0 --timeout 240 --json-out $O/drop_collective_n3.json &&
step drop_stop_n3 300 python -u bench_drop.py --peers 3 --backend nccl --model gpt2-tiny --batch 4 --seq 128 \
  --steps 16 --warmup 4 --fault stop --lease 2.0 --timeout 240 --json-out $O/drop_stop_n3.json &&
step drop_kill2_rejoin_n4 360 python -u bench_drop.py --peers 4 --backend nccl --model gpt2-tiny --batch 4 --seq 128 \
  --steps 16 --warmup 4 --fault collective --drop-peers 2,3 --rejoin --lease 2.0 --timeout 300 \
  --json-out $O/drop_kill2_rejoin_n4.json
