# Round-3 elastic rehearsals on ONE GPU (RCCL over loopback sockets, one NCCL_HOSTID per peer):
# PART=1: the RCCL GPU tests, a SIGKILL inside the averaging all-to-all (GPT-2-small, 3 peers x
# B=64, lease 2 s) and the sharded re-shard rehearsal (Llama-3.2-1B, 3 -> 2 peers, replicas=1).
# PART=2: SIGSTOP (lease-bound) and kill-2-then-rejoin (4 peers).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/el3
mkdir -p $O
run() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -n 3 $O/$name.log | cut -c1-800
  echo "rc=$rc"
  return $rc
}
D="python -u bench_drop.py --backend nccl --model gpt2 --seq 1024 --steps 16 --warmup 4 --lease 2.0"
if [ "${PART:-1}" = 1 ]; then
  run pytest_rccl 300 python -u -m pytest tests/test_rccl_rehearsal_gpu.py -x -q --timeout 240 --timeout-method thread &&
  run kill_n3 400 $D --peers 3 --batch 64 --fault collective --timeout 380 --json-out $O/kill_n3.json &&
  run reshard_n3 300 python -u scripts/rccl_rehearsal_launch.py --nproc 3 --expect-killed 2 --timeout 280 \
      --log-dir $O/reshard -- python -u scripts/reshard_rehearsal.py --model llama3.2-1b --seq 2048 --steps 8 --kill-at 4
  rc=$?
  cat $O/reshard/rank0.out $O/reshard/rank1.out 2>/dev/null | grep '^{' | cut -c1-600
  exit $rc
else
  run stop_n3 400 $D --peers 3 --batch 64 --fault stop --timeout 380 --json-out $O/stop_n3.json &&
  run kill2_rejoin_n4 500 $D --peers 4 --batch 32 --fault collective --drop-peers 2,3 --rejoin --timeout 480 \
      --json-out $O/kill2_rejoin_n4.json
fi
