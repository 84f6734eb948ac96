# Elastic drop rehearsal with RCCL communicators on ONE GPU (one NCCL_HOSTID per peer, loopback
# sockets; functional + latency evidence, not xGMI bandwidth). PART=1: the RCCL GPU tests and a
# SIGKILL inside the averaging all-to-all (GPT-2-small, 3 peers x B=64); PART=2: SIGSTOP (lease
# bound) and kill-2-then-rejoin (4 peers). Each step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/drop3
mkdir -p $O
run() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -n 3 $O/$name.log | cut -c1-600
  echo "rc=$rc"
  return $rc
}
D="python -u bench_drop.py --backend nccl --model gpt2 --seq 1024 --steps 16 --warmup 4 --lease 2.0"
if [ "${PART:-1}" = 1 ]; then
  run pytest_rccl 400 python -u -m pytest tests/test_rccl_rehearsal_gpu.py -x -q --timeout 300 --timeout-method thread &&
  run kill_n3 500 $D --peers 3 --batch 64 --fault collective --timeout 460 --json-out $O/kill_n3.json
else
  run stop_n3 500 $D --peers 3 --batch 64 --fault stop --timeout 460 --json-out $O/stop_n3.json &&
  run kill2_rejoin_n4 600 $D --peers 4 --batch 32 --fault collective --drop-peers 2,3 --rejoin --timeout 560 \
      --json-out $O/kill2_rejoin_n4.json
fi
