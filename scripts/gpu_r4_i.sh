# round 4, GPU call I: the whole GPU test suite on the current tree, the 30k-frame video job with the
# two-stage uplink on/off interleaved, then staged admission at 8 RCCL peers (stack dumps if it hangs).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/i || exit 1
O=gpurun_out/i
step() {  # name, seconds, command...  (rc 1 = failed tests / bench: logged, next step runs)
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step gpu_suite 660 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu
step xent_0a 120 env VCX_XENT_KEEP_E=0 python -u scripts/xent_ab.py
step xent_1a 120 env VCX_XENT_KEEP_E=1 python -u scripts/xent_ab.py
step xent_0b 120 env VCX_XENT_KEEP_E=0 python -u scripts/xent_ab.py
step xent_1b 120 env VCX_XENT_KEEP_E=1 python -u scripts/xent_ab.py
step video_ab 420 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both --uplink-ab
R="python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 120"
step rejoin_n8_staged 200 env VCX_ELASTIC_STAGE_JOINS=all VCX_ELASTIC_DEBUG=1 $R --json-out $O/rejoin_n8_staged.json
