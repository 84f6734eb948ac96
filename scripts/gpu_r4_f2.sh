# round 4, GPU call F2: config 4 kill-2-then-rejoin at 8 RCCL peers on one card with staged admission
# (membership trace on) and without it, then the steady-state 30k-frame video job with host spans.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/f2 || exit 1
O=gpurun_out/f2
step() {  # name, seconds, command...  (rc 1 = a failed bench: logged, next step runs)
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
R="python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 150"
step rejoin_n8_staged 240 env VCX_ELASTIC_STAGE_JOINS=all VCX_ELASTIC_DEBUG=1 $R --json-out $O/rejoin_n8_staged.json
step rejoin_n8_unstaged 240 env VCX_ELASTIC_STAGE_JOINS=off $R --json-out $O/rejoin_n8_unstaged.json
step video_30k 900 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both
