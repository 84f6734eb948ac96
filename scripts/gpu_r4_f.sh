# round 4, GPU call F: fused-BN numerics vs the torch bf16 path + ResNet oracle per path; SSD tail A/B with
# the chain-only mode; config 4 kill-2-then-rejoin at 8 peers with staged admission (and without, A/B);
# steady-state 30k-frame video job with host spans. Each step has its own limit; a crash ends the script.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/f || exit 1
O=gpurun_out/f
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step bn_diag 240 python -u scripts/bn_diag.py
R="python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 440"
step rejoin_n8_staged 480 env VCX_ELASTIC_STAGE_JOINS=1 $R --json-out $O/rejoin_n8_staged.json
step rejoin_n8_unstaged 480 env VCX_ELASTIC_STAGE_JOINS=off $R --json-out $O/rejoin_n8_unstaged.json
step video_30k 900 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both
