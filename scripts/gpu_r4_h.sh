# round 4, GPU call H: staged admission at 8 RCCL peers (init deferred to after the staged round's commit),
# every GEMM of the GPT-2 step by shape, and the 30k-frame video job with the two-stage uplink on/off
# interleaved (same process, same box).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/h || exit 1
O=gpurun_out/h
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
step gemm_shapes 400 python -u scripts/gemm_step_shapes.py
step video_ab 900 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both --uplink-ab
