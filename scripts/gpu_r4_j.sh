# round 4, GPU call J: bench x2 (one-exp cross-entropy default), detector trace (no fill kernels), 30k-frame
# video job (npy sink, one-stage vs two-stage uplink interleaved), staged admission at 8 RCCL peers with the
# old communicator's shutdown deferred.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/j || exit 1
O=gpurun_out/j
step() {  # name, seconds, command...  (rc 1 = failed bench: logged, next step runs)
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step bench1 300 python -u bench.py
step bench2 300 python -u bench.py
step detprof 200 bash scripts/gpu_det_prof.sh
step video_ab 480 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both --uplink-ab
step cfg5_prof 480 bash scripts/gpu_r4_k.sh
R="python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 120"
step rejoin_n8_staged 200 env VCX_ELASTIC_STAGE_JOINS=all VCX_ELASTIC_DEBUG=1 $R --json-out $O/rejoin_n8_staged.json
