# round 4, GPU call G: pipelined attention forward (tests + A/B), every GEMM of the GPT-2 step by shape,
# the whole GPU test suite, and two 1-GPU bench runs. Each step has its own limit; a crash ends it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g || exit 1
O=gpurun_out/g
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
step attn_tests 300 $PT -x tests/test_attention_gpu.py
step attn_variants 300 python -u scripts/attn_variants.py
step gemm_shapes 400 python -u scripts/gemm_step_shapes.py
step detprof 200 bash scripts/gpu_det_prof.sh
step bench1 300 python -u bench.py
step bench2 300 python -u bench.py
R="python -u bench_drop.py --peers 8 --backend nccl --model gpt2 --batch 2 --seq 256 --steps 16 --warmup 4 --fault collective --drop-peers 6,7 --rejoin --lease 2.0 --timeout 150"
step rejoin_n8_staged 240 env VCX_ELASTIC_STAGE_JOINS=all VCX_ELASTIC_DEBUG=1 $R --json-out $O/rejoin_n8_staged.json
step video_30k 600 python -u bench_video.py --frames 30000 --source-frames 3000 --job-repeats 3 --data-plane both
