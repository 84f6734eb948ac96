# round 4, GPU call B: gemm_ps (nt stores) tests + bench; vision tests (fused SSD tail), tail A/B, detector
# kernel trace and rel-error probe; ResNet-50 tests (1x1 GEMM convs, fused BN), config-3 A/B and kernel table.
# A step that fails its checks (rc 1) lets the next one run; a timeout, abort or crash ends the call.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rn50 gpurun_out/b || exit 1
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> gpurun_out/b/summary.txt
  timeout -k 10 "$secs" "$@" > gpurun_out/b/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/b/summary.txt
  [ $rc -le 1 ] || exit $rc
}
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step gemm_ps_tests 200 $PT tests/test_gemm_ps_gpu.py
step gemm_ps_bench 200 python -u scripts/gemm_ps_bench.py
step vision_tests 300 $PT tests/test_vision_gpu.py
step det_rel_err 120 python -u scripts/detector_rel_err.py
step detprof 200 bash scripts/gpu_det_prof.sh
step rn50_tests 240 $PT tests/test_models_gpu.py -k "resnet or batchnorm"
for m in conv:torch gemm:fused conv:fused gemm:torch gemm:fused conv:torch; do
  export VCX_RESNET_CONV1X1=${m%:*} VCX_RESNET_BN=${m#*:}
  step "rn50_ab_${m/:/_}" 200 python -u bench_configs.py --configs 3 --steps 10
done
unset VCX_RESNET_CONV1X1 VCX_RESNET_BN
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rn50/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/bench_configs.py --configs 3 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/rn50/run.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && f=$(find gpurun_out/rn50/trace -name "*kernel_trace.csv" | head -1) && \
  python3 scripts/prof_step_generic.py "$f" 45 > gpurun_out/rn50/step_kernels.txt && rm -f "$f"
