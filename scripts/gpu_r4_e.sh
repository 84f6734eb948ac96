# round 4, GPU call E: fused SSD tail v2 (128-deep steps, 8 waves) tests + A/B + kernel trace; ResNet tests
# (fused BN vs fp32, bottleneck oracle) verbose, every test run
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/e || exit 1
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> gpurun_out/e/summary.txt
  timeout -k 10 "$secs" "$@" > gpurun_out/e/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/e/summary.txt
  [ $rc -le 1 ] || exit $rc
}
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
step vision_tests 300 $PT -x tests/test_vision_gpu.py
step detprof 200 bash scripts/gpu_det_prof.sh
step rn50_tests 300 $PT -v tests/test_models_gpu.py -k "resnet or batchnorm"
