# round 4, GPU call N: vision tests (DetectionOutput parameters parsed at plan build) and the pointwise-GEMM
# A/B of the detector (nt / vision / auto).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/n || exit 1
O=gpurun_out/n
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)" >> $O/summary.txt
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit $rc
}
step vision_tests 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_vision_gpu.py
step pw_ab 240 python -u scripts/pw_gemm_ab.py
