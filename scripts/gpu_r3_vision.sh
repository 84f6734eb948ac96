# Round-3 detector + GEMM study session: vision kernel tests (fused dw->pw, dot2 depthwise, LDS
# epilogue, detection_out values), per-layer timing fused vs unfused, then the 4-wave GEMM bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vision_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_vision.log 2>&1
rc=$?; tail -n 4 $O/pytest_vision.log; echo "pytest_vision rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_fused.log 2>&1 || exit $?
VCX_DWPW_MAX_COUT=0 timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_unfused.log 2>&1 || exit $?
VCX_DWPW_MAX_COUT=1024 timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_fuseall.log 2>&1 || exit $?
tail -n 1 $O/layers_*.log
if [ -n "$GEMM4" ]; then
  timeout -k 10 200 python -u scripts/gemm_p_bench.py --gemm4 > $O/gemm4.log 2>&1; echo "gemm4 rc=$?"
  tail -n 20 $O/gemm4.log
fi
