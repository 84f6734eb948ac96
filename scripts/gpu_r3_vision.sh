# Round-3 detector session: vision kernel tests, per-layer timing (events, eager), the graphed
# network time, and a rocprofv3 kernel-trace of the detector for true per-kernel GPU times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vision_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_vision.log 2>&1
rc=$?; tail -n 4 $O/pytest_vision.log; echo "pytest_vision rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_fused.log 2>&1 || exit $?
VCX_DWPW=off timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_unfused.log 2>&1 || exit $?
grep -h -E "total_ms|detect_chunk|resize" $O/layers_*.log
cd /tmp && export TMPDIR=/tmp
VCX_DWPW=off timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/video_layers.py 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo "rocprof rc=$?"
exit 0
