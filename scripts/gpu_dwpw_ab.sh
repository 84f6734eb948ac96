# Persistent fused depthwise->pointwise kernel (dwpw_persist_kernel) A/B: vision GPU tests, then the
# detector's per-layer timing and chunk time for conv1-only / conv1..conv3 fusion, persistent or
# one tile per workgroup, two interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/dwpw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vision_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_vision.log 2>&1
rc=$?; tail -n 2 $O/pytest_vision.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for arm in "p1:VCX_DWPW_PERSIST=1" "p0:VCX_DWPW_PERSIST=0" "t3p1:VCX_DWPW=tile3,VCX_DWPW_PERSIST=1" "t3p0:VCX_DWPW=tile3,VCX_DWPW_PERSIST=0" "off:VCX_DWPW=off"; do
    name=${arm%%:*}; evs=$(echo "${arm#*:}" | tr ',' ' ')
    env $evs timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/${name}_$r.log 2>&1 || exit $?
    echo "$name r$r $(grep -h -o '"detect_chunk_ms": [0-9.]*, "mode": "eager"\|"dwpw": [0-9.]*\|"dw": [0-9.]*\|"pw": [0-9.]*' $O/${name}_$r.log | tr '\n' ' ')"
  done
done
