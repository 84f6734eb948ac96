# Multi-row blob kernel A/B: vision GPU tests, then video_layers.py (blob kernel time, eager chunk)
# with VCX_BLOB_ROWS=1 (8 rows per workgroup, default) and 0 (one row per workgroup), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/blob
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vision_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_vision.log 2>&1
rc=$?; tail -n 2 $O/pytest_vision.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    VCX_BLOB_ROWS=$v timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/rows${v}_$r.log 2>&1 || exit $?
    echo "rows=$v r$r $(grep -h -o '"detect_chunk_ms": [0-9.]*, "mode": "eager"\|"kernel": "blob_bilinear[^}]*' $O/rows${v}_$r.log | tr '\n' ' ')"
  done
done
