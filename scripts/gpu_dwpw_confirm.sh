# Same-box confirmation of the conv1..conv3 persistent fused default vs the previous conv1-only fusion:
# per-layer timing + eager chunk (video_layers.py) and the video bench's network-only figure, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/dwpwc
mkdir -p $O
for r in 1 2; do
  for arm in "default:VCX_DWPW=tile" "conv1only:VCX_DWPW=tile1"; do
    name=${arm%%:*}; evs=$(echo "${arm#*:}" | tr ',' ' ')
    env $evs timeout -k 10 120 python -u scripts/video_layers.py 10 > $O/layers_${name}_$r.log 2>&1 || exit $?
    env $evs timeout -k 10 200 python -u bench_video.py --no-job --iters 20 > $O/bv_${name}_$r.log 2>&1 || exit $?
    echo "$name r$r $(grep -h -o '"detect_chunk_ms": [0-9.]*, "mode": "eager"' $O/layers_${name}_$r.log) $(grep -h -o '"net_only_chunk_ms": [0-9.]*' $O/bv_${name}_$r.log)"
  done
done
