# Round-3 video job benchmark on one MI355X: engine + network + the whole job through the
# coordinator on both data planes, input pre-generated into a memory-mapped .npy (RAM-backed).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3video
mkdir -p $O
timeout -k 10 500 python -u bench_video.py --frames ${FRAMES:-3000} --iters 10 > $O/bench.log 2>&1
rc=$?
grep '^{' $O/bench.log | tail -1 | cut -c1-2000
echo "bench_video rc=$rc"
exit $rc
