set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 16 --warmup 8 > gpurun_out/bench.log 2>&1; tail -2 gpurun_out/bench.log
