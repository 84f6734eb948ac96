#!/bin/bash
# One GPU-box session: GPU tests, 1-GPU bench, kernel-trace profile. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEPS=${STEPS:-16}
echo "[gpu_round] pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
echo "[gpu_round] bench"
timeout -k 10 600 python bench.py --steps $STEPS --warmup 8 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
if [ "${PROFILE:-1}" = "1" ]; then
  echo "[gpu_round] rocprofv3"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
      python3 "$R/bench.py" --steps 4 --warmup 3 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; tail -3 "$R/gpurun_out/prof.log"; exit $rc
fi
