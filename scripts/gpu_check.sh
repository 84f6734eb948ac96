#!/bin/bash
# Focused GPU check: selected GPU tests, attention micro-bench, eager + hipGraph bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_attention_gpu.py tests/test_kernels_train_gpu.py tests/test_gpt2_gpu.py"}
echo "[gpu_check] pytest $TESTS"
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest $TESTS -x -q > gpurun_out/check_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/check_pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
if [ "${ATTN:-1}" = "1" ]; then
  echo "[gpu_check] attention micro-bench"
  timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1
  rc=$?; cat gpurun_out/attn_bench.log | cut -c1-120; [ $rc -ne 0 ] && { echo "attn rc=$rc"; exit $rc; }
fi
echo "[gpu_check] bench (eager)"
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
if [ "${GRAPH:-1}" = "1" ]; then
  echo "[gpu_check] bench (hipGraph)"
  timeout -k 10 300 python bench.py --graph 1 ${BENCH_ARGS:-} > gpurun_out/bench_graph.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_graph.log | cut -c1-300; exit $rc
fi
