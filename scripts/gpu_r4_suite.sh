# the whole GPU test suite, one process, per-test timeout (round-end tier rehearsal)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/suite || exit 1
timeout -k 10 1100 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/suite/gpu_suite.log 2>&1
echo "rc=$?" >> gpurun_out/suite/gpu_suite.log
