#!/bin/bash
# One GPU-box session: GPU tests, probes, 1-GPU bench and a kernel-trace profile. Every GPU step
# runs under its own time limit; a crash/timeout (rc > 1) ends the session, a plain test failure
# (pytest rc 1) does not.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: output to gpurun_out/<name>.log
  local name=$1 t=$2; shift 2
  echo "[session] $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAIL:-4} "gpurun_out/$name.log" | cut -c1-400
  echo "[session] $name rc=$rc"
  if [ $rc -gt 1 ]; then echo "[session] stopping after $name"; exit $rc; fi
  return 0
}
if [ "${PYTEST:-1}" = "1" ]; then
  step pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 180 --timeout-method thread
fi
for p in ${PROBES:-}; do
  TAIL=40 step "probe_$(basename $p .py)" 400 python -u $p
done
if [ "${BENCH:-1}" = "1" ]; then
  step bench 500 python -u bench.py --steps ${STEPS:-16} --warmup 8 ${BENCH_ARGS:-}
fi
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  echo "[session] rocprofv3 kernel trace"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
      python3 "$R/bench.py" --steps 4 --warmup 3 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; tail -2 "$R/gpurun_out/prof.log" | cut -c1-300; echo "[session] rocprof rc=$rc"; exit $rc
fi
