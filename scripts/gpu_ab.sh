#!/bin/bash
# A/B of bench.py under different environment settings in ONE GPU session (same device, same
# thermal state): AB="NAME1:VAR=val,VAR2=val NAME2:VAR=val ..." ; each arm runs ROUNDS times,
# interleaved. An ARGS=... entry (spaces written as +) adds bench.py arguments to that arm only.
# Results: gpurun_out/ab_<name>_<round>.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in $AB; do
    name=${arm%%:*}; envs=${arm#*:}
    args=""; evs=""
    for kv in $(echo "$envs" | tr ',' ' '); do
      case $kv in ARGS=*) args=$(echo "${kv#ARGS=}" | tr '+' ' ');; *) evs="$evs $kv";; esac
    done
    echo "[ab] round $r arm $name ($evs | $args)"
    env $evs timeout -k 10 300 python -u bench.py --steps ${STEPS:-16} --warmup 8 ${BENCH_ARGS:-} $args \
        > "gpurun_out/ab_${name}_${r}.log" 2>&1
    rc=$?
    grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gemm_lt_shapes": [0-9]*' "gpurun_out/ab_${name}_${r}.log" | tr '\n' ' '; echo
    [ $rc -ne 0 ] && { tail -5 "gpurun_out/ab_${name}_${r}.log"; exit $rc; }
  done
done
exit 0
