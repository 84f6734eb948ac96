#!/bin/bash
# Same-box A/B of the round-3 defaults against the round-2 compute path (VCX_MLP=lib, VCX_LN_FWD4=0),
# alternating arms so that clock drift hits both equally.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r3vr2; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/r3_$i.log 2>&1 || exit $?
  VCX_MLP=lib VCX_LN_FWD4=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/r2_$i.log 2>&1 || exit $?
  echo "run $i  r3 $(grep -o '"value": [0-9.]*' $O/r3_$i.log)  r2-path $(grep -o '"value": [0-9.]*' $O/r2_$i.log)"
done
