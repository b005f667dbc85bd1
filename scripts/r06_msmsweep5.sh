#!/bin/bash
# round 6: odd vs even window bits at 2^21 / 2^22 (planner default c = 18 there)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lg in 21 22; do
  timeout -k 10 400 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0 17,0,0,0,0,0 19,0,0,0,0,0 18,0,0,0,0,0 0,0,0,0,0,0" > gpurun_out/r06s5_$lg.log 2>&1 || { echo "sweep $lg failed"; tail gpurun_out/r06s5_$lg.log; exit 3; }
  cat gpurun_out/r06s5_$lg.log
done
