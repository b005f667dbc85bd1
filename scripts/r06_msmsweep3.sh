#!/bin/bash
# round 6: small-n MSM plans with the host Horner: planner default vs small windows / slot caps (2^14 .. 2^18)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lg in 14 15 16 17 18; do
  timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0 10,16,4,0,0,0 11,16,4,0,0,0 12,16,4,0,0,0 13,16,4,0,0,0 12,8,4,0,0,0 14,16,4,0,0,0 0,16,4,0,0,0 0,0,0,0,0,0" > gpurun_out/r06s3_$lg.log 2>&1 || { echo "sweep $lg failed"; tail gpurun_out/r06s3_$lg.log; exit 3; }
  cat gpurun_out/r06s3_$lg.log
done
