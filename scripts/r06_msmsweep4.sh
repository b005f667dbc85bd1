#!/bin/bash
# round 6: MSM plans at 2^19 / 2^20 with the host Horner (window bits x slot cap x segment slots)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lg in 19 20; do
  timeout -k 10 400 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0 13,16,4,0,0,0 14,16,4,0,0,0 15,16,4,0,0,0 16,16,4,0,0,0 17,16,4,0,0,0 13,32,8,0,0,0 15,32,8,0,0,0 17,32,8,0,0,0 13,16,8,0,0,0 15,16,8,0,0,0 0,0,0,0,0,0" > gpurun_out/r06s4_$lg.log 2>&1 || { echo "sweep $lg failed"; tail gpurun_out/r06s4_$lg.log; exit 3; }
  cat gpurun_out/r06s4_$lg.log
done
