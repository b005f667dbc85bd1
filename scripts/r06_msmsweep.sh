#!/bin/bash
# round 6: MSM plan sweep with the host Horner (window bits, slot cap, segment slots)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py 16 "0,0,0,0,0,0 12,0,0,0,0,0 13,0,0,0,0,0 14,0,0,0,0,0 16,0,0,0,0,0 15,8,0,0,0,0 15,32,0,0,0,0 15,0,2,0,0,0 15,0,8,0,0,0 14,0,2,0,0,0 13,0,2,0,0,0 13,0,8,0,0,0 0,0,0,0,0,1" > gpurun_out/r06s_16.log 2>&1 || { echo "16 failed"; tail gpurun_out/r06s_16.log; exit 3; }
cat gpurun_out/r06s_16.log
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py 20 "0,0,0,0,0,0 15,0,0,0,0,0 16,0,0,0,0,0 18,0,0,0,0,0 17,0,8,0,0,0 17,0,32,0,0,0 17,16,0,0,0,0 17,64,0,0,0,0" > gpurun_out/r06s_20.log 2>&1 || { echo "20 failed"; tail gpurun_out/r06s_20.log; exit 4; }
cat gpurun_out/r06s_20.log
