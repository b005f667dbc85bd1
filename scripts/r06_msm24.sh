#!/bin/bash
# round 6: window bits at 2^23 / 2^24 with the host window combination
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u fabric-token-sdk_amd/tools/msmtune.py 24 "0,0,0,0,0,0 20,0,0,0,0,0 21,0,0,0,0,0 22,0,0,0,0,0 18,0,0,0,0,0 0,0,0,0,0,0" > gpurun_out/r06m24.log 2>&1 || { echo "24 failed"; tail gpurun_out/r06m24.log; exit 3; }
cat gpurun_out/r06m24.log
timeout -k 10 500 python -u fabric-token-sdk_amd/tools/msmtune.py 23 "0,0,0,0,0,0 17,0,0,0,0,0 20,0,0,0,0,0 21,0,0,0,0,0 0,0,0,0,0,0" > gpurun_out/r06m23.log 2>&1 || { echo "23 failed"; tail gpurun_out/r06m23.log; exit 4; }
cat gpurun_out/r06m23.log
