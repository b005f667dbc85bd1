#!/bin/bash
# round 6: kernel chain of one n = 1 verify call (scripts/r06_seamtrace.py under rocprofv3 --kernel-trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/seamtr -o k -- python3 scripts/r06_seamtrace.py > gpurun_out/seamtr.log 2>&1 || { echo "trace failed"; tail gpurun_out/seamtr.log; exit 3; }
grep "last call" gpurun_out/seamtr.log
python3 fabric-token-sdk_amd/tools/ktrace.py $(find gpurun_out/seamtr -name '*kernel_trace.csv' | head -1) 34
