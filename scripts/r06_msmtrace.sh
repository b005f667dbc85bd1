#!/bin/bash
# round 6: kernel timeline of one 2^16 and one 2^20 MSM run (msmtune, default plan)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lg in 16 20; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mt$lg -o k -- python3 fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" > gpurun_out/mt$lg.log 2>&1 || { echo "trace $lg failed"; tail gpurun_out/mt$lg.log; exit 3; }
  f=$(find gpurun_out/mt$lg -name '*kernel_trace.csv' | head -1)
  python3 fabric-token-sdk_amd/tools/ktrace.py $f 30 > gpurun_out/mt${lg}_timeline.txt
  cat gpurun_out/mt$lg.log | grep n=2; cat gpurun_out/mt${lg}_timeline.txt
done
