#!/bin/bash
# round 6: kernel timelines of one 2^16 MSM for several plans (msmtune combos: C,T,S,P,R,G)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for combo in "12,16,4,0,0,0" "9,16,4,0,0,0" "10,16,4,0,0,0"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mt2_$i -o k -- python3 fabric-token-sdk_amd/tools/msmtune.py 16 "$combo" > gpurun_out/mt2_$i.log 2>&1 || { echo "trace $combo failed"; tail gpurun_out/mt2_$i.log; exit 3; }
  f=$(find gpurun_out/mt2_$i -name '*kernel_trace.csv' | head -1)
  echo "== $combo"; grep n=2 gpurun_out/mt2_$i.log
  python3 fabric-token-sdk_amd/tools/ktrace.py $f 32
done
