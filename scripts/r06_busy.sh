#!/bin/bash
# round 6: GPU busy timeline of the headline job (bench.py --steps 20 --warmup 5, legs off) under a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/busy -o k -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb --no-extras > gpurun_out/busy.log 2>&1 || { echo "trace failed"; tail gpurun_out/busy.log; exit 3; }
tail -1 gpurun_out/busy.log | cut -c1-200
f=$(find gpurun_out/busy -name '*kernel_trace.csv' | head -1)
python3 fabric-token-sdk_amd/tools/kbusy.py $f 140 2
python3 fabric-token-sdk_amd/tools/ktrace.py $f 40 | tail -42
