#!/bin/bash
# round 6: counting sort for small MSM plans vs rocPRIM radix sort (variant rsort); GPU MSM tests; 2^16 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06c_tests.log; exit 4; }
tail -1 gpurun_out/r06c_tests.log
for r in 1 2; do
  for lg in 14 16 17 18; do
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" > gpurun_out/r06c_one.log 2>&1 || { echo "csort $lg failed"; cat gpurun_out/r06c_one.log; exit 5; }
    echo "csort $(grep n=2 gpurun_out/r06c_one.log)"
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_rsort.so > gpurun_out/r06c_one.log 2>&1 || { echo "rsort $lg failed"; cat gpurun_out/r06c_one.log; exit 6; }
    echo "rsort $(grep n=2 gpurun_out/r06c_one.log)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mtc16 -o k -- python3 fabric-token-sdk_amd/tools/msmtune.py 16 "0,0,0,0,0,0" > gpurun_out/mtc16.log 2>&1 || { echo "trace failed"; exit 3; }
python3 fabric-token-sdk_amd/tools/ktrace.py $(find gpurun_out/mtc16 -name '*kernel_trace.csv' | head -1) 18
