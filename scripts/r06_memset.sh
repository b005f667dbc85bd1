#!/bin/bash
# round 6: MSM counts fused with the slot-count scan (new) vs the previous tree (prev)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06z_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z_tests.log; exit 4; }
tail -1 gpurun_out/r06z_tests.log
for r in 1 2 3; do
  for lg in 16 20; do
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" > gpurun_out/r06z_one.log 2>&1 || { echo "new $lg failed"; cat gpurun_out/r06z_one.log; exit 5; }
    echo "new  $(grep n=2 gpurun_out/r06z_one.log)"
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_prev.so > gpurun_out/r06z_one.log 2>&1 || { echo "prev $lg failed"; cat gpurun_out/r06z_one.log; exit 6; }
    echo "prev $(grep n=2 gpurun_out/r06z_one.log)"
  done
done
