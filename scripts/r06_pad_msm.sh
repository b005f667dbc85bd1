#!/bin/bash
# round 6: LDS region padding A/B (FTS_SQ_PAD 20 vs 0) and MSM graph replay / tree levels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_msm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06c_tests.log; exit 3; }
echo tests ok
for lg in 16 20 24; do
  timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,1 0,0,0,0,0,0 0,0,0,0,0,1 0,0,0,0,0,0" >> gpurun_out/r06c_msm.log 2>&1 || { echo "msmtune $lg failed"; tail -20 gpurun_out/r06c_msm.log; exit 4; }
done
echo msm ok
LIBS="new=default|old=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_pad0.so" bash scripts/pmc_lds.sh > gpurun_out/r06c_pmc.log 2>&1 || { echo pmc failed; exit 5; }
LIBS="new=default|old=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_pad0.so" ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/r06c_ab.log 2>&1 || { echo ab failed; exit 6; }
echo all ok
