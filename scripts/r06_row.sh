#!/bin/bash
# round 6: row-distributed Horner chain (FTS_MSM_ROW_HORNER 1 vs 0 = variant hq)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python fabric-token-sdk_amd/tools/rowbench.py > gpurun_out/r06g_rowbench.log 2>&1 || { echo rowbench failed; tail gpurun_out/r06g_rowbench.log; exit 3; }
cat gpurun_out/r06g_rowbench.log
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_msm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06g_tests.log; exit 4; }
echo tests ok
for r in 1 2; do
  for lg in 16 20 24; do
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" >> gpurun_out/r06g_msm_row.log 2>&1 || { echo "msmtune row $lg failed"; exit 5; }
    timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_hq.so >> gpurun_out/r06g_msm_hq.log 2>&1 || { echo "msmtune hq $lg failed"; exit 6; }
  done
done
echo row; grep "n=2" gpurun_out/r06g_msm_row.log; echo old; grep "n=2" gpurun_out/r06g_msm_hq.log
