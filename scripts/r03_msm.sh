#!/bin/bash
# Engine + MSM GPU tests, MSM check at 2^20 / 2^24 (defaults), seam sweep, smoke + bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
TESTS="tests/test_gpu_engine.py tests/test_msm.py" TEST_TIMEOUT=600 SMOKE=0 BENCH=0 bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py 20 "0,0,0 0,0,0,1" > gpurun_out/msmtune20.log 2>&1 || { echo "msmtune20 failed"; tail -5 gpurun_out/msmtune20.log; exit 6; }
cat gpurun_out/msmtune20.log
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py 24 "0,0,0 0,0,0,1" > gpurun_out/msmtune24.log 2>&1 || { echo "msmtune24 failed"; tail -5 gpurun_out/msmtune24.log; exit 7; }
cat gpurun_out/msmtune24.log
timeout -k 10 400 python -u fabric-token-sdk_amd/tools/seamsweep.py "" "hold_inflight=0,window_us=300" "hold_inflight=0,window_us=300,small_pass=1024" "hold_inflight=0,window_us=500,small_pass=4096" > gpurun_out/seamsweep.log 2>&1 || { echo "seam sweep failed"; tail -20 gpurun_out/seamsweep.log; exit 3; }
echo "seam sweep ok"
SKIP_TESTS=1 bash scripts/gpu_check.sh || exit $?
