#!/bin/bash
# round 6: MSM known-log tests and default-plan latency 2^14 .. 2^24 after the variable-base plan rule
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06p_tests.log; exit 4; }
tail -2 gpurun_out/r06p_tests.log
for lg in 14 15 16 17 18 19 20 21 22 23 24; do
  timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0 0,0,0,0,0,0" > gpurun_out/r06p_$lg.log 2>&1 || { echo "msmtune $lg failed"; tail gpurun_out/r06p_$lg.log; exit 5; }
  grep n=2 gpurun_out/r06p_$lg.log
done
