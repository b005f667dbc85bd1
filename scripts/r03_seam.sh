#!/bin/bash
# idemix GPU tests, seam sweep (engine options), then smoke + default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
TESTS=tests/test_idemix.py SMOKE=0 BENCH=0 TEST_TIMEOUT=300 bash scripts/gpu_check.sh || exit $?
timeout -k 10 400 python -u fabric-token-sdk_amd/tools/seamsweep.py "" "hold_inflight=1" "small_pass=1024" "small_pass=4096" "small_pass=4096,hold_inflight=1" "small_pass=4096,window_us=500" > gpurun_out/seamsweep.log 2>&1 || { echo "seam sweep failed"; tail -20 gpurun_out/seamsweep.log; exit 3; }
echo "seam sweep ok"
SKIP_TESTS=1 bash scripts/gpu_check.sh || exit $?
