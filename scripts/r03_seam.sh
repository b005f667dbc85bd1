#!/bin/bash
# Seam sweep (engine options) then GPU tests + smoke + default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
timeout -k 10 400 python -u fabric-token-sdk_amd/tools/seamsweep.py "" "hold_inflight=1" "small_pass=1024" "small_pass=4096" "small_pass=4096,hold_inflight=1" "small_pass=4096,window_us=500" > gpurun_out/seamsweep.log 2>&1 || { echo "seam sweep failed"; tail -20 gpurun_out/seamsweep.log; exit 3; }
echo "seam sweep ok"
bash scripts/gpu_check.sh || exit $?
