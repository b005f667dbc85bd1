#!/bin/bash
# Fexp/engine GPU tests, serial trace + PMC passes (profiles r03k), seam A/B, smoke + bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
timeout -k 10 200 python -u fabric-token-sdk_amd/tools/provebench.py --steps 16 > gpurun_out/prover_fresh.log 2>&1 || { echo "provebench failed"; tail -20 gpurun_out/prover_fresh.log; exit 8; }
cat gpurun_out/prover_fresh.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prover -o k -- python3 fabric-token-sdk_amd/tools/provebench.py --steps 4 --serial > gpurun_out/prof_prover.log 2>&1 || { echo "prover trace failed"; tail -20 gpurun_out/prof_prover.log; exit 9; }
echo "prover trace ok"
TESTS="tests/test_gpu_engine.py tests/test_gpu.py" TEST_TIMEOUT=600 SMOKE=0 BENCH=0 bash scripts/gpu_check.sh || exit $?
TAG=r03k SKIP_CHECK=1 bash scripts/r03_prof.sh || exit $?
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/seamsweep.py "" "small_pass=4096" "small_pass=4096,window_us=1000" > gpurun_out/seamsweep.log 2>&1 || { echo "seam sweep failed"; tail -20 gpurun_out/seamsweep.log; exit 3; }
echo "seam sweep ok"
SKIP_TESTS=1 bash scripts/gpu_check.sh || exit $?
