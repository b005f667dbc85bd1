#!/bin/bash
# Full GPU test suite, prover probe, smoke + default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python -u fabric-token-sdk_amd/tools/provebench.py --steps 16 --no-split > gpurun_out/prover_fresh.log 2>&1 || { echo "provebench failed"; tail -20 gpurun_out/prover_fresh.log; exit 8; }
cat gpurun_out/prover_fresh.log
TEST_TIMEOUT=900 bash scripts/gpu_check.sh || exit $?
