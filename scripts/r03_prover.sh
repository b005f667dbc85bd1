#!/bin/bash
# Prover regression probe: fresh-process prover with plan/upload vs device split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
timeout -k 10 240 python -u fabric-token-sdk_amd/tools/provebench.py --steps 16 > gpurun_out/prover_split.log 2>&1 || { echo "provebench failed"; tail -20 gpurun_out/prover_split.log; exit 8; }
cat gpurun_out/prover_split.log
