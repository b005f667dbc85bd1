#!/bin/bash
# callers debug, then GPU tests + smoke + a short bench (no cpu baseline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
FTZ_CALLERS_DEBUG=1 SEAM_SECONDS=1 timeout -k 10 200 python -u fabric-token-sdk_amd/tools/seamsweep.py "" > gpurun_out/seam1.log 2>&1; echo "seam rc=$?"; tail -4 gpurun_out/seam1.log
BENCH_ARGS="--steps 64 --no-cpu-baseline --no-seam" bash scripts/gpu_check.sh || exit $?
