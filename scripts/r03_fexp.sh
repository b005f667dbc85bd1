#!/bin/bash
# Round 3 check: VALU ceilings, GPU tests + smoke + bench, a kernel trace of a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u fabric-token-sdk_amd/tools/valupeak.py --out gpurun_out/valu_rates.json > gpurun_out/valupeak.log 2>&1 || { echo "valupeak failed"; tail -5 gpurun_out/valupeak.log; exit 3; }
tail -3 gpurun_out/valupeak.log
bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03a -o k -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-prover --msm 20 --distinct 4096 > gpurun_out/prof_r03a.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/prof_r03a.log; exit 6; }
echo trace ok
