#!/bin/bash
# round 6: LDS region stride 12 vs 20 vs previous rule (FTS_SQ_PAD 12 / 20 / 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06d_tests.log; exit 3; }
echo tests ok
L="p12=default|p20=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_pad20.so|p0=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_pad0.so"
LIBS="$L" bash scripts/pmc_lds.sh > gpurun_out/r06d_pmc.log 2>&1 || { echo pmc failed; exit 5; }
LIBS="$L" ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/r06d_ab.log 2>&1 || { echo ab failed; exit 6; }
echo all ok
