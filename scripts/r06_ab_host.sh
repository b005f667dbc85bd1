#!/bin/bash
# round 6: headline A/B on one box: HEAD vs HEAD without FTS_HOST64 (h32) vs the r06b tree (2eb2da2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS="new=default|h32=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_h32.so|r6b=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_r6b.so" ROUNDS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb" bash scripts/ab_lib.sh
